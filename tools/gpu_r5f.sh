# Round-5 session F: the small-n bulk launch as a persistent queue leaving
# CUs to the chains (k_update_multi_r, ACE_BULK_RESERVE).  Full GPU suite
# (its switch-neutrality test covers the reserve); bitwise check against the
# round's start; same-box C1 A/B of the reserve (0 / 1 / 2); C1 marks; one C2 line.
set -o pipefail
R=$GRAFT_REPO_ROOT
out=gpurun_out/r5f; mkdir -p $out
step() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
L=additivecausalexpansion_amd/libace_hip.so
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=8 --timeout 120 --timeout-method thread > $out/tests.log 2>&1
rc=$?; tail -12 $out/tests.log | grep -E "passed|failed|FAILED|ERROR"; if [ $rc -gt 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
step timeout -k 10 200 python tools/cmp_libs.py ab/libace_head.so $L 4096 SE > $out/cmp.txt 2>&1
cat $out/cmp.txt
ROUNDS=2 step timeout -k 10 400 bash tools/ab_envs.sh "ACE_BULK_RESERVE=0" "ACE_BULK_RESERVE=1" "ACE_BULK_RESERVE=2" -- --config C1 --steps 20 > $out/ab_c1.txt 2>&1; cat $out/ab_c1.txt
step env ACE_LIB_PATH=$PWD/ab/libace_wgt.so timeout -k 10 200 python tools/wg_timeline.py 4096 10 6 SE > $out/wgt_c1.txt 2>&1
head -32 $out/wgt_c1.txt
step timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-r6 > $out/bench_c2.json 2> $out/bench_c2.err
python -c "import json;d=json.load(open('$out/bench_c2.json'));print('C2', round(d['ms_per_step'],2), d['predict']['predict']['ms'], d['predict']['predict_marginal_ate']['ms'])"
cd /tmp && export TMPDIR=/tmp
step timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/$out/c1trace -o run -- python3 $R/bench.py --config C1 --steps 3 --warmup 2 --no-r6 --no-cpu-baseline > $R/$out/c1trace.log 2>&1
python3 $R/tools/shard_trace.py $R/$out/c1trace 25 > $R/$out/c1trace.txt; head -14 $R/$out/c1trace.txt
