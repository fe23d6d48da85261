# Round-5 session B: the full GPU suite on the round-5 tree (blocked / fused pivot,
# MFMA cross assembly, sharded group schedule), the inverse-accuracy probe, C2 / C1
# bench lines (old-pivot A/B), per-rank proxy timing of the sharded path, a C1 trace.
# Any GPU step that faults, aborts or times out ends the script (no later GPU step);
# test failures are results (pytest rc 1) and do not.
set -o pipefail
R=$GRAFT_REPO_ROOT
out=gpurun_out/r5b; mkdir -p $out
step() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=8 --timeout 120 --timeout-method thread > $out/tests.log 2>&1
rc=$?; tail -12 $out/tests.log | grep -E "passed|failed|FAILED|ERROR"; if [ $rc -gt 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
step timeout -k 10 300 python -u tools/inverse_probe.py gpurun_out/invp cur=ab/libace_cur.so new=additivecausalexpansion_amd/libace_hip.so pold=ab/libace_pold.so > $out/invp.log 2>&1
step timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-r6 > $out/bench_c2.json 2> $out/bench_c2.err
python -c "import json;d=json.load(open('$out/bench_c2.json'));print('C2', d['ms_per_step'], d['predict']['predict']['ms'], d['predict']['predict_marginal_ate']['ms'])"
step timeout -k 10 200 python bench.py --config C1 --steps 20 --warmup 3 --no-cpu-baseline --no-r6 > $out/bench_c1.json 2> $out/bench_c1.err
step env ACE_LIB_PATH=$PWD/ab/libace_pold.so timeout -k 10 200 python bench.py --config C1 --steps 20 --warmup 3 --no-cpu-baseline --no-r6 > $out/bench_c1_pold.json 2> $out/bench_c1_pold.err
python -c "import json;[print(f, json.load(open('$out/'+f))['ms_per_step']) for f in ('bench_c1.json','bench_c1_pold.json')]"
step env ACE_LIB_PATH=$PWD/ab/libace_proxy.so timeout -k 10 300 python bench.py --mode sharded --shard-config C3 --proxy 0/4 --steps 3 --warmup 1 > $out/proxy_c3_r0of4.json 2> $out/proxy_c3.err
step env ACE_LIB_PATH=$PWD/ab/libace_proxy.so timeout -k 10 300 python bench.py --mode sharded --shard-config C4 --proxy 0/8 --steps 3 --warmup 1 > $out/proxy_c4_r0of8.json 2> $out/proxy_c4.err
python -c "import json;[print(f, json.load(open('$out/'+f))['sharded']['ms_per_step'], json.load(open('$out/'+f))['sharded']['rank0_phase_ms_per_step']) for f in ('proxy_c3_r0of4.json','proxy_c4_r0of8.json')]"
cd /tmp && export TMPDIR=/tmp
step timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/$out/c1trace -o run -- python3 $R/bench.py --config C1 --steps 3 --warmup 2 --no-r6 --no-cpu-baseline > $R/$out/c1trace.log 2>&1
python3 $R/tools/shard_trace.py $R/$out/c1trace 25 > $R/$out/c1trace.txt; head -30 $R/$out/c1trace.txt
