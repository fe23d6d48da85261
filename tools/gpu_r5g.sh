# Round-5 session G: branch-free slice loops in the assembly / cross pair
# kernels (kval_nb); bulk launch enqueued before the next group's lookahead;
# small-n Q-first group boundary (ACE_QFIRST) with / without the bulk reserve.
# Full GPU suite; bitwise check against the round's start at C1 and C2 sizes;
# C1 A/B matrix; C2 A/B (round start / new / new with Q-first); C1 trace.
set -o pipefail
R=$GRAFT_REPO_ROOT
out=gpurun_out/r5g; mkdir -p $out
step() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
L=additivecausalexpansion_amd/libace_hip.so
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=8 --timeout 120 --timeout-method thread > $out/tests.log 2>&1
rc=$?; tail -12 $out/tests.log | grep -E "passed|failed|FAILED|ERROR"; if [ $rc -gt 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
step timeout -k 10 200 python tools/cmp_libs.py ab/libace_head.so $L 4096 SE > $out/cmp.txt 2>&1
step timeout -k 10 200 python tools/cmp_libs.py ab/libace_head.so $L 16384 Matern32 >> $out/cmp.txt 2>&1
cat $out/cmp.txt
ROUNDS=2 step timeout -k 10 500 bash tools/ab_envs.sh "ACE_QFIRST=0 ACE_BULK_RESERVE=0" "ACE_QFIRST=1 ACE_BULK_RESERVE=0" "ACE_QFIRST=1 ACE_BULK_RESERVE=1" "ACE_QFIRST=0 ACE_BULK_RESERVE=1" -- --config C1 --steps 20 > $out/ab_c1.txt 2>&1; cat $out/ab_c1.txt
ROUNDS=2 step timeout -k 10 500 bash tools/ab_libs.sh ab/libace_head.so $L -- --no-r6 > $out/ab_c2.txt 2>&1; cat $out/ab_c2.txt
ROUNDS=2 step timeout -k 10 300 bash tools/ab_envs.sh "ACE_QFIRST=1" > $out/ab_c2_qfirst.txt 2>&1; cat $out/ab_c2_qfirst.txt
cd /tmp && export TMPDIR=/tmp
step timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/$out/c1trace -o run -- python3 $R/bench.py --config C1 --steps 3 --warmup 2 --no-r6 --no-cpu-baseline > $R/$out/c1trace.log 2>&1
python3 $R/tools/shard_trace.py $R/$out/c1trace 25 > $R/$out/c1trace.txt; head -14 $R/$out/c1trace.txt
