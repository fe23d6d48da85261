# Round-5 session R: the next group's Q launch waits for the tail path's and the bulk launch's
# events on the side stream directly (ACE_QWAIT_DIRECT=1, in-tree) instead of through the main
# stream's combined event (ab/libace_qw0.so): full GPU suite, bitwise against qw0, C1 and C2 A/B,
# C1 trace.
set -o pipefail
R=$GRAFT_REPO_ROOT
out=gpurun_out/r5r; mkdir -p $out
step() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
L=additivecausalexpansion_amd/libace_hip.so
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=8 --timeout 120 --timeout-method thread > $out/tests.log 2>&1
rc=$?; tail -12 $out/tests.log | grep -E "passed|failed|FAILED|ERROR"; if [ $rc -gt 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
step timeout -k 10 200 python tools/cmp_libs.py ab/libace_qw0.so $L 4096 SE > $out/cmp.txt 2>&1
step timeout -k 10 200 python tools/cmp_libs.py ab/libace_qw0.so $L 16384 Matern32 >> $out/cmp.txt 2>&1
step timeout -k 10 200 python tools/cmp_libs.py ab/libace_qw0.so $L 8192 SE >> $out/cmp.txt 2>&1
cat $out/cmp.txt
ROUNDS=4 step timeout -k 10 400 bash tools/ab_libs.sh ab/libace_qw0.so $L -- --no-r6 --config C1 --steps 20 > $out/ab_c1.txt 2>&1; cat $out/ab_c1.txt
ROUNDS=2 step timeout -k 10 400 bash tools/ab_libs.sh ab/libace_qw0.so $L -- --no-r6 > $out/ab_c2.txt 2>&1; cat $out/ab_c2.txt
cd /tmp && export TMPDIR=/tmp
step timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$out/c1trace -o run -- python3 $R/bench.py --config C1 --steps 10 --warmup 2 --no-r6 --no-cpu-baseline > $R/$out/c1trace.log 2>&1
python3 $R/tools/shard_trace.py $R/$out/c1trace 25 > $R/$out/c1trace.txt; head -40 $R/$out/c1trace.txt
