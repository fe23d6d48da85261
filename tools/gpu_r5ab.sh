# Round-5 session AB: one event wait on the main stream before each bulk launch (E2 stands for
# the head path too) and no combined ev[2g+1] record (in-tree) against the committed tree
# (ab/libace_base.so): full GPU suite, bitwise, C2 and C1 A/B, C2 bulk-to-bulk gaps.
set -o pipefail
R=$GRAFT_REPO_ROOT
out=gpurun_out/r5ab; mkdir -p $out
step() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
L=additivecausalexpansion_amd/libace_hip.so
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=8 --timeout 120 --timeout-method thread > $out/tests.log 2>&1
rc=$?; tail -12 $out/tests.log | grep -E "passed|failed|FAILED|ERROR"; if [ $rc -gt 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
step timeout -k 10 200 python tools/cmp_libs.py ab/libace_base.so $L 4096 SE > $out/cmp.txt 2>&1
step timeout -k 10 200 python tools/cmp_libs.py ab/libace_base.so $L 16384 Matern32 >> $out/cmp.txt 2>&1
cat $out/cmp.txt
ROUNDS=3 step timeout -k 10 500 bash tools/ab_libs.sh ab/libace_base.so $L -- --no-r6 > $out/ab_c2.txt 2>&1; cat $out/ab_c2.txt
ROUNDS=3 step timeout -k 10 300 bash tools/ab_libs.sh ab/libace_base.so $L -- --no-r6 --config C1 --steps 20 > $out/ab_c1.txt 2>&1; cat $out/ab_c1.txt
cd /tmp && export TMPDIR=/tmp
step timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/$out/c2trace -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-r6 --no-cpu-baseline > $R/$out/c2trace.log 2>&1
python3 $R/tools/bulk_gaps.py $R/$out/c2trace
