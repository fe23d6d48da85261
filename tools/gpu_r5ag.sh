# Round-5 session AG: the final sums (k_final_sums: needs alpha and the pivots only) on the side
# stream beside the gradient instead of after its reductions (in-tree) against the committed tree
# (ab/libace_base.so): full GPU suite, bitwise, C1 and C2 A/B.
set -o pipefail
out=gpurun_out/r5ag; mkdir -p $out
step() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
L=additivecausalexpansion_amd/libace_hip.so
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=8 --timeout 120 --timeout-method thread > $out/tests.log 2>&1
rc=$?; tail -12 $out/tests.log | grep -E "passed|failed|FAILED|ERROR"; if [ $rc -gt 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
step timeout -k 10 200 python tools/cmp_libs.py ab/libace_base.so $L 4096 SE > $out/cmp.txt 2>&1
step timeout -k 10 200 python tools/cmp_libs.py ab/libace_base.so $L 16384 Matern32 >> $out/cmp.txt 2>&1
cat $out/cmp.txt
ROUNDS=4 step timeout -k 10 400 bash tools/ab_libs.sh ab/libace_base.so $L -- --no-r6 --config C1 --steps 20 > $out/ab_c1.txt 2>&1; cat $out/ab_c1.txt
ROUNDS=2 step timeout -k 10 400 bash tools/ab_libs.sh ab/libace_base.so $L -- --no-r6 > $out/ab_c2.txt 2>&1; cat $out/ab_c2.txt
