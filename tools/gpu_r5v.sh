# Round-5 session V: the side streams' rest-of-cross and tail updates of a group as persistent
# launches on the concurrent bulk launch's CU claims (ACE_SIDE_CLAIM=1, in-tree; the bulk
# leaves 2 CUs per engine, the side launches 1: the chain's CU) against ab/libace_sc0.so:
# full GPU suite, bitwise, C1 A/B, per-workgroup CU records.
set -o pipefail
out=gpurun_out/r5v; mkdir -p $out
step() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
L=additivecausalexpansion_amd/libace_hip.so
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=8 --timeout 120 --timeout-method thread > $out/tests.log 2>&1
rc=$?; tail -12 $out/tests.log | grep -E "passed|failed|FAILED|ERROR"; if [ $rc -gt 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
step timeout -k 10 200 python tools/cmp_libs.py ab/libace_sc0.so $L 4096 SE > $out/cmp.txt 2>&1
step timeout -k 10 200 python tools/cmp_libs.py ab/libace_sc0.so $L 8192 Matern32 >> $out/cmp.txt 2>&1
step timeout -k 10 200 python tools/cmp_libs.py ab/libace_sc0.so $L 2048 SE >> $out/cmp.txt 2>&1
cat $out/cmp.txt
ROUNDS=4 step timeout -k 10 400 bash tools/ab_libs.sh ab/libace_sc0.so $L -- --no-r6 --config C1 --steps 20 > $out/ab_c1.txt 2>&1; cat $out/ab_c1.txt
export ACE_LIB_PATH=$PWD/ab/libace_wgt.so
WGT_DUMP=$out/wgt_c1.npy step timeout -k 10 200 python tools/wg_timeline.py 4096 10 6 SE > $out/wgt_c1.txt 2>&1
head -3 $out/wgt_c1.txt
