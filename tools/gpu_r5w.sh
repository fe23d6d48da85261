# Round-5 session W: side claims (session V) plus split workgroups sized to fit beside no update
# workgroup from group 1 on (ACE_SPLIT_ALONE=1, in-tree) against side claims alone
# (ab/libace_sa0.so) and neither (ab/libace_sc0.so): bitwise, C1 A/B, per-workgroup CU records.
set -o pipefail
out=gpurun_out/r5w; mkdir -p $out
step() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
L=additivecausalexpansion_amd/libace_hip.so
step timeout -k 10 200 python tools/cmp_libs.py ab/libace_sc0.so $L 4096 SE > $out/cmp.txt 2>&1
step timeout -k 10 200 python tools/cmp_libs.py ab/libace_sc0.so $L 8192 Matern32 >> $out/cmp.txt 2>&1
cat $out/cmp.txt
ROUNDS=4 step timeout -k 10 500 bash tools/ab_libs.sh ab/libace_sc0.so ab/libace_sa0.so $L -- --no-r6 --config C1 --steps 20 > $out/ab_c1.txt 2>&1; cat $out/ab_c1.txt
export ACE_LIB_PATH=$PWD/ab/libace_wgt.so
WGT_DUMP=$out/wgt_c1.npy step timeout -k 10 200 python tools/wg_timeline.py 4096 10 6 SE > $out/wgt_c1.txt 2>&1
head -3 $out/wgt_c1.txt
