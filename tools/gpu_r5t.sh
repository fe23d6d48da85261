# Round-5 session T: per-workgroup records of one C1 evaluation (ab/libace_wgt.so,
# -DACE_DIAG_WGTIME) dumped raw, for the CU-sharing analysis of the chain's split
# workgroups (tools/wgt_cu.py).
set -o pipefail
out=gpurun_out/r5t; mkdir -p $out
step() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
export ACE_LIB_PATH=$PWD/ab/libace_wgt.so
WGT_DUMP=$out/wgt_c1.npy step timeout -k 10 200 python tools/wg_timeline.py 4096 10 6 SE > $out/wgt_c1.txt 2>&1
head -30 $out/wgt_c1.txt
