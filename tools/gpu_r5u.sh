# Round-5 session U: C1 with the chain's split (and head gather) workgroups given extra dynamic
# LDS so they cannot share a CU with a bulk / cross workgroup (ACE_XLDS_*, see ace_sweep.hip),
# and the per-workgroup records of the split-only setting.
set -o pipefail
out=gpurun_out/r5u; mkdir -p $out
step() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
ROUNDS=3 step timeout -k 10 500 bash tools/ab_envs.sh "" "ACE_XLDS_SPLIT=13312" "ACE_XLDS_SPLIT=13312 ACE_XLDS_Q=53248" "ACE_XLDS_SPLIT=5120 ACE_XLDS_BULK=8184" -- --config C1 --steps 20 > $out/ab_c1.txt 2>&1; cat $out/ab_c1.txt
export ACE_LIB_PATH=$PWD/ab/libace_wgt.so
ACE_XLDS_SPLIT=13312 WGT_DUMP=$out/wgt_c1_split.npy step timeout -k 10 200 python tools/wg_timeline.py 4096 10 6 SE > $out/wgt_c1_split.txt 2>&1
ACE_XLDS_SPLIT=13312 ACE_XLDS_Q=53248 WGT_DUMP=$out/wgt_c1_splitq.npy step timeout -k 10 200 python tools/wg_timeline.py 4096 10 6 SE > $out/wgt_c1_splitq.txt 2>&1
head -3 $out/wgt_c1_split.txt
