# Round-5 session Z: chain wave priority at C1 -- the split / pivot kernels at s_setprio 3
# instead of 1 (ab/libace_p3.so), the head gather k_update_q at the chain priority too (uq1:
# 1, uq3: 3), against the same build without (ab/libace_base.so); and base with the bulk
# leaving two CUs per engine (ACE_BULK_RESERVE=2).
set -o pipefail
out=gpurun_out/r5z; mkdir -p $out
step() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
ROUNDS=4 step timeout -k 10 600 bash tools/ab_libs.sh ab/libace_base.so ab/libace_p3.so ab/libace_uq1.so ab/libace_uq3.so -- --no-r6 --config C1 --steps 20 > $out/ab_c1.txt 2>&1; cat $out/ab_c1.txt
export ACE_LIB_PATH=$PWD/ab/libace_uq3.so
ROUNDS=3 step timeout -k 10 300 bash tools/ab_envs.sh "" "ACE_BULK_RESERVE=2" -- --config C1 --steps 20 > $out/ab_c1_r2.txt 2>&1; cat $out/ab_c1_r2.txt
