# Round-5 session AE: the assembly / bulk-order switches tuned at C2, measured at C1 (env A/B of
# the committed tree): persistent assembly off, group 0's tail path after the assembly / after
# its head path, bulk tile order super-blocks 1 and 4 (default 2).
set -o pipefail
out=gpurun_out/r5ae; mkdir -p $out
step() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
ROUNDS=3 step timeout -k 10 700 bash tools/ab_envs.sh "" "ACE_ASM_PERSIST=0" "ACE_ASM_TAIL=0" "ACE_ASM_TAIL=2" "ACE_UPD_ORDER=1" "ACE_UPD_ORDER=4" -- --config C1 --steps 20 > $out/ab_c1.txt 2>&1; cat $out/ab_c1.txt
