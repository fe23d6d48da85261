# The multi-panel kernel as the default two-step launch: bitwise tests of
# every schedule (single GPU and sharded), then single-GPU and sharded 1-rank
# C2 A/B against k_update_pair (ACE_MULTI2=0) and the round-2 pair schedule.
set -o pipefail
mkdir -p gpurun_out/g5
timeout -k 10 700 python -u -m pytest tests/test_gpu.py tests/test_shard_gpu.py tests/test_hostcomm_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "pair_steps or merged_cross_model or tile_order or cross_update or shard or hostcomm or host_comm or process" > gpurun_out/g5/tests.log 2>&1 || { tail -30 gpurun_out/g5/tests.log; exit 1; }
tail -2 gpurun_out/g5/tests.log
ROUNDS=${ROUNDS:-2} bash tools/ab_envs.sh "" "ACE_MULTI2=0" "ACE_GROUP_SCHED=0" || exit 1
AB_ENVS="ACE_MULTI2=0 ACE_X=1" bash tools/ab_shard_pair.sh C2
