# A/B: the pair kernels with scalar-base addressing (default schedule) vs
# the group schedule at Z = 2 on k_update_multi; bitwise tests first.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "pair_steps or merged_cross_model or tile_order or cross_update" > gpurun_out/ab_group_tests.log 2>&1 || { tail -30 gpurun_out/ab_group_tests.log; exit 1; }
tail -2 gpurun_out/ab_group_tests.log
ROUNDS=${ROUNDS:-3} bash tools/ab_envs.sh "" "ACE_GROUP_SCHED=1 ACE_MULTI2=1"
