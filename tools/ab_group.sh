# Group-schedule check: the bitwise tests of the sweep schedules, then the C2
# bench A/B of 2 / 3 / 4 steps per bulk launch (tools/ab_envs.sh).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "pair_steps or merged_cross_model" > gpurun_out/ab_group_tests.log 2>&1 || { tail -30 gpurun_out/ab_group_tests.log; exit 1; }
tail -2 gpurun_out/ab_group_tests.log
ROUNDS=${ROUNDS:-2} bash tools/ab_envs.sh "" "ACE_GROUP=3" "ACE_GROUP=4"
