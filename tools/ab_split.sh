# The assembly's second part split into a CU-masked part 3 and a part 4
# launched after the first group's head path (ACE_ASM_SPLIT = part 3's share):
# bitwise tests, bitwise against the previous build, C2 A/B, trace.
set -o pipefail
mkdir -p gpurun_out/sp
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "pair_steps or merged_cross_model or tile_order or cross_update" > gpurun_out/sp/tests.log 2>&1 || { tail -30 gpurun_out/sp/tests.log; exit 1; }
tail -1 gpurun_out/sp/tests.log
timeout -k 10 300 python tools/cmp_libs.py tools/libace_prev.so additivecausalexpansion_amd/libace_hip.so 16384 || exit 1
CMP_ENV_B="ACE_ASM_RESERVE=0" timeout -k 10 300 python tools/cmp_libs.py additivecausalexpansion_amd/libace_hip.so additivecausalexpansion_amd/libace_hip.so 3000 || exit 1
ROUNDS=3 bash tools/ab_envs.sh "" "ACE_ASM_SPLIT=1" "ACE_ASM_SPLIT=0.5" "ACE_ASM_SPLIT=0.85" || exit 1
NSHOW=1 bash tools/trace_group.sh sp ""
