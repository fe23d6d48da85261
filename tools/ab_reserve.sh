# The assembly's second part on a CU-masked stream that leaves R CUs to the
# first group's chains (ACE_ASM_RESERVE=R): bitwise check, C2 A/B, trace.
set -o pipefail
mkdir -p gpurun_out/rs
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "merged_cross_model" > gpurun_out/rs/tests.log 2>&1 || { tail -30 gpurun_out/rs/tests.log; exit 1; }
tail -1 gpurun_out/rs/tests.log
for R in 8 16; do
  CMP_ENV_B="ACE_ASM_RESERVE=$R" timeout -k 10 300 python tools/cmp_libs.py additivecausalexpansion_amd/libace_hip.so additivecausalexpansion_amd/libace_hip.so 16384 || exit 1
done
ROUNDS=3 bash tools/ab_envs.sh "" "ACE_ASM_RESERVE=8" "ACE_ASM_RESERVE=16" || exit 1
NSHOW=1 bash tools/trace_group.sh rs "ACE_ASM_RESERVE=8" "ACE_ASM_RESERVE=16"
