# Gradient slice loop unrolled by 2 (-DACE_GRAD_UNROLL=2): bitwise, C2 A/B.
set -o pipefail
for k in Matern32 SE; do
  timeout -k 10 300 python tools/cmp_libs.py additivecausalexpansion_amd/libace_hip.so tools/libace_unroll2.so 3001 $k || exit 1
done
ROUNDS=3 bash tools/ab_libs.sh additivecausalexpansion_amd/libace_hip.so tools/libace_unroll2.so -- --no-r6
