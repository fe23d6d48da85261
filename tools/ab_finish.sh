# Gradient finish with the column sums added once per slice: bitwise against
# the previous build (both kernels, odd n), then C2 A/B of the two builds.
set -o pipefail
for k in Matern32 SE; do
  for n in 16384 3001; do
    timeout -k 10 300 python tools/cmp_libs.py tools/libace_prev.so additivecausalexpansion_amd/libace_hip.so $n $k || exit 1
  done
done
ROUNDS=3 bash tools/ab_libs.sh tools/libace_prev.so additivecausalexpansion_amd/libace_hip.so -- --no-r6
