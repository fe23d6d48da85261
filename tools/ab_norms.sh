# Slice norms once per evaluation (TabView::norms) against per-tile norms:
# bitwise (both kernels, odd n), then C2 A/B.
set -o pipefail
for k in Matern32 SE; do
  for n in 16384 3001; do
    timeout -k 10 300 python tools/cmp_libs.py tools/libace_prev.so additivecausalexpansion_amd/libace_hip.so $n $k || exit 1
  done
done
CMP_ENV_B="ACE_NORMS=0" timeout -k 10 300 python tools/cmp_libs.py additivecausalexpansion_amd/libace_hip.so additivecausalexpansion_amd/libace_hip.so 5000 || exit 1
ROUNDS=3 bash tools/ab_envs.sh "" "ACE_NORMS=0"
