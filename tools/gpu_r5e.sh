# Round-5 session E: the split kernel's batched prologue loads and the head
# path's quartered panel GEMM (k_panel_gemm_q); prediction's cross kernel with
# both point sets staged and the cached prediction scratch.  Full GPU suite;
# bitwise check against the round's start; same-box C1 / C2 A/B; C1 marks; C2 kernel stats.
set -o pipefail
R=$GRAFT_REPO_ROOT
out=gpurun_out/r5e; mkdir -p $out
step() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
L=additivecausalexpansion_amd/libace_hip.so
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=8 --timeout 120 --timeout-method thread > $out/tests.log 2>&1
rc=$?; tail -12 $out/tests.log | grep -E "passed|failed|FAILED|ERROR"; if [ $rc -gt 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
step timeout -k 10 200 python tools/cmp_libs.py ab/libace_head.so $L 4096 SE > $out/cmp.txt 2>&1
step timeout -k 10 200 python tools/cmp_libs.py ab/libace_head.so $L 16384 Matern32 >> $out/cmp.txt 2>&1
cat $out/cmp.txt
ROUNDS=2 step timeout -k 10 400 bash tools/ab_libs.sh ab/libace_head.so $L ab/libace_pgt.so -- --no-r6 --config C1 --steps 20 > $out/ab_c1.txt 2>&1; cat $out/ab_c1.txt
ROUNDS=2 step timeout -k 10 500 bash tools/ab_libs.sh ab/libace_head.so $L -- --no-r6 > $out/ab_c2.txt 2>&1; cat $out/ab_c2.txt
step env ACE_LIB_PATH=$PWD/ab/libace_wgt.so timeout -k 10 200 python tools/wg_timeline.py 4096 10 6 SE > $out/wgt_c1.txt 2>&1
head -30 $out/wgt_c1.txt
step bash tools/run_prof.sh r5e/prof --steps 5 --warmup 1 --no-r6
python3 tools/kernel_stats_split.py $out/prof > $out/kernel_stats_split.csv; head -14 $out/kernel_stats_split.csv | cut -c1-160
