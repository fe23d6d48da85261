# Round-5 session H: pair-kernel tile staging with every global load issued
# before the LDS stores (mm_stage: assembly and gradient tiles); the gradient
# tile's finish over the whole workgroup.  Full GPU suite; comparison with the
# round's start (assembly / inverse bit-identical, gradient ulp-level); C2 A/B;
# C2 per-workgroup phases; rocprof kernel stats.
set -o pipefail
R=$GRAFT_REPO_ROOT
out=gpurun_out/r5h; mkdir -p $out
step() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
L=additivecausalexpansion_amd/libace_hip.so
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=8 --timeout 120 --timeout-method thread > $out/tests.log 2>&1
rc=$?; tail -12 $out/tests.log | grep -E "passed|failed|FAILED|ERROR"; if [ $rc -gt 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
step timeout -k 10 200 python tools/cmp_libs.py ab/libace_head.so $L 4096 SE > $out/cmp.txt 2>&1
step timeout -k 10 200 python tools/cmp_libs.py ab/libace_head.so $L 16384 Matern32 >> $out/cmp.txt 2>&1
cat $out/cmp.txt
ROUNDS=3 step timeout -k 10 600 bash tools/ab_libs.sh ab/libace_head.so $L -- --no-r6 > $out/ab_c2.txt 2>&1; cat $out/ab_c2.txt
ROUNDS=2 step timeout -k 10 300 bash tools/ab_libs.sh ab/libace_head.so $L -- --no-r6 --config C1 --steps 20 > $out/ab_c1.txt 2>&1; cat $out/ab_c1.txt
step env ACE_LIB_PATH=$PWD/ab/libace_wgt.so timeout -k 10 300 python tools/wg_timeline.py > $out/wgt_c2.txt 2>&1
grep -E "grad_mm|asm|phases" $out/wgt_c2.txt | head
step bash tools/run_prof.sh r5h/prof --steps 5 --warmup 1 --no-r6
python3 tools/kernel_stats_split.py $out/prof > $out/kernel_stats_split.csv; head -16 $out/kernel_stats_split.csv | cut -c1-150
