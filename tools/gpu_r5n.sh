# Round-5 session N: Z = 3 sweep steps per bulk launch for n <= 8192 (sweep_group_n), the
# evaluation's results read back by one copy, and the pivot-column lookahead in the 16-blocked
# pivot sweep.  Full GPU suite; bitwise comparison with the build before them at C1 / C2 sizes;
# C1 A/B per change (ab/libace_presw.so -> ab/libace_z3.so -> ab/libace_res.so -> in-tree); C2
# A/B against the build before them; the bulk reserve 1 / 2 / 0 at C1.
set -o pipefail
R=$GRAFT_REPO_ROOT
out=gpurun_out/r5n; mkdir -p $out
step() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
L=additivecausalexpansion_amd/libace_hip.so
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=8 --timeout 120 --timeout-method thread > $out/tests.log 2>&1
rc=$?; tail -12 $out/tests.log | grep -E "passed|failed|FAILED|ERROR"; if [ $rc -gt 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
step timeout -k 10 200 python tools/cmp_libs.py ab/libace_presw.so $L 4096 SE > $out/cmp.txt 2>&1
step timeout -k 10 200 python tools/cmp_libs.py ab/libace_presw.so $L 16384 Matern32 >> $out/cmp.txt 2>&1
cat $out/cmp.txt
ROUNDS=3 step timeout -k 10 300 bash tools/ab_libs.sh ab/libace_res.so $L -- --no-r6 --config C1 --steps 20 > $out/ab_c1_la.txt 2>&1; cat $out/ab_c1_la.txt
ROUNDS=3 step timeout -k 10 300 bash tools/ab_libs.sh ab/libace_z3.so ab/libace_res.so -- --no-r6 --config C1 --steps 20 > $out/ab_c1_res.txt 2>&1; cat $out/ab_c1_res.txt
ROUNDS=2 step timeout -k 10 300 bash tools/ab_libs.sh ab/libace_presw.so $L -- --no-r6 --config C1 --steps 20 > $out/ab_c1.txt 2>&1; cat $out/ab_c1.txt
ROUNDS=2 step timeout -k 10 400 bash tools/ab_libs.sh ab/libace_presw.so $L -- --no-r6 > $out/ab_c2.txt 2>&1; cat $out/ab_c2.txt
ROUNDS=2 step timeout -k 10 300 bash tools/ab_envs.sh "ACE_BULK_RESERVE=1" "ACE_BULK_RESERVE=2" "ACE_BULK_RESERVE=0" -- --config C1 --steps 20 > $out/ab_c1_reserve.txt 2>&1; cat $out/ab_c1_reserve.txt
