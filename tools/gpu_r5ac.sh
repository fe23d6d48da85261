# Round-5 session AC: at C2 the bulk launches are the critical path and the chains have slack --
# chain kernels at the default wave priority (ab/libace_p0.so, -DACE_CHAIN_PRIO=0) against
# s_setprio 1 (ab/libace_base.so, the committed tree), C2 A/B.
set -o pipefail
out=gpurun_out/r5ac; mkdir -p $out
step() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
ROUNDS=4 step timeout -k 10 700 bash tools/ab_libs.sh ab/libace_base.so ab/libace_p0.so -- --no-r6 > $out/ab_c2.txt 2>&1; cat $out/ab_c2.txt
