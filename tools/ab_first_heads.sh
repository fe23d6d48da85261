# The first group on the head / tail path: bitwise tests of the schedules,
# bitwise builds (prev = HEAD before, new = working tree, newpld72 = the split
# kernel's LDS in 72 KB), C2 A/B of the three, and a trace of the new build.
set -o pipefail
mkdir -p gpurun_out/fh
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "pair_steps or merged_cross_model" > gpurun_out/fh/tests.log 2>&1 || { tail -30 gpurun_out/fh/tests.log; exit 1; }
tail -1 gpurun_out/fh/tests.log
timeout -k 10 300 python tools/cmp_libs.py tools/libace_prev.so tools/libace_new.so || exit 1
timeout -k 10 300 python tools/cmp_libs.py tools/libace_new.so tools/libace_newpld72.so || exit 1
ROUNDS=3 bash tools/ab_libs.sh tools/libace_prev.so tools/libace_new.so tools/libace_newpld72.so -- --no-r6 || exit 1
NSHOW=2 bash tools/trace_group.sh fh ""
