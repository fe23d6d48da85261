# Effective clocks (GRBM_GUI_ACTIVE / 8 / wall, tools/clock_pmc.py) of the C2
# bench's kernels and of the bare fp64 MFMA loop (ab/probe_mfma_f64, built
# from tools/probe_mfma_f64.hip): one PMC pass each, with the kernel trace.
set -o pipefail
out=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $out/bench -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-r6 ${@:2} > $out/bench.log 2>&1 && \
timeout -s KILL 60 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $out/probe -o run -- $GRAFT_REPO_ROOT/ab/probe_mfma_f64 > $out/probe.log 2>&1 && \
python3 $GRAFT_REPO_ROOT/tools/clock_pmc.py $out/bench > $out/clock_bench.txt && \
python3 $GRAFT_REPO_ROOT/tools/clock_pmc.py $out/probe 0.2 > $out/clock_probe.txt && \
cat $out/clock_bench.txt $out/clock_probe.txt && grep "shape" $out/probe.log
