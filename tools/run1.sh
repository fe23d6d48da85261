set -o pipefail
mkdir -p gpurun_out/r1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r1/tests.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > gpurun_out/r1/bench.json 2> gpurun_out/r1/bench.err && \
cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r1/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/r1/prof.log 2>&1
