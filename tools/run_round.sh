# Full GPU check: tests, smoke, bench (with CPU baseline), rocprof kernel stats.
set -o pipefail
tag=${1:-v}
mkdir -p gpurun_out/$tag
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --durations=20 --timeout 120 --timeout-method thread > gpurun_out/$tag/tests.log 2>&1 && tail -1 gpurun_out/$tag/tests.log && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$tag/smoke.log 2>&1 && cat gpurun_out/$tag/smoke.log && \
timeout -k 10 400 python bench.py --steps 10 --warmup 2 > gpurun_out/$tag/bench.json 2> gpurun_out/$tag/bench.err && cut -c1-400 gpurun_out/$tag/bench.json && \
bash tools/run_prof.sh $tag/prof --steps 5 --warmup 1 > /dev/null
