# The handle path with the slice-norms table: its tests, then the bench's
# unchanged-R6 leg beside the fused model.
set -o pipefail
mkdir -p gpurun_out/r6n
timeout -k 10 600 python -u -m pytest tests/test_r6_handles_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6n/tests.log 2>&1 || { tail -30 gpurun_out/r6n/tests.log; exit 1; }
tail -1 gpurun_out/r6n/tests.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],2), 'r6', round(d['r6_drop_in']['ms_per_eval'],2), round(d['r6_drop_in']['vs_fused_ms_ratio'],4))" || exit 1
done
