# Handle-path (unchanged R6 sequence) GPU tests, then the bench with the
# round-3 direct path (ACE_DMAT_DIRECT=1) against the round-2 one (0).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_r6_handles_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r6t.log 2>&1 || { tail -30 gpurun_out/r6t.log; exit 1; }
tail -3 gpurun_out/r6t.log
for v in 1 0 1; do
  ACE_DMAT_DIRECT=$v timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r6ab_$v.json 2> gpurun_out/r6ab_$v.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/r6ab_$v.json'));print('direct=$v', d['ms_per_step'], d['r6_drop_in'])"
done
