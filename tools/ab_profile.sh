# A/B: bench ms/step with and without the per-launch HIP timing events
for i in $(seq ${ROUNDS:-3}); do
  for f in "" "--no-profile"; do
    timeout -k 5 100 python bench.py --steps 10 --warmup 2 --no-cpu-baseline $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('[$f]', round(d['ms_per_step'],2))" || exit 1
  done
done
