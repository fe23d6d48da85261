# A/B of several library builds in one call: args = .so paths; bench args via BENCH_ARGS
for i in 1 2; do
  for lib in "$@"; do
    ACE_LIB_PATH=$lib timeout -k 5 100 python bench.py --steps 8 --warmup 2 --no-cpu-baseline $BENCH_ARGS | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib'.split('/')[-1], round(d['ms_per_step'],2), round(d['roofline']['achieved'],2), {k: round(v,2) for k,v in d['phase_ms_per_step'].items()})" || exit 1
  done
done
