# A/B of an environment switch on the working tree's library: $1 = VAR=value for variant B
for i in 1 2; do
  for e in "" "$1"; do
    env $e timeout -k 5 100 python bench.py --steps 8 --warmup 2 --no-cpu-baseline ${@:2} | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('[$e]', round(d['ms_per_step'],2), round(d['roofline']['achieved'],2), {k: round(v,2) for k,v in d['phase_ms_per_step'].items()})" || exit 1
  done
done
