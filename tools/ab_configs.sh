# Single-GPU A/B of the default (Z = 4, head / tail lookahead) against the
# round-3 Z = 2 schedule at the other BASELINE configs' sizes (C1, C3).
set -o pipefail
for c in ${CONFIGS:-C1 C3}; do
  for i in $(seq ${ROUNDS:-2}); do
    for e in "" "ACE_GROUP=2 ACE_HEADS=0"; do
      env $e timeout -k 5 200 python bench.py --config $c --steps ${STEPS:-6} --warmup 2 --no-cpu-baseline --no-r6 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c [$e]', round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['phase_ms_per_step'].items()})" || exit 1
    done
  done
done
