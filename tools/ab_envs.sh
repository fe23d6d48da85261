# A/B/...: alternate bench runs of the working tree's library under several
# environment settings ("" = none); $ROUNDS rounds.
# usage: bash tools/ab_envs.sh "" "V=1" "V=2" [-- bench args]
envs=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do envs+=("$1"); shift; done; [ "$1" = "--" ] && shift
for i in $(seq ${ROUNDS:-3}); do
  for e in "${envs[@]}"; do
    env $e timeout -k 5 100 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-r6 "$@" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('[$e]', round(d['ms_per_step'],3), round(d['roofline']['achieved'],2), {k: round(v,2) for k,v in d['phase_ms_per_step'].items()}, {k: round(v,3) for k,v in (d.get('timeline_ms_per_eval') or {}).items() if v is not None})" || exit 1
  done
done
