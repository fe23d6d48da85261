# A/B/...: alternate bench runs of the given libraries (ACE_LIB_PATH), $ROUNDS rounds
# usage: bash tools/ab_libs.sh lib1 lib2 ... [-- bench args]
libs=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do libs+=("$1"); shift; done; [ "$1" = "--" ] && shift
for i in $(seq ${ROUNDS:-3}); do
  for lib in "${libs[@]}"; do
    ACE_LIB_PATH=$lib timeout -k 5 100 python bench.py --steps 10 --warmup 2 --no-cpu-baseline "$@" | python -c "import json,sys; d=json.loads(sys.stdin.read()); pr=d.get('predict') or {}; print('$lib'.split('/')[-1], round(d['ms_per_step'],2), round(d['roofline']['achieved'],2), {k: round(v,2) for k,v in d['phase_ms_per_step'].items()}, {k: round(v['ms'],2) for k,v in pr.items() if isinstance(v, dict) and 'ms' in v})" || exit 1
  done
done
