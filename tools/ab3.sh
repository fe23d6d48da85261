# A/B/C: HEAD build, working tree, NB=512 working tree
for i in 1 2; do
  for lib in tools/libace_A.so additivecausalexpansion_amd/libace_hip.so tools/libace_nb512.so; do
    ACE_LIB_PATH=$lib timeout -k 5 100 python bench.py --steps 8 --warmup 2 --no-cpu-baseline "$@" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib'.split('/')[-1], round(d['ms_per_step'],2), round(d['roofline']['achieved'],2), {k: round(v,2) for k,v in d['phase_ms_per_step'].items()})" || exit 1
  done
done
