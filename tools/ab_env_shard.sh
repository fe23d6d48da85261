# A/B of an env switch on the sharded leg (1 rank): $1 = VAR=value, $2 = config
for e in "" "$1"; do
  env $e timeout -k 5 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29531 bench.py --mode sharded --shard-config $2 --steps 1 --warmup 1 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read())['sharded']; print('[$e]', '$2', round(d['ms_per_step'],1), d['rank0_phase_ms_per_step'])" || exit 1
done
