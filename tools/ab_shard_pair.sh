# Sharded (1-rank RCCL) rates, same box: one-step schedule (ACE_PAIR=0),
# pair schedule with separate pack launches and full unpack (ACE_FUSE_PACK=0) and the
# default (ACE_X=1 is a no-op switch).  AB_ENVS overrides the list.  Args: configs (default C2).
set -o pipefail
mkdir -p gpurun_out/sp
port=29531
cfgs=${@:-C2}
timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-r6 > gpurun_out/sp/single.json 2> gpurun_out/sp/single.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/sp/single.json'));print('single C2', round(d['value'],3), round(d['ms_per_step'],1))"
for cfg in $cfgs; do
  for env in ${AB_ENVS:-ACE_PAIR=0 ACE_FUSE_PACK=0 ACE_X=1}; do
    port=$((port + 1))
    st=3; [ $cfg = C4 ] && st=2
    tag=${cfg}_${env%%=*}
    env $env timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $port bench.py --mode sharded --shard-config $cfg --steps $st --warmup 1 > gpurun_out/sp/$tag.json 2> gpurun_out/sp/$tag.err || exit 1
    python - gpurun_out/sp/$tag.json "$cfg $env" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.strip().startswith("{"):
        s = json.loads(l)["sharded"]
        print(sys.argv[2], round(s["evals_per_s"], 4), round(s["ms_per_step"], 1), "upd TF/s",
              round(s["rank0_update_kernel_tflops"] or 0, 1),
              {k: round(v, 1) for k, v in s["rank0_phase_ms_per_step"].items()})
PY
  done
done
