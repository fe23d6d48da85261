set -o pipefail
mkdir -p gpurun_out/bs
timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bs/single.json 2> gpurun_out/bs/single.err && \
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29521 bench.py --mode sharded --steps 3 --warmup 1 > gpurun_out/bs/sh_c2.json 2> gpurun_out/bs/sh_c2.err && \
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29522 bench.py --mode sharded --shard-config C3 --steps 2 --warmup 1 > gpurun_out/bs/sh_c3.json 2> gpurun_out/bs/sh_c3.err && \
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29523 bench.py --mode sharded --shard-config C4 --steps 1 --warmup 1 > gpurun_out/bs/sh_c4.json 2> gpurun_out/bs/sh_c4.err
rc=$?
cat gpurun_out/bs/*.json | cut -c1-600
exit $rc
