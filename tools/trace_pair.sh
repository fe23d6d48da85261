# Kernel traces of one single-GPU and one sharded (1-rank RCCL) C2 run on the
# same box, each summarised by tools/shard_trace.py with its largest idle gaps.
set -o pipefail
mkdir -p gpurun_out/tp
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tp/single -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-r6 --no-cpu-baseline > $R/gpurun_out/tp/single.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tp/sharded -o run -- python3 $R/bench.py --mode sharded --shard-config C2 --steps 2 --warmup 1 > $R/gpurun_out/tp/sharded.log 2>&1 || exit 1
cd $R
for t in single sharded; do echo "== $t"; python tools/shard_trace.py gpurun_out/tp/$t ${NGAPS:-12}; done
