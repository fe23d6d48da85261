# HIP API + kernel trace of a short single-GPU C2 bench and of the sharded
# 1-rank run: the host work between two evaluations (tools/host_gap.py).
set -o pipefail
mkdir -p gpurun_out/hg
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --output-format csv -d $R/gpurun_out/hg/single -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-r6 --no-cpu-baseline > $R/gpurun_out/hg/single.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --output-format csv -d $R/gpurun_out/hg/sharded -o run -- python3 $R/bench.py --mode sharded --shard-config C2 --steps 3 --warmup 1 > $R/gpurun_out/hg/sharded.log 2>&1 || exit 1
cd $R
for t in single sharded; do echo "== $t"; python tools/host_gap.py gpurun_out/hg/$t | head -60; done
