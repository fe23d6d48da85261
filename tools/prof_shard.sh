# Sharded GPU tests, the 1-rank pair-schedule A/B (tools/ab_shard_pair.sh)
# and a rocprofv3 kernel trace of one sharded C2 run (tools/shard_trace.py).
set -o pipefail
mkdir -p gpurun_out/shp
timeout -k 10 600 python -u -m pytest tests/test_shard_gpu.py tests/test_hostcomm_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/shp/tests.log 2>&1 || { tail -30 gpurun_out/shp/tests.log; exit 1; }
tail -2 gpurun_out/shp/tests.log
bash tools/ab_shard_pair.sh C2 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/shp/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --mode sharded --shard-config C2 --steps 2 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/shp/prof.log 2>&1
rc=$?
cd $GRAFT_REPO_ROOT && python tools/shard_trace.py gpurun_out/shp/prof | head -30
exit $rc
