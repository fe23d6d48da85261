# rocprofv3 kernel stats of the C2 bench (csv), written under gpurun_out/$1
set -o pipefail
out=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p $out
shift
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline "$@" > $out/bench.log 2>&1
rc=$?
find $out -name "*kernel_stats.csv" | head -3
tail -2 $out/bench.log | cut -c1-300
exit $rc
