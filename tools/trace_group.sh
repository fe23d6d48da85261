# Kernel traces of C2 single-GPU runs under environment settings ("" = none),
# each summarised per group by tools/group_timeline.py.
# usage: bash tools/trace_group.sh TAG "" "ACE_GROUP=4" ...
set -o pipefail
tag=$1; shift
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/$tag
cd /tmp && export TMPDIR=/tmp
i=0
for e in "$@"; do
  i=$((i+1))
  env $e timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/$tag/t$i -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-r6 --no-cpu-baseline > $R/gpurun_out/$tag/t$i.log 2>&1 || exit 1
  echo "== [$e]"; python3 $R/tools/group_timeline.py $R/gpurun_out/$tag/t$i ${NSHOW:-4} || exit 1
done
