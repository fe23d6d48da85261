# Group schedule A/B: pairs (default) / the group schedule at Z = 2 with
# k_update_pair / with k_update_multi / Z = 4; then a kernel trace at Z = 4.
set -o pipefail
mkdir -p gpurun_out/g4
ROUNDS=${ROUNDS:-2} bash tools/ab_envs.sh "" "ACE_GROUP_SCHED=1" "ACE_GROUP_SCHED=1 ACE_MULTI2=1" "ACE_GROUP=4" || exit 1
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
ACE_GROUP=4 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/g4/prof -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-r6 --no-cpu-baseline > $R/gpurun_out/g4/prof.log 2>&1 || exit 1
cd $R && python tools/shard_trace.py gpurun_out/g4/prof 10
