# Round-5 session M: C1 with 2, 3, 4 sweep steps per bulk launch (ACE_GROUP);
# C1 trace of the default.
set -o pipefail
R=$GRAFT_REPO_ROOT
out=gpurun_out/r5m; mkdir -p $out
step() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
ROUNDS=3 step timeout -k 10 400 bash tools/ab_envs.sh "ACE_GROUP=4" "ACE_GROUP=3" "ACE_GROUP=2" -- --config C1 --steps 20 > $out/ab_c1_group.txt 2>&1; cat $out/ab_c1_group.txt
cd /tmp && export TMPDIR=/tmp
step timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/$out/c1trace -o run -- python3 $R/bench.py --config C1 --steps 3 --warmup 2 --no-r6 --no-cpu-baseline > $R/$out/c1trace.log 2>&1
python3 $R/tools/shard_trace.py $R/$out/c1trace 25 > $R/$out/c1trace.txt; head -14 $R/$out/c1trace.txt
