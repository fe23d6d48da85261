# Round-5 session Q: the pivot update with one FMA per element for the pivot row and the rest
# (ab/libace_bp3.so, -DACE_PIVOT_BP=3, on top of bp1's ds_bpermute replication): bitwise
# against the in-tree build at C1 and C2 sizes, C1 A/B against in-tree and bp1, k_pivot's
# duration under rocprof.
set -o pipefail
R=$GRAFT_REPO_ROOT
out=gpurun_out/r5q; mkdir -p $out
step() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
L=additivecausalexpansion_amd/libace_hip.so
step timeout -k 10 200 python tools/cmp_libs.py $L ab/libace_bp3.so 4096 SE >> $out/cmp.txt 2>&1
step timeout -k 10 200 python tools/cmp_libs.py $L ab/libace_bp3.so 16384 Matern32 >> $out/cmp.txt 2>&1
step timeout -k 10 200 python tools/cmp_libs.py $L ab/libace_bp3.so 8192 Matern32 >> $out/cmp.txt 2>&1
cat $out/cmp.txt
ROUNDS=4 step timeout -k 10 500 bash tools/ab_libs.sh $L ab/libace_bp1.so ab/libace_bp3.so -- --no-r6 --config C1 --steps 20 > $out/ab_c1.txt 2>&1; cat $out/ab_c1.txt
cd /tmp && export TMPDIR=/tmp
export ACE_LIB_PATH=$R/ab/libace_bp3.so; step timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$out/c1trace_bp3 -o run -- python3 $R/bench.py --config C1 --steps 10 --warmup 2 --no-r6 --no-cpu-baseline > $R/$out/c1trace_bp3.log 2>&1
python3 $R/tools/shard_trace.py $R/$out/c1trace_bp3 25 > $R/$out/c1trace_bp3.txt; head -14 $R/$out/c1trace_bp3.txt
