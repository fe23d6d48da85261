# Round-5 session P: the 16-blocked pivot sweep's row replication on ds_bpermute (ab/libace_bp1.so,
# -DACE_PIVOT_BP=1) and with the column lookahead (bp2): bitwise against the in-tree build at C1 and
# C2 sizes, C1 A/B, and C1 kernel traces of the in-tree build and bp1.
set -o pipefail
R=$GRAFT_REPO_ROOT
out=gpurun_out/r5p; mkdir -p $out
step() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
L=additivecausalexpansion_amd/libace_hip.so
for v in bp1 bp2; do
  step timeout -k 10 200 python tools/cmp_libs.py $L ab/libace_$v.so 4096 SE >> $out/cmp.txt 2>&1
  step timeout -k 10 200 python tools/cmp_libs.py $L ab/libace_$v.so 16384 Matern32 >> $out/cmp.txt 2>&1
done
cat $out/cmp.txt
ROUNDS=4 step timeout -k 10 500 bash tools/ab_libs.sh $L ab/libace_bp1.so ab/libace_bp2.so -- --no-r6 --config C1 --steps 20 > $out/ab_c1.txt 2>&1; cat $out/ab_c1.txt
cd /tmp && export TMPDIR=/tmp
step timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$out/c1trace -o run -- python3 $R/bench.py --config C1 --steps 10 --warmup 2 --no-r6 --no-cpu-baseline > $R/$out/c1trace.log 2>&1
python3 $R/tools/shard_trace.py $R/$out/c1trace 25 > $R/$out/c1trace.txt; head -14 $R/$out/c1trace.txt
export ACE_LIB_PATH=$R/ab/libace_bp1.so; step timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$out/c1trace_bp1 -o run -- python3 $R/bench.py --config C1 --steps 10 --warmup 2 --no-r6 --no-cpu-baseline > $R/$out/c1trace_bp1.log 2>&1
python3 $R/tools/shard_trace.py $R/$out/c1trace_bp1 25 > $R/$out/c1trace_bp1.txt; head -14 $R/$out/c1trace_bp1.txt
