# Round-5 session D: the head GEMM back at one chunk in flight (A/B against the
# previous commit's depth 2 and the round's start); the small-n bulk cap
# (ACE_BULK_CAP) at C1; per-workgroup phase marks of the chain kernels at C1;
# the in-process 1-rank RCCL sharded C2 interleaved with single-GPU C2, and its trace.
set -o pipefail
R=$GRAFT_REPO_ROOT
out=gpurun_out/r5d; mkdir -p $out
step() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
L=additivecausalexpansion_amd/libace_hip.so
step timeout -k 10 200 python tools/cmp_libs.py ab/libace_head.so $L 4096 SE > $out/cmp.txt 2>&1
cat $out/cmp.txt
ROUNDS=2 step timeout -k 10 600 bash tools/ab_libs.sh ab/libace_head.so $L ab/libace_pg2.so ab/libace_s2n.so -- --no-r6 > $out/ab_c2.txt 2>&1; cat $out/ab_c2.txt
ROUNDS=2 step timeout -k 10 400 bash tools/ab_envs.sh "ACE_BULK_CAP=0" "ACE_BULK_CAP=64" "ACE_BULK_CAP=128" "ACE_BULK_CAP=192" -- --config C1 --steps 20 > $out/ab_c1_cap.txt 2>&1; cat $out/ab_c1_cap.txt
step env ACE_LIB_PATH=$PWD/ab/libace_wgt.so ACE_BULK_CAP=0 timeout -k 10 200 python tools/wg_timeline.py 4096 10 6 SE > $out/wgt_c1_cap0.txt 2>&1
step env ACE_LIB_PATH=$PWD/ab/libace_wgt.so ACE_BULK_CAP=128 timeout -k 10 200 python tools/wg_timeline.py 4096 10 6 SE > $out/wgt_c1_cap128.txt 2>&1
grep -A4 "per-workgroup phases" $out/wgt_c1_cap0.txt
for i in 1 2; do
  step timeout -k 10 200 python bench.py --mode sharded --shard-config C2 --steps 6 --warmup 2 > $out/sharded_c2_$i.json 2> $out/sharded_c2_$i.err
  step timeout -k 10 200 python bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-r6 > $out/single_c2_$i.json 2> $out/single_c2_$i.err
done
python -c "
import json
for f in ('sharded_c2_1','single_c2_1','sharded_c2_2','single_c2_2'):
    d=json.loads(open('$out/'+f+'.json').read().strip().split('\n')[-1]); print(f, round(d['ms_per_step'],2))"
cd /tmp && export TMPDIR=/tmp
step env ACE_BULK_CAP=128 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/$out/c1trace -o run -- python3 $R/bench.py --config C1 --steps 3 --warmup 2 --no-r6 --no-cpu-baseline > $R/$out/c1trace.log 2>&1
python3 $R/tools/shard_trace.py $R/$out/c1trace 25 > $R/$out/c1trace.txt; head -12 $R/$out/c1trace.txt
step timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/$out/shtrace -o run -- python3 $R/bench.py --mode sharded --shard-config C2 --steps 2 --warmup 1 > $R/$out/shtrace.log 2>&1
python3 $R/tools/shard_trace.py $R/$out/shtrace 25 > $R/$out/shtrace.txt; head -30 $R/$out/shtrace.txt
