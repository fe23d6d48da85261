# Round-5 session J: the sharded sweep on the single-GPU head / tail schedule
# (run_sweep_sharded_heads: head broadcast on the head path, tail broadcast +
# all-gather on the tail path over a second communicator); small-n tail
# launches on reserved queues.  Full GPU suite; sharded C2 (in-process 1-rank
# RCCL) against single-GPU C2, interleaved, with and without the head
# schedule; per-rank proxies C3 0/4, C4 0/8 both ways; C1 A/B; a sharded trace.
set -o pipefail
R=$GRAFT_REPO_ROOT
out=gpurun_out/r5j; mkdir -p $out
step() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=8 --timeout 120 --timeout-method thread > $out/tests.log 2>&1
rc=$?; tail -12 $out/tests.log | grep -E "passed|failed|FAILED|ERROR"; if [ $rc -gt 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
for i in 1 2; do
  step timeout -k 10 200 python bench.py --mode sharded --shard-config C2 --steps 6 --warmup 2 > $out/sh_heads_$i.json 2> $out/sh_heads_$i.err
  step env ACE_SHARD_HEADS=0 timeout -k 10 200 python bench.py --mode sharded --shard-config C2 --steps 6 --warmup 2 > $out/sh_groups_$i.json 2> $out/sh_groups_$i.err
  step timeout -k 10 200 python bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-r6 > $out/single_$i.json 2> $out/single_$i.err
done
python -c "
import json
for f in ('sh_heads_1','sh_groups_1','single_1','sh_heads_2','sh_groups_2','single_2'):
    d=json.loads(open('$out/'+f+'.json').read().strip().split('\n')[-1]); print(f, round(d['ms_per_step'],2))"
for hv in 1 0; do
  step env ACE_SHARD_HEADS=$hv ACE_LIB_PATH=$PWD/ab/libace_proxy.so timeout -k 10 300 python bench.py --mode sharded --shard-config C3 --proxy 0/4 --steps 3 --warmup 1 > $out/proxy_c3_h$hv.json 2> $out/proxy_c3_h$hv.err
  step env ACE_SHARD_HEADS=$hv ACE_LIB_PATH=$PWD/ab/libace_proxy.so timeout -k 10 300 python bench.py --mode sharded --shard-config C4 --proxy 0/8 --steps 3 --warmup 1 > $out/proxy_c4_h$hv.json 2> $out/proxy_c4_h$hv.err
done
python -c "
import json
for f in ('proxy_c3_h1','proxy_c3_h0','proxy_c4_h1','proxy_c4_h0'):
    d=json.loads(open('$out/'+f+'.json').read().strip().split('\n')[-1]); print(f, round(d['sharded']['ms_per_step'],2), {k: round(v,2) for k,v in d['sharded']['rank0_phase_ms_per_step'].items()})"
ROUNDS=2 step timeout -k 10 300 bash tools/ab_envs.sh "ACE_TAIL_RESERVE=0" "ACE_TAIL_RESERVE=1" -- --config C1 --steps 20 > $out/ab_c1.txt 2>&1; cat $out/ab_c1.txt
cd /tmp && export TMPDIR=/tmp
step timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/$out/shtrace -o run -- python3 $R/bench.py --mode sharded --shard-config C2 --steps 2 --warmup 1 > $R/$out/shtrace.log 2>&1
python3 $R/tools/shard_trace.py $R/$out/shtrace 20 > $R/$out/shtrace.txt; head -24 $R/$out/shtrace.txt
