# Round-5 session K: the sharded head schedule with group g+1's lookahead
# ordered after group g's tail path (E_PRE).  Sharded GPU tests first, then
# the full suite; sharded C2 vs single C2 interleaved; proxies; a trace.
set -o pipefail
R=$GRAFT_REPO_ROOT
out=gpurun_out/r5k; mkdir -p $out
step() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
timeout -k 10 600 python -u -m pytest tests/test_shard_gpu.py tests/test_hostcomm_gpu.py tests/test_fullsize_gpu.py -m gpu -v --maxfail=8 --timeout 150 --timeout-method thread > $out/tests_shard.log 2>&1
rc=$?; tail -12 $out/tests_shard.log | grep -E "passed|failed|FAILED|ERROR"; if [ $rc -ne 0 ]; then echo "pytest rc=$rc"; exit $rc; fi
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=8 --timeout 120 --timeout-method thread > $out/tests.log 2>&1
rc=$?; tail -12 $out/tests.log | grep -E "passed|failed|FAILED|ERROR"; if [ $rc -gt 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
for i in 1 2; do
  step timeout -k 10 200 python bench.py --mode sharded --shard-config C2 --steps 6 --warmup 2 > $out/sh_heads_$i.json 2> $out/sh_heads_$i.err
  step timeout -k 10 200 python bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-r6 > $out/single_$i.json 2> $out/single_$i.err
done
python -c "
import json
for f in ('sh_heads_1','single_1','sh_heads_2','single_2'):
    d=json.loads(open('$out/'+f+'.json').read().strip().split('\n')[-1]); print(f, round(d['ms_per_step'],2))"
step env ACE_LIB_PATH=$PWD/ab/libace_proxy.so timeout -k 10 300 python bench.py --mode sharded --shard-config C3 --proxy 0/4 --steps 3 --warmup 1 > $out/proxy_c3_r0of4.json 2> $out/proxy_c3.err
step env ACE_LIB_PATH=$PWD/ab/libace_proxy.so timeout -k 10 300 python bench.py --mode sharded --shard-config C4 --proxy 0/8 --steps 3 --warmup 1 > $out/proxy_c4_r0of8.json 2> $out/proxy_c4.err
python -c "
import json
for f in ('proxy_c3_r0of4','proxy_c4_r0of8'):
    d=json.loads(open('$out/'+f+'.json').read().strip().split('\n')[-1]); print(f, round(d['sharded']['ms_per_step'],2), {k: round(v,2) for k,v in d['sharded']['rank0_phase_ms_per_step'].items()})"
