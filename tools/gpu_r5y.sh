# Round-5 session Y: the sharded head schedule's next-group lookahead waiting for the tail
# path's and the bulk launch's events directly (E_READY2 / E_BULK) instead of through E_PRE.
# Sharded GPU tests, sharded C2 vs single C2, per-rank proxies old (ab/libace_proxy_old.so =
# the tree before) vs new (ab/libace_proxy.so) at C3 / 4 and C4 / 8.
set -o pipefail
out=gpurun_out/r5y; mkdir -p $out
step() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
timeout -k 10 600 python -u -m pytest tests/test_shard_gpu.py tests/test_hostcomm_gpu.py -m gpu -v --maxfail=8 --timeout 150 --timeout-method thread > $out/tests_shard.log 2>&1
rc=$?; tail -12 $out/tests_shard.log | grep -E "passed|failed|FAILED|ERROR"; if [ $rc -ne 0 ]; then echo "pytest rc=$rc"; exit $rc; fi
for i in 1 2; do
  step timeout -k 10 200 python bench.py --mode sharded --shard-config C2 --steps 6 --warmup 2 > $out/sh_heads_$i.json 2> $out/sh_heads_$i.err
  step timeout -k 10 200 python bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-r6 > $out/single_$i.json 2> $out/single_$i.err
done
python -c "
import json
for f in ('sh_heads_1','single_1','sh_heads_2','single_2'):
    d=json.loads(open('$out/'+f+'.json').read().strip().split('\n')[-1]); print(f, round(d['ms_per_step'],2))"
for i in 1 2; do
  for v in proxy_old proxy; do
    step env ACE_LIB_PATH=$PWD/ab/libace_$v.so timeout -k 10 300 python bench.py --mode sharded --shard-config C3 --proxy 0/4 --steps 3 --warmup 1 > $out/${v}_c3_$i.json 2> $out/${v}_c3_$i.err
    step env ACE_LIB_PATH=$PWD/ab/libace_$v.so timeout -k 10 300 python bench.py --mode sharded --shard-config C4 --proxy 0/8 --steps 3 --warmup 1 > $out/${v}_c4_$i.json 2> $out/${v}_c4_$i.err
  done
done
python -c "
import json
for i in (1, 2):
  for v in ('proxy_old', 'proxy'):
    for c in ('c3', 'c4'):
      f='%s_%s_%d' % (v, c, i); d=json.loads(open('$out/'+f+'.json').read().strip().split('\n')[-1]); print(f, round(d['sharded']['ms_per_step'],2))"
