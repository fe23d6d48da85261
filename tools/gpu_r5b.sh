# Round-5 session B: inverse-accuracy probe (r4 lib, blocked-pivot lib, old pivot),
# cross-assembly MFMA correctness (assembly / prediction / referee tests), the C2
# bench (predict leg), per-rank proxy timing of the sharded path, a C1 kernel trace.
# Any GPU step that fails, times out or faults ends the script (no later GPU step).
set -o pipefail
R=$GRAFT_REPO_ROOT
out=gpurun_out/r5b; mkdir -p $out
step() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
step timeout -k 10 300 python -u tools/inverse_probe.py gpurun_out/invp cur=ab/libace_cur.so new=additivecausalexpansion_amd/libace_hip.so pold=ab/libace_pold.so > $out/invp.log 2>&1
# test failures are results, not faults: keep going unless the runner itself died
timeout -k 10 400 python -u -m pytest tests/test_gpu.py tests/test_predict_gpu.py tests/test_referee_gpu.py -v --timeout 120 --timeout-method thread -k "assembly or pred or referee" > $out/tests.log 2>&1
rc=$?; tail -3 $out/tests.log; if [ $rc -gt 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
step timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-r6 > $out/bench_c2.json 2> $out/bench_c2.err
python -c "import json;d=json.load(open('$out/bench_c2.json'));print(d['ms_per_step'], d['predict'])"
step env ACE_LIB_PATH=$PWD/ab/libace_proxy.so timeout -k 10 300 python bench.py --mode sharded --shard-config C3 --proxy 0/4 --steps 3 --warmup 1 > $out/proxy_c3_r0of4.json 2> $out/proxy_c3.err
cut -c1-250 $out/proxy_c3_r0of4.json
step env ACE_LIB_PATH=$PWD/ab/libace_proxy.so timeout -k 10 300 python bench.py --mode sharded --shard-config C4 --proxy 0/8 --steps 3 --warmup 1 > $out/proxy_c4_r0of8.json 2> $out/proxy_c4.err
cut -c1-250 $out/proxy_c4_r0of8.json
cd /tmp && export TMPDIR=/tmp
step timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/$out/c1trace -o run -- python3 $R/bench.py --config C1 --steps 3 --warmup 2 --no-r6 --no-cpu-baseline > $R/$out/c1trace.log 2>&1
python3 $R/tools/shard_trace.py $R/$out/c1trace 25 > $R/$out/c1trace.txt; head -30 $R/$out/c1trace.txt
