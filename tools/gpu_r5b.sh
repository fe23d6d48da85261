# Round-5 session B: inverse-accuracy probe (r4 lib, blocked-pivot lib, old pivot),
# cross-assembly MFMA correctness (assembly / prediction tests) and the C2 bench
# (predict leg) with the new cross kernel.
set -o pipefail
out=gpurun_out/r5b; mkdir -p $out
timeout -k 10 300 python -u tools/inverse_probe.py gpurun_out/invp cur=ab/libace_cur.so new=additivecausalexpansion_amd/libace_hip.so pold=ab/libace_pold.so > $out/invp.log 2>&1 && \
timeout -k 10 400 python -u -m pytest tests/test_gpu.py tests/test_predict_gpu.py tests/test_referee_gpu.py -v --timeout 120 --timeout-method thread -k "assembly or pred or referee" > $out/tests.log 2>&1; tail -3 $out/tests.log; \
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-r6 > $out/bench_c2.json 2> $out/bench_c2.err && python -c "import json;d=json.load(open('$out/bench_c2.json'));print(d['ms_per_step'], d['predict'])"
