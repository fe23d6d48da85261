# Round-5 session A: numeric-drift probe (frozen libs), blocked-pivot correctness
# (sweep tests first), full GPU suite, C1/C2 bench with the old pivot A/B.
set -o pipefail
out=gpurun_out/r5a; mkdir -p $out
timeout -k 10 400 python -u tools/drift_probe.py gpurun_out/drift cur=ab/libace_cur.so r3=ab/libace_r3.so t4off=ab/libace_t4off.so aexp0=ab/libace_aexp0.so > $out/drift.log 2>&1 && \
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -k "invkernel or sweep or gather_pivot or split_panel or golden" > $out/sweep_tests.log 2>&1 && tail -2 $out/sweep_tests.log && \
timeout -k 10 200 python bench.py --config C1 --steps 20 --warmup 3 --no-cpu-baseline --no-r6 > $out/bench_c1.json 2> $out/bench_c1.err && cut -c1-300 $out/bench_c1.json && \
ACE_LIB_PATH=$PWD/ab/libace_pold.so timeout -k 10 200 python bench.py --config C1 --steps 20 --warmup 3 --no-cpu-baseline --no-r6 > $out/bench_c1_pold.json 2> $out/bench_c1_pold.err && cut -c1-300 $out/bench_c1_pold.json && \
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-r6 > $out/bench_c2.json 2> $out/bench_c2.err && cut -c1-300 $out/bench_c2.json && \
ACE_LIB_PATH=$PWD/ab/libace_pold.so timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-r6 > $out/bench_c2_pold.json 2> $out/bench_c2_pold.err && cut -c1-300 $out/bench_c2_pold.json && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/tests.log 2>&1; tail -3 $out/tests.log
