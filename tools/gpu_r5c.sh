# Round-5 session C: full GPU suite; bitwise check of the round-5 head-path load
# pipelines against the previous commit; same-box A/B (C2, C1) of previous commit /
# this tree / the tail path at normal priority; the 1-rank RCCL sharded C2 run (group
# schedule); per-rank proxies (C3 0/4, C4 0/8); rocprof kernel stats and PMC traffic of C2.
set -o pipefail
R=$GRAFT_REPO_ROOT
out=gpurun_out/r5c; mkdir -p $out
step() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=8 --timeout 120 --timeout-method thread > $out/tests.log 2>&1
rc=$?; tail -12 $out/tests.log | grep -E "passed|failed|FAILED|ERROR"; if [ $rc -gt 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
step timeout -k 10 200 python tools/cmp_libs.py ab/libace_head.so additivecausalexpansion_amd/libace_hip.so 4096 SE > $out/cmp.txt 2>&1
step timeout -k 10 200 python tools/cmp_libs.py ab/libace_head.so additivecausalexpansion_amd/libace_hip.so 16384 Matern32 >> $out/cmp.txt 2>&1
cat $out/cmp.txt
L=additivecausalexpansion_amd/libace_hip.so
ROUNDS=2 step timeout -k 10 600 bash tools/ab_libs.sh ab/libace_head.so $L ab/libace_s2n.so -- --no-r6 > $out/ab_c2.txt 2>&1; cat $out/ab_c2.txt
ROUNDS=2 step timeout -k 10 300 bash tools/ab_libs.sh ab/libace_head.so $L ab/libace_s2n.so -- --no-r6 --config C1 --steps 20 > $out/ab_c1.txt 2>&1; cat $out/ab_c1.txt
step env ACE_SYNC_TIMEOUT=150 timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr=127.0.0.1 --master-port=29533 bench.py --mode sharded --shard-config C2 --steps 6 --warmup 2 > $out/sharded_c2_rccl1.json 2> $out/sharded_c2_rccl1.err
python -c "import json;d=json.load(open('$out/sharded_c2_rccl1.json'));print('sharded C2 1-rank RCCL ms', d['ms_per_step'])"
step env ACE_LIB_PATH=$PWD/ab/libace_proxy.so timeout -k 10 300 python bench.py --mode sharded --shard-config C3 --proxy 0/4 --steps 3 --warmup 1 > $out/proxy_c3_r0of4.json 2> $out/proxy_c3.err
step env ACE_LIB_PATH=$PWD/ab/libace_proxy.so timeout -k 10 300 python bench.py --mode sharded --shard-config C4 --proxy 0/8 --steps 3 --warmup 1 > $out/proxy_c4_r0of8.json 2> $out/proxy_c4.err
python -c "import json;[print(f, json.load(open('$out/'+f))['sharded']['ms_per_step'], json.load(open('$out/'+f))['sharded']['rank0_phase_ms_per_step']) for f in ('proxy_c3_r0of4.json','proxy_c4_r0of8.json')]"
step bash tools/run_prof.sh r5c/prof --steps 5 --warmup 1 --no-r6
step bash tools/run_pmc.sh r5c/pmc > /dev/null
python3 tools/kernel_stats_split.py $out/prof > $out/kernel_stats_split.csv; head -12 $out/kernel_stats_split.csv; cat $out/pmc/pmc_traffic.json | head -30
