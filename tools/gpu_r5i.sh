# Round-5 check of the committed tree: full GPU suite, smoke, the default
# bench line (CPU baseline included), a C1 line, rocprof kernel stats and the
# PMC traffic passes of C2.
set -o pipefail
tag=${1:-r5i}
bash tools/run_round.sh $tag || exit $?
python3 tools/kernel_stats_split.py gpurun_out/$tag/prof > gpurun_out/$tag/kernel_stats_split.csv
timeout -k 10 200 python bench.py --config C1 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/$tag/bench_c1.json 2> gpurun_out/$tag/bench_c1.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/$tag/bench_c1.json'));print('C1', d['ms_per_step'])"
bash tools/run_pmc.sh $tag/pmc > /dev/null || exit $?
head -30 gpurun_out/$tag/pmc/pmc_traffic.json
