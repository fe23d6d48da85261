# Round-5 session AD: C1 records of the final tree -- rocprofv3 kernel stats of the C1 bench and
# the two PMC passes (FETCH_SIZE, WRITE_SIZE) at C1, so that a C1 bench line's roofline.traffic
# comes from its own configuration.
set -o pipefail
step() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
step bash tools/run_prof.sh r5ad/prof_c1 --config C1 --steps 20 --warmup 3 --no-r6
python3 tools/kernel_stats_split.py gpurun_out/r5ad/prof_c1 > gpurun_out/r5ad/kernel_stats_split_c1.csv
head -8 gpurun_out/r5ad/kernel_stats_split_c1.csv | cut -c1-160
CFG=C1 step bash tools/run_pmc.sh r5ad/pmc_c1 > /dev/null
head -20 gpurun_out/r5ad/pmc_c1/pmc_traffic.json
