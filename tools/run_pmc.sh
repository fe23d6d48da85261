# Two separate rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE) over a short bench
# (config ${CFG:-C2}); tools/pmc_traffic.py turns them into per-launch HBM bytes.
set -o pipefail
out=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/pmc_f -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config ${CFG:-C2} --steps 2 --warmup 1 --no-cpu-baseline --no-r6 > $out/pmc_f.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/pmc_w -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config ${CFG:-C2} --steps 2 --warmup 1 --no-cpu-baseline --no-r6 > $out/pmc_w.log 2>&1 && \
python3 $GRAFT_REPO_ROOT/tools/pmc_traffic.py $out/pmc_f $out/pmc_w ${CFG:-C2} > $out/pmc_traffic.json && cat $out/pmc_traffic.json
