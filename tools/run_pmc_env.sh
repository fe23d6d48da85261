# PMC traffic (two separate rocprofv3 passes) of a short C2 bench under an
# environment setting: $1 = tag, $2 = VAR=value (or "")
set -o pipefail
out=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  env $2 timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $out/pmc_$c -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $out/pmc_$c.log 2>&1 || exit 1
done
python3 $GRAFT_REPO_ROOT/tools/pmc_traffic.py $out/pmc_FETCH_SIZE $out/pmc_WRITE_SIZE > $out/pmc_traffic.json && python3 -c "import json; d=json.load(open('$out/pmc_traffic.json'))['kernels']['k_update_pair_bulk']; print('$2', round(d['traffic']/1e9,3), 'GB per bulk launch')"
