# L2 (TCC) attribution of the bulk update launch: separate rocprofv3 --pmc
# passes (each within gfx950's 4 TCC slots) over a short C2 bench, then
# tools/pmc_counters.py.  $1 = output tag under gpurun_out/.
set -o pipefail
out=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
i=0
for cs in "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" "TCC_HIT TCC_MISS" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $cs --output-format csv -d $out/p$i -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-r6 > $out/p$i.log 2>&1 || { echo "pass $i ($cs) failed"; tail -5 $out/p$i.log; exit 1; }
done
python3 $GRAFT_REPO_ROOT/tools/pmc_counters.py $out/p1 $out/p2 $out/p3 > $out/pmc_tcc.json && \
python3 $GRAFT_REPO_ROOT/tools/pmc_traffic.py $out/p4 $out/p5 > $out/pmc_traffic.json && \
python3 -c "
import json
d = json.load(open('$out/pmc_tcc.json'))['kernels']
for k, v in d.items():
    print(k, {c: round(x['mean_per_launch'] / 1e6, 2) for c, x in v.items()}, 'M per launch')
"
