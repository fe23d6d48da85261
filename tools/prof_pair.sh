# rocprofv3 kernel stats of a short C2 bench under two env settings:
# $1 = tag, $2 = VAR=value for the second run
set -o pipefail
out=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p $out/a $out/b
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/a -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 4 --warmup 1 > $out/a/bench.log 2>&1 && \
env $2 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/b -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 4 --warmup 1 > $out/b/bench.log 2>&1
for d in a b; do echo "== $d"; f=$(find $out/$d -name "*kernel_stats.csv" | head -1); python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
for r in rows[:14]: print(r['Name'][:60].ljust(60), r['Calls'].rjust(6), '%10.1f' % (float(r['AverageNs'])/1e3), '%10.2f' % (float(r['TotalDurationNs'])/1e6))
"; done
