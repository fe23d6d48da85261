#!/bin/bash
# One GPU session (gpurun -- 'bash tools/session.sh TAG STEP...'): the named
# steps in order, each under its own time limit, stopping at the first step
# that fails (a GPU step that faults, aborts or times out ends the session).
# Output under gpurun_out/TAG.  Replaces the per-session scripts of round 5
# (tools/gpu_r5*.sh, in git history before round 6).
#
# Steps:
#   tests          pytest -m gpu (verbose, slowest tests listed), with the
#                  measured-error log (ACE_ERROR_LOG -> errors.jsonl)
#   tests:EXPR     the GPU tests selected by -k EXPR
#   smoke          __graft_entry__.smoke()
#   bench          bench.py (C2, CPU baseline included)
#   bench_c1       bench.py --config C1 (no CPU baseline)
#   prof           rocprofv3 --kernel-trace --stats of the C2 bench + the
#                  bulk-launch split (tools/kernel_stats_split.py)
#   pmc            the FETCH_SIZE / WRITE_SIZE passes (tools/run_pmc.sh, CFG=C1|C2)
#   sq             the SQ counter passes (tools/run_sq.sh)
#   shard          the sharded model at world 1 over RCCL (C2, --mode sharded)
#   ab:ENV1,ENV2   alternating C2 bench runs under two switch settings
#                  (tools/ab_envs.sh; ROUNDS=2)
set -o pipefail
tag=${1:?tag}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/$tag; mkdir -p $out
cd $R
run() {  # run LIMIT_S LOG cmd...: bounded, logged, stops the session on failure
  local lim=$1 log=$2; shift 2
  timeout -k 10 $lim "$@" > $log 2>&1; local rc=$?
  if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; tail -20 $log; exit $rc; fi
}
runj() {  # runj LIMIT_S JSON cmd...: as run, stdout (the bench line) to JSON, stderr beside it
  local lim=$1 js=$2; shift 2
  timeout -k 10 $lim "$@" > $js 2> ${js%.json}.err; local rc=$?
  if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; tail -20 ${js%.json}.err; exit $rc; fi
}
for step in "$@"; do
  echo "== $step"
  case $step in
    tests)
      rm -f $out/errors.jsonl
      ACE_ERROR_LOG=$out/errors.jsonl run 900 $out/tests.log python -u -m pytest tests -m gpu -v \
        --durations=20 --timeout 900 --timeout-method thread
      tail -1 $out/tests.log
      python3 tools/error_table.py $out/errors.jsonl > $out/error_table.txt && tail -3 $out/error_table.txt ;;
    tests:*)
      run 900 $out/tests_k.log python -u -m pytest tests -m gpu -v -k "${step#tests:}" --timeout 900 \
        --timeout-method thread
      tail -1 $out/tests_k.log ;;
    smoke)
      run 200 $out/smoke.log python -c "import __graft_entry__ as g; g.smoke()"; cat $out/smoke.log ;;
    bench)
      runj 400 $out/bench.json python bench.py --steps 10 --warmup 2
      cut -c1-400 $out/bench.json ;;
    bench_c1)
      runj 300 $out/bench_c1.json python bench.py --config C1 --steps 20 --warmup 3 --no-cpu-baseline
      cut -c1-300 $out/bench_c1.json ;;
    prof)
      bash tools/run_prof.sh $tag/prof --steps 5 --warmup 1 > /dev/null || exit 1
      python3 tools/kernel_stats_split.py $out/prof > $out/kernel_stats_split.csv && head -5 $out/kernel_stats_split.csv ;;
    pmc)
      bash tools/run_pmc.sh $tag/pmc > $out/pmc.log 2>&1 || { tail -5 $out/pmc.log; exit 1; }
      tail -12 $out/pmc.log ;;
    sq)
      bash tools/run_sq.sh $tag/sq > $out/sq.log 2>&1 || { tail -5 $out/sq.log; exit 1; }
      tail -30 $out/sq.log ;;
    shard)
      runj 300 $out/shard.json python bench.py --mode sharded --shard-config C2 --steps 6 --warmup 2
      cut -c1-400 $out/shard.json ;;
    ab:*)
      IFS=, read -r a b <<< "${step#ab:}"
      ROUNDS=${ROUNDS:-2} run 600 $out/ab.txt bash tools/ab_envs.sh "$a" "$b" -- --steps 8
      cat $out/ab.txt ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
