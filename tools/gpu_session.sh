#!/bin/bash
# One GPU call of several bounded steps (each under its own timeout, chained
# with &&): $1 = tag, the rest = step names among
#   probe   tools/probe_mfma_f64 (fp64 MFMA layouts / rates), tools/probe_valu_rates
#   round   tools/run_round.sh (tests, smoke, bench, rocprof stats)
#   tests   the GPU test suite alone
#   bench   bench.py alone
#   tcc     tools/run_pmc_tcc.sh (L2 hit / miss, HBM traffic per launch)
#   repro   tools/repro_stall.sh on tools/libace_masked.so, then the default library
set -o pipefail
tag=$1; shift
mkdir -p gpurun_out/$tag
rc=0
for step in "$@"; do
  case $step in
    probe) timeout -k 10 120 ./tools/probe_mfma_f64 > gpurun_out/$tag/probe_mfma.txt 2>&1 && \
           timeout -k 10 120 ./tools/probe_valu_rates > gpurun_out/$tag/probe_valu.txt 2>&1; rc=$?
           tail -4 gpurun_out/$tag/probe_mfma.txt; cat gpurun_out/$tag/probe_valu.txt ;;
    round) bash tools/run_round.sh $tag; rc=$? ;;
    tests) timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --durations=20 --timeout 120 --timeout-method thread > gpurun_out/$tag/tests.log 2>&1; rc=$?; tail -3 gpurun_out/$tag/tests.log ;;
    bench) timeout -k 10 400 python bench.py --steps 10 --warmup 2 > gpurun_out/$tag/bench.json 2> gpurun_out/$tag/bench.err; rc=$?; cut -c1-600 gpurun_out/$tag/bench.json ;;
    repro) timeout -k 10 420 bash tools/repro_stall.sh tools/libace_masked.so 40 masked; rc=$?
           [ $rc -eq 0 ] && { timeout -k 10 200 bash tools/repro_stall.sh additivecausalexpansion_amd/libace_hip.so 10 default; rc=$?; } ;;
    tcc) bash tools/run_pmc_tcc.sh $tag/tcc; rc=$? ;;
    abgrad) bash tools/ab_grad.sh $tag tools/libace_tail.so tools/libace_tailexp.so; rc=$? ;;
    abnew) bash tools/ab_grad.sh $tag tools/libace_tail.so tools/libace_new.so; rc=$? ;;
    abstage) timeout -k 10 200 python tools/cmp_libs.py tools/libace_new.so tools/libace_stage.so 16384 Matern32 && \
             timeout -k 10 200 python tools/cmp_libs.py tools/libace_new.so tools/libace_stage.so 4096 SE && \
             { timeout -k 10 200 python tools/cmp_libs.py tools/libace_stage.so tools/libace_cur.so 16384 Matern32; \
               timeout -k 10 200 python tools/cmp_libs.py tools/libace_stage.so tools/libace_cur.so 4096 SE; true; } && \
             ROUNDS=3 bash tools/ab_libs.sh tools/libace_new.so tools/libace_stage.so tools/libace_cur.so -- --no-r6; rc=$? ;;
    abpersist) timeout -k 10 60 ./tools/probe_hwid > gpurun_out/$tag/probe_hwid.txt 2>&1; cat gpurun_out/$tag/probe_hwid.txt | tail -3
             timeout -k 10 200 python tools/cmp_libs.py tools/libace_new.so tools/libace_cur.so 16384 Matern32 && \
             CMP_ENV_B="ACE_ASM_PERSIST=1" timeout -k 10 200 python tools/cmp_libs.py tools/libace_cur.so tools/libace_cur.so 16384 Matern32 && \
             CMP_ENV_B="ACE_ASM_PERSIST=2" timeout -k 10 200 python tools/cmp_libs.py tools/libace_cur.so tools/libace_cur.so 4096 SE && \
             ROUNDS=3 bash tools/ab_envs.sh "" "ACE_ASM_PERSIST=1" "ACE_ASM_PERSIST=2"; rc=$? ;;
    trace) NSHOW=1 bash tools/trace_group.sh $tag/tg "" "ACE_ASM_PERSIST=1" > gpurun_out/$tag/timeline.txt 2>&1; rc=$?; head -c 6000 gpurun_out/$tag/timeline.txt ;;
    persist2) CMP_ENV_B="ACE_ASM_PERSIST=1" timeout -k 10 200 python tools/cmp_libs.py tools/libace_cur.so tools/libace_cur.so 16384 Matern32 && \
              CMP_ENV_B="ACE_ASM_PERSIST=2" timeout -k 10 200 python tools/cmp_libs.py tools/libace_cur.so tools/libace_cur.so 4096 SE && \
              NSHOW=1 bash tools/trace_group.sh $tag/tg "" "ACE_ASM_PERSIST=1" "ACE_ASM_PERSIST=2" > gpurun_out/$tag/timeline.txt 2>&1 && \
              ROUNDS=3 bash tools/ab_envs.sh "" "ACE_ASM_PERSIST=1" "ACE_ASM_PERSIST=2"; rc=$?; head -c 5000 gpurun_out/$tag/timeline.txt ;;
    persist3) CMP_ENV_B="ACE_ASM_PERSIST=1 ACE_ASM_TAIL=1 ACE_ASM_FILL=1" timeout -k 10 200 python tools/cmp_libs.py tools/libace_cur.so tools/libace_cur.so 16384 Matern32 && \
              CMP_ENV_B="ACE_ASM_PERSIST=2 ACE_ASM_FILL=1" timeout -k 10 200 python tools/cmp_libs.py tools/libace_cur.so tools/libace_cur.so 4096 SE && \
              NSHOW=1 bash tools/trace_group.sh $tag/tg "ACE_ASM_PERSIST=1 ACE_ASM_TAIL=1" "ACE_ASM_PERSIST=1 ACE_ASM_FILL=1" "ACE_ASM_PERSIST=1 ACE_ASM_TAIL=1 ACE_ASM_FILL=1" > gpurun_out/$tag/timeline.txt 2>&1 && \
              ROUNDS=3 bash tools/ab_envs.sh "" "ACE_ASM_PERSIST=1" "ACE_ASM_PERSIST=1 ACE_ASM_TAIL=1" "ACE_ASM_PERSIST=1 ACE_ASM_FILL=1" "ACE_ASM_PERSIST=1 ACE_ASM_TAIL=1 ACE_ASM_FILL=1" "ACE_ASM_PERSIST=2 ACE_ASM_FILL=1"; rc=$? ;;
    persist4) CMP_ENV_B="ACE_ASM_PERSIST=1 ACE_ASM_TAIL=2 ACE_ASM_FILL=1" timeout -k 10 200 python tools/cmp_libs.py tools/libace_cur.so tools/libace_cur.so 16384 Matern32 && \
              NSHOW=1 bash tools/trace_group.sh $tag/tg "ACE_ASM_PERSIST=1 ACE_ASM_TAIL=2" "ACE_ASM_PERSIST=1 ACE_ASM_TAIL=2 ACE_ASM_FILL=1" > gpurun_out/$tag/timeline.txt 2>&1 && \
              ROUNDS=3 bash tools/ab_envs.sh "" "ACE_ASM_PERSIST=1" "ACE_ASM_PERSIST=1 ACE_ASM_TAIL=1 ACE_ASM_FILL=1" "ACE_ASM_PERSIST=1 ACE_ASM_TAIL=2" "ACE_ASM_PERSIST=1 ACE_ASM_TAIL=2 ACE_ASM_FILL=1"; rc=$? ;;
    lead) ROUNDS=2 bash tools/ab_envs.sh "" "ACE_ASM_PERSIST=0" "ACE_ASM_TAIL=0 ACE_ASM_FILL=0" "ACE_ASM_TAIL=2"; rc=$? ;;
    evt) for i in 1 2 3; do for f in "" "--no-profile"; do timeout -k 5 100 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-r6 $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('[$f]', round(d['ms_per_step'],3))" || exit 1; done; done; rc=$? ;;
    cfgs) timeout -k 10 200 python bench.py --config C1 --steps 10 --warmup 2 --no-cpu-baseline --no-r6 > gpurun_out/$tag/bench_c1.json && \
          timeout -k 10 300 python bench.py --config C3 --steps 3 --warmup 1 --no-cpu-baseline --no-r6 > gpurun_out/$tag/bench_c3.json; rc=$?
          cut -c1-300 gpurun_out/$tag/bench_c1.json gpurun_out/$tag/bench_c3.json ;;
    wgt) ACE_LIB_PATH=tools/libace_wgt.so timeout -k 10 200 python tools/wg_timeline.py > gpurun_out/$tag/wgt.txt 2>&1; rc=$?; cat gpurun_out/$tag/wgt.txt | tail -30 ;;
    wgthot) ACE_LIB_PATH=tools/libace_wgthot.so timeout -k 10 200 python tools/wg_timeline.py > gpurun_out/$tag/wgthot.txt 2>&1; rc=$?; head -12 gpurun_out/$tag/wgthot.txt ;;
    hg) timeout -k 10 700 bash tools/host_gap.sh > gpurun_out/$tag/host_gap.txt 2>&1; rc=$?; head -60 gpurun_out/$tag/host_gap.txt ;;
    abbatch) timeout -k 10 200 python tools/cmp_libs.py additivecausalexpansion_amd/libace_hip.so tools/libace_cur.so 16384 Matern32 && \
             timeout -k 10 200 python tools/cmp_libs.py additivecausalexpansion_amd/libace_hip.so tools/libace_cur.so 4096 SE && \
             ROUNDS=3 bash tools/ab_libs.sh tools/libace_cur.so additivecausalexpansion_amd/libace_hip.so -- --no-r6; rc=$? ;;
    abg0) CMP_ENV_B="ACE_GATHER_PIV=1" timeout -k 10 200 python tools/cmp_libs.py additivecausalexpansion_amd/libace_hip.so additivecausalexpansion_amd/libace_hip.so 16384 Matern32 && \
          ROUNDS=3 bash tools/ab_envs.sh "" "ACE_GATHER_PIV=1" "ACE_HEADQ=0"; rc=$? ;;
    abprio) ROUNDS=3 bash tools/ab_envs.sh "" "ACE_MAIN_PRIO=0" "ACE_MAIN_PRIO=0 ACE_SIDE2_PRIO=2" "ACE_MAIN_PRIO=0 ACE_HEADQ=0"; rc=$? ;;
    abexp) timeout -k 10 200 python tools/cmp_libs.py tools/libace_cur.so tools/libace_exp256.so 16384 Matern32; \
           timeout -k 10 200 python tools/cmp_libs.py tools/libace_cur.so tools/libace_exp256.so 4096 SE; \
           ROUNDS=3 bash tools/ab_libs.sh tools/libace_cur.so tools/libace_exp256.so -- --no-r6; rc=$? ;;
    pmc) bash tools/run_pmc.sh $tag/pmc > /dev/null; rc=$?; head -c 3000 gpurun_out/$tag/pmc/pmc_traffic.json ;;
    sq) bash tools/run_sq.sh $tag/sq > /dev/null; rc=$?; cat gpurun_out/$tag/sq/sq.txt | head -80 ;;
    prof) bash tools/run_prof.sh $tag/prof --steps 5 --warmup 1 > /dev/null; rc=$? ;;
    *) echo "unknown step $step"; rc=2 ;;
  esac
  echo "[step $step rc=$rc]"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
