# Sharded tests + the 1-rank A/B + single/sharded traces + host-gap traces.
bash tools/prof_shard.sh > gpurun_out/rs_prof_shard.log 2>&1 || { tail -40 gpurun_out/rs_prof_shard.log; exit 1; }
cat gpurun_out/rs_prof_shard.log
NGAPS=8 bash tools/trace_pair.sh || exit 1
bash tools/host_gap.sh
