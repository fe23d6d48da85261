# Head / tail lookahead split (ACE_HEADS=1): bitwise tests, then C2 A/B
# against the group schedule under the given settings ($@, "" = default),
# then a kernel trace of the first setting.
set -o pipefail
mkdir -p gpurun_out/hd
python tools/prio_range.py
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "pair_steps or merged_cross_model" > gpurun_out/hd/tests.log 2>&1 || { tail -30 gpurun_out/hd/tests.log; exit 1; }
tail -2 gpurun_out/hd/tests.log
ROUNDS=${ROUNDS:-2} bash tools/ab_envs.sh "$@" || exit 1
NSHOW=3 bash tools/trace_group.sh hd "$1"
