# GPU test run: build nothing here (the .so is prebuilt in-tree)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread "$@" > gpurun_out/tests.log 2>&1
rc=$?
tail -5 gpurun_out/tests.log
exit $rc
