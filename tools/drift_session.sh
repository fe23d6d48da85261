set -o pipefail
mkdir -p gpurun_out/drift
timeout -k 10 400 python -u tools/drift_probe.py gpurun_out/drift cur=ab/libace_cur.so r3=ab/libace_r3.so t4off=ab/libace_t4off.so aexp0=ab/libace_aexp0.so > gpurun_out/drift/probe.log 2>&1
