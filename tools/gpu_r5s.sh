# Round-5 session S: host-side time per evaluation at C1 and C2 (ab/libace_ht.so, -DACE_HOST_TRACE:
# time outside the call, enqueue, wait), to tell the host's enqueue from the device's span.
set -o pipefail
out=gpurun_out/r5s; mkdir -p $out
step() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
export ACE_LIB_PATH=ab/libace_ht.so
step timeout -k 10 200 python bench.py --config C1 --steps 20 --warmup 3 --no-r6 --no-cpu-baseline > $out/c1.json 2> $out/c1_host.txt
tail -8 $out/c1_host.txt; cat $out/c1.json | cut -c1-300
step timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-r6 --no-cpu-baseline > $out/c2.json 2> $out/c2_host.txt
tail -4 $out/c2_host.txt
