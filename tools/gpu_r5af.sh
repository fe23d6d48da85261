# Round-5 session AF: C2 with Z = 3 sweep steps per bulk launch (ACE_GROUP=3) against the
# default Z = 4 (env A/B of the committed tree).
set -o pipefail
out=gpurun_out/r5af; mkdir -p $out
step() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
ROUNDS=3 step timeout -k 10 700 bash tools/ab_envs.sh "" "ACE_GROUP=3" > $out/ab_c2.txt 2>&1; cat $out/ab_c2.txt
