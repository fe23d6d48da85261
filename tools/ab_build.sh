#!/bin/bash
# Build libace_hip.so from a git revision (default HEAD) into ab/libace_<tag>.so (git-ignored; travels with gpurun)
# for in-call A/B timing against the working tree (ACE_LIB_PATH=...).
rev=${1:-HEAD}; tag=${2:-A}
mkdir -p /root/repo/ab
d=$(mktemp -d /tmp/ab.XXXX)
git -C /root/repo archive $rev additivecausalexpansion_amd/csrc include | tar -x -C $d
cd $d/additivecausalexpansion_amd && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wno-unused-result -ldl \
  -o /root/repo/ab/libace_$tag.so $(ls csrc/*.hip csrc/*.cpp) && echo built ab/libace_$tag.so from $rev
rm -rf $d
