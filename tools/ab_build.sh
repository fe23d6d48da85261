#!/bin/bash
# Build libace_hip.so from a git revision (default HEAD) into tools/libace_<tag>.so
# for in-call A/B timing against the working tree (ACE_LIB_PATH=...).
rev=${1:-HEAD}; tag=${2:-A}
d=$(mktemp -d /tmp/ab.XXXX)
git -C /root/repo archive $rev additivecausalexpansion_amd/csrc include | tar -x -C $d
cd $d/additivecausalexpansion_amd && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wno-unused-result -ldl \
  -o /root/repo/tools/libace_$tag.so $(ls csrc/*.hip csrc/*.cpp) && echo built tools/libace_$tag.so from $rev
rm -rf $d
