#!/bin/bash
# Build the working tree's library with extra compile flags into
# ab/libace_<tag>.so (A/B of compile-time variants): $1 = tag, rest = flags.
tag=$1; shift
mkdir -p /root/repo/ab
cd /root/repo/additivecausalexpansion_amd && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wno-unused-result -ldl "$@" \
  -o /root/repo/ab/libace_$tag.so $(ls csrc/*.hip csrc/*.cpp) && echo built ab/libace_$tag.so "$@"
