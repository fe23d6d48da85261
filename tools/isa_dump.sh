#!/bin/bash
# Device ISA of the gfx950 code objects of the HIP sources, for checking that
# a source change leaves the machine code unchanged (e.g. removing a
# compile-time A/B switch at its default):  tools/isa_dump.sh OUTDIR
# then `diff -r` two OUTDIRs.
set -e
out=${1:?outdir}; mkdir -p $out
B=/opt/rocm/lib/llvm/bin
for f in additivecausalexpansion_amd/csrc/*.hip; do
  b=$(basename $f .hip)
  ( /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC --cuda-device-only -c $f -o $out/$b.bundle
    $B/clang-offload-bundler --unbundle --type=o --input=$out/$b.bundle \
      --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$out/$b.co
    $B/llvm-objdump -d --no-show-raw-insn $out/$b.co | grep -v "file format" > $out/$b.s
    rm -f $out/$b.bundle ) &
done
wait
wc -l $out/*.s | tail -1
