#!/bin/bash
# Gradient-kernel A/B (round 4): the GPU tests that exercise the gradient on
# the working tree, result differences against the previous build
# (ab/libace_base.so, tools/cmp_libs.py: max relative difference of two
# C2-shaped evaluations), and alternating C2 bench runs of the given builds.
# usage: bash tools/ab_grad.sh tag lib...
tag=$1; shift
out=gpurun_out/$tag; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu.py tests/test_fullsize_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "grad or model or fullsize_against_torch or golden or c2" > $out/tests.log 2>&1; rc=$?
tail -2 $out/tests.log; [ $rc -ne 0 ] && exit $rc
for lib in "$@"; do
  timeout -k 10 200 python tools/cmp_libs.py ab/libace_base.so $lib 16384 Matern32
  timeout -k 10 200 python tools/cmp_libs.py ab/libace_base.so $lib 4096 SE
done
ROUNDS=${ROUNDS:-3} bash tools/ab_libs.sh ab/libace_base.so "$@" -- --no-r6
