"""Builds libace_hip.so in-tree for gfx950 with hipcc (no JIT cache: the
.so travels to the GPU box with the source snapshot)."""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SOURCES = ["csrc/ace_pairs.hip", "csrc/ace_pairs_mm.hip", "csrc/ace_sweep.hip", "csrc/ace_util.hip",
           "csrc/ace_api.cpp", "csrc/ace_host.cpp", "csrc/ace_shard.cpp"]
HEADERS = ["csrc/ace_internal.h", "csrc/ace_common.h", "../include/ace_hip.h"]
OUT = os.path.join(HERE, "libace_hip.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
         "-Wno-unused-result", "-ldl"]


def needs_build():
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    return any(os.path.getmtime(os.path.join(HERE, s)) > t for s in SOURCES + HEADERS)


def build(force=False, verbose=True):
    if not force and not needs_build():
        return OUT
    cmd = [HIPCC] + FLAGS + ["-o", OUT] + [os.path.join(HERE, s) for s in SOURCES]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True, cwd=HERE)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
