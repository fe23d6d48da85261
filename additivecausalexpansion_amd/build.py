"""Builds libace_hip.so in-tree for gfx950 with hipcc (no JIT cache: the
.so travels to the GPU box with the source snapshot).  Each source is
compiled to its own object in parallel (no device code crosses a
translation unit), then linked; an object is rebuilt only when its source
or a shared header is newer."""
from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
SOURCES = ["csrc/ace_pairs.hip", "csrc/ace_pairs_mm.hip", "csrc/ace_sweep.hip", "csrc/ace_util.hip",
           "csrc/ace_symm.hip", "csrc/ace_api.cpp", "csrc/ace_host.cpp", "csrc/ace_shard.cpp",
           "csrc/ace_predict.cpp", "csrc/ace_dmat.cpp", "csrc/ace_train.hip"]
HEADERS = ["csrc/ace_internal.h", "csrc/ace_common.h", "csrc/ace_model.h", "../include/ace_hip.h"]
OUT = os.path.join(HERE, "libace_hip.so")
OBJDIR = os.path.join(HERE, "build")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CFLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Wno-unused-result"]
LDFLAGS = ["--offload-arch=gfx950", "-shared", "-ldl"]


def _sources():
    return [s for s in SOURCES if os.path.exists(os.path.join(HERE, s))]


def _obj(src):
    return os.path.join(OBJDIR, os.path.basename(src) + ".o")


def _mtime(p):
    return os.path.getmtime(p) if os.path.exists(p) else -1.0


def needs_build():
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    return any(_mtime(os.path.join(HERE, s)) > t for s in _sources() + HEADERS)


def build(force=False, verbose=True):
    if not force and not needs_build():
        return OUT
    os.makedirs(OBJDIR, exist_ok=True)
    hdr = max(_mtime(os.path.join(HERE, h)) for h in HEADERS)
    todo = [s for s in _sources()
            if force or _mtime(_obj(s)) < max(_mtime(os.path.join(HERE, s)), hdr)]

    def compile_one(src):
        cmd = [HIPCC] + CFLAGS + ["-c", os.path.join(HERE, src), "-o", _obj(src)]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, cwd=HERE, capture_output=True, text=True)
        return src, r

    jobs = max(1, min(len(todo), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4))))
    with ThreadPoolExecutor(jobs) as ex:
        for src, r in ex.map(compile_one, todo):
            if r.returncode != 0:
                sys.stderr.write(r.stdout + r.stderr)
                raise subprocess.CalledProcessError(r.returncode, src)
    cmd = [HIPCC] + LDFLAGS + ["-o", OUT] + [_obj(s) for s in _sources()]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True, cwd=HERE)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
