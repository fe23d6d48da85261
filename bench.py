#!/usr/bin/env python3
"""Benchmark: log-marg-lik + gradient evaluations per second (BASELINE.json
`metric`) on the C2 configuration (n=16384, d=20, Matern32, ns basis B=10,
fp64) -- the largest configuration in BASELINE.json that fits one GPU.

A step is one `para_update` of the reference (R/kernel_SE_R6.R:40-62): the
device-resident model assembles the reduced kernel, inverts A = K + e^s I by
the MFMA Gauss-Jordan sweep (log det from its pivots) and computes every
gradient and both statistics; the host then takes the Nadam step with
norm clipping and the mu overwrite, exactly like the R6 class.  Inputs are
resident in HBM before the timed region.

Multi-GPU (torchrun, one process per GPU):
  * headline `value`: independent C2 replicas, one per GPU (per-GPU work
    fixed, "weak"): value = all ranks' evals / max-over-ranks time.  One C2
    evaluation fits a GPU, so replicas are the highest-throughput way to
    spend N GPUs on the n=16384 metric.
  * `sharded` leg (N > 1, after the replicas): ONE evaluation spread over
    all N GPUs -- A block-column-sharded, RCCL panel broadcast + all-gather
    per sweep step -- on the BASELINE config for that GPU
    count (C3 n=32768 at 4, C4 n=65536 at 8, C2-shaped n = 16384 N^(1/3)
    otherwise), with the weak-scaling efficiency of SURVEY §8d,
    E(N) = [n_N^3 / t_N / N] / [16384^3 / t_1], t_1 = this run's C2 step.
    A watchdog bounds it; the headline line is printed regardless, and a
    failed or timed-out leg then ends the run with exit status 3.
  * `--mode sharded`: the sharded leg alone (also at N = 1, where it runs the
    RCCL code path with one rank).

`--gpus N` is the world size.  Without a launcher (WORLD_SIZE unset) and
N > 1, bench.py starts `torch.distributed.run --nproc-per-node N` on itself as
a child process and exits with its status; under a launcher, WORLD_SIZE must
equal N (else exit 2).  `--launch-check` only rendezvouses and max-reduces.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--config C2]
                       [--mode auto|replicas|sharded] [--shard-config C4]
                       [--launch-check]
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "log-marg-lik+grad evals/sec at n=16384,d=20; Cholesky GF/s vs MFMA peak"
# MI355X dense fp64 matrix peak (AMD spec: 78.6 TFLOP/s fp64 vector and matrix;
# MI355X_MICROARCH.md lists no fp64 row, so the spec value is used).
FP64_MFMA_PEAK_TFLOPS = 78.6
HBM_PEAK_GBS = 8000.0
N1 = 16384  # C2


def _dist_init():
    # every launch path (self-launch child, external torchrun, --mode sharded):
    # RCCL shares buffers across processes by dmabuf IPC, which this host
    # driver requires; the HSA runtime reads the switch when HIP first
    # initialises, i.e. after this line
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world == 1 and "RANK" not in os.environ:
        return None, rank, world, local
    # torch first: its HIP runtime / RCCL are then the process-wide ones and
    # libace_hip.so binds to them by soname
    import torch
    import torch.distributed as dist
    backend = "nccl" if torch.cuda.is_available() else "gloo"
    if backend == "nccl":
        torch.cuda.set_device(local)
    dist.init_process_group(backend=backend)
    return dist, rank, world, local


def _barrier_sync(dist):
    if dist is not None:
        import torch
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        dist.barrier()


def _allreduce_max(dist, x):
    if dist is None:
        return x
    import torch
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def _newest_first_last(files):
    """Sort rNN_vMM_* profile files by (round, version) numerically."""
    import re
    return sorted(files, key=lambda f: [int(x) for x in re.findall(r"\d+", os.path.basename(f))])


def _pmc_files(config):
    """Committed PMC summaries (profiles/rNN_*pmc_traffic.json, oldest first)
    recorded at `config` (records without the key are the C2 runs of earlier
    rounds)."""
    import glob
    out = []
    for f in _newest_first_last(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_traffic.json"))):
        try:
            if json.load(open(f)).get("config", "C2") == config:
                out.append(f)
        except (ValueError, OSError):
            pass
    return out


def pmc_traffic(kernel="k_update", config="C2"):
    """HBM bytes per launch of `kernel` from the newest committed PMC summary
    of THIS configuration (profiles/rNN_pmc_traffic.json, written by
    tools/pmc_traffic.py from two separate rocprofv3 --pmc passes of this
    bench).  None when no record of the configuration exists."""
    files = _pmc_files(config)
    if not files:
        return None, None
    try:
        d = json.load(open(files[-1]))
        ks = d["kernels"]
        name = next((k for k in ks if k == kernel or k.startswith(kernel + "<")), None)
        return (ks[name]["traffic"] if name else None), os.path.relpath(files[-1], ROOT)
    except (KeyError, ValueError, OSError):
        return None, None


def rocprof_bulk_avg(config="C2"):
    """Average duration (ms) of the bulk update launch (k_update_multi; older
    summaries: k_update_pair) in the newest
    committed rocprofv3 kernel-trace summary (profiles/rNN_vMM_kernel_stats_split.csv,
    tools/kernel_stats_split.py: the bulk launches on their own line), for the
    cross-check against this run's HIP-event average."""
    import csv
    import glob
    if config != "C2":  # the committed summaries are of the C2 bench
        return None, None
    files = _newest_first_last(glob.glob(os.path.join(ROOT, "profiles", "r*_kernel_stats_split.csv")))
    if not files:
        return None, None
    try:
        for row in csv.DictReader(open(files[-1])):
            if row["Name"] in ("ace::k_update_multi[bulk]", "ace::k_update_pair[bulk]"):
                return float(row["AverageNs"]) / 1e6, os.path.relpath(files[-1], ROOT)
    except (KeyError, ValueError, OSError):
        pass
    return None, None


def rocprof_assembly_ms(config="C2"):
    """Per-evaluation kernel time of the assembly from the newest committed
    rocprofv3 summary: every k_asm_mm / k_asm_mm_q launch (the persistent
    queue's main launch AND the filler that takes its last tiles on the tail
    stream after group 0's lookahead), over the evaluations of that run (one
    k_aug_init per evaluation).  The HIP-event interval `assembly_kernel`
    brackets the main stream's launches only."""
    import csv
    import glob
    if config != "C2":
        return None, None
    files = _newest_first_last(glob.glob(os.path.join(ROOT, "profiles", "r*_kernel_stats_split.csv")))
    if not files:
        return None, None
    try:
        asm_ns, evals = 0.0, 0
        for row in csv.DictReader(open(files[-1])):
            name = row["Name"]
            if "k_asm_mm<" in name or "k_asm_mm_q<" in name:
                asm_ns += float(row["TotalDurationNs"])
            elif "k_aug_init(" in name:
                evals += int(row["Calls"])
        if evals == 0 or asm_ns == 0.0:
            return None, None
        return asm_ns / evals / 1e6, os.path.relpath(files[-1], ROOT)
    except (KeyError, ValueError, OSError):
        return None, None


def pair_hbm_gbs(asm_ms, grad_ms, config="C2"):
    """HBM GB/s of the fused assembly and gradient phases (SURVEY §8d asks for
    them beside their VALU/MFMA rates): PMC bytes per eval from the newest
    profiles/rNN_pmc_traffic.json (the assembly and gradient launches of
    each eval) over this run's phase times."""
    files = _pmc_files(config)
    if not files:
        return None
    try:
        ks = json.load(open(files[-1]))["kernels"]
        g = ks["k_grad_mm"]
        evals = g["launches"] / 2  # diagonal + strictly-lower gradient launch per eval
        # the assembly: its plain-grid parts (k_asm_mm) and, since round 4, the
        # persistent queue launches (k_asm_mm_q: main + filler)
        asm_b = sum(ks[k]["traffic"] * ks[k]["launches"] for k in ("k_asm_mm", "k_asm_mm_q")
                    if k in ks) / evals
        grad_b = g["traffic"] * g["launches"] / evals
    except (KeyError, ValueError, OSError, ZeroDivisionError):
        return None
    return {"assembly": asm_b / (asm_ms * 1e-3) / 1e9 if asm_ms else None,
            "gradient": grad_b / (grad_ms * 1e-3) / 1e9 if grad_ms else None,
            "bytes_per_eval": {"assembly": asm_b, "gradient": grad_b},
            "source": os.path.relpath(files[-1], ROOT)}


def cpu_baseline(cfg, timeout=240):
    """Rank 0 / N=1 only: the oracle leg in a subprocess (bounded)."""
    from additivecausalexpansion_amd.synthetic import CONFIGS
    n, p, B, kernel = CONFIGS[cfg]
    import glob
    fits = _newest_first_last(glob.glob(os.path.join(ROOT, "profiles", "r*_cpu_baseline.json")))
    cmd = [sys.executable, os.path.join(ROOT, "oracle", "cpu_baseline.py"), "--n", str(n),
           "--p", str(p), "--B", str(B), "--kernel", kernel, "--sample-n", "2048"]
    if fits:  # extrapolate with the measured exponents (oracle/cpu_scaling.py)
        cmd += ["--fit", fits[-1]]
    try:
        out = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, check=True)
        d = json.loads(out.stdout.strip().splitlines()[-1])
        return {k: d[k] for k in ("value", "unit", "cores", "host_nproc", "kind", "seconds_per_eval", "sample",
                          "measured_fit")
                if k in d}
    except Exception as e:  # the baseline is reported, never required
        return {"value": None, "unit": "evals/s", "cores": None, "kind": "port",
                "sample": f"failed: {type(e).__name__}: {e}"[:300]}


def shard_config(world, name=None):
    """(label, n, p, B, kernel) of the sharded leg for `world` GPUs."""
    from additivecausalexpansion_amd.synthetic import CONFIGS
    if name:
        return (name,) + tuple(CONFIGS[name])
    if world == 8:
        return ("C4",) + tuple(CONFIGS["C4"])
    if world == 4:
        return ("C3",) + tuple(CONFIGS["C3"])
    if world == 1:
        return ("C2",) + tuple(CONFIGS["C2"])
    n = int(round(N1 * world ** (1.0 / 3.0) / 256.0)) * 256
    return (f"C2-shape n={n}", n, 20, 10, "Matern32")


EXIT_SHARDED_FAILED = 3


def run_guarded(line, fn, timeout):
    """Runs the sharded leg fn() under a watchdog.  Returns (result, failed):
    an exception gives ({"error": ...}, True) and the caller prints the
    headline line, then exits EXIT_SHARDED_FAILED.  A leg still running
    after `timeout` s (a hung collective) prints the headline line with the
    error (rank 0) and ends the process at once with EXIT_SHARDED_FAILED:
    the line is never lost and the hang always shows in the exit status."""
    def watchdog():
        if line is not None:
            line["sharded"] = {"error": f"timed out after {timeout:.0f} s"}
            print(json.dumps(line), flush=True)
        sys.stderr.write(f"bench: sharded leg timed out after {timeout:.0f} s\n")
        sys.stderr.flush()
        os._exit(EXIT_SHARDED_FAILED)
    timer = threading.Timer(timeout, watchdog)
    timer.daemon = True
    timer.start()
    try:
        return fn(), False
    except Exception as e:  # the headline line is still printed by the caller
        return {"error": f"{type(e).__name__}: {e}"[:300]}, True
    finally:
        timer.cancel()


def make_step(kernel, p, B, theta, std_y, ctx, y, X, Z, model=None):
    import additivecausalexpansion_amd as ace
    Kc = ace.KernelClass_Matern32_R6 if kernel == "Matern32" else ace.KernelClass_SE_R6
    k = Kc(p, B, theta, std_y, ctx=ctx)
    opt = ace.set_optimizer("Nadam", k, 0.01, 0.0, 0.9, 0.999, True, 1.0)
    if model is None:
        model = k._ensure_model(y, X, Z)  # uploads X, Z, y once (resident in HBM)
    else:
        k.use_model(model, y, X, Z)
    state = {"it": 0}

    # ACE_BENCH_DIAG=1: timing of deliberately broken diagnostic builds
    # (tools/build_variant.sh -DACE_DIAG_SKIP=...): a non-finite gradient
    # keeps the parameters instead of ending the run
    diag = os.environ.get("ACE_BENCH_DIAG") == "1"
    theta0 = k.parameters.copy()

    def step():
        state["it"] += 1
        if not diag:
            return k.para_update(state["it"], y, X, Z, opt, verbose=False)
        try:
            return k.para_update(state["it"], y, X, Z, opt, verbose=False)
        except ace.AceError:
            k.parameters = theta0.copy()
            return [float("nan"), float("nan")]
    step.kernel_object = k
    return step, model


def timed_steps(dist, step, steps, warmup, model, profile=True):
    for _ in range(warmup):
        step()
    model.profile(profile)
    _barrier_sync(dist)
    t0 = time.perf_counter()
    stats = None
    for _ in range(steps):
        stats = step()
    _barrier_sync(dist)
    dt = time.perf_counter() - t0
    return _allreduce_max(dist, dt), stats


def predict_leg(k, model, p, B, nx=4096, reps=3):
    """Device prediction with the fit's resident inverse (Q6: the inverse of
    the last para_update, kernels at the current theta): pred_cpp and
    pred_marginal_cpp + ATE/ATT/ATU at nx test points against the n training
    points (R/kernel_SE_R6.R:75-97, src/pred_cpp.cpp:8-126).  Each call
    uploads X2 / Z2 (nx x (p + B - 1) doubles) and returns nx-long vectors
    over PCIe; the n x nx cross kernel and the A^-1 products stay in HBM."""
    import numpy as np
    from additivecausalexpansion_amd.synthetic import make_problem
    _, X2, Z2, _, _ = make_problem(nx, p, B, seed=77)
    dZ2 = np.asfortranarray(0.5 * Z2)
    zx = (np.arange(nx) % 3 == 0).astype(float)
    out = {"nx": nx, "n_train": model.n, "reps": reps,
           "note": "wall time per call incl. X2/Z2 upload and result download (small)"}
    calls = {
        "predict": lambda: model.predict(k.parameters, X2, Z2, 0.1, 1.3),
        "predict_marginal_ate": lambda: model.predict_marginal(k.parameters, X2, dZ2, zx, 1.3,
                                                               0.7, True),
    }
    for name, fn in calls.items():
        fn()  # warm (kernel tables, scratch)
        t0 = time.perf_counter()
        for _ in range(reps):
            r = fn()
        ms = (time.perf_counter() - t0) / reps * 1e3
        out[name] = {"ms": ms, "points_per_s": nx / (ms * 1e-3),
                     "finite": bool(np.all(np.isfinite(r["map"])) and np.all(np.isfinite(r["var"])))}
    return out


def r6_leg(kernel, p, B, theta, std_y, ctx, y, X, Z, iters=5, warmup=2):
    """The drop-in rate: the reference's UNCHANGED R6 para_update
    (R/kernel_SE_R6.R:40-62, R/kernel_Matern32_R6.R:39-60) over the .Call
    surface on device handles (r6.py, the sequence the R shim serves):
    kernmat_*_symmetric_cpp -> invkernel_cpp -> [mu_solution_cpp] ->
    grad_*_cpp -> Nadam -> mu_solution_cpp, per iteration.  Same data and
    theta as the headline steps; wall time per para_update.  The first two
    iterations allocate the two sweep buffers the loop then alternates
    between (a freed inverse handle's buffers are reused; in R the handles
    are freed by the collector): `ms_per_eval` is the median
    of the later iterations, `ms_first_two` what the allocating ones took."""
    import numpy as np
    from additivecausalexpansion_amd import set_optimizer
    from additivecausalexpansion_amd.r6 import R6KernelMatern32, R6KernelSE
    Kc = R6KernelMatern32 if kernel == "Matern32" else R6KernelSE
    k = Kc(p, B, theta, std_y, ctx=ctx)
    opt = set_optimizer("Nadam", k, 0.01, 0.0, 0.9, 0.999, True, 1.0)
    times = []
    st = None
    for it in range(1, warmup + iters + 1):
        t0 = time.perf_counter()
        st = k.para_update(it, y, X, Z, opt, verbose=False)
        times.append((time.perf_counter() - t0) * 1e3)
    ms = float(np.median(times[warmup:]))
    out = {"ms_per_eval": ms, "evals_per_s": 1e3 / ms, "iters": iters, "warmup": warmup,
           "ms_each": [round(t, 3) for t in times], "ms_first_two": times[:2],
           "last_stats": [float(st[0]), float(st[1])], "finite": bool(np.all(np.isfinite(st))),
           "path": "r6.py: kernmat_sym_dev -> invkernel_dev -> mu_solution_dev -> grad_dev "
                   "(virtual Kfull / elements, resident inverse)"}
    del k
    return out


def run_sharded(dist, rank, world, ctx, steps, warmup, name=None, proxy=False):
    """One evaluation over all ranks (block-column-sharded model, RCCL).
    proxy: rank `rank` of `world` alone in this process with the
    -DACE_DIAG_SHARD_PROXY library (tools/build_variant.sh): collectives are
    same-size device copies, results wrong, the rank's per-step time right."""
    import additivecausalexpansion_amd as ace
    from additivecausalexpansion_amd.synthetic import make_problem
    label, n, p, B, kernel = shard_config(world, name)
    uid = ace.comm_unique_id() if rank == 0 and not proxy else None
    if dist is not None:
        box = [uid]
        dist.broadcast_object_list(box, src=0)
        uid = box[0]
    y, X, Z, theta, std_y = make_problem(n, p, B, seed=2000)  # same data on every rank
    model = ace.DeviceModel(kernel, n, p, B, ctx=ctx, world=world, rank=rank, unique_id=uid,
                            sharded=True)
    step, model = make_step(kernel, p, B, theta, std_y, ctx, y, X, Z, model=model)
    dt, stats = timed_steps(dist, step, steps, warmup, model)
    upd_ms, upd_n, upd_work = model.kernel_time(0)
    asm_ms = model.kernel_time(1)[0]
    grad_ms = model.kernel_time(2)[0]
    model.profile(False)
    ms = dt / steps * 1e3
    out = {
        "config": label, "n": n, "p": p, "B": B, "kernel": kernel, "n_gpus": world,
        "parallelism": f"block-column shard x{world} (NB=256 cyclic), RCCL bcast+allgather/step",
        "steps": steps, "warmup": warmup, "ms_per_step": ms, "evals_per_s": 1e3 / ms,
        "dense_tflops_total": n ** 3 / (ms * 1e-3) / 1e12,
        "dense_tflops_per_gpu": n ** 3 / (ms * 1e-3) / 1e12 / world,
        "rank0_update_kernel_tflops": (upd_work / (upd_ms * 1e-3) / 1e12) if upd_ms else None,
        "rank0_phase_ms_per_step": {"update_kernel": upd_ms / steps, "assembly_kernel":
                                    asm_ms / steps, "gradient_kernel": grad_ms / steps},
        "last_stats": [float(stats[0]), float(stats[1])] if stats is not None else None,
    }
    model.close()
    return out


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def self_launch(a, argv):
    """`--gpus N > 1` without a launcher: start N ranks with
    torch.distributed.run as a CHILD process (never exec: nothing here has
    touched HIP yet, but the child must own the GPUs, not this process).
    The ranks inherit stdout, so rank 0's JSON line is the one line printed;
    the child's exit status is returned."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={a.gpus}", "--master-addr=127.0.0.1",
           f"--master-port={_free_port()}", os.path.abspath(__file__)] + list(argv)
    proc = subprocess.Popen(cmd, env=dict(os.environ))  # each rank: _dist_init's environment
    try:
        return proc.wait()
    except KeyboardInterrupt:
        proc.terminate()
        return proc.wait()


def launch_check(dist, rank, world):
    """--launch-check: the rendezvous and the max-over-ranks reduction only
    (no GPU work): rank 0 prints one line with the world size it saw."""
    got = _allreduce_max(dist, float(rank))
    if rank == 0:
        print(json.dumps({"launch_check": True, "n_gpus": world, "max_rank": int(got),
                          "backend": dist.get_backend() if dist is not None else None}), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="C2")
    ap.add_argument("--mode", default="auto", choices=["auto", "replicas", "sharded"])
    ap.add_argument("--shard-config", default=None)
    ap.add_argument("--shard-steps", type=int, default=2)
    ap.add_argument("--shard-timeout", type=float, default=240.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-r6", action="store_true", help="skip the unchanged-R6 drop-in leg")
    ap.add_argument("--no-profile", action="store_true",
                    help="diagnostic: no per-launch HIP events (no roofline / phase times)")
    ap.add_argument("--proxy", type=str, default=None, metavar="R/G",
                    help="diagnostic (--mode sharded, -DACE_DIAG_SHARD_PROXY library): time rank R "
                         "of a G-rank sharded evaluation alone on this GPU")
    ap.add_argument("--launch-check", action="store_true",
                    help="only rendezvous and max-reduce over the ranks (launcher test)")
    a = ap.parse_args()

    # --gpus N is the world size: a bare `bench.py --gpus N` launches N ranks
    # itself; under a launcher the two must agree
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and a.gpus > 1:
        sys.exit(self_launch(a, sys.argv[1:]))
    if env_world is not None and int(env_world) != a.gpus:
        sys.stderr.write(f"bench: --gpus {a.gpus} but WORLD_SIZE={env_world} "
                         "(the launcher's rank count must equal --gpus)\n")
        sys.exit(2)

    dist, rank, world, local = _dist_init()
    if a.launch_check:
        launch_check(dist, rank, world)
        return
    import additivecausalexpansion_amd as ace
    from additivecausalexpansion_amd.synthetic import CONFIGS, make_problem
    ctx = ace.Context(local)

    if a.mode == "sharded":
        if a.proxy:
            os.environ["ACE_BENCH_DIAG"] = "1"  # the proxy's gradients are not finite
            pr, pg = (int(x) for x in a.proxy.split("/"))
            sh = run_sharded(None, pr, pg, ctx, a.steps, a.warmup, a.shard_config, proxy=True)
            sh["proxy"] = {"rank": pr, "world": pg,
                           "note": "one rank alone, collectives replaced by same-size device copies"}
        else:
            sh = run_sharded(dist, rank, world, ctx, a.steps, a.warmup, a.shard_config)
        if rank == 0:
            line = {"metric": METRIC, "value": sh["evals_per_s"], "unit": "evals/s",
                    "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
                    "ms_per_step": sh["ms_per_step"], "higher_is_better": True,
                    "scaling": "weak", "vs_baseline": None, "dtype": "f64",
                    "data": "synthetic (seeded SURVEY.md §8d generator)",
                    "config": {"workload": f"{sh['config']} sharded para_update",
                               **{k: sh[k] for k in ("n", "p", "B", "kernel", "parallelism")}},
                    "sharded": sh}
            print(json.dumps(line), flush=True)
        if dist is not None:
            dist.barrier()
            dist.destroy_process_group()
        return

    n, p, B, kernel = CONFIGS[a.config]
    y, X, Z, theta, std_y = make_problem(n, p, B, seed=1000 + rank)
    step, model = make_step(kernel, p, B, theta, std_y, ctx, y, X, Z)
    dt_max, stats = timed_steps(dist, step, a.steps, a.warmup, model, not a.no_profile)
    upd_ms, upd_n, upd_work = model.kernel_time(0)
    asm_ms, _, asm_work = model.kernel_time(1)
    grad_ms, _, grad_work = model.kernel_time(2)
    sweep_ms, sweep_n, sweep_work = model.kernel_time(3)
    lead_ms, lead_n, _ = model.kernel_time(4)
    span_ms, span_n, _ = model.kernel_time(5)
    model.profile(False)
    pred = predict_leg(step.kernel_object, model, p, B) if rank == 0 else None
    r6 = None
    if rank == 0 and world == 1 and not a.no_r6:
        try:
            r6 = r6_leg(kernel, p, B, theta, std_y, ctx, y, X, Z)
            r6["vs_fused_ms_ratio"] = r6["ms_per_eval"] / (dt_max / a.steps * 1e3)
        except Exception as e:  # reported, never fatal for the headline
            r6 = {"error": f"{type(e).__name__}: {e}"[:300]}

    line = None
    if rank == 0:
        traffic, traffic_src = pmc_traffic("k_update_multi_bulk", a.config)
        if traffic is None:  # a summary from before the multi-panel kernel
            traffic, traffic_src = pmc_traffic("k_update_pair_bulk", a.config)
        rp_ms, rp_src = rocprof_bulk_avg(a.config)
        asm_rp_ms, asm_rp_src = rocprof_assembly_ms(a.config)
        naug = -(-n // 256) * 256 + 128
        nt = naug // 128
        # sweep steps per bulk launch, from the launch count (steps / groups)
        nsteps = -(-n // 256)
        zst = max(1, round(nsteps / (upd_n / a.steps))) if upd_n else 4
        # compulsory bytes of one bulk launch: every lower 128-tile of A read
        # and written once, plus the Z steps' W and Pn panels
        alg_bytes = nt * (nt + 1) // 2 * 128 * 128 * 8 * 2 + 2 * zst * naug * 256 * 8
        evals = a.steps * world
        value = evals / dt_max
        achieved = upd_work / (upd_ms * 1e-3) / 1e12 if upd_ms > 0 else None
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "evals/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": dt_max / a.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (seeded SURVEY.md §8d generator; no dataset exists for this metric)",
            "config": {
                "workload": (f"{a.config}: n={n}, d={p}, {kernel}, ns basis B={B}, fp64; one "
                             "para_update (kernel assembly + SPD inverse/log-det + all P gradients "
                             "+ RMSE/evidence + Nadam step) per step"),
                "n": n, "p": p, "B": B, "kernel": kernel,
                "parallelism": "single" if world == 1 else f"replicas x{world}",
            },
            "roofline": {
                "kernel": (f"k_update_multi (bulk sweep update, {zst} Gauss-Jordan steps per launch, "
                           f"K = {256 * zst} per 128x128 tile, v_mfma_f64_16x16x4_f64)"),
                "bound": "mfma",
                "achieved": achieved,
                "peak": FP64_MFMA_PEAK_TFLOPS,
                "unit": "TFLOP/s",
                "frac": (achieved / FP64_MFMA_PEAK_TFLOPS) if achieved else None,
                "traffic": traffic,
                "traffic_unit": "bytes/launch (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE)",
                "traffic_source": traffic_src,
                "algorithmic_bytes_per_launch": alg_bytes,
                "rocprof_avg_launch_ms": rp_ms,
                "rocprof_source": rp_src,
                "launches": upd_n,
                "avg_launch_ms": upd_ms / upd_n if upd_n else None,
                "algorithmic_flops_per_launch": upd_work / upd_n if upd_n else None,
                # the sweep as a whole: every update / cross / panel-GEMM flop
                # over the span from the first bulk launch's start to the last
                # one's end (the side streams' work runs inside it), per evaluation
                "sweep_span_ms": sweep_ms / sweep_n if sweep_n else None,
                "sweep_achieved": (sweep_work / (sweep_ms * 1e-3) / 1e12) if sweep_ms > 0 else None,
                "sweep_frac": ((sweep_work / (sweep_ms * 1e-3) / 1e12) / FP64_MFMA_PEAK_TFLOPS
                               if sweep_ms > 0 else None),
            },
            "dense_gflops_per_eval_wall": (n ** 3) / (dt_max / a.steps) / 1e9,
            "phase_ms_per_step": {"update_kernel": upd_ms / a.steps,
                                  "assembly_kernel": asm_ms / a.steps,
                                  "gradient_kernel": grad_ms / a.steps},
            # device timeline per evaluation (HIP events on the model's stream):
            # assembly main-launch end -> first bulk launch start, and the
            # span from the assembly's start to the gradient's end
            "timeline_ms_per_eval": {
                "assembly_end_to_first_bulk": lead_ms / lead_n if lead_n else None,
                "device_span": span_ms / span_n if span_n else None},
            "pair_kernels_tflops": {
                # (HIP events around the main stream's assembly launches: the
                # filler's share of the tiles runs after them on the tail
                # stream, so this overstates the rate; assembly_rocprof below
                # charges every assembly launch)
                "assembly": asm_work / (asm_ms * 1e-3) / 1e12 if asm_ms else None,
                "assembly_rocprof": (asm_work / a.steps / (asm_rp_ms * 1e-3) / 1e12) if asm_rp_ms else None,
                "assembly_rocprof_ms_per_eval": asm_rp_ms,
                "assembly_rocprof_source": asm_rp_src,
                "gradient": grad_work / (grad_ms * 1e-3) / 1e12 if grad_ms else None},
            "pair_kernels_hbm_gbs": pair_hbm_gbs(asm_ms / a.steps, grad_ms / a.steps, a.config),
            "last_stats": [float(stats[0]), float(stats[1])],
            "predict": pred,
            "r6_drop_in": r6,
        }
        if world == 1 and not a.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(a.config)

    failed = False
    if world > 1 and a.mode == "auto":
        model.close()

        def leg():
            sh = run_sharded(dist, rank, world, ctx, a.shard_steps, 1)
            t1 = dt_max / a.steps
            sh["weak_scaling_efficiency"] = (sh["n"] ** 3 / (sh["ms_per_step"] * 1e-3) / world) / (
                n ** 3 / t1) if a.config == "C2" else None
            return sh
        sh, failed = run_guarded(line, leg, a.shard_timeout)
        if line is not None:
            line["sharded"] = sh
            # SURVEY §8d's weak-scaling efficiency of ONE sharded evaluation
            # (the headline value above is N independent replicas)
            line["sharded_evals_per_s"] = sh.get("evals_per_s")
            line["sharded_weak_scaling_efficiency"] = sh.get("weak_scaling_efficiency")
    if line is not None:
        print(json.dumps(line), flush=True)
    if failed:  # peers may be stuck in a collective: no barrier; rc shows it
        sys.stdout.flush()
        os._exit(EXIT_SHARDED_FAILED)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
