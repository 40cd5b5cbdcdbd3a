#!/usr/bin/env python3
"""Throughput benchmark: GaPLAC log-marginal-likelihood evals/s at N=16384 fp64.

Workload (BASELINE.json configs[2], the configuration the metric is quoted on):
    SqExp(:t; l) + OU(:t; l=3) + Cat(:subject) + Noise,  N = 16384,  fp64,
    t ~ U(0, 10), subject = randint(0, N/3), v ~ N(0, 1), seed 2.
One step = one full logpdf evaluation (Gram build of all terms + 0.1 I, blocked Cholesky,
triangular solve, logdet -> scalar) through the C-ABI entry gaplac_logpdf_device with X
and v already resident in HBM. The SqExp lengthscale changes every step (an MCMC chain
proposing new hyperparameters), so nothing can be cached between steps.

Multi-GPU (--gpus N): each rank runs its own independent evaluations (replicas:
hyperparameter points / chains / select candidates), no data-path
collective; value = evals of all ranks / max wall time. Two ways to start it:

* under torch.distributed.run (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* in the env):
  this process is one rank, and WORLD_SIZE must equal --gpus;
* as plain `python bench.py --gpus N` (no WORLD_SIZE in the env): this process is only a
  launcher. It checks that N devices are visible (torch.cuda.device_count() does not
  initialise the GPU), starts N child processes of this script with the rank variables
  set (rendezvous on 127.0.0.1), never touches the GPU itself and never execs, and exits
  with the first failing child's status (the other ranks are then terminated).
Every rank asserts world size == --gpus and that its device exists; on a 1-GPU box
`--gpus 2` fails with a message instead of reporting n_gpus: 1.

With --gpus > 1 rank 0 also measures BASELINE configs[3] (N=65536) spread over all ranks
(extra.dist) and checks its logpdf against the single-GPU evaluation of the same input in
the same run (extra.dist.parity_vs_single, bar 1e-9 relative); a failed or non-matching
dist line makes the process exit non-zero (4) after the JSON line is printed. The leg runs
under its own deadline (--dist-deadline, 240 s, well inside the driver's limit and the
process group's 600 s collective timeout): a leg that hangs (a collective that never
completes) becomes an error in the line instead of a job killed with no line at all;
rank 0 prints the replicas line with dist_ok false and the process ends with status 4
without waiting for the hung collective (bounded_leg).

Prints ONE JSON line (rank 0).
"""
from __future__ import annotations

import argparse
import datetime
import json
import os
import platform
import socket
import subprocess
import sys
import threading
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

from gaplac_amd import configs as CF  # noqa: E402  (synthetic inputs of the BASELINE configs)

N_DEFAULT = CF.N2
PEAK_F64_TFLOPS = 78.6   # MI355X FP64 matrix, spec
PEAK_HBM_GBS = 8000.0    # MI355X HBM3E, spec (MI355X_MICROARCH.md)
LENGTHSCALES = CF.LENGTHSCALES_2
make_inputs = CF.config2_inputs
terms_for = CF.config2_terms


def _blas_threads() -> int:
    try:
        from threadpoolctl import threadpool_info
        return max((d.get("num_threads", 1) for d in threadpool_info() if d.get("user_api") == "blas"), default=1)
    except Exception:
        return os.cpu_count() or 1


def _host_cores() -> dict:
    """What the CPU baseline may use: the process's CPU affinity set, the pool's per-GPU
    CPU share (OMP_NUM_THREADS, set by the GPU pool and not overridden here) and the BLAS
    threads the oracle actually runs (all usable cores)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS")
    return {"affinity_cores": aff, "omp_num_threads": int(omp) if omp and omp.isdigit() else None,
            "blas_threads": _blas_threads()}


def _cores_note(h: dict) -> str:
    share = h["omp_num_threads"]
    if share and share < h["affinity_cores"]:
        return (f"{h['blas_threads']} BLAS threads = the pool's CPU share per GPU (OMP_NUM_THREADS={share}; "
                f"the affinity mask shows {h['affinity_cores']} CPUs of the shared host)")
    return f"{h['blas_threads']} BLAS threads of {h['affinity_cores']} CPUs in the affinity mask"


def cpu_baseline(N: int, budget_s: float = 25.0):
    """Time the oracle (numpy Gram + scipy/OpenBLAS dpotrf + dtrsv) on the host cores."""
    from oracle import restatement as R
    hc = _host_cores()
    threads = hc["blas_threads"]
    X, v = make_inputs(N)
    n_small = 2048
    Xs, vs = make_inputs(n_small)
    R.logpdf(Xs, terms_for(1.5), 0.1, vs)  # warm up BLAS threads / page in
    times = []
    t_start = time.perf_counter()
    for i in range(8):
        t0 = time.perf_counter()
        R.logpdf(X, terms_for(LENGTHSCALES[i % len(LENGTHSCALES)]), 0.1, v)
        times.append(time.perf_counter() - t0)
        if time.perf_counter() - t_start > budget_s:
            break
    med = float(np.median(times))
    cpu = platform.processor() or platform.machine()
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    cpu = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {
        "value": 1.0 / med,
        "unit": "evals/s",
        "cores": int(threads),
        "kind": "port",
        "host_cores": hc,
        "sample": f"{len(times)} full evals at N={N} (same workload, seed 2), median {med:.2f} s; "
                  f"numpy Gram + scipy-openblas dpotrf('U') + dtrsv, {_cores_note(hc)}, on {cpu}",
    }


# PMC traffic of the dominant kernel (tools/profile_round.sh: FETCH_SIZE / WRITE_SIZE
# passes over the same command, corrected per MI355X_MICROARCH.md; per launch).
TRAFFIC_FILE = os.path.join("profiles", "r06g8_traffic_syrk.json")
TRAFFIC_FILE_CINV = os.path.join("profiles", "r06g8_traffic_cinv.json")


def load_traffic(name=TRAFFIC_FILE):
    path = os.path.join(HERE, name)
    try:
        with open(path) as f:
            d = json.load(f)
        return d.get("bytes_per_launch"), os.path.relpath(path, HERE)
    except (OSError, ValueError):
        return None, None


DIST_PARITY_BAR = 1e-9  # relative, north_star's fp64 bar
DIST_DEADLINE_S = 240.0  # the configs[3] leg's own deadline (--dist-deadline)
NONROOT_GRACE_S = 60.0   # other ranks wait this much longer, so rank 0 prints first


def bounded_leg(rank: int, fn, deadline_s: float, device=None):
    """Run one collective leg (fn) on a worker thread under a deadline: (result, expired).

    A leg that does not finish in deadline_s (rank 0; the other ranks NONROOT_GRACE_S
    later, so that rank 0 reports first) returns ({"error": ...}, True) and leaves its
    thread behind, blocked in whatever collective hung: the caller must then end the
    process with os._exit (a clean shutdown would wait for that collective). An exception
    in fn is returned as {"error": ...} on rank 0 and re-raised on the others (the launcher
    then stops the job, non-zero). device: the thread's torch device (torch keeps the
    current device per thread)."""
    box = {}

    def target():
        try:
            if device is not None:
                import torch
                torch.cuda.set_device(device)
            box["value"] = fn()
        except BaseException as e:  # reported below
            box["error"] = e

    th = threading.Thread(target=target, name="bounded-leg", daemon=True)
    th.start()
    th.join(deadline_s if rank == 0 else deadline_s + NONROOT_GRACE_S)
    if th.is_alive():
        return {"error": f"deadline: the leg did not finish within {deadline_s:.0f} s (a collective that never "
                         f"completed?); not waited for", "deadline_s": deadline_s}, True
    if "error" in box:
        if rank != 0:
            raise box["error"]
        return {"error": repr(box["error"])[:400]}, False
    return box["value"], False


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int, argv, need_gpus: bool = True, poll_s: float = 0.2) -> int:
    """Start n ranks of this script as child processes and wait for them.

    The parent never touches the GPU (device_count() only counts devices on this image)
    and never execs; each child gets RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* and the
    same argv. Returns 0 if every rank exited 0, otherwise the first failure's status
    (a signal maps to 128 + signo), after terminating the ranks still running."""
    if need_gpus:
        import torch
        have = torch.cuda.device_count()
        if have < n:
            print(f"bench: --gpus {n} needs {n} visible GPUs, this node shows {have}", file=sys.stderr, flush=True)
            return 2
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env))
    rc = 0
    pending = set(range(n))
    while pending:
        for r in sorted(pending):
            c = procs[r].poll()
            if c is None:
                continue
            pending.discard(r)
            if c != 0 and rc == 0:
                rc = c if c > 0 else 128 - c
                print(f"bench: rank {r} exited with status {c}; stopping the other ranks", file=sys.stderr, flush=True)
                for q in pending:
                    procs[q].terminate()
        if pending:
            time.sleep(poll_s)
    return rc


def rank_env(args):
    """(rank, world, local_rank) from the launcher's env, checked against --gpus."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench: --gpus {args.gpus} but WORLD_SIZE={world}: launch one rank per GPU "
                         f"(torch.distributed.run --nproc-per-node {args.gpus}, or plain python bench.py --gpus N)")
    return rank, world, local_rank


def init_rank(args):
    """Select this rank's GPU and join the job's process group (nccl = RCCL)."""
    rank, world, local_rank = rank_env(args)
    import torch
    import torch.distributed as dist
    have = torch.cuda.device_count()
    if local_rank >= have:
        raise SystemExit(f"bench: rank {rank} wants GPU {local_rank} but only {have} are visible")
    torch.cuda.set_device(local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank),
                                timeout=datetime.timedelta(seconds=600))
        assert dist.get_world_size() == world == args.gpus, (dist.get_world_size(), world, args.gpus)
    return rank, world, local_rank, torch, dist


def main_launcher_check(args):
    """--mode launcher-check: the rank side of the launcher without a GPU (gloo). Every
    rank checks its env against --gpus, all-reduces its rank, runs a stand-in collective
    leg through bounded_leg (the configs[3] leg's wrapper), and rank 0 prints one JSON
    line; --fail-rank r makes rank r exit 3 (tests the launcher's failure path);
    --hang-rank r makes rank r never join the leg's collective, so the leg hangs on every
    other rank (tests that a hang ends as a printed line with dist_ok false, status 4)."""
    rank, world, _ = rank_env(args)
    import torch
    import torch.distributed as dist
    if rank == args.fail_rank:
        raise SystemExit(3)
    dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=600))
    assert dist.get_world_size() == world
    t = torch.tensor([float(rank)], dtype=torch.float64)
    dist.all_reduce(t)
    ranks = [None] * world
    dist.all_gather_object(ranks, {"rank": rank, "pid": os.getpid()})

    def leg():
        if rank == args.hang_rank:
            time.sleep(1e6)  # never joins: the others block in the all_reduce below
        u = torch.ones(1, dtype=torch.float64)
        dist.all_reduce(u)
        return {"value": float(u.item()), "parity_ok": True}

    t0 = time.perf_counter()
    dist_line, expired = bounded_leg(rank, leg, args.dist_deadline)
    if rank == 0:
        out = {"metric": "launcher-check", "n_gpus": world, "rank_sum": float(t.item()),
               "pids": [r["pid"] for r in ranks], "extra": {"dist": dist_line},
               "dist_leg_s": round(time.perf_counter() - t0, 3)}
        out["dist_ok"] = "error" not in dist_line and bool(dist_line.get("parity_ok"))
        print(json.dumps(out), flush=True)
        if not out["dist_ok"]:
            print(f"bench: stand-in dist leg FAILED: {dist_line.get('error')}", file=sys.stderr, flush=True)
    if expired:
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(4)  # never wait for the hung collective
    dist.destroy_process_group()
    return 0 if rank != 0 or out["dist_ok"] else 4


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--n", type=int, default=N_DEFAULT)
    ap.add_argument("--skip-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--no-extra", action="store_true",
                    help="skip the extra size legs (N=4096, N=65536, select, two chains): profiling runs")
    ap.add_argument("--no-profile", action="store_true", help="skip the per-kernel event pass")
    ap.add_argument("--profile-steps", type=int, default=2, help="eager steps timed per kernel after the timed region")
    ap.add_argument("--mode", choices=("replicas", "dist", "single", "select", "grad", "posterior", "rand",
                                       "launcher-check"),
                    default="replicas",
                    help="replicas (default, the headline metric): independent evals per GPU; dist: one "
                         "evaluation spread over all ranks (BASELINE configs[3], N=65536); single: the "
                         "single-GPU path at --n (comparison line for dist); select: BASELINE configs[4], "
                         "64 candidate formulas x N=8192 through gaplac_logpdf_batch, sharded over ranks; "
                         "grad: logpdf + gradient (gaplac_logpdf_grad, the mcmc/NUTS step) on the configs[2] workload; "
                         "posterior: mean_and_var(posterior(fx, y), xs) at --m test points; rand: one FiniteGP draw; "
                         "launcher-check: the multi-rank launcher on gloo without a GPU (tests)")
    ap.add_argument("--m", type=int, default=1024, help="posterior mode: test points")
    ap.add_argument("--loopback", type=int, default=0,
                    help="dist mode on ONE GPU: emulate this many ranks in-process (schedule timing only)")
    ap.add_argument("--spw", type=int, default=4, help="dist mode: super-panel width in 128-column tiles")
    ap.add_argument("--no-dist", action="store_true",
                    help="replicas mode with --gpus > 1: skip the configs[3] distributed extra line")
    ap.add_argument("--dist-deadline", type=float, default=DIST_DEADLINE_S,
                    help="seconds the configs[3] leg (--gpus > 1) may take before it is reported as failed")
    ap.add_argument("--fail-rank", type=int, default=-1, help=argparse.SUPPRESS)  # launcher-check only
    ap.add_argument("--hang-rank", type=int, default=-1, help=argparse.SUPPRESS)  # launcher-check only
    argv = sys.argv[1:]
    args = ap.parse_args(argv)
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return launch_ranks(args.gpus, argv, need_gpus=args.mode != "launcher-check")
    if args.mode == "launcher-check":
        return main_launcher_check(args)
    if args.mode in ("dist", "single"):
        return main_dist(args)
    if args.mode == "select":
        return main_select(args)
    if args.mode == "grad":
        return main_grad(args)
    if args.mode in ("posterior", "rand"):
        return main_post(args)

    rank, world, local_rank, torch, dist = init_rank(args)

    from gaplac_amd.backend import Context

    N = args.n
    X, v = make_inputs(N)
    dX = torch.from_numpy(np.ascontiguousarray(X.T)).to("cuda")  # (2, N) row-major == N x 2 col-major
    dv = torch.from_numpy(v).to("cuda")
    torch.cuda.synchronize()
    ctx = Context(local_rank)

    def step(i):
        # replicas: every rank walks its own lengthscale sequence
        lval = LENGTHSCALES[(i + rank) % len(LENGTHSCALES)]
        return ctx.logpdf_device(N, 2, dX.data_ptr(), N, terms_for(lval), CF.NOISE_VAR, dv.data_ptr())

    for i in range(args.warmup):
        step(i)

    # The timed region: the production schedule, no instrumentation.
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    lp = None
    for i in range(args.steps):
        lp = step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0

    # Roofline pass: the same steps with hipEvents recorded on s_main (the launching
    # stream) around every bulk tile_syrk launch (gaplac_set_profiling mode 2).
    st_ev = None
    if not args.no_profile:
        ctx.reset_stats()
        ctx.set_profiling(2)
        for i in range(max(1, min(args.steps, 5))):
            step(i)
        ctx.set_profiling(0)
        st_ev = ctx.stats()

    # Per-kernel breakdown (extra): per-launch device timestamps wired into every kernel
    # (first workgroup start / last wave end on the 100 MHz s_memrealtime clock).
    st = None
    if not args.no_profile and args.profile_steps > 0:
        ctx.reset_stats()
        ctx.set_profiling(True)
        for i in range(args.profile_steps):
            step(i)
        ctx.set_profiling(False)
        st = ctx.stats()

    # Gram kernel alone (extra.gram): in the evaluation its second launch deliberately
    # shares the GPU with the first super-panel's chain (2 workgroups per CU), so the
    # in-situ rate is a schedule figure; the kernel's roofline is this standalone launch of
    # the same Gram (configs[2] terms, all lower tiles, plain grid, best of 5, hipEvents).
    gram_alone = None
    if not args.no_profile and rank == 0:
        gram_alone = ctx.gram_time(X, terms_for(LENGTHSCALES[0]), CF.NOISE_VAR, v, reps=5)

    full_run = not args.no_profile and not args.no_extra  # profiled runs keep to the timed schedule
    # Throughput with two chains per GPU (extra, not the headline): independent evaluations
    # in flight on two lanes (gaplac_logpdf_batch), filling the latency-bound tail of one
    # evaluation's panel chain with the other's bulk updates.
    two = None
    n4096 = None
    n65536 = None
    select4 = None
    if full_run and rank == 0:
        models = [terms_for(LENGTHSCALES[i % len(LENGTHSCALES)]) for i in range(8)]
        ctx.logpdf_batch(X, models[:2], CF.NOISE_VAR, v)
        tb = time.perf_counter()
        for _ in range(2):
            ctx.logpdf_batch(X, models, CF.NOISE_VAR, v)
        two = 16 / (time.perf_counter() - tb)
        n4096 = measure_config1(ctx, torch)
        n65536 = measure_config3_single(local_rank, torch)
        select4 = measure_config4(local_rank, torch)

    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # BASELINE configs[3] across the job's GPUs (N=65536, one evaluation spread over all
    # ranks, panel broadcasts over RCCL): an extra line beside the replicas headline.
    dist_line = None
    dist_expired = False
    if world > 1 and not args.no_dist:
        ctx.close()  # free the N=16384 workspace before the 65536 one
        single_lp = n65536["last_logpdf"] if n65536 else None
        dist_line, dist_expired = bounded_leg(
            rank, lambda: measure_config3_dist(rank, world, local_rank, torch, dist, single_lp=single_lp),
            args.dist_deadline, device=local_rank)

    total_evals = args.steps * world
    value = total_evals / elapsed
    ms_per_step = elapsed / args.steps * 1e3

    if rank != 0:
        if dist_expired:
            os._exit(4)  # the leg's collective never completed: do not wait for it
        if world > 1:
            dist.destroy_process_group()
        return

    roofline = None
    if st_ev and st_ev["syrk_launches"] > 0 and st_ev["syrk_ms"] > 0:
        flops_per_launch = st_ev["syrk_flops"] / st_ev["syrk_launches"]
        avg_s = st_ev["syrk_ms"] / st_ev["syrk_launches"] / 1e3
        achieved = flops_per_launch / avg_s / 1e12
        traffic, traffic_src = load_traffic()
        roofline = {
            "bound": "mfma",
            "kernel": "tile_syrk_kernel (bulk trailing update, 128x128 tiles, K=512 or 1024 (paired), LDS-DMA staged, "
                      "fp64 MFMA 16x16x4); since round 6 each triangle launch runs beside the next steps' band launches "
                      "(split bulk updates, DESIGN.md §3.8), so its launch time includes the GPU share the bands take: "
                      "bulk_phase below is the same code's throughput over the time it is in flight",
            "achieved": round(achieved, 3),
            "peak": PEAK_F64_TFLOPS,
            "unit": "TFLOP/s",
            "frac": round(achieved / PEAK_F64_TFLOPS, 4),
            "traffic": traffic,
            "traffic_source": traffic_src,
            "traffic_algorithmic": st_ev["syrk_bytes"] / st_ev["syrk_launches"],
            "flops_per_launch": flops_per_launch,
            "avg_launch_ms": st_ev["syrk_ms"] / st_ev["syrk_launches"],
            "launches": st_ev["syrk_launches"],
            "timing": "hipEvents recorded on the launching stream around every tile_syrk_kernel launch, "
                      "in a pass of the same steps right after the (uninstrumented) timed region; cf. "
                      "profiles/*kernel_stats.csv (rocprofv3 --kernel-trace --stats of the same command)",
        }
        if st_ev.get("bulk_union_ms", 0) > 0:
            bph = st_ev["bulk_flops"] / (st_ev["bulk_union_ms"] / 1e3) / 1e12
            roofline["bulk_phase"] = {
                "kernels": "tile_syrk_kernel + tile_band_kernel (the same tile_syrk_body: triangle updates, bands, "
                           "split heads, whole-tile lookaheads) over the super-panel phase",
                "achieved": round(bph, 3), "frac": round(bph / PEAK_F64_TFLOPS, 4),
                "flops": st_ev["bulk_flops"], "launches": st_ev["bulk_launches"],
                "union_ms": st_ev["bulk_union_ms"],
                "timing": "union of the launches' hipEvent intervals (each on its own stream), same pass"}
    eval_flops = N ** 3 / 3.0 + N ** 2
    eval_tflops = eval_flops * (value / world) / 1e12
    extra = {
        "whole_eval": {
            "flops_per_eval": eval_flops,
            "achieved_tflops_per_gpu": round(eval_tflops, 3),
            "frac_of_fp64_peak": round(eval_tflops / PEAK_F64_TFLOPS, 4),
        },
        "gram": None,
        "last_logpdf": lp,
        "two_chains_evals_per_s": two,
        "n4096": n4096,
        "n65536": n65536,
        "select": select4,
        "select_share8": select4.get("share8") if select4 else None,
        "dist": dist_line,
    }
    if gram_alone:
        g_ms, g_bytes = gram_alone
        gbs = g_bytes / (g_ms / 1e3) / 1e9
        extra["gram"] = {"bound": "hbm", "kernel": "gram_kernel, all lower tiles in one launch (configs[2] terms)",
                         "achieved_GBs": round(gbs, 1), "peak_GBs": PEAK_HBM_GBS, "frac": round(gbs / PEAK_HBM_GBS, 4),
                         "launch_ms": round(g_ms, 4), "bytes_algorithmic": g_bytes,
                         "timing": "hipEvents around the launch on its stream, best of 5 (gaplac_gram_time)"}
    if st and st["gram_launches"] > 0 and st["gram_ms"] > 0:
        gbs = st["gram_bytes"] / (st["gram_ms"] / 1e3) / 1e9
        (extra["gram"] if extra["gram"] else extra)["gram_in_situ"] = {
            "achieved_GBs": round(gbs, 1), "frac": round(gbs / PEAK_HBM_GBS, 4),
            "ms_per_eval": st["gram_ms"] / max(st["evals"], 1),
            "note": "both Gram launches of an evaluation beside the first super-panel's chain (device stamps)"}
    if st and st["evals"] > 0:
        extra["profiled_span_ms_per_eval"] = st["total_ms"] / st["evals"]
        extra["diag_ms_per_eval"] = st["panel_ms"] / st["evals"]
        extra["trsm_ms_per_eval"] = st["trsm_ms"] / st["evals"]
        extra["colupd_ms_per_eval"] = st["colupd_ms"] / st["evals"]
        extra["syrk_ms_per_eval"] = st["syrk_ms"] / st["evals"]
        extra["small_update_ms_per_eval"] = st["small_ms"] / st["evals"]
        if st["syrk_launches"]:
            extra["syrk_avg_launch_ms_stamps"] = st["syrk_ms"] / st["syrk_launches"]

    cpu = None
    if world == 1 and not args.skip_cpu:
        cpu = cpu_baseline(N)

    out = {
        "metric": "log-marginal-likelihood evals/sec at N=16384 fp64",
        "value": value,
        "unit": "evals/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (seeded t~U(0,10), subject~randint(0,N/3), v~N(0,1); inputs resident in HBM)",
        "config": {
            "workload": f"BASELINE configs[2]: SqExp(:t;l in {list(LENGTHSCALES)})+OU(:t;l=3)+Cat(:subject)+Noise, N={N}, noise 0.1",
            "N": N,
            "terms": 4,
            "parallelism": "replicas" if world > 1 else "single",
        },
        "roofline": roofline,
        "cpu_baseline": cpu,
        "extra": extra,
    }
    rc = 0
    if dist_line is not None:
        # a failed or non-matching configs[3] line must not hide behind a good replicas
        # headline: the line is printed, then the process exits non-zero
        out["dist_ok"] = "error" not in dist_line and bool(dist_line.get("parity_ok"))
        if not out["dist_ok"]:
            why = dist_line.get("error") or f"parity_vs_single {dist_line.get('parity_vs_single')} > {DIST_PARITY_BAR}"
            print(f"bench: configs[3] distributed line FAILED: {why}", file=sys.stderr, flush=True)
            rc = 4
    print(json.dumps(out), flush=True)
    if dist_expired:
        sys.stderr.flush()
        os._exit(rc)  # the leg's thread is still blocked in a collective: do not wait for it
    if world > 1:
        dist.destroy_process_group()
    return rc


def measure_config1(ctx, torch, steps: int = 8):
    """BASELINE configs[1] (SqExp(:x), N=4096, l swept over {0.5, 1, 1.5, 3}) on this GPU:
    evals/s with inputs resident in HBM, and the whole evaluation against the fp64 MFMA
    peak (at nt = 33 tile columns every trailing update is small: the quadrant kernel)."""
    x, v = CF.config1_inputs()
    N = x.shape[0]
    dx = torch.from_numpy(x).to("cuda")
    dvv = torch.from_numpy(v).to("cuda")

    def one(i):
        return ctx.logpdf_device(N, 1, dx.data_ptr(), N, CF.config1_terms(CF.LENGTHSCALES_1[i % 4]), CF.NOISE_VAR,
                                 dvv.data_ptr())

    for i in range(2):
        one(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        one(i)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    flops = N ** 3 / 3.0 + N ** 2
    tf = flops / dt / 1e12
    return {"workload": f"BASELINE configs[1]: SqExp(:x; l in {list(CF.LENGTHSCALES_1)}), N={N}, noise 0.1",
            "evals_per_s": 1.0 / dt, "ms_per_eval": dt * 1e3, "achieved_tflops": round(tf, 3),
            "roofline": {"bound": "mfma", "kernel": "whole evaluation (F = N^3/3 + N^2)", "achieved": round(tf, 3),
                         "peak": PEAK_F64_TFLOPS, "unit": "TFLOP/s", "frac": round(tf / PEAK_F64_TFLOPS, 4)}}


def measure_config3_single(local_rank: int, torch, steps: int = 2, inputs=None):
    """BASELINE configs[3]'s workload (SqExp(:x; l=1.5), N=65536, seed 3) as ONE evaluation
    on ONE GPU: the north_star's 64k point and the 1-GPU base of the configs[3]
    strong-scaling curve. Its own context (34 GB workspace), freed afterwards."""
    from gaplac_amd.backend import Context
    x, v = CF.config3_inputs() if inputs is None else inputs
    N = x.shape[0]
    dx = torch.from_numpy(x).to("cuda")
    dvv = torch.from_numpy(v).to("cuda")
    c = Context(local_rank)
    try:
        def one():
            return c.logpdf_device(N, 1, dx.data_ptr(), N, CF.CONFIG3_TERMS, CF.NOISE_VAR, dvv.data_ptr())

        one()  # warmup: workspace, tile lists
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        lp = None
        for _ in range(steps):
            lp = one()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / steps
    finally:
        c.close()
        del dx, dvv
        torch.cuda.empty_cache()
    flops = N ** 3 / 3.0 + N ** 2
    tf = flops / dt / 1e12
    return {"workload": f"BASELINE configs[3] workload on 1 GPU: SqExp(:x; l=1.5), N={N}, noise 0.1",
            "evals_per_s": 1.0 / dt, "ms_per_eval": dt * 1e3, "steps": steps, "last_logpdf": lp,
            "roofline": {"bound": "mfma", "kernel": "whole evaluation (F = N^3/3 + N^2)", "achieved": round(tf, 3),
                         "peak": PEAK_F64_TFLOPS, "unit": "TFLOP/s", "frac": round(tf / PEAK_F64_TFLOPS, 4)}}


def measure_config4(local_rank: int, torch, steps: int = 2):
    """BASELINE configs[4] (select: 64 candidate formulas at N=8192, one gaplac_logpdf_batch
    call per step, the batched persistent tail of DESIGN.md §3.4) on this GPU, as an extra
    beside the headline; --mode select runs the same workload on its own. Its own context,
    freed afterwards."""
    from gaplac_amd.backend import Context
    N = CF.N4
    X, y = CF.config4_inputs(N)
    models = select_models()
    from gaplac_amd.replicas import shard
    # one GPU's share of the 8-GPU job (replicas.shard: rank 0's 8 of the 64 formulas)
    share8 = [models[i] for i in shard(len(models), 0, 8)]
    c = Context(local_rank)
    try:
        c.logpdf_batch(X, models, CF.NOISE_VAR, y)  # warmup: workspaces, task lists
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = None
        for _ in range(steps):
            out, _ = c.logpdf_batch(X, models, CF.NOISE_VAR, y)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / steps
        c.logpdf_batch(X, share8, CF.NOISE_VAR, y)  # warmup: the 8-model task list
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(2 * steps):
            c.logpdf_batch(X, share8, CF.NOISE_VAR, y)
        torch.cuda.synchronize()
        dt8 = (time.perf_counter() - t0) / (2 * steps)
    finally:
        c.close()
        torch.cuda.empty_cache()
    flops = len(models) * (N ** 3 / 3.0 + N ** 2)
    tf = flops / dt / 1e12
    rate64, rate8 = len(models) / dt, len(share8) / dt8
    return {"workload": f"BASELINE configs[4]: {len(models)} candidate formulas, N={N}, noise 0.1 (host inputs)",
            "evals_per_s": rate64, "ms_per_step": dt * 1e3, "steps": steps,
            "n_finite": int(np.isfinite(out).sum()),
            "roofline": {"bound": "mfma", "kernel": "whole batch (64 x (N^3/3 + N^2))", "achieved": round(tf, 3),
                         "peak": PEAK_F64_TFLOPS, "unit": "TFLOP/s", "frac": round(tf / PEAK_F64_TFLOPS, 4)},
            "share8": {"workload": f"one GPU's share of configs[4] on 8 GPUs: {len(share8)} formulas "
                                   f"(replicas.shard rank 0), N={N}, one gaplac_logpdf_batch call",
                       "evals_per_s": rate8, "ms_per_call": dt8 * 1e3, "ratio_to_64": rate8 / rate64}}


def measure_config3_dist(rank: int, world: int, local_rank: int, torch, dist, steps: int = 3,
                         single_lp: float | None = None, inputs=None):
    """BASELINE configs[3]: SqExp(:x; l=1.5), N=65536, one evaluation over all ranks of the
    job (1-D block-column cyclic Cholesky, panel broadcasts with RCCL over xGMI,
    gaplac_amd/distributed.py). Strong scaling: the work per evaluation is fixed.

    Rank 0 checks the distributed logpdf against the single-GPU evaluation of the same
    input (single_lp, or one evaluated here): parity_vs_single, bar DIST_PARITY_BAR.
    A failure on another rank raises (the launcher then stops the job, non-zero)."""
    try:
        line = _config3_dist(rank, world, local_rank, torch, dist, steps, inputs)
    except Exception as e:
        if rank != 0:
            raise
        return {"error": repr(e)[:400]}
    if rank == 0:
        if single_lp is None:
            single_lp = measure_config3_single(local_rank, torch, steps=1, inputs=inputs)["last_logpdf"]
        rel = abs(line["last_logpdf"] - single_lp) / abs(single_lp)
        line.update(single_gpu_logpdf=single_lp, parity_vs_single=rel, parity_bar=DIST_PARITY_BAR,
                    parity_ok=bool(rel <= DIST_PARITY_BAR))
    return line


def _config3_dist(rank: int, world: int, local_rank: int, torch, dist, steps: int, inputs=None):
    from gaplac_amd import distributed as DI
    x, v = CF.config3_inputs() if inputs is None else inputs  # (inputs: tests, a smaller N)
    N = x.shape[0]
    dx = torch.from_numpy(x).to("cuda")
    dvv = torch.from_numpy(v).to("cuda")
    r = DI.DistRank(local_rank, world, rank, spw=DI.DEFAULT_SPW)
    layout = "snake" if world > 1 and r.owner(world) == world - 1 else "round-robin"
    tr = DI.TorchTransport(device=torch.device("cuda", local_rank), timing=True)

    def one():
        return DI.logpdf_dist_device([r], tr, N, 1, dx.data_ptr(), N, CF.CONFIG3_TERMS, CF.NOISE_VAR,
                                     dvv.data_ptr())

    one()  # warmup (workspace, lists, RCCL communicator)
    tr.reset_timing()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    lp = None
    for _ in range(steps):
        lp = one()
    torch.cuda.synchronize()
    dist.barrier()
    el = time.perf_counter() - t0
    t = torch.tensor([el, tr.bcast_ms() / steps], dtype=torch.float64, device="cuda")
    allt = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(allt, t)
    r.close()
    el = max(float(a[0].item()) for a in allt)
    bc = [round(float(a[1].item()), 3) for a in allt]
    flops = N ** 3 / 3.0 + N ** 2
    tf = flops * steps / el / 1e12 / world
    return {"workload": f"BASELINE configs[3]: SqExp(:x; l=1.5), N={N}, noise 0.1, one evaluation over {world} GPUs",
            "value": steps / el, "unit": "evals/s", "ms_per_eval": el / steps * 1e3, "scaling": "strong",
            "ranks_seen": len(allt), "bcast_ms_per_eval_per_rank": bc, "last_logpdf": lp,
            "achieved_tflops_per_gpu": round(tf, 3), "frac_of_fp64_peak": round(tf / PEAK_F64_TFLOPS, 4),
            "transport": "torch.distributed nccl (RCCL) broadcast on the library's comm stream",
            "layout": layout, "tail_gather": "off (DESIGN.md §7.4)"}


def cpu_grad_baseline(N: int):
    """One oracle gradient evaluation (numpy Gram, scipy-openblas dpotrf + dpotri, numpy
    dK/dtheta contractions) at N on the host cores."""
    from oracle import restatement as R
    X, v = make_inputs(N)
    Xs, vs = make_inputs(1024)
    R.logpdf_grad_potri(Xs, terms_for(1.5), 0.1, vs)
    t0 = time.perf_counter()
    R.logpdf_grad_potri(X, terms_for(1.5), 0.1, v)
    dt = time.perf_counter() - t0
    try:
        from threadpoolctl import threadpool_info
        threads = max((d.get("num_threads", 1) for d in threadpool_info() if d.get("user_api") == "blas"), default=1)
    except Exception:
        threads = os.cpu_count() or 1
    return {"value": 1.0 / dt, "unit": "grad evals/s", "cores": int(threads), "kind": "port",
            "sample": f"1 full logpdf+gradient eval at N={N} (same workload), {dt:.1f} s: numpy Gram, scipy-openblas "
                      f"dpotrf + dpotri ({threads} BLAS threads), numpy dK/dtheta contractions (1 thread)"}


def main_grad(args):
    """logpdf + gradient evals/s (the mcmc NUTS step: gaplac_logpdf_grad_device), replicas."""
    rank, world, local_rank, torch, dist = init_rank(args)
    from gaplac_amd.backend import Context

    N = args.n
    X, v = make_inputs(N)
    dX = torch.from_numpy(np.ascontiguousarray(X.T)).to("cuda")
    dv = torch.from_numpy(v).to("cuda")
    torch.cuda.synchronize()
    ctx = Context(local_rank)

    def step(i):
        lval = LENGTHSCALES[(i + rank) % len(LENGTHSCALES)]
        return ctx.logpdf_grad_device(N, 2, dX.data_ptr(), N, terms_for(lval), 0.1, dv.data_ptr())

    for i in range(args.warmup):
        step(i)
    ctx.reset_stats()
    ctx.set_profiling(0 if args.no_profile else 2)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = None
    for i in range(args.steps):
        res = step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ctx.set_profiling(0)
    st_ev = ctx.stats()
    st = None
    if not args.no_profile and args.profile_steps > 0:
        ctx.reset_stats()
        ctx.set_profiling(True)
        for i in range(args.profile_steps):
            step(i)
        ctx.set_profiling(False)
        st = ctx.stats()
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return
    value = args.steps * world / elapsed
    Np = (N + 1 + 127) // 128 * 128
    m = (N + 127) // 128
    # -C^{-1} tiles: algorithmic flops of the lower triangle of Y Y^T (Y = L^{-T} upper
    # triangular): sum_{i >= j} 2 (N - i) = N^3/3 + O(N^2)
    cinv_flops = N ** 3 / 3.0
    roofline = None
    if st_ev["cinv_launches"] > 0 and st_ev["cinv_ms"] > 0:
        avg_s = st_ev["cinv_ms"] / st_ev["cinv_launches"] / 1e3
        ach = cinv_flops / avg_s / 1e12
        roofline = {"bound": "mfma",
                    "kernel": "cinv_contract_kernel (-C^{-1} = -L^{-T} L^{-1} lower tiles on fp64 MFMA 16x16x4, each "
                              "contracted with every dC/dtheta in place: never stored)",
                    "achieved": round(ach, 3), "peak": PEAK_F64_TFLOPS, "unit": "TFLOP/s",
                    "frac": round(ach / PEAK_F64_TFLOPS, 4), "traffic": load_traffic(TRAFFIC_FILE_CINV)[0],
                    "traffic_source": load_traffic(TRAFFIC_FILE_CINV)[1],
                    # Y's upper triangle read once (the -C^{-1} tiles are not written)
                    "traffic_algorithmic": 8.0 * Np * (Np + 1) / 2,
                    "flops_per_launch": cinv_flops, "avg_launch_ms": avg_s * 1e3,
                    "launches": st_ev["cinv_launches"],
                    "timing": "hipEvents on s_main around every cinv_contract_kernel launch inside the timed region"}
    grad_flops = N ** 3  # potrf N^3/3 + identity rows (L^{-T}) N^3/3 + C^{-1} N^3/3
    tf = grad_flops * (value / world) / 1e12
    extra = {"whole_eval": {"flops_per_eval": grad_flops, "achieved_tflops_per_gpu": round(tf, 3),
                            "frac_of_fp64_peak": round(tf / PEAK_F64_TFLOPS, 4)},
             "last_logpdf": res[0], "last_dparam": [float(x) for x in res[2]], "last_dnoise": res[3]}
    if st_ev["syrk_launches"] > 0 and st_ev["syrk_ms"] > 0:
        extra["tile_syrk_tflops"] = round(st_ev["syrk_flops"] / (st_ev["syrk_ms"] / 1e3) / 1e12, 3)
    if st and st["evals"] > 0:
        e = st["evals"]
        extra.update(profiled_span_ms_per_eval=st["total_ms"] / e, syrk_ms_per_eval=st["syrk_ms"] / e,
                     identity_rows_ms_per_eval=st["grad_rows_ms"] / e, cinv_ms_per_eval=st["cinv_ms"] / e,
                     contract_ms_per_eval=st["contract_ms"] / e, diag_ms_per_eval=st["panel_ms"] / e,
                     trsm_ms_per_eval=st["trsm_ms"] / e, colupd_ms_per_eval=st["colupd_ms"] / e)
    cpu = None
    if world == 1 and not args.skip_cpu:
        cpu = cpu_grad_baseline(N)
    out = {
        "metric": f"log-marginal-likelihood + gradient evals/sec at N={N} fp64 (mcmc NUTS step)",
        "value": value, "unit": "grad evals/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (seeded t~U(0,10), subject~randint(0,N/3), v~N(0,1); inputs resident in HBM)",
        "config": {"workload": f"BASELINE configs[2] terms, gradient w.r.t. v, every term parameter and the noise, N={N}",
                   "N": N, "terms": 4, "parallelism": "replicas" if world > 1 else "single"},
        "roofline": roofline, "cpu_baseline": cpu, "extra": extra,
    }
    print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main_post(args):
    """posterior: mean_and_var(posterior(FiniteGP(X, 0.1), y), xs) over M test points
    (gaplac_posterior_mean_var; src/plotting.jl:8-12); rand: rand(FiniteGP(X, 0.1)) = L z
    (gaplac_rand; CLI/src/sample.jl:25). configs[2] kernel and inputs; replicas over ranks."""
    rank, world, local_rank, torch, dist = init_rank(args)
    from gaplac_amd.backend import Context

    N, M = args.n, args.m
    X, v = make_inputs(N)
    rng = np.random.default_rng(5)
    Xs = np.column_stack([rng.uniform(0.0, 10.0, M), rng.integers(0, max(1, N // 3), M).astype(np.float64)])
    ctx = Context(local_rank)
    post = args.mode == "posterior"

    def step(i):
        lval = LENGTHSCALES[(i + rank) % len(LENGTHSCALES)]
        if post:
            return ctx.posterior_mean_var(X, terms_for(lval), 0.1, v, Xs)
        return ctx.rand(X, terms_for(lval), 0.1, v)

    for i in range(args.warmup):
        step(i)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return
    value = args.steps * world / elapsed
    # potrf N^3/3, plus the M cross-covariance rows through the factor (N^2 M) / L z (N^2)
    flops = N ** 3 / 3.0 + (float(N) * N * M if post else float(N) * N)
    tf = flops * value / world / 1e12
    cpu = None
    if world == 1 and not args.skip_cpu:
        from oracle import restatement as R
        t1 = time.perf_counter()
        if post:
            R.posterior_mean_var(X, terms_for(1.5), 0.1, v, Xs)
        else:
            R.rand_from(X, terms_for(1.5), 0.1, v)
        dt = time.perf_counter() - t1
        cpu = {"value": 1.0 / dt, "unit": "evals/s", "cores": _blas_threads(), "kind": "port",
               "sample": f"1 full evaluation at N={N}{f', M={M}' if post else ''} (same workload), {dt:.1f} s: numpy Gram"
                         f" + scipy-openblas dpotrf + " + ("dpotrs / dtrsm" if post else "dtrmv")}
    what = f"posterior mean_and_var at M={M} test points" if post else "rand(FiniteGP) draws"
    out = {
        "metric": f"{what}: evals/sec at N={N} fp64",
        "value": value, "unit": "evals/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (seeded t~U(0,10), subject~randint(0,N/3); host inputs, PCIe-inclusive)",
        "config": {"workload": f"BASELINE configs[2] kernel, N={N}" + (f", M={M}" if post else ""), "N": N,
                   "M": M if post else None, "parallelism": "replicas" if world > 1 else "single"},
        "roofline": None, "cpu_baseline": cpu,
        "extra": {"flops_per_eval": flops, "achieved_tflops_per_gpu": round(tf, 3),
                  "frac_of_fp64_peak": round(tf / PEAK_F64_TFLOPS, 4)},
    }
    print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


make_inputs_dist = CF.config3_inputs
select_models = CF.select_models


def main_select(args):
    """Batched select over 64 formulas (one gaplac_logpdf_batch call per rank; candidates
    sharded round-robin over ranks, results all-gathered: gaplac_amd/replicas.py)."""
    rank, world, local_rank, torch, dist = init_rank(args)
    from gaplac_amd import replicas
    from gaplac_amd.backend import Context

    N = args.n if args.n != N_DEFAULT else CF.N4
    X, y = CF.config4_inputs(N)
    models = select_models()
    ctx = Context(local_rank)
    mine = replicas.shard(len(models), rank, world)

    def step():
        out, info = ctx.logpdf_batch(X, [models[u] for u in mine], 0.1, y)
        if world > 1:
            return replicas.gather_results(mine, list(out), len(models), device=torch.device("cuda", local_rank))
        return out

    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    if rank == 0:
        value = args.steps * len(models) / elapsed
        out = {
            "metric": f"select: log-marginal-likelihood evals/sec, {len(models)} formulas x N={N} fp64",
            "value": value, "unit": "evals/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "strong",
            "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (seeded x~U(-5,5), t~U(0,10), subject~randint(0,N/3), y~N(0,1))",
            "config": {"workload": f"BASELINE configs[4]: {len(models)} candidate formulas, N={N}, noise 0.1", "N": N,
                       "parallelism": f"candidates round-robin over {world} rank(s)"},
            "extra": {"n_finite": int(np.isfinite(res).sum())},
        }
        print(json.dumps(out), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


def main_dist(args):
    """One evaluation spread over the ranks of the job (strong scaling: total work fixed)."""
    rank, world, local_rank, torch, dist = init_rank(args)
    from gaplac_amd import distributed as DI
    from gaplac_amd.backend import Context

    N = args.n if args.n != N_DEFAULT else CF.N3
    x, v = make_inputs_dist(N)
    dX = torch.from_numpy(x).to("cuda")
    dv = torch.from_numpy(v).to("cuda")
    terms = CF.CONFIG3_TERMS
    nranks = args.loopback if args.loopback > 0 else world
    if args.mode == "single":
        ctx = Context(local_rank)
        step = lambda: ctx.logpdf_device(N, 1, dX.data_ptr(), N, terms, 0.1, dv.data_ptr())
        parallelism = "single"
    else:
        if args.loopback > 0 or world == 1:
            nranks = max(1, args.loopback)
            ranks = [DI.DistRank(local_rank, nranks, r, spw=args.spw) for r in range(nranks)]
            tr = DI.LoopbackTransport()
        else:
            ranks = [DI.DistRank(local_rank, world, rank, spw=args.spw)]
            tr = DI.TorchTransport(device=torch.device("cuda", local_rank))
        step = lambda: DI.logpdf_dist_device(ranks, tr, N, 1, dX.data_ptr(), N, terms, 0.1, dv.data_ptr())
        parallelism = f"1-D block-column cyclic over {nranks} rank(s)" + (" (in-process loopback)" if args.loopback else "")
    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    lp = None
    for _ in range(args.steps):
        lp = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    if rank == 0:
        value = args.steps / elapsed
        flops = N ** 3 / 3.0 + N ** 2
        tf_per_gpu = flops * value / 1e12 / max(1, world)
        out = {
            "metric": f"log-marginal-likelihood evals/sec at N={N} fp64 (one evaluation over all GPUs)",
            "value": value, "unit": "evals/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "strong",
            "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (seeded x~U(-5,5), v~N(0,1); inputs resident in HBM)",
            "config": {"workload": f"BASELINE configs[3]: SqExp(:x; l=1.5), N={N}, noise 0.1", "N": N,
                       "parallelism": parallelism, "spw": args.spw, "mode": args.mode},
            "extra": {"achieved_tflops_per_gpu": round(tf_per_gpu, 3),
                      "frac_of_fp64_peak": round(tf_per_gpu / PEAK_F64_TFLOPS, 4), "last_logpdf": lp},
        }
        print(json.dumps(out), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main() or 0)
