"""Parametrised A/B runner (replaces the round-3 one-off tools/gpu_r03*.sh scripts).

Every arm is a library build and/or environment switches; the arms are run alternately
(rep 1: a b c, rep 2: a b c, ...) so drift on the box hits every arm alike. Per arm and rep:

* ms per evaluation at the --ns sizes (tools/ab_n.py: configs[2]-style terms, inputs in HBM);
* with --select: bench.py --mode select (configs[4], 64 formulas x N=8192);
* with --grad / --posterior: bench.py --mode grad / posterior (N=16384);
* with --tests (first rep only): the listed GPU test files against that arm's library.

usage (on the GPU box):
  python tools/ab.py TAG [--reps 2] [--ns 16384,4096] [--select] [--grad] [--posterior]
                     [--tests tests/test_gpu_configs.py,...] ARM [ARM ...]
  ARM = name[:lib=path][:VAR=value]...     e.g.  cur   new:lib=tools/bin/lib_new.so
                                                 tail64:GAPLAC_TAIL_S=64
Writes gpurun_out/TAG/ab.txt (one line per measurement); every child runs under its own
time limit and the first failure ends the run (non-zero exit).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def parse_arm(spec: str):
    parts = spec.split(":")
    env = {}
    for p in parts[1:]:
        k, v = p.split("=", 1)
        if k == "lib":
            env["GAPLAC_LIB_PATH"] = os.path.join(ROOT, v) if not os.path.isabs(v) else v
        else:
            env[k] = v
    return parts[0], env


def run(cmd, env, limit, out):
    full = dict(os.environ, **env)
    r = subprocess.run(["timeout", "-k", "10", str(limit)] + cmd, env=full, cwd=ROOT, capture_output=True, text=True)
    if r.returncode != 0:
        out.write(f"FAILED ({r.returncode}): {' '.join(cmd)}\n{r.stdout[-3000:]}\n{r.stderr[-3000:]}\n")
        out.flush()
        sys.stdout.write(f"FAILED ({r.returncode}): {' '.join(cmd)}\n{r.stderr[-2000:]}\n")
        raise SystemExit(1)
    return r.stdout


def bench_line(text: str) -> dict:
    return json.loads([s for s in text.strip().splitlines() if s.startswith("{")][-1])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("arms", nargs="+")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--ns", default="16384,4096")
    ap.add_argument("--select", action="store_true")
    ap.add_argument("--grad", action="store_true")
    ap.add_argument("--posterior", action="store_true")
    ap.add_argument("--tests", default="")
    a = ap.parse_args()
    os.makedirs(os.path.join(ROOT, "gpurun_out", a.tag), exist_ok=True)
    arms = [parse_arm(s) for s in a.arms]
    with open(os.path.join(ROOT, "gpurun_out", a.tag, "ab.txt"), "a") as out:
        def emit(s):
            print(s, flush=True)
            out.write(s + "\n")
            out.flush()

        for rep in range(1, a.reps + 1):
            for name, env in arms:
                if rep == 1 and a.tests:
                    txt = run([sys.executable, "-u", "-m", "pytest", *a.tests.split(","), "-m", "gpu", "-x", "-q",
                               "--timeout", "200", "--timeout-method", "thread"], env, 400, out)
                    emit(f"{name} tests: {txt.strip().splitlines()[-1]}")
                if a.ns:
                    txt = run([sys.executable, "-u", "tools/ab_n.py", "GAPLAC_NONE", "-", a.ns], env, 300, out)
                    for line in txt.splitlines():
                        if line.startswith("N="):
                            emit(f"{name} rep{rep} {line}")
                for mode, flag in (("select", a.select), ("grad", a.grad), ("posterior", a.posterior)):
                    if flag:
                        d = bench_line(run([sys.executable, "bench.py", "--mode", mode, "--steps", "4", "--warmup", "1",
                                            "--skip-cpu", "--no-profile"], env, 300, out))
                        emit(f"{name} rep{rep} {mode} {d['value']:.2f} /s {d['ms_per_step']:.2f} ms")


if __name__ == "__main__":
    main()
