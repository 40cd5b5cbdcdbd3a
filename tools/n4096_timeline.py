"""configs[1] (N = 4096, whole matrix in the persistent tail): where one evaluation's wall
time goes outside the tail kernel. Run mode (default) times K resident evaluations with
perf_counter (as bench.py's measure_config1); under rocprofv3 --kernel-trace the analysis
mode splits each evaluation (init_result_kernel .. reduce_final_kernel) into its kernels
and the gaps between them.
usage: python tools/n4096_timeline.py run [K]
       python tools/n4096_timeline.py analyse TRACE_DIR"""
import csv
import statistics
import sys
import time


def run(k):
    sys.path.insert(0, ".")
    import torch
    from gaplac_amd.backend import Context
    from gaplac_amd import configs as CF
    x, v = CF.config1_inputs()
    N = x.shape[0]
    dx = torch.from_numpy(x).to("cuda")
    dv = torch.from_numpy(v).to("cuda")
    ctx = Context(0)

    def one(i):
        return ctx.logpdf_device(N, 1, dx.data_ptr(), N, CF.config1_terms(CF.LENGTHSCALES_1[i % 4]), CF.NOISE_VAR,
                                 dv.data_ptr())

    for i in range(4):
        one(i)
    torch.cuda.synchronize()
    ts = []
    for i in range(k):
        t0 = time.perf_counter()
        one(i)
        ts.append((time.perf_counter() - t0) * 1e6)
    print(f"wall per evaluation: median {statistics.median(ts):.1f} us, min {min(ts):.1f}, "
          f"mean {statistics.mean(ts):.1f} ({k} evaluations)", flush=True)


def analyse(d):
    tr = list(csv.DictReader(open(f"{d}/run_kernel_trace.csv")))
    tr.sort(key=lambda r: int(r["Start_Timestamp"]))
    short = lambda n: n.split("(")[0].replace("gaplac::", "").removeprefix("void ").split("<")[0]
    evs, cur = [], None
    for r in tr:
        n = short(r["Kernel_Name"])
        if n in ("init_result_kernel", "init_result_ctl_kernel"):  # (the latter: Gram inside the tail)
            cur = []
        if cur is not None:
            cur.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), n))
            if n == "reduce_final_kernel":
                evs.append(cur)
                cur = None
    evs = evs[4:]  # the warm-up evaluations
    if not evs:
        print("no complete evaluation in the trace")
        return
    span, parts, gaps, starts = [], {}, {}, []
    for k, ev in enumerate(evs):
        t0 = ev[0][0]
        span.append((ev[-1][1] - t0) / 1e3)
        if k:
            starts.append((t0 - evs[k - 1][-1][1]) / 1e3)
        prev_end, prev_n = None, None
        for s, e, n in ev:
            parts.setdefault(n, []).append((e - s) / 1e3)
            if prev_end is not None:
                gaps.setdefault(f"{prev_n} -> {n}", []).append((s - prev_end) / 1e3)
            prev_end, prev_n = e, n
    med = statistics.median
    print(f"{len(evs)} evaluations: kernel span (init start .. reduce end) median {med(span):.1f} us, "
          f"min {min(span):.1f}")
    if starts:
        print(f"  idle between evaluations (host sync + next submit): median {med(starts):.1f} us")
    for n, v in parts.items():
        print(f"  {n:24s} median {med(v):8.1f} us")
    for n, v in gaps.items():
        print(f"  gap {n:44s} median {med(v):6.1f} us")


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(int(sys.argv[2]) if len(sys.argv) > 2 else 40)
    else:
        analyse(sys.argv[2])
