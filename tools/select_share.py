"""configs[4]'s per-GPU share at 8 GPUs: gaplac_logpdf_batch over 8 of the 64 formulas
(replicas.shard rank 0) at N = 8192, against the 64-model batch, for several
GAPLAC_BATCH_LAG values (read at context creation).
usage: python tools/select_share.py [lag ...]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from gaplac_amd import configs as CF
    from gaplac_amd.backend import Context
    from gaplac_amd.replicas import shard
    import bench
    lags = [int(a) for a in sys.argv[1:]] or [-1]
    N = CF.N4
    X, y = CF.config4_inputs(N)
    models = bench.select_models()
    share = [models[i] for i in shard(len(models), 0, 8)]
    ref = None
    for lag in lags:
        if lag >= 0:
            os.environ["GAPLAC_BATCH_LAG"] = str(lag)
        else:
            os.environ.pop("GAPLAC_BATCH_LAG", None)
        with Context(0) as c:
            out = {}
            for name, ms in (("share8", share), ("all64", models)):
                got, _ = c.logpdf_batch(X, ms, CF.NOISE_VAR, y)
                reps = 6 if name == "share8" else 2
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(reps):
                    got, _ = c.logpdf_batch(X, ms, CF.NOISE_VAR, y)
                torch.cuda.synchronize()
                dt = (time.perf_counter() - t0) / reps
                out[name] = len(ms) / dt
                if name == "share8":
                    ref = got if ref is None else ref
                    out["bitwise_vs_first"] = bool((got == ref).all())
        print(json.dumps({"lag": lag, **out, "ratio": out["share8"] / out["all64"]}), flush=True)


if __name__ == "__main__":
    main()
