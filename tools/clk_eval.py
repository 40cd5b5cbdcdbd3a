"""Diagnostic: the configs[2] evaluation at N=16384 with per-launch device slots
(profiling mode 1), for a -DGAPLAC_CLOCK library (GAPLAC_LIB_PATH): its bulk launches print
the clock they held and their per-workgroup cycles on stderr. A timing-only build (e.g.
GAPLAC_CHAIN_SKIP) may report a non-PD result: ignored."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from gaplac_amd import configs as CF  # noqa: E402
from gaplac_amd.backend import Context, PosDefException  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
X, v = CF.config2_inputs(N)
dX = torch.from_numpy(np.ascontiguousarray(X.T)).to("cuda")
dv = torch.from_numpy(v).to("cuda")
c = Context(0)
for i in range(8):
    if i == 5:
        c.set_profiling(True)
    try:
        c.logpdf_device(N, 2, dX.data_ptr(), N, CF.config2_terms(1.5), CF.NOISE_VAR, dv.data_ptr())
    except PosDefException:
        pass
c.set_profiling(False)
print(c.stats())
