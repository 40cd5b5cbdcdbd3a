"""gaplac_amd — MI355X-native backend for GaPLAC's GP log-marginal-likelihood path.

The hot path (Gram build + blocked Cholesky + triangular solve + logdet) lives in the
HIP library `_lib/libgaplac_hip.so` (C-ABI: include/gaplac.h). The Python modules mirror
the reference's formula/kernel API (src/gp_parts.jl, src/abstractgp_translations.jl,
src/interface.jl) and call the library through ctypes.
"""
__version__ = "0.1.0"
