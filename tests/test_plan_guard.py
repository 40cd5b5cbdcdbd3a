"""Launch-footprint guard, on the CPU: gaplac_plan_check walks the real
host schedule of one evaluation without a device — every launch gaplac_logpdf /
gaplac_logpdf_grad / gaplac_posterior_mean_var would enqueue — and checks the element
range each launch's grid touches (derived from the same tile counts and decodes as the
kernels) against the workspace the context allocates. The sweep covers N = 1..300, where
the round-1 fault lived (the second Gram launch's tile count for N < 255), the padding
edges and larger orders; the negative control shrinks the workspace by one element, which
the last Gram tile must hit.
"""
import ctypes

import pytest

from gaplac_amd import _native

SIZES = list(range(1, 301)) + [383, 384, 385, 511, 512, 513, 1000, 2047, 4095, 4096, 4097, 16384, 65536]


def plan(N, mode, M=0, spw=4):
    lib = _native.load()
    launches, violations = ctypes.c_int64(), ctypes.c_int64()
    msg = ctypes.create_string_buffer(256)
    rc = lib.gaplac_plan_check(N, mode, M, spw, ctypes.byref(launches), ctypes.byref(violations), msg, 256)
    assert rc == 0, (N, mode, M, spw, rc)
    return launches.value, violations.value, msg.value.decode()


@pytest.mark.parametrize("spw", [1, 2, 4, 5, 8])
@pytest.mark.parametrize("mode,M", [(0, 0), (1, 0), (2, 1), (2, 130), (2, 1000), (2, 6016), (2, 6200)])
def test_every_launch_inside_the_workspace(mode, M, spw):
    for N in SIZES:
        if mode == 1 and N > 16384:
            continue  # the gradient's identity rows double the workspace; 64k is covered by logpdf
        launches, violations, msg = plan(N, mode, M, spw)
        assert launches > 0
        assert violations == 0, (N, mode, M, spw, msg)


def test_launch_counts_follow_the_schedule():
    # N = 16384 (nt = 129): one diagonal block per tile column plus TRSMs, column updates,
    # bulk updates, the Gram in two parts and the reduction, except for the last 80 tile
    # columns, which are one persistent tail launch: 49 chain columns
    l0, v0, _ = plan(16384, 0)
    assert v0 == 0 and 49 * 3 < l0 < 49 * 6 + 10
    l1, _, _ = plan(16384, 1)
    assert l1 > l0  # the gradient adds the identity-row launches and the C^-1 tiles
    # the posterior's cross-covariance rows ride in the same tail while they fit beside its
    # 80 columns (M <= 48 tile rows): the super-panel phase's extra-row launches only
    l2, v2, _ = plan(16384, 2, M=1024)
    l3, v3, _ = plan(16384, 2, M=48 * 128 + 1)  # 49 tile rows: no tail, every column a super-panel
    assert v2 == v3 == 0 and l0 < l2 < l3


@pytest.mark.parametrize("N", [1, 127, 128, 129, 254, 255, 300, 4096])
@pytest.mark.parametrize("mode", [0, 1, 2])
def test_negative_control_short_workspace_is_reported(N, mode):
    launches, violations, msg = plan(N, mode + 8, M=64 if mode == 2 else 0)
    assert violations >= 1
    assert "outside" not in msg and "touches elements" in msg


def test_bad_arguments():
    lib = _native.load()
    z = ctypes.c_int64()
    for args in ((0, 0, 0, 4), (10, 3, 0, 4), (10, 2, 0, 4), (10, 0, 0, 0), (10, 0, 0, 9)):
        assert lib.gaplac_plan_check(*args, ctypes.byref(z), ctypes.byref(z), None, 0) == _native.E_ARG


def schedule(N, spw=4, depth=0, ext=1, pair_m=40):
    lib = _native.load()
    msg = ctypes.create_string_buffer(256)
    n = ctypes.c_int64()
    rc = lib.gaplac_plan_check_schedule(N, spw, depth, ext, pair_m, ctypes.byref(n), msg, 256)
    return rc, n.value, msg.value.decode()


@pytest.mark.parametrize("depth", [0, 2, 3, 4, 5, 6, 7, 8])
@pytest.mark.parametrize("ext", [0, 1])
def test_single_gpu_schedule_applies_every_panel_once_in_order(depth, ext):
    """the deferred bulk updates at every depth (GAPLAC_PAIR_DEPTH 2..8, 0 =
    auto) and with / without the band extension: a dry walk of the real schedule records
    every update and factorisation, and every tile column gets every earlier panel column
    exactly once, in order, before its diagonal block or the persistent tail."""
    for N in (1, 127, 1000, 4096, 10239, 10240, 12000, 16384, 20000, 33000, 40000, 50000, 65536):
        for spw, pair_m in ((4, 40), (4, 8), (2, 24), (3, 16)):
            rc, n, msg = schedule(N, spw, depth, ext, pair_m)
            assert rc == 0 and n >= 1, (N, spw, depth, ext, pair_m, msg)


def test_schedule_records_cover_the_superpanel_phase():
    # N = 65536: 513 tile columns, the last 80 in the persistent tail, the rest in
    # super-panels: at least one factorisation record per non-tail column plus updates
    rc, n, msg = schedule(65536)
    assert rc == 0, msg
    assert n > 2 * (513 - 80)
