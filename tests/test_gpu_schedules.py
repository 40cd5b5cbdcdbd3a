"""The factorisation schedule's alternatives against the oracle and against each other
(DESIGN.md §3.1, §4): every switch below changes only the order and grouping of the same
updates, so each must reproduce the oracle's logpdf, logdet and quad (1e-12 relative at
these sizes) and agree with the default schedule.

* GAPLAC_TAIL_S: the last tile columns factored right-looking on one stream (serial tail;
  1000 makes it everything after the first super-panel, 0 turns it off);
* GAPLAC_SPW: the super-panel width;
* GAPLAC_PAIR_M / GAPLAC_BAND_TILES_M: paired bulk updates (every other step the columns
  beyond the next bands receive two super-panels at once; 1: whenever possible), bands as
  whole tiles or quadrants;
* GAPLAC_SERIAL: everything on one stream;
* GAPLAC_TAILK=0: the serial tail as per-column launches instead of the persistent dataflow
  kernel (tail_kernel);
A matrix with at most GAPLAC_TAIL_S tile columns lies whole in the persistent tail (library
default 80); the schedules here run with 32 unless they say otherwise, so the larger sizes
go through super-panels and then the tail.
The settings are read when a context is created (gaplac_ctx_create). A product-group
formula (PRODUCT_TERMS) runs through the main schedules too.
"""
import os

import numpy as np
import pytest

from gaplac_amd._native import CAT, NOISE, OU, SQEXP
from gaplac_amd.backend import Context
from oracle import restatement as R
from tests.conftest import gpu_available

pytestmark = pytest.mark.gpu

SCHEDULES = {
    "default": {},
    "serial_everything": {"GAPLAC_TAIL_S": "1000"},
    "no_serial_tail": {"GAPLAC_TAIL_S": "0"},
    "spw3_serial8": {"GAPLAC_SPW": "3", "GAPLAC_TAIL_S": "8"},
    "spw1_no_tail": {"GAPLAC_SPW": "1", "GAPLAC_TAIL_S": "0"},
    "pair_all": {"GAPLAC_PAIR_M": "1"},
    "pair_band_whole_tiles": {"GAPLAC_PAIR_M": "1", "GAPLAC_BAND_TILES_M": "1"},
    "no_pair": {"GAPLAC_PAIR_M": "0"},
    "pair_spw3_whole": {"GAPLAC_PAIR_M": "1", "GAPLAC_SPW": "3", "GAPLAC_BAND_TILES_M": "1"},
    "pair_no_tail": {"GAPLAC_PAIR_M": "1", "GAPLAC_TAIL_S": "0"},
    "serial_stream": {"GAPLAC_SERIAL": "1"},
    "tail_launches": {"GAPLAC_TAILK": "0"},
    "tailk_everything": {"GAPLAC_TAIL_S": "1000"},
    "tailk_spw1": {"GAPLAC_SPW": "1", "GAPLAC_TAIL_S": "40"},
    "whole_tail_80": {"GAPLAC_TAIL_S": "80"},
    "whole_tail_128": {"GAPLAC_TAIL_S": "128"},
}
SIZES = [1, 127, 129, 700, 2049, 3000, 9000]
TERMS = [(SQEXP, 0, 1.5, 0), (OU, 0, 3.0, 1), (CAT, 1, 0.0, 2), (NOISE, -1, 1.0, 3)]
# SqExp * Cat + OU (a product group)
PRODUCT_TERMS = [(SQEXP, 0, 1.5, 0), (CAT, 1, 0.0, 0), (OU, 0, 3.0, 1)]


def inputs(N):
    rng = np.random.default_rng(N)
    X = np.column_stack([rng.uniform(0, 10, N), rng.integers(0, max(1, N // 3), N).astype(float)])
    return X, rng.standard_normal(N)


def make_ctx(env):
    # the super-panel schedules at these sizes: a 32-column tail, except where a schedule
    # says otherwise (the library default, 80, puts every size here whole in the tail)
    env = {"GAPLAC_TAIL_S": "32", **env}
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return Context(0)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


@pytest.fixture(scope="module")
def ctxs():
    if not gpu_available():
        pytest.skip("no GPU")
    cs = {name: make_ctx(env) for name, env in SCHEDULES.items()}
    yield cs
    for c in cs.values():
        c.close()


@pytest.mark.parametrize("N", SIZES)
def test_schedules_match_oracle_and_each_other(ctxs, N):
    X, v = inputs(N)
    rl, rd, rq = R.logpdf(X, TERMS, 0.1, v)
    base = ctxs["default"].logpdf(X, TERMS, 0.1, v, full=True)
    for name, c in ctxs.items():
        lp, ld, q = c.logpdf(X, TERMS, 0.1, v, full=True)
        assert abs(lp - rl) <= 1e-12 * abs(rl), (name, lp, rl)
        assert abs(ld - rd) <= 1e-12 * abs(rl), (name, ld, rd)
        assert abs(q - rq) <= 1e-12 * abs(rl), (name, q, rq)
        assert abs(lp - base[0]) <= 1e-12 * abs(rl), (name, lp, base[0])


@pytest.mark.parametrize("N", [3000, 9000])
def test_schedules_product_group(ctxs, N):
    X, v = inputs(N)
    rl, rd, rq = R.logpdf(X, PRODUCT_TERMS, 0.1, v)
    for name in ("default", "no_pair", "serial_stream", "pair_all"):
        lp, ld, q = ctxs[name].logpdf(X, PRODUCT_TERMS, 0.1, v, full=True)
        assert abs(lp - rl) <= 1e-12 * abs(rl), (name, lp, rl)
        assert abs(q - rq) <= 1e-12 * abs(rl), (name, q, rq)


def test_serial_tail_reports_posdef_failure(ctxs):
    # a zero pivot inside the serial tail: Cat-only without noise (exactly singular),
    # the same info from every schedule
    N = 1500  # distinct categories for 1000 rows (identity), then repeated triples: the first
    # zero pivot is at row 1002, tile column 7, inside the serial tail by default
    cats = np.concatenate([np.arange(1000), 1000 + np.repeat(np.arange(500 // 2 + 1), 2)[:500]])
    X = np.column_stack([np.zeros(N), cats.astype(float)])
    infos = set()
    for name, c in ctxs.items():
        out, info = c.logpdf_batch(X, [[(CAT, 1, 0.0, 0)]], 0.0, np.ones(N))
        assert info[0] > 0, name
        infos.add(int(info[0]))
    assert infos == {1002}
