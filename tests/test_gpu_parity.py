"""Parity of the HIP path (through the C-ABI) against the CPU restatement in oracle/.

Tolerance: the north_star bar, <= 1e-9 relative on logpdf (fp64). Observed agreement is
~1e-15 at these sizes; a tighter 1e-12 check on small cases guards against silent
precision regressions. The oracle is "parity unpinned" by the reference itself (no Julia
here, see oracle/restatement.py) — it is cross-checked against scikit-learn in
tests/test_oracle.py.
"""
import numpy as np
import pytest

from gaplac_amd import abstractgps as AG
from gaplac_amd import formula as F
from gaplac_amd._native import CAT, LINEAR, NOISE, OU, SQEXP
from gaplac_amd.backend import ArgumentError, Context, PosDefException
from oracle import restatement as R
from tests.conftest import gpu_available
from tests.golden_io import load_cases

pytestmark = pytest.mark.gpu
RTOL = 1e-9

CASES = load_cases()


@pytest.fixture(scope="module")
def ctx():
    if not gpu_available():
        pytest.skip("no GPU")
    c = Context(0)
    yield c
    c.close()


def rel(a, b):
    return abs(a - b) / max(abs(b), 1e-300)


@pytest.mark.parametrize("case", CASES, ids=[c["name"][:60] for c in CASES])
def test_golden_fixtures(ctx, case):
    if case["info"]:
        with pytest.raises(PosDefException) as ei:
            ctx.logpdf(case["X"], case["terms"], case["noise"], case["v"])
        assert ei.value.info == case["info"]
        return
    lp, ld, q = ctx.logpdf(case["X"], case["terms"], case["noise"], case["v"], full=True)
    assert rel(lp, case["logpdf"]) <= RTOL
    assert rel(ld, case["logdet"]) <= RTOL * max(1.0, abs(case["logpdf"]) / max(abs(case["logdet"]), 1e-300))
    assert rel(q, case["quad"]) <= RTOL * max(1.0, abs(case["logpdf"]) / max(abs(case["quad"]), 1e-300))
    if case["N"] <= 1024:
        assert rel(lp, case["logpdf"]) <= 1e-12


def test_gram_time_measures_the_same_gram(ctx):
    # gaplac_gram_time (bench.py extra.gram) builds the Gram into the workspace: its bytes
    # follow the documented formula and a logpdf right after it still matches the oracle
    rng = np.random.default_rng(5)
    N = 1000
    X = np.column_stack([rng.uniform(0, 10, N), rng.integers(0, 7, N).astype(float)])
    v = rng.standard_normal(N)
    terms = [(SQEXP, 0, 1.5, 0), (OU, 0, 3.0, 1), (CAT, 1, 0.0, 2), (NOISE, -1, 1.0, 3)]
    ms, nbytes = ctx.gram_time(X, terms, 0.1, v, reps=3)
    Np = (N + 1 + 127) // 128 * 128
    assert nbytes == 8.0 * Np * (Np + 1) / 2 + 8.0 * N * 3
    assert 0.0 < ms < 1000.0
    assert rel(ctx.logpdf(X, terms, 0.1, v), R.logpdf(X, terms, 0.1, v)[0]) <= 1e-12
    with pytest.raises(ArgumentError):
        ctx.gram_time(X, terms, 0.1, v, reps=0)


@pytest.mark.parametrize("case", [c for c in CASES if c["N"] <= 1024 and not c["info"]][:12],
                         ids=lambda c: c["name"][:60])
def test_gram_entrywise(ctx, case):
    G = ctx.gram(case["X"], case["terms"], case["noise"])
    Gr = R.gram(case["X"], case["terms"], case["noise"])
    assert np.max(np.abs(G - Gr)) <= 1e-13 * max(1.0, np.max(np.abs(Gr)))
    assert abs(G.sum() - case["gram_sum"]) <= 1e-12 * max(1.0, abs(case["gram_sum"]))


SIZES = [1, 2, 3, 64, 127, 128, 129, 255, 256, 257, 383, 385, 640, 1000, 2049]
TERMSETS = {
    "sqexp": [(SQEXP, 0, 1.5, 0)],
    "ou": [(OU, 0, 0.7, 0)],
    "composite": [(SQEXP, 0, 1.5, 0), (OU, 0, 3.0, 1), (CAT, 1, 0.0, 2), (NOISE, -1, 1.0, 3)],
    "linear_cat": [(LINEAR, 0, 0.5, 0), (CAT, 1, 0.0, 1)],
    "product": [(SQEXP, 0, 2.0, 0), (CAT, 1, 0.0, 0), (OU, 0, 1.0, 1)],
}


@pytest.mark.parametrize("name", sorted(TERMSETS))
@pytest.mark.parametrize("N", SIZES)
def test_random_sizes_vs_oracle(ctx, N, name):
    rng = np.random.default_rng(N * 31 + len(name))
    X = np.column_stack([rng.uniform(-5, 5, N), rng.integers(0, max(1, N // 4), N).astype(float)])
    v = rng.standard_normal(N)
    terms = TERMSETS[name]
    lp, ld, q = ctx.logpdf(X, terms, 0.1, v, full=True)
    rl, rd, rq = R.logpdf(X, terms, 0.1, v)
    assert rel(lp, rl) <= RTOL
    assert abs(ld - rd) <= RTOL * abs(rl)
    assert abs(q - rq) <= RTOL * abs(rl)


@pytest.mark.parametrize("N", [129, 300, 700])
def test_factor_and_solve_match_lapack(ctx, N):
    rng = np.random.default_rng(N)
    X = rng.uniform(-5, 5, (N, 1))
    v = rng.standard_normal(N)
    terms = [(SQEXP, 0, 1.0, 0), (LINEAR, 0, 0.1, 1)]
    L, z = ctx.factor(X, terms, 0.1, v)
    Lr = R.cholesky_lower(X, terms, 0.1)
    assert np.linalg.norm(L - Lr) <= 1e-12 * np.linalg.norm(Lr)
    import scipy.linalg
    zr = scipy.linalg.solve_triangular(Lr, v, lower=True)
    assert np.linalg.norm(z - zr) <= 1e-11 * np.linalg.norm(zr)


def test_deterministic_bitwise(ctx):
    rng = np.random.default_rng(5)
    X = rng.uniform(0, 10, (1500, 1))
    v = rng.standard_normal(1500)
    a = ctx.logpdf(X, [(SQEXP, 0, 1.5, 0), (OU, 0, 3.0, 1)], 0.1, v, full=True)
    b = ctx.logpdf(X, [(SQEXP, 0, 1.5, 0), (OU, 0, 3.0, 1)], 0.1, v, full=True)
    assert a == b


def test_posdef_failure_matches_lapack_info(ctx):
    g = np.array([5.0, 1, 2, 3, 4, 6, 7, 8, 9, 2, 11.0])
    with pytest.raises(PosDefException) as ei:
        ctx.logpdf(g, [(CAT, 0, 0.0, 0)], 0.0, np.ones(len(g)))
    assert ei.value.info == 10
    # NaN input: OpenBLAS potf2 (the reference's LAPACK) tests ajj <= 0 only, so a NaN
    # pivot raises nothing and logpdf is NaN — on both sides
    x = np.array([np.nan, 0.5, 1.0])
    assert np.isnan(ctx.logpdf(x, [(SQEXP, 0, 1.0, 0)], 0.1, np.ones(3)))
    assert np.isnan(R.logpdf(x, [(SQEXP, 0, 1.0, 0)], 0.1, np.ones(3))[0])
    # the context stays usable after a failure
    assert np.isfinite(ctx.logpdf(np.arange(4.0), [(SQEXP, 0, 1.0, 0)], 0.1, np.ones(4)))


def test_argument_errors(ctx):
    X = np.arange(10.0)[:, None]
    v = np.ones(10)
    for bad in ([(SQEXP, 0, 0.0, 0)], [(OU, 0, -1.0, 0)], [(LINEAR, 0, -0.5, 0)], [(9, 0, 1.0, 0)],
                [(SQEXP, 3, 1.0, 0)], [(SQEXP, 0, 1.0, 0)] * 17,
                [(SQEXP, 0, 1.0, 0), (CAT, 0, 0.0, 1), (OU, 0, 1.0, 0)]):
        with pytest.raises(ArgumentError):
            ctx.logpdf(X, bad, 0.1, v)
    with pytest.raises(ArgumentError):
        ctx.logpdf(X, [(SQEXP, 0, 1.0, 0)], -0.1, v)
    assert ctx.logpdf(np.zeros((0, 1)), [(SQEXP, 0, 1.0, 0)], 0.1, np.zeros(0)) == 0.0


def test_batch_matches_individual(ctx):
    rng = np.random.default_rng(9)
    N = 500
    X = np.column_stack([rng.uniform(0, 10, N), rng.integers(0, 50, N).astype(float)])
    v = rng.standard_normal(N)
    models = [[(SQEXP, 0, l, 0)] for l in (0.5, 1.0, 2.0)] + [[(OU, 0, 1.0, 0), (CAT, 1, 0.0, 1)],
                                                            [(CAT, 1, 0.0, 0)]]
    out, info = ctx.logpdf_batch(X, models, 0.1, v)
    assert np.all(info == 0)
    for m, lp in zip(models, out):
        assert rel(lp, R.logpdf(X, m, 0.1, v)[0]) <= RTOL
    # a non-PD model inside a batch reports its own info and does not poison the others
    out, info = ctx.logpdf_batch(X, [[(CAT, 1, 0.0, 0)], [(SQEXP, 0, 1.0, 0), (NOISE, -1, 0.1, 1)]], 0.0, v)
    assert info[0] > 0 and np.isnan(out[0]) and info[1] == 0 and np.isfinite(out[1])


def test_batch_lanes_bitwise_equal_to_single_evals(ctx):
    """Models evaluated together (N = 3000: the whole matrix in the persistent tail, so one
    tail launch for 8 models) give exactly the single-eval results (same
    kernels, same tasks per model), with a non-PD model in the middle."""
    rng = np.random.default_rng(12)
    N = 3000
    X = np.column_stack([rng.uniform(-5, 5, N), rng.uniform(0, 10, N), rng.integers(0, 900, N).astype(float)])
    v = rng.standard_normal(N)
    models = [[(SQEXP, 0, l, 0)] for l in (0.5, 1.0, 2.0, 4.0)] + [
        [(OU, 1, 1.0, 0), (CAT, 2, 0.0, 1)], [(CAT, 2, 0.0, 0)], [(LINEAR, 0, 0.5, 0), (SQEXP, 1, 2.0, 1)],
        [(SQEXP, 1, 1.0, 0), (OU, 1, 3.0, 1), (CAT, 2, 0.0, 2)]]
    out, info = ctx.logpdf_batch(X, models, 0.1, v)
    for m, lp, inf in zip(models, out, info):
        assert inf == 0
        assert lp == ctx.logpdf(X, m, 0.1, v)
    # noise 0 for the batch; every model but one carries its own Noise term
    models2 = [m + [(NOISE, -1, 0.1, len(m))] for m in models[:6]]
    models2.insert(3, [(CAT, 2, 0.0, 0)])
    out, info = ctx.logpdf_batch(X, models2, 0.0, v)
    with pytest.raises(PosDefException) as e:
        ctx.logpdf(X, models2[3], 0.0, v)
    assert info[3] == e.value.info and np.isnan(out[3])
    for i, m in enumerate(models2):
        if i != 3:
            assert info[i] == 0 and out[i] == ctx.logpdf(X, m, 0.0, v)


def test_abstractgps_frontend_and_select(ctx):
    import pandas as pd
    from tests.golden_io import GOLDEN
    import os
    df = pd.read_csv(os.path.join(GOLDEN, "data", "input_pair_109.tsv"), sep="\t")
    table = {c: df[c].to_numpy() for c in df.columns if c != "SampleID"}
    spec = F.gp_spec("bug ~| Cat(:PersonID) + Linear(:nutrient) + SqExp(:Date; l=30)")
    gp, vars_ = AG.make_gp(spec)
    fx = AG.FiniteGP(gp, AG.design_matrix(table, vars_), 0.1)
    lp = AG.logpdf(fx, table["bug"], ctx=ctx)
    ref = R.logpdf(AG.design_matrix(table, vars_), fx.terms, 0.1, table["bug"])[0]
    assert rel(lp, ref) <= RTOL
    bayes, lp1, lp2 = AG.select_formulae("bug ~| SqExp(:Date; l=30)", "bug ~| OU(:Date; l=30)", table, ctx=ctx)
    assert bayes == lp1 - lp2


def test_large_n_properties(ctx):
    """N = 16384 (the benchmark size): the oracle once, plus a size-independent property:
    permuting the observations (rows of X with v) leaves logpdf unchanged."""
    N = 16384
    rng = np.random.default_rng(2)
    X = np.column_stack([rng.uniform(0, 10, N), rng.integers(0, N // 3, N).astype(float)])
    v = rng.standard_normal(N)
    terms = [(SQEXP, 0, 1.5, 0), (OU, 0, 3.0, 1), (CAT, 1, 0.0, 2), (NOISE, -1, 1.0, 3)]
    lp = ctx.logpdf(X, terms, 0.1, v)
    ref = R.logpdf(X, terms, 0.1, v)[0]
    assert rel(lp, ref) <= RTOL
    perm = rng.permutation(N)
    lp2 = ctx.logpdf(X[perm], terms, 0.1, v[perm])
    assert rel(lp2, lp) <= RTOL


def test_batch_on_lanes_bitwise_equal_to_single_evals():
    """Beyond the whole-matrix tail (GAPLAC_TAIL_S=32, N = 7000: 55 tile columns, super-
    panels then the tail) the models run concurrently on batch lanes: again exactly the
    single-eval results."""
    if not gpu_available():
        pytest.skip("no GPU")
    import os
    old = os.environ.get("GAPLAC_TAIL_S")
    os.environ["GAPLAC_TAIL_S"] = "32"
    try:
        c = Context(0)
    finally:
        if old is None:
            os.environ.pop("GAPLAC_TAIL_S")
        else:
            os.environ["GAPLAC_TAIL_S"] = old
    try:
        rng = np.random.default_rng(13)
        N = 7000
        X = np.column_stack([rng.uniform(0, 10, N), rng.integers(0, 2000, N).astype(float)])
        v = rng.standard_normal(N)
        models = [[(SQEXP, 0, l, 0), (CAT, 1, 0.0, 1)] for l in (0.7, 1.5)] + [[(OU, 0, 2.0, 0)], [(SQEXP, 0, 1.0, 0)]]
        out, info = c.logpdf_batch(X, models, 0.1, v)
        for m, lp, inf in zip(models, out, info):
            assert inf == 0 and lp == c.logpdf(X, m, 0.1, v)
        ref = R.logpdf(X, models[3], 0.1, v)[0]
        assert abs(out[3] - ref) <= 1e-9 * abs(ref)
    finally:
        c.close()


def test_batched_tail_sets_reused_bitwise_equal_to_single_evals():
    """The batched tail with 3 models per launch over 11 models: four launches
    alternate between the two workspace sets (each launch's Grams on s_panel beside the
    previous launch's tail), so every set is reused while the other is in flight; a
    non-positive-definite model sits in the middle. Every result is exactly the single
    evaluation's."""
    if not gpu_available():
        pytest.skip("no GPU")
    import os
    old = {k: os.environ.get(k) for k in ("GAPLAC_BATCH_W", "GAPLAC_BATCH_LAG")}
    os.environ.update({"GAPLAC_BATCH_W": "3", "GAPLAC_BATCH_LAG": "5"})
    try:
        c = Context(0)
    finally:
        for k, val in old.items():
            if val is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = val
    try:
        rng = np.random.default_rng(29)
        N = 1500
        X = np.column_stack([rng.uniform(0, 10, N), rng.integers(0, 400, N).astype(float)])
        v = rng.standard_normal(N)
        models = [[(SQEXP, 0, 0.5 + 0.25 * i, 0), (CAT, 1, 0.0, 1), (NOISE, -1, 0.1, 2)] for i in range(10)]
        models.insert(5, [(CAT, 1, 0.0, 0)])  # noise 0 below: singular
        for rep in range(2):
            out, info = c.logpdf_batch(X, models, 0.0, v)
            for i, m in enumerate(models):
                if i == 5:
                    with pytest.raises(PosDefException) as e:
                        c.logpdf(X, m, 0.0, v)
                    assert info[i] == e.value.info and np.isnan(out[i])
                else:
                    assert info[i] == 0 and out[i] == c.logpdf(X, m, 0.0, v), (rep, i)
        ref = R.logpdf(X, models[7], 0.0, v)[0]
        assert rel(out[7], ref) <= RTOL
    finally:
        c.close()
