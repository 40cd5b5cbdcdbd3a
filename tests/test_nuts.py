"""The mcmc sampler driver (gaplac_amd/nuts.py) on CPU: a target with a known law, and the
mcmc model of CLI/src/mcmc.jl:31-39 driven through the oracle's log density + gradient
(the GPU run of BASELINE configs[0] is tests/test_gpu_mcmc.py)."""
import math

import numpy as np

from gaplac_amd import nuts
from gaplac_amd.mcmc import MCMCModel
from oracle import restatement as R


class _Gauss:
    """ℓ ~ Uniform(0, 20), fx ~ N(0, I_d): in θ space u is standard logistic."""

    def __init__(self, d):
        self.N = d

    def logdensity_and_gradient(self, ell, fx):
        fx = np.asarray(fx)
        return -math.log(20.0) - 0.5 * float(fx @ fx), 0.0, -fx


def test_nuts_recovers_a_known_law():
    chain = nuts.sample(_Gauss(3), 3000, seed=4)
    fx = np.array([chain[f"fx[{i}]"] for i in (1, 2, 3)])
    assert np.all(np.abs(fx.mean(axis=1)) < 0.12)
    assert np.all(np.abs(fx.var(axis=1) - 1.0) < 0.15)
    ell = np.array(chain["ℓ"])
    assert 0.0 < ell.min() and ell.max() < 20.0
    assert abs(ell.mean() - 10.0) < 1.0          # Uniform(0, 20): mean 10, var 33.3
    assert abs(ell.var() - 400.0 / 12.0) < 5.0
    assert 0.4 < np.mean(chain["acceptance_rate"]) < 0.95  # adapted towards δ = 0.65
    assert len(chain["lp"]) == 3000 and chain["iteration"][0] == 301  # 300 warm-up draws discarded


class _OracleCtx:
    """The oracle's logpdf_grad in the place of the library (tests only)."""

    def __init__(self):
        self.calls = 0

    def logpdf_grad(self, X, terms, noise, v):
        self.calls += 1
        return R.logpdf_grad(X, terms, noise, v)


def config0_table(n=50, seed=0):
    rng = np.random.default_rng(seed)
    x = rng.uniform(-5, 5, n)
    K = np.exp(-0.5 * ((x[:, None] - x[None, :]) / 1.5) ** 2) + 1e-9 * np.eye(n)
    y = np.linalg.cholesky(K) @ rng.standard_normal(n)
    return {"x": x, "y": y}


def test_mcmc_model_chain_through_oracle_density(tmp_path):
    ctx = _OracleCtx()
    model = MCMCModel("y ~| SqExp(:x)", config0_table(30), ["x"], ctx=ctx)
    chain = nuts.sample(model, 40, seed=2, n_adapts=20)
    assert len(chain["ℓ"]) == 40 and all(0 < v < 20 for v in chain["ℓ"])
    assert all(np.isfinite(chain["lp"]))
    # one library call per density evaluation (the memo only dedupes identical points)
    assert ctx.calls == model.memo.calls <= chain["_density_calls"]
    out = tmp_path / "mcmc.tsv"
    from gaplac_amd.select import df_output, select_chains
    c = dict(chain)
    c.pop("_density_calls")
    df_output(c, str(out))
    head = out.read_text().splitlines()[0].split("\t")
    assert head[:3] == ["iteration", "chain", "ℓ"] and "lp" in head
    bayes, lp1, lp2 = select_chains(str(out), str(out))
    assert bayes == 0.0 and math.isfinite(lp1)


def test_lp_column_is_the_linked_space_log_density():
    # Turing 0.21 / DynamicPPL 0.19: the HMC step sets the VarInfo's logp to the sampler's
    # log density, which in linked space includes the logit log-Jacobian, so :lp equals
    # log_density on every draw (the column omitted the Jacobian)
    chain = nuts.sample(_Gauss(2), 50, seed=1, n_adapts=10)
    assert chain["lp"] == chain["log_density"]
    f = nuts.Unconstrained(_Gauss(2))
    for ell, a, b in zip(chain["ℓ"], chain["fx[1]"], chain["fx[2]"]):
        theta = f.to_theta(ell, [a, b])
        logp, _, lp_constrained = f(theta)
        s = ell / 20.0
        assert abs(logp - (lp_constrained + math.log(20.0 * s * (1.0 - s)))) <= 1e-9 * max(1.0, abs(logp))


def test_find_good_stepsize_bisects_into_the_acceptance_band():
    f = nuts.Unconstrained(_Gauss(3))
    rng = np.random.default_rng(5)
    theta = rng.uniform(-2, 2, 4)
    logp, grad, lp = f(theta)
    cur = nuts._State(theta, None, logp, grad, lp)
    eps = nuts.find_good_stepsize(f, cur, np.random.default_rng(7))
    # the final step size's one-step acceptance, from the same momentum draw
    r = np.random.default_rng(7).standard_normal(4)
    s0 = nuts._State(theta, r, logp, grad, lp)
    s1 = nuts._leapfrog(f, s0, eps)
    acc = min(1.0, math.exp(-(nuts._energy(s1) - nuts._energy(s0))))
    assert 0.25 <= acc <= 1.0 and eps > 0.0
