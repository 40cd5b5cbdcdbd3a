"""NUTS driver for `gaplac mcmc` (BASELINE configs[0], CLI/src/mcmc.jl:31-44):

    chain = sample(inference_engine(y, x, formula, inferable), NUTS(0.65), samples)
    GaPLAC._df_output(chain, args)

The sampler is the host side of the mcmc path: every leapfrog step is ONE log density +
gradient evaluation (MCMCModel.logdensity_and_gradient -> gaplac_logpdf_grad on the GPU,
answered for all ForwardDiff chunks by one library call). It restates what Turing 0.21's
NUTS(0.65) does with it, in the unconstrained space Turing samples in:

  * ℓ ~ Uniform(0, 20) is mapped by Bijectors' logit transform, ℓ = 20 σ(u), and the log
    density gets the log-Jacobian log(20 σ(u) (1 - σ(u))); fx is unconstrained;
  * the no-U-turn sampler with multinomial sampling over the trajectory (AdvancedHMC's
    NUTS{MultinomialTS, GeneralisedNoUTurn}; the classic end-point U-turn test here), max
    tree depth 10, divergence at an energy error above 1000;
  * step size: AdvancedHMC's find_good_stepsize (a doubling / halving crossing search
    around acceptance 1/2 from ε = 0.1, then bisection into [1/4, 3/4]), then Nesterov dual averaging
    towards acceptance δ = 0.65 (γ = 0.05, t0 = 10, κ = 0.75) over n_adapts =
    min(samples ÷ 10, 1000) warm-up iterations (Turing's default), which are discarded.
    The metric stays the identity (Turing also adapts a diagonal metric in windows; that
    only changes efficiency, not the target distribution).

Output columns follow MCMCChains' table: iteration, chain, ℓ, fx[1..N], lp (Turing's :lp,
which `select --chains` reads: in Turing 0.21 / DynamicPPL 0.19 the HMC step stores the
sampler's log density, i.e. the log joint in the LINKED space including the logit
log-Jacobian, so lp == log_density), n_steps, is_accept,
acceptance_rate, log_density, hamiltonian_energy, hamiltonian_energy_error,
tree_depth, numerical_error, step_size, nom_step_size.
"""
from __future__ import annotations

import math
from typing import Callable, Dict, List, Optional, Tuple

import numpy as np

ELL_HI = 20.0
MAX_DEPTH = 10
MAX_DELTA_H = 1000.0


def _sigmoid(u: float) -> float:
    return 1.0 / (1.0 + math.exp(-u)) if u >= 0 else math.exp(u) / (1.0 + math.exp(u))


class Unconstrained:
    """θ = (u, fx) with ℓ = 20 σ(u): log density and gradient of the model in the space the
    sampler moves in (log joint + log-Jacobian of the logit bijection)."""

    def __init__(self, model):
        self.model = model
        self.calls = 0

    def to_theta(self, ell: float, fx) -> np.ndarray:
        p = ell / ELL_HI
        return np.concatenate([[math.log(p) - math.log1p(-p)], np.asarray(fx, dtype=np.float64)])

    def ell(self, theta) -> float:
        return ELL_HI * _sigmoid(float(theta[0]))

    def __call__(self, theta) -> Tuple[float, np.ndarray, float]:
        """(log density in θ, gradient, log joint in the constrained space)."""
        self.calls += 1
        u = float(theta[0])
        s = _sigmoid(u)
        ell = ELL_HI * s
        if not (0.0 < ell < ELL_HI):
            return -math.inf, np.full(theta.shape, math.nan), -math.inf
        lp, dell, dfx = self.model.logdensity_and_gradient(ell, theta[1:])
        logj = math.log(ELL_HI) + math.log(s) + math.log1p(-s)
        g = np.empty_like(theta)
        g[0] = dell * ell * (1.0 - s) + (1.0 - 2.0 * s)
        g[1:] = dfx
        return lp + logj, g, lp


class _State:
    __slots__ = ("theta", "r", "logp", "grad", "lp")

    def __init__(self, theta, r, logp, grad, lp):
        self.theta, self.r, self.logp, self.grad, self.lp = theta, r, logp, grad, lp


def _leapfrog(f, s: _State, eps: float) -> _State:
    r = s.r + 0.5 * eps * s.grad
    theta = s.theta + eps * r
    logp, grad, lp = f(theta)
    return _State(theta, r + 0.5 * eps * grad, logp, grad, lp)


def _uturn(left: _State, right: _State) -> bool:
    d = right.theta - left.theta
    return bool(np.dot(d, left.r) < 0.0 or np.dot(d, right.r) < 0.0)


def _energy(s: _State) -> float:
    return -s.logp + 0.5 * float(np.dot(s.r, s.r))


def _build(f, s: _State, v: int, depth: int, eps: float, H0: float, rng):
    """Subtree of 2^depth leapfrog steps from s in direction v:
    (left, right, proposal, log weight, stop, divergent, sum of acceptance stats, n)."""
    if depth == 0:
        s1 = _leapfrog(f, s, v * eps)
        H = _energy(s1) if math.isfinite(s1.logp) else math.inf
        dH = H - H0
        div = not (dH <= MAX_DELTA_H)
        acc = 0.0 if not math.isfinite(dH) else min(1.0, math.exp(-dH))
        return s1, s1, s1, (-dH if math.isfinite(dH) else -math.inf), div, div, acc, 1
    l1, r1, p1, w1, stop1, div1, a1, n1 = _build(f, s, v, depth - 1, eps, H0, rng)
    if stop1:
        return l1, r1, p1, w1, True, div1, a1, n1
    edge = r1 if v > 0 else l1
    l2, r2, p2, w2, stop2, div2, a2, n2 = _build(f, edge, v, depth - 1, eps, H0, rng)
    left, right = (l1, r2) if v > 0 else (l2, r1)
    w = np.logaddexp(w1, w2)
    prop = p2 if (math.isfinite(w2) and rng.uniform() < math.exp(w2 - w)) else p1
    stop = stop2 or _uturn(left, right)
    return left, right, prop, w, stop, div2, a1 + a2, n1 + n2


def nuts_transition(f, cur: _State, eps: float, rng) -> Tuple[_State, Dict[str, float]]:
    """One NUTS iteration from cur (theta, logp, grad known); returns the new state and its
    statistics."""
    d = cur.theta.shape[0]
    r0 = rng.standard_normal(d)
    s0 = _State(cur.theta, r0, cur.logp, cur.grad, cur.lp)
    H0 = _energy(s0)
    left = right = s0
    prop = s0
    logw = 0.0
    depth = 0
    acc_sum, n_tot, div = 0.0, 0, False
    while depth < MAX_DEPTH:
        v = 1 if rng.uniform() < 0.5 else -1
        if v > 0:
            _, right, p2, w2, stop, div, a, n = _build(f, right, v, depth, eps, H0, rng)
        else:
            left, _, p2, w2, stop, div, a, n = _build(f, left, v, depth, eps, H0, rng)
        acc_sum += a
        n_tot += n
        if not stop and math.isfinite(w2) and rng.uniform() < min(1.0, math.exp(w2 - logw)):
            prop = p2  # biased progressive sampling between the old tree and the new half
        logw = np.logaddexp(logw, w2)
        depth += 1
        if stop or _uturn(left, right):
            break
    H = _energy(_State(prop.theta, prop.r, prop.logp, prop.grad, prop.lp))
    stats = {"n_steps": n_tot, "is_accept": True, "acceptance_rate": acc_sum / max(n_tot, 1),
             "log_density": prop.logp, "hamiltonian_energy": H, "hamiltonian_energy_error": H - H0,
             "tree_depth": depth, "numerical_error": bool(div)}
    return _State(prop.theta, None, prop.logp, prop.grad, prop.lp), stats


def find_good_stepsize(f, cur: _State, rng, eps: float = 0.1, max_iters: int = 100) -> float:
    """AdvancedHMC 0.3's find_good_stepsize (what Turing's NUTS(0.65) calls when its initial
    ε is 0): from ε = 0.1, double (acceptance of one leapfrog step above 1/2) or halve it
    until the acceptance crosses 1/2, then bisect between the two neighbours until the
    acceptance lies in [1/4, 3/4]. Restated from the published algorithm (the package is
    not vendored in the reference); the constants are AdvancedHMC's defaults."""
    a_min, a_cross, a_max = 0.25, 0.5, 0.75
    r = rng.standard_normal(cur.theta.shape[0])
    s0 = _State(cur.theta, r, cur.logp, cur.grad, cur.lp)
    H0 = _energy(s0)

    def dH(e):  # H - H' (exp of it is the MH acceptance ratio)
        s1 = _leapfrog(f, s0, e)
        return -(_energy(s1) - H0) if math.isfinite(s1.logp) else -math.inf

    direction = 1 if dH(eps) > math.log(a_cross) else -1
    eps2 = eps
    for _ in range(max_iters):
        eps2 = 2.0 * eps if direction == 1 else 0.5 * eps
        d = dH(eps2)
        if (direction == 1 and not d > math.log(a_cross)) or (direction == -1 and not d < math.log(a_cross)):
            break
        eps = eps2
    lo, hi = (eps, eps2) if eps < eps2 else (eps2, eps)  # lo: high acceptance, hi: low
    for _ in range(max_iters):
        mid = 0.5 * (lo + hi)
        d = dH(mid)
        a = math.exp(min(d, 0.0)) if math.isfinite(d) else 0.0  # min(1, exp(dH))
        if a > a_max or d > 0.0:
            lo = mid
        elif a < a_min:
            hi = mid
        else:
            lo = mid
            break
    return lo


class DualAveraging:
    """Nesterov dual averaging of log ε towards the target acceptance δ (Hoffman & Gelman
    2014, Alg. 5)."""

    def __init__(self, eps0: float, delta: float = 0.65, gamma: float = 0.05, t0: float = 10.0,
                 kappa: float = 0.75):
        self.mu = math.log(10.0 * eps0)
        self.delta, self.gamma, self.t0, self.kappa = delta, gamma, t0, kappa
        self.hbar = 0.0
        self.logeps_bar = 0.0
        self.m = 0

    def update(self, acc: float) -> float:
        self.m += 1
        m = self.m
        self.hbar = (1 - 1 / (m + self.t0)) * self.hbar + (self.delta - acc) / (m + self.t0)
        logeps = self.mu - math.sqrt(m) / self.gamma * self.hbar
        eta = m ** -self.kappa
        self.logeps_bar = eta * logeps + (1 - eta) * self.logeps_bar
        return math.exp(logeps)

    def final(self) -> float:
        return math.exp(self.logeps_bar)


def sample(model, samples: int, seed: int = 0, delta: float = 0.65, n_adapts: Optional[int] = None,
           init: Optional[Tuple[float, np.ndarray]] = None,
           callback: Optional[Callable[[int, float], None]] = None) -> Dict[str, List]:
    """sample(model, NUTS(δ), samples) for an mcmc.MCMCModel. Returns the chain table."""
    rng = np.random.default_rng(seed)
    f = Unconstrained(model)
    N = model.N
    if n_adapts is None:
        n_adapts = min(samples // 10, 1000)
    if init is None:  # Turing's default initialisation: uniform in [-2, 2] in θ space
        theta = rng.uniform(-2.0, 2.0, N + 1)
    else:
        theta = f.to_theta(*init)
    logp, grad, lp = f(theta)
    cur = _State(theta, None, logp, grad, lp)
    eps = find_good_stepsize(f, cur, rng)
    da = DualAveraging(eps, delta)
    cols: Dict[str, List] = {"iteration": [], "chain": [], "ℓ": []}
    for i in range(N):
        cols[f"fx[{i + 1}]"] = []
    for k in ("lp", "n_steps", "is_accept", "acceptance_rate", "log_density", "hamiltonian_energy",
              "hamiltonian_energy_error", "tree_depth", "numerical_error", "step_size", "nom_step_size"):
        cols[k] = []
    for it in range(n_adapts + samples):
        step = eps
        cur, st = nuts_transition(f, cur, eps, rng)
        if it < n_adapts:
            eps = da.update(st["acceptance_rate"])
            if it == n_adapts - 1:
                eps = da.final()
            continue
        cols["iteration"].append(it + 1)
        cols["chain"].append(1)
        cols["ℓ"].append(f.ell(cur.theta))
        for i in range(N):
            cols[f"fx[{i + 1}]"].append(float(cur.theta[1 + i]))
        cols["lp"].append(cur.logp)  # Turing's :lp = the linked-space log density
        for k in ("n_steps", "is_accept", "acceptance_rate", "log_density", "hamiltonian_energy",
                  "hamiltonian_energy_error", "tree_depth", "numerical_error"):
            cols[k].append(st[k])
        cols["step_size"].append(step)
        cols["nom_step_size"].append(step)
        if callback is not None:
            callback(it, f.ell(cur.theta))
    cols["_density_calls"] = f.calls  # not a column: how many log density + gradient evaluations
    return cols


def run(formula: str, table, infer, samples: int, seed: int = 0, output: Optional[str] = None, ctx=None):
    """`gaplac mcmc FORMULA --data ... --samples n --infer v...` (CLI/src/mcmc.jl:10-44):
    build the model, sample, write the chain (src/utils.jl:30-40). Returns the chain."""
    from .mcmc import MCMCModel
    from .select import df_output
    model = MCMCModel(formula, table, infer, ctx=ctx)
    chain = sample(model, samples, seed=seed)
    calls = chain.pop("_density_calls")
    df_output(chain, output)
    chain["_density_calls"] = calls
    chain["_library_calls"] = model.memo.calls
    return chain
