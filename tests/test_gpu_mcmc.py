"""BASELINE configs[0] on the GPU: `./gaplac mcmc "y ~| SqExp(:x)" --data data.tsv
--samples 500 --infer x` on N = 50 observations (README.md "Fitting parameters";
CLI/src/mcmc.jl:10-44), every leapfrog step's log density + gradient through
gaplac_logpdf_grad (one library call per step).

* The full 500-sample run: the chain table, ℓ inside its prior's support, finite :lp, one
  library call per density evaluation, and `select --chains` on the written file.
* The sampler driven by the GPU and by the oracle from the same seed follows the same
  trajectory: the first iterations' ℓ agree to 1e-6 (the densities agree to ~1e-15; the
  tree building only compares them).
"""
import math

import numpy as np
import pytest

from gaplac_amd import nuts
from gaplac_amd.backend import Context
from gaplac_amd.mcmc import MCMCModel
from tests.conftest import gpu_available
from tests.test_nuts import _OracleCtx, config0_table

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    if not gpu_available():
        pytest.skip("no GPU")
    c = Context(0)
    yield c
    c.close()


def test_config0_mcmc_500_samples(ctx, tmp_path):
    out = tmp_path / "mcmc.tsv"
    chain = nuts.run("y ~| SqExp(:x)", config0_table(50), ["x"], 500, seed=7, output=str(out), ctx=ctx)
    ell = np.array(chain["ℓ"])
    assert len(ell) == 500 and np.all((ell > 0) & (ell < 20))
    assert np.all(np.isfinite(chain["lp"]))
    assert chain["_library_calls"] == chain["_density_calls"]
    assert np.mean(chain["acceptance_rate"]) > 0.3
    from gaplac_amd.select import select_chains
    bayes, lp1, _ = select_chains(str(out), str(out))
    assert bayes == 0.0 and math.isfinite(lp1)


def test_gpu_and_oracle_density_drive_the_same_chain(ctx):
    table = config0_table(50, seed=3)
    gpu = nuts.sample(MCMCModel("y ~| SqExp(:x)", table, ["x"], ctx=ctx), 15, seed=11, n_adapts=10)
    ref = nuts.sample(MCMCModel("y ~| SqExp(:x)", table, ["x"], ctx=_OracleCtx()), 15, seed=11, n_adapts=10)
    assert np.allclose(gpu["ℓ"], ref["ℓ"], rtol=1e-6, atol=0)
    assert np.allclose(gpu["lp"], ref["lp"], rtol=1e-6, atol=0)
    assert gpu["tree_depth"] == ref["tree_depth"]
