"""Generate the golden fixtures in tests/golden/*.json from the CPU restatement.

Run from the repo root:  python tests/golden/make_golden.py

Inputs are seeded synthetic draws (SURVEY.md §8c case list) and the reference's own
input data files test/testin/input_pair_{109,1609}.tsv (copied verbatim into
tests/golden/data/). Expected outputs come from oracle/restatement.py, which is
"parity unpinned" (no Julia here; see its header). Floats are stored with float.hex()
so they round-trip exactly. Each case also records the Distances.jl-style (gemm
distance) logpdf, to show the size of the distance-rounding ambiguity the 1e-9
tolerance covers.
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import restatement as R  # noqa: E402
from gaplac_amd import formula as F, kernels as K  # noqa: E402
from gaplac_amd.abstractgps import design_matrix  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")


def hexs(a):
    return [float(x).hex() for x in np.ravel(a, order="F")]


def read_tsv(path):
    import pandas as pd
    df = pd.read_csv(path, sep="\t")
    df = df.dropna()  # select.jl:38-39: disallowmissing(df[completecases(df), :])
    return {c: df[c].to_numpy() for c in df.columns if c != "SampleID"}


def case(name, X, terms, noise, v, formula=None, vars_=None, note=""):
    X = np.asarray(X, dtype=np.float64)
    if X.ndim == 1:
        X = X[:, None]
    v = np.asarray(v, dtype=np.float64)
    rec = {"name": name, "formula": formula, "vars": vars_, "note": note, "N": int(X.shape[0]),
           "D": int(X.shape[1]), "noise": float(noise).hex(),
           "terms": [[int(k), int(c), float(p).hex(), int(g)] for (k, c, p, g) in terms],
           "X": hexs(X), "v": hexs(v)}
    C = R.gram(X, terms, noise)
    rec["gram_sum"] = float(C.sum()).hex()
    rec["gram_diag_sum"] = float(np.trace(C)).hex()
    try:
        lp, ld, q = R.logpdf(X, terms, noise, v)
        rec.update(info=0, logpdf=lp.hex(), logdet=ld.hex(), quad=q.hex())
        # gradient (gaplac_logpdf_grad): d/dv, d/dparam per term, d/dnoise, and the
        # per-entry magnitude scale the parity tolerance is stated against
        _, dv, dparam, dnoise = R.logpdf_grad(X, terms, noise, v)
        sc, scn = R.logpdf_grad_scale(X, terms, noise, v)
        rec.update(dv=hexs(dv), dparam=hexs(dparam), dnoise=float(dnoise).hex(),
                   dparam_scale=hexs(sc), dnoise_scale=float(scn).hex())
        try:
            lpg, _, _ = R.logpdf(X, terms, noise, v, distances="gemm")
            rec["logpdf_gemm_distances"] = lpg.hex()
            rec["gemm_rel_diff"] = abs(lpg - lp) / abs(lp)
        except R.PosDefException:
            pass
    except R.PosDefException as e:
        rec.update(info=e.info, logpdf=None, logdet=None, quad=None)
    return rec


def main():
    cases = []
    # (1) SqExp l in {1, 1.5, 0.3}, N in {50, 256, 1024}, x ~ U(-5, 5)
    for N in (50, 256, 1024):
        for l in (1.0, 1.5, 0.3):
            rng = np.random.default_rng(1000 + N)
            x = rng.uniform(-5, 5, N)
            y = rng.standard_normal(N)
            f = f"y ~| SqExp(:x; l={l})"
            terms, vars_ = K.lower_formula(F.gp_spec(f).formula)
            cases.append(case(f"sqexp_N{N}_l{l}", x, terms, 0.1, y, f, vars_))
    # (2) reference data: test/testin/input_pair_109.tsv (N=921), bug as the response
    tab = read_tsv(os.path.join(OUT, "data", "input_pair_109.tsv"))
    for f in ("bug ~| OU(:nutrient; l=1.5)", "bug ~| Linear(:nutrient)", "bug ~| Linear(:nutrient; c=2)",
              "bug ~| Cat(:PersonID)", "bug ~| Cat(:PersonID) + Linear(:nutrient) + SqExp(:Date; l=30)",
              "bug ~| Cat(:StoolPairs) + OU(:Date; l=100)"):
        sp = F.gp_spec(f)
        terms, vars_ = K.lower_formula(sp.formula)
        X = design_matrix(tab, vars_)
        cases.append(case("pair109:" + f, X, terms, 0.1, tab[F.response(sp)], f, vars_))
    # input_pair_1609.tsv has 2 missing Dates -> completecases -> N = 921
    tab2 = read_tsv(os.path.join(OUT, "data", "input_pair_1609.tsv"))
    f = "bug ~| SqExp(:Date; l=50) + Cat(:PersonID)"
    sp = F.gp_spec(f)
    terms, vars_ = K.lower_formula(sp.formula)
    cases.append(case("pair1609:" + f, design_matrix(tab2, vars_), terms, 0.1, tab2["bug"], f, vars_,
                      note="completecases drops the 2 rows with missing Date"))
    # (3) composite SqExp + OU + Cat + Noise (extension: Noise, duplicated :t)
    rng = np.random.default_rng(2)
    N = 700
    t = rng.uniform(0, 10, N)
    subj = rng.integers(0, N // 3, N).astype(float)
    v = rng.standard_normal(N)
    f = "y ~| SqExp(:t; l=1.5) + OU(:t; l=3) + Cat(:subject) + Noise"
    terms, vars_ = K.lower_formula(F.gp_spec(f).formula)
    cases.append(case("composite_N700", np.column_stack([t, t, subj]), terms, 0.1, v, f, vars_,
                      note="extension: Noise = 1.0*delta_ij by index; SqExp(:t)+OU(:t) reuses :t (SURVEY Q3)"))
    # (4) non-PD known answers: Cat-only, no noise -> the first repeated level is an
    #     exactly-zero pivot (all arithmetic exact in 0/1), info = its 1-based position
    cats = np.array([3, 1, 4, 5, 9, 2, 6, 8, 7, 0, 11, 12, 4, 13], dtype=float)
    cases.append(case("nonpd_cat_no_noise", cats, [(R.CAT, 0, 0.0, 0)], 0.0, np.ones(len(cats)),
                      "y ~| Cat(:g)", ["g"], note="level 4 repeats at position 13 -> info 13"))
    cats2 = np.concatenate([np.arange(300.0), [17.0], np.arange(300.0, 420.0)])
    cases.append(case("nonpd_cat_block3", cats2, [(R.CAT, 0, 0.0, 0)], 0.0, np.ones(len(cats2)),
                      "y ~| Cat(:g)", ["g"], note="repeat at position 301 (third 128-block) -> info 301"))
    # (5) top-level product: reference lowering (sum, Q1) and the product extension
    rng = np.random.default_rng(5)
    N = 300
    a = rng.uniform(-3, 3, N)
    b = rng.integers(0, 20, N).astype(float)
    v = rng.standard_normal(N)
    f = "y ~| SqExp(:a) * Cat(:b)"
    terms, vars_ = K.lower_formula(F.gp_spec(f).formula)
    cases.append(case("toplevel_product_as_reference", np.column_stack([a, b]), terms, 0.1, v, f, vars_,
                      note="reference kernel() sums the factors of a top-level product (SURVEY Q1)"))
    terms, vars_ = K.lower_formula(F.gp_spec(f).formula, products=True)
    cases.append(case("toplevel_product_extension", np.column_stack([a, b]), terms, 0.1, v, f, vars_,
                      note="extension: true Hadamard product"))
    f = "y ~| SqExp(:a) * Cat(:b) + Linear(:a; c=0.5) + OU(:a; l=0.7) * SqExp(:a; l=2)"
    terms, vars_ = K.lower_formula(F.gp_spec(f).formula, products=True)
    cases.append(case("nested_products_extension", np.column_stack([a, b, a, a, a]), terms, 0.1, v, f, vars_,
                      note="extension: nested products (the reference errors, Q1)"))
    # (6) edges: N=1, N=2, padding boundaries 127/128/129
    for N in (1, 2, 127, 128, 129):
        rng = np.random.default_rng(77 + N)
        x = rng.uniform(-5, 5, N)
        v = rng.standard_normal(N)
        terms = [(R.SQEXP, 0, 1.5, 0), (R.LINEAR, 0, 0.25, 1)]
        cases.append(case(f"edge_N{N}", x, terms, 0.1, v, "y ~| SqExp(:x; l=1.5) + Linear(:x; c=0.25)", ["x", "x"]))
    for c in cases:
        fn = "case_" + "".join(ch if ch.isalnum() else "_" for ch in c["name"])[:80] + ".json"
        with open(os.path.join(OUT, fn), "w") as fh:
            json.dump(c, fh)
    with open(os.path.join(OUT, "index.json"), "w") as fh:
        json.dump(sorted("case_" + "".join(ch if ch.isalnum() else "_" for ch in c["name"])[:80] + ".json"
                         for c in cases), fh, indent=1)
    print(f"wrote {len(cases)} cases")
    for c in cases:
        print(f"  {c['name'][:70]:70s} N={c['N']:5d} info={c['info']} logpdf={float.fromhex(c['logpdf']) if c['logpdf'] else None} gemm_rel={c.get('gemm_rel_diff')}")


if __name__ == "__main__":
    main()
