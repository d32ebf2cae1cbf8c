"""The oracle (CPU restatement) against the golden fixtures generated from the reference."""
import numpy as np
import pytest

from oracle import kde_oracle as O
from tests import golden_cases as G


@pytest.mark.parametrize("name", G.kde_case_names())
def test_fit_matches_reference(name):
    c = G.load_kde_case(name)
    X, L = c["X"], c["eff_losses"]
    split = O.bohb_split(X, L, int(c["min_points"]))
    assert split is not None
    good, bad = split
    # the rows in the reference's own order, ties included (numpy 1.26.4's argsort, oracle/np_argsort.py)
    np.testing.assert_array_equal(good, c["good_idx"])
    np.testing.assert_array_equal(bad, c["bad_idx"])
    # bandwidths in the reference's own row order are bit-exact
    np.testing.assert_array_equal(O.normal_reference_bw(X[c["good_idx"]]), c["bw_good"])
    np.testing.assert_array_equal(O.normal_reference_bw(X[c["bad_idx"]]), c["bw_bad"])
    np.testing.assert_array_equal(O.num_levels(X[good], c["var_type"]), c["nlev_good"])
    np.testing.assert_array_equal(O.num_levels(X[bad], c["var_type"]), c["nlev_bad"])


@pytest.mark.parametrize("name", G.kde_case_names())
def test_pdf_and_selection_match_reference(name):
    c = G.load_kde_case(name)
    X, C = c["X"], c["cands"]
    if name == "d32m":
        C = C[:64]
    good, bad = X[c["good_idx"]], X[c["bad_idx"]]
    vt = c["var_type"]
    l = O.pdf_many(good, c["bw_good"], vt, C)
    g = O.pdf_many(bad, c["bw_bad"], vt, C)
    # this process's numpy exp differs from numpy 1.26.4's in the last ulp: products of D of them
    rtol = 1e-13 if X.shape[1] < 24 else 4e-13
    np.testing.assert_allclose(l, c["pdf_l"][:len(C)], rtol=rtol, atol=0, equal_nan=True)
    np.testing.assert_allclose(g, c["pdf_g"][:len(C)], rtol=rtol, atol=0, equal_nan=True)
    if len(C) == len(c["cands"]) and not name.startswith("neartie"):
        # (near ties are decided by the reference numpy's own exp rounding; this restatement uses the
        # process's numpy -- the C oracle's exact mode pins them, test_c_oracle_matches_reference)
        chosen, _ = O.select(l, g)
        assert chosen == c["chosen"]
    # the reference's own scores pick the recorded index (pins py_score/py_argmin)
    assert O.py_argmin([O.py_score(a, b) for a, b in zip(c["pdf_l"], c["pdf_g"])]) == c["chosen"]


@pytest.mark.parametrize("name", G.kde_case_names())
def test_log_pdf_restatement(name):
    c = G.load_kde_case(name)
    X, C = c["X"], c["cands"][:64]
    for rows, bw, ref in ((c["good_idx"], c["bw_good"], c["pdf_l"]), (c["bad_idx"], c["bw_bad"], c["pdf_g"])):
        lp = O.log_pdf_many(X[rows], bw, c["var_type"], C)
        ref = ref[:len(C)]
        with np.errstate(divide="ignore", invalid="ignore"):
            lref = np.where(ref > 0, np.log(ref), np.where(np.isnan(ref), np.nan, -np.inf))
        fin = np.isfinite(lref) & (ref > 1e-300)
        np.testing.assert_allclose(lp[fin], lref[fin], rtol=1e-9, atol=1e-9)
        assert np.array_equal(np.isnan(lp), np.isnan(lref))


@pytest.mark.parametrize("which", ["sh_promotion", "sh_ties"])
def test_sh_promotion_matches_reference(which):
    for c in G.load_sh(which):
        losses = np.where(c["crashed"], np.nan, c["losses"])
        adv = O.sh_advance(losses, c["k"])
        np.testing.assert_array_equal(adv, c["sh_adv"])
        assert adv.sum() == c["sh_count"]
        k_sr = max(1, c["k"] * (1 - 0.5))
        adv = O.sh_advance(losses, k_sr)
        np.testing.assert_array_equal(adv, c["sr_adv"])


def test_np_argsort_restatement_known_answers():
    """numpy 1.26.4's own argsort of tie-heavy float64 arrays (+-inf, +-0, NaN, quantised, sorted,
    periodic, sizes 1..10000: the bitonic networks, both partitions, the std::sort fallbacks)."""
    from oracle import np_argsort as NA
    z = np.load(G.GOLDEN + "/np_argsort.npz")
    assert str(z["numpy"]) == "1.26.4" and bool(z["avx512_skx"])
    x, order, off = z["x"], z["order"], z["off"]
    for i in range(off.size - 1):
        a = x[off[i]:off[i + 1]]
        np.testing.assert_array_equal(NA.argsort(a), order[off[i]:off[i + 1]], err_msg="case %d n=%d" % (i, a.size))


def test_hb_brackets_match_reference():
    for t in G.load_brackets():
        m, budgets = O.hb_budgets(t["eta"], t["min_budget"], t["max_budget"])
        assert m == t["max_SH_iter"]
        # np.power differs by <=1 ulp between numpy 1.26 (fixture) and 2.x for non-integer eta
        np.testing.assert_allclose(budgets, np.array(t["budgets"]), rtol=5e-16, atol=0)
        for it in t["iterations"]:
            s, ns = O.hb_bracket(it["it"], t["eta"], m)
            assert ns == it["num_configs"]
            np.testing.assert_allclose(budgets[(-s - 1):], np.array(it["budgets"]), rtol=5e-16, atol=0)


@pytest.mark.parametrize("name", G.kde_case_names())
def test_c_oracle_matches_reference(name):
    """Fast mode (libm exp, sequential sums; the CPU baseline) to rounding; exact mode (numpy 1.26.4's
    exp and pairwise sums) bit for bit, and the reference's chosen index from both."""
    from oracle import c_oracle
    c = G.load_kde_case(name)
    X, C = c["X"], c["cands"]
    for exact in (False, True):
        l = c_oracle.kde_pdf(X[c["good_idx"]], c["bw_good"], c["var_type"], c["nlev_good"], C, exact=exact)
        g = c_oracle.kde_pdf(X[c["bad_idx"]], c["bw_bad"], c["var_type"], c["nlev_bad"], C, exact=exact)
        if exact:
            np.testing.assert_array_equal(l, c["pdf_l"])
            np.testing.assert_array_equal(g, c["pdf_g"])
            assert c_oracle.bohb_select(l, g)[0] == c["chosen"]
        else:
            np.testing.assert_allclose(l, c["pdf_l"], rtol=1e-12, atol=0, equal_nan=True)
            np.testing.assert_allclose(g, c["pdf_g"], rtol=1e-12, atol=0, equal_nan=True)
            if not name.startswith("neartie"):  # near ties are decided by the reference's own rounding
                assert c_oracle.bohb_select(l, g)[0] == c["chosen"]


def test_c_oracle_np_exp_known_answers():
    """The oracle's restatement of numpy 1.26.4's float64 exp (SVML) against that numpy's outputs."""
    from oracle import c_oracle
    z = np.load(G.GOLDEN + "/np_exp.npz")
    assert str(z["numpy"]) == "1.26.4"
    np.testing.assert_array_equal(c_oracle.np_exp(z["x"]).view(np.uint64), z["y"].view(np.uint64))
