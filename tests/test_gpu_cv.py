"""GPU parity of the cross-validation bandwidth objectives (hbx_kde_cv_terms through
hpbandster_amd.cv.CVObjective) against statsmodels 0.12.2's outputs (tests/golden/cv_*.npz) and the
oracle's per-observation sums.

Tolerances: per-observation sums and objectives within 1e-13 relative (the GPU's exp and numpy's differ
by an ulp; summation order is the reference's); selected bandwidths within 1e-6 relative (Nelder-Mead
from the same start on objectives that agree to ~1e-15 follows the same path; the bound allows one
late tie-break to differ).
"""
import numpy as np
import pytest

from oracle import kde_oracle as O
from tests.test_oracle_cv import CASES, load

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", CASES)
def test_terms_match_oracle(device, name):
    from hpbandster_amd.cv import CVObjective
    c = load(name)
    vt = str(c["var_type"])
    obj = CVObjective(c["X"], vt, device=device)
    for p in c["bw_points"]:
        F, L = obj.terms(p)
        Fo, Lo = O.cv_terms(c["X"], p, vt)
        np.testing.assert_allclose(F, Fo, rtol=1e-13, atol=0)
        np.testing.assert_allclose(L, Lo, rtol=1e-13, atol=0)


@pytest.mark.parametrize("name", CASES)
def test_objectives_match_statsmodels(device, name):
    from hpbandster_amd.cv import CVObjective
    c = load(name)
    obj = CVObjective(c["X"], str(c["var_type"]), device=device)
    np.testing.assert_array_equal(obj.normal_reference(), c["h0"])
    for p, im, lo in zip(c["bw_points"], c["imse"], c["loo"]):
        np.testing.assert_allclose(obj.imse(p), im, rtol=1e-13)
        np.testing.assert_allclose(obj.loo_likelihood(p), lo, rtol=1e-13)


@pytest.mark.parametrize("name", CASES)
@pytest.mark.parametrize("method", ["cv_ls", "cv_ml"])
def test_bandwidth_selection_matches_statsmodels(device, name, method):
    from hpbandster_amd.cv import select_bandwidth
    c = load(name)
    bw = select_bandwidth(c["X"], str(c["var_type"]), method, device=device)
    np.testing.assert_allclose(bw, c["bw_" + method], rtol=1e-6)


def test_negative_and_large_bandwidths(device):
    """Nelder-Mead probes outside the valid range (h < 0, categorical h > 1); the kernel computes the
    reference's arithmetic there too (NaN/inf where statsmodels produces them)."""
    from hpbandster_amd.cv import CVObjective
    c = load("mixed")
    vt = str(c["var_type"])
    obj = CVObjective(c["X"], vt, device=device)
    for p in ([-0.1, 0.2, 0.5, 0.5], [0.1, 0.2, 1.3, -0.2], [0.3, 0.01, 0.99, 1.0]):
        p = np.array(p)
        F, L = obj.terms(p)
        Fo, Lo = O.cv_terms(c["X"], p, vt)
        np.testing.assert_allclose(F, Fo, rtol=1e-13, atol=0, equal_nan=True)
        np.testing.assert_allclose(L, Lo, rtol=1e-13, atol=0, equal_nan=True)


def test_single_level_and_singleton_columns(device):
    """A categorical column with one level (c - 1 = 0: the reference divides by zero) and one whose
    only other level is held by a single row (its leave-one-out column has one level)."""
    from hpbandster_amd.cv import CVObjective
    rs = np.random.RandomState(5)
    n = 40
    X = np.column_stack([rs.rand(n), np.zeros(n), np.zeros(n), rs.randint(0, 2, n)]).astype(float)
    X[7, 2] = 1.0
    vt = "cuuu"
    obj = CVObjective(X, vt, device=device)
    for p in ([0.2, 0.3, 0.4, 0.5], [0.05, 0.9, 0.1, 0.2]):
        p = np.array(p)
        F, L = obj.terms(p)
        Fo, Lo = O.cv_terms(X, p, vt)
        np.testing.assert_allclose(F, Fo, rtol=1e-13, atol=0, equal_nan=True)
        np.testing.assert_allclose(L, Lo, rtol=1e-13, atol=0, equal_nan=True)


def test_more_than_one_sum_buffer(device):
    """n > 8192: numpy's sum runs over 8192-element buffers; rows checked against the oracle."""
    from hpbandster_amd.cv import CVObjective
    rs = np.random.RandomState(9)
    n = 9000
    X = np.column_stack([rs.rand(n), rs.rand(n), rs.randint(0, 3, n)]).astype(float)
    vt = "ccu"
    obj = CVObjective(X, vt, device=device)
    p = O.normal_reference_bw(X)
    F, L = obj.terms(p)
    rows = [0, 1, 4095, 8191, 8192, 8999]
    Fo, Lo = O.cv_terms(X, p, vt, rows=rows)
    np.testing.assert_allclose(F[rows], Fo[rows], rtol=1e-13, atol=0)
    np.testing.assert_allclose(L[rows], Lo[rows], rtol=1e-13, atol=0)
    assert np.all(np.isfinite(F)) and np.all(F > 0) and np.all(L > 0)


def test_minimal_and_wide(device):
    """n = D + 1 (the smallest the reference accepts) and D = 32 (24c + 8u)."""
    from hpbandster_amd.cv import CVObjective
    rs = np.random.RandomState(3)
    for n, dc, du in ((4, 2, 1), (120, 24, 8)):
        X = np.column_stack([rs.rand(n, dc), rs.randint(0, 4, (n, du))]).astype(float)
        vt = "c" * dc + "u" * du
        obj = CVObjective(X, vt, device=device)
        p = O.normal_reference_bw(X)
        p[dc:] = np.minimum(p[dc:], 0.9)
        F, L = obj.terms(p)
        Fo, Lo = O.cv_terms(X, p, vt)
        np.testing.assert_allclose(F, Fo, rtol=1e-13, atol=0)
        np.testing.assert_allclose(L, Lo, rtol=1e-13, atol=0)


def test_rejects_bad_shapes(device):
    from hpbandster_amd.cv import CVObjective
    with pytest.raises(ValueError):
        CVObjective(np.zeros((3, 3)), "ccc", device=device)
    obj = CVObjective(np.random.rand(10, 2), "cc", device=device)
    with pytest.raises(ValueError):
        obj.terms([0.1])
