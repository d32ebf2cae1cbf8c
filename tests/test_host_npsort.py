"""CPU: libhbx's host restatement of numpy 1.26.4's np.argsort (hbx_np_argsort_host, hbx_sh_advance_host)
-- the one-bracket promotion with tied losses across the k-th place (HB_iteration.py:180-182) -- against
numpy 1.26.4's own outputs (tests/golden/np_argsort.npz: 206 arrays, random, few-distinct, all-equal,
+-0, +-inf, NaN, sizes 1 ... 20000), the reference's tied promotion masks (sh_ties.npz) and the Python
restatement (oracle/np_argsort.py) on random tie-heavy brackets; and the drop-in's advance_mask policy."""
import os

import numpy as np
import pytest

from hpbandster_amd import _native as N
from hpbandster_amd import promote

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def host_argsort(x):
    x = np.ascontiguousarray(x, dtype=np.float64)
    o = np.empty(x.shape[0], dtype=np.int64)
    N.check(N.lib().hbx_np_argsort_host(x.ctypes.data, x.shape[0], o.ctypes.data))
    return o


def test_known_answers_numpy_1_26_4():
    z = np.load(os.path.join(GOLDEN, "np_argsort.npz"))
    x, order, off = z["x"], z["order"], z["off"]
    for j in range(len(off) - 1):
        a, b = off[j], off[j + 1]
        assert np.array_equal(host_argsort(x[a:b]), order[a:b]), j


@pytest.mark.parametrize("seed", range(6))
def test_matches_python_restatement_on_tied_brackets(seed):
    from oracle import np_argsort as NA
    rs = np.random.RandomState(seed)
    for n in (2, 9, 63, 64, 65, 200, 257, 300, 1000, 3001):
        x = np.round(rs.rand(n), int(rs.randint(0, 3)))
        if seed % 3 == 1:
            x[rs.rand(n) < 0.2] = np.inf
        if seed % 3 == 2:
            x[rs.rand(n) < 0.05] = np.nan
        assert np.array_equal(host_argsort(x), NA.argsort(x)), n


def test_reference_tied_promotions():
    """sh_ties.npz / sh_promotion.npz: the reference's own SuccessiveHalving and SuccessiveResampling masks
    (tied losses across the k-th place, crashed runs) through the drop-in's host policy."""
    from tests import golden_cases as G
    n = 0
    for which in ("sh_ties", "sh_promotion"):
        for c in G.load_sh(which):
            losses = np.where(c["crashed"], np.nan, c["losses"])
            assert np.array_equal(promote.advance_mask(losses, c["k"]), c["sh_adv"])
            assert np.array_equal(promote.advance_mask(losses, max(1, c["k"] * (1 - 0.5))), c["sr_adv"])
            n += 1
    assert n > 10


def test_advance_host_equals_mask_of_first_k():
    from oracle import np_argsort as NA
    rs = np.random.RandomState(3)
    for n in (81, 1000, 4096):
        x = np.round(rs.rand(n), 1)
        for k in (1, n // 3, n // 2, n - 1):
            adv = np.empty(n, dtype=np.bool_)
            scr = np.empty(n, dtype=np.int64)
            N.check(N.lib().hbx_sh_advance_host(x.ctypes.data, n, k, adv.ctypes.data, scr.ctypes.data))
            assert np.array_equal(adv, NA.ranks_advance(x, k))
            assert np.array_equal(promote.advance_mask(x, k), adv)  # the drop-in's policy takes this path
