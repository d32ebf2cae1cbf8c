"""Seeded synthetic inputs for the KDE acquisition and promotion workloads.

Shared by the golden-fixture generator (run under the oracle interpreter), the tests and
``bench.py``.  Only the legacy ``numpy.random.RandomState`` stream is used, which is frozen
across numpy releases, so the same seed reproduces the same arrays bit for bit under
numpy 1.26 (oracle interpreter) and numpy 2.2 (engine interpreter).

Seeds follow SURVEY.md section 8(d): observations = 1, losses = 2, candidates = 3.
Continuous dims are U[0,1); categorical dims are integer codes ``randint(0, L)`` stored as
float64, exactly what ``Configuration.get_array()`` yields for a categorical hyperparameter.
Continuous columns come first, then categorical columns (the order a name-sorted
configuration space with ``x*`` continuous and ``y*`` categorical names produces).
"""

import hashlib

import numpy as np

SEED_OBS = 1
SEED_LOSS = 2
SEED_CAND = 3


def _levels_list(du, levels):
    if np.isscalar(levels):
        return [int(levels)] * du
    levels = [int(l) for l in levels]
    if len(levels) != du:
        raise ValueError("need one level count per categorical dim")
    return levels


def make_points(rs, n, dc, du, levels):
    """n points: dc U[0,1) columns followed by du integer-code columns (float64)."""
    lv = _levels_list(du, levels)
    xc = rs.rand(n, dc) if dc else np.zeros((n, 0))
    xu = np.empty((n, du))
    for d in range(du):
        xu[:, d] = rs.randint(0, lv[d], size=n)
    return np.ascontiguousarray(np.hstack([xc, xu]), dtype=np.float64)


def make_observations(n_obs, dc, du, levels, seed=SEED_OBS):
    return make_points(np.random.RandomState(seed), n_obs, dc, du, levels)


def make_losses(n_obs, seed=SEED_LOSS):
    losses = np.random.RandomState(seed).rand(n_obs)
    if np.unique(losses).size != n_obs:
        raise AssertionError("synthetic losses must be tie-free")
    return losses


def make_candidates(n_cand, dc, du, levels, seed=SEED_CAND):
    return make_points(np.random.RandomState(seed), n_cand, dc, du, levels)


CAND_BLOCK = 1 << 16


def make_candidates_blocked(lo, hi, dc, du, levels, seed=SEED_CAND):
    """Rows [lo, hi) of an unbounded seeded candidate stream: block b (rows b*CAND_BLOCK ...) is
    ``make_points(RandomState([seed, b]), CAND_BLOCK, ...)``.  Any slice is reproducible without drawing
    the rows before it, so every rank of a sharded run draws only its own shard, the weak-scaling set at N
    ranks (rank r: rows [r Nc, (r+1) Nc)) is a prefix of config #4's 1e7 set, and the oracle's full-size
    winners (tests/golden/full_winners.json) cover every rank count from one scan."""
    if hi < lo or lo < 0:
        raise ValueError("bad row range")
    out = np.empty((hi - lo, dc + du))
    b0, b1 = lo // CAND_BLOCK, (hi + CAND_BLOCK - 1) // CAND_BLOCK
    for b in range(b0, b1):
        blk = make_points(np.random.RandomState([seed, b]), CAND_BLOCK, dc, du, levels)
        r0, r1 = max(lo, b * CAND_BLOCK), min(hi, (b + 1) * CAND_BLOCK)
        out[r0 - lo:r1 - lo] = blk[r0 - b * CAND_BLOCK:r1 - b * CAND_BLOCK]
    return out


def var_type_string(dc, du):
    return "c" * dc + "u" * du


def bohb_split_sizes(n, min_points, top_n_percent=15):
    """Good/bad row counts of BOHB.new_result (reference bohb.py:224-225)."""
    n_good = max(min_points, (top_n_percent * n) // 100)
    n_bad = max(min_points, ((100 - top_n_percent) * n) // 100)
    return n_good, n_bad


def make_bracket_losses(n_brackets, n_configs, seed=SEED_LOSS):
    """[B, n] fp64 losses, tie-free within every bracket (config #5)."""
    rs = np.random.RandomState(seed)
    losses = rs.rand(n_brackets, n_configs)
    return losses


def sha256_array(a):
    a = np.ascontiguousarray(a)
    h = hashlib.sha256()
    h.update(str(a.dtype).encode())
    h.update(str(a.shape).encode())
    h.update(a.tobytes())
    return h.hexdigest()
