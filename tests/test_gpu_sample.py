"""GPU candidate sampler: distributional parity with BOHB's rule (bohb.py:133-147).

The reference draws from numpy's global RNG; the GPU draws from Philox, so parity is distributional:
* datum index ~ U{0..n-1}                                   (chi-square)
* continuous dim | datum m ~ scipy.stats.truncnorm(-m/bw, (1-m)/bw, loc=m, scale=3 bw)
  -- the reference's own distribution object as the CDF    (Kolmogorov-Smirnov)
* categorical dim | datum m: P(m) = (1-bw) + bw/t, P(other) = bw/t   (chi-square)
The draws are deterministic (seeded, counter-based), so the p-value thresholds cannot flake.
"""
import numpy as np
import pytest
import scipy.stats as sps

from tests import golden_cases as G

pytestmark = pytest.mark.gpu

P_MIN = 1e-4


def _pair(name):
    from hpbandster_amd import kde
    c = G.load_kde_case(name)
    pair = kde.fit_pair_from_rows(c["X"], c["good_idx"], c["bad_idx"], c["var_type"], c["bw_good"], c["bw_bad"],
                                  c["nlev_good"], c["nlev_bad"])
    return c, pair


def _levels(c, pair):
    # categorical dims: a choice count covering every code of the fixture
    return np.array([0 if t == "c" else int(np.nanmax(c["X"][:, d])) + 2 for d, t in enumerate(c["var_type"])])


def test_deterministic_and_counter_additive(device):
    c, pair = _pair("mixed8")
    lv = _levels(c, pair)
    a, da, _ = pair.good.sample(lv, 3.0, 1000, seed=123, counter_base=0)
    b, db, _ = pair.good.sample(lv, 3.0, 1000, seed=123, counter_base=0)
    assert np.array_equal(a.cpu().numpy(), b.cpu().numpy(), equal_nan=True)
    tail, dt, _ = pair.good.sample(lv, 3.0, 400, seed=123, counter_base=600)
    assert np.array_equal(a[600:].cpu().numpy(), tail.cpu().numpy(), equal_nan=True)
    assert np.array_equal(da[600:].cpu().numpy(), dt.cpu().numpy())
    other, _, _ = pair.good.sample(lv, 3.0, 1000, seed=124, counter_base=0)
    assert not np.array_equal(a.cpu().numpy(), other.cpu().numpy())


def test_datum_index_uniform(device):
    c, pair = _pair("mixed8")
    lv = _levels(c, pair)
    n = pair.good.nobs
    _, datum, _ = pair.good.sample(lv, 3.0, 200 * n, seed=5, counter_base=0)
    cnt = np.bincount(datum.cpu().numpy(), minlength=n)
    assert cnt.size == n
    assert sps.chisquare(cnt).pvalue > P_MIN


@pytest.mark.parametrize("name", ["mixed8", "d8c", "hgt1"])
def test_marginals_match_reference_distribution(device, name):
    c, pair = _pair(name)
    lv = _levels(c, pair)
    bw = pair.good.bw
    data = pair.good.data
    n = pair.good.nobs
    Nc = 4000 * n if n < 50 else 400000
    cands, datum, err = pair.good.sample(lv, 3.0, Nc, seed=77, counter_base=1 << 40)
    cands, datum = cands.cpu().numpy(), datum.cpu().numpy()
    assert not err.cpu().numpy().any()
    rs = np.random.RandomState(0)
    checked = 0
    for j in rs.choice(n, size=min(n, 4), replace=False):
        sel = cands[datum == j]
        assert len(sel) > 1000
        for d, t in enumerate(lv):
            m = data[j, d]
            x = sel[:, d]
            if t == 0:
                ref = sps.truncnorm(-m / bw[d], (1 - m) / bw[d], loc=m, scale=3.0 * bw[d])
                assert x.min() >= m - 3.0 * m - 1e-12 and x.max() <= m + 3.0 * (1 - m) + 1e-12  # the quirk's support
                assert sps.kstest(x, ref.cdf).pvalue > P_MIN, (name, j, d)
            else:
                h = bw[d]
                obs = np.bincount(x.astype(np.int64), minlength=t)[:t]
                assert obs.sum() == len(x)  # every draw is a valid level
                keep = min(max(1 - h, 0.0), 1.0)  # rand() < 1 - bw (never true for bw > 1)
                exp = np.full(t, (1 - keep) / t)
                exp[int(m)] += keep
                assert sps.chisquare(obs, exp * len(x)).pvalue > P_MIN, (name, j, d)
            checked += 1
    assert checked >= 4


def test_host_and_gpu_samplers_agree_in_distribution(device):
    """Two-sample KS between the reference rule on the host (global numpy RNG, scipy truncnorm) and
    the GPU draws, per continuous dim, pooled over data."""
    from hpbandster_amd import configspace as CS
    from hpbandster_amd.config_generators import BOHB
    c, pair = _pair("d8c")
    space = CS.ConfigurationSpace(seed=1)
    for d in range(8):
        space.add_hyperparameter(CS.UniformFloatHyperparameter("x%d" % d, lower=0, upper=1))
    cg = BOHB(space, device=device)
    np.random.seed(3)
    host = cg.sample_candidates(pair.good, 3000)
    gpu, _, _ = pair.good.sample(cg.vartypes, cg.bw_factor, 60000, seed=9, counter_base=0)
    gpu = gpu.cpu().numpy()
    for d in range(8):
        assert sps.ks_2samp(host[:, d], gpu[:, d]).pvalue > P_MIN, d


def test_domain_error_flags_nan_datum(device):
    from hpbandster_amd import kde
    rs = np.random.RandomState(2)
    X = rs.rand(40, 3)
    good = np.arange(0, 12)
    bad = np.arange(12, 40)
    bwg = np.array([0.2, 0.3, 0.25])
    pair = kde.fit_pair_from_rows(X, good, bad, "ccc", bwg, bwg, [0, 0, 0], [0, 0, 0])
    pair.good.X_dev[5, 1] = float("nan")  # an inactive (NaN) continuous value in a good row
    cands, datum, err = pair.good.sample([0, 0, 0], 3.0, 5000, seed=1, counter_base=0)
    datum, err = datum.cpu().numpy(), err.cpu().numpy()
    assert np.array_equal(err.astype(bool), datum == 5)
    assert err.any()


def _toy_bohb(device, sampler):
    from hpbandster_amd import configspace as CS
    from hpbandster_amd.config_generators import BOHB
    space = CS.ConfigurationSpace(seed=4)
    for i in range(3):
        space.add_hyperparameter(CS.UniformFloatHyperparameter("x%d" % i, lower=-1, upper=1))
    space.add_hyperparameter(CS.CategoricalHyperparameter("c", ["a", "b", "c"]))
    cg = BOHB(space, device=device, num_samples=256, sampler=sampler, sampler_seed=42)

    class Job(object):
        pass

    rs = np.random.RandomState(4)
    for k in range(30):
        cfg = space.sample_configuration().get_dictionary()
        j = Job()
        j.id, j.kwargs, j.exception, j.timestamps = (0, 0, k), {"config": cfg, "budget": 1.0}, None, {}
        j.result = {"loss": float(rs.rand()), "info": None}
        cg.new_result(j)
    return cg, space


def test_bohb_gpu_sampler_batch_equals_sequential(device):
    seq_cg, seq_space = _toy_bohb(device, "gpu")
    np.random.seed(1)
    seq = [seq_cg.get_config(1.0) for _ in range(20)]
    bat_cg, bat_space = _toy_bohb(device, "gpu")
    np.random.seed(1)
    bat = bat_cg.get_config_batch(1.0, 20)
    assert sum(i["model_based_pick"] for _, i in seq) >= 8
    assert seq == bat
    assert seq_cg._sample_counter == bat_cg._sample_counter > 0


def test_phi_table_gives_identical_draws(device):
    c, pair = _pair("mixed8")
    lv = _levels(c, pair)
    a, _, _ = pair.good.sample(lv, 3.0, 3000, seed=8, counter_base=17, table=True)
    b, _, _ = pair.good.sample(lv, 3.0, 3000, seed=8, counter_base=17, table=False)
    assert np.array_equal(a.cpu().numpy(), b.cpu().numpy(), equal_nan=True)


def test_norm_ppf_matches_scipy_ndtri(device):
    """The sampler's inversion routine (fp32 guess + one fp64 Halley step) against scipy's ndtri
    (the inverse scipy's truncnorm uses), over the whole range the sampler can hit."""
    import torch
    from scipy.special import ndtri
    from hpbandster_amd import _native as N
    p = np.concatenate([np.logspace(-300, -1, 4000), np.linspace(0.05, 0.95, 4001), 1 - np.logspace(-16, -1, 2000),
                        np.random.RandomState(1).rand(20000)])
    pd = torch.from_numpy(p).to(device)
    z = torch.empty_like(pd)
    N.check(N.lib().hbx_norm_ppf(N.ptr(pd), p.size, N.ptr(z), N.stream_handle()))
    z = z.cpu().numpy()
    ref = ndtri(p)
    err = np.abs(z - ref) / np.maximum(np.abs(ref), 1e-300)
    central = (p > 1e-300) & (np.abs(ref) > 1e-3)
    assert err[central].max() < 1e-12, err[central].max()
    assert np.abs(z - ref)[~central].max() < 1e-14


