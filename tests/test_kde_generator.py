"""KernelDensityEstimator (reference config_generators/kde.py) against the reference's own run.

tests/golden/kdegen_*.npz hold a seeded schedule of get_config / new_result calls through the
reference's methods (tests/golden/gen_kde_generator.py: statsmodels 0.12.2 cv_ls bandwidths).

* CPU: the host logic (training-set rule, borrowing from other budgets, refit cadence, proposals and
  their global-RNG consumption) with the recorded bandwidths standing in for the fit: refit steps
  exact; training data and proposal vectors within 1e-12 relative (scipy 1.15's truncnorm inversion
  differs from 1.7.1's in the last ulp; the RNG stream itself is the same).
* GPU: the whole generator, cv_ls bandwidths selected on the GPU (hbx_kde_cv_terms): same refits,
  training data within the proposals' tolerance, bandwidths within 1e-6 relative (Nelder-Mead's xtol=1e-3 stopping rule on objectives equal to
  ~1e-13), proposals within 1e-5 relative, same kinds.
"""
import os

import numpy as np
import pytest

from hpbandster_amd import configspace as CS
from hpbandster_amd.dispatch import Job

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CASES = ["d3", "d2"]


def _load(name):
    return dict(np.load(os.path.join(HERE, "kdegen_%s.npz" % name)))


def _space(D):
    space = CS.ConfigurationSpace(seed=11)  # gen_golden.make_space
    for d in range(D):
        space.add_hyperparameter(CS.UniformFloatHyperparameter("x%02d" % d, 0.0, 1.0))
    return space


def _run(c, gen, space, result_form):
    """Replay the fixture's schedule; returns (vectors, refits)."""
    budgets = list(c["budgets"])
    np.random.seed(int(c["seed"]))
    rs = np.random.RandomState(int(c["seed"]) + 100)
    vectors, refits = [], []
    for step in range(int(c["steps"])):
        b = budgets[step % len(budgets)]
        cfg, info = gen.get_config(b)
        vec = CS.Configuration(space, cfg).get_array()
        loss = float(np.sum((np.asarray(vec) - 0.3) ** 2) + 0.05 * rs.rand() / b)
        job = Job((0, 0, step), config=cfg, budget=b)
        job.result = {"result": {"loss": loss}} if result_form == "nested" else {"loss": loss, "info": {}}
        before = dict(gen.kde_models)
        gen.new_result(job)
        for bb, m in gen.kde_models.items():
            if before.get(bb) is not m:
                refits.append((step, bb, np.asarray(m.bw), np.asarray(m.data)))
        vectors.append(vec)
    return np.array(vectors), refits


def _refit_data(c):
    off = np.concatenate([[0], np.cumsum(c["refit_n"])])
    return [c["refit_data"][off[i]:off[i + 1]] for i in range(len(c["refit_n"]))]


@pytest.mark.parametrize("result_form", ["nested", "flat"])
@pytest.mark.parametrize("name", CASES)
def test_host_logic_with_recorded_bandwidths(name, result_form):
    from hpbandster_amd.config_generators.kde import CVKDEModel, KernelDensityEstimator
    c = _load(name)
    D = int(c["D"])
    space = _space(D)
    recorded = list(zip(c["refit_bw"], _refit_data(c)))
    seen = []

    class Replay(KernelDensityEstimator):
        def fit_model(self, train_data):
            bw, data = recorded[len(seen)]
            np.testing.assert_allclose(train_data, data, rtol=1e-12)  # the reference's training set
            seen.append(1)
            return CVKDEModel(train_data, bw, self.var_type)

    gen = Replay(space, top_n_percent=int(c["top_pct"]), update_after_n_points=int(c["update_after"]),
                 min_points_in_model=int(c["min_points"]))
    vectors, refits = _run(c, gen, space, result_form)
    assert len(seen) == len(recorded)
    assert [r[0] for r in refits] == list(c["refit_step"])
    assert [r[1] for r in refits] == list(c["refit_budget"])
    np.testing.assert_allclose(vectors, c["vectors"], rtol=1e-12)


def test_constructor_defaults():
    from hpbandster_amd.config_generators import KernelDensityEstimator
    space = _space(4)
    gen = KernelDensityEstimator(space)
    assert gen.min_points_in_model == 5 and gen.var_type == "cccc"
    assert gen.top_n_percent == 10 and gen.update_after_n_points == 50
    cfg, info = gen.get_config(1.0)  # no model: a prior sample, as a (dict, info) pair
    assert sorted(cfg) == ["x00", "x01", "x02", "x03"] and info == {}


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
def test_generator_on_gpu_matches_reference_run(device, name):
    from hpbandster_amd.config_generators.kde import KernelDensityEstimator
    c = _load(name)
    D = int(c["D"])
    space = _space(D)
    gen = KernelDensityEstimator(space, top_n_percent=int(c["top_pct"]),
                                 update_after_n_points=int(c["update_after"]),
                                 min_points_in_model=int(c["min_points"]), device=device)
    vectors, refits = _run(c, gen, space, "nested")
    assert [r[0] for r in refits] == list(c["refit_step"])
    for (step, b, bw, data), bw_ref, data_ref in zip(refits, c["refit_bw"], _refit_data(c)):
        np.testing.assert_allclose(data, data_ref, rtol=1e-5, atol=1e-9)
        np.testing.assert_allclose(bw, bw_ref, rtol=1e-6)
    np.testing.assert_allclose(vectors, c["vectors"], rtol=1e-5, atol=1e-9)
