"""GPU: the reference's threading: the Pyro dispatcher thread runs new_result -- the KDE
refit -- without the master's lock while the main thread runs get_config (HB_master.py:192-208,
dispatcher.py:303).  The engine must be reentrant and a model swap atomic: every get_config must see
one whole (good, bad) snapshot and pick exactly what acquiring on that snapshot picks."""
import threading

import numpy as np
import pytest

from hpbandster_amd import configspace as CS
from hpbandster_amd.dispatch import Job

pytestmark = pytest.mark.gpu


def _space(D):
    space = CS.ConfigurationSpace(seed=3)
    for d in range(D):
        space.add_hyperparameter(CS.UniformFloatHyperparameter("x%02d" % d, 0.0, 1.0))
    return space


def test_new_result_thread_races_get_config(device, monkeypatch):
    from hpbandster_amd import kde
    from hpbandster_amd.config_generators.bohb import BOHB
    D = 6
    space = _space(D)
    cg = BOHB(space, random_fraction=0.0, num_samples=256, device=device)
    rs = np.random.RandomState(5)
    X = rs.rand(400, D)
    L = ((X - 0.4) ** 2).sum(1) + 0.01 * rs.rand(400)

    def feed(lo, hi):
        for i in range(lo, hi):
            job = Job((0, 0, i), config=CS.Configuration(space, vector=X[i]).get_dictionary(), budget=1.0)
            job.result = {"loss": float(L[i]), "info": None}
            cg.new_result(job)

    feed(0, 40)  # a first model
    seen = []
    orig = kde.KDEPair.acquire
    orig_mapped = kde.KDEPair.acquire_mapped  # (the host sampler's call: candidates in mapped host memory)

    def recording_acquire(self, cands, *a, **k):
        res = orig_mapped(self, cands, *a, **k)
        seen.append((self, np.array(cands, copy=True), res))
        return res

    monkeypatch.setattr(kde.KDEPair, "acquire_mapped", recording_acquire)
    errors = []

    def dispatcher():
        try:
            feed(40, 400)
        except Exception as e:  # pragma: no cover - reported below
            errors.append(e)

    t = threading.Thread(target=dispatcher)
    np.random.seed(7)
    picks = []
    t.start()
    while t.is_alive() or len(picks) < 50:
        cfg, info = cg.get_config(1.0)
        picks.append((cfg, info))
        if len(picks) > 2000:
            break
    t.join(120)
    assert not errors, errors
    assert len(set(id(p) for p, _, _ in seen)) > 3, "the model must have been swapped while sampling"
    assert all(info["model_based_pick"] for _, info in picks)
    # each pick: the acquisition on the snapshot it saw, bit for bit, and the returned configuration
    for (pair, cands, res), (cfg, _) in zip(seen, picks):
        again = orig(pair, cands)
        assert (again.index, again.score) == (res.index, res.score)
        np.testing.assert_allclose(CS.Configuration(space, cfg).get_array(), cands[res.index], rtol=1e-15)


def test_refit_on_other_thread_and_stream_is_identical(device):
    """A refit enqueued from another thread on an explicit stream gives the same model as one on the
    main thread's current stream (the engine takes the tensors' device stream, not the thread's)."""
    import torch
    from hpbandster_amd import kde
    from hpbandster_amd import synthetic as S
    X = S.make_observations(3000, 16, 4, 3)
    L = S.make_losses(3000)
    vt = S.var_type_string(16, 4)
    a = kde.fit_pair(X, L, vt, 21, device=device)
    out = {}

    def other():
        s = torch.cuda.Stream(device=device)
        out["pair"] = kde.fit_pair(X, L, vt, 21, device=device, stream=s)
        s.synchronize()

    t = threading.Thread(target=other)
    t.start()
    t.join(120)
    b = out["pair"]
    C = S.make_candidates(5000, 16, 4, 3)
    Cd = torch.from_numpy(C).to(device)
    for ka, kb in ((a.good, b.good), (a.bad, b.bad)):
        np.testing.assert_array_equal(ka.bw, kb.bw)
        np.testing.assert_array_equal(ka.rows_dev.cpu().numpy(), kb.rows_dev.cpu().numpy())
        assert ka.variant == kb.variant
        for ea, eb in zip(ka.logpdf_est(Cd), kb.logpdf_est(Cd)):  # same tables -> same fp32 sums
            np.testing.assert_array_equal(ea, eb)
    ra, rb = a.acquire(C), b.acquire(C)
    assert (ra.index, ra.score) == (rb.index, rb.score)
