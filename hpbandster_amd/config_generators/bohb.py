"""BOHB -- drop-in for hpbandster/config_generators/bohb.py with the KDE work on the MI355X.

Same constructor kwargs, same ``get_config`` / ``new_result`` behaviour and the same consumption of
the global numpy RNG (``np.random.rand`` / ``randint`` and ``scipy.stats.truncnorm.rvs``, in the
reference's order), so a seeded run proposes the same configurations.  What moved to the GPU:

* ``new_result``: the per-budget refit (argsort of the losses, good/bad split, normal-reference
  bandwidths, observed level counts -- bohb.py:220-246) runs in libhbx.so (``kde.fit_pair``);
* ``get_config``: the ``num_samples`` candidates are scored against l (good) and g (bad) and the
  first index of min max(1e-8, g)/max(l, 1e-8) is selected exactly (bohb.py:124-161) by
  ``KDEPair.acquire`` -- fp32 matrix-core scoring of every candidate, fp64 re-score of the ones that
  can still be the minimum.

``kde_models[budget]`` holds a ``KDEPair`` whose ``['good']`` / ``['bad']`` expose ``.data``,
``.bw`` and ``.pdf`` like the statsmodels objects of the reference.
"""

import traceback

import numpy as np
import scipy.stats as sps

from .. import _native
from ..kde import ObservationStore
from .base import base_config_generator
from ._cs import ConfigSpace


def _rng_snapshot(gen):
    return (np.random.get_state(), gen.configspace.random.get_state(), gen._sample_counter)


def _rng_same(a, b):
    """Two snapshots of (global RNG, configspace RNG, GPU sampler counter) equal."""
    for x, y in ((a[0], b[0]), (a[1], b[1])):
        if x[0] != y[0] or x[2:] != y[2:] or not np.array_equal(x[1], y[1]):
            return False
    return a[2] == b[2]


def _rng_set(gen, snap):
    np.random.set_state(snap[0])
    gen.configspace.random.set_state(snap[1])
    gen._sample_counter = snap[2]


class SpeculativeBatch(object):
    """get_config results computed ahead in one batched acquisition (BOHB.get_config_batch_spec)."""

    def __init__(self, gen, out, before, after, version):
        self.gen, self.out, self.after, self.version = gen, out, after, version
        self.served = 0
        _rng_set(gen, before)  # nothing consumed yet: pop() moves the RNGs call by call

    def valid(self):
        """The next result is exactly the sequential call's: same model, RNGs where the last call left them."""
        g = self.gen
        if self.served >= len(self.out) or g._model_version != self.version:
            return False
        if self.served == 0:
            return True
        return _rng_same(_rng_snapshot(g), self.after[self.served - 1])

    def pop(self):
        r = self.out[self.served]
        _rng_set(self.gen, self.after[self.served])
        self.served += 1
        return r


class BOHB(base_config_generator):
    def __init__(self, configspace, min_points_in_model=None, top_n_percent=15, num_samples=64,
                 random_fraction=1 / 3, bandwidth_factor=3, device=None, sampler="host", sampler_seed=None,
                 **kwargs):
        super().__init__(**kwargs)
        # sampler 'host': the reference's draws from the global numpy RNG (seeded runs reproduce the
        # reference's proposals); 'gpu': the same rule drawn on the GPU from a Philox stream
        # (distributional parity; for large num_samples, where host sampling dominates)
        if sampler not in ("host", "gpu"):
            raise ValueError("sampler must be 'host' or 'gpu'")
        self.sampler = sampler
        if sampler_seed is None and sampler == "gpu":
            sampler_seed = int.from_bytes(np.random.bytes(8), "little")
        self.sampler_seed = sampler_seed
        self._sample_counter = 0
        self.top_n_percent = top_n_percent
        self.configspace = configspace
        self.bw_factor = bandwidth_factor
        self.min_points_in_model = min_points_in_model
        if min_points_in_model is None:
            self.min_points_in_model = len(self.configspace.get_hyperparameters()) + 1
        self.num_samples = num_samples
        self.random_fraction = random_fraction
        self.device = device

        hps = self.configspace.get_hyperparameters()
        self.kde_vartypes = ""
        self.vartypes = []
        for h in hps:  # bohb.py:69-75
            if hasattr(h, 'choices'):
                self.kde_vartypes += 'u'
                self.vartypes += [len(h.choices)]
            else:
                self.kde_vartypes += 'c'
                self.vartypes += [0]
        self.vartypes = np.array(self.vartypes, dtype=int)
        # engine limits: D <= 256 dims; categorical codes are level indices < 1024 (the
        # level count runs on a 1024-bit map); beyond 64 continuous / 32 categorical dims the KDEs are
        # exact-only (every candidate re-scored in fp64, no fp32 pre-selection)
        if len(self.vartypes) > _native.lib().hbx_max_dims():
            raise ValueError("hpbandster_amd supports at most %d hyperparameters (got %d)"
                             % (_native.lib().hbx_max_dims(), len(self.vartypes)))
        if (self.vartypes > 1024).any():
            raise ValueError("hpbandster_amd supports categorical hyperparameters with at most 1024 choices")

        self.cat_probs = []
        self.configs = dict()
        self.losses = dict()
        self.good_config_rankings = dict()
        self.kde_models = dict()
        self._stores = dict()  # budget -> ObservationStore: the budget's rows resident in HBM
        self._model_version = 0  # bumped whenever kde_models changes (speculative batches check it)

    # -- candidates ---------------------------------------------------------------------------
    def sample_candidates(self, kde_good, num_samples):
        """bohb.py:133-147: around a random good observation, truncnorm per continuous dim (bounds
        from bw, scale bandwidth_factor * bw), keep-or-resample per categorical dim.  Global RNG."""
        D = len(self.vartypes)
        cands = np.empty((num_samples, D), dtype=np.float64)
        data = kde_good.data
        bws = kde_good.bw
        for i in range(num_samples):
            idx = np.random.randint(0, len(data))
            for d, (m, bw, t) in enumerate(zip(data[idx], bws, self.vartypes)):
                if t == 0:
                    cands[i, d] = sps.truncnorm.rvs(-m / bw, (1 - m) / bw, loc=m, scale=self.bw_factor * bw)
                else:
                    if np.random.rand() < (1 - bw):
                        cands[i, d] = m
                    else:
                        cands[i, d] = np.random.randint(t)
        return cands

    def draw_candidates(self, pair, num_samples):
        """Candidates of one get_config call (or of several back to back): host numpy array, or with
        the GPU sampler a device tensor plus its per-candidate domain-error flags."""
        if self.sampler == "host":
            return self.sample_candidates(pair['good'], num_samples), None
        cands, _, err = pair['good'].sample(self.vartypes, self.bw_factor, num_samples, self.sampler_seed,
                                            self._sample_counter)
        self._sample_counter += num_samples
        return cands, err

    def get_config(self, budget):
        sample = None
        info_dict = {}
        if len(self.kde_models.keys()) == 0 or np.random.rand() < self.random_fraction:
            sample = self.configspace.sample_configuration().get_dictionary()
            info_dict['model_based_pick'] = False

        if sample is None:
            try:
                budget = max(self.kde_models.keys())  # always the largest-budget model (bohb.py:124)
                pair = self.kde_models[budget]        # immutable snapshot (new_result swaps entries)
                cands, err = self.draw_candidates(pair, self.num_samples)
                res = pair.acquire(cands)
                if err is not None and bool(err.any()):
                    raise ValueError("truncnorm domain error: a sampled datum has no valid bounds")
                if res.index < 0:
                    self.logger.debug("Sampling based optimization with %i samples failed -> using random configuration"
                                      % self.num_samples)
                    sample = self.configspace.sample_configuration().get_dictionary()
                    info_dict['model_based_pick'] = False
                else:
                    best_vector = cands[res.index]
                    if err is not None:
                        best_vector = best_vector.cpu().numpy()
                    self.logger.debug('best_vector: {}, {}'.format(best_vector, res.score))
                    sample = ConfigSpace.Configuration(self.configspace, vector=best_vector).get_dictionary()
                    info_dict['model_based_pick'] = True
            except _native.HbxError:
                raise  # the engine failed: never hide it behind a random configuration
            except Exception:
                self.logger.warning("Sampling based optimization with %i samples failed\n %s \nUsing random configuration"
                                    % (self.num_samples, traceback.format_exc()))
                sample = self.configspace.sample_configuration().get_dictionary()
                info_dict['model_based_pick'] = False
        return sample, info_dict

    def get_config_batch_spec(self, budget, k):
        """k get_config calls drawn and scored now (ONE hbx_kde_acquire_batch pass), handed out one at a
        time by the returned SpeculativeBatch -- each only while it is exactly what the sequential call
        would return at that moment: the model unchanged (no refit since, ``_model_version``) and every
        RNG the calls consume (numpy's global one, the configspace's, the GPU sampler's counter) in the
        state the previous call left.  The RNGs are rewound to the state after call 1 at once, so
        anything else drawing in between (a worker, another generator) sees the sequential stream."""
        before = _rng_snapshot(self)
        after = []
        out = self.get_config_batch(budget, k, _snapshots=after)
        spec = SpeculativeBatch(self, out, before, after, self._model_version)
        return spec

    def get_config_batch(self, budget, k, _snapshots=None):
        """``[self.get_config(budget) for _ in range(k)]`` with one GPU pass for all model-based calls.

        Valid while no result arrives in between (the model is fixed): an SH stage's first
        ``num_configs[0]`` samples (HB_iteration.py:136-138).  The global numpy RNG is consumed in the
        same order as k sequential calls (the draws of a call do not depend on earlier calls' scores)
        and the configspace RNG is consumed in call order, so the returned list is identical to the
        sequential one.
        """
        plan = []  # per call: None (random pick) or the row offset of its candidates
        blocks = []
        pair = None
        g_after = []  # numpy's global RNG state after each call's draws (speculative batches)
        counter0 = self._sample_counter
        for _ in range(int(k)):
            if _snapshots is not None and plan:
                g_after.append(np.random.get_state())
            if len(self.kde_models.keys()) == 0 or np.random.rand() < self.random_fraction:
                plan.append(None)
                continue
            if pair is None:
                pair = self.kde_models[max(self.kde_models.keys())]  # bohb.py:124
            if self.sampler == "gpu":
                plan.append(len(blocks) * self.num_samples)
                blocks.append(None)
                continue
            try:  # a sampling error falls back to a random configuration for this call only, after
                # consuming the global RNG exactly as the sequential call would (bohb.py:163-166)
                block = self.sample_candidates(pair['good'], self.num_samples)
            except Exception:
                self.logger.warning("Sampling based optimization with %i samples failed\n %s \nUsing random "
                                    "configuration" % (self.num_samples, traceback.format_exc()))
                plan.append(None)
                continue
            plan.append(len(blocks) * self.num_samples)
            blocks.append(block)
        if _snapshots is not None and plan:
            g_after.append(np.random.get_state())
        results, bad = [], None
        if blocks:
            if self.sampler == "gpu":  # one draw for all calls: same Philox counters as call by call
                cands, err = self.draw_candidates(pair, len(blocks) * self.num_samples)
                bad = err.view(len(blocks), self.num_samples).any(dim=1).cpu().numpy()
            else:
                cands = np.concatenate(blocks, axis=0)
            results = pair.acquire_batch(cands, self.num_samples)
        out = []
        nmodel = 0
        for i, off in enumerate(plan):
            if _snapshots is not None and i > 0:  # call i-1 is complete: every RNG's state after it
                _snapshots.append((g_after[i - 1], self.configspace.random.get_state(),
                                   counter0 + nmodel * self.num_samples))
            if off is not None:
                nmodel += 1
            if off is None:
                out.append((self.configspace.sample_configuration().get_dictionary(), {'model_based_pick': False}))
                continue
            res = results[off // self.num_samples]
            if bad is not None and bad[off // self.num_samples]:
                self.logger.warning("Sampling based optimization with %i samples failed (truncnorm domain error)"
                                    "\nUsing random configuration" % self.num_samples)
                out.append((self.configspace.sample_configuration().get_dictionary(), {'model_based_pick': False}))
            elif res.index < 0:
                self.logger.debug("Sampling based optimization with %i samples failed -> using random configuration"
                                  % self.num_samples)
                out.append((self.configspace.sample_configuration().get_dictionary(), {'model_based_pick': False}))
            else:
                vec = cands[off + res.index]
                if bad is not None:
                    vec = vec.cpu().numpy()
                out.append((ConfigSpace.Configuration(self.configspace, vector=vec).get_dictionary(),
                            {'model_based_pick': True}))
        if _snapshots is not None and plan:
            _snapshots.append((g_after[-1], self.configspace.random.get_state(),
                               counter0 + nmodel * self.num_samples))
        return out

    # -- observations ---------------------------------------------------------------------------
    def new_result(self, job):
        super().new_result(job)
        if job.result is None:
            loss = np.inf  # crashed runs count as bad configurations (bohb.py:189-192)
        else:
            loss = job.result["loss"]
        budget = job.kwargs["budget"]
        if budget not in self.configs.keys():
            self.configs[budget] = []
            self.losses[budget] = []
        if max(list(self.kde_models.keys()) + [-np.inf]) > budget:  # bohb.py:204-205
            return
        conf = ConfigSpace.Configuration(self.configspace, job.kwargs["config"])
        vec = conf.get_array()
        self.configs[budget].append(vec)
        self.losses[budget].append(loss)
        store = self._stores.get(budget)
        if store is None:
            store = self._stores[budget] = ObservationStore(len(self.kde_vartypes), self.kde_vartypes,
                                                            device=self.device)
        store.add(vec, loss)
        if len(self.configs[budget]) <= self.min_points_in_model + 1:
            return
        # one refit call: the new row to the device, argsort, split, bandwidths, both KDEs prepared
        pair = store.refit(self.min_points_in_model, self.top_n_percent)
        if pair is None:  # bohb.py:234-237: too few rows for a KDE
            return
        self.kde_models[budget] = pair  # atomic swap: a concurrent get_config keeps its snapshot
        self._model_version += 1
        self.logger.debug('done building a new model for budget %f based on %i/%i split\nBest loss for this '
                          'budget:%f\n\n\n\n\n' % (budget, pair.good.nobs, pair.bad.nobs,
                                                       np.min(store.losses_host)))
