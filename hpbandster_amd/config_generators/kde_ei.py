"""KDEEI -- drop-in for hpbandster/config_generators/kde_ei.py with the KDE work on the MI355X.

Continuous-only KDEs (var_type 'c' * D, kde_ei.py:63), the same l/g acquisition as BOHB with the
candidate perturbation truncnorm(scale = 2 bw) (kde_ei.py:119-142), and the float split rule
n_good = int(max(top% * N / 100., min_points)) with refits every ``update_after_n_points`` results
(kde_ei.py:146-215).  mode='sampling' runs the batched GPU acquisition; mode='DE' keeps the
reference's scipy differential evolution (a sequential optimiser), evaluating each point with the
GPU's exact fp64 pdf.
"""

import numpy as np
import scipy.optimize as spo
import scipy.stats as sps

from ..kde import ObservationStore
from .base import base_config_generator
from ._cs import ConfigSpace


class KDEEI(base_config_generator):
    def __init__(self, configspace, top_n_percent=10, update_after_n_points=1, min_points_in_model=None,
                 mode='sampling', num_samples=64, random_fraction=0.5, device=None, **kwargs):
        super(KDEEI, self).__init__(**kwargs)
        self.top_n_percent = top_n_percent
        self.update_after_n_points = update_after_n_points
        self.configspace = configspace
        self.min_points_in_model = min_points_in_model
        if min_points_in_model is None:
            self.min_points_in_model = len(self.configspace.get_hyperparameters()) + 1
        self.mode = mode
        self.num_samples = num_samples
        self.random_fraction = random_fraction
        self.device = device
        self.var_type = "c" * len(self.configspace.get_hyperparameters())
        self.configs = dict()
        self.losses = dict()
        self.kde_models = dict()
        self._stores = dict()  # budget -> ObservationStore (rows resident in HBM)

    def get_config(self, budget):
        sample = None
        info_dict = {}
        if len(self.kde_models.keys()) == 0 or np.random.rand() < self.random_fraction:
            sample = self.configspace.sample_configuration().get_dictionary()
            info_dict['model_based_pick'] = False

        if sample is None:
            budget = max(self.kde_models.keys())
            pair = self.kde_models[budget]
            if self.mode == 'DE':
                l, g = pair['good'].pdf, pair['bad'].pdf
                minimize_me = lambda x: max(1e-8, g(x)) / max(l(x), 1e-8)  # noqa: E731
                dim = len(self.configspace.get_hyperparameters())
                maxiter = self.num_samples // (15 * dim) + 1  # 15*dim: scipy's default population
                res = spo.differential_evolution(minimize_me, [(0, 1)] * dim, maxiter=maxiter, init='random')
                sample = ConfigSpace.Configuration(self.configspace, vector=res.x)
            if self.mode == 'sampling':
                kde_good = pair['good']
                D = len(kde_good.bw)
                cands = np.empty((self.num_samples, D), dtype=np.float64)
                for i in range(self.num_samples):
                    idx = np.random.randint(0, len(kde_good.data))
                    for d, (m, bw) in enumerate(zip(kde_good.data[idx], 2 * kde_good.bw)):
                        cands[i, d] = sps.truncnorm.rvs(-m / bw, (1 - m) / bw, loc=m, scale=bw)
                res = pair.acquire(cands)
                if res.index < 0:
                    self.logger.debug("Sampling based optimization with %i samples failed -> using random "
                                      "configuration" % self.num_samples)
                    sample = self.configspace.sample_configuration().get_dictionary()
                    info_dict['model_based_pick'] = False
                else:
                    sample = ConfigSpace.Configuration(self.configspace, vector=cands[res.index]).get_dictionary()
                    info_dict['model_based_pick'] = True
        return sample, info_dict

    def new_result(self, job):
        super(KDEEI, self).new_result(job)
        if job.result is None:  # crashed runs are skipped (kde_ei.py:164-168)
            return
        budget = job.kwargs["budget"]
        loss = job.result["loss"]
        if budget not in self.configs.keys():
            self.configs[budget] = []
            self.losses[budget] = []
        conf = ConfigSpace.Configuration(self.configspace, job.kwargs['config'])
        vec = conf.get_array()
        self.configs[budget].append(vec)
        self.losses[budget].append(loss)
        store = self._stores.get(budget)
        if store is None:
            store = self._stores[budget] = ObservationStore(len(self.var_type), self.var_type, device=self.device)
        store.add(vec, loss)
        if len(self.configs[budget]) <= self.min_points_in_model:
            return
        if len(self.configs[budget]) % self.update_after_n_points == 0:
            pair = store.refit(self.min_points_in_model, self.top_n_percent, split_rule="kde_ei")
            if pair is None:
                return
            self.kde_models[budget] = pair
            self.logger.debug('done building a new model for budget %f based on %i/%i split'
                              % (budget, pair.good.nobs, pair.bad.nobs))
