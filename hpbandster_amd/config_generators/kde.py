"""KernelDensityEstimator (reference: hpbandster/config_generators/kde.py:9-147).

The reference's fourth generator: per budget, a product-Gaussian KDE over the best ``top_n_percent``
configurations with **cross-validated** bandwidths (``KDEMultivariate(..., bw='cv_ls')``,
kde.py:145-147) and proposals drawn around a random training point (kde.py:69-75).  What moved to the
GPU: the bandwidth selection.  Every Nelder-Mead step evaluates statsmodels' ``imse`` objective, an
O(n^2 D) sum over observation pairs, and that runs in libhbx.so (``hbx_kde_cv_terms`` through
``cv.CVObjective``); the simplex search, the training-set rule and the proposals stay on the host, in
the reference's order, with the same consumption of the global numpy RNG.

Deviations, each where the reference cannot run as written:

* ``__init__(..., *kwargs)`` forwards a tuple as ``**kwargs`` (kde.py:12,33), a TypeError for any
  call; here the base-class keyword arguments are accepted as ``**kwargs`` (the evident intent).
* ``new_result`` reads ``job.result['result']['loss']`` (kde.py:119), but the dispatcher's jobs carry
  ``{'loss': ..., 'info': ...}`` (dispatcher.py:9-32).  Both forms are accepted; a failed job
  (``result is None``) is recorded with loss +inf instead of raising.
* With no model, the reference returns a bare dict (kde.py:65); here ``(dict, {})`` as the
  ``get_config`` contract (base.py:32-51) and ``HB_iteration`` require.
"""

import numpy as np
import scipy.stats as sps

from .base import base_config_generator
from ._cs import ConfigSpace


class CVKDEModel(object):
    """What the reference keeps of a fitted ``KDEMultivariate``: the training data and bandwidths."""

    __slots__ = ("data", "bw", "var_type")

    def __init__(self, data, bw, var_type):
        self.data, self.bw, self.var_type = data, bw, var_type


class KernelDensityEstimator(base_config_generator):
    def __init__(self, configspace, top_n_percent=10, update_after_n_points=50, min_points_in_model=None,
                 bw_method="cv_ls", device=None, **kwargs):
        super(KernelDensityEstimator, self).__init__(**kwargs)
        self.top_n_percent = top_n_percent
        self.update_after_n_points = update_after_n_points
        self.configspace = configspace
        self.min_points_in_model = min_points_in_model
        if min_points_in_model is None:  # kde.py:38-39
            self.min_points_in_model = len(self.configspace.get_hyperparameters()) + 1
        # kde.py:43: continuous spaces only
        self.var_type = "c" * len(self.configspace.get_hyperparameters())
        self.bw_method = bw_method  # the reference hard-codes 'cv_ls'; 'cv_ml' is the other CV rule
        self.device = device
        self.configs = dict()
        self.losses = dict()
        self.kde_models = dict()

    def fit_model(self, train_data):
        """KDEMultivariate(data=train_data, var_type='c'*D, bw='cv_ls') (kde.py:145-147): the CV
        bandwidths selected on the GPU (SM:_kernel_base.py:103-139, 279-332)."""
        from ..cv import CVObjective
        obj = CVObjective(train_data, self.var_type, device=self.device)
        return CVKDEModel(obj.data, obj.select(self.bw_method), self.var_type)

    def get_config(self, budget):
        """kde.py:50-78."""
        if len(self.kde_models.keys()) == 0:
            return self.configspace.sample_configuration().get_dictionary(), {}
        if budget not in self.kde_models.keys():
            budget = sorted(self.kde_models.keys())[-1]
        kde = self.kde_models[budget]
        idx = np.random.randint(0, len(self.kde_models[budget].data))
        vector = [sps.truncnorm.rvs(-m / bw, (1 - m) / bw, loc=m, scale=bw)
                  for m, bw in zip(self.kde_models[budget].data[idx], kde.bw)]
        if np.any(np.array(vector) > 1) or np.any(np.array(vector) < 0):
            raise RuntimeError("truncated normal sampling problems!")
        sample = ConfigSpace.Configuration(self.configspace, vector=vector)
        return sample.get_dictionary(), {}

    @staticmethod
    def _loss(job):
        r = job.result
        if r is None:
            return np.inf
        if isinstance(r, dict) and isinstance(r.get("result"), dict):  # the form kde.py:119 reads
            r = r["result"]
        return r["loss"]

    def new_result(self, job):
        """kde.py:80-147: record, and every ``update_after_n_points`` results on a budget refit that
        budget's model on the best configurations (borrowing from larger budgets first when short)."""
        super(KernelDensityEstimator, self).new_result(job)
        budget = job.kwargs["budget"]
        if budget not in self.configs.keys():
            self.configs[budget] = []
            self.losses[budget] = []
        conf = ConfigSpace.Configuration(self.configspace, job.kwargs['config'])
        self.configs[budget].append(conf.get_array())
        self.losses[budget].append(self._loss(job))

        if len(self.configs[budget]) % self.update_after_n_points != 0:
            return
        train_configs, train_losses = [], []
        train_configs.extend(self.configs[budget])
        train_losses.extend(self.losses[budget])
        n = int(self.top_n_percent * len(train_configs) / 100.)
        remaining_budgets = list(self.configs.keys())
        remaining_budgets.remove(budget)
        remaining_budgets.sort(reverse=True)
        for b in remaining_budgets:
            if n >= self.min_points_in_model:
                break
            train_configs.extend(self.configs[b])
            train_losses.extend(self.losses[b])
            n = int(self.top_n_percent * len(train_configs) / 100.)
        if len(train_losses) < self.min_points_in_model:
            return
        n = max(self.min_points_in_model, n)
        idx = np.argsort(train_losses)
        train_data = (np.array(train_configs)[idx])[:n]
        self.kde_models[budget] = self.fit_model(train_data)


__all__ = ["KernelDensityEstimator", "CVKDEModel"]
