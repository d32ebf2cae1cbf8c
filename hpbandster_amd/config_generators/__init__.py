"""Config generators: the get_config/new_result drop-ins (BOHB, KDEEI and KernelDensityEstimator run their
KDE work on the GPU)."""
from .base import base_config_generator  # noqa: F401
from .random_sampling import RandomSampling  # noqa: F401


def __getattr__(name):  # BOHB / KDEEI import scipy; load them lazily
    if name == "BOHB":
        from .bohb import BOHB
        return BOHB
    if name == "KDEEI":
        from .kde_ei import KDEEI
        return KDEEI
    if name == "KernelDensityEstimator":
        from .kde import KernelDensityEstimator
        return KernelDensityEstimator
    raise AttributeError(name)
