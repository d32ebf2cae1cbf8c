"""RandomSampling (reference: hpbandster/config_generators/random_sampling.py:6-29)."""

from .base import base_config_generator


class RandomSampling(base_config_generator):
    def __init__(self, configspace, **kwargs):
        super().__init__(**kwargs)
        self.configspace = configspace

    def get_config(self, budget):
        return (self.configspace.sample_configuration().get_dictionary(), {})
