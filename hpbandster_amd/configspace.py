"""Minimal ConfigSpace-compatible configuration space (host side, no compute).

HpBandSter's config generators talk to ``ConfigSpace`` through a handful of calls
(``get_hyperparameters()``, ``hasattr(h, 'choices')``, ``sample_configuration()``,
``Configuration(cs, values).get_array()`` and ``Configuration(cs, vector=v).get_dictionary()``;
see ``hpbandster/config_generators/bohb.py:63-77,110,160,211-212`` in the reference).
ConfigSpace is not installed in this image, so the engine ships this small stand-in with
the same surface and the same vector encoding conventions:

* ``UniformFloatHyperparameter``: vector = (v - lower) / (upper - lower) (log space if ``log``).
* ``UniformIntegerHyperparameter``: encoded through a float range widened by 0.49999 on both
  sides, decoded by rounding (ConfigSpace's convention); no ``choices`` -> BOHB type ``'c'``.
* ``CategoricalHyperparameter``: vector = index into ``choices``; BOHB type ``'u'``.
* ``OrdinalHyperparameter``: vector = index into ``sequence``; no ``choices`` -> type ``'c'``.

Hyperparameters are kept sorted by name, which is the order ConfigSpace uses for
unconditioned spaces, so ``get_array()`` columns line up with ``get_hyperparameters()``.
When the real ``ConfigSpace`` package is importable the engine uses it instead
(see ``hpbandster_amd.config_generators._cs``).
"""

import math

import numpy as np


class Hyperparameter(object):
    def __init__(self, name):
        self.name = name

    def __repr__(self):
        return "%s(%r)" % (type(self).__name__, self.name)


class UniformFloatHyperparameter(Hyperparameter):
    def __init__(self, name, lower, upper, default_value=None, log=False):
        super().__init__(name)
        if not lower < upper:
            raise ValueError("lower must be < upper for %s" % name)
        if log and lower <= 0:
            raise ValueError("log-scaled hyperparameter %s needs lower > 0" % name)
        self.lower = float(lower)
        self.upper = float(upper)
        self.log = bool(log)
        self.default_value = default_value

    def _bounds(self):
        if self.log:
            return math.log(self.lower), math.log(self.upper)
        return self.lower, self.upper

    def _transform(self, vector_value):
        lo, hi = self._bounds()
        v = vector_value * (hi - lo) + lo
        return math.exp(v) if self.log else float(v)

    def _inverse_transform(self, value):
        lo, hi = self._bounds()
        v = math.log(value) if self.log else float(value)
        return (v - lo) / (hi - lo)

    def _sample_vector(self, rng):
        return rng.uniform()


class UniformIntegerHyperparameter(UniformFloatHyperparameter):
    def __init__(self, name, lower, upper, default_value=None, log=False):
        Hyperparameter.__init__(self, name)
        self.int_lower = int(lower)
        self.int_upper = int(upper)
        self.lower = lower - 0.49999
        self.upper = upper + 0.49999
        self.log = bool(log)
        if log:
            self.lower = max(self.lower, 1e-12)
        self.default_value = default_value

    def _transform(self, vector_value):
        v = int(round(super()._transform(vector_value)))
        return min(max(v, self.int_lower), self.int_upper)


class CategoricalHyperparameter(Hyperparameter):
    def __init__(self, name, choices, default_value=None):
        super().__init__(name)
        self.choices = tuple(choices)
        if len(self.choices) == 0:
            raise ValueError("categorical %s needs at least one choice" % name)
        self.default_value = default_value

    def _transform(self, vector_value):
        return self.choices[int(vector_value)]

    def _inverse_transform(self, value):
        return float(self.choices.index(value))

    def _sample_vector(self, rng):
        return float(rng.randint(len(self.choices)))


class OrdinalHyperparameter(Hyperparameter):
    def __init__(self, name, sequence, default_value=None):
        super().__init__(name)
        self.sequence = tuple(sequence)
        self.default_value = default_value

    def _transform(self, vector_value):
        return self.sequence[int(round(vector_value))]

    def _inverse_transform(self, value):
        return float(self.sequence.index(value))

    def _sample_vector(self, rng):
        return float(rng.randint(len(self.sequence)))


class ConfigurationSpace(object):
    def __init__(self, seed=None):
        self._hps = {}
        self.random = np.random.RandomState(seed)

    def seed(self, seed):
        self.random = np.random.RandomState(seed)

    def add_hyperparameter(self, hp):
        if hp.name in self._hps:
            raise ValueError("hyperparameter %s already present" % hp.name)
        self._hps[hp.name] = hp
        return hp

    def add_hyperparameters(self, hps):
        for h in hps:
            self.add_hyperparameter(h)
        return hps

    def get_hyperparameters(self):
        return [self._hps[k] for k in sorted(self._hps)]

    def get_hyperparameter_names(self):
        return sorted(self._hps)

    def get_hyperparameter(self, name):
        return self._hps[name]

    def sample_configuration(self, size=1):
        hps = self.get_hyperparameters()
        out = []
        for _ in range(size):
            vec = np.array([h._sample_vector(self.random) for h in hps], dtype=np.float64)
            out.append(Configuration(self, vector=vec))
        return out[0] if size == 1 else out

    def __len__(self):
        return len(self._hps)


class Configuration(object):
    def __init__(self, configuration_space, values=None, vector=None):
        self.configuration_space = configuration_space
        hps = configuration_space.get_hyperparameters()
        if (values is None) == (vector is None):
            raise ValueError("exactly one of values / vector must be given")
        if values is not None:
            missing = [h.name for h in hps if h.name not in values]
            if missing:
                raise ValueError("missing values for %s" % missing)
            self._vector = np.array([h._inverse_transform(values[h.name]) for h in hps],
                                    dtype=np.float64)
        else:
            vec = np.asarray(vector, dtype=np.float64).reshape(-1)
            if vec.shape[0] != len(hps):
                raise ValueError("vector has %d entries, space has %d" % (vec.shape[0], len(hps)))
            self._vector = np.ascontiguousarray(vec)

    def get_array(self):
        return self._vector

    def get_dictionary(self):
        hps = self.configuration_space.get_hyperparameters()
        return {h.name: h._transform(v) for h, v in zip(hps, self._vector)}

    def __getitem__(self, key):
        return self.get_dictionary()[key]

    def __eq__(self, other):
        return isinstance(other, Configuration) and np.array_equal(self._vector, other._vector)

    def __repr__(self):
        return "Configuration(%r)" % (self.get_dictionary(),)
