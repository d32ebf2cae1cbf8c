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

import ctypes
import logging
import threading
import traceback

import numpy as np
import scipy.stats as sps

from .. import _native
from ..kde import ACQ_DOMAIN_ERR, ObservationStore, mapped_candidates
from .base import base_config_generator
from ._cs import ConfigSpace


class _MT(object):
    """The raw MT19937 state (key[624] words + position: 2500 bytes) of a legacy ``RandomState`` -- a
    snapshot, compare or restore in ~1 us, where ``get_state`` / ``set_state`` cost ~60 us each (they
    build and parse the state tuple).  The Gaussian cache of the legacy generator is not part of it:
    BOHB's draws (``rand``, ``randint``, scipy's truncnorm by inversion of a uniform) never touch it.
    The layout is numpy's ``mt19937_state``; ``mt_layout_ok()`` checks it against ``get_state`` /
    ``set_state`` once per process before anything relies on it."""
    NB = 624 * 4 + 4

    def __init__(self, rs):
        bg = rs._bit_generator
        if type(bg).__name__ != "MT19937":
            raise TypeError("not an MT19937 RandomState")
        self.rs, self.addr, self.lock = rs, bg.ctypes.state_address, bg.lock

    def snap(self):
        return ctypes.string_at(self.addr, self.NB)

    def load(self, raw):
        ctypes.memmove(self.addr, raw, self.NB)


_LAYOUT = [None]


def mt_layout_ok():
    """Once per process: the raw bytes at the bit generator's state address are get_state()'s key words
    and position, and load() of another state's bytes gives that state's get_state() (and its next
    draws).  False (never raising) when numpy's layout is not the one assumed: the raw-state users then
    step aside -- speculative batches are not made, the host draws take scipy's per-element path."""
    if _LAYOUT[0] is None:
        try:
            a, b = np.random.RandomState(20240917), np.random.RandomState(77)
            a.random_sample(700)  # position off the block boundary
            ma, mb = _MT(a), _MT(b)
            st = a.get_state(legacy=True)
            ok = ma.snap() == np.asarray(st[1], dtype="<u4").tobytes() + np.int32(st[2]).tobytes()
            mb.load(ma.snap())
            sb = b.get_state(legacy=True)
            ok = ok and np.array_equal(sb[1], st[1]) and sb[2] == st[2]
            ok = ok and np.array_equal(a.random_sample(3), b.random_sample(3))
            _LAYOUT[0] = bool(ok)
        except Exception:
            _LAYOUT[0] = False
        if not _LAYOUT[0]:
            logging.getLogger('hpbandster').warning(
                "numpy's MT19937 state layout is not the assumed one: speculative batches and the fast host draws "
                "are off (results unchanged)")
    return _LAYOUT[0]


_GLOBAL = [None]


def _global_mt():
    """_MT of numpy's global RandomState (the one np.random.rand / randint / scipy's rvs draw from), or
    None when its raw state cannot be used."""
    R = np.random.mtrand._rand
    g = _GLOBAL[0]
    if g is None or g.rs is not R:
        if not mt_layout_ok():
            return None
        try:
            g = _GLOBAL[0] = _MT(R)
        except (TypeError, AttributeError):
            return None
    return g


_HOSTDRAW = [None]


def host_draw_ok():
    """Once per process: hbx_bohb_draw (libhbx's restatement of the draws, on numpy's own state) agrees with
    numpy and scipy -- random_sample and randint streams, and a small get_config draw against the
    per-element scipy path, values and final state bit for bit.  False (never raising) otherwise: the
    per-element path then runs."""
    if _HOSTDRAW[0] is None:
        ok = False
        try:
            ok = mt_layout_ok() and int(_native.lib().hbx_mt_state_bytes()) == _MT.NB
            if ok:
                L = _native.lib()
                a, b = np.random.RandomState(5), np.random.RandomState(5)
                ma = _MT(a)
                out = np.empty(1500)
                _native.check(L.hbx_mt_draw(ma.addr, 0, out.size, 0, out.ctypes.data))
                ok = np.array_equal(out, b.random_sample(out.size))
                for high in (1, 2, 3, 4, 7, 100, 1000, 65537, 2 ** 31 + 5):
                    o = np.empty(64)
                    _native.check(L.hbx_mt_draw(ma.addr, 1, o.size, high, o.ctypes.data))
                    ok = ok and np.array_equal(o, [b.randint(0, high) for _ in range(o.size)])
                ok = ok and ma.snap() == _MT(b).snap()
            if ok:
                rs = np.random.RandomState(11)
                data = np.column_stack([rs.rand(9, 3), rs.randint(0, 3, (9, 2))]).astype(np.float64)
                data[4, 0], data[2, 1] = 0.0, 1.0
                kde = _HostModel(data, np.array([0.2, 0.05, 0.6, 0.4, 0.9]))
                lv = np.array([0, 0, 0, 3, 4])
                a, b = np.random.RandomState(6), np.random.RandomState(6)
                fast = _draw_fast(kde, lv, 3, 16, a, _MT(a))
                slow = _draw_rvs(kde, lv, 3, 16, b)
                ok = np.array_equal(fast, slow) and _MT(a).snap() == _MT(b).snap()
        except Exception:
            ok = False
        _HOSTDRAW[0] = bool(ok)
        if not ok:
            logging.getLogger('hpbandster').warning(
                "hbx_bohb_draw disagrees with numpy/scipy here: BOHB draws candidates element by element")
    return _HOSTDRAW[0]


class _HostModel(object):
    """The two fields of a KDE the draws read (``data`` rows and ``bw``)."""

    def __init__(self, data, bw):
        self.data, self.bw = data, bw


def _draw_rvs(kde_good, levels, bw_factor, num_samples, R):
    """bohb.py:133-147 element by element: R.randint for the datum, one scipy truncnorm.rvs per continuous
    dim (bounds from bw, scale bw_factor * bw), keep-or-resample per categorical dim."""
    D = len(levels)
    cands = np.empty((num_samples, D), dtype=np.float64)
    data = kde_good.data
    bws = kde_good.bw
    for i in range(num_samples):
        idx = R.randint(0, len(data))
        for d, (m, bw, t) in enumerate(zip(data[idx], bws, levels)):
            if t == 0:
                cands[i, d] = sps.truncnorm.rvs(-m / bw, (1 - m) / bw, loc=m, scale=bw_factor * bw, random_state=R)
            else:
                if R.rand() < (1 - bw):
                    cands[i, d] = m
                else:
                    cands[i, d] = R.randint(t)
    return cands


class _TruncnormTerms(object):
    """The uniform-independent terms of scipy's ``truncnorm._ppf`` for one KDE's observation rows, filled
    row by row as draws first pick them (a model serves every call until the next refit, and BOHB's datum is
    one of its good rows: after a call or two every row is in).  Per (row, continuous dim), with a = -m/bw,
    b = (1 - m)/bw (scipy 1.15 ``_continuous_distns.py``, ``truncnorm_gen._ppf`` / ``_log_gauss_mass``):
    ``lp`` = log_ndtr(a) where a < 0 (``ppf_left``), log_ndtr(-b) otherwise (``ppf_right``); ``mass`` =
    log1p(-ndtr(a) - ndtr(-b)), the central case of ``_log_gauss_mass``; ``ok`` False where that case does not
    apply (b <= 0: a datum at the upper bound, a > 0, non-finite bounds) -- those elements take scipy's own
    ``_ppf``."""

    def __init__(self, data, bw):
        self.data, self.bw = data, bw
        n, D = data.shape
        self.lp = np.empty((n, D))
        self.mass = np.empty((n, D))
        self.left = np.zeros((n, D), dtype=np.bool_)
        self.ok = np.zeros((n, D), dtype=np.bool_)
        self.have = np.zeros(n, dtype=np.bool_)

    def fill(self, rows, cont):
        import scipy.special as sc
        r = np.unique(rows[~self.have[rows]])
        if r.size:
            m = self.data[np.ix_(r, cont)]
            h = self.bw[cont]
            with np.errstate(all="ignore"):  # (a zero bandwidth: no inversion is asked for that dim)
                a, b = -m / h, (1 - m) / h
                left = a < 0
                self.lp[np.ix_(r, cont)] = sc.log_ndtr(np.where(left, a, -b))
                self.mass[np.ix_(r, cont)] = sc.log1p(-sc.ndtr(a) - sc.ndtr(-b))
            self.left[np.ix_(r, cont)] = left
            self.ok[np.ix_(r, cont)] = (b > 0) & (a <= 0) & np.isfinite(a) & np.isfinite(b)
            self.have[r] = True


_LOG2 = [None]


def _ppf_from_terms(q, lp, mass, left):
    """scipy's truncnorm._ppf at uniforms q from the terms above, the same numpy / scipy.special ufuncs in the
    same order: log_Phi_x = logsumexp([lp, log(q) + mass]) (log1p(-q) on the right), scipy 1.15's
    ``_logsumexp`` for two real rows (the larger one taken out of the sum: (log1p(exp(lo - hi)) + log(m)) + hi,
    m the number of rows equal to the larger), then ndtri_exp (negated on the right).  Formed here as
    log1p(exp(min - max)) + max: for m = 1, log(m) = 0 adds nothing to log1p(.) >= 0; for m = 2 (the rows
    equal), exp(0) = 1 and log1p(1) is log(2) (checked by ppf_terms_ok), where scipy adds log(2) to log1p(0) = 0.
    Elementwise, so a subset gives the values the whole array would.  Non-finite log_Phi_x inputs come back as
    ``bad`` positions for scipy's own _ppf."""
    import scipy.special as sc
    with np.errstate(all="ignore"):
        x = np.where(left, np.log(q), np.log1p(-q))
        x += mass
        hi = np.maximum(lp, x)
        s = np.minimum(lp, x)
        s -= hi
        np.exp(s, out=s)
        np.log1p(s, out=s)
        s += hi
        y = sc.ndtri_exp(s)
    np.negative(y, out=y, where=~left)
    return y, ~np.isfinite(hi)


_PPF = [None]


def ppf_terms_ok():
    """Once per process: _ppf_from_terms equals scipy's own truncnorm._ppf bit for bit over BOHB's range and its
    edges (uniforms 0, tiny, near 1; a datum at 0 (a = -0: the right case), at 1 (b = 0: scipy's path), near the
    bounds; narrow and wide bandwidths).  False (never raising) otherwise: the draws then invert through scipy's
    _ppf, as before."""
    if _PPF[0] is None:
        ok = False
        try:
            rs = np.random.RandomState(17)
            nr, nd = 200, 20
            m = rs.rand(nr, nd)
            m[:4] = 0.0
            m[4:6] = 1.0
            m[6:10] = rs.choice([1e-12, 1 - 1e-12, 1e-300, 0.5], (4, nd))
            h = np.exp(rs.uniform(np.log(1e-4), np.log(5.0), nd))
            q = rs.rand(nr, nd)
            q[10:12] = 0.0
            q[12:16] = rs.choice([1e-300, 1e-17, 1 - 2 ** -53, 0.5], (4, nd))
            t = _TruncnormTerms(m, h)
            t.fill(np.arange(nr), np.arange(nd))
            with np.errstate(all="ignore"):
                ref = sps.truncnorm._ppf(q, -m / h, (1 - m) / h)
            y, bad = _ppf_from_terms(q, t.lp, t.mass, t.left)
            use = t.ok & ~bad
            ok = bool(use.sum() > nr * nd - 3 * nd) and np.array_equal(y[use].view(np.uint64),
                                                                       ref[use].view(np.uint64))
            one = np.ones(4)  # the equal-rows case of the logsumexp (_ppf_from_terms)
            ok = ok and np.array_equal(np.log1p(one).view(np.uint64), np.log(one + one).view(np.uint64))
        except Exception:
            ok = False
        _PPF[0] = bool(ok)
        if not ok:
            logging.getLogger('hpbandster').warning(
                "the truncnorm inversion terms disagree with scipy's truncnorm._ppf here: BOHB inverts through scipy")
    return _PPF[0]


def _draw_fast(kde_good, levels, bw_factor, num_samples, R, mt, out=None):
    """The same draws in one native call on R's own MT19937 state (hbx_bohb_draw, the reference's
    consumption order), then the truncnorm inversion of the call's uniforms and rvs's ``* scale + loc`` --
    the arithmetic rvs applies to each uniform, elementwise, so the values are the per-element path's bit for
    bit (checked by host_draw_ok and tests/test_host_draw.py).  The inversion reuses the model's per-row terms
    (``_TruncnormTerms``; scipy's own ``truncnorm._ppf`` when ppf_terms_ok() fails and for the elements the
    terms do not cover).  A domain error raises ValueError with R left where scipy's raise leaves it."""
    data = kde_good.data
    if not (isinstance(data, np.ndarray) and data.dtype == np.float64 and data.flags.c_contiguous):
        data = np.ascontiguousarray(data, dtype=np.float64)
    bws = np.ascontiguousarray(kde_good.bw, dtype=np.float64)
    lv = np.ascontiguousarray(levels, dtype=np.int64)
    n, D = data.shape
    vals = np.empty((num_samples, D)) if out is None else out
    if not vals.flags.c_contiguous:
        raise ValueError("_draw_fast: out must be C-contiguous")
    cap = num_samples * D
    uni = np.empty(cap)
    comp = np.empty(2 * cap, dtype=np.int64)
    datum = np.empty(num_samples, dtype=np.int64)
    stop = ctypes.c_int64(-1)
    nc = ctypes.c_int64(0)
    with mt.lock:
        rc = _native.lib().hbx_bohb_draw(mt.addr, data.ctypes.data, n, D, bws.ctypes.data, lv.ctypes.data,
                                         float(bw_factor), num_samples, vals.ctypes.data, uni.ctypes.data, None,
                                         datum.ctypes.data, ctypes.addressof(stop), comp.ctypes.data,
                                         ctypes.addressof(nc))
    if rc == 1:
        raise ValueError("Domain error in arguments (truncnorm bounds of candidate %d, dim %d; bohb.py:141)"
                         % divmod(stop.value, D))
    _native.check(rc)
    k = nc.value
    if k == 0:
        return vals
    # the elements to invert, in draw order: uniform q, element index e, term index ti = datum D + dim
    q, e, ti = uni[:k], comp[:k], comp[cap:cap + k]
    flat = vals.reshape(-1)
    loc = flat.take(e)
    h = bws.take(ti % D)
    if ppf_terms_ok():
        t = getattr(kde_good, "_tn_terms", None)
        if t is None or t.data is not data or t.bw is not bws or t.lp.shape != (n, D):
            t = _TruncnormTerms(data, bws)
            try:
                kde_good._tn_terms = t
            except AttributeError:  # (an object that takes no attributes: terms for this call only)
                pass
        t.fill(datum, np.flatnonzero(lv == 0))
        y, bad = _ppf_from_terms(q, t.lp.reshape(-1).take(ti), t.mass.reshape(-1).take(ti),
                                 t.left.reshape(-1).take(ti))
        rest = bad | ~t.ok.reshape(-1).take(ti)
        if rest.any():
            y[rest] = sps.truncnorm._ppf(q[rest], -loc[rest] / h[rest], (1 - loc[rest]) / h[rest])
    else:
        y = sps.truncnorm._ppf(q, -loc / h, (1 - loc) / h)
    flat[e] = y * (bw_factor * h) + loc
    return vals


class SpeculativeBatch(object):
    """get_config results computed ahead in one batched acquisition (BOHB.get_config_batch_spec).

    The draws were made from a PRIVATE copy of the global RNG: nothing outside changes until a result is
    served.  ``take()`` serves result j only when it is exactly what the sequential call would return at
    that moment -- the model unchanged (``_model_version``), the GPU sampler's counter and the global
    RNG's raw state equal to those before call j -- and then moves the global RNG (under its lock, so no
    other thread's draw can fall between the check and the move) and the counter to where call j leaves
    them.  A random pick (and its warning) is made only when served, from the configspace's own RNG, as
    the sequential call makes it."""

    def __init__(self, gen, entries, states, counters, version):
        self.gen, self.entries, self.states, self.counters, self.version = gen, entries, states, counters, version
        self.mt = _global_mt()
        self.served = 0

    def __len__(self):
        return len(self.entries)

    def _valid_at(self, j):
        g = self.gen
        return g._model_version == self.version and g._sample_counter == self.counters[j]

    def take(self):
        """The next result, or None when it is not the sequential call's (or the batch is used up)."""
        j = self.served
        if j >= len(self.entries) or not self._valid_at(j):
            return None
        mt = self.mt
        with mt.lock:
            if mt.snap() != self.states[j]:
                return None
            mt.load(self.states[j + 1])
        self.gen._sample_counter = self.counters[j + 1]
        self.served += 1
        return self.gen._serve(self.entries[j])

    def continues(self):
        """Every result served and nothing changed since: a longer batch would have stayed valid."""
        j = self.served
        return j == len(self.entries) and self._valid_at(j) and self.mt.snap() == self.states[j]


class BOHB(base_config_generator):
    def __init__(self, configspace, min_points_in_model=None, top_n_percent=15, num_samples=64,
                 random_fraction=1 / 3, bandwidth_factor=3, device=None, sampler="host", sampler_seed=None,
                 speculative="auto", **kwargs):
        super().__init__(**kwargs)
        # speculative batches (SuccessiveHalving serving a stage's back-to-back requests from one batched
        # acquisition): 'auto' = with the GPU sampler only (the host sampler's scipy draws cost ~100x the
        # acquisition, so batching them gains nothing and risks drawing for calls never served),
        # 'always', 'never'
        if speculative not in ("auto", "always", "never"):
            raise ValueError("speculative must be 'auto', 'always' or 'never'")
        self.speculative = speculative
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
        self._calls = 0  # get_config calls so far
        self._pick_tls = threading.local()  # GPU sampler: this thread's draw / pick buffers (_pick)

    # -- candidates ---------------------------------------------------------------------------
    def sample_candidates(self, kde_good, num_samples, rng=None, out=None):
        """bohb.py:133-147: around a random good observation, truncnorm per continuous dim (bounds
        from bw, scale bandwidth_factor * bw), keep-or-resample per categorical dim.  Global RNG (or
        ``rng``, a RandomState drawn from in the same order).  One native call for every draw of the call
        plus one vectorised truncnorm inversion (``_draw_fast``); the values and the RNG's state after the
        call are the reference's per-element path's bit for bit (``_draw_rvs``, which runs instead when
        host_draw_ok() finds numpy or scipy not as assumed)."""
        R = np.random.mtrand._rand if rng is None else rng
        if host_draw_ok():
            mt = _global_mt() if rng is None else getattr(self, "_rng_mt", (None, None))[1]
            if mt is None or mt.rs is not R:
                try:
                    mt = _MT(R)
                except (TypeError, AttributeError):  # a legacy RandomState over another bit generator (PCG64 ...)
                    mt = None
                if rng is not None and mt is not None:
                    self._rng_mt = (R, mt)
            if mt is not None:
                return _draw_fast(kde_good, self.vartypes, self.bw_factor, num_samples, R, mt, out)
        c = _draw_rvs(kde_good, self.vartypes, self.bw_factor, num_samples, R)
        if out is None:
            return c
        out[...] = c
        return out

    def get_config(self, budget):
        sample = None
        info_dict = {}
        self._calls += 1
        if len(self.kde_models.keys()) == 0 or np.random.rand() < self.random_fraction:
            sample = self.configspace.sample_configuration().get_dictionary()
            info_dict['model_based_pick'] = False

        if sample is None:
            try:
                budget = max(self.kde_models.keys())  # always the largest-budget model (bohb.py:124)
                pair = self.kde_models[budget]        # immutable snapshot (new_result swaps entries)
                if self.sampler == "gpu":
                    # one wait: the draws, the acquisition, the domain-error flag and the winning row come back
                    # together (no separate device reduction and row copy)
                    res, best_vector = self._pick(pair, self._sample_counter)
                    self._sample_counter += self.num_samples
                    if res.flags & ACQ_DOMAIN_ERR:
                        raise ValueError("truncnorm domain error: a sampled datum has no valid bounds")
                else:  # drawn into mapped host memory, which the acquisition's kernels read in place
                    cands = self.sample_candidates(pair['good'], self.num_samples,
                                                   out=mapped_candidates(self.num_samples, len(self.vartypes)))
                    res = pair.acquire_mapped(cands)
                    best_vector = cands[res.index].copy() if res.index >= 0 else None
                if res.index < 0:
                    self.logger.debug("Sampling based optimization with %i samples failed -> using random configuration"
                                      % self.num_samples)
                    sample = self.configspace.sample_configuration().get_dictionary()
                    info_dict['model_based_pick'] = False
                else:
                    if self.logger.isEnabledFor(logging.DEBUG):  # (formatting the vector costs ~0.1 ms)
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

    # -- one GPU-sampler call: draws and acquisition, one wait ----------------------------------------
    def _pick(self, pair, counter):
        """The call's num_samples draws on the Philox `counter` (hbx_kde_sample) and their acquisition with the
        pick on the host (hbx_kde_acquire_bound with the draws' error flags and the winning row): (AcqResult,
        winning row or None).  The draw buffers are kept per thread and reused; the native calls go straight
        through when the thread's current device is the model's and the draw needs no Phi table."""
        import torch
        g = pair.good
        n, D = self.num_samples, len(self.vartypes)
        t = self._pick_tls
        keep = getattr(t, "keep", None)
        wsb = pair.workspace_bytes(n)
        if keep is None or keep[3].numel() < wsb or keep[0].device != g.device:
            keep = t.keep = (torch.empty((n, D), dtype=torch.float64, device=g.device),
                             torch.empty(n, dtype=torch.int64, device=g.device),
                             torch.empty(n, dtype=torch.uint8, device=g.device),
                             torch.empty(wsb, dtype=torch.uint8, device=g.device), np.empty(D))
        cands, datum, err, ws, row = keep
        if (pair._cur_dev is not None and pair._raw_stream is not None and pair._cur_dev() == pair._dev_index
                and n < 4 * g.nobs):
            from ..kde import _levels_on_device
            L = _native.lib()
            lvb = getattr(self, "_lv_bytes", None)
            if lvb is None:
                self._lv_np = np.ascontiguousarray(self.vartypes, dtype=np.int32)
                lvb = self._lv_bytes = self._lv_np.tobytes()
                self._bw_off = int(L.hbx_kde_param_bw_offset())
            lvd = _levels_on_device(lvb, self._lv_np, g.device)
            sh = pair._raw_stream(pair._dev_index)
            if sh != pair._home:
                pair._order(sh)
            _native.check(L.hbx_kde_sample(g.X_dev.data_ptr(), g.k_vars, g.rows_dev.data_ptr(), g.nobs,
                                           g.params.data_ptr() + self._bw_off, lvd.data_ptr(), None,
                                           float(self.bw_factor), int(self.sampler_seed) & (2 ** 64 - 1),
                                           int(counter) & (2 ** 64 - 1), 0, n, cands.data_ptr(), datum.data_ptr(),
                                           err.data_ptr(), sh))
            res = pair.acquire_pick(cands, err, ws, row, sh)
        else:
            with _native.on_device(g.device):
                g.sample(self.vartypes, self.bw_factor, n, self.sampler_seed, counter, out=keep[:3])
                res = pair.acquire_pick(cands, err, ws, row)
        return res, (row.copy() if res.index >= 0 else None)

    # -- several get_config calls in one GPU pass ----------------------------
    def speculation_enabled(self):
        return self.speculative == "always" or (self.speculative == "auto" and self.sampler == "gpu")

    def spec_fingerprint(self):
        """(model version, GPU sampler counter): the same before and after an interval in which no result
        refitted the model.  A hint for SuccessiveHalving's batch sizes only -- every speculative result is
        checked against the full RNG state when served, and a batch cut short by another draw from the
        global RNG drops the sizes back to one."""
        return (self._model_version, self._sample_counter)

    def spec_unchanged(self, fp):
        return fp[0] == self._model_version and fp[1] == self._sample_counter

    def get_config_batch_spec(self, budget, k):
        """k get_config calls drawn and scored now (ONE hbx_kde_acquire_batch pass) from a private copy of
        the global RNG, handed out one at a time by the returned SpeculativeBatch -- each only while it is
        exactly what the sequential call would return at that moment (see SpeculativeBatch).  Returns None
        when the global RNG cannot be copied (not a legacy MT19937 RandomState)."""
        g = _global_mt()
        if g is None:
            return None
        rs = getattr(self, "_spec_rs", None)
        if rs is None:
            rs = self._spec_rs = np.random.RandomState()
            self._spec_mt = _MT(rs)
        pm = self._spec_mt
        states = [g.snap()]
        pm.load(states[0])
        counters = [self._sample_counter]
        version = self._model_version
        entries = self._batch_entries(k, rs, states, counters, pm)
        return SpeculativeBatch(self, entries, states, counters, version)

    def get_config_batch(self, budget, k):
        """``[self.get_config(budget) for _ in range(k)]`` with one GPU pass for all model-based calls.

        Valid while no result arrives in between (the model is fixed): an SH stage's first
        ``num_configs[0]`` samples (HB_iteration.py:136-138).  The global numpy RNG is consumed in the
        same order as k sequential calls (the draws of a call do not depend on earlier calls' scores)
        and the configspace RNG in call order, so the returned list is identical to the sequential one.
        """
        return [self._serve(e) for e in self._batch_entries(k, np.random.mtrand._rand)]

    def _batch_entries(self, k, R, states=None, counters=None, mt=None):
        """The draws of k calls from RandomState R (and the GPU sampler's counter), their candidates scored
        in one batched acquisition.  Per call an entry: ('model', best vector, score) or ('random', log
        level, message) -- the random configuration itself is drawn from the configspace's RNG when the
        entry is served.  With ``states`` / ``counters``: R's raw state (``mt``) and the counter after
        every call are appended."""
        plan = []  # per call: None (random pick), ('err', message) or the row offset of its candidates
        blocks = []
        pair = None
        counter = self._sample_counter
        for _ in range(int(k)):
            if len(self.kde_models.keys()) == 0 or R.rand() < self.random_fraction:
                plan.append(None)
            else:
                if pair is None:
                    pair = self.kde_models[max(self.kde_models.keys())]  # bohb.py:124
                if self.sampler == "gpu":
                    plan.append(len(blocks) * self.num_samples)
                    blocks.append(None)
                    counter += self.num_samples
                else:
                    try:  # a sampling error falls back to a random configuration for this call only, after
                        # consuming the RNG exactly as the sequential call would (bohb.py:163-166)
                        block = self.sample_candidates(pair['good'], self.num_samples, rng=R)
                        plan.append(len(blocks) * self.num_samples)
                        blocks.append(block)
                    except Exception:
                        plan.append(("err", "Sampling based optimization with %i samples failed\n %s \nUsing random "
                                            "configuration" % (self.num_samples, traceback.format_exc())))
            if states is not None:
                states.append(mt.snap())
                counters.append(counter)
        entries = []
        if not blocks:
            return [("random", None, None) if p is None else ("random", "warning", p[1]) for p in plan]
        if self.sampler == "gpu":  # one draw for all calls: the same Philox counters as call by call
            cands, _, err = pair['good'].sample(self.vartypes, self.bw_factor, len(blocks) * self.num_samples,
                                                self.sampler_seed, self._sample_counter if states is None
                                                else counters[0])
            if states is None:
                self._sample_counter += len(blocks) * self.num_samples
        else:
            cands, err = np.concatenate(blocks, axis=0), None
        results = pair.acquire_batch(cands, self.num_samples)
        # the winners' rows in one gather (one device-to-host copy for a device candidate set)
        win = [off + results[off // self.num_samples].index for off in plan
               if type(off) is int and results[off // self.num_samples].index >= 0]
        if err is not None:
            import torch
            bad = err.view(len(blocks), self.num_samples).any(dim=1).cpu().numpy()
            rows = cands[torch.as_tensor(win, dtype=torch.int64, device=cands.device)].cpu().numpy() if win else None
        else:
            bad, rows = None, cands[win] if win else None
        w = 0
        for off in plan:
            if off is None:
                entries.append(("random", None, None))
            elif type(off) is tuple:
                entries.append(("random", "warning", off[1]))
            else:
                res = results[off // self.num_samples]
                if bad is not None and bad[off // self.num_samples]:
                    if res.index >= 0:
                        w += 1
                    entries.append(("random", "warning", "Sampling based optimization with %i samples failed "
                                                         "(truncnorm domain error)\nUsing random configuration"
                                                         % self.num_samples))
                elif res.index < 0:
                    entries.append(("random", "debug", "Sampling based optimization with %i samples failed -> "
                                                       "using random configuration" % self.num_samples))
                else:
                    entries.append(("model", rows[w], res.score))
                    w += 1
        return entries

    def _serve(self, e):
        """One get_config result from a batch entry (the logging and random draws of bohb.py:124-169 happen
        here, when the result is handed out)."""
        if e[0] == "model":
            if self.logger.isEnabledFor(logging.DEBUG):
                self.logger.debug('best_vector: {}, {}'.format(e[1], e[2]))
            return (ConfigSpace.Configuration(self.configspace, vector=e[1]).get_dictionary(),
                    {'model_based_pick': True})
        if e[1] == "warning":
            self.logger.warning(e[2])
        elif e[1] == "debug":
            self.logger.debug(e[2])
        return self.configspace.sample_configuration().get_dictionary(), {'model_based_pick': False}

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
        if self.logger.isEnabledFor(logging.DEBUG):
            self.logger.debug('done building a new model for budget %f based on %i/%i split\nBest loss for this '
                              'budget:%f\n\n\n\n\n' % (budget, pair.good.nobs, pair.bad.nobs,
                                                           np.min(store.losses_host)))
