"""The speculative-batch machinery of BOHB (config_generators/bohb.py), host side only: the raw MT19937
state access, the private-RNG draws (identical to the global RNG's, scipy's truncnorm included), and
SpeculativeBatch.take()'s rule -- a result is served only from the exact global state the sequential call
would start from, the state then moved to where that call leaves it, never replayed."""
import threading

import numpy as np
import scipy.stats as sps

from hpbandster_amd.config_generators import bohb as B


class _Gen(object):
    """A stand-in generator: what SpeculativeBatch reads and calls."""

    def __init__(self):
        self._model_version = 3
        self._sample_counter = 0
        self.served = []

    def _serve(self, e):
        self.served.append(e)
        return e


def _draws(R, k):
    out = []
    for _ in range(k):
        out.append(R.rand())
        out.append(float(sps.truncnorm.rvs(-0.5, 1.5, loc=0.2, scale=0.3, random_state=R)))
        out.append(int(R.randint(7)))
    return out


def test_raw_state_snapshot_and_private_copy():
    g = B._global_mt()
    np.random.seed(11)
    snap = g.snap()
    assert len(snap) == B._MT.NB
    want = _draws(np.random.mtrand._rand, 5)
    g.load(snap)  # back to the snapshot: the same draws again
    assert _draws(np.random.mtrand._rand, 5) == want
    rs = np.random.RandomState()
    pm = B._MT(rs)
    pm.load(snap)  # a private copy draws exactly what the global RNG drew
    assert _draws(rs, 5) == want
    assert g.snap() != snap  # the global RNG moved on its own


def _batch(gen, k):
    """A batch of k 'calls', each drawing from a private copy: states[j] before call j."""
    g = B._global_mt()
    rs = np.random.RandomState()
    pm = B._MT(rs)
    states = [g.snap()]
    pm.load(states[0])
    entries = []
    for j in range(k):
        entries.append(("call", j, rs.rand()))
        states.append(pm.snap())
    return B.SpeculativeBatch(gen, entries, states, [gen._sample_counter] * (k + 1), gen._model_version)


def test_take_serves_in_order_and_moves_the_global_state():
    np.random.seed(5)
    seq = [np.random.rand() for _ in range(4)]
    after_seq = B._global_mt().snap()
    np.random.seed(5)
    gen = _Gen()
    spec = _batch(gen, 4)
    assert B._global_mt().snap() != after_seq  # building the batch drew nothing from the global RNG
    got = [spec.take()[2] for _ in range(4)]
    assert got == seq
    assert B._global_mt().snap() == after_seq  # left where four sequential calls leave it
    assert spec.take() is None and spec.continues()


def test_take_refuses_after_a_foreign_draw_and_never_replays_it():
    np.random.seed(6)
    gen = _Gen()
    spec = _batch(gen, 3)
    first = spec.take()
    other = np.random.rand()  # another thread draws between two requests
    assert spec.take() is None  # the next result would not be the sequential call's
    assert not spec.continues()
    np.random.seed(6)
    np.random.rand()
    assert np.random.rand() == other  # the foreign draw got the value after call 0: nothing replayed
    assert first[1] == 0


def test_take_refuses_after_a_refit():
    np.random.seed(7)
    gen = _Gen()
    spec = _batch(gen, 3)
    spec.take()
    gen._model_version += 1
    assert spec.take() is None


def test_concurrent_draws_are_never_duplicated():
    """A thread drawing from the global RNG throughout, while batches are served: no value repeats."""
    np.random.seed(8)
    stop, vals = threading.Event(), []

    def worker():
        while not stop.is_set():
            vals.append(np.random.rand())
    t = threading.Thread(target=worker)
    t.start()
    try:
        for _ in range(200):
            gen = _Gen()
            spec = _batch(gen, 4)
            while spec.take() is not None:
                pass
    finally:
        stop.set()
        t.join()
    assert len(vals) > 50
    assert len(set(vals)) == len(vals)
