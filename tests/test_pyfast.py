"""_hbxfast (hbx_pyfast.c), advance_mask's buffer-protocol call into hbx_sh_advance_state: it is built
in-tree, loads, and hands every buffer it cannot take straight back (rc 1) without touching the GPU --
wrong dtype, wrong rank, a mask of the wrong size or type, more configurations than the staging holds."""
import ctypes
import importlib.util
import os

import numpy as np
import pytest


def _load():
    from hpbandster_amd import _native as N
    from hpbandster_amd import build as B
    path = B.pyfast_path()
    if not os.path.exists(path):
        pytest.skip("_hbxfast not built (run __graft_entry__.build())")
    spec = importlib.util.spec_from_file_location("hpbandster_amd._hbxfast", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod, N


def test_pyfast_rejects_what_it_cannot_take():
    mod, N = _load()
    with pytest.raises(RuntimeError):
        mod.advance(0, 8, np.zeros(4), np.zeros(4, np.bool_), 1.0, 0)  # no entry yet
    mod.set_entry(ctypes.cast(N.lib().hbx_sh_advance_state, ctypes.c_void_p).value)
    state = (ctypes.c_int64 * 6)()
    sa = ctypes.addressof(state)
    ok = np.zeros(4, np.bool_)
    assert mod.advance(sa, 8, np.zeros(4, np.float32), ok, 1.0, 0) == 1
    assert mod.advance(sa, 8, np.zeros((2, 2)), ok, 1.0, 0) == 1
    assert mod.advance(sa, 8, np.zeros(4), np.zeros(5, np.bool_), 1.0, 0) == 1
    assert mod.advance(sa, 8, np.zeros(4), np.zeros(4, np.int32), 1.0, 0) == 1
    assert mod.advance(sa, 2, np.zeros(4), ok, 1.0, 0) == 1
    assert mod.advance(sa, 8, np.zeros(0), np.zeros(0, np.bool_), 1.0, 0) == 1
    assert mod.advance(sa, 8, np.zeros(8)[::2], ok, 1.0, 0) == 1  # not contiguous
    assert mod.advance(sa, 8, b"12345678", ok, 1.0, 0) == 1
    assert list(state) == [0] * 6  # nothing was called
