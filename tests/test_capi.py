"""The C-ABI library loads and exports every entry point include/hbx.h declares (no GPU needed)."""
import ctypes
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(ROOT, "include", "hbx.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(hbx_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_entry_points():
    names = header_functions()
    assert "hbx_kde_acquire" in names and "hbx_sh_promote" in names and "hbx_kde_fit" in names
    assert len(names) >= 18


def test_library_exports_every_header_symbol():
    from hpbandster_amd import _native as N
    L = N.lib()
    for name in header_functions():
        assert hasattr(L, name), name
        assert name in N.SIGNATURES, "ctypes signature missing for %s" % name


def test_host_side_helpers():
    from hpbandster_amd import _native as N
    L = N.lib()
    assert L.hbx_version().decode().startswith("hbx")
    assert L.hbx_max_dims() == 256
    assert L.hbx_kde_param_bytes() > 0 and L.hbx_acq_result_bytes() == 48
    assert L.hbx_kde_est_bytes() == 16
    a, b, s = np.zeros(1, np.int32), np.zeros(1, np.int32), np.zeros(1, np.int32)
    assert L.hbx_kde_bucket(24, 8, a.ctypes.data, b.ctypes.data, s.ctypes.data) == 0
    assert (a[0], b[0]) == (24, 8) and s[0] == 28 * 80 + 64 * 8
    tf = L.hbx_kde_table_floats(100, 24, 8)  # capacity: largest layout prepare may pick, 2 chunks
    assert tf % 2 == 0 and tf // 2 >= 28 * 80 + 64 * 4 * 16 * 2
    assert L.hbx_kde_bucket(100, 0, a.ctypes.data, b.ctypes.data, s.ctypes.data) == -3
    assert b"continuous" in L.hbx_last_error()
    assert L.hbx_kde_workspace_bytes(1000, 100) > 1000 * 16


def test_errors_are_reported_not_swallowed():
    from hpbandster_amd import _native as N
    L = N.lib()
    rc = L.hbx_kde_acquire(None, 10, 3, 0, None, None, None, None, 0, None, None, None, None, 0, 4, 0,
                           10, None, None, None, 0, None, None)
    assert rc == -1
    with pytest.raises(N.HbxError):
        N.check(rc)


# Philox4x32-10 known-answer vectors (Random123 kat_vectors: counter, key -> output)
PHILOX_KAT = [
    ([0, 0, 0, 0], [0, 0], [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]),
    ([0xffffffff] * 4, [0xffffffff] * 2, [0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd]),
    ([0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344], [0xa4093822, 0x299f31d0],
     [0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1]),
]


@pytest.mark.parametrize("ctr,key,want", PHILOX_KAT)
def test_philox_known_answers(ctr, key, want):
    """The sampler's generator (hbx_philox.h, host build of the same function the kernel uses)."""
    from hpbandster_amd import _native as N
    c, k, o = np.array(ctr, np.uint32), np.array(key, np.uint32), np.zeros(4, np.uint32)
    N.check(N.lib().hbx_philox4x32_10(N.ptr(c), N.ptr(k), N.ptr(o)))
    assert [int(v) for v in o] == want


def test_pair_binding_host_side():
    """hbx_kde_pair_bind keeps the fixed arguments of a KDE pair (no GPU: host memory only); bad ones give
    NULL and the error text, and the bound call refuses a NULL pair."""
    from hpbandster_amd import _native as N
    L = N.lib()
    h = L.hbx_kde_pair_bind(32, 1, 2, 3, 4, 0, 5, 6, 7, 8, 0, 24, 8, 10000)
    assert h
    L.hbx_kde_pair_free(h)
    assert not L.hbx_kde_pair_bind(0, 1, 2, 3, 4, 0, 5, 6, 7, 8, 0, 24, 8, 10000)
    assert b"hbx_kde_pair_bind" in L.hbx_last_error()
    assert not L.hbx_kde_pair_bind(32, None, 2, 3, 4, 0, 5, 6, 7, 8, 0, 24, 8, 10000)
    rec = ctypes.create_string_buffer(64)
    assert L.hbx_kde_acquire_bound(None, None, 0, 0, None, 0, None, None, None, rec, None) != 0
    L.hbx_kde_pair_free(None)
