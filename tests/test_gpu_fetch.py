"""hbx_fetch (include/hbx.h) and hbx_kde_acquire_bound: device bytes to the host without a blocking
synchronisation -- through the thread's mapped buffer (<= 4096 aligned bytes, a completion word) or a
copy plus stream polling (larger / unaligned) -- and the acquisition whose final kernel stores its record
into mapped memory: the same bytes as the workspace's record."""
import ctypes
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("nbytes,offset", [(0, 0), (4, 0), (48, 0), (4096, 0), (4100, 0), (100000, 0), (48, 1), (47, 4)])
def test_fetch_sizes_and_alignment(device, nbytes, offset):
    import torch
    from hpbandster_amd import _native as N
    src = torch.randint(0, 256, (nbytes + offset + 8,), dtype=torch.uint8, device=device)
    want = src[offset:offset + nbytes].cpu().numpy()
    dst = ctypes.create_string_buffer(max(nbytes, 1))
    N.check(N.lib().hbx_fetch(dst, src.data_ptr() + offset, nbytes, N.stream_handle(None, device)))
    assert np.frombuffer(dst.raw[:nbytes], dtype=np.uint8).tobytes() == want.tobytes()


def test_fetch_waits_for_queued_work_and_threads(device):
    """The record fetched after a long queue of work is the final value; two threads each with their own
    mapped buffer."""
    import torch
    from hpbandster_amd import _native as N
    out = {}

    def run(tag):
        x = torch.zeros(1 << 22, dtype=torch.float32, device=device)
        for _ in range(20):
            x += 1.0
        s = x[-4:].view(torch.uint8)
        dst = ctypes.create_string_buffer(16)
        N.check(N.lib().hbx_fetch(dst, s.data_ptr(), 16, N.stream_handle(None, device)))
        out[tag] = np.frombuffer(dst.raw, dtype=np.float32)

    ts = [threading.Thread(target=run, args=(i,)) for i in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    for i in range(2):
        assert (out[i] == 20.0).all()


def test_acquire_host_record_equals_workspace_record(device):
    import torch
    from hpbandster_amd import kde
    from hpbandster_amd import synthetic as S
    X = S.make_observations(800, 6, 2, 3, seed=5)
    pair = kde.fit_pair(X, S.make_losses(800, seed=6), S.var_type_string(6, 2), 9, device=device)
    C = torch.from_numpy(S.make_candidates(3000, 6, 2, 3, seed=7)).to(device)
    ws = torch.empty(pair.workspace_bytes(3000), dtype=torch.uint8, device=device)
    r_host = pair.acquire(C, workspace=ws, index_base=11)  # hbx_kde_acquire_bound
    off = pair.result_offset()
    r_ws = kde.AcqResult.from_bytes(ws[off:off + kde.RESULT_BYTES].cpu().numpy().tobytes())
    r_async = kde.AcqResult.from_bytes(kde.fetch_bytes(pair.acquire(C, workspace=ws, index_base=11, sync=False)))
    for r in (r_ws, r_async):
        assert (r.index, r.score, r.pdf_l, r.pdf_g, r.shortlist, r.flags) == \
               (r_host.index, r_host.score, r_host.pdf_l, r_host.pdf_g, r_host.shortlist, r_host.flags)
    empty = pair.acquire(C[:0], workspace=ws)
    assert empty.index == -1


def test_bound_pair_record_equals_the_async_record(device):
    """hbx_kde_acquire_bound (the drop-in's synchronous call: the pair's fixed arguments bound once) stores the
    same 48 bytes as hbx_kde_acquire with every argument passed (fetched from its workspace), and the record
    published to mapped memory equals the workspace's -- over many back-to-back calls (the completion word per
    call); with err and row_out (one wait for the whole pick) the record is the same, the row is the winner's,
    and a set error flag comes back as HBX_ACQ_DOMAIN_ERR."""
    import torch
    from hpbandster_amd import _native as N
    from hpbandster_amd import kde
    from hpbandster_amd import synthetic as S
    X = S.make_observations(1200, 24, 8, 4, seed=15)
    pair = kde.fit_pair(X, S.make_losses(1200, seed=16), S.var_type_string(24, 8), 33, device=device)
    C = torch.from_numpy(S.make_candidates(20000, 24, 8, 4, seed=17)).to(device)
    ws = torch.empty(pair.workspace_bytes(20000), dtype=torch.uint8, device=device)
    L = N.lib()
    sh = N.stream_handle(None, device)
    off = pair.result_offset()
    err = torch.zeros(20000, dtype=torch.uint8, device=device)
    for base in (0, 5, 1 << 33):
        a, c = ctypes.create_string_buffer(64), ctypes.create_string_buffer(64)
        N.check(L.hbx_kde_acquire_bound(pair._bound, C.data_ptr(), 20000, base, ws.data_ptr(), ws.numel(), None,
                                        None, sh, a, None))
        w = ws[off:off + kde.RESULT_BYTES].cpu().numpy().tobytes()
        N.check(L.hbx_kde_acquire(C.data_ptr(), 20000, 32, base, *pair._kde_args, None, None, ws.data_ptr(),
                                  ws.numel(), None, sh))
        b = kde.fetch_bytes(ws[off:off + kde.RESULT_BYTES])
        assert a.raw[:kde.RESULT_BYTES] == b == w
        r = kde.AcqResult.from_bytes(a.raw[:kde.RESULT_BYTES])
        assert r.index >= base
        row = np.full(32, np.nan)
        N.check(L.hbx_kde_acquire_bound(pair._bound, C.data_ptr(), 20000, base, ws.data_ptr(), ws.numel(),
                                        err.data_ptr(), None, sh, c, row.ctypes.data))
        assert c.raw[:kde.RESULT_BYTES] == a.raw[:kde.RESULT_BYTES]
        np.testing.assert_array_equal(row, C[r.index - base].cpu().numpy())
    err[17] = 1
    rec = pair.acquire_pick(C, err, ws, row)
    assert rec.flags & kde.ACQ_DOMAIN_ERR and rec.index == r.index - (1 << 33)
    seen = {pair.acquire(C[i * 1000:(i + 1) * 1000]).index for i in range(20)}
    assert len(seen) > 1 and min(seen) >= 0


def test_tagged_record_words_interleaved_with_fetches(device):
    """hbx_kde_acquire_bound's record travels as sequence-tagged words in the thread's mapped buffer, beside
    hbx_fetch's untagged bytes: 300 calls alternating with fetches on the same thread (their data written where
    no tag is read), picks with and without rows, varying candidate sets -- every record equals the workspace's
    record and every row the winner's."""
    import torch
    from hpbandster_amd import _native as N
    from hpbandster_amd import kde
    from hpbandster_amd import synthetic as S
    X = S.make_observations(400, 24, 8, 4, seed=25)
    pair = kde.fit_pair(X, S.make_losses(400, seed=26), S.var_type_string(24, 8), 33, device=device)
    C = torch.from_numpy(S.make_candidates(6400, 24, 8, 4, seed=27)).to(device)
    ws = torch.empty(pair.workspace_bytes(6400), dtype=torch.uint8, device=device)
    L = N.lib()
    sh = N.stream_handle(None, device)
    off = pair.result_offset()
    err = torch.zeros(6400, dtype=torch.uint8, device=device)
    junk = torch.randint(0, 256, (4096,), dtype=torch.uint8, device=device)
    rs = np.random.RandomState(3)
    for it in range(300):
        lo = int(rs.randint(0, 6336))
        n = int(rs.randint(1, 65))
        dst = ctypes.create_string_buffer(4096)  # a fetch first: arbitrary bytes through the same mapped buffer
        N.check(L.hbx_fetch(dst, junk.data_ptr(), 4096, sh))
        a = ctypes.create_string_buffer(64)
        row = np.full(32, np.nan)
        pick = it % 2 == 1
        N.check(L.hbx_kde_acquire_bound(pair._bound, C[lo:].data_ptr(), n, lo, ws.data_ptr(), ws.numel(),
                                        err.data_ptr() if pick else None, None, sh, a,
                                        row.ctypes.data if pick else None))
        w = kde.fetch_bytes(ws[off:off + kde.RESULT_BYTES])
        assert a.raw[:kde.RESULT_BYTES] == w, it
        r = kde.AcqResult.from_bytes(w)
        if pick and r.index >= 0:
            np.testing.assert_array_equal(row, C[r.index].cpu().numpy())


def test_mapped_buffers_pooled_across_short_lived_threads(device):
    """Each thread that fetches, acquires or refits holds device-mapped host buffers (include/hbx.h
    hbx_fetch); when it ends they go back to a process-wide pool with their sequence numbers: 40 short-lived
    threads one after another, each a fetch, a bound acquisition and a refit, allocate no buffer past the first
    thread's -- and every record, fetched value and refit is right (a pooled buffer's old completion word and
    tags never pass for the new owner's)."""
    import torch
    from hpbandster_amd import _native as N
    from hpbandster_amd import kde
    from hpbandster_amd import synthetic as S
    Lb = N.lib()
    X = S.make_observations(340, 6, 2, 3, seed=41)
    Ls = S.make_losses(340, seed=42)
    vt = S.var_type_string(6, 2)
    store = kde.ObservationStore(8, vt, device=device, capacity=400)
    store.add(X[:300], Ls[:300])
    C = torch.from_numpy(S.make_candidates(2000, 6, 2, 3, seed=43)).to(device)
    sh = N.stream_handle(None, device)
    out, errors = [], []

    def run(i):
        try:
            torch.cuda.set_device(device)
            src = torch.full((12,), i, dtype=torch.int32, device=device)
            dst = ctypes.create_string_buffer(48)
            N.check(Lb.hbx_fetch(dst, src.data_ptr(), 48, sh))
            assert (np.frombuffer(dst.raw, dtype=np.int32) == i).all()
            store.add(X[300 + i:301 + i], Ls[300 + i:301 + i])
            pair = store.refit(9)
            ref = kde.fit_pair(X[:301 + i], Ls[:301 + i], vt, 9, device=device)
            r = pair.acquire(C)
            r_ref = ref.acquire(C)
            out.append((i, r.index, r.score, r_ref.index, r_ref.score))
        except Exception as e:  # noqa: BLE001 (re-raised on the main thread)
            errors.append((i, e))

    def one(i):
        t = threading.Thread(target=run, args=(i,))
        t.start()
        t.join()

    one(0)
    base = int(Lb.hbx_mapped_host_buffers())
    for i in range(1, 40):
        one(i)
    assert not errors, errors
    assert int(Lb.hbx_mapped_host_buffers()) == base
    assert len(out) == 40
    for i, a, sa, b, sb in out:
        assert (a, sa) == (b, sb), i
