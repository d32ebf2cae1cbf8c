"""The drop-in's refit (ObservationStore.refit -> hbx_kde_refit_sync: the appended rows carried in the
sort launch's kernel arguments when they fit, else copied through the scratch; the column statistics written
by the fit launch; the table launch's last block finishing each KDE) against the separate preparation of the
same split (hbx_kde_prepare through fit_pair_from_rows) -- the same kernel instance, the same acquisition
records and fp32 ln-pdf estimates bit for bit (every table element the scoring reads) -- and against the
oracle's split and np.std bandwidths; at up to 1024 rows (one sort launch), above (the segmented sort), and at
D = 1 (numpy's pairwise column sum); rows staged from device memory give the same blocks."""
import numpy as np
import pytest

from oracle import kde_oracle as O

pytestmark = pytest.mark.gpu

SHAPES = [  # (dc, du, levels, n, n_new)
    (24, 8, 4, 400, 1),
    (8, 0, 0, 1000, 1),
    (16, 4, 3, 120, 7),     # 7 x 21 = 147 staged doubles: inline
    (24, 8, 4, 300, 12),    # 12 x 33 = 396: through the scratch
    (6, 2, 5, 1024, 1),     # the one-launch sort's cap exactly
    (40, 0, 0, 200, 1),
    (24, 8, 4, 1500, 1),    # above the cap: the segmented sort, rows through the scratch
    (1, 0, 0, 300, 1),      # D = 1 (numpy's pairwise column sum)
]


def _store_pair(device, dc, du, lev, n, n_new, seed):
    from hpbandster_amd import kde
    from hpbandster_amd import synthetic as S
    X = S.make_observations(n, dc, du, lev, seed=seed)
    L = S.make_losses(n, seed=seed + 1)
    vt = S.var_type_string(dc, du)
    store = kde.ObservationStore(dc + du, vt, device=device, capacity=n + 8)
    store.add(X[:n - n_new], L[:n - n_new])
    store.refit(dc + du + 1)
    store.add(X[n - n_new:], L[n - n_new:])
    return X, L, vt, store.refit(dc + du + 1)


@pytest.mark.parametrize("dc,du,lev,n,n_new", SHAPES)
def test_one_launch_refit_equals_prepare(device, dc, du, lev, n, n_new):
    from hpbandster_amd import kde
    from hpbandster_amd import synthetic as S
    X, L, vt, pair = _store_pair(device, dc, du, lev, n, n_new, 31 + n)
    g_idx, b_idx = O.bohb_split(X, L, dc + du + 1)
    np.testing.assert_array_equal(pair.good.rows_dev.cpu().numpy(), g_idx)
    np.testing.assert_array_equal(pair.bad.rows_dev.cpu().numpy(), b_idx)
    np.testing.assert_array_equal(pair.good.bw, O.normal_reference_bw(X[g_idx]))
    np.testing.assert_array_equal(pair.bad.bw, O.normal_reference_bw(X[b_idx]))
    np.testing.assert_array_equal(pair.good.nlev, O.num_levels(X[g_idx], vt))
    np.testing.assert_array_equal(pair.bad.nlev, O.num_levels(X[b_idx], vt))
    ref = kde.fit_pair_from_rows(X, g_idx, b_idx, vt, pair.good.bw, pair.bad.bw, pair.good.nlev, pair.bad.nlev,
                                 device=device)
    for a, b in ((pair.good, ref.good), (pair.bad, ref.bad)):
        assert (a.variant, a.dc_pad, a.du_pad, a.kc) == (b.variant, b.dc_pad, b.du_pad, b.kc)
    C = S.make_candidates(700, dc, du, lev, seed=5 + n)
    if du:
        C[::3, dc:] = X[g_idx[np.arange(len(C[::3])) % len(g_idx)], dc:]
    r1, l1, g1 = pair.acquire(C, logs=True)
    r2, l2, g2 = ref.acquire(C, logs=True)
    assert (r1.index, r1.score, r1.pdf_l, r1.pdf_g) == (r2.index, r2.score, r2.pdf_l, r2.pdf_g)
    np.testing.assert_array_equal(np.asarray(l1), np.asarray(l2))
    np.testing.assert_array_equal(np.asarray(g1), np.asarray(g2))


def test_device_staged_rows_equal_host_rows(device):
    """hbx_kde_refit (rows staged in device memory) and hbx_kde_refit_sync (rows from host memory) give the same
    output block, parameter blocks and tables."""
    import torch
    from hpbandster_amd import _native as N
    from hpbandster_amd import kde
    from hpbandster_amd import synthetic as S
    dc, du, lev, n, n_new = 24, 8, 4, 500, 3
    D = dc + du
    X = S.make_observations(n, dc, du, lev, seed=77)
    L = S.make_losses(n, seed=78)
    vt = np.array([0] * dc + [1] * du, dtype=np.int32)
    ng, nb = kde.bohb_split_sizes(n, D + 1)
    Lb = N.lib()
    outs = []
    for host in (True, False):
        Xd = torch.zeros((n, D), dtype=torch.float64, device=device)
        Ld = torch.zeros(n, dtype=torch.float64, device=device)
        Xd[:n - n_new] = torch.from_numpy(X[:n - n_new]).to(device)
        Ld[:n - n_new] = torch.from_numpy(L[:n - n_new]).to(device)
        st = np.concatenate([X[n - n_new:].reshape(-1), L[n - n_new:]])
        ob, sb, pb = (int(Lb.hbx_kde_refit_out_bytes(n, D)), int(Lb.hbx_kde_refit_scratch_bytes(n, D)),
                      int(Lb.hbx_kde_param_bytes()))
        dcp, dup = kde.scoring_bucket(vt)
        tgf, tbf = int(Lb.hbx_kde_table_floats(ng, dcp, dup)), int(Lb.hbx_kde_table_floats(nb, dcp, dup))
        out = torch.zeros(ob, dtype=torch.uint8, device=device)
        scr = torch.zeros(sb, dtype=torch.uint8, device=device)
        pg, pbd = (torch.zeros(pb, dtype=torch.uint8, device=device) for _ in range(2))
        tg = torch.zeros(tgf, dtype=torch.float32, device=device)
        tb = torch.zeros(tbf, dtype=torch.float32, device=device)
        fg, fb = kde.bandwidth_factor(ng, D), kde.bandwidth_factor(nb, D)
        if host:
            hb = np.empty(ob, dtype=np.uint8)
            N.call("hbx_kde_refit_sync", N.ptr(Xd), N.ptr(Ld), n, D, vt.ctypes.data, st.ctypes.data, n_new, ng, nb,
                   fg, fb, N.ptr(pg), N.ptr(tg), tgf, N.ptr(pbd), N.ptr(tb), tbf, N.ptr(out), N.ptr(scr), sb,
                   N.stream_handle(), hb.ctypes.data)
        else:
            sd = torch.from_numpy(st).to(device)
            N.call("hbx_kde_refit", N.ptr(Xd), N.ptr(Ld), n, D, vt.ctypes.data, N.ptr(sd), n_new, ng, nb, fg, fb,
                   N.ptr(pg), N.ptr(tg), tgf, N.ptr(pbd), N.ptr(tb), tbf, N.ptr(out), N.ptr(scr), sb,
                   N.stream_handle())
        torch.cuda.synchronize()
        kp = int(Lb.hbx_kde_param_bytes())
        outs.append((out.cpu().numpy(), tg.cpu().numpy().view(np.int32), tb.cpu().numpy().view(np.int32),
                     Xd.cpu().numpy(), Ld.cpu().numpy(), kp))
    a, b = outs
    for x, y in zip(a[:5], b[:5]):
        np.testing.assert_array_equal(x, y)
    np.testing.assert_array_equal(a[3], X)
    np.testing.assert_array_equal(a[4], L)


@pytest.mark.parametrize("dc,du,lev,n,n_new", [(24, 8, 4, 400, 1), (8, 0, 0, 1000, 2), (24, 8, 4, 3000, 1),
                                               (70, 0, 0, 300, 1), (4, 40, 3, 200, 1)])
def test_sync_refit_publishes_the_output_block(device, dc, du, lev, n, n_new):
    """hbx_kde_refit_sync's host copy of the output block (published by the finishing workgroups through mapped
    host memory -- the table launch's last blocks, or the separate finish launch when a KDE is exact-only) equals
    the device block and the block of hbx_kde_refit (rows staged in device memory); three calls in a row (the
    sequence), a block larger than the first mapped buffer (it grows)."""
    import torch
    from hpbandster_amd import _native as N
    from hpbandster_amd import kde
    from hpbandster_amd import synthetic as S
    D = dc + du
    X = S.make_observations(n, dc, du, lev, seed=91 + n)
    L = S.make_losses(n, seed=92 + n)
    vt = np.array([0] * dc + [1] * du, dtype=np.int32)
    ng, nb = kde.bohb_split_sizes(n, D + 1)
    Lb = N.lib()
    ob, sb, pb = (int(Lb.hbx_kde_refit_out_bytes(n, D)), int(Lb.hbx_kde_refit_scratch_bytes(n, D)),
                  int(Lb.hbx_kde_param_bytes()))
    dcp, dup = kde.scoring_bucket(vt)
    tgf, tbf = int(Lb.hbx_kde_table_floats(ng, dcp, dup)), int(Lb.hbx_kde_table_floats(nb, dcp, dup))
    fg, fb = kde.bandwidth_factor(ng, D), kde.bandwidth_factor(nb, D)
    st = np.concatenate([X[n - n_new:].reshape(-1), L[n - n_new:]])
    blocks = []
    for call in ("hbx_kde_refit", "hbx_kde_refit_sync", "hbx_kde_refit_sync", "hbx_kde_refit_sync"):
        Xd = torch.zeros((n, D), dtype=torch.float64, device=device)
        Ld = torch.zeros(n, dtype=torch.float64, device=device)
        Xd[:n - n_new] = torch.from_numpy(X[:n - n_new]).to(device)
        Ld[:n - n_new] = torch.from_numpy(L[:n - n_new]).to(device)
        out = torch.zeros(ob, dtype=torch.uint8, device=device)
        scr = torch.zeros(sb, dtype=torch.uint8, device=device)
        pg, pbd = (torch.zeros(pb, dtype=torch.uint8, device=device) for _ in range(2))
        tg = torch.zeros(max(tgf, 1), dtype=torch.float32, device=device)
        tb = torch.zeros(max(tbf, 1), dtype=torch.float32, device=device)
        sd = torch.from_numpy(st).to(device)  # (hbx_kde_refit: the staged rows in device memory)
        args = [N.ptr(Xd), N.ptr(Ld), n, D, vt.ctypes.data, st.ctypes.data if call == "hbx_kde_refit_sync" else
                N.ptr(sd), n_new, ng, nb, fg, fb, N.ptr(pg), N.ptr(tg), tgf, N.ptr(pbd), N.ptr(tb), tbf, N.ptr(out),
                N.ptr(scr), sb, N.stream_handle()]
        host = np.full(ob, 0xAB, dtype=np.uint8)
        if call == "hbx_kde_refit_sync":
            N.call(call, *args, host.ctypes.data)
        else:
            N.call(call, *args)
        torch.cuda.synchronize()
        dev_block = out.cpu().numpy()
        if call == "hbx_kde_refit_sync":
            np.testing.assert_array_equal(host, dev_block)
        blocks.append(dev_block)
    for b in blocks[1:]:
        np.testing.assert_array_equal(b, blocks[0])
    info = blocks[0][8 * n + 24 * D:].view(np.int32)
    if dc > 64:
        assert (info[0] >> 5) & 1 and (info[8] >> 5) & 1  # exact-only KDEs: the finish launch published


def test_sync_refit_rejects_bad_codes_then_recovers(device):
    """A categorical code that is not an integer in [0, 1024) makes hbx_kde_refit_sync fail with the drop-in's
    message (its level-count check on the host block); the thread's next call on valid rows succeeds."""
    import torch
    from hpbandster_amd import _native as N
    from hpbandster_amd import kde
    from hpbandster_amd import synthetic as S
    dc, du, lev, n = 6, 2, 3, 120
    D = dc + du
    vt = np.array([0] * dc + [1] * du, dtype=np.int32)
    ng, nb = kde.bohb_split_sizes(n, D + 1)
    Lb = N.lib()
    ob, sb, pb = (int(Lb.hbx_kde_refit_out_bytes(n, D)), int(Lb.hbx_kde_refit_scratch_bytes(n, D)),
                  int(Lb.hbx_kde_param_bytes()))
    dcp, dup = kde.scoring_bucket(vt)
    tgf, tbf = int(Lb.hbx_kde_table_floats(ng, dcp, dup)), int(Lb.hbx_kde_table_floats(nb, dcp, dup))
    for bad in (True, False):
        X = S.make_observations(n, dc, du, lev, seed=7)
        if bad:
            X[:, dc] = 0.5  # every row: not an integer code, in both sets
        L = S.make_losses(n, seed=8)
        Xd = torch.from_numpy(X).to(device)
        Ld = torch.from_numpy(L).to(device)
        out = torch.zeros(ob, dtype=torch.uint8, device=device)
        scr = torch.zeros(sb, dtype=torch.uint8, device=device)
        pg, pbd = (torch.zeros(pb, dtype=torch.uint8, device=device) for _ in range(2))
        tg = torch.zeros(tgf, dtype=torch.float32, device=device)
        tb = torch.zeros(tbf, dtype=torch.float32, device=device)
        host = np.zeros(ob, dtype=np.uint8)
        args = [N.ptr(Xd), N.ptr(Ld), n, D, vt.ctypes.data, None, 0, ng, nb, kde.bandwidth_factor(ng, D),
                kde.bandwidth_factor(nb, D), N.ptr(pg), N.ptr(tg), tgf, N.ptr(pbd), N.ptr(tb), tbf, N.ptr(out),
                N.ptr(scr), sb, N.stream_handle(), host.ctypes.data]
        if bad:
            with pytest.raises(N.HbxError, match="categorical codes"):
                N.call("hbx_kde_refit_sync", *args)
        else:
            N.call("hbx_kde_refit_sync", *args)
            torch.cuda.synchronize()
            np.testing.assert_array_equal(host, out.cpu().numpy())
            g_idx, _ = O.bohb_split(X, L, D + 1)
            np.testing.assert_array_equal(host[:8 * n].view(np.int64)[:ng], g_idx)


def test_sync_refit_every_published_word_over_many_calls(device):
    """300 back-to-back refits through the drop-in's store (hbx_kde_refit_sync), one row more each time, the
    store's device arrays growing on the way: the host block each call returned (the models' bw / nlev / rows
    views) equals the device output block word for word."""
    from hpbandster_amd import _native as N
    from hpbandster_amd import kde
    from hpbandster_amd import synthetic as S
    dc, du, lev, n0, calls = 24, 8, 4, 200, 300
    D = dc + du
    X = S.make_observations(n0 + calls, dc, du, lev, seed=123)
    L = S.make_losses(n0 + calls, seed=124)
    store = kde.ObservationStore(D, S.var_type_string(dc, du), device=device, capacity=64)
    store.add(X[:n0], L[:n0])
    for i in range(calls):
        store.add(X[n0 + i], L[n0 + i])
        pair = store.refit(D + 1)
        host = pair.good.bw
        while host.base is not None:
            host = host.base
        ob = int(N.lib().hbx_kde_refit_out_bytes(n0 + i + 1, D))
        assert host.nbytes == ob
        np.testing.assert_array_equal(host.view(np.uint8), pair._keep[0][:ob].cpu().numpy())


def test_refit_then_acquire_on_another_stream(device):
    """A model refit on the current stream and used at once from another stream (a side stream of another
    thread's work): hbx_kde_refit_sync returns with the refit's launches complete, so the acquisition there sees
    the finished parameter blocks and tables -- its record equals the same acquisition on the refit's stream."""
    import torch
    from hpbandster_amd import kde
    from hpbandster_amd import synthetic as S
    dc, du, lev, n0 = 24, 8, 4, 400
    D = dc + du
    X = S.make_observations(n0 + 20, dc, du, lev, seed=125)
    L = S.make_losses(n0 + 20, seed=126)
    C = torch.from_numpy(S.make_candidates(4096, dc, du, lev, seed=127)).to(device)
    store = kde.ObservationStore(D, S.var_type_string(dc, du), device=device)
    store.add(X[:n0], L[:n0])
    side = torch.cuda.Stream(device)
    for i in range(20):
        store.add(X[n0 + i], L[n0 + i])
        pair = store.refit(D + 1)
        with torch.cuda.stream(side):
            r = pair.acquire(C, stream=side)
        torch.cuda.synchronize()
        ref = pair.acquire(C)
        assert (r.index, r.score, r.pdf_l, r.pdf_g) == (ref.index, ref.score, ref.pdf_l, ref.pdf_g)
