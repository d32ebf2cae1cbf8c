"""GPU parity: batched successive-halving promotion against the reference's golden masks."""
import numpy as np
import pytest

from oracle import kde_oracle as O
from tests import golden_cases as G

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("policy", ["gpu", "auto"])
def test_promotion_matches_reference(device, policy):
    from hpbandster_amd import promote
    for c in G.load_sh():
        losses = np.where(c["crashed"], np.nan, c["losses"])
        adv = promote.advance_mask(losses, c["k"], device=device, policy=policy)
        np.testing.assert_array_equal(adv, c["sh_adv"])
        adv = promote.advance_mask(losses, max(1, c["k"] * (1 - 0.5)), device=device, policy=policy)
        np.testing.assert_array_equal(adv, c["sr_adv"])


def test_size_policy_equals_gpu_path(device):
    """advance_mask's size policy (host ranking of tie-free brackets up to HOST_MAX) gives the GPU path's
    masks: tie-free, straddling and non-straddling ties, -0.0 against 0.0, non-finite losses, fractional,
    zero, NaN and oversized k, at sizes across the argsort / partition switch and past 1024."""
    from hpbandster_amd import promote
    rs = np.random.RandomState(77)
    for n in (1, 2, 3, 27, 81, 255, 256, 257, 700, 1024, 1025, 3000):
        for trial in range(4):
            if trial == 0:
                losses = rs.rand(n)
            elif trial == 1:
                losses = np.round(rs.rand(n) * 5) / 5
            elif trial == 2:
                losses = rs.rand(n)
                losses[rs.rand(n) < 0.1] = rs.choice([np.inf, -np.inf, np.nan, -0.0, 0.0])
            else:
                losses = rs.randn(n) * 10.0 ** rs.randint(-3, 3, n)
            for k in (n // 3, max(1, n // 2) + 0.5, 0, n, n + 4, float("nan"), 1):
                want = promote.advance_mask(losses, k, device=device, policy="gpu")
                got = promote.advance_mask(losses, k, device=device, policy="auto")
                np.testing.assert_array_equal(got, want, err_msg="n=%d trial=%d k=%r" % (n, trial, k))


def test_advance_mask_on_a_non_current_device():
    """The one-bracket state entry launches on the staging's device whatever device is current on the
    calling thread (a dispatcher thread's is 0): needs two visible GPUs."""
    import torch
    from hpbandster_amd import promote
    if not torch.cuda.is_available() or torch.cuda.device_count() < 2:
        pytest.skip("needs two GPUs")
    d1 = torch.device("cuda", 1)
    losses = np.random.RandomState(3).rand(500)
    want = np.argsort(np.argsort(losses)) < 166
    with torch.cuda.device(0):
        np.testing.assert_array_equal(promote.advance_mask(losses, 166, device=d1, policy="gpu"), want)
        assert torch.cuda.current_device() == 0


@pytest.mark.parametrize("B,n", [(1, 1), (3, 5000), (64, 1000), (1000, 81), (7, 4097)])
def test_batched_promotion_matches_oracle(device, B, n):
    from hpbandster_amd import promote
    rs = np.random.RandomState(B * 7 + n)
    lens = rs.randint(max(1, n // 2), n + 1, size=B)
    seg = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    loss = rs.rand(seg[-1])
    loss[rs.rand(seg[-1]) < 0.05] = np.inf
    loss[rs.rand(seg[-1]) < 0.02] = np.nan
    loss[rs.rand(seg[-1]) < 0.01] = -np.inf
    k = np.maximum(lens // 3, 1).astype(np.float64)
    adv = promote.promote_segments(loss, seg, k, device=device)
    for b in range(B):
        s, e = seg[b], seg[b + 1]
        np.testing.assert_array_equal(adv[s:e], O.sh_advance(loss[s:e], k[b]))


def test_promotion_ties_stable_and_numpy(device):
    from hpbandster_amd import promote
    loss = np.array([1.0] * 40 + [0.5] * 10)
    adv = promote.advance_mask(loss, 15, device=device, ties="stable", policy="gpu")
    assert adv[40:].all() and adv[:5].all() and not adv[5:40].any()
    # numpy 1.26.4's argsort of this array starts [40..45, 48, 49, 46, 47, 0, 1, 4, 5, 2, 3, ...]
    adv = promote.advance_mask(loss, 15, device=device)
    assert sorted(np.nonzero(adv)[0].tolist()) == [0, 1, 2, 4, 5] + list(range(40, 50))


def test_one_bracket_entries_agree(device):
    """hbx_sh_promote_one (stream-ordered: the selection launch, then the re-rank launch that works only on
    a straddling tie) on device buffers, and advance_mask (the mapped one-call path: a second launch only
    when the selection reports the tie), on tie-free, straddling-tie and non-straddling-tie brackets."""
    import torch
    from hpbandster_amd import _native as N
    from hpbandster_amd import promote
    rs = np.random.RandomState(21)
    cases = [(rs.rand(1000), 333), (np.array([1.0] * 40 + [0.5] * 10), 15), (np.round(rs.rand(1024), 1), 500),
             (np.array([0.25] * 7 + [0.75] * 9), 7), (np.array([3.0]), 1), (np.round(rs.rand(81), 2), 27)]
    for losses, k in cases:
        n = len(losses)
        for ties, mode in (("numpy", N.ORDER_NUMPY), ("stable", N.ORDER_STABLE)):
            want = promote.advance_mask(losses, k, device=device, ties=ties, policy="gpu")
            assert want.sum() == min(k, n)
            ld = torch.from_numpy(losses).to(device)
            ad = torch.full((n,), 7, dtype=torch.uint8, device=device)
            scr = torch.full((4 * n,), -1, dtype=torch.int32, device=device)
            N.check(N.lib().hbx_sh_promote_one(ld.data_ptr(), n, float(k), ad.data_ptr(),
                                               scr.data_ptr() if mode == N.ORDER_NUMPY else None, mode, None, 0,
                                               N.stream_handle()))
            torch.cuda.synchronize()
            np.testing.assert_array_equal(ad.cpu().numpy().astype(bool), want, err_msg="%s n=%d" % (ties, n))
            if ties == "numpy" and len(np.unique(losses)) == n:
                np.testing.assert_array_equal(want, np.argsort(np.argsort(losses)) < k)


def test_advance_state_sequence_wraps(device):
    """hbx_sh_advance_state's sequence number wraps from 2^31 - 2 to 1 (the completion word is never 0 or
    negative for a finished call) and a straddling tie (completion word -seq, then the re-rank launch)
    on either side of the wrap still yields numpy's masks."""
    from hpbandster_amd import promote
    tie = np.array([1.0] * 40 + [0.5] * 10)
    want_tie = promote.advance_mask(tie, 15, device=device, policy="gpu")
    assert sorted(np.nonzero(want_tie)[0].tolist()) == [0, 1, 2, 4, 5] + list(range(40, 50))
    rnd = np.random.RandomState(5).rand(700)
    want_rnd = np.argsort(np.argsort(rnd)) < 233
    st = promote._staging(device).get(700)
    st.state[5] = 0x7ffffffe - 2
    seqs = []
    for i in range(6):
        losses, k, want = (tie, 15, want_tie) if i % 2 else (rnd, 233, want_rnd)
        np.testing.assert_array_equal(promote.advance_mask(losses, k, device=device, policy="gpu"), want,
                                      err_msg="call %d" % i)
        seqs.append(int(st.state[5]))
    assert seqs == [0x7ffffffe - 1, 0x7ffffffe, 1, 2, 3, 4], seqs


def test_config5_shape_with_fit(device):
    """B=1e3 brackets x 1e3 configs (config #5 at 1/10 the brackets): promotion + per-bracket refit."""
    import torch
    from hpbandster_amd import _native as N
    from hpbandster_amd import kde
    from hpbandster_amd import synthetic as S
    B, n, D = 1000, 1000, 8
    losses = S.make_bracket_losses(B, n)
    seg = np.arange(B + 1, dtype=np.int64) * n
    from hpbandster_amd import promote
    adv = promote.promote_segments(losses.reshape(-1), seg, np.full(B, 333.0), device=device)
    assert adv.reshape(B, n).sum(1).tolist() == [333] * B
    for b in (0, 17, B - 1):
        np.testing.assert_array_equal(adv.reshape(B, n)[b], O.sh_advance(losses[b], 333))
    # batched KDE refit of every bracket (D=8 continuous)
    X = np.random.RandomState(4).rand(B * n, D)
    L = N.lib()
    dev = device
    Xd = torch.from_numpy(X).to(dev)
    ld = torch.from_numpy(losses.reshape(-1)).to(dev)
    segd = torch.from_numpy(seg).to(dev)
    order = torch.empty(B * n, dtype=torch.int64, device=dev)
    sb = int(L.hbx_sort_scratch_bytes(B * n))
    scr = torch.empty(sb, dtype=torch.uint8, device=dev)
    N.call("hbx_seg_argsort", N.ptr(ld), N.ptr(segd), B, n, B * n, N.ptr(order), N.ptr(scr), sb, N.stream_handle())
    ng, nb = kde.bohb_split_sizes(n, D + 1)
    ngd = torch.full((B,), ng, dtype=torch.int64, device=dev)
    nbd = torch.full((B,), nb, dtype=torch.int64, device=dev)
    fg = torch.full((B,), kde.bandwidth_factor(ng, D), dtype=torch.float64, device=dev)
    fb = torch.full((B,), kde.bandwidth_factor(nb, D), dtype=torch.float64, device=dev)
    vt = torch.zeros(D, dtype=torch.int32, device=dev)
    bwg = torch.empty((B, D), dtype=torch.float64, device=dev)
    bwb = torch.empty((B, D), dtype=torch.float64, device=dev)
    nlg = torch.empty((B, D), dtype=torch.int32, device=dev)
    nlb = torch.empty((B, D), dtype=torch.int32, device=dev)
    N.call("hbx_kde_fit", N.ptr(Xd), D, N.ptr(segd), B, N.ptr(order), N.ptr(ngd), N.ptr(nbd), N.ptr(fg), N.ptr(fb),
           N.ptr(vt), N.ptr(bwg), N.ptr(bwb), N.ptr(nlg), N.ptr(nlb), N.stream_handle())
    bwg, bwb = bwg.cpu().numpy(), bwb.cpu().numpy()
    for b in (0, 5, B - 1):
        Xb, Lb = X[b * n:(b + 1) * n], losses[b]
        good, bad = O.bohb_split(Xb, Lb, D + 1)
        np.testing.assert_array_equal(bwg[b], O.normal_reference_bw(Xb[good]))
        np.testing.assert_array_equal(bwb[b], O.normal_reference_bw(Xb[bad]))


def test_config5_full_shape_every_mask(device):
    """Config #5 at its full shape: 1e4 brackets x 1e3 configs, eta = 3 (k = 333): every one of the 1e7
    mask bytes against argsort(argsort(losses)) < k per bracket (HB_iteration.py:179-182; numpy's
    stable argsort, vectorised over the brackets -- the synthetic losses have no ties, so any argsort
    ranks them alike); and the same brackets sharded over two 'ranks' (independent calls on the two
    halves, no collective) give the same masks."""
    from hpbandster_amd import promote
    from hpbandster_amd import synthetic as S
    B, n, k = 10000, 1000, 333
    losses = S.make_bracket_losses(B, n)
    assert all(len(np.unique(r)) == n for r in losses[:50])
    want = np.argsort(np.argsort(losses, axis=1, kind="stable"), axis=1, kind="stable") < k
    seg = np.arange(B + 1, dtype=np.int64) * n
    adv = promote.promote_segments(losses.reshape(-1), seg, np.full(B, float(k)), device=device)
    np.testing.assert_array_equal(adv.reshape(B, n), want)
    h = B // 2
    a0 = promote.promote_segments(losses[:h].reshape(-1), seg[:h + 1], np.full(h, float(k)), device=device)
    a1 = promote.promote_segments(losses[h:].reshape(-1), seg[:B - h + 1], np.full(B - h, float(k)), device=device)
    np.testing.assert_array_equal(np.concatenate([a0, a1]), adv)


@pytest.mark.parametrize("B,n", [(300, 1024), (97, 200), (5, 1), (64, 3)])
def test_wave_kernel_identical_to_block_kernel(device, B, n):
    """Launches whose brackets are all <= 1024 configurations run the register-resident wave kernel; one
    longer bracket in the launch sends every bracket to the LDS block kernel.  Same (loss, position) order:
    the shared brackets' order, masks and counts identical, masks equal to the oracle; empty brackets, ties
    and non-finite losses included."""
    from hpbandster_amd import promote
    rs = np.random.RandomState(B + n)
    lens = rs.randint(0, n + 1, size=B)
    seg = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    loss = np.round(rs.rand(seg[-1]) * 50) / 50  # many ties
    loss[rs.rand(seg[-1]) < 0.05] = np.inf
    loss[rs.rand(seg[-1]) < 0.03] = np.nan
    loss[rs.rand(seg[-1]) < 0.01] = -np.inf
    k = np.maximum(lens * 0.34, 1.0)
    a1, o1, c1 = (t.cpu().numpy() for t in promote.promote_segments(loss, seg, k, device=device, return_order=True))
    long = rs.rand(1100)  # a bracket beyond the wave kernel's 1024
    loss2 = np.concatenate([loss, long])
    seg2 = np.concatenate([seg, [seg[-1] + long.size]]).astype(np.int64)
    a0, o0, c0 = (t.cpu().numpy() for t in promote.promote_segments(loss2, seg2, np.concatenate([k, [300.0]]),
                                                                      device=device, return_order=True))
    np.testing.assert_array_equal(a1[:seg[-1]], a0[:seg[-1]])
    np.testing.assert_array_equal(o1[:seg[-1]], o0[:seg[-1]])
    np.testing.assert_array_equal(c1[:B], c0[:B])
    for b in range(B):
        s, e = seg[b], seg[b + 1]
        np.testing.assert_array_equal(a1[s:e].astype(bool), O.sh_advance(loss[s:e], k[b]))


@pytest.mark.parametrize("B,n", [(200, 1024), (33, 100), (1, 1000), (3, 1500), (1, 10000), (4, 3000)])
def test_seg_argsort_is_numpy_stable_argsort(device, B, n):
    """hbx_seg_argsort (the refit's split, bohb.py:220): np.argsort order (-inf < finite < +inf < NaN),
    ties by position, through the wave kernel (segments <= 1024) or the counting-rank kernel
    (1024 < segments <= 65536), and the block kernel (a segment beyond 65536 in the same launch)."""
    import torch
    from hpbandster_amd import _native as N
    rs = np.random.RandomState(B * 3 + n)
    lens = rs.randint(0, n + 1, size=B)
    lens[0] = n
    seg = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    loss = np.round(rs.rand(seg[-1]) * 40) / 40
    loss[rs.rand(seg[-1]) < 0.04] = np.inf
    loss[rs.rand(seg[-1]) < 0.04] = np.nan
    loss[rs.rand(seg[-1]) < 0.02] = -np.inf
    loss[rs.rand(seg[-1]) < 0.03] = -0.0  # equal to 0.0 for numpy's sort: ties by position
    loss[rs.rand(seg[-1]) < 0.03] = 0.0
    L = N.lib()
    outs = []
    for extra in (0, 70000):  # 70000: one segment beyond the counting rank's limit -> the block kernel
        lv = np.concatenate([loss, rs.rand(extra)])
        sg = np.concatenate([seg, [seg[-1] + extra]]).astype(np.int64) if extra else seg
        ld = torch.from_numpy(lv).to(device)
        segd = torch.from_numpy(sg).to(device)
        nt = int(sg[-1])
        sb = int(L.hbx_sort_scratch_bytes(nt))
        scr = torch.empty(max(sb, 1), dtype=torch.uint8, device=device)
        order = torch.full((max(nt, 1),), -1, dtype=torch.int64, device=device)
        N.call("hbx_seg_argsort", N.ptr(ld), N.ptr(segd), len(sg) - 1, int(np.diff(sg).max()), nt, N.ptr(order),
               N.ptr(scr), sb, N.stream_handle())
        outs.append(order.cpu().numpy()[:seg[-1]])
    np.testing.assert_array_equal(outs[0], outs[1])
    for b in range(B):
        s, e = seg[b], seg[b + 1]
        np.testing.assert_array_equal(outs[0][s:e], np.argsort(loss[s:e], kind="stable"))


@pytest.mark.parametrize("crashed", [True, False])
@pytest.mark.parametrize("B,n", [(400, 1024), (97, 200), (5, 1), (64, 3), (2000, 81)])
def test_select_kernel_identical_to_sort(device, B, n, crashed):
    """Mask-only promotion (order not requested) runs the radix select of the k-th (loss, position);
    with the order requested the wave sort runs.  Masks and counts identical on tie-heavy brackets
    with empty, all-equal, all-crashed ones and k = 0, fractional, NaN and larger than the bracket.
    Without CRASHED (non-finite) entries every bracket takes the select kernel's all-finite path."""
    from hpbandster_amd import promote
    rs = np.random.RandomState(3 * B + n)
    lens = rs.randint(0, n + 1, size=B)
    lens[0] = n
    seg = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    loss = np.round(rs.rand(seg[-1]) * 30) / 30
    loss[rs.rand(seg[-1]) < 0.3] = 0.5
    if crashed:
        loss[rs.rand(seg[-1]) < 0.05] = np.inf
        loss[rs.rand(seg[-1]) < 0.03] = np.nan
        loss[rs.rand(seg[-1]) < 0.01] = -np.inf
    loss[rs.rand(seg[-1]) < 0.01] = -0.0
    loss[rs.rand(seg[-1]) < 0.01] = 0.0
    if B > 3:
        loss[seg[1]:seg[2]] = 0.25       # all equal
        loss[seg[2]:seg[3]] = np.nan if crashed else -0.0  # all crashed / all zero
    k = np.maximum(lens * rs.choice([0.0, 0.34, 0.5, 0.999, 1.7], size=B), 0.0)
    k[::7] = np.floor(k[::7])
    if B > 5:
        k[4] = np.nan
        k[5] = np.inf
    a_sel = promote.promote_segments(loss, seg, k, device=device)
    a_srt, _, c_srt = promote.promote_segments(loss, seg, k, device=device, return_order=True)
    np.testing.assert_array_equal(a_sel, a_srt.cpu().numpy().astype(bool))
    for b in range(B):
        s, e = seg[b], seg[b + 1]
        np.testing.assert_array_equal(a_sel[s:e], O.sh_advance(loss[s:e], k[b]))


def test_select_kernel_counts_and_extreme_keys(device):
    """Counts from the select kernel; keys differing only in the lowest bits and across signs."""
    import torch
    from hpbandster_amd import _native as N
    base = np.array([1.0, np.nextafter(1.0, 2), np.nextafter(np.nextafter(1.0, 2), 2), -1.0, -np.nextafter(1.0, 2),
                     5e-324, -5e-324, 0.0, -0.0, 1e308, -1e308])
    rs = np.random.RandomState(5)
    L = N.lib()
    for trial in range(20):
        loss = rs.permutation(np.concatenate([base, rs.choice(base, 40)]))
        n = loss.shape[0]
        for kk in range(0, n + 2):
            ld = torch.from_numpy(loss).to(device)
            seg = torch.tensor([0, n], dtype=torch.int64, device=device)
            kd = torch.tensor([float(kk)], dtype=torch.float64, device=device)
            adv = torch.empty(n, dtype=torch.uint8, device=device)
            cnt = torch.empty(1, dtype=torch.int64, device=device)
            N.check(L.hbx_sh_promote(N.ptr(ld), N.ptr(seg), 1, n, n, N.ptr(kd), None, N.ptr(adv), N.ptr(cnt), None, 0,
                                     N.stream_handle()))
            want = O.sh_advance(loss, kk, stable=True)  # hbx_sh_promote: ties by position
            np.testing.assert_array_equal(adv.cpu().numpy().astype(bool), want, err_msg="k=%d" % kk)
            assert int(cnt.item()) == int(want.sum())


@pytest.mark.parametrize("dist", ["lognormal", "exponents", "signed", "lowbits", "clustered", "uniform"])
def test_select_kernel_search_paths(device, dist):
    """The select kernel's three search stages on 1024-config brackets: interpolation hits (uniform),
    misses on skewed or clustered losses, bisection across exponents and signs, and brackets whose
    losses differ only in their lowest mantissa bits.  Masks equal argsort(argsort(losses)) < k."""
    from hpbandster_amd import promote
    rs = np.random.RandomState(len(dist))
    B, n = 96, 1024
    lens = rs.randint(n // 2, n + 1, size=B)
    lens[0] = n
    seg = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    N = int(seg[-1])
    if dist == "lognormal":
        loss = np.exp(rs.randn(N) * 4)
    elif dist == "exponents":
        loss = 10.0 ** rs.uniform(-300, 300, N)
    elif dist == "signed":
        loss = rs.randn(N) * 10.0 ** rs.randint(-5, 5, N)
    elif dist == "lowbits":
        loss = 0.75 + rs.randint(0, 4096, N) * np.spacing(0.75)
    elif dist == "clustered":
        loss = np.round(rs.rand(N) * 7) + rs.rand(N) * 1e-9
    else:
        loss = rs.rand(N)
    k = np.floor(lens * rs.uniform(0.01, 0.99, size=B))
    a_sel = promote.promote_segments(loss, seg, k, device=device)
    for b in range(B):
        s, e = seg[b], seg[b + 1]
        np.testing.assert_array_equal(a_sel[s:e], O.sh_advance(loss[s:e], k[b]), err_msg="bracket %d" % b)
