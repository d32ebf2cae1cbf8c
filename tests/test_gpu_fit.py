"""Batched KDE refit of many segments (hbx_kde_fit; config #5's per-bracket refit, bohb.py:220-246): the
lane-per-column kernel (64 add chains per wave, codes of up to 1000 levels through its window passes) and, at
D = 1, the per-column gather kernel, against numpy's own np.std(axis=0) / np.unique on the same split -- bit
for bit, ragged segments, segments longer than 1024 rows, empty and oversized sets, wide and invalid level
codes."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _case(D, dc, seed):
    rs = np.random.RandomState(seed)
    B = 16384 // (2 * D) + 9  # enough columns for the many-segment kernels
    lens = rs.randint(40, 900, size=B)
    lens[3] = 1024  # the LDS capacity exactly
    lens[5] = 1500  # beyond it: the gather path inside the kernel
    lens[7] = 2
    seg = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    N = int(seg[-1])
    X = rs.rand(N, D)
    levels = [4, 100, 1000]
    for d in range(dc, D):
        X[:, d] = rs.randint(0, levels[d % 3], size=N)
    orders = []
    for b in range(B):
        loss = np.round(rs.rand(lens[b]), 2)  # ties: the order is the host's, handed over as is
        orders.append(np.argsort(loss, kind="stable"))
    order = np.concatenate(orders).astype(np.int64)
    ng = np.array([max(D + 1, 15 * n // 100) for n in lens], dtype=np.int64)
    nb = np.array([max(D + 1, 85 * n // 100) for n in lens], dtype=np.int64)
    ng[7] = nb[7] = 0  # not refit
    nb[9] = lens[9] + 1  # more than the segment holds: not refit
    ng[11] = 0
    if D > dc:
        X[seg[13] + order[seg[13]], dc] = 2.5  # best row of segment 13: a code that is not an integer
    return B, lens, seg, X, order, ng, nb


def _run(device, D, dc, seed):
    import torch
    from hpbandster_amd import _native as N
    from hpbandster_amd import kde
    B, lens, seg, X, order, ng, nb = _case(D, dc, seed)
    vt = np.array([0] * dc + [1] * (D - dc), dtype=np.int32)
    fg = np.array([kde.bandwidth_factor(max(int(v), 1), D) for v in ng])
    fb = np.array([kde.bandwidth_factor(max(int(v), 1), D) for v in nb])
    ins = [torch.from_numpy(a).to(device) for a in (X, seg, order, ng, nb, fg, fb, vt)]
    outs = [torch.empty((B, D), dtype=torch.float64, device=device) for _ in range(2)] + \
           [torch.empty((B, D), dtype=torch.int32, device=device) for _ in range(2)]
    Xd, segd, od, ngd, nbd, fgd, fbd, vtd = ins
    N.call("hbx_kde_fit", N.ptr(Xd), D, N.ptr(segd), B, N.ptr(od), N.ptr(ngd), N.ptr(nbd), N.ptr(fgd),
           N.ptr(fbd), N.ptr(vtd), *[N.ptr(o) for o in outs], N.stream_handle())
    torch.cuda.synchronize()
    bwg, bwb, nlg, nlb = (o.cpu().numpy() for o in outs)
    for b in range(B):
        n = int(lens[b])
        Xb = X[seg[b]:seg[b + 1]]
        rows = order[seg[b]:seg[b + 1]]
        for ns, fac, bw, nl, rsel in ((ng[b], fg[b], bwg[b], nlg[b], rows[:max(int(ng[b]), 0)]),
                                      (nb[b], fb[b], bwb[b], nlb[b], rows[n - int(nb[b]):] if nb[b] > 0 else rows[:0])):
            if ns <= 0 or ns > n:
                assert np.isnan(bw).all(), b
                assert (nl == 0).all(), b
                continue
            data = Xb[rsel]
            np.testing.assert_array_equal(bw, 1.06 * np.std(data, axis=0) * fac, err_msg="segment %d" % b)
            for d in range(D):
                if d < dc:
                    assert nl[d] == 0
                    continue
                col = data[:, d]
                want = -1 if (col != np.floor(col)).any() else len(np.unique(col))
                assert nl[d] == want, (b, d, nl[d], want)


@pytest.mark.parametrize("D,dc", [(32, 24), (13, 9), (40, 40), (2, 1)])
def test_batched_fit_many_segments_bit_exact(device, D, dc):
    _run(device, D, dc, 100 + D)


@pytest.mark.parametrize("dc", [1, 0])
def test_batched_fit_gather_kernel_bit_exact(device, dc):
    """D = 1 (one continuous or one categorical dim): the per-column gather kernel."""
    _run(device, 1, dc, 7)
