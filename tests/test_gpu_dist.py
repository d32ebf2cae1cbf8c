"""GPU: the candidate-sharded acquisition (the reference loop bohb.py:133-152 split over
GPUs) -- the RCCL winner exchange at world size 1, the device reduction of gathered records, a
two-process run sharing the box's GPU (gloo transport), and BASELINE config #4's shape (1e7 candidates
x 1e4 observations x D = 32) sharded 8 ways through index_base on one MI355X."""
import os
import socket
import struct

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _pair_and_cands(device, dc=24, du=8, lev=4, n_obs=3000, n_cand=50000):
    from hpbandster_amd import kde
    from hpbandster_amd import synthetic as S
    X = S.make_observations(n_obs, dc, du, lev)
    L = S.make_losses(n_obs)
    pair = kde.fit_pair(X, L, S.var_type_string(dc, du), dc + du + 1, device=device)
    return pair, S.make_candidates(n_cand, dc, du, lev)


def test_rccl_exchange_world1_matches_acquire(device):
    """hbx_argmax_allreduce over libhbx's own RCCL communicator (one rank): the exchanged winner is the
    local acquisition's record."""
    from hpbandster_amd.distributed import WinnerExchange, acquire_sharded
    pair, C = _pair_and_cands(device)
    want = pair.acquire(C)
    x = WinnerExchange(device, transport="rccl")
    try:
        idx, score, g = acquire_sharded(pair, C, 0, x)
        assert (idx, score) == (want.index, want.score)
        assert g.shortlist == want.shortlist
        # a second exchange over the same communicator, shifted index base
        idx2, _, _ = acquire_sharded(pair, C[:1000], 5000, x)
        assert idx2 == 5000 + pair.acquire(C[:1000]).index
    finally:
        x.close()


def test_torch_transport_world1_matches_acquire(device):
    """The fallback exchange (device records all-gathered on torch's process group, then the device reduction)
    at one rank: the exchanged winner is the local acquisition's record."""
    from hpbandster_amd.distributed import WinnerExchange, acquire_sharded
    pair, C = _pair_and_cands(device)
    want = pair.acquire(C)
    x = WinnerExchange(device, transport="torch")
    idx, score, g = acquire_sharded(pair, C, 0, x)
    assert (idx, score) == (want.index, want.score)
    assert g.shortlist == want.shortlist


def _rec(index, score, rel=1e-13, flags=0):
    from hpbandster_amd.kde import RESULT_FMT
    return struct.pack(RESULT_FMT, index, score, rel, flags, 3, 1, 0.5, 0.25)


@pytest.mark.parametrize("case", ["distinct", "tie", "none", "near", "nan"])
def test_device_reduction_of_records(device, case):
    """hbx_argmax_records (the reduction hbx_argmax_allreduce runs after its all-gather) against the
    host restatement: smallest score, ties to the smallest global index, invalid records skipped, near
    winners flagged."""
    import torch
    from hpbandster_amd import _native as N
    from hpbandster_amd.distributed import reduce_records_host
    from hpbandster_amd.kde import AcqResult, ACQ_NEAR_TIE
    recs = {"distinct": [(5, 2.0), (900, 1.5), (40, 3.0)],
            "tie": [(700, 1.5), (12, 1.5), (40, 3.0)],
            "none": [(-1, np.nan), (-1, np.nan)],
            "near": [(700, 1.5 * (1 + 1e-14)), (12, 1.5), (40, 1.5 * (1 + 1e-6))],
            "nan": [(3, np.nan), (9, np.inf), (11, 4.0)]}[case]
    raw = b"".join(_rec(i, s) for i, s in recs)
    d = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(device)
    out = torch.empty(48, dtype=torch.uint8, device=device)
    N.check(N.lib().hbx_argmax_records(N.ptr(d), len(recs), N.ptr(out), N.stream_handle(None, device)))
    g = AcqResult.from_bytes(out.cpu().numpy().tobytes())
    hs = [AcqResult.from_bytes(_rec(i, s)) for i, s in recs]
    best, near = reduce_records_host(hs)
    if best < 0:
        assert g.index == -1
        return
    assert g.index == hs[best].index and g.score == hs[best].score
    assert bool(g.flags & ACQ_NEAR_TIE) == (len(near) > 1) == (case in ("near", "tie"))
    assert g.shortlist == 3 * len(recs)


def _two_rank_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from hpbandster_amd.distributed import WinnerExchange, acquire_sharded, shard_range
        device = torch.device("cuda", 0)
        torch.cuda.set_device(device)
        pair, C = _pair_and_cands(device, n_cand=40000)
        out = []
        for lo_n in (40000, 777, 3):  # shards of different lengths (one rank may hold 1 candidate)
            lo, hi = shard_range(lo_n, rank, world)
            x = WinnerExchange(device, transport="records")
            idx, score, _ = acquire_sharded(pair, C[lo:hi], lo, x)
            out.append((idx, score))
        q.put((rank, out, None))
    except Exception as e:  # report to the parent instead of hanging it
        import traceback
        q.put((rank, None, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def test_two_ranks_share_the_gpu_gloo_records():
    """Two processes (one per 'GPU', both on the box's one MI355X), each scoring its shard with global
    indices; the gloo records transport + device reduction give the unsharded acquisition's winner."""
    import multiprocessing as mp
    import torch
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_two_rank_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = dict()
    for _ in range(2):
        rank, out, err = q.get(timeout=180)
        assert err is None, err
        got[rank] = out
    for p in ps:
        p.join(60)
    device = torch.device("cuda", 0)
    pair, C = _pair_and_cands(device, n_cand=40000)
    for k, n in enumerate((40000, 777, 3)):
        want = pair.acquire(C[:n])
        assert got[0][k] == got[1][k] == (want.index, want.score), (n, got, want)


def test_config4_shape_sharded_8_ways(device):
    """BASELINE config #4 on one MI355X: 1e7 candidates x 1e4 observations (1500 good / 8500 bad),
    D = 32 (24c + 8u, 4 levels) -- the set whose winner the C oracle pinned by scoring every candidate
    (tests/golden/full_winners.json, prefix_10000000).  The acquisition that also reports ln-pdfs (the
    precise scoring instance) and the 8 per-rank shards (index_base = shard start) reduced by the
    exchange's rule both return the pinned winner, score and pdfs bit for bit."""
    import json
    import torch
    from hpbandster_amd import kde
    from hpbandster_amd import synthetic as S
    from hpbandster_amd.distributed import reduce_records_host, shard_range
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "full_winners.json")) as fh:
        e = json.load(fh)["config3_prefixes"]["prefix_10000000"]
    dc, du, lev = 24, 8, 4
    X = S.make_observations(10000, dc, du, lev)
    L = S.make_losses(10000)
    vt = S.var_type_string(dc, du)
    pair = kde.fit_pair(X, L, vt, dc + du + 1, device=device)
    assert (pair.good.nobs, pair.bad.nobs) == (1500, 8500)
    Nc = 10_000_000
    C = torch.from_numpy(S.make_candidates_blocked(0, Nc, dc, du, lev)).to(device)
    ws = torch.empty(pair.workspace_bytes(Nc), dtype=torch.uint8, device=device)
    res, logl, logg = pair.acquire(C, workspace=ws, logs=True)
    recs = []
    for k in range(8):
        lo, hi = shard_range(Nc, k, 8)
        recs.append(pair.acquire(C[lo:hi], index_base=lo, workspace=ws))
    best, _ = reduce_records_host(recs)
    for r in (res, recs[best]):
        assert r.index == e["winner"] and float(r.score).hex() == e["score_hex"]
        assert float(r.pdf_l).hex() == e["pdf_l_hex"] and float(r.pdf_g).hex() == e["pdf_g_hex"]
    # the reported ln-pdf estimates of the winner agree with its exact pdfs
    np.testing.assert_allclose([logl[e["winner"]], logg[e["winner"]]], np.log([res.pdf_l, res.pdf_g]), rtol=1e-4)
