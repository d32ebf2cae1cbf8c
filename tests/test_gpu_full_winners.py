"""GPU: the benchmarked configurations' winners at FULL size against the C oracle's scan of every
candidate (tests/golden/full_winners.json, written by tests/golden/gen_full_winners.py from the
reference's own fitted models: bohb.py:133-152's loop over all 1e5 / 1e6 / ... / 1e7 candidates).

Per workload: the inputs' checksums and the model's bandwidths equal the pinned ones, and
hbx_kde_acquire returns the pinned index, score, pdf_l and pdf_g bit for bit -- config #2 (1e5 x 1e3 x
8c), config #3 (1e6 x 1e4 x 24c+8u), the weak-scaling sets of 2 / 4 / 8 ranks (their first N x 1e6 rows,
sharded as the ranks shard them) and config #4 (1e7, whole and in 8 shards)."""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(HERE, "golden", "full_winners.json")) as _fh:
    PINNED = json.load(_fh)


def _check(rec, entry):
    assert rec.index == entry["winner"], (rec.index, entry["winner"])
    assert float(rec.score).hex() == entry["score_hex"]
    assert float(rec.pdf_l).hex() == entry["pdf_l_hex"] and float(rec.pdf_g).hex() == entry["pdf_g_hex"]


def _model_check(pair, entry, X, L):
    from hpbandster_amd import synthetic as S
    assert S.sha256_array(X) == entry["sha_X"] and S.sha256_array(L) == entry["sha_losses"]
    assert (pair.good.nobs, pair.bad.nobs) == (entry["n_good"], entry["n_bad"])
    assert [float(v).hex() for v in pair.good.bw] == entry["bw_good_hex"]
    assert [float(v).hex() for v in pair.bad.bw] == entry["bw_bad_hex"]


def test_config2_full_winner(device):
    import torch
    from hpbandster_amd import kde
    from hpbandster_amd import synthetic as S
    e = PINNED["config2"]
    X, L = S.make_observations(1000, 8, 0, 0), S.make_losses(1000)
    C = S.make_candidates(100_000, 8, 0, 0)
    assert S.sha256_array(C) == e["sha_cands"]
    pair = kde.fit_pair(X, L, S.var_type_string(8, 0), 9, device=device)
    _model_check(pair, e, X, L)
    _check(pair.acquire(torch.from_numpy(C).to(device)), e)


@pytest.fixture(scope="module")
def config3(device):
    from hpbandster_amd import kde
    from hpbandster_amd import synthetic as S
    X, L = S.make_observations(10_000, 24, 8, 4), S.make_losses(10_000)
    pair = kde.fit_pair(X, L, S.var_type_string(24, 8), 33, device=device)
    _model_check(pair, PINNED["config3_model"], X, L)
    return pair


@pytest.mark.parametrize("n", [1_000_000, 2_000_000, 4_000_000, 8_000_000, 10_000_000])
def test_config3_and_config4_full_winners(device, config3, n):
    """The headline set (1e6), the weak-scaling sets at 2 / 4 / 8 ranks (rank r scores rows [r 1e6, (r+1)
    1e6), global indices) and config #4's 1e7 (whole, and in 8 shards as the 8-GPU run shards it)."""
    import torch
    from hpbandster_amd import synthetic as S
    from hpbandster_amd.distributed import reduce_records_host, shard_range
    e = PINNED["config3_prefixes"]["prefix_%d" % n]
    C = S.make_candidates_blocked(0, n, 24, 8, 4)
    assert S.sha256_array(C) == e["sha_cands"]
    C = torch.from_numpy(C).to(device)
    ws = torch.empty(config3.workspace_bytes(n), dtype=torch.uint8, device=device)
    if n in (1_000_000, 10_000_000):
        _check(config3.acquire(C, workspace=ws), e)
    shards = {1_000_000: 1, 2_000_000: 2, 4_000_000: 4, 8_000_000: 8, 10_000_000: 8}[n]
    if shards > 1:
        recs = []
        for k in range(shards):
            lo, hi = shard_range(n, k, shards) if n == 10_000_000 else (k * 1_000_000, (k + 1) * 1_000_000)
            recs.append(config3.acquire(C[lo:hi], index_base=lo, workspace=ws))
        best, _ = reduce_records_host(recs)
        _check(recs[best], e)
