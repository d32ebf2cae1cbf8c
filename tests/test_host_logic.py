"""CPU tests of the engine's host-side logic (no GPU): Hyperband math, the SuccessiveHalving state
machine, the BOHB candidate sampler's RNG parity, the ConfigSpace stand-in, result logging, and the
multi-rank winner exchange over gloo.  The promotion kernel is replaced by the oracle ONLY here."""
import json
import os

import numpy as np
import pytest

from hpbandster_amd import HB_master as M
from hpbandster_amd import configspace as CS
from oracle import kde_oracle as O
from tests import golden_cases as G


def test_hb_budgets_and_brackets_match_reference():
    for t in G.load_brackets():
        m, budgets = M.hb_budgets(t["eta"], t["min_budget"], t["max_budget"])
        assert m == t["max_SH_iter"]
        np.testing.assert_allclose(budgets, t["budgets"], rtol=5e-16, atol=0)
        for it in t["iterations"]:
            s, ns = M.hb_bracket(it["it"], t["eta"], m)
            assert ns == it["num_configs"]


def test_hb_budgets_random_bit_identical_to_oracle():
    """Budgets are dict keys in the reference (float equality matters, HB_master.py:93-94): 4000 random
    (eta, min_budget, max_budget) give the oracle's restatement of the reference expressions bit for bit,
    and every bracket's num_configs (HB_master.py:161-168)."""
    rs = np.random.RandomState(0)
    done = 0
    while done < 4000:
        eta = float(rs.choice([2, 3, 4, 2.5, 1.5, 5, 10]))
        mx = float(rs.choice([1, 9, 27, 81, 100, 243, 1000, 3.7, 64])) * 10.0 ** rs.randint(-3, 3)
        mn = mx / eta ** rs.randint(0, 8) * float(rs.choice([1, 1, 0.9, 1.1, 0.5]))
        if not 0 < mn <= mx:
            continue
        done += 1
        m, budgets = M.hb_budgets(eta, mn, mx)
        mo, bo = O.hb_budgets(eta, mn, mx)
        assert m == mo
        assert np.array_equal(budgets, bo) and budgets.tobytes() == bo.tobytes(), (eta, mn, mx)
        for it in range(2 * m):
            assert M.hb_bracket(it, eta, m) == O.hb_bracket(it, eta, m)


class _Job(object):
    def __init__(self, cid, cfg, b, loss):
        self.id, self.kwargs, self.timestamps = cid, {"config": cfg, "budget": b}, {}
        self.result = None if loss is None else {"loss": loss, "info": None}
        self.exception = None if loss is not None else "crash"


@pytest.mark.parametrize("cls_name", ["SuccessiveHalving", "SuccessiveResampling"])
def test_successive_halving_state_machine(monkeypatch, cls_name):
    from hpbandster_amd import HB_iteration as H
    monkeypatch.setattr(H.promote, "advance_mask", lambda losses, k, device=None: O.sh_advance(losses, k))
    cls = getattr(H, cls_name)
    for c in G.load_sh():
        n = len(c["losses"])
        cnt = [0]

        def sampler(b):
            cnt[0] += 1
            return {"i": cnt[0]}, {}
        sh = cls(iter_number=0, num_configs=[n, c["k"], 1], budgets=[1.0, 3.0, 9.0], config_sampler=sampler)
        jobs = [sh.get_next_run() for _ in range(n)]
        for (cid, cfg, b), l, cr in zip(jobs, c["losses"], c["crashed"]):
            sh.register_result(_Job(cid, cfg, b, None if cr else float(l)))
        sh.get_next_run()
        adv = np.array([sh.data[cid]["status"] in ("QUEUED", "RUNNING") for cid, _, _ in jobs])
        np.testing.assert_array_equal(adv, c["sh_adv"] if cls_name == "SuccessiveHalving" else c["sr_adv"])


@pytest.mark.parametrize("name", G.getcfg_names())
def test_bohb_candidate_sampler_rng_parity(name):
    """The host sampler consumes the global RNG exactly like bohb.py:109-147."""
    from types import SimpleNamespace
    from hpbandster_amd import synthetic as S
    from hpbandster_amd.config_generators.bohb import BOHB
    g = G.load_getcfg(name)
    dc, du, lv, n = g["dc"], g["du"], g["levels"], g["n_obs"]
    lvs = [int(v) for v in lv] if len(lv) > 1 else [int(lv[0])] * du
    space = CS.ConfigurationSpace(seed=11)
    for d in range(dc):
        space.add_hyperparameter(CS.UniformFloatHyperparameter("x%02d" % d, 0.0, 1.0))
    for d in range(du):
        space.add_hyperparameter(CS.CategoricalHyperparameter("y%02d" % d, list(range(lvs[d]))))
    cg = BOHB(space)
    X = S.make_observations(n, dc, du, lv if len(lv) > 1 else int(lv[0]))
    L = S.make_losses(n)
    good, bad = O.bohb_split(X, L, dc + du + 1)
    kde_good = SimpleNamespace(data=X[good], bw=O.normal_reference_bw(X[good]))
    for r in g["records"]:
        np.random.seed(int(r["seed"]))
        model_based = not (np.random.rand() < cg.random_fraction)
        assert model_based == bool(r["model_based"])
        if model_based:
            cands = cg.sample_candidates(kde_good, cg.num_samples)
            # scipy's truncnorm differs by <= a few ulp between 1.7 (fixture) and this interpreter
            np.testing.assert_allclose(cands, r["cands"], rtol=1e-12, atol=1e-12)


def test_configspace_roundtrip():
    cs = CS.ConfigurationSpace(seed=1)
    cs.add_hyperparameter(CS.UniformFloatHyperparameter("lr", 1e-4, 1e-1, log=True))
    cs.add_hyperparameter(CS.CategoricalHyperparameter("act", ["relu", "tanh", "elu"]))
    cs.add_hyperparameter(CS.UniformIntegerHyperparameter("units", 16, 256))
    assert [h.name for h in cs.get_hyperparameters()] == ["act", "lr", "units"]
    c = cs.sample_configuration()
    d = c.get_dictionary()
    v = CS.Configuration(cs, values=d).get_array()
    d2 = CS.Configuration(cs, vector=v).get_dictionary()
    assert d2["act"] == d["act"] and d2["units"] == d["units"]
    assert abs(d2["lr"] - d["lr"]) <= 1e-12 * d["lr"]
    assert hasattr(cs.get_hyperparameters()[0], "choices") and not hasattr(cs.get_hyperparameters()[1], "choices")


def test_json_result_logger_format(tmp_path):
    from hpbandster_amd.utils import json_result_logger, logged_results_to_HB_result
    lg = json_result_logger(str(tmp_path))
    j = _Job((0, 0, 0), {"x": 0.5}, 1.0, 0.25)
    j.timestamps = {"submitted": 10.0, "started": 10.5, "finished": 11.0}
    lg(j)
    j2 = _Job((0, 0, 0), {"x": 0.5}, 3.0, 0.2)
    j2.timestamps = {"submitted": 12.0, "started": 12.5, "finished": 13.0}
    lg(j2)
    lines = open(os.path.join(tmp_path, "configs.json")).read().splitlines()
    assert json.loads(lines[0]) == [[0, 0, 0], {"x": 0.5}] and len(lines) == 1
    res = [json.loads(l) for l in open(os.path.join(tmp_path, "results.json"))]
    assert res[1][1] == 3.0 and res[1][3]["loss"] == 0.2
    hb = logged_results_to_HB_result(str(tmp_path))
    assert hb.get_incumbent_id() == (0, 0, 0)
    with pytest.raises(FileExistsError):
        json_result_logger(str(tmp_path))


def test_shard_ranges_cover_everything():
    from hpbandster_amd.distributed import shard_range
    for n, w in ((10, 3), (1000000, 8), (7, 8), (0, 2)):
        got = [shard_range(n, r, w) for r in range(w)]
        assert got[0][0] == 0 and got[-1][1] == n
        assert all(a[1] == b[0] for a, b in zip(got, got[1:]))


def _gloo_worker(rank, world, port, shards, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from hpbandster_amd.distributed import reduce_winners
    score, idx = shards[rank]
    q.put((rank, reduce_winners(score, idx)))
    dist.destroy_process_group()


@pytest.mark.parametrize("case", ["distinct", "tie", "none_left", "all_none"])
def test_winner_exchange_gloo_world2(case):
    """World-size-2 exchange of local winners (the N>1 path of bench.py / acquire_sharded)."""
    import multiprocessing as mp
    import socket
    c = G.load_kde_case("mixed8")
    X, C = c["X"], c["cands"]
    l = O.pdf_many(X[c["good_idx"]], c["bw_good"], c["var_type"], C)
    g = O.pdf_many(X[c["bad_idx"]], c["bw_bad"], c["var_type"], C)
    scores = np.array([O.py_score(a, b) for a, b in zip(l, g)])
    if case == "tie":  # duplicate the global winner into the second shard
        scores[400] = scores[c["chosen"]]
    if case == "none_left":
        scores[:250] = np.nan
    if case == "all_none":
        scores[:] = np.nan
    want = O.py_argmin(scores)
    shards = []
    for lo, hi in ((0, 250), (250, 500)):
        i = O.py_argmin(scores[lo:hi])
        shards.append((float(scores[lo + i]) if i >= 0 else np.nan, lo + i if i >= 0 else -1))
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_gloo_worker, args=(r, 2, port, shards, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = dict(q.get(timeout=120) for _ in range(2))
    for p in ps:
        p.join(60)
    assert out[0][0] == out[1][0] == want


def _subgroup_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from hpbandster_amd.distributed import broadcast_from_group_root
    grp = dist.new_group([1, 2])  # every rank creates it; only 1 and 2 belong
    if rank in (1, 2):
        got = broadcast_from_group_root(b"uid-of-rank-%d" % rank, grp, 2)
        q.put((rank, got))
    dist.barrier()
    dist.destroy_process_group()


def test_rccl_uid_broadcast_in_a_subgroup_without_global_rank0():
    """WinnerExchange's RCCL unique id travels from the GROUP's rank 0 (global rank 1 here): world size
    3, subgroup {1, 2} (broadcast_object_list takes a global source rank)."""
    import multiprocessing as mp
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_subgroup_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in ps:
        p.start()
    out = dict(q.get(timeout=120) for _ in range(2))
    for p in ps:
        p.join(60)
    assert out == {1: b"uid-of-rank-1", 2: b"uid-of-rank-1"}


def test_promotion_size_policy_host_rank():
    """advance_mask's host ranking (tie-free brackets up to HOST_MAX): the reference's argsort(argsort) < k
    mask (HB_iteration.py:180) wherever the k-th and (k+1)-th smallest losses differ; None -- the GPU's
    numpy-order path -- where tied losses straddle the k-th place or a loss is not finite."""
    from hpbandster_amd import promote as P
    rs = np.random.RandomState(9)
    for n in (1, 2, 5, 81, 256, 257, 1000, 4096):
        x = rs.rand(n)
        for k in (0, 1, n // 3, n // 2 + 0.5, n - 1, n, n + 3, float("nan"), -1.0):
            m = P._host_rank(x, P._threshold(k, n), n)
            assert m is not None
            want = (np.argsort(np.argsort(x)) < k) if k == k and k > 0 else np.zeros(n, bool)
            np.testing.assert_array_equal(m, want, err_msg="n=%d k=%r" % (n, k))
    tie = np.array([1.0] * 40 + [0.5] * 10)
    assert P._host_rank(tie, 15, 50) is None            # straddling tie: numpy 1.26.4's order decides
    assert P._host_rank(tie, 10, 50) is not None        # the tie is wholly above the k-th place
    assert P._host_rank(np.array([-0.0, 0.0, 1.0]), 1, 3) is None  # -0.0 == 0.0 ties
    for bad in (np.inf, -np.inf, np.nan):
        y = rs.rand(300)
        y[17] = bad
        assert P._host_rank(y, 100, 300) is None
        assert P._host_rank(y[:100], 30, 100) is None
    assert P._threshold(4.5, 10) == 5 and P._threshold(3, 10) == 3 and P._threshold(20, 10) == 10
