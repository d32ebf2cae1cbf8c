"""Load the golden fixtures written by tests/golden/gen_golden.py.

Large cases store only seeds + sha256 of their inputs; the inputs are regenerated with
hpbandster_amd.synthetic (legacy RandomState streams, identical across numpy versions) and
checked against the recorded hashes before use.
"""
import glob
import json
import os

import numpy as np

from hpbandster_amd import synthetic as S

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

_REGEN = {
    "d8c": lambda: (S.make_observations(1000, 8, 0, 2), S.make_losses(1000), S.make_candidates(1000, 8, 0, 2)),
    "d32m": lambda: (S.make_observations(10000, 24, 8, 4), S.make_losses(10000),
                     S.make_candidates(256, 24, 8, 4)),
    "tie_q1m": lambda: (S.make_observations(3000, 6, 2, [3, 4], seed=87), tie_losses(3000, 1, 0.1, 88)[0],
                        S.make_candidates(400, 6, 2, [3, 4], seed=89)),
    "tie_d32": lambda: (S.make_observations(2000, 24, 8, 4, seed=90), tie_losses(2000, 3, 0.05, 91)[0],
                        S.make_candidates(256, 24, 8, 4, seed=92)),
}


def tie_losses(n, decimals, crash_frac, seed):
    """Quantised losses and crash flags of the tie fixtures (tests/golden/gen_golden.py:tie_losses)."""
    rs = np.random.RandomState(seed)
    L = np.round(rs.rand(n), decimals)
    crashed = rs.rand(n) < crash_frac
    return L, crashed


def kde_case_names():
    return sorted(os.path.basename(p)[4:-4] for p in glob.glob(os.path.join(GOLDEN, "kde_*.npz")))


def load_kde_case(name):
    z = np.load(os.path.join(GOLDEN, "kde_%s.npz" % name))
    c = {k: z[k] for k in z.files}
    if "X" not in c:
        X, L, C = _REGEN[name]()
        assert S.sha256_array(X) == str(c["sha_X"]), name
        assert S.sha256_array(L) == str(c["sha_losses"]), name
        assert S.sha256_array(C) == str(c["sha_cands"]), name
        c.update(X=X, losses=L, cands=C)
    c["var_type"] = str(c["var_type"])
    c["chosen"] = int(c["chosen"])
    if "crashed" in c:
        c["eff_losses"] = np.where(c["crashed"], np.inf, c["losses"])
    else:
        c["eff_losses"] = c["losses"]
    c["name"] = name
    return c


def load_getcfg(name):
    z = np.load(os.path.join(GOLDEN, "getcfg_%s.npz" % name))
    recs = []
    for i in range(int(z["n_records"])):
        recs.append({k: z["r%02d_%s" % (i, k)] for k in ("seed", "model_based", "cands", "chosen", "vec")})
    return dict(dc=int(z["dc"]), du=int(z["du"]), levels=z["levels"], n_obs=int(z["n_obs"]), records=recs)


def getcfg_names():
    return sorted(os.path.basename(p)[7:-4] for p in glob.glob(os.path.join(GOLDEN, "getcfg_*.npz")))


def load_sh(which="sh_promotion"):
    z = np.load(os.path.join(GOLDEN, which + ".npz"))
    cases = []
    for i in range(int(z["n_cases"])):
        cases.append(dict(losses=z["b%02d_losses" % i], crashed=z["b%02d_crashed" % i], k=int(z["b%02d_k" % i]),
                          sh_adv=z["sh%02d_adv" % i], sr_adv=z["sr%02d_adv" % i],
                          sh_count=int(z["sh%02d_count" % i]), sr_count=int(z["sr%02d_count" % i])))
    return cases


def load_brackets():
    with open(os.path.join(GOLDEN, "hb_brackets.json")) as fh:
        return json.load(fh)


def load_e2e():
    z = np.load(os.path.join(GOLDEN, "e2e_toy.npz"))
    recs = []
    for i in range(int(z["n_records"])):
        recs.append({k: z["r%03d_%s" % (i, k)] for k in ("budget", "x", "model_based", "cands")})
    with open(os.path.join(GOLDEN, "e2e_toy_runs.json")) as fh:
        runs = json.load(fh)
    return recs, runs
