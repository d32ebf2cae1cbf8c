"""Survivor count of a coarse scoring pre-screen at config #3 (CPU, fp64; tools only).

For every candidate: exact ln l, ln g (fp64 logsumexp over all observations) and the per-candidate
rigorous exponent error of a coarse pass that keeps one f16 product per continuous dim
(xh.Xh: the xh.Xl + xl.X' terms given up, <= 2^-10 |x''_d| max_j |X'_jd| per dim, log2 units) on top of
the FAST pass's own bound.  Survivors = candidates whose score interval reaches the smallest upper end
(they would go on to the precise pass).  Candidates: U[0,1) (bench) and BOHB's sampler rule.

    python tools/prescreen_survivors.py [--cand 1000000]
"""
import argparse
import math
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hpbandster_amd import synthetic as S  # noqa: E402

LOG2E = 1.4426950408889634


def kde_parts(data, dc, du):
    n, D = data.shape
    bw = 1.06 * np.std(data, axis=0) * n ** (-1. / (4 + D))
    nlev = [np.unique(data[:, d]).size for d in range(dc, D)]
    mu = data[:, :dc].mean(0)
    s = math.sqrt(LOG2E / 2) / bw[:dc]
    Xp = s * (data[:, :dc] - mu)
    xmax = np.abs(Xp).max(0)
    return dict(bw=bw, nlev=nlev, mu=mu, s=s, Xp=Xp, xmax=xmax, n=n, data=data)


def ln_pdf(K, C, dc, du):
    """exact fp64 ln pdf of every candidate row of C (log space, the reference's value up to rounding)."""
    xp = K["s"] * (C[:, :dc] - K["mu"])
    Xp = K["Xp"]
    t = -(np.sum(xp * xp, 1)[:, None] + np.sum(Xp * Xp, 1)[None, :] - 2 * xp @ Xp.T)  # log2 units
    for u in range(du):
        h = K["bw"][dc + u]
        c = K["nlev"][u]
        a, b = 1 - h, h / (c - 1)
        m = C[:, dc + u][:, None] == K["data"][:, dc + u][None, :]
        t += np.where(m, math.log2(abs(a)), math.log2(b))
    mx = t.max(1)
    lse2 = mx + np.log2(np.exp2(t - mx[:, None]).sum(1))
    norm = -math.log(K["n"]) - np.log(K["bw"][:dc]).sum() - 0.5 * dc * math.log(2 * math.pi)
    bnd = 2 * np.abs(xp) @ K["xmax"]  # sum_d |x''_d| max|X'_d|
    return lse2 * math.log(2) + norm, bnd


def bohb_candidates(Kg, n, dc, du, levels, rs):
    from scipy.stats import truncnorm
    data, bw = Kg["data"], Kg["bw"]
    idx = rs.randint(0, data.shape[0], size=n)
    C = np.empty((n, dc + du))
    for d in range(dc):
        m = data[idx, d]
        a, b = (0 - m) / bw[d], (1 - m) / bw[d]
        C[:, d] = truncnorm.rvs(a, b, loc=m, scale=3 * bw[d], random_state=rs)
    for u in range(du):
        d = dc + u
        keep = rs.rand(n) < (1 - bw[d])
        C[:, d] = np.where(keep, data[idx, d], rs.randint(0, levels, size=n))
    return C


def survivors(lnl, lng, wl, wg):
    lc = math.log(1e-8)
    sc = np.maximum(lng, lc) - np.maximum(lnl, lc)
    w = wl + wg
    hi_min = np.min(sc + w)
    order = np.sort(sc)
    return int(np.sum(sc - w <= hi_min)), order[:5] - order[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cand", type=int, default=1_000_000)
    ap.add_argument("--chunk", type=int, default=2000)
    a = ap.parse_args()
    torch.set_num_threads(os.cpu_count())
    dc, du, L, nobs = 24, 8, 4, 10_000
    X = S.make_observations(nobs, dc, du, L)
    losses = S.make_losses(nobs)
    ng, nb = S.bohb_split_sizes(nobs, dc + du + 1)
    idx = np.argsort(losses)
    Kg, Kb = kde_parts(X[idx[:ng]], dc, du), kde_parts(X[idx[-nb:]], dc, du)
    sets = {"uniform": S.make_candidates(a.cand, dc, du, L),
            "bohb_sampler": bohb_candidates(Kg, a.cand, dc, du, L, np.random.RandomState(9))}
    fast_bound = 0.0089 + 0.002  # FAST pass: one-hot lo parts + rounding (log2 units), bench shape
    for name, C in sets.items():
        lnl = np.empty(a.cand)
        lng = np.empty(a.cand)
        bl = np.empty(a.cand)
        bg = np.empty(a.cand)
        for i0 in range(0, a.cand, a.chunk):
            c = C[i0:i0 + a.chunk]
            lnl[i0:i0 + len(c)], bl[i0:i0 + len(c)] = ln_pdf(Kg, c, dc, du)
            lng[i0:i0 + len(c)], bg[i0:i0 + len(c)] = ln_pdf(Kb, c, dc, du)
        ln2 = math.log(2)
        for label, cw in (("fast", 0.0), ("coarse", 2.0 ** -10)):
            wl = (fast_bound + cw * bl) * ln2
            wg = (fast_bound + cw * bg) * ln2
            n_s, gaps = survivors(lnl, lng, wl, wg)
            print("%-13s %-7s survivors %7d  mean half-width %.4f ln  (bnd mean l %.1f g %.1f)  top gaps %s"
                  % (name, label, n_s, np.mean(wl + wg), bl.mean(), bg.mean(), np.round(gaps, 4)), flush=True)


if __name__ == "__main__":
    main()
