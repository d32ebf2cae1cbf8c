#!/usr/bin/env python
"""bench.py -- BOHB KDE acquisition throughput on MI355X (BASELINE.json metric).

One "step" = one acquisition over one batch of synthetic candidates resident in HBM:
score every candidate against the good (l) and bad (g) KDE of config #3's observation set
(1e4 observations, D = 32: 24 continuous + 8 categorical with 4 levels; BOHB split 1500 / 8500),
then select the first index of min max(1e-8, g)/max(l, 1e-8) exactly, and bring the winner to the
host.  Per GPU: 1e6 candidates (config #3).  With N GPUs every rank scores its own 1e6-candidate
shard (global indices rank*1e6 + i) and the local winners meet in one RCCL all_gather
(weak scaling; config #4's 1e7 candidates at N=8 is `--candidates 1250000`).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

Rank 0 prints ONE JSON line.  value = all ranks' (candidate, observation) pairs / max-over-ranks
time.  roofline: the scoring kernel (kde_logpdf, two launches per step), timed with HIP events on
its own stream inside the timed region; algorithmic work W = 3*Dc + 2*Du + 4 = 92 flops per pair
 against the 157.3 TFLOP/s fp32 vector peak.  cpu_baseline: the C oracle
(oracle/kde_oracle.c, fp64, OpenMP) on the host cores, on a bounded candidate sample.
"""

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "candidate KDE evals/sec (cand×obs pairs) at D=32, 1/2/4/8 MI355X; % VALU peak"
PEAK_FP32_TFLOPS = 157.3  # MI355X_MICROARCH.md: peak FP32 vector (= f32 MFMA) rate


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--candidates", type=int, default=1_000_000, help="candidates per GPU")
    ap.add_argument("--obs", type=int, default=10_000)
    ap.add_argument("--dc", type=int, default=24)
    ap.add_argument("--du", type=int, default=8)
    ap.add_argument("--levels", type=int, default=4)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample time")
    ap.add_argument("--no-cpu", action="store_true")
    return ap.parse_args()


def cpu_baseline(X, good_rows, bad_rows, pair, var_type, cands, target_s):
    """C oracle (fp64, OpenMP over candidates) on the host cores, bounded sample."""
    from oracle import c_oracle
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
    Xg, Xb = X[good_rows], X[bad_rows]
    args_g = (Xg, pair.good.bw, var_type, pair.good.nlev)
    args_b = (Xb, pair.bad.bw, var_type, pair.bad.nlev)
    n = max(threads, 16)
    t_used = 0.0
    while True:
        t0 = time.perf_counter()
        c_oracle.kde_pdf(*args_g, cands[:n], nthreads=threads)
        c_oracle.kde_pdf(*args_b, cands[:n], nthreads=threads)
        dt = time.perf_counter() - t0
        if dt >= target_s * 0.5 or n >= cands.shape[0]:
            break
        t_used += dt
        n = int(min(cands.shape[0], max(2 * n, n * (target_s / max(dt, 1e-3)))))
    pairs = n * (Xg.shape[0] + Xb.shape[0])
    return {"value": pairs / dt, "unit": "pairs/s", "cores": threads, "kind": "port",
            "sample": "%d of the %d candidates x %d observations (D=%d), fp64 C oracle, %.1f s"
                      % (n, cands.shape[0], Xg.shape[0] + Xb.shape[0], X.shape[1], dt)}


def load_traffic(workload):
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(p) as fh:
            d = json.load(fh)
        if d.get("workload") == workload:
            return d.get("bytes_per_launch")
    except (OSError, ValueError):
        pass
    return None


def main():
    a = parse()
    import torch
    import torch.distributed as dist
    from hpbandster_amd import kde
    from hpbandster_amd import synthetic as S

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        log("note: --gpus %d but WORLD_SIZE %d; using WORLD_SIZE" % (a.gpus, world))
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=device)

    D = a.dc + a.du
    var_type = S.var_type_string(a.dc, a.du)
    X = S.make_observations(a.obs, a.dc, a.du, a.levels)
    losses = S.make_losses(a.obs)
    pair = kde.fit_pair(X, losses, var_type, D + 1, device=device)
    Ng, Nb = pair.good.nobs, pair.bad.nobs
    Nc = a.candidates
    cands = S.make_candidates(Nc, a.dc, a.du, a.levels, seed=S.SEED_CAND + rank)
    c_dev = torch.from_numpy(cands).to(device)
    base = rank * Nc
    ws = torch.empty(pair.workspace_bytes(Nc), dtype=torch.uint8, device=device)
    ev = kde.ScoreEvents()
    log("rank %d/%d: %d candidates x (%d + %d) observations, D=%d" % (rank, world, Nc, Ng, Nb, D))

    def step():
        rv = pair.acquire(c_dev, index_base=base, workspace=ws, sync=False, events=ev)
        loc = torch.stack([rv[8:16].view(torch.float64)[0], rv[0:8].view(torch.int64)[0].to(torch.float64)])
        if world > 1:
            allr = [torch.empty_like(loc) for _ in range(world)]
            dist.all_gather(allr, loc)
            allr = torch.stack(allr)
        else:
            allr = loc[None]
        h = allr.cpu().numpy()  # the winner reaches the host (what BOHB needs)
        ok = (h[:, 1] >= 0) & (h[:, 0] < np.inf)
        if not ok.any():
            return -1, np.nan
        sc = np.where(ok, h[:, 0], np.inf)
        best = np.min(sc)
        idx = int(np.min(h[(sc == best), 1]))
        return idx, best

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_l = t_g = 0.0
    t0 = time.perf_counter()
    winner = None
    for s in range(a.steps):
        winner = step()
        ml, mg = ev.elapsed_ms()  # step() synchronised on the result: events are complete
        t_l += ml
        t_g += mg
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    last = kde.AcqResult.from_bytes(ws[int(pair.result_offset()):int(pair.result_offset()) + kde.RESULT_BYTES]
                                    .cpu().numpy().tobytes())
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    pairs_step = world * Nc * (Ng + Nb)
    value = pairs_step * a.steps / el
    W = 3 * a.dc + 2 * a.du + 4
    avg_l, avg_g = t_l / a.steps, t_g / a.steps
    achieved = W * Nc * (Ng + Nb) / ((avg_l + avg_g) * 1e-3) / 1e12
    workload = "kde_acquisition_d%d_%dc%du_obs%d_cand%d" % (D, a.dc, a.du, a.obs, Nc)
    traffic = load_traffic(workload)
    out = {
        "metric": METRIC, "value": value, "unit": "pairs/s", "n_gpus": world, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": el / a.steps * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f32", "data": "synthetic",
        "config": {"workload": workload, "candidates_per_gpu": Nc, "observations": a.obs, "n_good": Ng,
                   "n_bad": Nb, "dims": "%dc+%du" % (a.dc, a.du), "levels": a.levels,
                   "parallelism": "candidate-sharded x%d, RCCL all_gather of local winners" % world,
                   "winner": winner[0], "shortlist": last.shortlist},
        "roofline": {"bound": "valu", "achieved": achieved, "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
                     "frac": achieved / PEAK_FP32_TFLOPS, "traffic": traffic,
                     "kernel": "kde_logpdf_kernel<24,8,false> (l and g launches)",
                     "flops_per_pair": W, "ms_per_launch": {"l": avg_l, "g": avg_g}},
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not a.no_cpu:
        try:
            out["cpu_baseline"] = cpu_baseline(X, pair.good.rows_dev.cpu().numpy(), pair.bad.rows_dev.cpu().numpy(),
                                               pair, var_type, cands, a.cpu_seconds)
        except Exception as e:  # the baseline is a side measurement; report why it is missing
            out["cpu_baseline"] = {"error": repr(e)}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
