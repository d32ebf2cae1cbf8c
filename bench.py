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
time.  roofline: the scoring kernel (kde_logpdf: l and g in one pair launch per step), timed with HIP events on
its own stream inside the timed region; algorithmic work W = 3*Dc + 2*Du + 4 = 92 flops per pair
 against the 2516.6 TFLOP/s dense f16 MFMA peak the kernel runs on (the fp32 VALU
basis, 157.3 TFLOP/s, beside it).  cpu_baseline: the C oracle
(oracle/kde_oracle.c, fp64, OpenMP) on the host cores, on a bounded candidate sample.
"""

import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "candidate KDE evals/sec (cand×obs pairs) at D=32, 1/2/4/8 MI355X; % VALU peak"
PEAK_FP32_TFLOPS = 157.3   # MI355X_MICROARCH.md: peak FP32 vector (= f32 MFMA) rate
PEAK_F16_MFMA_TFLOPS = 2516.6  # MI355X_MICROARCH.md: dense BF16/FP16 MFMA (~2.5 PF; no sparsity credit)
PEAK_FP64_TFLOPS = 78.6    # MI355X FP64 vector peak (AMD spec; not in MI355X_MICROARCH.md)
CLOCK_GHZ = 2.4            # spec engine clock (the chip holds ~2.0-2.1 GHz under this load)
N_SIMD = 1024              # 256 CUs x 4 SIMDs


def kernel_model(kde_obj, dc, du):
    """Name and per-256-pair cost model of the scoring kernel a prepared KDE runs.

    hbx_score_h.hip (16x16 tiles, variant bit 4): one output tile = 16 candidates x 16 observations =
    256 pairs per SIMD:
      matrix pipe: NSC dense 16x16x32 f16 MFMAs + KC/2 sparse 16x16x64 (16 cycles each)
      issue:       8 cycles held per matrix instruction + 4 v_exp_f32 (8 each) + 4 v_add_f32 (4 each)
    hbx_score_h32.hip (32x32 tiles, variant bit 6): one tile = 1024 pairs:
      matrix pipe: h32_nd(NSC) = ceil((6 + 24 NSC) / 16) dense 32x32x16 f16 MFMAs (3 slots per
                   continuous dim, 6 for the C_j / c_i pieces) + KP = ceil(KC / 2) sparse 32x32x32 (32
                   cycles each; the acquisition's FAST instance multiplies the one-hot hi parts only, the
                   precise one adds KP for the lo parts)
      issue:       8 cycles held per matrix instruction + 16 v_exp_f32 + 16 v_add_f32
    both quoted per 256 pairs (MI355X_MICROARCH.md, 'vector-instruction ISSUE cost').  Dense-equivalent
    matrix work: 2 x 32 x (NSC + KC) flops per pair either way."""
    v = kde_obj.variant
    signed, kc, hmode, h32 = v & 1, (v >> 1) & 7, (v >> 4) & 1, (v >> 6) & 1
    if not hmode:
        return {"kernel": "kde_logpdf_%s_kernel (f32 MFMA fallback)" % ("oh" if kc else ""), "model": None}
    nsc = (4 * kde_obj.dc_pad + 31) // 32
    if h32:
        coarse = bool((v >> 7) & 1) and not signed  # the acquisition's coarse pre-screen instance
        nd = (6 + (8 if coarse else 24) * nsc + 15) // 16  # h32c_nd / h32_nd dense steps
        kp = (kc + 1) // 2  # 32-position one-hot steps
        fast = kp > 0 and not coarse  # the acquisition's instance
        n_mat = nd + kp * (1 if (fast or coarse) else 2) + (kp if signed else 0)  # per 1024 pairs (+ parity)
        valu = 16 * 8 + 16 * 4 + (32 * 4 if signed else 0)  # exp2, add (+ fract, fma when signed)
        if signed:
            name = "kde_logpdf_h32s_kernel<%d,%d,%s>" % (nsc, kp, "true" if fast else "false")
        else:
            name = "kde_logpdf_h32_kernel<%d,%d,%s,%s>" % (nsc, kp, "true" if fast else "false",
                                                           "true" if coarse else "false")
        return {"kernel": name,
                "model": {"matrix_instr_per_1024_pairs": n_mat, "sparse_onehot": kc > 0,
                          "pipe_cycles": 32 * n_mat / 4, "issue_cycles": (8 * n_mat + valu) / 4,
                          "bound_cycles": max(32 * n_mat, 8 * n_mat + valu) / 4,
                          "dense_equiv_flops_per_pair": 2 * (16 * nd + 32 * (n_mat - nd))}}
    sparse = (not signed) and kc > 0 and kc % 2 == 0
    n_mat = nsc + (kc // 2 if sparse else kc)
    pipe = 16 * n_mat
    issue = 8 * n_mat + 4 * 8 + 4 * 4
    return {"kernel": "kde_logpdf_h_kernel<%d,%d,%s>" % (nsc, kc, "true" if signed else "false"),
            "model": {"matrix_instr_per_tile": n_mat, "sparse_onehot": bool(sparse), "pipe_cycles": pipe,
                      "issue_cycles": issue, "bound_cycles": max(pipe, issue),
                      "dense_equiv_flops_per_pair": 2 * 32 * (nsc + kc)}}


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


def parse(argv=None):
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
    ap.add_argument("--no-config5", action="store_true", help="skip the secondary SH-promotion line")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="winner exchange: nccl (= RCCL over xGMI) or gloo (CPU, multi-process rehearsal)")
    ap.add_argument("--share-gpu", action="store_true", help="ranks share the visible GPUs (rehearsal only)")
    ap.add_argument("--total-candidates", type=int, default=None,
                    help="strong scaling: the main line scores this many candidates in total, sharded over the "
                         "ranks (config #4: 10000000); default: --candidates per GPU (weak)")
    ap.add_argument("--strong-total", type=int, default=10_000_000,
                    help="N>1: the config #4 side line (this many candidates in total over the ranks); 0 = off")
    ap.add_argument("--profile-tag", default=None,
                    help="profiles/ directory holding the rocprofv3 summaries of this very run (recorded in the line)")
    ap.add_argument("--launch-check", action="store_true",
                    help="ranks report (rank, world size) as JSON and exit before any GPU call (tests the launcher)")
    return ap.parse_args(argv)


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def plan_launch(gpus, env, argv, script):
    """How this process runs ``--gpus N`` (decided before any GPU call):
    ("run", world) -- this process is one rank of `world` (WORLD_SIZE set by a launcher, or N = 1 alone);
    ("spawn", cmd) -- N > 1 without a launcher: run N ranks as children of torch.distributed.run (one process
    per GPU, rendezvous on 127.0.0.1) and exit with their status;
    ("error", msg) -- WORLD_SIZE disagrees with --gpus: measuring another rank count than asked is refused."""
    ws = env.get("WORLD_SIZE")
    if ws is None:
        if gpus <= 1:
            return "run", 1
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(gpus),
               "--master-addr", "127.0.0.1", "--master-port", str(free_port()), script] + list(argv)
        return "spawn", cmd
    if int(ws) != gpus:
        return "error", "--gpus %d but WORLD_SIZE %s: launch %d ranks, or pass --gpus %s" % (gpus, ws, gpus, ws)
    return "run", int(ws)


def host_info():
    """Core counts and CPU model of the host the baseline runs on."""
    model = None
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    quota, qcpus = None, None
    try:  # the job's cgroup CPU quota ("max" or "<quota_us> <period_us>")
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q = fh.read().split()
        if q[0] != "max":
            qcpus = int(q[0]) / int(q[1])
        quota = q[0] if q[0] == "max" else "%.1f cpus" % qcpus
    except (OSError, ValueError, IndexError, ZeroDivisionError):
        pass
    return {"nproc": os.cpu_count(), "affinity": len(os.sched_getaffinity(0)), "cpu_model": model,
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS"), "cgroup_cpu_max": quota, "cgroup_cpus": qcpus}


_CPU_PDFS = [None]     # (pdf_l, pdf_g) of cpu_baseline's candidate sample (C oracle, fp64)
_PRECISE_OUT = [None]  # (ln l, ln g) of precise_line over every candidate (hbx_kde_logpdf_rtol)


def logpdf_oracle_check(rtol=1e-5):
    """precise_logpdf at full size against the C oracle: the GPU's ln l(x), ln g(x) of the candidates whose pdfs
    cpu_baseline computed anyway (its bounded sample: the first n candidates), relative error
    |ln p_gpu - ln p_oracle| / max(1, |ln p_oracle|) -- the north-star contract (1e-5)."""
    if _CPU_PDFS[0] is None or _PRECISE_OUT[0] is None:
        return None
    res = {}
    worst = 0.0
    for name, ref, got in (("l", _CPU_PDFS[0][0], _PRECISE_OUT[0][0]), ("g", _CPU_PDFS[0][1], _PRECISE_OUT[0][1])):
        n = ref.shape[0]
        with np.errstate(divide="ignore"):
            lr = np.log(ref)
        fin = np.isfinite(lr)
        err = np.abs(got[:n][fin] - lr[fin]) / np.maximum(1.0, np.abs(lr[fin]))
        res[name] = {"candidates": int(fin.sum()), "max_rel_err": float(err.max()) if err.size else None,
                     "not_finite_in_oracle": int((~fin).sum())}
        worst = max(worst, float(err.max()) if err.size else 0.0)
    res.update(max_rel_err=worst, rtol=rtol, ok=bool(worst <= rtol),
               checker="oracle/kde_oracle.c (fp64, the reference's arithmetic with libm exp), cpu_baseline's sample")
    return res


def cpu_baseline(X, good_rows, bad_rows, pair, var_type, cands, target_s):
    """CPU baselines on the host cores, bounded samples of the same workload:
    * value: the C oracle (oracle/kde_oracle.c, fp64, the reference's arithmetic, OpenMP over
      candidates) with one thread per host core this process may run on: the affinity mask, capped by the
      job's cgroup CPU quota when there is one (the GPU box's lease grants 16 of its 256 cores: 256 threads
      under a 16-CPU quota measured 6.0e7 pairs/s against 1.5e8 with 16, profiles/r04/bench.json notes);
    * reference_as_called: the reference's own path, KDEMultivariate.pdf for l and g per candidate
      (bohb.py:149), single core -- statsmodels is not installed on the box, so its numpy restatement
      oracle.kde_oracle.pdf stands in (bit-identical to statsmodels on every golden fixture), level
      counts recomputed per call as statsmodels does; a candidate subsample, linear in Nc."""
    from oracle import c_oracle
    from oracle import kde_oracle as O
    hi = host_info()
    threads = hi["affinity"] or 1
    if hi["cgroup_cpus"]:
        threads = max(1, min(threads, int(math.ceil(hi["cgroup_cpus"]))))
    Xg, Xb = X[good_rows], X[bad_rows]
    args_g = (Xg, pair.good.bw, var_type, pair.good.nlev)
    args_b = (Xb, pair.bad.bw, var_type, pair.bad.nlev)
    n = max(threads, 16)
    while True:
        t0 = time.perf_counter()
        pl = c_oracle.kde_pdf(*args_g, cands[:n], nthreads=threads)
        pg = c_oracle.kde_pdf(*args_b, cands[:n], nthreads=threads)
        dt = time.perf_counter() - t0
        if dt >= target_s * 0.5 or n >= cands.shape[0]:
            break
        n = int(min(cands.shape[0], max(2 * n, n * (target_s / max(dt, 1e-3)))))
    _CPU_PDFS[0] = (pl, pg)  # the sample's oracle pdfs: precise_logpdf's full-size check (main)
    nobs = Xg.shape[0] + Xb.shape[0]
    out = {"value": n * nobs / dt, "unit": "pairs/s", "cores": threads, "kind": "port",
           "sample": "%d of the %d candidates x %d observations (D=%d), fp64 C oracle (reference arithmetic), "
                     "%d OpenMP threads = the affinity mask (%d cores) capped by the job's cgroup quota (%s), %.1f s"
                     % (n, cands.shape[0], nobs, X.shape[1], threads, hi["affinity"], hi["cgroup_cpu_max"], dt)}
    out.update(hi)
    m, t_ref = 0, 0.0
    t0 = time.perf_counter()
    while t_ref < min(4.0, target_s / 3) and m < cands.shape[0]:
        O.pdf(Xg, pair.good.bw, var_type, cands[m])
        O.pdf(Xb, pair.bad.bw, var_type, cands[m])
        m += 1
        t_ref = time.perf_counter() - t0
    out["reference_as_called"] = {"value": m * nobs / t_ref, "unit": "pairs/s", "cores": 1,
                                  "kind": "numpy restatement of KDEMultivariate.pdf (statsmodels absent on the box)",
                                  "sample": "%d candidates, KDEMultivariate.pdf arithmetic per candidate "
                                            "(numpy restatement, single core), %.1f s" % (m, t_ref)}
    return out


def reference_loop_baseline(device, n_obs=400, dims=(24, 8), calls=3):
    """CPU baseline of the one-worker loop at default sizes (VERDICT r04 missing #3), the reference's own
    arithmetic on one core: a model-based get_config = bohb.py:133-152 -- the per-element draws (one scipy
    truncnorm.rvs per continuous element, rand / randint per categorical one) and KDEMultivariate.pdf of l
    and g per candidate (statsmodels is not installed on the box: oracle.kde_oracle.pdf, its numpy
    restatement, bit-identical on every golden fixture) -- and a refit = bohb.py:220-246 (np.argsort, the
    good / bad rows, 1.06 std n^(-1/(4+D)), np.unique level counts).  Beside bench's
    sh_stage_interleaved_host_sampler (the drop-in on the same loop shape)."""
    from oracle import kde_oracle as O
    from hpbandster_amd import kde
    from hpbandster_amd import synthetic as S
    from hpbandster_amd.config_generators import bohb as Bm
    D = sum(dims)
    vt = S.var_type_string(*dims)
    X = S.make_observations(n_obs, dims[0], dims[1], 4, seed=51)
    Lo = S.make_losses(n_obs, seed=52)
    pair = kde.fit_pair(X, Lo, vt, D + 1, device=device)
    good = Bm._HostModel(X[pair.good.rows_dev.cpu().numpy()], pair.good.bw)
    Xb = X[pair.bad.rows_dev.cpu().numpy()]
    lv = np.array([0] * dims[0] + [4] * dims[1])
    R = np.random.RandomState(5)
    t0 = time.perf_counter()
    for _ in range(calls):
        cands = Bm._draw_rvs(good, lv, 3, 64, R)
        best, bi = np.inf, -1
        for i in range(64):
            v = O.py_score(O.pdf(good.data, good.bw, vt, cands[i]), O.pdf(Xb, pair.bad.bw, vt, cands[i]))
            if v < best:
                best, bi = v, i
    get_ms = (time.perf_counter() - t0) / calls * 1e3
    t0 = time.perf_counter()
    for _ in range(10):
        idx = np.argsort(Lo)
        ng, nb = kde.bohb_split_sizes(n_obs, D + 1)
        for rows, n in ((idx[:ng], ng), (idx[-nb:], nb)):
            data = X[rows]
            bw = 1.06 * np.std(data, axis=0) * n ** (-1. / (4 + D))
            lev = [np.unique(data[:, d]).size for d in range(D) if vt[d] == "u"]
    refit_ms = (time.perf_counter() - t0) / 10 * 1e3
    return {"workload": "one_worker_loop_d%d_obs%d_64cand" % (D, n_obs), "cores": 1,
            "ms_per_model_based_get_config": get_ms, "ms_per_refit": refit_ms,
            "ms_per_request_at_random_fraction_1_3": 2. / 3 * get_ms + refit_ms,
            "kind": "reference arithmetic in numpy/scipy on one core (KDEMultivariate.pdf as its numpy restatement)",
            "sample": "%d model-based get_config calls, 10 refits" % calls}


def config5(device, B=10_000, n=1_000, reps=10, rank=0, world=1, dist=None):
    """Secondary line: BASELINE config #5, batched successive-halving promotion (eta=3 -> k=333) over
    B brackets x n configs (fp64 losses resident in HBM) plus one batched KDE refit of every bracket
    (D = 32: 24 continuous + 8 categorical, bandwidths and level counts).  Brackets are independent: with N ranks each promotes its own B/N brackets (no
    collective; weak scaling of the bracket count per GPU is not applied -- the total stays B).
    Algorithmic HBM bytes per promoted config: 8 (loss read) + 1 (mask written)."""
    import torch
    from hpbandster_amd import _native as N
    from hpbandster_amd import kde
    from hpbandster_amd import synthetic as S
    from hpbandster_amd.distributed import shard_range
    L = N.lib()
    b0, b1 = shard_range(B, rank, world)
    Bl = b1 - b0
    losses = torch.from_numpy(S.make_bracket_losses(B, n)[b0:b1].reshape(-1)).to(device)
    seg = torch.arange(Bl + 1, dtype=torch.int64, device=device) * n
    k = torch.full((Bl,), float(n // 3), dtype=torch.float64, device=device)
    adv = torch.empty(Bl * n, dtype=torch.uint8, device=device)
    nadv = torch.empty(Bl, dtype=torch.int64, device=device)
    sh = N.stream_handle(None, device)
    # numpy's tie order (the drop-in's): the selection flags brackets whose ties straddle k, a re-rank
    # kernel follows (a pool of 64 workgroups, exiting at once when none is flagged)
    sb = int(L.hbx_sh_promote_scratch_bytes(Bl, n, Bl * n, 0, N.ORDER_NUMPY))
    scr = torch.empty(sb, dtype=torch.uint8, device=device)
    kev = kde.ScoreEvents()  # stamped at the selection kernel's start and end (hipExtLaunchKernel)

    def promote(ev=None):  # mask only (what process_results needs): the O(n) select kernel
        N.check(L.hbx_sh_promote_ex(N.ptr(losses), N.ptr(seg), Bl, n, Bl * n, N.ptr(k), None, N.ptr(adv),
                                    N.ptr(nadv), N.ptr(scr), sb, N.ORDER_NUMPY, ev, sh))
    promote()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for _ in range(reps):
        promote()
    e1.record()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    ms_call = e0.elapsed_time(e1) / reps
    kms = []
    for _ in range(reps):  # the selection kernel alone, what rocprof's kernel trace shows
        promote(kev.address)
        torch.cuda.synchronize()
        kms.append(kev.elapsed_ms(True)[0])
    ms = float(np.median(kms))
    ok = bool((nadv == n // 3).all().item())
    if dist is not None:
        t = torch.tensor([wall, ms, 0.0 if ok else 1.0], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall, ms, ok = float(t[0]), float(t[1]), float(t[2]) == 0.0
    # batched refit of every bracket's KDE pair at config #3's dims ("plus per-bracket fit on
    # D=32"): numpy-order argsort of each bracket's losses, good = head / bad = tail, normal-reference
    # bandwidths (np.std bit for bit) and observed level counts of 24 continuous + 8 categorical dims.
    # Observations drawn on the device (1e7 x 32 f64 = 2.56 GB resident)
    dc, du, lev = 24, 8, 4
    D = dc + du
    g = torch.Generator(device=device)
    g.manual_seed(4 + rank)
    X = torch.empty((Bl * n, D), dtype=torch.float64, device=device)
    X[:, :dc] = torch.rand((Bl * n, dc), dtype=torch.float64, device=device, generator=g)
    X[:, dc:] = torch.randint(0, lev, (Bl * n, du), device=device, generator=g).to(torch.float64)
    order = torch.empty(Bl * n, dtype=torch.int64, device=device)
    sb = int(L.hbx_sort_scratch_bytes(Bl * n))
    scr = torch.empty(sb, dtype=torch.uint8, device=device)
    ng, nb = kde.bohb_split_sizes(n, D + 1)
    ngd = torch.full((Bl,), ng, dtype=torch.int64, device=device)
    nbd = torch.full((Bl,), nb, dtype=torch.int64, device=device)
    fg = torch.full((Bl,), kde.bandwidth_factor(ng, D), dtype=torch.float64, device=device)
    fb = torch.full((Bl,), kde.bandwidth_factor(nb, D), dtype=torch.float64, device=device)
    vt = torch.tensor([0] * dc + [1] * du, dtype=torch.int32, device=device)
    bwg = torch.empty((Bl, D), dtype=torch.float64, device=device)
    bwb = torch.empty((Bl, D), dtype=torch.float64, device=device)
    nlg = torch.empty((Bl, D), dtype=torch.int32, device=device)
    nlb = torch.empty((Bl, D), dtype=torch.int32, device=device)

    def refit():
        N.check(L.hbx_seg_argsort_ex(N.ptr(losses), N.ptr(seg), Bl, n, Bl * n, N.ptr(order), N.ptr(scr), sb,
                                     N.ORDER_NUMPY, sh))
        N.check(L.hbx_kde_fit(N.ptr(X), D, N.ptr(seg), Bl, N.ptr(order), N.ptr(ngd), N.ptr(nbd), N.ptr(fg),
                              N.ptr(fb), N.ptr(vt), N.ptr(bwg), N.ptr(bwb), N.ptr(nlg), N.ptr(nlb), sh))
    refit()
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        refit()
    e1.record()
    torch.cuda.synchronize()
    ms_fit = e0.elapsed_time(e1) / reps
    # spot check against the host restatement (oracle-free: numpy's order restated in this module's
    # tests; here the tie-free losses make any argsort numpy's)
    b = Bl // 2
    rows = np.argsort(S.make_bracket_losses(B, n)[b0 + b], kind="stable")
    Xb = X[b * n:(b + 1) * n].cpu().numpy()
    good_b, bad_b = Xb[rows[:ng]], Xb[rows[-nb:]]
    lev_ok = all(int(nlg[b, d]) == len(np.unique(good_b[:, d])) and int(nlb[b, d]) == len(np.unique(bad_b[:, d]))
                 for d in range(dc, D))
    bw_ok = bool(np.array_equal(bwg[b].cpu().numpy(), 1.06 * np.std(good_b, axis=0) * ng ** (-1. / (4 + D))) and
                 np.array_equal(bwb[b].cpu().numpy(), 1.06 * np.std(bad_b, axis=0) * nb ** (-1. / (4 + D))) and lev_ok)
    # algorithmic HBM bytes: losses read (8) and the order written and read (16) per config, each set's rows
    # read ONCE: (ng + nb) D 8 per bracket (the deviation pass is a re-read a kernel holding the rows on chip
    # would not make; the wave kernel makes it, profiles/r06/side/)
    fit_bytes = Bl * (24 * n + (ng + nb) * D * 8)
    fit_gbs = fit_bytes / (ms_fit * 1e-3) / 1e9
    del X
    torch.cuda.empty_cache()
    gbs = Bl * n * 9 / (ms * 1e-3) / 1e9
    # the reference rule on the host (HB_iteration.py:180-182: argsort(argsort(losses)) < k per bracket),
    # a bracket subsample, x B
    Lh = S.make_bracket_losses(B, n)
    nb_cpu = 200
    t0 = time.perf_counter()
    for b in range(nb_cpu):
        _ = np.argsort(np.argsort(Lh[b])) < n // 3
    cpu_s = (time.perf_counter() - t0) / nb_cpu * B
    out = {"workload": "sh_promotion_B%d_n%d_eta3" % (B, n), "brackets_per_rank": Bl, "ranks": world,
           "configs_per_s": B * n / (wall / reps), "ms_per_launch": ms, "masks_ok": ok,
           "ms_per_call": ms_call, "tie_order": "numpy",
           "timing": "ms_per_launch: median of the selection kernel's start/end stamps (hipExtLaunchKernel); "
                     "ms_per_call: events around back-to-back calls (selection + numpy-order re-rank launch)",
           "roofline": {"bound": "hbm", "achieved": gbs, "peak": 8000.0, "unit": "GB/s", "frac": gbs / 8000.0,
                        "bytes_per_config": 9, "kernel": "sh_select_kernel"},
           "refit_all_brackets_ms": ms_fit, "refit_dims": "%dc+%du (L=%d)" % (dc, du, lev),
           "refit_bandwidths_spot_check": bw_ok,
           "refit_roofline": {"bound": "hbm", "achieved": fit_gbs, "peak": 8000.0, "unit": "GB/s",
                              "frac": fit_gbs / 8000.0, "bytes": fit_bytes,
                              "basis": "losses 8 + order 16 per config, + (n_good + n_bad) D 8 per bracket: every row read once"},
           "cpu_reference_rule": {"s_for_all_brackets": cpu_s, "cores": 1,
                                  "sample": "%d brackets of numpy argsort(argsort) < k, x %d" % (nb_cpu, B)}}
    return out


def blocked_candidates(lo, hi, dc, du, levels, device):
    """Rows [lo, hi) of the seeded candidate stream (synthetic.make_candidates_blocked: U[0,1) continuous,
    U{0..L-1} categorical, block b of 65536 rows from RandomState([3, b])), drawn on the host and moved to
    the device.  Any slice is drawn without the rows before it, so every rank draws only its own shard, the
    weak set at N ranks is the first N x 1e6 rows and config #4 is the first 1e7 -- the sets whose winners
    the C oracle pinned at full size (tests/golden/full_winners.json)."""
    import torch
    from hpbandster_amd import synthetic as S
    return torch.from_numpy(S.make_candidates_blocked(lo, hi, dc, du, levels)).to(device)


_PINNED = [None]


def pinned_winners():
    """tests/golden/full_winners.json (data: the C oracle's full-size winners, tests/golden/gen_full_winners.py)."""
    if _PINNED[0] is None:
        try:
            with open(os.path.join(ROOT, "tests", "golden", "full_winners.json")) as fh:
                _PINNED[0] = json.load(fh)
        except (OSError, ValueError):
            _PINNED[0] = {}
    return _PINNED[0]


def winner_check(entry, index, score, pdf_l=None, pdf_g=None):
    """The acquisition's winner against a pinned one: index, score (and the pdfs when given) bit for bit.
    None when nothing is pinned for this workload."""
    if not entry:
        return None
    ok = index == entry["winner"] and float(score).hex() == entry["score_hex"]
    if pdf_l is not None:
        ok = ok and float(pdf_l).hex() == entry["pdf_l_hex"] and float(pdf_g).hex() == entry["pdf_g_hex"]
    return {"winner_ok": bool(ok), "pinned_winner": entry["winner"], "pinned_score": entry["score"],
            "pinned_margin_rel": entry["margin_rel"], "pinned_by": "tests/golden/full_winners.json (C oracle, %s)"
                                                                 % ("exact over every candidate" if not entry.get("screen")
                                                                    else "screen + exact re-score")}


def pinned_prefix(n, dc, du, levels, obs):
    """The pinned entry of the blocked stream's first n rows at config #3's model, if any."""
    if (dc, du, levels, obs) != (24, 8, 4, 10_000):
        return None
    return pinned_winners().get("config3_prefixes", {}).get("prefix_%d" % n)


def config4_line(pair, device, dc, du, levels, Nc=10_000_000, shards=8, reps=3):
    """Side line: BASELINE config #4's whole workload on ONE MI355X -- 1e7 candidates x config #3's 1e4
    observations (D = 32) -- as one acquisition, and as the 8 per-rank shards of the 8-GPU run
    (index_base = shard start, here one after another on this GPU) reduced by the exchange's rule.
    The winners must agree.  Candidates are drawn on the device (U[0,1) continuous, U{0..L-1}
    categorical; the scoring cost is data independent)."""
    import torch
    from hpbandster_amd import kde
    from hpbandster_amd.distributed import reduce_records_host, shard_range
    C = blocked_candidates(0, Nc, dc, du, levels, device)
    ws = torch.empty(pair.workspace_bytes(Nc), dtype=torch.uint8, device=device)
    r = pair.acquire(C, workspace=ws)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        r = pair.acquire(C, workspace=ws)
    el = (time.perf_counter() - t0) / reps
    recs = []
    for k in range(shards):
        lo, hi = shard_range(Nc, k, shards)
        recs.append(pair.acquire(C[lo:hi], index_base=lo, workspace=ws))
    best, near = reduce_records_host(recs)
    sharded = recs[best].index if best >= 0 else -1
    del C, ws
    torch.cuda.empty_cache()
    pairs = Nc * (pair.good.nobs + pair.bad.nobs)
    out = {"workload": "kde_acquisition_d%d_%dc%du_obs%d_cand%d_one_gpu" % (dc + du, dc, du,
                                                                          pair.good.nobs + pair.bad.nobs, Nc),
           "value": pairs / el, "unit": "pairs/s", "ms_per_acquisition": el * 1e3, "winner": r.index,
           "winner_8_shards": sharded, "winners_identical": r.index == sharded, "shortlist": r.shortlist,
           "candidates": "rows [0, %d) of synthetic.make_candidates_blocked (seed 3)" % Nc}
    chk = winner_check(pinned_prefix(Nc, dc, du, levels, pair.good.nobs + pair.bad.nobs), r.index, r.score,
                       r.pdf_l, r.pdf_g)
    if chk:
        chk["winner_ok"] = chk["winner_ok"] and sharded == r.index
        out.update(chk)
    return out


def strong_line(pair, device, a, rank, world, dist, xchg, reps=10):
    """Side line at N > 1: BASELINE config #4 -- a fixed total of candidates (1e7) x config #3's
    observations, sharded over the ranks (each scores shard_range(total, rank, N) with global indices,
    drawn on its own device: config4_line's set, so the winner is config4_line's at every N), one winner
    exchange per step; max-over-ranks time (strong scaling)."""
    import torch
    from hpbandster_amd import kde
    from hpbandster_amd.distributed import shard_range
    lo, hi = shard_range(a.strong_total, rank, world)
    Nc = hi - lo
    C = blocked_candidates(lo, hi, a.dc, a.du, a.levels, device)
    ws = torch.empty(pair.workspace_bytes(Nc), dtype=torch.uint8, device=device)

    def step():
        rv = pair.acquire(C, index_base=lo, workspace=ws, sync=False)
        if xchg is not None:
            rv = xchg.exchange(rv)
        return kde.AcqResult.from_bytes(kde.fetch_bytes(rv))

    step()
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        r = step()
    torch.cuda.synchronize()
    dist.barrier()
    el = time.perf_counter() - t0
    t = torch.tensor([el], dtype=torch.float64, device=device if dist.get_backend() == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    el = float(t.item())
    del C, ws
    torch.cuda.empty_cache()
    pairs = a.strong_total * (pair.good.nobs + pair.bad.nobs)
    out = {"workload": "kde_acquisition_d%d_obs%d_total%d_sharded" % (a.dc + a.du, a.obs, a.strong_total),
           "scaling": "strong", "value": pairs * reps / el, "unit": "pairs/s", "ms_per_step": el / reps * 1e3,
           "candidates_per_rank": Nc, "ranks": world, "winner": r.index}
    chk = winner_check(pinned_prefix(a.strong_total, a.dc, a.du, a.levels, a.obs), r.index, r.score)
    if chk:
        out.update(chk)
    return out


def promote_dropin(device, n=1000, reps=50):
    """Side line: the drop-in SuccessiveHalving.process_results at one bracket of n configurations
    (HB_iteration.py:149-190 as HpBandSter calls it: one bracket per call), wall clock per call, beside
    the reference's own arithmetic on the host (the dict walk, argsort(argsort(losses)) < k, the status
    updates) restated in numpy."""
    from hpbandster_amd.HB_iteration import SuccessiveHalving
    rs = np.random.RandomState(8)

    def make():
        sh = SuccessiveHalving(0, [n, n // 3, 1], [1.0, 3.0, 9.0], lambda b: ({}, {}), device=device)
        for i in range(n):
            cid = (0, 0, i)
            sh.data[cid] = {'config': {}, 'config_info': {}, 'results': {1.0: {'loss': float(rs.rand())}},
                            'time_stamps': {}, 'exceptions': {}, 'status': 'REVIEW', 'budget': 1.0}
        sh.actual_num_configs[0] = n
        return sh

    def host_rule(sh):  # the reference's process_results body (HB_iteration.py:162-190) in numpy
        sh.SH_iter += 1
        ids = [c for c in sh.data.keys() if sh.data[c]['status'] == 'REVIEW']
        budgets = [sh.data[c]['budget'] for c in ids]
        losses = np.array([sh.data[c]['results'][budgets[0]]['loss'] for c in ids])
        ranks = np.argsort(np.argsort(losses))
        advance = ranks < sh.num_configs[sh.SH_iter]
        for i, c in enumerate(ids):
            if advance[i]:
                sh.data[c]['status'] = 'QUEUED'
                sh.data[c]['budget'] = sh.budgets[sh.SH_iter]
                sh.actual_num_configs[sh.SH_iter] += 1
            else:
                sh.data[c]['status'] = 'TERMINATED'
        return advance

    sh0 = make()
    sh0.process_results()
    res = {}
    for name, fn in (("gpu", lambda sh: sh.process_results()), ("host_numpy", host_rule)):
        shs = [make() for _ in range(reps)]
        t0 = time.perf_counter()
        for sh in shs:
            fn(sh)
        res[name] = (time.perf_counter() - t0) / reps * 1e3
    # the ranking step alone: advance_mask under the size policy (host for tie-free brackets <= HOST_MAX),
    # forced onto the GPU (mapped losses + one-wave select kernel + completion word), and numpy's rule
    from hpbandster_amd import promote
    losses = rs.rand(n)
    k = n // 3

    def per_call(fn, r=reps * 20):
        fn()
        t0 = time.perf_counter()
        for _ in range(r):
            fn()
        return (time.perf_counter() - t0) / r * 1e3
    rank_auto = per_call(lambda: promote.advance_mask(losses, k, device=device))
    rank_gpu = per_call(lambda: promote.advance_mask(losses, k, device=device, policy="gpu"))
    rank_host = per_call(lambda: np.argsort(np.argsort(losses)) < k)
    tie = np.round(losses, 1)  # tied losses straddle the k-th place: numpy 1.26.4's order, on the GPU
    rank_tie = per_call(lambda: promote.advance_mask(tie, k, device=device))
    return {"workload": "process_results_one_bracket_n%d" % n, "ms_per_call": res["gpu"],
            "host_numpy_ms_per_call": res["host_numpy"], "rank_step_ms": rank_auto,
            "rank_step_gpu_ms": rank_gpu, "rank_step_tied_ms": rank_tie, "host_rank_step_ms": rank_host,
            "policy": "host when tie-free and n <= %d (promote.HOST_MAX), else GPU" % promote.HOST_MAX}


def batched(pair, device, dc, du, levels, calls=81, per_call=64, reps=20):
    """Side measurement: one SH stage's get_config calls at the reference's real size
    (bohb.py:23 num_samples=64; 81 = the first stage of an eta=3 bracket) against config #3's model:
    81 sequential acquisitions of 64 candidates vs one batched pass; wall time per call, winners
    reaching the host in both cases (what BOHB needs)."""
    import torch
    from hpbandster_amd import synthetic as S
    C = torch.from_numpy(S.make_candidates(calls * per_call, dc, du, levels, seed=S.SEED_CAND + 7)).to(device)
    ws1 = torch.empty(pair.workspace_bytes(per_call), dtype=torch.uint8, device=device)
    wsb = torch.empty(pair.batch_workspace_bytes(calls * per_call, per_call), dtype=torch.uint8, device=device)
    rb = torch.empty(calls * kde_result_bytes(), dtype=torch.uint8, device=device)

    def seq():
        outs = [pair.acquire(C[i * per_call:(i + 1) * per_call], workspace=ws1, sync=False).clone()
                for i in range(calls)]
        return torch.stack(outs).cpu()

    def bat():
        return pair.acquire_batch(C, per_call, workspace=wsb, results=rb, sync=False).cpu()

    a, b = seq(), bat()
    same = bool(torch.equal(a.reshape(-1), b.reshape(-1)))
    res = {}
    for name, fn in (("sequential", seq), ("batched", bat)):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        res[name] = (time.perf_counter() - t0) / reps
    return {"workload": "sh_stage_%dx%d_get_config" % (calls, per_call), "calls": calls,
            "candidates_per_call": per_call, "records_identical": same,
            "ms_sequential": res["sequential"] * 1e3, "ms_batched": res["batched"] * 1e3,
            "get_config_per_s_batched": calls / res["batched"], "speedup": res["sequential"] / res["batched"]}


def sh_stage_line(device, n_obs=400, stage=81, reps=5, interleaved=False, sampler="gpu", dims=(24, 8)):
    """Side measurement (SURVEY 8f row 1 through the drop-in): the first stage of an eta=3 bracket -- 81
    configurations requested through SuccessiveHalving.get_next_run, as HpBandSter.run requests them --
    from BOHB (config #3's dims, 24c + 8u, GPU sampler, num_samples=64) with speculative batching (batches
    of 1, 2, 4, ... while fully served) against one get_config per request; the proposals must be identical.
    interleaved: every request is followed by its run's result (new_result, which refits the model) -- one
    worker, where no batch survives; the timed loop includes the refits."""
    import torch
    from hpbandster_amd import configspace as CS
    from hpbandster_amd.config_generators import BOHB
    from hpbandster_amd.HB_iteration import SuccessiveHalving
    from hpbandster_amd import synthetic as S

    class Job(object):
        pass

    def job(cid, cfg, loss):
        j = Job()
        j.id, j.exception, j.timestamps = cid, None, {}
        j.kwargs = {"config": cfg, "budget": 1.0}
        j.result = {"loss": float(loss), "info": None}
        return j

    def make(spec):
        space = CS.ConfigurationSpace(seed=3)
        for i in range(dims[0]):
            space.add_hyperparameter(CS.UniformFloatHyperparameter("x%02d" % i, lower=0, upper=1))
        for i in range(dims[1]):
            space.add_hyperparameter(CS.CategoricalHyperparameter("y%02d" % i, ["a", "b", "c", "d"]))
        cg = BOHB(space, device=device, sampler=sampler, sampler_seed=77, speculative=spec)
        X = S.make_observations(n_obs, dims[0], dims[1], 4, seed=51)
        Lo = S.make_losses(n_obs, seed=52)
        for i in range(n_obs):
            cg.new_result(job((0, 0, i), CS.Configuration(space, vector=X[i]).get_dictionary(), Lo[i]))
        return cg, space

    def run(batch):
        cg, space = make("auto" if batch else "never")
        np.random.seed(5)
        space.seed(6)
        sh = SuccessiveHalving(0, [stage, stage // 3, stage // 9, 3, 1], [1.0, 3.0, 9.0, 27.0, 81.0], cg.get_config,
                               device=device, batch_sampling=batch)
        lr = np.random.RandomState(9)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        cfgs = []
        for _ in range(stage):
            cid, cfg, _ = sh.get_next_run()
            cfgs.append(cfg)
            if interleaved:
                cg.new_result(job((1,) + tuple(cid[1:]), cfg, lr.rand()))
        torch.cuda.synchronize()
        return time.perf_counter() - t0, cfgs

    res = {}
    for r in range(reps):  # alternated, either one first in turn, best of reps each
        for batch in ((False, True) if r % 2 == 0 else (True, False)):
            t, c = run(batch)
            if batch not in res or t < res[batch][0]:
                res[batch] = (t, c)
    return {"workload": "sh_stage_%d_get_next_run_d%d_obs%d%s%s" % (stage, sum(dims), n_obs,
                                                                  "_interleaved" if interleaved else "",
                                                                  "_host_sampler" if sampler == "host" else ""),
            "ms_sequential": res[False][0] * 1e3, "ms_batched": res[True][0] * 1e3,
            "ms_per_request": res[True][0] * 1e3 / stage,
            "sequential_is": "speculative='never': one draw + acquisition per call",
            "speedup": res[False][0] / res[True][0], "proposals_identical": res[False][1] == res[True][1],
            "note": ("SuccessiveHalving.get_next_run x %d, each followed by its result (new_result + refit); "
                     "batched = the default drop-in (with results in between no batch survives: one call at a time)"
                     % stage)
            if interleaved else
                    ("SuccessiveHalving.get_next_run x %d without results in between (a filled job queue); "
                     "batched = the default drop-in: speculative batches of 1, 2, 4, ... (hbx_kde_acquire_batch)"
                     % stage)}


def threaded_run_line(device, n_iterations=16, workers=8, reps=7, dims=(24, 8)):
    """Side line: the drop-in HpBandSter.run with BOHB (GPU sampler) and `workers` in-process zero-cost workers
    (dispatch.ThreadedDispatcher: results reach job_callback -> new_result on the dispatcher thread while the
    master loop requests runs, HB_master.py:170-177,192-208), job_queue_sizes=(-1, 0) with the queue sized to
    the workers (the reference's BOHB optimizer settings): wall time of the whole run with speculative batches
    (speculative='auto', the default) against one draw + acquisition per call ('never'), alternated, best of
    `reps` each (median and best).  Thread timing makes the proposals differ from run to run.  (Round 6 measured here the next
    call computed ahead of it, which the drop-in then had: 0.69x, i.e. slower -- it was removed.)"""
    from hpbandster_amd.config_generators import BOHB
    from hpbandster_amd.dispatch import ThreadedDispatcher
    from hpbandster_amd.HB_master import HpBandSter
    CS, space, _ = _space_and_jobs(dims)

    def compute(config, budget, working_directory):
        return {"loss": float(sum(v for v in config.values() if isinstance(v, float))) / budget, "info": None}

    def run(spec):
        np.random.seed(7)
        space.seed(8)
        cg = BOHB(space, device=device, sampler="gpu", sampler_seed=5, speculative=spec, min_points_in_model=40)
        disp = ThreadedDispatcher(compute, n_workers=workers)
        m = HpBandSter("bench", cg, eta=3, min_budget=1, max_budget=27, job_queue_sizes=(-1, 0),
                       dynamic_queue_size=True, dispatcher=disp)
        m.adjust_queue_size(workers)
        t0 = time.perf_counter()
        res = m.run(n_iterations)
        el = time.perf_counter() - t0
        m.shutdown()
        return el, len(res.get_all_runs()), cg._calls

    res = {"never": [], "auto": []}
    for r in range(reps):
        for spec in (("never", "auto") if r % 2 == 0 else ("auto", "never")):
            res[spec].append(run(spec))
    med = {k: float(np.median([e[0] for e in v])) for k, v in res.items()}
    best = {k: min(e[0] for e in v) for k, v in res.items()}
    return {"workload": "hpbandster_run_%d_iterations_%d_threaded_workers_d%d" % (n_iterations, workers, sum(dims)),
            "ms_never_median": med["never"] * 1e3, "ms_auto_median": med["auto"] * 1e3,
            "ms_never_best": best["never"] * 1e3, "ms_auto_best": best["auto"] * 1e3,
            "speedup_median": med["never"] / med["auto"], "runs": res["auto"][0][1], "reps": reps,
            "get_config_calls_never": res["never"][0][2],
            "note": "BOHB(sampler='gpu'), zero-cost compute, results on the dispatcher thread; speedup = never / auto "
                    "(speculative batches of back-to-back requests)"}


def _space_and_jobs(dims, levels=4):
    from hpbandster_amd import configspace as CS

    class Job(object):
        pass

    def job(cid, cfg, loss):
        j = Job()
        j.id, j.exception, j.timestamps = cid, None, {}
        j.kwargs = {"config": cfg, "budget": 1.0}
        j.result = {"loss": float(loss), "info": None}
        return j

    space = CS.ConfigurationSpace(seed=3)
    for i in range(dims[0]):
        space.add_hyperparameter(CS.UniformFloatHyperparameter("x%02d" % i, lower=0, upper=1))
    for i in range(dims[1]):
        space.add_hyperparameter(CS.CategoricalHyperparameter("y%02d" % i, ["abcdefgh"[j] for j in range(levels)]))
    return CS, space, job


def get_config_line(device, n_obs=400, dims=(24, 8), calls=30, slow_calls=3):
    """Side line: the DEFAULT drop-in's get_config -- BOHB(space) with the host sampler,
    num_samples=64, bohb.py's draws from the global numpy RNG -- at config #3's dims (24c + 8u) against a
    400-observation model, ms per model-based call (random_fraction=0, so every call samples and scores):
    the draws made by hbx_bohb_draw on numpy's own MT19937 state + one vectorised truncnorm inversion,
    against the same BOHB with the per-element scipy path the reference runs (bohb.py:133-147: one
    truncnorm.rvs per continuous element); the proposals and the global RNG's state must be identical."""
    from hpbandster_amd.config_generators import BOHB
    from hpbandster_amd.config_generators import bohb as Bm
    from hpbandster_amd import synthetic as S
    CS, space, job = _space_and_jobs(dims)
    cg = BOHB(space, device=device, random_fraction=0.0)
    X = S.make_observations(n_obs, dims[0], dims[1], 4, seed=51)
    Lo = S.make_losses(n_obs, seed=52)
    for i in range(n_obs):
        cg.new_result(job((0, 0, i), CS.Configuration(space, vector=X[i]).get_dictionary(), Lo[i]))

    def run(k):
        np.random.seed(5)
        t0 = time.perf_counter()
        out = [cg.get_config(1.0)[0] for _ in range(k)]
        return (time.perf_counter() - t0) / k, out, Bm._global_mt().snap()

    assert Bm.host_draw_ok()
    run(2)
    reps = [run(calls) for _ in range(7)]  # the same 30 calls (seed 5) seven times: median and best per call
    fast, cf, sf = reps[0]
    times = sorted(r[0] for r in reps)
    fast = times[len(times) // 2]
    saved = Bm._HOSTDRAW[0]
    try:
        Bm._HOSTDRAW[0] = False  # the per-element scipy path
        slow, cs, ss = run(slow_calls)
    finally:
        Bm._HOSTDRAW[0] = saved
    _, cf3, sf3 = run(slow_calls)
    return {"workload": "get_config_default_d%d_obs%d_64cand" % (sum(dims), n_obs), "ms_per_call": fast * 1e3,
            "ms_per_call_best": times[0] * 1e3, "timing": "median (and best) of 7 runs of the same %d calls" % calls,
            "ms_per_call_per_element_draws": slow * 1e3, "speedup": slow / fast,
            "proposals_identical": cs == cf3, "global_rng_identical": ss == sf3,
            "model_based_calls": calls,
            "note": "BOHB defaults (host sampler, num_samples=64) with random_fraction=0; per_element = bohb.py's "
                    "scipy truncnorm.rvs per continuous element (what the reference's get_config draws), the rest "
                    "of the call identical (GPU acquisition)"}


def precise_line(pair, c_dev, device, rtol=1e-5, reps=5):
    """Side line: the ln-pdf contract at config #3 -- hbx_kde_logpdf_rtol (the precise
    instance: 3 f16 products per continuous dim, the one-hot hi and lo parts, then every candidate whose
    rigorous bound does not guarantee rtol re-evaluated in fp64 log space on the device) for l(x) and g(x)
    over the same 1e6 candidates (bohb.py:126-129: what a caller who wants the densities gets).  Time per
    KDE call from HIP events on its stream; the fraction of candidates re-evaluated in fp64 read from the
    call's scratch counter."""
    import torch
    from hpbandster_amd import _native as N
    L = N.lib()
    Nc = int(c_dev.shape[0])
    sh = N.stream_handle(None, device)
    sb = int(L.hbx_kde_logpdf_rtol_scratch_bytes(Nc))
    scr = torch.empty(sb, dtype=torch.uint8, device=device)
    out = torch.empty(Nc, dtype=torch.float64, device=device)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    res = {}
    keep = []
    for name, k in (("l", pair.good), ("g", pair.bad)):
        def call():
            N.check(L.hbx_kde_logpdf_rtol(N.ptr(c_dev), Nc, k.k_vars, N.ptr(k.params), N.ptr(k.table), N.ptr(k.X_dev),
                                          N.ptr(k.rows_dev), k.dc_pad, k.du_pad, k.variant, float(rtol), N.ptr(out),
                                          N.ptr(scr), sb, sh))
        call()
        torch.cuda.synchronize()
        ms = []
        for _ in range(reps):
            e0.record()
            call()
            e1.record()
            torch.cuda.synchronize()
            ms.append(e0.elapsed_time(e1))
        refined = int(scr[:4].view(torch.int32).item())
        res[name] = {"ms_per_call": float(np.median(ms)), "observations": k.nobs, "fp64_reevaluated": refined,
                     "fp64_fraction": refined / Nc, "finite": bool(torch.isfinite(out).all().item())}
        keep.append(out.cpu().numpy())
    _PRECISE_OUT[0] = tuple(keep)
    t = res["l"]["ms_per_call"] + res["g"]["ms_per_call"]
    pairs = Nc * (pair.good.nobs + pair.bad.nobs)
    rate = pairs / (t * 1e-3)
    W = 92  # SURVEY 8d algorithmic flops per pair at 24c + 8u
    return {"workload": "kde_logpdf_rtol%g_d32_obs%d_cand%d" % (rtol, pair.good.nobs + pair.bad.nobs, Nc),
            "value": rate, "unit": "pairs/s", "ms_l_plus_g": t, "rtol": rtol, "kernel": "kde_logpdf_dd_kernel<24,8,2,LUT,SG> (fp32 direct differences, packed VALU, observation rows staged once per call and read through scalar loads, categorical matches through LDS tables, a rigorous per-candidate bound)",
            "fp64_kernel": "kde_logpdf_tiled_kernel (the candidates that bound rejects)", "per_kde": res,
            "roofline": {"bound": "valu", "achieved": W * rate / 1e12, "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
                         "frac": W * rate / 1e12 / PEAK_FP32_TFLOPS,
                         "basis": "W = 92 algorithmic flops per pair over the whole hbx_kde_logpdf_rtol call (the fp32 "
                                  "direct-difference pass, then fp64 for the candidates its bound rejects) vs the packed "
                                  "fp32 vector peak"}}


def config2_line(device, reps=50):
    """Side measurement: BASELINE config #2 (1e5 candidates x 1e3 observations x 8 continuous dims,
    BOHB split 150 / 850), whole acquisitions with the winner on the host, as the main line."""
    import torch
    from hpbandster_amd import kde
    from hpbandster_amd import synthetic as S
    X = S.make_observations(1000, 8, 0, 0)
    pair = kde.fit_pair(X, S.make_losses(1000), S.var_type_string(8, 0), 9, device=device)
    Nc = 100_000
    c_dev = torch.from_numpy(S.make_candidates(Nc, 8, 0, 0)).to(device)
    ws = torch.empty(pair.workspace_bytes(Nc), dtype=torch.uint8, device=device)
    for _ in range(5):
        r = pair.acquire(c_dev, workspace=ws)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        r = pair.acquire(c_dev, workspace=ws)
    el = (time.perf_counter() - t0) / reps
    pairs = Nc * (pair.good.nobs + pair.bad.nobs)
    # the scoring launch's own time (HIP events at its start and end, separate calls after the timed ones)
    ev = kde.ScoreEvents()
    launch = []
    for _ in range(20):
        pair.acquire(c_dev, workspace=ws, events=ev)
        launch.append(ev.elapsed_ms(True)[0])
    lm = float(np.median(launch))
    fpp = 3 * 8 + 4  # 3 Dc + 2 Du + 4 flops per pair
    tf = fpp * pairs / (lm * 1e-3) / 1e12
    chk = winner_check(pinned_winners().get("config2"), r.index, r.score, r.pdf_l, r.pdf_g) or {}
    return {"workload": "kde_acquisition_d8_8c_obs1000_cand100000", "value": pairs / el, "unit": "pairs/s",
            "ms_per_step": el * 1e3, "winner": r.index, "variant": int(pair.bad.variant), **chk,
            "scoring_launch_ms": lm, "step_minus_scoring_ms": el * 1e3 - lm,
            "roofline": {"bound": "mfma", "achieved": tf, "peak": PEAK_F16_MFMA_TFLOPS, "unit": "TFLOP/s",
                         "frac": tf / PEAK_F16_MFMA_TFLOPS, "flops_per_pair": fpp,
                         "kernel": ("kde_logpdf_h32_pair1_kernel<1,0> (l and g in one launch, one candidate column "
                                    "tile per wave)" if os.environ.get("HBX_PAIR1", "1") != "0" else
                                    "kde_logpdf_h32_pair_kernel<1,0,false,true> (l and g in one launch)"),
                         "timing": "median of 20 launches' start/end events"}}


def refit_line(X, losses, var_type, device, reps=20):
    """Side measurement: one BOHB refit at config #3's observation set as
    new_result runs it (bohb.py:211-251): one new observation appended to the budget's rows resident in
    HBM, then ``hbx_kde_refit_sync`` (split, bandwidths, level counts, both KDEs prepared for scoring; the
    output block published to mapped host memory) -- beside the same arithmetic in host numpy (argsort, row gathers,
    1.06 std n^(-1/(4+D)), unique level counts), and the refit from host arrays (all rows uploaded)."""
    import torch
    from hpbandster_amd import kde
    D = X.shape[1]
    n0 = X.shape[0] - reps - 1
    store = kde.ObservationStore(D, var_type, device=device, capacity=2 * X.shape[0])
    store.add(X[:n0], losses[:n0])
    store.refit(D + 1)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    gpu_ms = []
    t0 = time.perf_counter()
    for r in range(reps):
        store.add(X[n0 + r], losses[n0 + r])
        e0.record()
        store.refit(D + 1)  # ends with a stream synchronisation: e1 below is already complete when read
        e1.record()
        e1.synchronize()
        gpu_ms.append(e0.elapsed_time(e1))
    inc_ms = (time.perf_counter() - t0) / reps * 1e3
    kde.fit_pair(X, losses, var_type, D + 1, device=device)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        kde.fit_pair(X, losses, var_type, D + 1, device=device)
    full_ms = (time.perf_counter() - t0) / 5 * 1e3
    ng, nb = kde.bohb_split_sizes(X.shape[0], D + 1)
    t0 = time.perf_counter()
    for _ in range(reps):
        idx = np.argsort(losses)
        for rows, n in ((idx[:ng], ng), (idx[-nb:], nb)):
            data = X[rows]
            bw = 1.06 * np.std(data, axis=0) * n ** (-1. / (4 + D))
            lev = [np.unique(data[:, d]).size for d in range(D) if var_type[d] == "u"]
    host_ms = (time.perf_counter() - t0) / reps * 1e3
    return {"workload": "bohb_refit_obs%d_d%d" % X.shape, "ms_per_refit": inc_ms, "host_numpy_ms": host_ms,
            "ms_per_refit_host_arrays": full_ms,
            "stream_ms_median": float(np.median(gpu_ms)),
            "stream_ms_note": "events bracketing store.refit on its stream: the kernels plus the host's enqueue gaps "
                              "(wall clock ms_per_refit adds add(), allocation and the read-back)",
            "note": "wall clock per new_result refit: one row appended in HBM, one hbx_kde_refit_sync (its output block published to mapped host memory); "
                    "host_arrays = every row uploaded"}


def cv_line(device, n=4096, D=8, reps=5):
    """Side measurement: the cv_ls objective of KernelDensityEstimator's fit
    (KDEMultivariate.imse, fp64 in the reference's operation order) at n observations: 2 n^2 pair
    terms (convolution F and leave-one-out L) per evaluation, one hbx_kde_cv_terms launch; plus a whole
    Nelder-Mead bandwidth selection.  Synthetic U[0,1) data, D continuous dims."""
    import torch
    from hpbandster_amd.cv import CVObjective
    X = np.random.RandomState(5).rand(n, D)
    obj = CVObjective(X, "c" * D, device=device)
    h0 = obj.normal_reference()
    obj.imse(h0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(reps):
        obj.imse(h0 * (1 + 0.01 * k))
    ms = (time.perf_counter() - t0) / reps * 1e3
    e0 = obj.evals
    t0 = time.perf_counter()
    obj.select("cv_ls")
    sel = time.perf_counter() - t0
    return {"workload": "cv_ls_imse_obs%d_d%d" % (n, D), "ms_per_eval": ms,
            "pair_terms_per_s": 2 * n * n / (ms * 1e-3), "select_s": sel, "select_evals": obj.evals - e0,
            "dtype": "f64"}


def sampler_line(pair, device, dc, du, levels, Nc, ws, reps=10):
    """Side measurement: BOHB's candidate rule for Nc candidates drawn on the GPU
    (Philox + truncnorm inversion), alone and followed by the acquisition -- a whole model-based
    get_config at Nc candidates.  HBM roofline of the sampler: 8 B written per (candidate, dim)."""
    import torch
    from hpbandster_amd import kde
    lv = np.array([0] * dc + [levels] * du)
    D = dc + du

    def samp(k):
        return pair.good.sample(lv, 3.0, Nc, seed=1234, counter_base=k * Nc)[0]

    samp(0)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for k in range(reps):
        samp(k + 1)
    e1.record()
    torch.cuda.synchronize()
    ms_call = e0.elapsed_time(e1) / reps  # the Python call per launch (allocations, argument checks): host-bound
    # the launch itself: back-to-back native calls into kept output buffers with their arguments built once, so
    # the host enqueues far faster than the kernel runs and the events bracket kernel time (and the 1-byte-per-
    # candidate flag memset each launch does)
    from hpbandster_amd import _native as N
    g = pair.good
    L = N.lib()
    out = (torch.empty((Nc, D), dtype=torch.float64, device=device), torch.empty(Nc, dtype=torch.int64, device=device),
           torch.empty(Nc, dtype=torch.uint8, device=device))
    g.sample(lv, 3.0, Nc, seed=1234, counter_base=0, out=out)  # the levels on the device, the Phi table built
    fixed = (g.X_dev.data_ptr(), D, g.rows_dev.data_ptr(), g.nobs,
             g.params.data_ptr() + int(L.hbx_kde_param_bw_offset()), g._lv_dev.data_ptr(),
             g._tab.data_ptr() if getattr(g, "_tab", None) is not None else None, 3.0, 1234)
    tail = (Nc, out[0].data_ptr(), out[1].data_ptr(), out[2].data_ptr(), N.stream_handle(None, device))
    fn = L.hbx_kde_sample
    torch.cuda.synchronize()
    nl = 4 * reps
    e0.record()
    for k in range(nl):
        fn(*fixed, (k + 1) * Nc, 0, *tail)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / nl
    t0 = time.perf_counter()
    for k in range(reps):
        r = pair.acquire(samp(k + 100), workspace=ws)
    torch.cuda.synchronize()
    ms_e2e = (time.perf_counter() - t0) / reps * 1e3
    # the acquisition alone on BOHB-distributed candidates (around the good observations, bohb.py:133-147):
    # its scoring launch and how many candidates the exact re-score takes (data dependent)
    ev = kde.ScoreEvents()
    C = samp(7)
    pair.acquire(C, workspace=ws, events=ev)
    launch, shortlists = [], []
    for k in range(reps):
        rr = pair.acquire(C, workspace=ws, events=ev)
        ml, mg = ev.elapsed_ms(True)
        launch.append(ml)
        shortlists.append(rr.shortlist)
    gbs = Nc * D * 8 / (ms * 1e-3) / 1e9
    return {"workload": "gpu_sampler_cand%d_d%d" % (Nc, D), "ms_per_launch": ms,
            "ms_per_python_call": ms_call, "timing": "ms_per_launch: events around %d back-to-back native launches "
            "(flag memset + kernel) into kept buffers; ms_per_python_call: the same around DeviceKDE.sample calls "
            "(host-bound: allocations and argument handling per call)" % nl,
            "candidates_per_s": Nc / (ms * 1e-3),
            "roofline": {"bound": "hbm", "achieved": gbs, "peak": 8000.0, "unit": "GB/s", "frac": gbs / 8000.0,
                         "bytes_per_element": 8},
            "ms_sample_plus_acquire": ms_e2e, "last_winner": r.index,
            "bohb_distributed_acquisition": {"pair_launch_ms_median": float(np.median(launch)),
                                             "shortlist": int(np.max(shortlists)), "winner": rr.index}}


def kde_result_bytes():
    from hpbandster_amd import kde
    return kde.RESULT_BYTES


PROFILE_SET = "profiles/r06/final4"


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


def load_clock(workload):
    """Effective engine clock under the scoring kernel (GRBM_GUI_ACTIVE / 8 / duration) from the
    committed PMC record of this workload (tools/profile_round.sh), else None."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(p) as fh:
            d = json.load(fh)
        if d.get("workload") == workload:
            return d.get("clock_ghz")
    except (OSError, ValueError):
        pass
    return None


def main():
    a = parse()
    # before anything touches the GPU: N ranks however bench.py was started
    how, what = plan_launch(a.gpus, os.environ, sys.argv[1:], os.path.abspath(__file__))
    if how == "error":
        log("error: " + what)
        sys.exit(2)
    if how == "spawn":
        import subprocess
        log("launching %d ranks: %s" % (a.gpus, " ".join(what)))
        env = dict(os.environ)
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        env["HBX_BENCH_SPAWNED"] = "1"
        sys.exit(subprocess.call(what, env=env))
    world = what
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.launch_check:
        print(json.dumps({"rank": rank, "world": world, "local_rank": local,
                          "spawned": os.environ.get("HBX_BENCH_SPAWNED") == "1"}), flush=True)
        return
    import torch
    import torch.distributed as dist
    from hpbandster_amd import kde
    from hpbandster_amd import synthetic as S

    # one process per GPU; --share-gpu maps every rank onto the visible devices round-robin (rehearsal
    # of the multi-process path on a 1-GPU box, with --backend gloo: RCCL refuses two ranks per GPU)
    ndev = torch.cuda.device_count()
    if not a.share_gpu and local >= ndev:
        log("error: rank %d needs GPU %d but %d are visible (--share-gpu rehearses several ranks on one)"
            % (rank, local, ndev))
        sys.exit(2)
    dev_idx = local % ndev if a.share_gpu else local
    torch.cuda.set_device(dev_idx)
    device = torch.device("cuda", dev_idx)
    comm_dev = device if a.backend == "nccl" else torch.device("cpu")
    if world > 1:
        if a.backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group(a.backend)

    D = a.dc + a.du
    var_type = S.var_type_string(a.dc, a.du)
    X = S.make_observations(a.obs, a.dc, a.du, a.levels)
    losses = S.make_losses(a.obs)
    pair = kde.fit_pair(X, losses, var_type, D + 1, device=device)
    Ng, Nb = pair.good.nobs, pair.bad.nobs
    from hpbandster_amd.distributed import shard_range
    if a.total_candidates:  # strong scaling: this rank's contiguous shard of ONE seeded set, global indices
        lo, hi = shard_range(a.total_candidates, rank, world)
        Nc, base = hi - lo, lo
    else:  # weak: rank r scores rows [r Nc, (r+1) Nc) of the stream -- at N ranks the first N Nc rows
        Nc, base = a.candidates, rank * a.candidates
    cands = S.make_candidates_blocked(base, base + Nc, a.dc, a.du, a.levels)
    c_dev = torch.from_numpy(cands).to(device)
    ws = torch.empty(pair.workspace_bytes(Nc), dtype=torch.uint8, device=device)
    ev = kde.ScoreEvents()
    # l and g in one launch of the pair kernel (hbx_kde.hip launch_score2): same hmode instance for both
    # KDEs, not switched off
    fused = (kernel_model(pair.bad, a.dc, a.du)["model"] is not None and pair.good.variant == pair.bad.variant
             and os.environ.get("HBX_SCORE_PAIR", "1") != "0")
    log("rank %d/%d: %d candidates x (%d + %d) observations, D=%d" % (rank, world, Nc, Ng, Nb, D))

    xchg = None
    if world > 1:  # one collective per step: RCCL all-gather of the 48-byte records + device reduction
        from hpbandster_amd.distributed import WinnerExchange
        try:
            xchg = WinnerExchange(device, transport="rccl" if a.backend == "nccl" else "records")
        except Exception as e:  # libhbx's communicator refused: the same exchange on torch's process group
            if a.backend != "nccl":
                raise
            log("rank %d: hbx_rccl_comm_init failed (%r): exchanging the records on torch's nccl group" % (rank, e))
            xchg = WinnerExchange(device, transport="torch")

    def step(ev):
        if xchg is None:  # one rank: the acquisition's record reaches the host in the same native call
            r = pair.acquire(c_dev, index_base=base, workspace=ws, events=ev)
            return r.index, r.score
        rv = pair.acquire(c_dev, index_base=base, workspace=ws, sync=False, events=ev)
        rv = xchg.exchange(rv)
        # the winner reaches the host (what BOHB needs); the exact scores are the pinned reference's
        # float64 values bit for bit, so the (score, index) reduction is the reference's pick
        r = kde.AcqResult.from_bytes(kde.fetch_bytes(rv))
        return r.index, r.score

    for _ in range(a.warmup):
        step(ev)
    # every timed step stamps its scoring launch with its own events, read after the timed region (the
    # reads are measurement, not part of a step)
    evs = [kde.ScoreEvents() for _ in range(a.steps)]
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    winner = None
    for s in range(a.steps):
        winner = step(evs[s])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    t_l = t_g = 0.0
    launch_ms = []  # the scoring launch of every timed step (HIP events on its stream)
    for e in evs:
        ml, mg = e.elapsed_ms(fused)
        t_l += ml
        t_g += mg
        launch_ms.append(ml + mg)
    last = kde.AcqResult.from_bytes(ws[int(pair.result_offset()):int(pair.result_offset()) + kde.RESULT_BYTES]
                                    .cpu().numpy().tobytes())
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=comm_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    pairs_step = (a.total_candidates if a.total_candidates else world * Nc) * (Ng + Nb)
    value = pairs_step * a.steps / el
    W = 3 * a.dc + 2 * a.du + 4
    avg_l, avg_g = t_l / a.steps, t_g / a.steps
    kernel_rate = Nc * (Ng + Nb) / ((avg_l + avg_g) * 1e-3)  # pairs/s inside the scoring launches
    achieved = W * kernel_rate / 1e12
    workload = "kde_acquisition_d%d_%dc%du_obs%d_cand%d" % (D, a.dc, a.du, a.obs, Nc)
    if a.total_candidates:
        workload = "kde_acquisition_d%d_%dc%du_obs%d_total%d_sharded" % (D, a.dc, a.du, a.obs, a.total_candidates)
    traffic = load_traffic(workload)
    km = kernel_model(pair.bad, a.dc, a.du)
    if fused:
        km["kernel"] = km["kernel"].replace("_kernel<", "_pair_kernel<")
    mfma_util = issue_bound = None
    if km["model"]:
        m = km["model"]
        mfma_tf = kernel_rate * m["dense_equiv_flops_per_pair"] / 1e12
        mfma_util = {"achieved": mfma_tf, "peak": PEAK_F16_MFMA_TFLOPS, "unit": "TFLOP/s",
                     "frac": mfma_tf / PEAK_F16_MFMA_TFLOPS,
                     "flops_per_pair": m["dense_equiv_flops_per_pair"],
                     "note": "dense-equivalent f16 matrix-core work of the formulation the kernel runs"}
        peak_pairs = N_SIMD * CLOCK_GHZ * 1e9 * 256 / m["bound_cycles"]
        issue_bound = dict(m, clock_ghz=CLOCK_GHZ, peak_pairs_per_s=peak_pairs, achieved_pairs_per_s=kernel_rate,
                           frac=kernel_rate / peak_pairs)
        clk = load_clock(workload)
        if clk:  # the same model at the clock the chip was measured to hold under this kernel
            issue_bound["measured_clock_ghz"] = clk
            issue_bound["frac_at_measured_clock"] = kernel_rate / (N_SIMD * clk * 1e9 * 256 / m["bound_cycles"])
    out = {
        "metric": METRIC, "value": value, "unit": "pairs/s", "n_gpus": world, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": el / a.steps * 1e3, "higher_is_better": True,
        "scaling": "strong" if a.total_candidates else "weak",
        "vs_baseline": None,
        "dtype": ("f16 MFMA coarse pre-screen (1 product per dim, rigorous bound), f32 accumulate, f64 re-score"
                  if (pair.bad.variant >> 7) & 1 else "f16 hi/lo MFMA (3 products per dim), f32 accumulate, f64 re-score"),
        "data": "synthetic",
        "config": {"workload": workload, "candidates_per_gpu": Nc,
                   "total_candidates": a.total_candidates or world * Nc, "observations": a.obs, "n_good": Ng,
                   "n_bad": Nb, "dims": "%dc+%du" % (a.dc, a.du), "levels": a.levels,
                   "parallelism": ("one GPU, no collective (the final argmin kernel publishes the record to the host)"
                                   if world == 1 else "candidate-sharded x%d, %s" % (
                       world, "one collective per step: hbx_argmax_allreduce (RCCL all-gather of result records)"
                       if xchg.transport == "rccl" else
                       "one collective per step: all_gather of the device records on torch's nccl group (RCCL)"
                       if xchg.transport == "torch" else "gloo all_gather of result records (rehearsal)")),
                   "winner": winner[0], "shortlist": last.shortlist,
                   "candidates": "rows [%d, %d) of synthetic.make_candidates_blocked (seed 3) per rank, the first %d "
                                 "rows in all" % (base, base + Nc, pairs_step // (Ng + Nb)),
                   "world_size_rccl": xchg.rccl_world_size() if xchg is not None else None,
                   "launcher": ("bench.py -> torch.distributed.run" if os.environ.get("HBX_BENCH_SPAWNED") == "1"
                                else "torch.distributed.run" if "WORLD_SIZE" in os.environ else "single process")},
        # the kernel runs on the f16 matrix cores: priced against their dense peak (no sparsity
        # credit), with SURVEY 8d's algorithmic W flops per pair; the formulation's own matrix work and
        # the VALU-basis figure SURVEY 8d first proposed are reported beside it
        "roofline": {"bound": "mfma", "achieved": achieved, "peak": PEAK_F16_MFMA_TFLOPS, "unit": "TFLOP/s",
                     "frac": achieved / PEAK_F16_MFMA_TFLOPS, "traffic": traffic,
                     "traffic_source": ("carried, not counted in this run: HBM bytes per launch from the committed PMC "
                                        "record of this workload (profiles/pmc_traffic.json: rocprofv3 --pmc "
                                        "FETCH_SIZE / WRITE_SIZE passes, tools/profile_round.sh)") if traffic else None,
                     "valu_basis": {"peak": PEAK_FP32_TFLOPS, "frac": achieved / PEAK_FP32_TFLOPS},
                     "kernel": km["kernel"] + (" (l and g in one launch)" if fused else " (l and g launches)"),
                     "flops_per_pair": W,
                     "basis": "SURVEY 8d: W = 3 Dc + 2 Du + 4 algorithmic flops per pair x pairs per launch / "
                              "launch time vs the dense f16 MFMA peak; the exact hi/lo f16 formulation does "
                              "%s dense-equivalent flops per pair (mfma_util); vs the fp32 VALU peak "
                              "(valu_basis) frac > 1" % (km["model"] or {}).get("dense_equiv_flops_per_pair", "-"),
                     "ms_per_launch": ({"l+g": avg_l + avg_g, "pairs_per_launch": Nc * (Ng + Nb)} if fused else
                                       {"l": avg_l, "g": avg_g, "mean": (avg_l + avg_g) / 2}),
                     # every timed step's launch: what rocprofv3's kernel trace of the same run must show
                     "launch_ms_stats": {"mean": float(np.mean(launch_ms)), "median": float(np.median(launch_ms)),
                                         "min": float(np.min(launch_ms)), "max": float(np.max(launch_ms)),
                                         "samples": len(launch_ms),
                                         "timing": "HIP events on the launch stream around the scoring launch(es) "
                                                   "of each timed step"},
                     # the committed same-session set for this workload (bench line + the same bench under
                     # rocprofv3 + PMC passes: tools/profile_round.sh); traffic and measured clock come
                     # from its pmc_traffic.json (copied to profiles/pmc_traffic.json)
                     "profiles": a.profile_tag or PROFILE_SET,
                     "mfma_util": mfma_util, "issue_bound": issue_bound},
        "cpu_baseline": None,
    }
    chk = winner_check(pinned_prefix(pairs_step // (Ng + Nb), a.dc, a.du, a.levels, a.obs), winner[0], winner[1],
                       last.pdf_l if world == 1 else None, last.pdf_g if world == 1 else None)
    out["config"].update(chk or {"winner_ok": None, "pinned_by": "no pinned winner for this workload"})
    if world > 1 and a.strong_total and not a.total_candidates:
        try:  # config #4 beside the weak line: the same total at every N (strong scaling)
            out["strong_config4"] = strong_line(pair, device, a, rank, world, dist, xchg)
        except Exception as e:
            out["strong_config4"] = {"error": repr(e)}
    if not a.no_config5:  # every rank promotes its share of the brackets
        try:
            out["config5"] = config5(device, rank=rank, world=world, dist=dist if world > 1 else None)
        except Exception as e:  # a side measurement; report why it is missing
            out["config5"] = {"error": repr(e)}
    if rank == 0 and not a.no_config5:
        try:
            out["promote_dropin"] = promote_dropin(device)
            out["promote_dropin_n81"] = promote_dropin(device, n=81)
        except Exception as e:
            out["promote_dropin"] = {"error": repr(e)}
        if world == 1:
            try:
                out["config4_single_gpu"] = config4_line(pair, device, a.dc, a.du, a.levels)
            except Exception as e:
                out["config4_single_gpu"] = {"error": repr(e)}
        try:
            out["batched_acquisition"] = batched(pair, device, a.dc, a.du, a.levels)
        except Exception as e:
            out["batched_acquisition"] = {"error": repr(e)}
        try:
            out["sh_stage"] = sh_stage_line(device)
        except Exception as e:
            out["sh_stage"] = {"error": repr(e)}
        try:  # HpBandSter.run with 8 threaded zero-cost workers, results on the dispatcher thread
            out["threaded_run"] = threaded_run_line(device)
        except Exception as e:
            out["threaded_run"] = {"error": repr(e)}
        try:
            out["sh_stage_interleaved"] = sh_stage_line(device, interleaved=True, reps=7)
        except Exception as e:
            out["sh_stage_interleaved"] = {"error": repr(e)}
        try:  # the default drop-in's get_config (host sampler) against the per-element draws
            out["get_config_default"] = get_config_line(device)
        except Exception as e:
            out["get_config_default"] = {"error": repr(e)}
        try:  # one worker with the default (host) sampler at default sizes: request, result, refit
            out["sh_stage_interleaved_host_sampler"] = sh_stage_line(device, n_obs=400, stage=81, reps=3,
                                                                     interleaved=True, sampler="host")
        except Exception as e:
            out["sh_stage_interleaved_host_sampler"] = {"error": repr(e)}
        try:
            out["gpu_sampler"] = sampler_line(pair, device, a.dc, a.du, a.levels, Nc, ws)
        except Exception as e:
            out["gpu_sampler"] = {"error": repr(e)}
        try:
            out["precise_logpdf"] = precise_line(pair, c_dev, device)
        except Exception as e:
            out["precise_logpdf"] = {"error": repr(e)}
        try:
            out["config2"] = config2_line(device)
        except Exception as e:
            out["config2"] = {"error": repr(e)}
        try:
            out["refit"] = refit_line(X, losses, var_type, device)
        except Exception as e:
            out["refit"] = {"error": repr(e)}
        try:
            out["cv_objective"] = cv_line(device)
        except Exception as e:
            out["cv_objective"] = {"error": repr(e)}
    if rank == 0 and world == 1 and not a.no_cpu:
        try:
            out["cpu_baseline"] = cpu_baseline(X, pair.good.rows_dev.cpu().numpy(), pair.bad.rows_dev.cpu().numpy(),
                                               pair, var_type,
                                               cands,
                                               a.cpu_seconds)
        except Exception as e:  # the baseline is a side measurement; report why it is missing
            out["cpu_baseline"] = {"error": repr(e)}
        try:
            out["cpu_baseline"]["reference_loop"] = reference_loop_baseline(device)
        except Exception as e:
            out["cpu_baseline"]["reference_loop"] = {"error": repr(e)}
        if isinstance(out.get("precise_logpdf"), dict) and "error" not in out["precise_logpdf"]:
            try:
                out["precise_logpdf"]["oracle_check"] = logpdf_oracle_check()
            except Exception as e:
                out["precise_logpdf"]["oracle_check"] = {"error": repr(e)}
    if world > 1:
        out["cpu_baseline_note"] = ("the CPU baseline is measured on rank 0 at N=1 only (bench contract): see that "
                                    "line's cpu_baseline")
    if rank == 0:
        print(json.dumps(out), flush=True)
    if xchg is not None:
        xchg.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
