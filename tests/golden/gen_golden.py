#!/opt/conda/bin/python3.9 -B
"""Generate the golden fixtures under tests/golden/ from the reference itself.

Run ONLY in the build container, where /root/reference and the oracle interpreter exist:

    PYTHONDONTWRITEBYTECODE=1 /opt/conda/bin/python3.9 -B tests/golden/gen_golden.py

What runs here (and nowhere else):
  * the reference's own ``hpbandster/config_generators/bohb.py``, ``kde_ei.py``,
    ``HB_iteration.py``, ``HB_master.py`` and ``HB_result.py``, loaded by file path;
  * statsmodels 0.12.2 ``KDEMultivariate`` (the third-party arithmetic BOHB calls,
    ``bohb.py:245-246``), scipy 1.7.1 ``truncnorm`` and numpy 1.26.4.

Shims: ``ConfigSpace`` is absent, so ``hpbandster_amd/configspace.py``
is registered under that name; ``statsmodels.api`` is broken in this interpreter, so a stub
exposing ``nonparametric.KDEMultivariate`` is registered; ``hpbandster.distributed.dispatcher``
imports Pyro4 (absent), so a synchronous in-process dispatcher stands in for it.  Nothing from
the reference is copied into the repository: only inputs/outputs (npz/json data) are written.
"""

import importlib.util
import json
import os
import sys
import time
import types
import warnings

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"

warnings.filterwarnings("ignore")


def _load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def load_reference():
    if not os.path.isdir(os.path.join(REF, "hpbandster")):
        raise SystemExit("gen_golden.py needs the reference at %s (build container only)" % REF)
    sys.dont_write_bytecode = True

    cs = _load("ConfigSpace", os.path.join(REPO, "hpbandster_amd", "configspace.py"))
    synth = _load("hbx_synthetic", os.path.join(REPO, "hpbandster_amd", "synthetic.py"))

    import statsmodels
    from statsmodels.nonparametric.kernel_density import KDEMultivariate
    sm_api = types.ModuleType("statsmodels.api")
    sm_api.nonparametric = types.SimpleNamespace(KDEMultivariate=KDEMultivariate)
    sys.modules["statsmodels.api"] = sm_api
    statsmodels.api = sm_api

    root = os.path.join(REF, "hpbandster")
    for pkg, sub in (("hpbandster", ""), ("hpbandster.config_generators", "config_generators"),
                     ("hpbandster.distributed", "distributed")):
        m = types.ModuleType(pkg)
        m.__path__ = [os.path.join(root, sub)] if sub else [root]
        sys.modules[pkg] = m

    disp = types.ModuleType("hpbandster.distributed.dispatcher")

    class Job(object):
        """Field-compatible with the reference Job (dispatcher.py:9-32)."""

        def __init__(self, id, *args, **kwargs):
            self.id = id
            self.args = args
            self.kwargs = kwargs
            self.timestamps = {}
            self.result = None
            self.exception = None
            self.worker_name = None

        def time_it(self, which):
            self.timestamps[which] = time.time()

    class SyncDispatcher(object):
        """Runs every submitted job immediately and calls back synchronously."""
        compute = None

        def __init__(self, new_result_callback, queue_callback=None, **kwargs):
            self.new_result_callback = new_result_callback

        def run(self):
            return

        def number_of_workers(self):
            return 1

        def shutdown(self, shutdown_workers=False):
            return

        def submit_job(self, id, **kwargs):
            job = Job(id, **kwargs)
            job.time_it("submitted")
            job.time_it("started")
            res = SyncDispatcher.compute(kwargs["config"], kwargs["budget"])
            job.time_it("finished")
            if res is None:
                job.exception = "RuntimeError: simulated failure"
            else:
                job.result = res
            self.new_result_callback(job)
            return job

    disp.Job = Job
    disp.Dispatcher = SyncDispatcher
    sys.modules["hpbandster.distributed.dispatcher"] = disp

    ref = types.SimpleNamespace()
    ref.utils = _load("hpbandster.utils", os.path.join(root, "utils.py"))
    ref.base = _load("hpbandster.config_generators.base", os.path.join(root, "config_generators", "base.py"))
    ref.bohb = _load("hpbandster.config_generators.bohb", os.path.join(root, "config_generators", "bohb.py"))
    ref.kde_ei = _load("hpbandster.config_generators.kde_ei", os.path.join(root, "config_generators", "kde_ei.py"))
    ref.HB_iteration = _load("hpbandster.HB_iteration", os.path.join(root, "HB_iteration.py"))
    ref.HB_result = _load("hpbandster.HB_result", os.path.join(root, "HB_result.py"))
    ref.HB_master = _load("hpbandster.HB_master", os.path.join(root, "HB_master.py"))
    ref.Job = Job
    ref.SyncDispatcher = SyncDispatcher
    ref.cs = cs
    ref.synth = synth
    ref.KDEMultivariate = KDEMultivariate
    return ref


# ----------------------------------------------------------------------------------------
# helpers


def make_space(cs, dc, du, levels):
    """x00.. continuous in [0,1], y00.. categorical with integer choices (sorted: x* then y*)."""
    space = cs.ConfigurationSpace(seed=11)
    lv = [levels] * du if np.isscalar(levels) else list(levels)
    for d in range(dc):
        space.add_hyperparameter(cs.UniformFloatHyperparameter("x%02d" % d, 0.0, 1.0))
    for d in range(du):
        space.add_hyperparameter(cs.CategoricalHyperparameter("y%02d" % d, list(range(lv[d]))))
    return space


def vec_to_dict(space, cs, vec):
    return cs.Configuration(space, vector=vec).get_dictionary()


def py_score(l, g):
    """bohb.py:129 minimize_me, with Python max() semantics (NaN asymmetry)."""
    return max(1e-8, g) / max(l, 1e-8)


def py_argmin(scores):
    """bohb.py:150-152: strict <, best starts at +inf, first index wins."""
    best, best_i = np.inf, -1
    for i, v in enumerate(scores):
        if v < best:
            best, best_i = v, i
    return best_i


def fit_through_bohb(ref, X, losses, dc, du, levels, crashed=None, top_n_percent=15):
    """Feed every row through the reference BOHB.new_result (one budget) and return the model."""
    space = make_space(ref.cs, dc, du, levels)
    cg = ref.bohb.BOHB(space, top_n_percent=top_n_percent)
    for i in range(X.shape[0]):
        job = ref.Job((0, 0, i), config=vec_to_dict(space, ref.cs, X[i]), budget=1.0)
        if crashed is not None and crashed[i]:
            job.result = None
            job.exception = "crash"
        else:
            job.result = {"loss": float(losses[i]), "info": None}
        cg.new_result(job)
    return space, cg


def kde_case(ref, name, X, losses, cands, dc, du, levels, crashed=None, store_inputs=True, extra=None):
    space, cg = fit_through_bohb(ref, X, losses, dc, du, levels, crashed)
    model = cg.kde_models[1.0]
    good, bad = model["good"], model["bad"]
    vt = cg.kde_vartypes
    assert vt == "c" * dc + "u" * du, vt

    # recover the row order of good/bad data (bohb.py:229-232) and check it
    eff_losses = np.where(crashed, np.inf, losses) if crashed is not None else losses
    idx = np.argsort(eff_losses)
    n = X.shape[0]
    n_good, n_bad = ref.synth.bohb_split_sizes(n, cg.min_points_in_model)
    good_idx, bad_idx = idx[:n_good], idx[-n_bad:]
    assert np.array_equal(good.data, X[good_idx]), name
    assert np.array_equal(bad.data, X[bad_idx]), name

    nlev_good = np.array([np.unique(good.data[:, d]).size if vt[d] == "u" else 0 for d in range(len(vt))])
    nlev_bad = np.array([np.unique(bad.data[:, d]).size if vt[d] == "u" else 0 for d in range(len(vt))])

    pdf_l = np.atleast_1d(good.pdf(cands)).astype(np.float64)
    pdf_g = np.atleast_1d(bad.pdf(cands)).astype(np.float64)
    # per-candidate calls as bohb.py:149 makes them, must agree bit for bit
    for i in range(min(16, cands.shape[0])):
        lv, gv = good.pdf(list(cands[i])), bad.pdf(list(cands[i]))
        assert (lv == pdf_l[i]) or (np.isnan(lv) and np.isnan(pdf_l[i])), name
        assert (gv == pdf_g[i]) or (np.isnan(gv) and np.isnan(pdf_g[i])), name
    scores = np.array([py_score(l, g) for l, g in zip(pdf_l, pdf_g)])
    chosen = py_argmin(scores)

    out = dict(
        dc=dc, du=du, levels=np.atleast_1d(levels), var_type=np.array(vt),
        n_obs=n, min_points=cg.min_points_in_model,
        good_idx=good_idx.astype(np.int64), bad_idx=bad_idx.astype(np.int64),
        bw_good=np.asarray(good.bw, dtype=np.float64), bw_bad=np.asarray(bad.bw, dtype=np.float64),
        nlev_good=nlev_good, nlev_bad=nlev_bad,
        pdf_l=pdf_l, pdf_g=pdf_g, scores=scores, chosen=np.int64(chosen),
        sha_X=np.array(ref.synth.sha256_array(X)), sha_losses=np.array(ref.synth.sha256_array(losses)),
        sha_cands=np.array(ref.synth.sha256_array(cands)),
    )
    if crashed is not None:
        out["crashed"] = crashed.astype(np.bool_)
    if store_inputs:
        out.update(X=X, losses=losses, cands=cands)
    if extra:
        out.update(extra)
    path = os.path.join(HERE, "kde_%s.npz" % name)
    np.savez_compressed(path, **out)
    print("wrote %s  n=%d D=%d Nc=%d chosen=%d  nan(l)=%d nan(g)=%d zero(l)=%d" % (
        os.path.basename(path), n, dc + du, cands.shape[0], chosen,
        np.isnan(pdf_l).sum(), np.isnan(pdf_g).sum(), (pdf_l == 0).sum()))


def gen_kde_cases(ref):
    S = ref.synth
    # config #1 shape: toy function, D=1
    X = S.make_observations(40, 1, 0, 2); L = S.make_losses(40); C = S.make_candidates(64, 1, 0, 2)
    kde_case(ref, "d1", X, L, C, 1, 0, 2)

    # config #2 shape: D=8 continuous, 1e3 observations (1e3-candidate slice of 1e5)
    X = S.make_observations(1000, 8, 0, 2); L = S.make_losses(1000); C = S.make_candidates(1000, 8, 0, 2)
    kde_case(ref, "d8c", X, L, C, 8, 0, 2, store_inputs=False)

    # config #3 shape: D=32 (24c + 8u, L=4), 1e4 observations (256-candidate slice)
    X = S.make_observations(10000, 24, 8, 4); L = S.make_losses(10000); C = S.make_candidates(256, 24, 8, 4)
    kde_case(ref, "d32m", X, L, C, 24, 8, 4, store_inputs=False)

    # mixed levels, a few crashed runs (loss=+inf, bohb.py:189-192)
    X = S.make_observations(300, 5, 3, [2, 3, 5]); L = S.make_losses(300)
    crashed = np.random.RandomState(7).rand(300) < 0.05
    C = S.make_candidates(500, 5, 3, [2, 3, 5])
    kde_case(ref, "mixed8", X, L, C, 5, 3, [2, 3, 5], crashed=crashed)

    # categorical bandwidth > 1 -> negative Aitchison-Aitken match weight (hard part 2)
    X = S.make_observations(40, 2, 3, 10); L = S.make_losses(40); C = S.make_candidates(400, 2, 3, 10)
    # candidates that copy observed categories so matches actually occur
    C[:200, 2:] = X[np.random.RandomState(9).randint(0, 40, 200)][:, 2:]
    kde_case(ref, "hgt1", X, L, C, 2, 3, 10)

    # constant categorical column in the data: h=0, mismatch -> 0/0 = NaN
    X = S.make_observations(60, 3, 2, 4); X[:, 3] = 2.0
    L = S.make_losses(60); C = S.make_candidates(300, 3, 2, 4)
    kde_case(ref, "constcat", X, L, C, 3, 2, 4)

    # constant continuous column: bw=0 -> every pdf NaN -> no model-based pick
    X = S.make_observations(50, 3, 1, 3); X[:, 1] = 0.25
    L = S.make_losses(50); C = S.make_candidates(100, 3, 1, 3)
    kde_case(ref, "constcont", X, L, C, 3, 1, 3)

    # tight clusters + spread candidates: far candidates underflow to pdf=0 in fp64
    rs = np.random.RandomState(21)
    X = 0.5 + 1e-3 * rs.rand(80, 6); L = S.make_losses(80)
    C = rs.rand(400, 6); C[:20] = X[:20] + 1e-4 * rs.rand(20, 6)
    kde_case(ref, "far", X, L, C, 6, 0, 2)

    # duplicated candidates: exact score ties -> first index wins (strict <)
    X = S.make_observations(120, 4, 2, 3); L = S.make_losses(120)
    C0 = S.make_candidates(50, 4, 2, 3)
    C = np.vstack([C0, C0[::-1], C0])
    kde_case(ref, "dups", X, L, C, 4, 2, 3)

    # categorical-only space: many exact ties
    X = S.make_observations(100, 0, 4, 3); L = S.make_losses(100); C = S.make_candidates(300, 0, 4, 3)
    kde_case(ref, "catonly", X, L, C, 0, 4, 3)


# ----------------------------------------------------------------------------------------
# near ties: candidates whose reference scores differ from the best one by a few ulps (the GPU's fp64
# exp and numpy's may order them differently -- the engine must re-resolve them in numpy's arithmetic)


def near_tie_candidates(ref, X, L, base, dc, du, levels, seed, max_ulps):
    """base candidates + copies of the reference's best one with continuous coordinates moved by
    1..max_ulps ulps (and exact duplicates), shuffled so copies sit before and after it."""
    space, cg = fit_through_bohb(ref, X, L, dc, du, levels)
    model = cg.kde_models[1.0]
    l = np.atleast_1d(model["good"].pdf(base))
    g = np.atleast_1d(model["bad"].pdf(base))
    best = py_argmin([py_score(a, b) for a, b in zip(l, g)])
    rs = np.random.RandomState(seed)
    copies = []
    for k in range(48):
        c = base[best].copy()
        if k % 8 != 0:  # every 8th copy is an exact duplicate
            for _ in range(1 + k % 3):
                d = rs.randint(dc)
                for _ in range(rs.randint(1, max_ulps + 1)):
                    c[d] = np.nextafter(c[d], np.inf if rs.rand() < 0.5 else -np.inf)
        copies.append(c)
    C = np.vstack([base, np.array(copies)])
    return C[rs.permutation(C.shape[0])]


def gen_neartie_cases(ref):
    S = ref.synth
    X = S.make_observations(300, 8, 0, 2); L = S.make_losses(300); B = S.make_candidates(200, 8, 0, 2)
    kde_case(ref, "neartie_c", X, L, near_tie_candidates(ref, X, L, B, 8, 0, 2, 61, 2), 8, 0, 2)
    X = S.make_observations(400, 5, 3, [2, 3, 4]); L = S.make_losses(400); B = S.make_candidates(200, 5, 3, [2, 3, 4])
    kde_case(ref, "neartie_m", X, L, near_tie_candidates(ref, X, L, B, 5, 3, [2, 3, 4], 62, 40), 5, 3, [2, 3, 4])


# ----------------------------------------------------------------------------------------
# get_config: the reference's own sampler + selection, recording every candidate it scored


class _PdfRecorder(object):
    def __init__(self, kde, sink):
        self._kde = kde
        self._sink = sink

    def __getattr__(self, k):
        return getattr(self._kde, k)

    def pdf(self, x):
        v = self._kde.pdf(x)
        self._sink.append((np.array(x, dtype=np.float64), float(v)))
        return v


def gen_get_config(ref, cases=None):
    S = ref.synth
    if cases is None:
        cases = [("d8c", 8, 0, 2, 200), ("mixed", 5, 3, [2, 3, 5], 150), ("hgt1", 2, 3, 10, 40)]
    for name, dc, du, lv, n in cases:
        X = S.make_observations(n, dc, du, lv)
        L = S.make_losses(n)
        space, cg = fit_through_bohb(ref, X, L, dc, du, lv)
        model = cg.kde_models[1.0]
        records = []
        for seed in range(12):
            good_sink, bad_sink = [], []
            cg.kde_models[1.0] = {"good": _PdfRecorder(model["good"], good_sink),
                                  "bad": _PdfRecorder(model["bad"], bad_sink)}
            np.random.seed(1000 + seed)
            cfg, info = cg.get_config(1.0)
            cg.kde_models[1.0] = model
            vec = ref.cs.Configuration(space, values=cfg).get_array()
            if info["model_based_pick"]:
                cands = np.array([v for v, _ in bad_sink])
                assert np.array_equal(cands, np.array([v for v, _ in good_sink]))
                scores = [py_score(l, g) for (_, l), (_, g) in zip(good_sink, bad_sink)]
                ci = py_argmin(scores)
                assert np.allclose(cands[ci], vec), name
            else:
                cands = np.zeros((0, dc + du))
                ci = -1
            records.append(dict(seed=1000 + seed, model_based=bool(info["model_based_pick"]),
                                cands=cands, chosen=ci, vec=vec))
        out = dict(dc=dc, du=du, levels=np.atleast_1d(lv), n_obs=n)
        for i, r in enumerate(records):
            for k, v in r.items():
                out["r%02d_%s" % (i, k)] = v
        out["n_records"] = len(records)
        path = os.path.join(HERE, "getcfg_%s.npz" % name)
        np.savez_compressed(path, **out)
        print("wrote %s  model-based picks %d/%d" % (
            os.path.basename(path), sum(r["model_based"] for r in records), len(records)))


def gen_get_config_more(ref):
    """Round 6: one continuous dim (config #1's shape), categorical dims only (2-7 levels), and a wider
    mixed space with more observations -- the same recording as gen_get_config."""
    gen_get_config(ref, [("d1", 1, 0, 2, 24), ("cat6", 0, 6, [2, 3, 4, 5, 6, 7], 90),
                         ("d24m", 16, 8, 4, 400)])


# ----------------------------------------------------------------------------------------
# successive halving promotion (HB_iteration.py:149-190, 208-250)


def run_sh(ref, cls, losses, k, crashed):
    n = losses.shape[0]
    counter = [0]

    def sampler(budget):
        counter[0] += 1
        return {"i": counter[0]}, {}

    sh = cls(iter_number=0, num_configs=[n, k, 1], budgets=[1.0, 3.0, 9.0], config_sampler=sampler)
    jobs = []
    for _ in range(n):
        cid, cfg, b = sh.get_next_run()
        jobs.append((cid, cfg, b))
    for (cid, cfg, b), l, c in zip(jobs, losses, crashed):
        job = ref.Job(cid, config=cfg, budget=b)
        job.result = None if c else {"loss": float(l), "info": None}
        sh.register_result(job)
    nxt = sh.get_next_run()  # triggers process_results
    adv = np.array([sh.data[cid]["status"] in ("QUEUED", "RUNNING") for cid, _, _ in jobs])
    return adv, sh.actual_num_configs[1]


def gen_sh(ref):
    rs = np.random.RandomState(31)
    sizes = [1, 2, 3, 7, 27, 81, 100, 333, 1000, 1023, 1024, 1025, 2048]
    out = {}
    for i, n in enumerate(sizes):
        losses = rs.rand(n)
        crashed = rs.rand(n) < 0.1
        losses[crashed & (rs.rand(n) < 0.5)] = np.inf  # non-finite losses also crash
        for tag, cls in (("sh", ref.HB_iteration.SuccessiveHalving),
                         ("sr", ref.HB_iteration.SuccessiveResampling)):
            k = max(n // 3, 1)
            adv, count = run_sh(ref, cls, losses, k, crashed)
            out["%s%02d_adv" % (tag, i)] = adv
            out["%s%02d_count" % (tag, i)] = count
        out["b%02d_losses" % i] = losses
        out["b%02d_crashed" % i] = crashed
        out["b%02d_k" % i] = max(n // 3, 1)
    out["n_cases"] = len(sizes)
    np.savez_compressed(os.path.join(HERE, "sh_promotion.npz"), **out)
    print("wrote sh_promotion.npz (%d cases)" % len(sizes))


# ----------------------------------------------------------------------------------------
# Hyperband bracket tables (HB_master.py:93-94, 161-168)


class _Recorder(object):
    seen = []

    def __init__(self, iter_number, num_configs, budgets, config_sampler, **kw):
        _Recorder.seen.append((iter_number, list(num_configs), [float(b) for b in budgets]))
        self.is_finished = True
        self.data = {}


def gen_brackets(ref):
    tables = []
    for eta, mn, mx in ((2, 1, 64), (3, 1, 81), (3, 0.01, 1), (3, 1, 9), (4, 0.5, 32), (2.5, 1, 100)):
        _Recorder.seen = []
        hb = ref.HB_master.HpBandSter(run_id="0", config_generator=types.SimpleNamespace(get_config=None),
                                      working_directory="/tmp/hbx_golden_wd", eta=eta,
                                      min_budget=mn, max_budget=mx)
        hb.run(2 * hb.max_SH_iter, iteration_class=_Recorder)
        tables.append(dict(eta=eta, min_budget=mn, max_budget=mx, max_SH_iter=int(hb.max_SH_iter),
                           budgets=[float(b) for b in hb.budgets],
                           iterations=[dict(it=i, num_configs=n, budgets=b) for i, n, b in _Recorder.seen]))
    with open(os.path.join(HERE, "hb_brackets.json"), "w") as fh:
        json.dump(tables, fh, indent=1)
    print("wrote hb_brackets.json")


# ----------------------------------------------------------------------------------------
# end to end (config #1 semantics): reference HpBandSter.run + BOHB on the toy function,
# driven by a synchronous dispatcher in one thread (deterministic order)


def gen_e2e(ref):
    cs = ref.cs
    space = cs.ConfigurationSpace(seed=5)
    space.add_hyperparameter(cs.UniformFloatHyperparameter("x", lower=0, upper=1))
    noise = np.random.RandomState(17)

    def compute(config, budget):
        if noise.rand() < 0.2:
            return None
        res = [config["x"] + noise.randn() / budget for _ in range(int(budget))]
        return {"loss": float(np.mean(res)), "info": res}

    ref.SyncDispatcher.compute = staticmethod(compute)
    np.random.seed(123)
    logdir = os.path.join(HERE, "e2e_log")
    # the reference's own json_result_logger writes the run's configs.json / results.json (fixture)
    cg = ref.bohb.BOHB(space, directory=logdir, overwrite=True)
    records = []
    orig_get = cg.get_config
    sink = {}

    def get_config(budget):
        good_sink, bad_sink = [], []
        model = None
        if cg.kde_models:
            b = max(cg.kde_models.keys())
            model = cg.kde_models[b]
            cg.kde_models[b] = {"good": _PdfRecorder(model["good"], good_sink),
                                "bad": _PdfRecorder(model["bad"], bad_sink)}
        cfg, info = orig_get(budget)
        if model is not None:
            cg.kde_models[b] = model
        cands = np.array([v for v, _ in bad_sink]) if bad_sink else np.zeros((0, 1))
        records.append(dict(budget=budget, x=cfg["x"], model_based=bool(info["model_based_pick"]),
                            cands=cands))
        return cfg, info

    cg.get_config = get_config
    hb = ref.HB_master.HpBandSter(run_id="0", config_generator=cg, working_directory="/tmp/hbx_golden_wd",
                                  eta=2, min_budget=1, max_budget=64)
    res = hb.run(4)
    runs = []
    for cid, d in res.data.items():
        for b, r in d["results"].items():
            runs.append([list(cid), float(b), None if r is None else r["loss"], d["config"]["x"]])
    runs.sort()
    inc = res.get_incumbent_id()
    runs = dict(runs=runs, incumbent=None if inc is None else list(inc))
    out = dict(n_records=len(records))
    for i, r in enumerate(records):
        for k, v in r.items():
            out["r%03d_%s" % (i, k)] = v
    np.savez_compressed(os.path.join(HERE, "e2e_toy.npz"), **out)
    with open(os.path.join(HERE, "e2e_toy_runs.json"), "w") as fh:
        json.dump(runs, fh)
    # the reference's reload of that log into an HB_result, and what its API returns
    sys.modules["hpbandster"].HB_result = ref.HB_result.HB_result
    hr = ref.utils.logged_results_to_HB_result(logdir)

    def run_rec(r):
        return [list(r.config_id), r.budget, r.loss, r.info, r.time_stamps, r.error_logs]

    outs = dict(
        HB_config=hr.HB_config, incumbent=list(hr.get_incumbent_id()), num_iterations=hr.num_iterations(),
        trajectory_all=hr.get_incumbent_trajectory(all_budgets=True),
        trajectory_max=hr.get_incumbent_trajectory(all_budgets=False),
        all_runs=[run_rec(r) for r in hr.get_all_runs()],
        all_runs_largest=[run_rec(r) for r in hr.get_all_runs(only_largest_budget=True)],
        learning_curves=[[list(k), v] for k, v in hr.get_learning_curves().items()],
        id2config=[[list(k), v] for k, v in hr.get_id2config_mapping().items()],
        runs_by_id={str(list(k)): [run_rec(r) for r in hr.get_runs_by_id(k)] for k in list(hr.data.keys())[:5]},
        repr_first=repr(hr.get_all_runs()[0]))
    for t in ("trajectory_all", "trajectory_max"):
        outs[t]["config_ids"] = [list(c) for c in outs[t]["config_ids"]]
    with open(os.path.join(HERE, "e2e_hb_result.json"), "w") as fh:
        json.dump(outs, fh)
    print("wrote e2e_toy.npz (%d get_config calls, %d model-based), e2e_toy_runs.json (%d runs)" % (
        len(records), sum(r["model_based"] for r in records), len(runs["runs"])))


# ----------------------------------------------------------------------------------------
# KDEEI (config_generators/kde_ei.py): the reference's own refits and sampling-mode proposals


def gen_kdeei(ref):
    S = ref.synth
    cs = ref.cs
    for name, dc, n, top, upd, crash_rate in (("d4", 4, 80, 10, 1, 0.1), ("d8", 8, 200, 15, 3, 0.0)):
        space = cs.ConfigurationSpace(seed=13)
        for d in range(dc):
            space.add_hyperparameter(cs.UniformFloatHyperparameter("x%02d" % d, 0.0, 1.0))
        X = S.make_observations(n, dc, 0, 2)
        L = S.make_losses(n)
        crashed = np.random.RandomState(17).rand(n) < crash_rate
        cg = ref.kde_ei.KDEEI(space, top_n_percent=top, update_after_n_points=upd)
        fits = []
        for i in range(n):
            job = ref.Job((0, 0, i), config=vec_to_dict(space, cs, X[i]), budget=1.0)
            if crashed[i]:
                job.result, job.exception = None, "crash"
            else:
                job.result = {"loss": float(L[i]), "info": None}
            cg.new_result(job)
            if 1.0 in cg.kde_models and (not fits or fits[-1][0] is not cg.kde_models[1.0]["good"]):
                m = cg.kde_models[1.0]
                fits.append((m["good"], i, np.asarray(m["good"].bw), np.asarray(m["bad"].bw),
                             np.asarray(m["good"].data), np.asarray(m["bad"].data)))
        model = cg.kde_models[1.0]
        records = []
        for seed in range(10):
            good_sink, bad_sink = [], []
            cg.kde_models[1.0] = {"good": _PdfRecorder(model["good"], good_sink),
                                  "bad": _PdfRecorder(model["bad"], bad_sink)}
            np.random.seed(2000 + seed)
            cfg, info = cg.get_config(1.0)
            cg.kde_models[1.0] = model
            vec = cs.Configuration(space, values=cfg).get_array()
            cands = np.array([v for v, _ in bad_sink]) if info["model_based_pick"] else np.zeros((0, dc))
            ci = py_argmin([py_score(l, g) for (_, l), (_, g) in zip(good_sink, bad_sink)]) if len(cands) else -1
            records.append(dict(seed=2000 + seed, model_based=bool(info["model_based_pick"]), cands=cands,
                                chosen=ci, vec=vec))
        out = dict(dc=dc, n=n, top_n_percent=top, update_after_n_points=upd, X=X, losses=L, crashed=crashed,
                   n_fits=len(fits), fit_at=np.array([f[1] for f in fits]))
        for k, (_, at, bg, bb, dg, db) in enumerate(fits[-3:]):
            out.update({"fit%d_at" % k: at, "fit%d_bw_good" % k: bg, "fit%d_bw_bad" % k: bb,
                        "fit%d_good" % k: dg, "fit%d_bad" % k: db})
        for i, r in enumerate(records):
            for k, v in r.items():
                out["r%02d_%s" % (i, k)] = v
        out["n_records"] = len(records)
        np.savez_compressed(os.path.join(HERE, "kdeei_%s.npz" % name), **out)
        print("wrote kdeei_%s.npz  fits %d  model-based picks %d/%d" % (
            name, len(fits), sum(r["model_based"] for r in records), len(records)))


# ----------------------------------------------------------------------------------------
# numpy's float64 exp as the reference's numpy evaluates it (known-answer vectors for the engine's and
# the oracle's restatement of it)


def gen_npexp(ref):
    rs = np.random.RandomState(71)
    x = np.concatenate([
        -rs.rand(5000) * 50, (rs.rand(5000) - 0.5) * 1500, (rs.rand(1500) - 0.5) * 1e-6,
        -(rs.randn(5000) ** 2) / (2 * 0.01 ** 2), -707.7 - rs.rand(2500) * 40, -745.2 + rs.rand(1500) * 2,
        np.array([0.0, -0.0, 5e-324, -5e-324, 1e-300, -1e-300, 2.0 ** -54, -2.0 ** -54, 709.78, 709.79, -745.13,
                  -745.14, -708.3964, -707.7032713517042, np.inf, -np.inf])])
    np.savez_compressed(os.path.join(HERE, "np_exp.npz"), x=x, y=np.exp(x), numpy=np.array(np.__version__))
    print("wrote np_exp.npz (%d values, numpy %s)" % (x.size, np.__version__))


# ----------------------------------------------------------------------------------------
# tied losses: crashed runs (+inf, bohb.py:189-192) and quantised losses.  numpy's default argsort is
# not stable (bohb.py:229, HB_iteration.py:180), so these pin the reference's own tie order end to end


def tie_losses(n, decimals, crash_frac, seed):
    rs = np.random.RandomState(seed)
    L = np.round(rs.rand(n), decimals)
    crashed = rs.rand(n) < crash_frac
    return L, crashed


def gen_tie_cases(ref):
    S = ref.synth
    # many crashed runs: the bad KDE's +inf rows, in numpy's order
    X = S.make_observations(400, 5, 3, [2, 3, 5], seed=81)
    L, cr = tie_losses(400, 3, 0.3, 82)
    kde_case(ref, "tie_inf", X, L, S.make_candidates(500, 5, 3, [2, 3, 5], seed=83), 5, 3, [2, 3, 5], crashed=cr)
    # losses rounded to 2 decimals: 100 distinct values over 1000 runs, ties across the good/bad boundary
    X = S.make_observations(1000, 8, 0, 2, seed=84)
    L, cr = tie_losses(1000, 2, 0.0, 85)
    kde_case(ref, "tie_q2", X, L, S.make_candidates(600, 8, 0, 2, seed=86), 8, 0, 2, crashed=cr)
    # > 256 rows per partition (numpy's unrolled partition), 1 decimal + 10 % crashed, mixed dims
    X = S.make_observations(3000, 6, 2, [3, 4], seed=87)
    L, cr = tie_losses(3000, 1, 0.1, 88)
    kde_case(ref, "tie_q1m", X, L, S.make_candidates(400, 6, 2, [3, 4], seed=89), 6, 2, [3, 4], crashed=cr,
             store_inputs=False)
    # config #3's dims (24c + 8u, L=4), 3 decimals + 5 % crashed
    X = S.make_observations(2000, 24, 8, 4, seed=90)
    L, cr = tie_losses(2000, 3, 0.05, 91)
    kde_case(ref, "tie_d32", X, L, S.make_candidates(256, 24, 8, 4, seed=92), 24, 8, 4, crashed=cr,
             store_inputs=False)


def gen_sh_ties(ref):
    """promotion masks where tied losses straddle the k-th place (and crashed runs are filtered)"""
    rs = np.random.RandomState(41)
    sizes = [5, 9, 27, 64, 65, 81, 100, 257, 333, 1000, 1024, 2048, 3000]
    out = {}
    for i, n in enumerate(sizes):
        q = 1 if n < 100 else 2
        losses = np.round(rs.rand(n), q)
        crashed = rs.rand(n) < 0.05
        for tag, cls in (("sh", ref.HB_iteration.SuccessiveHalving),
                         ("sr", ref.HB_iteration.SuccessiveResampling)):
            k = max(n // 3, 1)
            adv, count = run_sh(ref, cls, losses, k, crashed)
            out["%s%02d_adv" % (tag, i)] = adv
            out["%s%02d_count" % (tag, i)] = count
        out["b%02d_losses" % i] = losses
        out["b%02d_crashed" % i] = crashed
        out["b%02d_k" % i] = max(n // 3, 1)
    out["n_cases"] = len(sizes)
    np.savez_compressed(os.path.join(HERE, "sh_ties.npz"), **out)
    print("wrote sh_ties.npz (%d cases)" % len(sizes))


def gen_np_argsort(ref):
    """numpy's own argsort of float64 on tie-heavy inputs (the third-party order oracle/np_argsort.py
    restates: numpy 1.26.4, AVX512_SKX dispatch)."""
    rs = np.random.RandomState(43)
    xs, outs, offs = [], [], [0]

    def add(a):
        a = np.ascontiguousarray(a, dtype=np.float64)
        xs.append(a)
        outs.append(np.argsort(a).astype(np.int32))
        offs.append(offs[-1] + a.size)

    for n in list(range(1, 70)) + [255, 256, 257, 258, 300, 511, 512, 513, 1000, 4097, 10000]:
        add(rs.randint(0, 3, size=n).astype(float))
    for t in range(120):
        n = int(np.exp(rs.uniform(np.log(2), np.log(4000))))
        kind = t % 8
        if kind == 0:
            a = np.round(rs.rand(n), 2)
        elif kind == 1:
            a = rs.rand(n); a[rs.rand(n) < 0.3] = np.inf
        elif kind == 2:
            a = rs.randint(0, 50, size=n).astype(float); a[rs.rand(n) < 0.1] = np.inf
        elif kind == 3:
            a = rs.choice([-0.0, 0.0, 1.0, -1.0, np.inf, -np.inf], size=n)
        elif kind == 4:
            a = rs.rand(n); a[rs.rand(n) < 0.05] = np.nan; a[rs.rand(n) < 0.2] = 0.5
        elif kind == 5:
            a = np.sort(rs.randint(0, 20, size=n).astype(float))
            if rs.rand() < 0.5:
                a = a[::-1].copy()
        elif kind == 6:
            a = np.round(rs.randn(n) * 3, 0)
        else:
            a = (np.arange(n) % rs.randint(2, 9)).astype(float)
        add(a)
    for n in (300, 1000, 4000):  # depth budget spent -> std::sort on the sub-ranges
        add(np.concatenate([np.arange(n // 2), np.arange(n // 2)[::-1]]).astype(float))
        b = np.arange(n, dtype=float); b[8::max(1, (n - 1) // 8)] = 1e9; add(b)
    np.savez_compressed(os.path.join(HERE, "np_argsort.npz"), x=np.concatenate(xs), order=np.concatenate(outs),
                        off=np.array(offs, dtype=np.int64), numpy=np.array(np.__version__),
                        avx512_skx=np.array(bool(np.core._multiarray_umath.__cpu_features__["AVX512_SKX"])))
    print("wrote np_argsort.npz (%d arrays, %d values, numpy %s)" % (len(xs), offs[-1], np.__version__))


GENERATORS = ["kde", "neartie", "getcfg", "getcfg_more", "sh", "brackets", "e2e", "npexp", "kdeei", "ties", "shties", "npargsort"]


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", nargs="*", default=None, help="subset of %s" % GENERATORS)
    a = ap.parse_args()
    t0 = time.time()
    ref = load_reference()
    todo = a.only or GENERATORS
    fns = {"kde": gen_kde_cases, "neartie": gen_neartie_cases, "getcfg": gen_get_config,
           "getcfg_more": gen_get_config_more, "sh": gen_sh,
           "brackets": gen_brackets, "e2e": gen_e2e, "npexp": gen_npexp,
           "kdeei": gen_kdeei, "ties": gen_tie_cases, "shties": gen_sh_ties, "npargsort": gen_np_argsort}
    for name in todo:
        fns[name](ref)
    with open(os.path.join(HERE, "PROVENANCE.json"), "w") as fh:
        json.dump(dict(generator="tests/golden/gen_golden.py", interpreter=sys.version.split()[0],
                       numpy=np.__version__, scipy=__import__("scipy").__version__,
                       statsmodels=__import__("statsmodels").__version__,
                       reference="/root/reference (HpBandSter snapshot, read-only)"), fh, indent=1)
    print("done in %.1fs" % (time.time() - t0))


if __name__ == "__main__":
    main()
