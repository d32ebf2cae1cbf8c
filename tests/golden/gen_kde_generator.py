#!/opt/conda/bin/python3.9 -B
"""Golden run of the reference's KernelDensityEstimator generator (config_generators/kde.py).

    PYTHONDONTWRITEBYTECODE=1 /opt/conda/bin/python3.9 -B tests/golden/gen_kde_generator.py

Build container only (reference + statsmodels 0.12.2 + scipy 1.7.1), with gen_golden.py's shims.
The reference's constructor cannot run as written (``super().__init__(**kwargs)`` on the tuple of
``*kwargs``, kde.py:12,33: TypeError), so the object is made with ``__new__`` and given the attributes
that constructor assigns (kde.py:35-47); ``get_config`` and ``new_result`` are the reference's own
methods.  Jobs carry ``{'result': {'loss': ...}}``, the form kde.py:119 reads.  A fixed schedule of
new_result(job) / get_config(budget) calls under ``np.random.seed`` is recorded: every proposal
vector, every refit's bandwidths and training data.  Writes tests/golden/kdegen_<case>.npz (data only).
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gen_golden as GG  # noqa: E402


def loss_of(vec, budget, rs):
    """A smooth toy objective with budget-dependent noise (independent RandomState)."""
    v = np.asarray(vec)
    return float(np.sum((v - 0.3) ** 2) + 0.05 * rs.rand() / budget)


def run_case(ref, kde_mod, name, D, steps, budgets, update_after, top_pct, min_points, seed):
    cs = ref.cs
    space = GG.make_space(cs, D, 0, 0)
    K = kde_mod.KernelDensityEstimator
    gen = K.__new__(K)
    ref.base.base_config_generator.__init__(gen)
    gen.top_n_percent = top_pct
    gen.update_after_n_points = update_after
    gen.configspace = space
    gen.min_points_in_model = min_points
    gen.var_type = "c" * len(space.get_hyperparameters())
    gen.configs, gen.losses, gen.kde_models = dict(), dict(), dict()

    np.random.seed(seed)
    rs = np.random.RandomState(seed + 100)
    vectors, kinds, bud_log, losses = [], [], [], []
    refits = []  # (step, budget, bw, data)
    for step in range(steps):
        b = budgets[step % len(budgets)]
        out = gen.get_config(b)
        if isinstance(out, tuple):  # model-based proposal
            cfg, kind = out[0], 1
        else:  # kde.py:65 returns a bare dict without a model
            cfg, kind = out, 0
        vec = cs.Configuration(space, cfg).get_array()
        loss = loss_of(vec, b, rs)
        job = ref.Job((0, 0, step), config=cfg, budget=b)
        job.result = {"result": {"loss": loss}}
        before = dict(gen.kde_models)
        gen.new_result(job)
        for bb, m in gen.kde_models.items():
            if before.get(bb) is not m:
                refits.append((step, bb, np.array(m.bw, dtype=np.float64), np.array(m.data, dtype=np.float64)))
        vectors.append(vec)
        kinds.append(kind)
        bud_log.append(b)
        losses.append(loss)
    np.savez(os.path.join(HERE, "kdegen_%s.npz" % name), D=D, steps=steps, budgets=np.array(budgets, float),
             update_after=update_after, top_pct=top_pct, min_points=min_points, seed=seed,
             vectors=np.array(vectors), kinds=np.array(kinds), budget_log=np.array(bud_log),
             losses=np.array(losses), refit_step=np.array([r[0] for r in refits]),
             refit_budget=np.array([r[1] for r in refits], float),
             refit_bw=np.array([r[2] for r in refits]),
             refit_data=np.concatenate([r[3] for r in refits]) if refits else np.zeros((0, D)),
             refit_n=np.array([len(r[3]) for r in refits]))
    print("%s: %d steps, %d refits, %d model-based proposals" % (name, steps, len(refits), sum(kinds)))


def main():
    ref = GG.load_reference()
    kde_mod = GG._load("hpbandster.config_generators.kde",
                       os.path.join(GG.REF, "hpbandster", "config_generators", "kde.py"))
    run_case(ref, kde_mod, "d3", D=3, steps=60, budgets=[1.0, 3.0], update_after=10, top_pct=30,
             min_points=4, seed=7)
    run_case(ref, kde_mod, "d2", D=2, steps=45, budgets=[9.0], update_after=15, top_pct=40, min_points=3,
             seed=8)


if __name__ == "__main__":
    main()
