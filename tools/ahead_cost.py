"""Host time of one computed-ahead launch, piece by piece (GPU box): python tools/ahead_cost.py"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from hpbandster_amd import configspace as CS
    from hpbandster_amd.config_generators import BOHB
    from hpbandster_amd import synthetic as S
    dev = torch.device("cuda", 0)

    class Job(object):
        pass
    space = CS.ConfigurationSpace(seed=3)
    for i in range(24):
        space.add_hyperparameter(CS.UniformFloatHyperparameter("x%02d" % i, lower=0, upper=1))
    for i in range(8):
        space.add_hyperparameter(CS.CategoricalHyperparameter("y%02d" % i, ["a", "b", "c", "d"]))
    cg = BOHB(space, device=dev, sampler="gpu", sampler_seed=77)
    X = S.make_observations(400, 24, 8, 4, seed=51)
    Lo = S.make_losses(400, seed=52)
    for i in range(400):
        j = Job()
        j.id, j.exception, j.timestamps = (0, 0, i), None, {}
        j.kwargs = {"config": CS.Configuration(space, vector=X[i]).get_dictionary(), "budget": 1.0}
        j.result = {"loss": float(Lo[i]), "info": None}
        cg.new_result(j)
    pair = cg.kde_models[1.0]
    t = {k: [] for k in ("hint", "buffer", "sample", "acquire_ahead", "serve", "configspace")}
    for r in range(60):
        t0 = time.perf_counter()
        cg._next_call_is_random()
        t1 = time.perf_counter()
        with cg._ahead_lock:
            buf, keep = cg._pick_buffer(pair)
        t2 = time.perf_counter()
        cands, _, err = pair['good'].sample(cg.vartypes, cg.bw_factor, cg.num_samples, cg.sampler_seed, 64 * r,
                                            out=keep[:3])
        t3 = time.perf_counter()
        cg._pick_seq += 1
        pair.acquire_ahead(cands, err, keep[3], buf, cg._pick_seq)
        t4 = time.perf_counter()
        from hpbandster_amd.config_generators.bohb import _Ahead
        a = _Ahead(pair, 0, 0, cg._pick_seq, keep, buf, None, 0)
        res, bad, row = cg._serve_ahead(a)
        t5 = time.perf_counter()
        CS.Configuration(space, vector=row).get_dictionary()
        t6 = time.perf_counter()
        for k, v in zip(t, (t1 - t0, t2 - t1, t3 - t2, t4 - t3, t5 - t4, t6 - t5)):
            t[k].append(v * 1e6)
    print(json.dumps({k: round(float(np.median(v)), 1) for k, v in t.items()}))


if __name__ == "__main__":
    main()
