"""Where an interleaved request's time goes (GPU box): the bench's sh_stage_interleaved loop with
new_result and get_next_run timed separately, speculative='never' vs 'auto' (computed ahead).
    python tools/ahead_probe.py"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import bench
    from hpbandster_amd import configspace as CS
    from hpbandster_amd.config_generators import BOHB
    from hpbandster_amd.HB_iteration import SuccessiveHalving
    from hpbandster_amd import synthetic as S
    dev = torch.device("cuda", 0)

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
        for i in range(24):
            space.add_hyperparameter(CS.UniformFloatHyperparameter("x%02d" % i, lower=0, upper=1))
        for i in range(8):
            space.add_hyperparameter(CS.CategoricalHyperparameter("y%02d" % i, ["a", "b", "c", "d"]))
        cg = BOHB(space, device=dev, sampler="gpu", sampler_seed=77, speculative=spec)
        X = S.make_observations(400, 24, 8, 4, seed=51)
        Lo = S.make_losses(400, seed=52)
        for i in range(400):
            cg.new_result(job((0, 0, i), CS.Configuration(space, vector=X[i]).get_dictionary(), Lo[i]))
        return cg, space

    out = {}
    for rep in range(3):
        for spec in ("never", "auto"):
            cg, space = make(spec)
            np.random.seed(5)
            space.seed(6)
            sh = SuccessiveHalving(0, [81, 27, 9, 3, 1], [1.0, 3.0, 9.0, 27.0, 81.0], cg.get_config, device=dev,
                                   batch_sampling=spec != "never")
            lr = np.random.RandomState(9)
            tg, tn = [], []
            torch.cuda.synchronize()
            for _ in range(81):
                t0 = time.perf_counter()
                cid, cfg, _ = sh.get_next_run()
                t1 = time.perf_counter()
                cg.new_result(job((1,) + tuple(cid[1:]), cfg, lr.rand()))
                t2 = time.perf_counter()
                tg.append(t1 - t0)
                tn.append(t2 - t1)
            k = "%s_%d" % (spec, rep)
            out[k] = {"get_next_run_us": float(np.median(tg) * 1e6), "new_result_us": float(np.median(tn) * 1e6),
                      "total_ms": float((sum(tg) + sum(tn)) * 1e3), "stats": dict(cg._ahead_stats)}
            print(k, json.dumps(out[k]), flush=True)


if __name__ == "__main__":
    main()
