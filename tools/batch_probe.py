"""Per-request time of an SH stage's 81 back-to-back get_next_run (GPU box), batched (default drop-in) vs
speculative='never', with cProfile of the batched run's top host functions: python tools/batch_probe.py"""
import cProfile
import io
import json
import os
import pstats
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from hpbandster_amd import configspace as CS
    from hpbandster_amd.config_generators import BOHB
    from hpbandster_amd.HB_iteration import SuccessiveHalving
    from hpbandster_amd import synthetic as S
    dev = torch.device("cuda", 0)

    class Job(object):
        pass

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
            j = Job()
            j.id, j.exception, j.timestamps = (0, 0, i), None, {}
            j.kwargs = {"config": CS.Configuration(space, vector=X[i]).get_dictionary(), "budget": 1.0}
            j.result = {"loss": float(Lo[i]), "info": None}
            cg.new_result(j)
        return cg, space

    for spec in ("never", "auto", "auto"):
        cg, space = make(spec)
        np.random.seed(5)
        space.seed(6)
        sh = SuccessiveHalving(0, [81, 27, 9, 3, 1], [1.0, 3.0, 9.0, 27.0, 81.0], cg.get_config, device=dev,
                               batch_sampling=spec != "never")
        ts = []
        pr = cProfile.Profile() if spec == "auto" else None
        if pr:
            pr.enable()
        for _ in range(81):
            t0 = time.perf_counter()
            sh.get_next_run()
            ts.append((time.perf_counter() - t0) * 1e6)
        if pr:
            pr.disable()
        ts = np.array(ts)
        print(spec, json.dumps({"total_ms": float(ts.sum() / 1e3), "median_us": float(np.median(ts)),
                                "p90_us": float(np.percentile(ts, 90)), "max_us": float(ts.max()),
                                "largest": [round(float(x)) for x in sorted(ts)[-8:]]}), flush=True)
        if pr:
            s = io.StringIO()
            pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(18)
            print(s.getvalue()[-4000:])


if __name__ == "__main__":
    main()
