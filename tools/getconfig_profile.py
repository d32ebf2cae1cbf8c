"""Where the default drop-in's get_config time goes (GPU box): BOHB with the host sampler, 64 candidates,
24c + 8u against 400 observations, cProfile over 200 model-based calls.  python tools/getconfig_profile.py"""
import cProfile
import os
import pstats
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import bench
    from hpbandster_amd.config_generators import BOHB
    from hpbandster_amd import synthetic as S
    dev = torch.device("cuda", 0)
    CS, space, job = bench._space_and_jobs((24, 8))
    cg = BOHB(space, device=dev, random_fraction=0.0)
    X = S.make_observations(400, 24, 8, 4, seed=51)
    Lo = S.make_losses(400, seed=52)
    for i in range(400):
        cg.new_result(job((0, 0, i), CS.Configuration(space, vector=X[i]).get_dictionary(), Lo[i]))
    np.random.seed(5)
    for _ in range(20):
        cg.get_config(1.0)
    t0 = time.perf_counter()
    for _ in range(200):
        cg.get_config(1.0)
    print("ms per call %.4f" % ((time.perf_counter() - t0) / 200 * 1e3))
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(200):
        cg.get_config(1.0)
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(22)


if __name__ == "__main__":
    main()
