"""Where the one-worker loop's time goes (GPU box): SuccessiveHalving.get_next_run followed by its result
(new_result + refit) for 81 requests, BOHB(sampler='gpu') at 24c + 8u against 400 observations -- bench.py's
sh_stage_interleaved -- under cProfile.   python tools/interleaved_profile.py"""
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
    from hpbandster_amd.HB_iteration import SuccessiveHalving
    from hpbandster_amd import synthetic as S
    dev = torch.device("cuda", 0)
    CS, space, job = bench._space_and_jobs((24, 8))
    cg = BOHB(space, device=dev, sampler="gpu", sampler_seed=77, speculative="never")
    X = S.make_observations(400, 24, 8, 4, seed=51)
    Lo = S.make_losses(400, seed=52)
    for i in range(400):
        cg.new_result(job((0, 0, i), CS.Configuration(space, vector=X[i]).get_dictionary(), Lo[i]))
    lr = np.random.RandomState(9)

    def loop(n):
        sh = SuccessiveHalving(0, [81, 27, 9, 3, 1], [1.0, 3.0, 9.0, 27.0, 81.0], cg.get_config, device=dev,
                               batch_sampling=False)
        for _ in range(n):
            cid, cfg, _ = sh.get_next_run()
            cg.new_result(job((1,) + tuple(cid[1:]), cfg, lr.rand()))

    loop(20)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    loop(81)
    torch.cuda.synchronize()
    print("ms per request+result %.4f" % ((time.perf_counter() - t0) / 81 * 1e3))
    pr = cProfile.Profile()
    pr.enable()
    loop(81)
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
