"""The ln-pdf contract line of bench.py (precise_logpdf) alone (GPU box): python tools/precise_probe.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import bench
    from hpbandster_amd import kde
    from hpbandster_amd import synthetic as S
    dev = torch.device("cuda", 0)
    X = S.make_observations(10000, 24, 8, 4)
    pair = kde.fit_pair(X, S.make_losses(10000), S.var_type_string(24, 8), 33, device=dev)
    C = torch.from_numpy(S.make_candidates_blocked(0, 1000000, 24, 8, 4)).to(dev)
    print(json.dumps(bench.precise_line(pair, C, dev, reps=5)))


if __name__ == "__main__":
    main()
