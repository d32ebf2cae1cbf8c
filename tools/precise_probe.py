"""The ln-pdf contract line of bench.py (precise_logpdf) alone, with the tiled fp64 kernel and the
per-point one (GPU box): python tools/precise_probe.py"""
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
    C = torch.from_numpy(S.make_candidates(1000000, 24, 8, 4)).to(dev)
    out = {}
    for t in ("1", "0"):
        os.environ["HBX_LOGPDF_TILED"] = t
        out["tiled" if t == "1" else "per_point"] = bench.precise_line(pair, C if t == "1" else C[:20000].contiguous(),
                                                                       dev, reps=3 if t == "1" else 1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
