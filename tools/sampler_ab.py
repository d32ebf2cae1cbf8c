"""The GPU sampler's two kernels on config #3's good KDE (1e6 x 32 candidates), alternating (GPU box):
    python tools/sampler_ab.py
pair: one (candidate, pair of dims) per lane (default); candidate: one candidate per lane
(HBX_SAMPLE_LANES=candidate).  bench.sampler_line's launch time and HBM fraction for each."""
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
    ws = torch.empty(pair.workspace_bytes(1000000), dtype=torch.uint8, device=dev)
    out = []
    for lanes in ("pair", "candidate", "pair", "candidate"):
        os.environ["HBX_SAMPLE_LANES"] = lanes
        d = bench.sampler_line(pair, dev, 24, 8, 4, 1000000, ws)
        out.append({"lanes": lanes, "ms_per_launch": d["ms_per_launch"], "hbm_frac": d["roofline"]["frac"],
                    "ms_sample_plus_acquire": d["ms_sample_plus_acquire"]})
    print(json.dumps(out))


if __name__ == "__main__":
    main()
