"""The ln-pdf contract line of bench.py (precise_logpdf) alone (GPU box):
    python tools/precise_probe.py            -> the line
    python tools/precise_probe.py --ab N     -> N alternations of the LUT categorical path (HBX_DD_LUT=1) and the
                                                packed-match path (HBX_DD_LUT=0), ms for l + g, and the largest
                                                difference between the two paths' ln-pdfs (both within the contract)"""
import json
import os
import sys

import numpy as np

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
    if len(sys.argv) > 2 and sys.argv[1] == "--ab":
        outs = {}
        for r in range(int(sys.argv[2])):
            for lut in ("1", "0"):
                os.environ["HBX_DD_LUT"] = lut
                line = bench.precise_line(pair, C, dev, reps=5)
                outs[lut] = bench._PRECISE_OUT[0]
                print(json.dumps({"round": r, "HBX_DD_LUT": lut, "ms_l_plus_g": line["ms_l_plus_g"],
                                  "fp64_fraction": {k: v["fp64_fraction"] for k, v in line["per_kde"].items()}}),
                      flush=True)
        d = max(float(np.max(np.abs(a - b) / np.maximum(1.0, np.abs(b)))) for a, b in zip(outs["1"], outs["0"]))
        print(json.dumps({"max_rel_diff_lut_vs_packed": d}))
        return
    print(json.dumps(bench.precise_line(pair, C, dev, reps=5)))


if __name__ == "__main__":
    main()
