"""The ln-pdf contract line of bench.py (precise_logpdf) alone (GPU box):
    python tools/precise_probe.py            -> the line
    python tools/precise_probe.py --ab N [VAR] -> N alternations of VAR=1 and VAR=0 (default HBX_DD_LUT: the LUT
                                                categorical path against the packed-match path; HBX_DD_SG: the
                                                scalar-staged against the LDS-staged kernel), ms for l + g, and the
                                                largest difference between the two paths' ln-pdfs"""
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
        var = sys.argv[3] if len(sys.argv) > 3 else "HBX_DD_LUT"
        outs = {}
        for r in range(int(sys.argv[2])):
            for lut in ("1", "0"):
                os.environ[var] = lut
                line = bench.precise_line(pair, C, dev, reps=5)
                outs[lut] = bench._PRECISE_OUT[0]
                print(json.dumps({"round": r, var: lut, "ms_l_plus_g": line["ms_l_plus_g"],
                                  "fp64_fraction": {k: v["fp64_fraction"] for k, v in line["per_kde"].items()}}),
                      flush=True)
        d = max(float(np.max(np.abs(a - b) / np.maximum(1.0, np.abs(b)))) for a, b in zip(outs["1"], outs["0"]))
        print(json.dumps({"var": var, "max_rel_diff_1_vs_0": d}))
        return
    print(json.dumps(bench.precise_line(pair, C, dev, reps=5)))


if __name__ == "__main__":
    main()
