"""Config #5's refit of every bracket (bench.config5's refit_all_brackets line) with the lane-per-column fit
kernel and with the LDS kernel, alternated on one box (GPU box): python tools/fit_ab.py [rounds]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import bench
    dev = torch.device("cuda", 0)
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    for r in range(rounds):
        for mode in ("1", "0"):
            os.environ["HBX_FIT_WAVE"] = mode
            c = bench.config5(dev)
            print(json.dumps({"round": r, "fit_wave": mode, "refit_all_brackets_ms": c["refit_all_brackets_ms"],
                              "frac": c["refit_roofline"]["frac"], "bw_check": c["refit_bandwidths_spot_check"],
                              "ms_per_launch": c["ms_per_launch"]}), flush=True)


if __name__ == "__main__":
    main()
