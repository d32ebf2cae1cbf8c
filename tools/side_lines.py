"""Selected bench.py side lines alone (GPU box): python tools/side_lines.py promote sh_stage ..."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import bench
    dev = torch.device("cuda", 0)
    out = {}
    for name in sys.argv[1:]:
        if name == "promote":
            out["promote_dropin"] = bench.promote_dropin(dev)
            out["promote_dropin_n81"] = bench.promote_dropin(dev, n=81)
        elif name == "sh_stage":
            out["sh_stage"] = bench.sh_stage_line(dev)
            out["sh_stage_interleaved"] = bench.sh_stage_line(dev, interleaved=True, reps=7)
            out["sh_stage_interleaved_host_sampler"] = bench.sh_stage_line(dev, n_obs=100, stage=27, reps=3,
                                                                           interleaved=True, sampler="host",
                                                                           dims=(4, 2))
        elif name == "config2":
            out["config2"] = bench.config2_line(dev)
        print(json.dumps({name: {k: v for k, v in out.items()}}), flush=True)


if __name__ == "__main__":
    main()
