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
        elif name == "threaded":
            out["threaded_run"] = bench.threaded_run_line(dev)
        elif name == "getconfig":
            out["get_config_default"] = bench.get_config_line(dev)
        elif name == "refit":
            from hpbandster_amd import synthetic as S
            X = S.make_observations(10000, 24, 8, 4)
            out["refit"] = bench.refit_line(X, S.make_losses(10000), S.var_type_string(24, 8), dev)
        elif name == "precise":
            from hpbandster_amd import kde
            from hpbandster_amd import synthetic as S
            X = S.make_observations(10000, 24, 8, 4)
            pair = kde.fit_pair(X, S.make_losses(10000), S.var_type_string(24, 8), 33, device=dev)
            out["precise_logpdf"] = bench.precise_line(pair, bench.blocked_candidates(0, 1_000_000, 24, 8, 4, dev), dev)
        elif name == "config2":
            out["config2"] = bench.config2_line(dev)
        elif name == "config5":
            out["config5"] = bench.config5(dev)
        elif name == "sampler":
            import numpy as np
            import torch
            from hpbandster_amd import kde
            from hpbandster_amd import synthetic as S
            X = S.make_observations(10000, 24, 8, 4)
            pair = kde.fit_pair(X, S.make_losses(10000), S.var_type_string(24, 8), 33, device=dev)
            ws = torch.empty(pair.workspace_bytes(1_000_000), dtype=torch.uint8, device=dev)
            out["gpu_sampler"] = bench.sampler_line(pair, dev, 24, 8, 4, 1_000_000, ws)
        print(json.dumps({name: {k: v for k, v in out.items()}}), flush=True)


if __name__ == "__main__":
    main()
