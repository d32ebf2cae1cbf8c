"""The secondary kernels' workloads alone (GPU box), for rocprofv3 kernel traces and PMC passes
(tools/profile_side.sh): config #2's acquisition (kde_logpdf_h32_pair1_kernel<1,0>), the ln-pdf
contract at config #3 (kde_logpdf_dd_kernel<24,8,2>), the GPU sampler (kde_sample_pair_kernel), config #5's
refit of every bracket (seg_argsort_wave_kernel + kde_fit_wave_kernel) and its promotion (sh_select_kernel).
Each workload is bench.py's own side line with fewer repetitions; the JSON lines it prints are that line.

    python tools/side_kernels.py [config2 precise sampler config5 ...]
"""
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
    which = sys.argv[1:] or ["config2", "precise", "sampler", "config5"]
    pair = c_dev = ws = None
    if {"precise", "sampler"} & set(which):
        X = S.make_observations(10000, 24, 8, 4)
        pair = kde.fit_pair(X, S.make_losses(10000), S.var_type_string(24, 8), 33, device=dev)
        c_dev = bench.blocked_candidates(0, 1_000_000, 24, 8, 4, dev)
        ws = torch.empty(pair.workspace_bytes(1_000_000), dtype=torch.uint8, device=dev)
    for name in which:
        if name == "config2":
            out = bench.config2_line(dev, reps=20)
        elif name == "precise":
            out = bench.precise_line(pair, c_dev, dev, reps=3)
        elif name == "sampler":
            out = bench.sampler_line(pair, dev, 24, 8, 4, 1_000_000, ws, reps=3)
        elif name == "config5":
            out = bench.config5(dev, reps=3)
        else:
            raise SystemExit("unknown workload %s" % name)
        torch.cuda.synchronize()
        print(json.dumps({name: out}), flush=True)


if __name__ == "__main__":
    main()
