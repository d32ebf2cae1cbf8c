"""Kernel timeline of the drop-in's synchronous acquisition (KDEPair.acquire, no timing events) at
config #2 and config #3 -- what a step spends beyond the scoring launch.  Run on the box:
    rocprofv3 --kernel-trace --output-format csv -d DIR -o run -- python3 tools/tail_timeline.py run
    python3 tools/tail_timeline.py show DIR/.../run_kernel_trace.csv
'run' prints each config's wall time per call; 'show' prints the last 3 steps of each config: every kernel
from one scoring launch to the next, its duration and the gap before it (us)."""
import csv
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CONFIGS = {"config2": (8, 0, 0, 1000, 100_000, 9), "config3": (24, 8, 4, 10000, 1_000_000, 33)}
if os.environ.get("TAIL_SMALL"):  # get_config-sized calls: 64 candidates against 400 / 10000 observations
    CONFIGS = {"config2": (24, 8, 4, 400, 64, 33), "config3": (24, 8, 4, 10000, 64, 33)}


def run(reps=40):
    import torch
    from hpbandster_amd import kde
    from hpbandster_amd import synthetic as S
    dev = torch.device("cuda", 0)
    out = {}
    for name, (dc, du, lev, nobs, Nc, mp) in CONFIGS.items():
        X = S.make_observations(nobs, dc, du, lev)
        pair = kde.fit_pair(X, S.make_losses(nobs), S.var_type_string(dc, du), mp, device=dev)
        C = torch.from_numpy(S.make_candidates(Nc, dc, du, lev)).to(dev)
        for _ in range(5):
            r = pair.acquire(C)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            r = pair.acquire(C)
        out[name] = {"us_per_call": (time.perf_counter() - t0) / reps * 1e6, "winner": r.index}
        time.sleep(0.01)  # a visible break between the configs in the trace
    print(json.dumps(out))


def show(path):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # configs are separated by the longest gap in the trace
    gaps = [(int(rows[i + 1]["Start_Timestamp"]) - int(rows[i]["End_Timestamp"]), i) for i in range(len(rows) - 1)]
    cut = max(gaps)[1] + 1
    for name, part in (("config2", rows[:cut]), ("config3", rows[cut:])):
        idx = [i for i, r in enumerate(part) if "kde_logpdf_h" in r["Kernel_Name"]]
        print("=== %s (%d scoring launches)" % (name, len(idx)))
        tails = []
        for a, b in zip(idx[:-1], idx[1:]):
            tails.append((int(part[b]["Start_Timestamp"]) - int(part[a]["End_Timestamp"])) / 1e3)
        if tails:
            tails.sort()
            print("scoring end -> next scoring start, median %.1f us" % tails[len(tails) // 2])
        for a, b in zip(idx[-4:-1], idx[-3:]):
            print("--- step")
            prev_end = None
            for r in part[a:b + 1]:
                s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
                gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
                print("%8.1f gap %7.1f us  %s" % ((e - s) / 1e3, gap, r["Kernel_Name"][:70]))
                prev_end = e


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run()
    else:
        show(sys.argv[2])
