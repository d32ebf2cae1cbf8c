"""Steady-state per-kernel durations from a rocprofv3 kernel_trace.csv: drop the first `--skip` calls
of each kernel (clock ramp / first-launch costs), report mean and median of the rest.

    python tools/ksteady.py gpurun_out/<run>/trace/run_kernel_trace.csv [--skip 2] [--match kde_]
"""
import argparse
import collections
import csv
import statistics

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--skip", type=int, default=2)
ap.add_argument("--match", default="")
a = ap.parse_args()
calls = collections.defaultdict(list)
for r in sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"])):
    if a.match in r["Kernel_Name"]:
        calls[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(calls.items(), key=lambda kv: -sum(kv[1])):
    w = v[a.skip:] if len(v) > a.skip else v
    print("%-72s calls %3d  steady mean %10.1f us  median %10.1f us  (all-call mean %10.1f us)"
          % (k[:72], len(v), statistics.mean(w), statistics.median(w), statistics.mean(v)))
