"""Aggregate rocprofv3 --pmc counter_collection.csv files: per kernel, per-dispatch mean of every counter.

    python tools/pmc_summary.py gpurun_out/<name> [--traffic-out profiles/pmc_traffic.json --workload W]
"""
import argparse
import collections
import csv
import glob
import json
import os

ap = argparse.ArgumentParser()
ap.add_argument("dir")
ap.add_argument("--traffic-out")
ap.add_argument("--workload")
ap.add_argument("--kernel", default="kde_logpdf_h_pair_kernel")
ap.add_argument("--trace", help="kernel_trace.csv of the same command: the kernel's median duration, for the "
                                "effective clock GRBM_GUI_ACTIVE / 8 XCDs / duration (MI355X_MICROARCH.md)")
a = ap.parse_args()
vals = collections.defaultdict(lambda: collections.defaultdict(list))
grids = collections.defaultdict(collections.Counter)  # kernel -> grid sizes of its profiled dispatches
for p in glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True):
    per = collections.defaultdict(float)
    names = {}
    for row in csv.DictReader(open(p)):
        key = (row["Dispatch_Id"], row["Counter_Name"])
        per[key] += float(row["Counter_Value"])  # sum over dimensions (XCD/SE instances)
        if row["Dispatch_Id"] not in names:
            grids[row["Kernel_Name"]][int(row.get("Grid_Size") or row.get("Grid_Size_X") or 0)] += 1
        names[row["Dispatch_Id"]] = row["Kernel_Name"]
    for (d, c), v in per.items():
        vals[names[d]][c].append(v)
out = {}
for k, cs in vals.items():
    out[k] = {c: sum(v) / len(v) for c, v in cs.items()}
    out[k]["dispatches"] = max(len(v) for v in cs.values())
for k in sorted(out, key=lambda k: -out[k].get("SQ_BUSY_CYCLES", 0)):
    print(k[:90])
    print("   ", json.dumps({c: round(v, 1) for c, v in sorted(out[k].items())}))
if a.traffic_out:
    ks = [k for k in out if a.kernel in k]
    assert ks, "kernel %s not profiled" % a.kernel
    # gfx950: FETCH_SIZE (KB) counts half the bytes of wide coalesced reads (MI355X_MICROARCH.md, HBM)
    fetch = sum(out[k].get("FETCH_SIZE", 0) * out[k]["dispatches"] for k in ks) / sum(out[k]["dispatches"] for k in ks)
    write = sum(out[k].get("WRITE_SIZE", 0) * out[k]["dispatches"] for k in ks) / sum(out[k]["dispatches"] for k in ks)
    rec = {"workload": a.workload, "kernel": a.kernel, "fetch_size_kb_raw": fetch, "write_size_kb": write,
           "bytes_per_launch": 2 * fetch * 1024 + write * 1024,
           "note": "HBM-side bytes per launch (%s) = 2 x FETCH_SIZE + WRITE_SIZE "
                   "(gfx950 FETCH_SIZE halving, MI355X_MICROARCH.md); from tools/profile_round.sh"
                   % ("l and g in one launch" if any("pair" in k for k in ks) else "mean over the l and g launches")}
    if a.trace:
        import statistics
        rows = [r for r in csv.DictReader(open(a.trace)) if a.kernel in r["Kernel_Name"]]
        grid = lambda r: int(r.get("Grid_Size") or r.get("Grid_Size_X") or 0)  # noqa: E731
        # the traced launches with the grid the counter passes profiled (the main step's; the traced bench
        # also runs side lines whose grids differ)
        gc = collections.Counter()
        for k in ks:
            gc.update(grids[k])
        gpmc = gc.most_common(1)[0][0] if gc else 0
        durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9 for r in rows if grid(r) == gpmc]
        rec["grid"] = gpmc
        grbm = sum(out[k].get("GRBM_GUI_ACTIVE", 0) * out[k]["dispatches"] for k in ks) / \
            sum(out[k]["dispatches"] for k in ks)
        if durs and grbm:
            med = statistics.median(durs)
            rec["kernel_median_s"] = med
            rec["clock_ghz"] = grbm / 8 / med / 1e9
            rec["clock_note"] = ("effective engine clock during the kernel: GRBM_GUI_ACTIVE (sum over 8 XCDs) / 8 / "
                                 "median kernel duration of the traced run")
    json.dump(rec, open(a.traffic_out, "w"), indent=1)
    print(json.dumps(rec))
