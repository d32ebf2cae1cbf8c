"""Check a bench line against the rocprofv3 kernel trace of the SAME process (tools/profile_round.sh).

The scoring kernel: its launches with the main step's grid, in time order, the first `warmup` dropped,
the next `steps` taken -- the launches the line timed with HIP events.  Reports rocprof's mean / median
of those, the line's event mean, and roofline.frac recomputed from rocprof (within 3 % of the line's is
the bar).  Likewise config #5's select kernel and the refit kernels.

    python tools/trace_vs_line.py <run_kernel_trace.csv> <bench_traced.json> [<bench.json>]

(bench.json: the same session's untraced line -- a 20 us kernel's HIP-event stamps move by ~10 us under
the tracer, so the short kernels are compared with the untraced line too.)
"""
import csv
import json
import statistics
import sys


def rows(path):
    out = []
    for r in csv.DictReader(open(path)):
        g = r.get("Grid_Size") or r.get("Grid_Size_X") or "0"
        out.append((int(r["Start_Timestamp"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3,
                    r["Kernel_Name"], int(g)))
    return sorted(out)


def load_line(path):
    line = None
    for ln in open(path):
        ln = ln.strip()
        if ln.startswith("{"):
            line = json.loads(ln)
    assert line is not None, "no JSON line in %s" % path
    return line


def main():
    trace, line_path = sys.argv[1], sys.argv[2]
    line = load_line(line_path)
    plain = load_line(sys.argv[3]) if len(sys.argv) > 3 else None
    R = rows(trace)
    rf = line["roofline"]
    kname = rf["kernel"].split("<")[0].split(" ")[0]
    k = [r for r in R if r[2].startswith(kname) or (" " + kname) in r[2]]
    assert k, "kernel %s not in the trace" % kname
    grid = k[0][3]
    main = [r for r in k if r[3] == grid][line["warmup"]:line["warmup"] + line["steps"]]
    d = [r[1] for r in main]
    mean_us, med_us = statistics.mean(d), statistics.median(d)
    st = rf["launch_ms_stats"]
    pairs = rf["ms_per_launch"].get("pairs_per_launch") or line["config"]["candidates_per_gpu"] * (
        line["config"]["n_good"] + line["config"]["n_bad"])
    frac_trace = rf["flops_per_pair"] * pairs / (mean_us * 1e-6) / (rf["peak"] * 1e12)
    print("scoring kernel %s: %d launches of grid %d" % (kname, len(d), grid))
    print("  rocprof mean %.1f us  median %.1f us  min %.1f  max %.1f" % (mean_us, med_us, min(d), max(d)))
    print("  line HIP-event mean %.1f us  median %.1f us (launch + rescue pass)" % (st["mean"] * 1e3,
                                                                                    st["median"] * 1e3))
    print("  line ms_per_step %.1f us: rocprof mean <= step: %s" % (line["ms_per_step"] * 1e3,
                                                                     mean_us <= line["ms_per_step"] * 1e3))
    print("  roofline.frac line %.4f  from rocprof %.4f  (%.2f %%)" % (rf["frac"], frac_trace,
                                                                       100 * (frac_trace / rf["frac"] - 1)))
    c5 = line.get("config5") or {}
    sel = [r[1] for r in R if "sh_select_kernel" in r[2]]
    if sel and "ms_per_launch" in c5:
        big = [r[1] for r in R if "sh_select_kernel" in r[2] and r[3] == max(x[3] for x in R if "sh_select" in x[2])]
        m = statistics.mean(big[1:]) if len(big) > 1 else big[0]
        gbs = c5["roofline"]["bytes_per_config"] * 1e7 / (m * 1e-6) / 1e9
        print("config5 sh_select_kernel: rocprof mean %.1f us over %d launches, traced line %.1f us; HBM frac "
              "from rocprof %.3f, traced line %.3f" % (m, len(big) - 1, c5["ms_per_launch"] * 1e3, gbs / 8000.0,
                                                      c5["roofline"]["frac"]))
        if plain and "ms_per_launch" in (plain.get("config5") or {}):
            p5 = plain["config5"]
            print("  untraced line of the session: %.1f us, HBM frac %.3f (%.2f %% from rocprof's)" % (
                p5["ms_per_launch"] * 1e3, p5["roofline"]["frac"], 100 * (p5["roofline"]["frac"] / (gbs / 8000.0) - 1)))
    rf_line = line.get("refit") or {}
    names = ("kde_refit_meta", "seg_rank", "seg_argsort", "seg_tie_flag", "seg_np_order", "kde_fit_col", "kde_colstats",
             "kde_params", "kde_table", "kde_prep_finish")
    per = {}
    for r in R:
        for nm in names:
            if r[2].startswith(nm) or (" " + nm) in r[2]:
                per.setdefault(nm, []).append(r[1])
    if per and "ms_per_refit" in rf_line:
        print("refit kernels (median us per call over the run): " +
              ", ".join("%s %.1f" % (nm, statistics.median(v)) for nm, v in per.items()))
        print("  sum of medians %.1f us; line stream_ms_median %.1f us, wall ms_per_refit %.1f us" % (
            sum(statistics.median(v) for v in per.values()), rf_line.get("stream_ms_median", float("nan")) * 1e3,
            rf_line["ms_per_refit"] * 1e3))


if __name__ == "__main__":
    main()
