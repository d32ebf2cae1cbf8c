"""Per-kernel roofline of the secondary kernels from ONE session (tools/profile_side.sh): steady durations
from the rocprofv3 kernel trace (no counters), counters per dispatch from the --pmc passes of the same
script, and each kernel's fraction of its roofline on its algorithmic basis (BASES below).

    python tools/side_roofline.py <kernel_trace.csv> <dir with pmc*/ passes> [--skip 2]

Derived columns (MI355X_MICROARCH.md: SQ_* time counters count quad-cycles summed over waves, GRBM_GUI_ACTIVE
is summed over the 8 XCDs, FETCH_SIZE counts half the bytes of wide coalesced reads):
  clock_ghz      GRBM_GUI_ACTIVE / 8 / steady duration (reads high below ~0.3 ms dispatches)
  hbm_bytes      2 FETCH_SIZE + WRITE_SIZE (KiB -> bytes)
  valu_busy      4 SQ_ACTIVE_INST_VALU / (1024 SIMDs x kernel cycles): the SIMDs' VALU-busy share
  mfma_busy      SQ_VALU_MFMA_BUSY_CYCLES / (1024 x kernel cycles)
  waves_per_simd 4 SQ_WAVE_CYCLES / kernel cycles / 1024: average resident waves per SIMD
  wait_frac      SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES: share of wave time waiting on a dependency (memory, LDS)
Writes side_pmc.json (every counter and derived value per kernel) beside the text table.
"""
import argparse
import collections
import csv
import glob
import json
import os
import statistics

N_SIMD = 1024
HBM = 8000.0          # GB/s
F16_MFMA = 2516.6     # TFLOP/s dense
FP32_VALU = 157.3     # TFLOP/s

# kernel substring -> (basis text, bound, work per dispatch, unit); work in bytes (hbm) or flops (mfma/valu).
# Shapes are tools/side_kernels.py's (= bench.py's side lines).
NC2, NOBS2 = 100_000, 1000                     # config #2
NC3, NG3, NB3 = 1_000_000, 1500, 8500          # config #3
B5, N5, D5 = 10_000, 1000, 32                  # config #5
NG5, NB5 = 150, 850                            # bohb_split_sizes(1000, 33)
BASES = [
    ("kde_logpdf_h32_pair1_kernel<1, 0>",
     "config #2: 28 flops/pair (SURVEY 8d, 3 Dc + 4) x 1e5 x 1e3 pairs (one column tile per wave)", "mfma",
     28.0 * NC2 * NOBS2),
    ("kde_logpdf_h32_pair_kernel<1, 0, false, true>",
     "config #2 with HBX_PAIR1=0: 28 flops/pair x 1e5 x 1e3 pairs", "mfma", 28.0 * NC2 * NOBS2),
    ("kde_logpdf_h32_pair_kernel<3, 1, false, true>",
     "config #3 headline: 92 flops/pair x 1e6 x 1e4 pairs", "mfma", 92.0 * NC3 * (NG3 + NB3)),
    ("kde_logpdf_dd_kernel<24, 8, 2",
     "config #3 ln-pdf pass: 92 flops/pair x 1e6 x (1500 + 8500) pairs over the l and g dispatches' mean durations",
     "valu", 92.0 * NC3 * (NG3 + NB3) / 2),
    ("kde_sample_pair_kernel",
     "1e6 x 32 f64 values written (8 B each) + the datum index (8 B) and flag (1 B) per candidate", "hbm",
     NC3 * (D5 * 8 + 9)),
    ("kde_fit_wave_kernel",
     "config #5: every set's rows read once ((150 + 850) x 32 x 8 B per bracket) + the order read (8 B per row)",
     "hbm", B5 * (NG5 + NB5) * (D5 * 8 + 8)),
    ("seg_argsort_wave_kernel",
     "config #5: losses read (8 B) + order written (8 B) per configuration", "hbm", B5 * N5 * 16),
    ("sh_select_kernel",
     "config #5: losses read (8 B) + mask written (1 B) per configuration", "hbm", B5 * N5 * 9),
    # the acquisition's tail after the scoring launch (config #2 when run alone): latency-bound chains, no
    # roofline -- durations and counters only
    ("kde_combine_kernel", "acquisition tail: score intervals, segment minima (36 B per candidate)", "lat", 0),
    ("kde_shortlist_kernel", "acquisition tail: the shortlist predicate per candidate", "lat", 0),
    ("kde_exact_kernel", "acquisition tail: fp64 re-score of the shortlist (numpy order)", "lat", 0),
    ("kde_final_kernel", "acquisition tail: argmin, record published to mapped host memory", "lat", 0),
]


def trace_durations(path, skip):
    calls = collections.defaultdict(list)
    for r in sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"])):
        calls[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    return {k: (v[skip:] if len(v) > skip else v) for k, v in calls.items()}


def pmc_counters(d):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        per, names = collections.defaultdict(float), {}
        for row in csv.DictReader(open(p)):
            per[(row["Dispatch_Id"], row["Counter_Name"])] += float(row["Counter_Value"])
            names[row["Dispatch_Id"]] = row["Kernel_Name"]
        for (disp, c), v in per.items():
            vals[names[disp]][c].append(v)
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in vals.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("pmcdir")
    ap.add_argument("--skip", type=int, default=2)
    a = ap.parse_args()
    durs = trace_durations(a.trace, a.skip)
    pmc = pmc_counters(a.pmcdir)
    rec = {}
    for sub, basis, bound, work in BASES:
        names = [k for k in durs if sub in k]
        if not names:
            continue
        name = max(names, key=lambda k: sum(durs[k]))  # (the SG dd kernel beside its LDS twin's early exits)
        ds = durs[name]
        dur = statistics.mean(ds)
        if "dd_kernel" in sub and len(ds) >= 2:  # l and g dispatches (1500 / 8500 observations): split at the
            srt = sorted(ds)                        # largest gap, work / (mean l + mean g) = the mean of the pair
            cut = max(range(1, len(srt)), key=lambda i: srt[i] - srt[i - 1])
            dur = (statistics.mean(srt[:cut]) + statistics.mean(srt[cut:])) / 2
        c = next((pmc[k] for k in pmc if sub in k), {})
        r = {"kernel": name, "dispatches_traced": len(ds), "dur_us_mean": dur * 1e6,
             "dur_us_median": statistics.median(ds) * 1e6, "basis": basis, "bound": bound}
        if bound == "lat":
            r.update(achieved=0.0, peak=None, unit=None, frac=0.0)
        elif bound == "hbm":
            ach = work / dur / 1e9
            r.update(achieved=ach, peak=HBM, unit="GB/s", frac=ach / HBM, algorithmic_bytes=work)
        else:
            peak = F16_MFMA if bound == "mfma" else FP32_VALU
            ach = work / dur / 1e12
            r.update(achieved=ach, peak=peak, unit="TFLOP/s", frac=ach / peak, algorithmic_flops=work)
        if c:
            cyc = c.get("GRBM_GUI_ACTIVE", 0) / 8
            if cyc:
                r["clock_ghz"] = cyc / dur / 1e9
                r["valu_busy"] = 4 * c.get("SQ_ACTIVE_INST_VALU", 0) / (N_SIMD * cyc)
                r["mfma_busy"] = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (N_SIMD * cyc)
                r["waves_per_simd"] = 4 * c.get("SQ_WAVE_CYCLES", 0) / cyc / N_SIMD
            if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
                hb = (2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024
                r["hbm_bytes_pmc"] = hb
                r["hbm_gbs_pmc"] = hb / dur / 1e9
            if c.get("SQ_WAVES"):
                r["valu_per_wave"] = c.get("SQ_INSTS_VALU", 0) / c["SQ_WAVES"]
                r["salu_per_wave"] = c.get("SQ_INSTS_SALU", 0) / c["SQ_WAVES"]
                r["mfma_per_wave"] = c.get("SQ_INSTS_MFMA", 0) / c["SQ_WAVES"]
            if c.get("SQ_WAVE_CYCLES"):
                r["wait_frac"] = c.get("SQ_WAIT_INST_ANY", 0) / c["SQ_WAVE_CYCLES"]
            r["counters"] = c
        rec[sub] = r
    print("%-48s %9s %7s %9s %6s %6s %6s %6s %8s %6s" % ("kernel", "us", "frac", "achieved", "clock", "valu",
                                                          "mfma", "w/simd", "GB/s pmc", "wait"))
    for sub, r in rec.items():
        print("%-48s %9.2f %7.3f %9.1f %6.2f %6.3f %6.3f %6.2f %8.0f %6.3f" % (
            sub[:48], r["dur_us_mean"], r["frac"], r["achieved"], r.get("clock_ghz", 0), r.get("valu_busy", 0),
            r.get("mfma_busy", 0), r.get("waves_per_simd", 0), r.get("hbm_gbs_pmc", 0), r.get("wait_frac", 0)))
    for sub, r in rec.items():
        print("  %s: %s %s per wave: VALU %.0f SALU %.0f MFMA %.0f" % (
            sub[:40], r["bound"], r["basis"], r.get("valu_per_wave", 0), r.get("salu_per_wave", 0),
            r.get("mfma_per_wave", 0)))
    others = sorted(((statistics.mean(v) * len(v), k) for k, v in durs.items()), reverse=True)[:12]
    print("largest kernels of the traced run (total steady time):")
    for t, k in others:
        print("  %10.1f us  %s" % (t * 1e6, k[:100]))
    json.dump(rec, open(os.path.join(a.pmcdir, "side_pmc.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
