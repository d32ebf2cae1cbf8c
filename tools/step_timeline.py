"""Kernel timeline of the last headline steps from a rocprofv3 kernel trace (run on the box after
    rocprofv3 --kernel-trace --output-format csv -d DIR -o run -- python3 tools/step_breakdown.py --steps 10):
    python tools/step_timeline.py DIR/.../run_kernel_trace.csv
Prints, for the last 3 scoring launches, every kernel from that launch to the next one: name, duration and
the gap before it (us)."""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "kde_logpdf_h32_pair_kernel" in r["Kernel_Name"]]
    for a, b in zip(idx[-4:-1], idx[-3:]):
        print("--- step")
        prev_end = None
        for r in rows[a:b + 1]:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
            print("%8.1f gap %7.1f us  %s" % ((e - s) / 1e3, gap, r["Kernel_Name"][:70]))
            prev_end = e


if __name__ == "__main__":
    main()
