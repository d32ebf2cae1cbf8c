"""Per-kernel median durations and the last dispatches of a rocprofv3 kernel trace (csv):
    python3 tools/trace_tail.py DIR/.../run_kernel_trace.csv [last]"""
import csv
import sys
from collections import defaultdict


def main(path, last=8):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    dur = defaultdict(list)
    for r in rows:
        dur[r["Kernel_Name"][:60]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print("kernel (median us, count)")
    for k, v in sorted(dur.items(), key=lambda kv: -sorted(kv[1])[len(kv[1]) // 2]):
        v.sort()
        print("%8.2f %6d  %s" % (v[len(v) // 2], len(v), k))
    print("last %d dispatches: duration, gap before (us)" % last)
    prev = None
    for r in rows[-last:]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        print("%8.2f gap %8.2f  %s" % ((e - s) / 1e3, (s - prev) / 1e3 if prev else 0.0, r["Kernel_Name"][:60]))
        prev = e


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 8)
