"""Sum a rocprofv3 --pmc counter_collection.csv per kernel: one line of name, then the counters summed
over its dispatches (the format of profiles/r02/pmc_sh_select.txt).
    python3 tools/pmc_kernels.py <dir with *counter_collection.csv> [name filter]"""
import csv
import glob
import json
import sys
from collections import defaultdict

d = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
tot = defaultdict(lambda: defaultdict(float))
disp = defaultdict(set)
for p in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
    for x in csv.DictReader(open(p)):
        k = x["Kernel_Name"]
        if flt not in k:
            continue
        tot[k][x["Counter_Name"]] += float(x["Counter_Value"])
        disp[k].add(x["Dispatch_Id"])
for k in sorted(tot, key=lambda k: -sum(tot[k].values())):
    row = {c: round(v, 1) for c, v in sorted(tot[k].items())}
    row["dispatches"] = len(disp[k])
    print(k[:90])
    print("   ", json.dumps(row))
