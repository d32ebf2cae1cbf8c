"""Per-kernel VGPR / scratch / occupancy from a hipcc -S listing: python tools/isa_stats.py file.s [filter]"""
import re
import sys

cur = None
rows = []
for line in open(sys.argv[1]):
    m = re.match(r"^(_Z\w+):", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    if cur is None:
        continue
    for key in ("NumVgprs", "ScratchSize", "Occupancy"):
        m = re.match(r"^; %s: (\d+)" % key, line)
        if m and key not in cur:
            cur[key] = int(m.group(1))
flt = sys.argv[2] if len(sys.argv) > 2 else ""
for r in rows:
    if flt in r["name"] and "NumVgprs" in r:
        print("%-70s vgpr %3d scratch %4d occ %d" % (r["name"][:70], r["NumVgprs"], r.get("ScratchSize", -1),
                                                   r.get("Occupancy", -1)))
