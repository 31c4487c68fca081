"""Per-launch timeline of the last call of a kernel sequence in a rocprofv3 kernel trace.
Usage: python tools/trace_last.py <kernel_trace.csv> <first kernel name substring> [min_us]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
first = sys.argv[2]
min_us = float(sys.argv[3]) if len(sys.argv) > 3 else 0.0
idx = [i for i, r in enumerate(rows) if first in r["Kernel_Name"]]
s = idx[-1]
t0 = int(rows[s]["Start_Timestamp"])
prev = t0
tot = {}
for r in rows[s:]:
    a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    nm = r["Kernel_Name"].replace("hdb::(anonymous namespace)::", "").replace("void ", "").split("(")[0]
    nm = nm.split("<")[0][:48] if "rocprim" in nm else nm[:48]
    tot[nm] = tot.get(nm, 0) + (b - a) / 1e3
    if (b - a) / 1e3 >= min_us or (a - prev) / 1e3 >= 10:
        print(f"{(a - t0) / 1e3:9.1f} gap {(a - prev) / 1e3:7.1f} dur {(b - a) / 1e3:8.1f}  {nm}")
    prev = b
print("total span", (prev - t0) / 1e3, "us")
for k, v in sorted(tot.items(), key=lambda x: -x[1])[:25]:
    print(f"{v:9.1f}  {k}")
