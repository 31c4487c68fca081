"""Per-partition kernel split of a rocprofv3 --stats csv (tools/c2_part.py runs: reps + 1 calls).
usage: python tools/kstats.py <kernel_stats.csv> <partitions>"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
R = float(sys.argv[2])
agg = {}
for r in rows:
    n = r["Name"]
    if "rocprim" in n or "hipcub" in n:
        k = "rocprim/hipcub"
    elif "fillBuffer" in n:
        k = "fill"
    elif "copyBuffer" in n:
        k = "copy"
    else:
        k = re.sub(r"\(anonymous namespace\)::", "", n).split("(")[0][-50:]
    a = agg.setdefault(k, [0.0, 0])
    a[0] += float(r["TotalDurationNs"])
    a[1] += int(r["Calls"])
tot = sum(v[0] for v in agg.values())
for k, (t, c) in sorted(agg.items(), key=lambda x: -x[1][0]):
    print(f"{t / 1e3 / R:9.1f} us/part {c / R:7.1f} calls  {k}")
print(f"total {tot / 1e3 / R:.1f} us/part")
