"""Per-kernel PMC totals from rocprofv3 counter_collection CSVs (one dir per pass).
usage: python tools/kernel_counters.py <substring of kernel name> <pass dir> ..."""
import csv
import glob
import sys
from collections import defaultdict

pat = sys.argv[1]
tot = defaultdict(float)
disp = defaultdict(set)
for d in sys.argv[2:]:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if pat in r["Kernel_Name"]:
                tot[r["Counter_Name"]] += float(r["Counter_Value"])
                disp[r["Counter_Name"]].add(r["Dispatch_Id"])
for k, v in sorted(tot.items()):
    print(f"{k:32s} {v:20.0f}  dispatches {len(disp[k])}")
