"""Summarises rocprofv3 --pmc passes (tools/profile_bench.sh) per kernel: counter value per
dispatch averaged over dispatches.  HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE is
in KiB and reports 1/2 of the bytes of wide coalesced reads on gfx950 (doubled here, flagged
as such); WRITE_SIZE in KiB, exact for streaming stores."""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"hdb::(\w+)", name)
    return m.group(1) if m else name.split("(")[0][-60:]


def load(d):
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = short(row.get("Kernel_Name", "?"))
                acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return acc


def main(out):
    res = {}
    for sub in ("fetch", "write", "sq", "lds"):
        for k, cs in load(os.path.join(out, sub)).items():
            r = res.setdefault(k, {})
            for c, v in cs.items():
                r[c + "_per_dispatch"] = sum(v) / len(v)
                r["dispatches_" + sub] = len(v)
    for k, r in res.items():
        fb = r.get("FETCH_SIZE_per_dispatch")
        wb = r.get("WRITE_SIZE_per_dispatch")
        if fb is not None:
            r["hbm_read_bytes_per_launch"] = 2 * 1024 * fb  # x2: gfx950 FETCH_SIZE halves wide reads
        if wb is not None:
            r["hbm_write_bytes_per_launch"] = 1024 * wb
        if fb is not None and wb is not None:
            r["hbm_bytes_per_launch"] = r["hbm_read_bytes_per_launch"] + r["hbm_write_bytes_per_launch"]
    json.dump(res, sys.stdout, indent=1, sort_keys=True)


if __name__ == "__main__":
    main(sys.argv[1])
