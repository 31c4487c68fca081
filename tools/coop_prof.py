"""Phase timestamps of the cooperative Prim (coop2, prim_coop_slots = 3) from a build with
-DHDB_COOP_PROF (HDBMI_EXTRA_FLAGS=-DHDB_COOP_PROF HDBMI_OUT=lib_prof build_lib.py; run with
HDBMI_LIB=.../lib_prof/libhdbmi.so).  Prints the median cycles between phases of steps
1024..1087 of workgroup 0.  usage: python tools/coop_prof.py [n] [d]"""
import ctypes as C
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
pkg = importlib.import_module("232-hierarchical-density-based-clustering-using-mapreduce_amd")
from importlib import import_module
A = import_module("232-hierarchical-density-based-clustering-using-mapreduce_amd._capi")
n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
d = int(sys.argv[2]) if len(sys.argv) > 2 else 8
rng = np.random.default_rng(0)
X = torch.from_numpy(rng.normal(size=(n, d)) * 10).cuda()
core = torch.from_numpy(np.abs(rng.normal(0.5, 0.1, n))).cuda()
ids = torch.arange(n, dtype=torch.int32).cuda()
ctx = pkg.Context.get(0)
ctx.use_torch_stream()
star = pkg.HDBSCANStar(ctx)
ctx.set_option("prim_coop_slots", int(os.environ.get("SLOTS", "4")))
if os.environ.get("BUBBLES"):
    rngb = np.random.default_rng(1)
    eB = torch.from_numpy(np.abs(rngb.normal(0.3, 0.1, n))).cuda()
    nnB = torch.from_numpy(np.abs(rngb.normal(0.2, 0.05, n))).cuda()
    nB = torch.from_numpy(rngb.integers(1, 9, n).astype(np.int32)).cuda()
    pkg.HdbscanDataBubbles(ctx).constructMSTBubbles(X, nB, eB, nnB, ids, core, True)
else:
    star.constructMST(X, core, True, None, ids)
torch.cuda.synchronize()
buf = (C.c_ulonglong * 512)()
A.lib().hdb_debug_coop_prof(buf)
t8 = np.array(buf, dtype=np.int64).reshape(64, 8)
t = t8[:, :6]
names = ["mrd+wave reduce+sync", "fold+publish", "poll (tags)", "fold+row load", "final sync", "-> next step"]
dif = np.diff(t, axis=1)
nxt = t[1:, 0] - t[:-1, 5]
print(f"n={n} d={d} cycles/step median {np.median(t[1:, 0] - t[:-1, 0]):.0f}")
for j in range(5):
    print(f"  {names[j]:22s} median {np.median(dif[:, j]):7.0f}  p90 {np.percentile(dif[:, j], 90):7.0f}")
print(f"  {names[5]:22s} median {np.median(nxt):7.0f}")
if np.any(t8[:, 6]):  # slots 4/5 kernels: relaxation / wave minimum split of phase 0
    print(f"    relax (mrd + key)      median {np.median(t8[:, 6] - t8[:, 0]):7.0f}")
    print(f"    wave min + last lane   median {np.median(t8[:, 7] - t8[:, 6]):7.0f}")
    print(f"    park + barrier         median {np.median(t8[:, 1] - t8[:, 7]):7.0f}")
