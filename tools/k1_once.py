"""One warm K1 launch at config-2 size (1M x 3, minPts 4, EXCL_SELF) -- the PMC target."""
import importlib, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
pkg = importlib.import_module("232-hierarchical-density-based-clustering-using-mapreduce_amd")
from bench import make_blobs
X = torch.from_numpy(make_blobs(1_000_000, 3, 20, 1)).cuda()
ctx = pkg.Context.get(0); ctx.use_torch_stream()
star = pkg.HDBSCANStar(ctx)
star.calculateCoreDistances(X, 4, None, 2)
torch.cuda.synchronize()
star.calculateCoreDistances(X, 4, None, 2)
torch.cuda.synchronize()
print("done")
