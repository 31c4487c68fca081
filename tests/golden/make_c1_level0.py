"""Generates tests/golden/c1_level0_model.npz: the inputs of C1's level-0 bubble model (the
18,135 non-empty bubbles of Skin_NonSkin at the reference's my_args, Main.java:71) and the
result of the INDEPENDENT pure-Python transcription (oracle/java_transcription.py) on them.

C1 hinges on this one model: it throws the reference's own "Cluster cannot have less than 0
points" (Clusters.java:45-46) and, under D10, the whole file becomes one exact leaf.  The
transcription has its own JDK 8 HashMap/TreeSet emulation and shares no code with the C
oracle (hdb_oracle.c) or the product (local_model.cpp); tests/test_java_transcription.py
checks that the C oracle throws at the same cluster label, level and point count.

Inputs are built as oracle/mr_driver.py does at iteration 0: D2 sample ids (seed 20210101),
nearest sample (FirstStep.java:74-85), CombineStep statistics, D4 compaction.
Run in the build container (CPU; ~3 min):  python tests/golden/make_c1_level0.py
"""
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from conftest import load_skin  # noqa: E402
from oracle import java_transcription as J  # noqa: E402
from oracle import mr_driver as M  # noqa: E402
from oracle import oracle as O  # noqa: E402

MIN_PTS, MCL, K, SEED = 4, 4, 0.2, 20210101


def model_inputs():
    X = load_skin()
    sp = M.sample_ids(X.shape[0], K, None, SEED, 0, 0)
    near, _ = O.nearest_sample(X, X[sp])
    st = O.bubble_stats(X, near, sp.shape[0], "combine")
    nonempty = np.nonzero(st["info"][:, 2] > 0)[0]
    return st["rep"][nonempty], st["info"][nonempty], sp.shape[0]


def main(out=os.path.join(HERE, "c1_level0_model.npz")):
    t0 = time.time()
    rep, info, m = model_inputs()
    print(f"inputs: {m} samples, {rep.shape[0]} non-empty bubbles ({time.time() - t0:.1f} s)", flush=True)
    t1 = time.time()
    code, label, level, pts = 0, 0, np.nan, 0
    labels = np.zeros(0, np.int32)
    try:
        r = J.local_model(rep, info, MIN_PTS, MCL)
        labels = r["labels"]
    except J.JavaException as e:
        code = e.code
        if isinstance(e.detail, dict):
            label, level, pts = e.detail["label"], e.detail["level"], e.detail["num_points"]
    print(f"transcription: code {code} label {label} level {level!r} numPoints {pts} ({time.time() - t1:.1f} s)")
    np.savez_compressed(out, rep=rep, info=info, samples=m, min_pts=MIN_PTS, mcl=MCL, code=code, label=label,
                        level=level, num_points=pts, labels=labels)
    print("wrote", out, os.path.getsize(out), "bytes")


if __name__ == "__main__":
    main(*sys.argv[1:])
