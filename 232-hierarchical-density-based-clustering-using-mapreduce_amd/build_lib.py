"""Builds libhdbmi.so (HIP, gfx950) in-tree with hipcc -- no JIT cache, no CMake.

Usage: python build_lib.py [--jobs N] [--force]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.environ.get("HDBMI_OUT") or os.path.join(HERE, "lib")
LIB = os.path.join(OUT, "libhdbmi.so")
SOURCES = ["context.cpp", "capi.cpp", "local_model.cpp", "flat.cpp", "formats.cpp", "knn.hip", "nearest.hip", "prim.hip",
           "bubbles.hip", "merge.hip", "spatial.hip", "knn_mfma.hip", "flat.hip", "comm.cpp"] + [f"knn_d{d}.hip" for d in (1, 2, 3, 4, 5, 6, 8, 16)]
HEADERS = ["common.hpp", "internal.hpp", "knn_impl.hpp", "sort.hpp", "ssort.hpp"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

# -ffp-contract=off: the reference (Java) never fuses a*b+c; bit-exact parity needs the same.
FLAGS = [*os.environ.get("HDBMI_EXTRA_FLAGS", "").split(),
         "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math",
         "--offload-arch=gfx950", "-munsafe-fp-atomics", "-Wno-unused-result"]


def _obj(src: str) -> str:
    return os.path.join(OUT, "obj", src + ".o")


def _deps(src: str) -> list:
    """src plus the csrc headers it includes, transitively"""
    seen, todo = [], [src]
    while todo:
        f = todo.pop()
        if f in seen:
            continue
        seen.append(f)
        with open(os.path.join(CSRC, f)) as fh:
            for line in fh:
                m = re.match(r'\s*#\s*include\s+"([^"/]+)"', line)
                if m and m.group(1) in HEADERS:
                    todo.append(m.group(1))
    return seen


def _stamp(src: str) -> str:
    h = hashlib.sha1()
    for f in _deps(src):
        with open(os.path.join(CSRC, f), "rb") as fh:
            h.update(fh.read())
    with open(os.path.join(HERE, "..", "include", "hdbmi.h"), "rb") as fh:
        h.update(fh.read())
    h.update(" ".join(FLAGS).encode())
    return h.hexdigest()


def _compile(src: str, force: bool) -> str:
    obj = _obj(src)
    stamp = obj + ".sha"
    st = _stamp(src)
    if not force and os.path.exists(obj) and os.path.exists(stamp) and open(stamp).read() == st:
        return obj
    os.makedirs(os.path.dirname(obj), exist_ok=True)
    lang = ["-x", "hip"] if src.endswith(".hip") else ["-x", "hip"]
    cmd = [HIPCC, *FLAGS, *lang, "-c", os.path.join(CSRC, src), "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError(f"hipcc failed for {src}")
    with open(stamp, "w") as fh:
        fh.write(st)
    return obj


def build(jobs: int | None = None, force: bool = False) -> str:
    os.makedirs(OUT, exist_ok=True)
    jobs = jobs or min(16, os.cpu_count() or 4)
    with cf.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, force), SOURCES))
    newest = max(os.path.getmtime(o) for o in objs)
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < newest:
        cmd = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", LIB, *objs]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            sys.stderr.write(r.stdout + r.stderr)
            raise RuntimeError("link failed")
    return LIB


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=None)
    ap.add_argument("--force", action="store_true")
    a = ap.parse_args()
    print(build(a.jobs, a.force))
