"""The reference's record formats on either side of the hot path,
backed by csrc/formats.cpp through the C-ABI (host code; no device needed).

* ``MapperDataset_github`` / ``read_dataset`` -- the dataset text -> points
  (MapperDataset_github.java:12-20): ``s.split(" ")`` + ``Double.parseDouble``, one point per
  line, numbered in file order.  ``strict=False`` is deviation D1: runs of
  blanks/tabs separate fields and the first ``d`` columns are kept (Skin_NonSkin.txt is
  TAB-separated with a trailing label column).
* ``format_local_mst`` -- CreateLocalMST's local-MST text (CreateLocalMST.java:110-123):
  ``"v1 v2 w f1 f2 node"`` lines joined by ``\\n``, ``w`` via ``Double.toString``.
* ``parse_local_mst`` -- UnionFindReducer.call's parse of those records
  (UnionFindReducer.java:22-45).
* ``double_to_string`` -- ``Double.toString`` (Java layout, shortest round-trip digits).

Malformed fields raise ``NumberFormatException`` and short lines
``ArrayIndexOutOfBoundsException``, as the Java does.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from ._capi import check, lib, ptr


def double_to_string(v: float) -> str:
    """Double.toString(v)."""
    buf = C.create_string_buffer(40)
    n = lib().hdb_format_double(float(v), buf, 40)
    if n < 0:
        check(n, "hdb_format_double")
    return buf.value.decode()


def _as_bytes(text_or_path) -> bytes:
    if isinstance(text_or_path, (bytes, bytearray)):
        return bytes(text_or_path)
    if isinstance(text_or_path, str) and "\n" not in text_or_path and os.path.exists(text_or_path):
        with open(text_or_path, "rb") as fh:
            return fh.read()
    return str(text_or_path).encode()


def read_dataset(text_or_path, d: int = 0, strict: bool = False) -> np.ndarray:
    """The whole dataset as an ``n x d`` FP64 array in file order (the ids the reference's
    ``count`` assigns).  ``d = 0``: the first line's field count."""
    raw = _as_bytes(text_or_path)
    n, dd = C.c_int64(), C.c_int32()
    L = lib()
    check(L.hdb_parse_points(raw, len(raw), int(d), int(strict), None, 0, C.byref(n), C.byref(dd)),
          "hdb_parse_points")
    X = np.empty((n.value, dd.value), dtype=np.float64)
    check(L.hdb_parse_points(raw, len(raw), int(d), int(strict), ptr(X), n.value, C.byref(n), C.byref(dd)),
          "hdb_parse_points")
    return X


class MapperDataset_github:
    """PairFunction<String, Integer, Tuple2<Integer, double[]>> (MapperDataset_github.java:6-21):
    ``call(line)`` returns ``(0, (count, point))`` with a running ``count`` from 0."""

    def __init__(self, d: int = 0, strict: bool = True):
        self.count = -1
        self.d = d
        self.strict = strict

    def call(self, s: str):
        X = read_dataset(s.encode(), self.d, self.strict)
        if X.shape[0] != 1:
            raise ValueError("call() takes one line")
        self.count += 1
        return 0, (self.count, X[0])


def format_local_mst(va, vb, w, fake1=None, fake2=None, node=None) -> str:
    """CreateLocalMST.java:110-123 text for one local MST (edges in the given order)."""
    va = np.ascontiguousarray(np.asarray(va), dtype=np.int32)
    vb = np.ascontiguousarray(np.asarray(vb), dtype=np.int32)
    w = np.ascontiguousarray(np.asarray(w), dtype=np.float64)
    ne = va.shape[0]
    if vb.shape[0] != ne or w.shape[0] != ne:
        raise ValueError("va, vb, w must have the same length")
    extra = [None if a is None else np.ascontiguousarray(np.asarray(a), dtype=np.int32) for a in (fake1, fake2, node)]
    for a in extra:
        if a is not None and a.shape[0] != ne:
            raise ValueError("fake1/fake2/node must match the edge count")
    L = lib()
    n = C.c_int64()
    args = [ptr(va), ptr(vb), ptr(w), *[ptr(a) for a in extra], ne]
    check(L.hdb_format_mst_records(*args, None, 0, C.byref(n)), "hdb_format_mst_records")
    buf = C.create_string_buffer(n.value + 1)
    check(L.hdb_format_mst_records(*args, buf, n.value + 1, C.byref(n)), "hdb_format_mst_records")
    return buf.raw[: n.value].decode()


def parse_local_mst(text):
    """UnionFindReducer.java:22-45: the records of one text value as arrays
    ``(va, vb, w, fake1, fake2, node)``."""
    raw = text.encode() if isinstance(text, str) else bytes(text)
    L = lib()
    n = C.c_int64()
    check(L.hdb_parse_mst_records(raw, len(raw), None, None, None, None, None, None, 0, C.byref(n)),
          "hdb_parse_mst_records")
    ne = n.value
    va, vb, f1, f2, nd = (np.empty(ne, np.int32) for _ in range(5))
    w = np.empty(ne, np.float64)
    check(L.hdb_parse_mst_records(raw, len(raw), ptr(va), ptr(vb), ptr(w), ptr(f1), ptr(f2), ptr(nd), ne,
                                  C.byref(n)), "hdb_parse_mst_records")
    return va, vb, w, f1, f2, nd
