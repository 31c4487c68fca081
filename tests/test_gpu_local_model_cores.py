"""hdb_local_model_cores (round 6): the local model from bubble cores computed beforehand by
hdb_bubble_core_distances equals hdb_local_model (labels, quicksorted MST, inter-cluster edges) --
the driver's cores-first schedule relies on it (LocalModelReduceByKey.java:88-104)."""
import importlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def A():
    importlib.import_module("232-hierarchical-density-based-clustering-using-mapreduce_amd")
    return importlib.import_module("232-hierarchical-density-based-clustering-using-mapreduce_amd._capi")


def run(A, ctx, rep, info, core, min_pts, mcs):
    b, d = rep.shape
    ne = 2 * b - 1
    lab = np.zeros(b, np.int32)
    mva, mvb, mw = np.zeros(ne, np.int32), np.zeros(ne, np.int32), np.zeros(ne)
    iva, ivb, iw = np.zeros(ne, np.int32), np.zeros(ne, np.int32), np.zeros(ne)
    nic = np.zeros(1, np.int64)
    if core is None:
        rc = A.lib().hdb_local_model(ctx.h, A.ptr(rep), A.ptr(info), b, d, min_pts, mcs, 0, A.ptr(lab), A.ptr(mva),
                                     A.ptr(mvb), A.ptr(mw), A.ptr(iva), A.ptr(ivb), A.ptr(iw), A.ptr(nic))
    else:
        rc = A.lib().hdb_local_model_cores(ctx.h, A.ptr(rep), A.ptr(info), b, d, min_pts, mcs, 0, A.ptr(core),
                                           A.ptr(lab), A.ptr(mva), A.ptr(mvb), A.ptr(mw), A.ptr(iva), A.ptr(ivb),
                                           A.ptr(iw), A.ptr(nic))
    k = int(nic[0])
    return rc, lab, mva, mvb, mw.view(np.uint64), iva[:k], ivb[:k], iw[:k].view(np.uint64)


@pytest.mark.parametrize("b,d,min_pts,mcs,rounded", [(2, 3, 2, 2, False), (300, 3, 4, 4, True),
                                                     (2500, 8, 4, 4, False), (5000, 2, 9, 8, True)])
def test_local_model_cores_equal(A, b, d, min_pts, mcs, rounded):
    rng = np.random.default_rng(b + d)
    ctr = rng.uniform(-20, 20, (12, d))
    rep = ctr[rng.integers(0, 12, b)] + rng.normal(0, 1, (b, d))
    if rounded:  # ties in the distances and the cores
        rep = np.round(rep)
    info = np.stack([rng.uniform(0.1, 1.0, b), rng.uniform(0.05, 0.5, b),
                     rng.integers(1, 40, b).astype(float)], 1)
    if rounded:
        info[:, :2] = np.round(info[:, :2], 1)
    rep, info = np.ascontiguousarray(rep), np.ascontiguousarray(info)
    ctx = A.Context.get(0)
    nB = np.ascontiguousarray(info[:, 2].astype(np.int32))
    core = np.zeros(b)
    assert A.lib().hdb_bubble_core_distances(ctx.h, A.ptr(rep), A.ptr(nB), A.ptr(np.ascontiguousarray(info[:, 0])),
                                             A.ptr(np.ascontiguousarray(info[:, 1])), b, d, min_pts, 0,
                                             A.ptr(core)) == 0
    ref = run(A, ctx, rep, info, None, min_pts, mcs)
    got = run(A, ctx, rep, info, core, min_pts, mcs)
    assert ref[0] == got[0]
    for x, y in zip(ref[1:], got[1:]):
        assert np.array_equal(x, y)


def test_local_model_cores_requires_core(A):
    ctx = A.Context.get(0)
    rep, info = np.zeros((4, 2)), np.ones((4, 3))
    lab = np.zeros(4, np.int32)
    assert A.lib().hdb_local_model_cores(ctx.h, A.ptr(rep), A.ptr(info), 4, 2, 2, 2, 0, None, A.ptr(lab), None, None,
                                         None, None, None, None, None) != 0
