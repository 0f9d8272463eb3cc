"""CPU checks of the hierarchy LOD cut restatement (oracle/gs_oracle.c gso_expand_to_size /
gso_interpolation_weights, the checker for csrc/lod.hip) and of the synthetic tree the config-5
workload uses (gs_train/synthetic.py synthetic_lod_hierarchy).

gaussianhierarchy is not vendored in the reference, so parity against the extension itself is
UNPINNED; what is pinned here: the C restatement equals a direct pure-Python transcription of the
published cut on small trees, and the cut has the defining property of an LOD cut on a tree
whose projected sizes shrink towards the leaves -- every leaf is covered by exactly one rendered
node."""
from __future__ import annotations

import math
import os

import numpy as np
import pytest
import torch

import gs_oracle as O
from gs_train.synthetic import synthetic_lod_hierarchy, tau_threshold


def _py_size(b, v):
    if all(b[k] <= v[k] <= b[4 + k] for k in range(3)):
        return np.float32(np.finfo(np.float32).max)
    c = [np.float32(max(b[k], min(b[4 + k], v[k]))) for k in range(3)]
    d = [np.float32(v[k] - c[k]) for k in range(3)]
    s = np.float32(np.float32(d[0] * d[0]) + np.float32(d[1] * d[1]))
    s = np.float32(s + np.float32(d[2] * d[2]))
    return np.float32(b[3] / np.float32(math.sqrt(s)))


def _py_cut(nodes, boxes, target, v):
    """Pure-Python transcription of the published expand_to_size / get_interpolation_weights."""
    ri, pi, ni = [], [], []
    for i, n in enumerate(nodes):
        s = _py_size(boxes[i], v)
        if s >= target:
            c = n[3]
        elif n[1] < 0 or _py_size(boxes[n[1]], v) >= target:
            c = n[3] + n[4]
        else:
            c = 0
        for k in range(c):
            ri.append(n[2] + k)
            pi.append(-1 if n[1] < 0 else nodes[n[1]][2])
            ni.append(i)
    w, kids = [], []
    for i in ni:
        p = nodes[i][1]
        t, kk = np.float32(1.0), 1
        if p >= 0:
            kk = nodes[p][6]
            sp = _py_size(boxes[p], v)
            if not sp > np.float32(2.0) * target:
                s = _py_size(boxes[i], v)
                s0 = max(np.float32(0.5) * sp, s)
                diff = np.float32(sp - s0)
                if diff > 0:
                    tdiff = max(np.float32(0.0), np.float32(target - s0))
                    t = max(np.float32(np.float32(1.0) - np.float32(tdiff / diff)), np.float32(0.0))
        w.append(t)
        kids.append(kk)
    return (np.array(ri, np.int32), np.array(pi, np.int32), np.array(ni, np.int32), np.array(w, np.float32),
            np.array(kids, np.int32))


@pytest.fixture(scope="module")
def tree():
    h = synthetic_lod_hierarchy(3000, 640, 360, "cpu", seed=3, branching=4, skybox=7, zmin=0.5, zmax=6.0,
                                log_scale_mean=-3.0)
    return h, h["nodes"].numpy(), h["boxes"].reshape(-1, 8).numpy()


def test_synthetic_tree_is_consistent(tree):
    h, nodes, boxes = tree
    N = nodes.shape[0]
    assert h["means3D"].shape[0] == N + 7 and nodes[0, 1] == -1 and (nodes[1:, 1] >= 0).all()
    np.testing.assert_array_equal(nodes[:, 2], np.arange(N))
    for i in range(N):
        d, p, start, cl, cm, sc, cc = nodes[i]
        assert cl + cm == 1
        if cc:
            kids = np.arange(sc, sc + cc)
            assert (nodes[kids, 1] == i).all() and (nodes[kids, 0] == d + 1).all()
            assert (boxes[kids, :3] >= boxes[i, :3]).all() and (boxes[kids, 4:7] <= boxes[i, 4:7]).all()
            assert (boxes[kids, 3] <= boxes[i, 3]).all()
        else:
            assert cl == 1 and cm == 0


@pytest.mark.parametrize("tau,vp", [(0.0, None), (6.0, None), (40.0, None), (120.0, (0.2, -0.1, 1.5)),
                                    (15.0, (100.0, 0.0, 0.0))])
def test_cut_oracle_matches_python_and_covers_every_leaf_once(tree, tau, vp):
    h, nodes, boxes = tree
    v = np.asarray(h["campos"] if vp is None else vp, np.float32)
    thr = np.float32(tau_threshold(tau, h["tanfovx"], h["W"]))
    ri, pi, ni = O.expand_to_size(nodes, boxes, thr, v)
    w, k = O.interpolation_weights(ni, thr, nodes, boxes, v)
    pri, ppi, pni, pw, pk = _py_cut(nodes.tolist(), boxes.tolist(), thr, v.tolist())
    for a, b in ((ri, pri), (pi, ppi), (ni, pni), (w, pw), (k, pk)):
        np.testing.assert_array_equal(a, b)
    # LOD-cut property: the rendered nodes' subtrees partition the leaves
    N = nodes.shape[0]
    leaf_of = np.zeros(N, np.int64)
    covered = np.zeros(N, np.int64)
    for i in range(N - 1, -1, -1):  # children are stored after their parents
        if nodes[i, 6] == 0:
            leaf_of[i] = 1
        if nodes[i, 1] >= 0:
            leaf_of[nodes[i, 1]] += leaf_of[i]
    assert leaf_of[0] == int((nodes[:, 6] == 0).sum())
    covered[ni] = leaf_of[ni]
    assert covered.sum() == leaf_of[0]
    assert len(np.unique(ni)) == len(ni)
    assert ((w >= 0) & (w <= 1)).all() and (w[pi < 0] == 1).all()
    assert (ri == ni).all()  # one Gaussian per node, Gaussian i belongs to node i


def test_viewpoint_inside_root_box_expands_to_leaves(tree):
    h, nodes, boxes = tree
    v = 0.5 * (boxes[0, :3] + boxes[0, 4:7])  # inside every enclosing box: infinite projected size
    ri, pi, ni = O.expand_to_size(nodes, boxes, np.float32(1.0), v)
    # every node whose box contains v is expanded; everything else is cut at its first small node
    assert 0 not in set(ni.tolist())


def test_hier_file_round_trip(tmp_path):
    """gaussian_hierarchy.load_hierarchy / write_hierarchy (scene/gaussian_model.py:347, 437-445):
    the uncompressed .hier layout restated in _C.py (parity-unpinned: the gaussianhierarchy writer
    is not vendored and no reference-written file is available) -- round trip, exact byte size, and
    loud failures for the compressed variant and for trailing bytes."""
    import numpy as np
    import torch
    from gaussian_hierarchy._C import load_hierarchy, write_hierarchy
    rng = np.random.default_rng(3)
    P, N = 1000, 400
    xyz = torch.tensor(rng.normal(size=(P, 3)), dtype=torch.float32)
    shs = torch.tensor(rng.normal(size=(P, 16, 3)), dtype=torch.float32)
    opac = torch.tensor(rng.random((P, 1)), dtype=torch.float32)
    scales = torch.tensor(rng.normal(-4, 1, size=(P, 3)), dtype=torch.float32)
    rots = torch.tensor(rng.normal(size=(P, 4)), dtype=torch.float32)
    nodes = torch.tensor(rng.integers(-1, P, size=(N, 7)), dtype=torch.int32)
    boxes = torch.tensor(rng.normal(size=(N, 2, 4)), dtype=torch.float32)
    path = str(tmp_path / "h.hier")
    write_hierarchy(path, xyz, shs, opac, scales, rots, nodes, boxes)
    assert os.path.getsize(path) == 4 + P * (3 + 4 + 3 + 1 + 48) * 4 + 4 + N * 7 * 4 + N * 8 * 4
    got = load_hierarchy(path)
    for a, b in zip(got, (xyz, shs, opac, scales, rots, nodes, boxes)):
        assert a.shape == b.shape and a.dtype == b.dtype and torch.equal(a, b)
    raw = open(path, "rb").read()
    with open(path, "wb") as f:
        f.write(np.int32(-P).tobytes() + raw[4:])
    with pytest.raises(NotImplementedError):
        load_hierarchy(path)
    with open(path, "wb") as f:
        f.write(raw + b"\0\0\0\0")
    with pytest.raises(ValueError):
        load_hierarchy(path)
