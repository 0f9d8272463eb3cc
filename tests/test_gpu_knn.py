"""GPU parity of the nearest-neighbour scale initialisation (csrc/knn.hip, include/gsr_knn.h;
the drop-in simple_knn._C.distCUDA2) with the C restatement gso_knn_mean_dist2 (bit-exact: the
box pruning is conservative and the distance order is shared).  simple-knn itself is not
vendored in the reference, so this row is parity-unpinned against the real extension
(oracle/gs_oracle.c)."""
from __future__ import annotations

import numpy as np
import pytest
import torch

import gs_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _dist(p):
    from simple_knn._C import distCUDA2
    return distCUDA2(torch.tensor(p, device=DEV)).cpu().numpy()


def _street_cloud(n, seed):
    """A LiDAR/SfM-like cloud: a ground plane, two facades and clutter, over a 100 m street."""
    rng = np.random.default_rng(seed)
    k = n // 4
    ground = np.stack([rng.uniform(-50, 50, k), rng.uniform(-8, 8, k), rng.normal(0, 0.02, k)], 1)
    left = np.stack([rng.uniform(-50, 50, k), -8 + rng.normal(0, 0.05, k), rng.uniform(0, 12, k)], 1)
    right = np.stack([rng.uniform(-50, 50, k), 8 + rng.normal(0, 0.05, k), rng.uniform(0, 12, k)], 1)
    rest = rng.normal(0, 3, (n - 3 * k, 3)) * [10, 1, 1]
    return np.concatenate([ground, left, right, rest]).astype(np.float32)


@pytest.mark.parametrize("case", ["normal", "street", "duplicates", "grid"])
def test_knn_matches_oracle_bitwise(case):
    rng = np.random.default_rng(5)
    if case == "normal":
        p = rng.normal(size=(20_000, 3)).astype(np.float32)
    elif case == "street":
        p = _street_cloud(20_000, 6)
    elif case == "duplicates":
        p = rng.normal(size=(5_000, 3)).astype(np.float32)
        p = np.concatenate([p, p[:700], p[:50]])  # repeated positions: zero distances
    else:  # integer lattice: massive ties
        g = np.arange(22, dtype=np.float32)
        p = np.stack(np.meshgrid(g, g, g, indexing="ij"), -1).reshape(-1, 3)
        p = p[rng.permutation(len(p))]
    np.testing.assert_array_equal(_dist(p), O.knn_mean_dist2(p))


@pytest.mark.parametrize("n", [1, 2, 3, 4, 63, 64, 65, 4095, 4097])
def test_knn_small_and_ragged_sizes(n):
    p = np.random.default_rng(n).normal(size=(n, 3)).astype(np.float32)
    np.testing.assert_array_equal(_dist(p), O.knn_mean_dist2(p))


def test_knn_degenerate_extent():
    p = np.zeros((300, 3), np.float32)
    p[:, 0] = np.arange(300)  # all on one axis: zero extent in y and z
    np.testing.assert_array_equal(_dist(p), O.knn_mean_dist2(p))
    assert _dist(np.zeros((0, 3), np.float32)).shape == (0,)


def test_knn_large_cloud_spot_checks():
    """1M points (the bench scene size): every value against the brute force for 3000 queries."""
    p = _street_cloud(1_000_000, 7)
    got = _dist(p)
    q = np.random.default_rng(8).choice(len(p), 3000, replace=False)
    np.testing.assert_array_equal(got[q], O.knn_mean_dist2_at(p, q))
    assert np.isfinite(got).all() and (got >= 0).all()
