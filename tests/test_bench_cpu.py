"""bench.py's line-shaping helpers on the CPU: the roofline's algorithmic bytes follow SURVEY.md 8(d)
for render_bwd (44 K + 24 Npix + 40 Pv; the dense zero gradient rows are booked under
preprocess_bwd), and the secondary legs' prose moves to the detail file while their numbers stay."""
from __future__ import annotations

import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def test_render_bwd_bytes_are_survey_8d():
    import bench
    P, Pv, K, T, npix, P1 = 1_000_000, 900_000, 13_885_166, 8160, 1920 * 1080, 2_624_626
    b = bench.algorithmic_bytes(P, Pv, K, T, npix, P1, M=16, Pl=38_637)
    assert b["render_bwd"] == 44 * K + 24 * npix + 40 * Pv
    assert b["render_fwd"] == 44 * K + 24 * npix
    # the zero rows (56 + 12 M B per Gaussian) are in preprocess_bwd's figure
    b0 = bench.algorithmic_bytes(P, Pv, K, T, npix, P1, M=16, Pl=0)
    assert b0["preprocess_bwd"] == 4 * P + (56 + 12 * 16) * P


def test_compact_legs_moves_prose_only():
    import bench
    out = {"metric": "m", "config": {"workload": "kept"},
           "config5": {"ms_per_frame": 3.5, "workload": "long text", "data": "d",
                       "render_post_order": {"ms_per_frame": 4.0, "workload": "w2", "raster_stages_ms": {"a": 1}}},
           "config3_proxy": {"chunk_wall_s": 50.0, "iteration_ms": {"mean": 1.7, "source": "events"}}}
    detail = {}
    bench.compact_legs(out, detail)
    assert out["config"]["workload"] == "kept"  # the metric's own config keeps its workload
    assert out["config5"] == {"ms_per_frame": 3.5, "render_post_order": {"ms_per_frame": 4.0}}
    assert out["config3_proxy"] == {"chunk_wall_s": 50.0, "iteration_ms": {"mean": 1.7}}
    assert detail["prose"]["config5.workload"] == "long text"
    assert detail["prose"]["config3_proxy.iteration_ms.source"] == "events"
    assert detail["config5_render_post_order_stages_ms"] == {"a": 1}


def test_compact_legs_moves_descriptive_numbers():
    import bench
    out = {"config3_proxy": {"chunk_wall_s": 50.0, "seed": 0, "P_init": 330000,
                             "variant": {"spatial_rows": True, "chunk_wall_s": 49.4, "slowest3": [[1, 2.0]]}},
           "config5": {"ms_per_frame": 3.3, "nodes": 50, "raster_stages_ms": {"render_fwd": 0.4, "render_bwd": 0.0}},
           "config": {"gaussians": 1}}
    detail = {}
    bench.compact_legs(out, detail)
    assert out["config3_proxy"] == {"chunk_wall_s": 50.0, "variant": {"spatial_rows": True, "chunk_wall_s": 49.4}}
    assert out["config5"] == {"ms_per_frame": 3.3, "raster_stages_ms": {"render_fwd": 0.4}}
    assert out["config"] == {"gaussians": 1}  # the metric's own config is never touched
    assert detail["moved"]["config3_proxy.variant.slowest3"] == [[1, 2.0]] and detail["moved"]["config5.nodes"] == 50


def test_dispersion_of_step_times():
    import bench
    d = bench.dispersion([0.65, 0.66, 0.70, 0.64, 0.90])
    assert d["median_ms"] == 0.66 and d["min_ms"] == 0.64 and d["max_ms"] == 0.9 and d["n"] == 5
    assert bench.dispersion([]) is None
