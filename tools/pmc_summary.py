"""Summarise rocprofv3 runs into profiles/<tag>_*.json for bench.py / DESIGN.md.

    python tools/pmc_summary.py --trace DIR --fetch DIR --write DIR --out profiles/r01_pmc.json

--trace: a `rocprofv3 --kernel-trace --stats --output-format csv` directory (kernel_stats.csv)
--fetch / --write: `rocprofv3 --pmc FETCH_SIZE` and `--pmc WRITE_SIZE` runs (separate passes:
the two do not fit one pass of the 4 TCC slots).  gfx950 corrections (MI355X_MICROARCH.md,
HBM): FETCH_SIZE is in KiB and reports half the bytes of wide (16 B/lane) streaming reads, so
read bytes = 2 * FETCH_SIZE * 1024; WRITE_SIZE * 1024 is exact for 16 B/lane stores.
The FETCH doubling is exact only for wide coalesced reads; gathers (the render kernels' 4..16 B
per-lane gathers) are uncalibrated, so both the raw and the corrected figure are kept.
"""
import argparse
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

STAGE_OF = [("render_bwd_kernel<true, true>", "render_bwd"), ("render_bwd_kernel<true, false>", "render_bwd:records"),
            ("render_bwd_kernel<false, true>", "render_bwd:nodepth"),
            ("render_bwd_kernel<false, false>", "render_bwd:nodepth_records"),
            ("render_bwd_kernel<true>", "render_bwd"), ("render_bwd_kernel<false>", "render_bwd:nodepth"),
            ("render_bwd_kernel", "render_bwd"), ("render_fwd_seg", "render_fwd:pool"),
            ("render_fwd_cleanup", "render_fwd:cleanup"), ("render_fwd", "render_fwd"),
            ("preprocess_bwd_kernel", "preprocess_bwd"), ("record_sum_kernel", "record_sum"),
            ("preprocess_color_kernel<true", "sh_color:cut"), ("preprocess_color_kernel", "sh_color"),
            ("lod_count_kernel", "lod:count"), ("lod_put_kernel", "lod:put"), ("lod_weights_kernel", "lod:weights"), ("preprocess_kernel", "preprocess"),
            ("depth_gather_kernel", "depth_gather"), ("dsort_upsweep", "depth_sort:upsweep"),
            ("dsort_pass_kernel<0>", "depth_sort:pass0"), ("dsort_pass_kernel<1>", "depth_sort:pass1"),
            ("dsort_pass_kernel<2>", "depth_sort:pass2"), ("dsort_pass_kernel<3>", "depth_sort:pass3"),
            ("sb_count_kernel", "bin_superblocks:count"), ("sb_colscan_kernel", "bin_superblocks:colscan"),
            ("sb_base_kernel", "bin_superblocks:base"), ("sb_scatter_kernel", "bin_superblocks:scatter"),
            ("tile_bin_kernel", "bin_tiles"), ("tile_order_kernel", "tile_order"), ("mark_visible", "mark_visible"),
            ("l1_ssim_fwd", "loss_fwd"), ("l1_ssim_bwd", "loss_bwd"), ("sparse_adam", "adam"),
            ("exposure_", "exposure"), ("densify_stats", "densify"), ("adam_rowlist", "adam:rows"),
            ("adam_compact", "adam:compact"), ("grad_live_list", "grad_live:list"), ("grad_live", "grad_live"),
            ("grad_range", "grad_live"), ("l1_ssim_stream", "loss:ssim_stream")]
# rocPRIM kernels are all `trampoline_kernel<wrapped_<algo>_config<cfg, KeyT, ...>>`: the algorithm
# and key type tell the depth sort (u32 keys over P) from the tile sort (u16 keys over K).
ROCPRIM = re.compile(r"wrapped_(\w+?)_config<[^,]+(?:<[^>]*>)?, (unsigned \w+)")


def stage(name):
    for k, v in STAGE_OF:
        if k in name:
            return v
    m = ROCPRIM.search(name)
    if m:
        algo, key = m.groups()
        if algo == "scan":
            return "depth_sort_scan:scan"
        if "lookback" in name:
            return "rocprim:init_lookback"
        who = "tile_sort" if key == "unsigned short" else "sort_u32"
        return f"{who}:{algo}"
    if "init_lookback" in name:
        return "rocprim:init_lookback"
    return name.replace("(anonymous namespace)::", "").split("(")[0][:60]


def read_pmc(d, counter):
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            vals[stage(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return vals


SQ_COUNTERS = ("SQ_INSTS_VALU", "SQ_INSTS_VALU_TRANS_F32", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM",
               "SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_ANY",
               "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_LDS_BANK_CONFLICT", "SQ_WAIT_INST_LDS", "GRBM_GUI_ACTIVE",
               "SQ_INSTS_VALU_FMA_F32", "SQ_INSTS_VALU_MUL_F32", "SQ_INSTS_VALU_ADD_F32", "TCC_HIT_sum", "TCC_MISS_sum",
               "TCC_EA0_RDREQ_sum", "TCP_TOTAL_CACHE_ACCESSES_sum", "TCP_TCC_READ_REQ_sum")


def read_sq(dirs):
    """Per-launch averages of the SQ / GRBM counters of every stage (several --pmc passes)."""
    out = defaultdict(dict)
    for d in dirs:
        for c in SQ_COUNTERS:
            for s, v in read_pmc(d, c).items():
                out[s][c] = sum(v) / len(v)
    return out


def read_stats(d):
    out = {}
    for f in glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            s = stage(r["Name"])
            e = out.setdefault(s, {"calls": 0, "total_ns": 0.0})
            e["calls"] += int(r["Calls"])
            e["total_ns"] += float(r["TotalDurationNs"])
    for e in out.values():
        e["avg_us"] = e["total_ns"] / max(1, e["calls"]) / 1e3
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace")
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--out", required=True)
    ap.add_argument("--sq", action="append", default=[], help="rocprofv3 --pmc SQ_* pass directories")
    ap.add_argument("--note", default="")
    a = ap.parse_args()
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import kernel_source_sha
    # the kernel sources this profile describes (bench.py reports traffic / rocprof times only from
    # a profile of the sources that run)
    res = {"note": a.note, "source_sha": kernel_source_sha(), "kernels": {}}
    stats = read_stats(a.trace) if a.trace else {}
    fetch = read_pmc(a.fetch, "FETCH_SIZE") if a.fetch else {}
    write = read_pmc(a.write, "WRITE_SIZE") if a.write else {}
    sq = read_sq(a.sq)
    for s in sorted(set(stats) | set(fetch) | set(write) | set(sq)):
        e = dict(stats.get(s, {}))
        if s in fetch:
            f = sum(fetch[s]) / len(fetch[s])
            e["fetch_size_kib_raw"] = f
            e["read_bytes_corrected"] = 2 * f * 1024
        if s in write:
            w = sum(write[s]) / len(write[s])
            e["write_size_kib"] = w
            e["write_bytes"] = w * 1024
        if "read_bytes_corrected" in e and "write_bytes" in e:
            e["hbm_bytes_per_launch"] = e["read_bytes_corrected"] + e["write_bytes"]
        if s in sq:
            e["sq"] = sq[s]
            # VALU issue: a wave64 VALU instruction holds its SIMD for 2 cycles (MI355X_MICROARCH.md,
            # v_fma_f32 row); GRBM_GUI_ACTIVE is summed over the 8 XCDs
            g = sq[s].get("GRBM_GUI_ACTIVE")
            v = sq[s].get("SQ_INSTS_VALU")
            if g and v:
                e["valu_issue_frac"] = v * 2.0 / (1024 * g / 8.0)
        res["kernels"][s] = e
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    json.dump(res, open(a.out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
