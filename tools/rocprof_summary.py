"""Summarise rocprofv3 outputs into profiles/ (committed evidence).

Usage: python tools/rocprof_summary.py <prof_dir> <round_tag> [command] [warm-up launches to skip]
  <prof_dir>/trace/run_kernel_stats.csv          (--kernel-trace --stats)
  <prof_dir>/trace/run_kernel_trace.csv[.gz]     (per-dispatch durations: steady-state averages)
  <prof_dir>/pmc_fetch/run_counter_collection.csv (--pmc FETCH_SIZE, its own pass)
  <prof_dir>/pmc_write/run_counter_collection.csv (--pmc WRITE_SIZE, its own pass)

HBM bytes per launch follow MI355X_MICROARCH.md §HBM: FETCH_SIZE/WRITE_SIZE are KiB; on gfx950
FETCH_SIZE reads half the bytes of a wide (16 B/lane) coalesced stream, so the corrected read
side is 2 x FETCH_SIZE for such kernels.  Our kernels mix widths, so both the raw and the x2
figures are kept; `hbm_bytes_per_launch` uses the raw FETCH (lower bound) + WRITE and
`hbm_bytes_per_launch_fetch_x2` the corrected 2 x FETCH + WRITE (what bench.py reports as traffic).
"""
from __future__ import annotations

import csv
import gzip
import json
import re
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def short(name: str) -> str:
    m = re.search(r"::([A-Za-z0-9_]+)(?:<[^(]*>)?\(", name)
    base = m.group(1) if m else name.split("(")[0]
    return base


VALU_PEAK_G = 1024 * 2.4 / 4.0  # G wave64 VALU instructions / s at one per quad-cycle (the r1-r4 pricing)
N_SIMD = 1024
N_XCD = 8


def valu_busy(insts, dual_quads, grbm):
    """VALU issue occupancy of a launch: each SIMD issues at most one VALU instruction per quad-cycle,
    or two (one from each of two waves) when both are full-rate forms; SQ_ACTIVE_INST_VALU2 counts
    those dual quad-cycles.  Quad-cycles with a VALU issue = SQ_INSTS_VALU - SQ_ACTIVE_INST_VALU2
    (summed over the SIMDs); the launch lasted GRBM_GUI_ACTIVE / 8 cycles (one GRBM per XCD).
    Calibrated on tools/valu_probe.hip (profiles/r5_valu_probe_pmc.md): every pure-VALU loop of the
    47 forms, full- or half-rate, reads 0.93-0.95 (the rest is its loop branch and ramp)."""
    if insts is None or dual_quads is None or not grbm:
        return None
    return (insts - dual_quads) * 4 / N_SIMD / (grbm / N_XCD)

KERNEL_TAG = {
    "fast_nms_kernel": "orb.fast_nms", "select_kernel": "orb.select", "fast_redo_kernel": "orb.fast_redo",
    "select_redo_kernel": "orb.select_redo", "describe_kernel": "orb.describe", "describe_blurred_kernel": "orb.describe",
    "match_kernel": "match.two_way", "match_fp4_kernel": "match.two_way", "build_schur": "ba.build_schur", "cholesky_solve": "ba.cholesky_solve",
    "point_linearize": "ba.point_linearize", "cam_linearize": "ba.cam_linearize",
    "point_backsub": "ba.point_backsub", "edge_schur": "ba.edge_schur", "chol_tiles": "ba.cholesky_solve", "drop_edges": "ba.drop_edges", "export_state": "ba.export_state", "update_state": "ba.update_state",
    "outlier_pass": "ba.outlier_pass", "reduce3": "ba.reduce", "linearize_finish": "ba.linearize_finish",
    "schur_pairs": "ba.schur_pairs", "schur_chunks": "ba.schur_pairs", "schur_finish": "ba.schur_finish",
    "linearize_kernel": "ba.linearize", "update_evaluate": "ba.update_evaluate",
    "tether_eval": "ba.tether_eval", "refresh_membership": "ba.refresh_membership",
    "pose_ba_kernel": "pose.ba", "radius_match_kernel": "match.radius", "radius_post_kernel": "match.radius_post", "indexed_match_kernel": "match.indexed",
    "bow_leaves_kernel": "bow.leaves", "remap_linear_kernel": "image.remap", "remap_boxes_kernel": "image.boxes",
    "undistort_map_kernel": "image.map", "undistort_kernel": "orb.undistort", "synth_scene_kernel": "synth.scene",
    "synth_frames_kernel": "synth.frames", "fast_score_map_kernel": "orb.fast_score", "orient_kernel": "orb.orient",
    "resize_linear_kernel": "orb.resize", "resize_band_kernel": "orb.pyramid", "resize_rows_kernel": "orb.pyramid",
    "orient_rows_kernel": "orb.orient", "radius_band_index_kernel": "match.radius_index",
    "csort_count": "ba.sort_count", "csort_scan": "ba.sort_scan", "csort_scatter": "ba.sort_scatter",
}


def _open(path: Path):
    """The CSV or its gzip (tools/profile_round.sh compresses the counter files on the box)."""
    gz = path.with_name(path.name + ".gz")
    return gzip.open(gz, "rt") if gz.exists() else open(path)


def _exists(path: Path) -> bool:
    return path.exists() or path.with_name(path.name + ".gz").exists()


def read_stats(path: Path):
    rows = []
    with _open(path) as f:
        for r in csv.DictReader(f):
            rows.append({"kernel": short(r["Name"]), "calls": int(r["Calls"]),
                         "avg_us": float(r["AverageNs"]) / 1e3, "total_ms": float(r["TotalDurationNs"]) / 1e6,
                         "pct": float(r["Percentage"])})
    return rows


def read_pmc(path: Path, counter: str, skip: int = 0):
    """Per-kernel mean of `counter` per dispatch, without each kernel's first `skip` dispatches
    (the bench's warm-up launches: the first ORB batch runs without the candidate gate)."""
    per = defaultdict(list)
    if not _exists(path):
        return {}
    with _open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] != counter:
                continue
            per[short(r["Kernel_Name"])].append((int(r.get("Dispatch_Id") or 0), float(r["Counter_Value"])))
    out = {}
    for k, v in per.items():
        v.sort()
        v = v[skip:] if len(v) > skip else v
        out[k] = sum(x for _, x in v) / len(v)
    return out


def read_trace(path: Path, skip: int = 0):
    """Per-kernel (launches, mean duration in us) from the kernel trace, without each kernel's first
    `skip` dispatches — the steady-state launch time bench.py's HIP events measure."""
    per = defaultdict(list)
    if not _exists(path):
        return {}
    with _open(path) as f:
        for r in csv.DictReader(f):
            per[short(r["Kernel_Name"])].append(
                (int(r.get("Dispatch_Id") or 0), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
    out = {}
    for k, v in per.items():
        v.sort()
        v = v[skip:] if len(v) > skip else v
        out[k] = (len(v), sum(x for _, x in v) / len(v))
    return out


def main():
    prof = Path(sys.argv[1])
    tag = sys.argv[2]
    cmd = sys.argv[3] if len(sys.argv) > 3 else "python bench.py"
    skip = int(sys.argv[4]) if len(sys.argv) > 4 else 0  # warm-up launches per kernel to leave out
    out_dir = ROOT / "profiles"
    out_dir.mkdir(exist_ok=True)
    stats = read_stats(prof / "trace" / "run_kernel_stats.csv")
    trace = read_trace(prof / "trace" / "run_kernel_trace.csv", skip)
    fetch = read_pmc(prof / "pmc_fetch" / "run_counter_collection.csv", "FETCH_SIZE", skip)
    write = read_pmc(prof / "pmc_write" / "run_counter_collection.csv", "WRITE_SIZE", skip)
    valu = read_pmc(prof / "pmc_valu" / "run_counter_collection.csv", "SQ_INSTS_VALU", skip)
    mfma = read_pmc(prof / "pmc_valu" / "run_counter_collection.csv", "SQ_VALU_MFMA_BUSY_CYCLES", skip)
    dual = read_pmc(prof / "pmc_valu" / "run_counter_collection.csv", "SQ_ACTIVE_INST_VALU2", skip)
    grbm = read_pmc(prof / "pmc_valu" / "run_counter_collection.csv", "GRBM_GUI_ACTIVE", skip)
    lines = [f"# rocprofv3 summary — {tag}", "",
             "`rocprofv3 --kernel-trace --stats` (durations) and separate `--pmc FETCH_SIZE` / `--pmc WRITE_SIZE` "
             f"passes of `{cmd}` on one MI355X.  KiB counters converted to bytes; FETCH x2 is the "
             "gfx950 wide-stream correction (MI355X_MICROARCH.md §HBM).", "",
             "VALU issue (own pass): `VALU busy` = (SQ_INSTS_VALU - SQ_ACTIVE_INST_VALU2) x 4 / (1024 SIMDs x "
             "GRBM_GUI_ACTIVE / 8) — the quad-cycles in which a SIMD issued VALU work (one instruction, or two "
             "full-rate ones from two waves) over the launch's cycles; tools/valu_probe.hip loops of every "
             "form read 0.93-0.95 (profiles/r5_valu_probe_pmc.md).  `VALU G inst/s` is the raw rate; the "
             "r1-r4 `frac` priced it at one instruction per quad-cycle (614 G/s).", "",
             f"Steady-state columns (avg µs steady, counters) leave out each kernel's first {skip} launches "
             "(the command's warm-up steps; the first ORB batch runs without the candidate gate), from the "
             "per-dispatch kernel trace and counter rows.", "",
             "| kernel | calls | avg µs (all) | avg µs steady | total ms | % | FETCH MB/launch (raw) | FETCH x2 | WRITE MB/launch | VALU G inst/s | VALU busy |",
             "|---|---|---|---|---|---|---|---|---|---|---|"]
    # provenance: the kernel sources the counters were collected on (written on the GPU box by
    # tools/profile_round.sh; bench.py reports traffic only for matching sources)
    sha_file = prof / "sources_sha"
    if sha_file.exists():
        sha = sha_file.read_text().strip()
    else:
        sys.path.insert(0, str(ROOT))
        from mageslam_amd.build import kernel_sources_sha

        sha = kernel_sources_sha()
    summary = {"_meta": {"tag": tag, "kernel_sources_sha": sha, "command": cmd, "skipped_warmup_launches": skip}}
    # per-file hashes, recorded only when this tree is the one the counters were collected on
    sys.path.insert(0, str(ROOT))
    from mageslam_amd.build import kernel_file_shas, kernel_sources_sha as _now_sha

    if _now_sha() == sha:
        summary["_meta"]["kernel_file_shas"] = kernel_file_shas()
    for r in stats:
        k = r["kernel"]
        f = fetch.get(k)
        w = write.get(k)
        fmb = f * 1024 / 1e6 if f is not None else None
        wmb = w * 1024 / 1e6 if w is not None else None
        v = valu.get(k)
        steady = trace[k][1] if k in trace else r["avg_us"]
        vrate = v / (steady * 1e-6) / 1e9 if v is not None and steady > 0 else None
        vfrac = valu_busy(v, dual.get(k), grbm.get(k))
        lines.append(f"| {k} | {r['calls']} | {r['avg_us']:.1f} | {steady:.1f} | {r['total_ms']:.2f} | {r['pct']:.1f} | "
                     f"{'' if fmb is None else f'{fmb:.3f}'} | {'' if fmb is None else f'{2 * fmb:.3f}'} | "
                     f"{'' if wmb is None else f'{wmb:.3f}'} | {'' if vrate is None else f'{vrate:.0f}'} | "
                     f"{'' if vfrac is None else f'{vfrac:.2f}'} |")
        tagname = KERNEL_TAG.get(k)
        if tagname:
            summary[tagname] = {"avg_us": r["avg_us"], "calls": r["calls"], "avg_us_steady": steady,
                                "steady_launches": trace[k][0] if k in trace else None, "skipped_warmup_launches": skip,
                                "fetch_bytes_per_launch": None if f is None else f * 1024,
                                "write_bytes_per_launch": None if w is None else w * 1024,
                                "hbm_bytes_per_launch": None if (f is None or w is None) else (f + w) * 1024,
                                "hbm_bytes_per_launch_fetch_x2": None if (f is None or w is None) else (2 * f + w) * 1024,
                                "valu_insts_per_launch": v, "valu_busy": vfrac,
                                "valu_dual_quads_per_launch": dual.get(k), "grbm_gui_active_per_launch": grbm.get(k),
                                "mfma_busy_cycles_per_launch": mfma.get(k)}
    (out_dir / f"{tag}_rocprof.md").write_text("\n".join(lines) + "\n")
    (out_dir / f"{tag}_pmc_summary.json").write_text(json.dumps(summary, indent=1))
    print("\n".join(lines))


if __name__ == "__main__":
    main()
