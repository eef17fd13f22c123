#!/usr/bin/env python3
"""bench.py — MAGE-SLAM hot path on MI355X: ORB extract + match @720p (headline) and local-BA
iterations (50 KF x 5000 pts), with roofline and CPU-baseline fields.

Step = one batch of B synthetic 1280x720 frames (resident in HBM before timing): ORB extraction
(FAST/NMS -> retain/ANMS -> blur+rBRIEF) of every frame and the two-way Hamming match of each
frame against its predecessor (SURVEY.md §8(d) unit of work).  Multi-GPU (C5): one independent
sequence per rank (seed + rank), no collective in the data path ("scaling": "weak"); after the
timed region rank 0 gathers each rank's per-frame (keypoints, matches) summary over RCCL.

Launch: python bench.py [--gpus 1 --steps K --warmup W]; for N > 1 via torch.distributed.run.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

import numpy as np  # noqa: E402

METRIC = "frames/sec ORB extract+match @720p; local-BA iters/sec (50 KF, 5k pts)"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md: 8.0 TB/s; 6.29 measured)
FP64_PEAK_TFLOPS = 78.6  # MI355X fp64 (vector = matrix), SURVEY.md §8(d)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--batch", type=int, default=256, help="frames per step")
    p.add_argument("--frames", type=int, default=1024, help="resident sequence length per rank")
    p.add_argument("--width", type=int, default=1280)
    p.add_argument("--height", type=int, default=720)
    p.add_argument("--features", type=int, default=2000)
    p.add_argument("--ba-iters", type=int, default=30)
    p.add_argument("--ba-warmup", type=int, default=3)
    p.add_argument("--no-ba", action="store_true")
    p.add_argument("--pose-problems", type=int, default=2048, help="pose-only BA problems per launch")
    p.add_argument("--pose-iters", type=int, default=20)
    p.add_argument("--no-pose", action="store_true")
    p.add_argument("--track-frames", type=int, default=1000, help="C4 tracking-loop sequence length (SURVEY §8(d))")
    p.add_argument("--track-warmup", type=int, default=16, help="C4 warm-up frames (untimed run before the timed one)")
    p.add_argument("--track-parity-frames", type=int, default=600, help="frames of the C4 oracle parity run (>= 6 local-BA windows)")
    p.add_argument("--no-local-ba", action="store_true", help="C4 without the local BA after each keyframe")
    p.add_argument("--track-depth-noise", type=float, default=0.02,
                   help="C4 depth-error leg: new map points' depth error (rms fraction; 0: leg off)")
    p.add_argument("--no-tracking", action="store_true")
    p.add_argument("--trajectory-csv", default="", help="rank 0 writes the gathered trajectories (ExportFossilCsv)")
    p.add_argument("--cpu-sample-s", type=float, default=12.0, help="budget per CPU baseline leg")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--streams", type=int, default=1,
                   help="HIP streams the ORB batches are pipelined over (the headline uses 1: with overlapping "
                        "batches the per-kernel durations behind the roofline stretch)")
    p.add_argument("--pipelined-streams", type=int, default=2,
                   help="also report the ORB rate pipelined over this many streams (0: skip; 1 GPU runs only)")
    p.add_argument("--no-all-cores", action="store_true", help="skip the all-host-cores CPU baselines")
    p.add_argument("--no-rbrief31", action="store_true", help="skip the rBRIEF-31 variant leg")
    p.add_argument("--rbrief31-steps", type=int, default=10)
    p.add_argument("--orb-variant", default="c2", choices=["c2", "rbrief31"],
                   help="profiling only: the variant the ORB leg runs (the headline is c2)")
    p.add_argument("--ba-many-child", action="store_true", help=argparse.SUPPRESS)
    p.add_argument("--profile", type=int, default=1, help="per-kernel HIP-event timing in the timed region")
    p.add_argument("--batch-parity", type=int, default=4,
                   help="frames of the last timed ORB batch checked against the oracle (0: off)")
    p.add_argument("--cpu-dry-run", action="store_true", help="gloo rehearsal of the multi-rank flow (tests)")
    p.add_argument("--rehearse-one-gpu", action="store_true",
                   help="multi-rank rehearsal on a one-GPU box: every rank on cuda:0, gloo collectives (the flow "
                        "of the C5 configuration; times are not a scaling measurement)")
    return p.parse_args()


def orb_bytes_per_frame(w, h, n):
    # frame read + keypoint/descriptor write + two descriptor-set reads + matches
    return w * h + n * (28 + 32) + 2 * n * 32 + n * 16


def ba_flops(g, trials_per_iter):
    """F = 330 E + trials * (sum_p [40 + 144 f_p + 108 f_p (f_p + 1)] + n^3/3 + 2 n^2)."""
    free = g.fixed[g.cam] == 0
    f_p = np.bincount(g.pt[free], minlength=len(g.points)).astype(np.float64)
    n = 6 * int((g.fixed == 0).sum())
    schur = float(np.sum(40 + 144 * f_p + 108 * f_p * (f_p + 1)))
    return 330.0 * len(g.cam) + trials_per_iter * (schur + n ** 3 / 3 + 2 * n ** 2)


# the source files a kernel tag is built from (a committed summary's counters stay valid for the
# kernel while these are unchanged)
KERNEL_FILES = {
    "orb.": ["orb.hip", "orb_tables.hpp", "lds_sort.hpp", "common.hpp"],
    "match.": ["match.hip", "radius.hip", "band_index.hpp", "lds_sort.hpp", "common.hpp"],
    "ba.": ["ba.hip", "ba_math.hpp", "common.hpp"],
    "pose.": ["pose.hip", "ba_math.hpp", "common.hpp"],
}


def load_pmc(kernel, field="hbm_bytes_per_launch", summary="pmc_summary.json"):
    """(`field` of `kernel`, provenance) from a committed rocprofv3 PMC summary (default: HBM
    bytes per launch of the ORB-only profile; pmc_summary_ba.json: the full bench profile, which
    holds the BA kernels).  The summary records the hash of the kernel sources it was collected on;
    counters of other sources are stale and not reported (None)."""
    from mageslam_amd.build import kernel_sources_sha

    f = ROOT / "profiles" / summary
    if not f.exists():
        return None, "no committed PMC summary"
    try:
        d = json.loads(f.read_text())
    except Exception as e:
        return None, f"unreadable PMC summary ({e})"
    meta = d.get("_meta", {})
    sha, now = meta.get("kernel_sources_sha"), kernel_sources_sha()
    files = next((v for k, v in KERNEL_FILES.items() if kernel.startswith(k)), None)
    fshas = meta.get("kernel_file_shas")
    if sha != now and fshas and files:
        # the whole tree changed since the profile, but maybe not this kernel's own sources
        from mageslam_amd.build import kernel_file_shas

        cur = kernel_file_shas()
        changed = [f for f in files if fshas.get(f) != cur.get(f)]
        if not changed:
            return d.get(kernel, {}).get(field), \
                f"profiles/{summary} ({meta.get('tag')}, kernel sources {sha}; {', '.join(files)} unchanged since)"
        return None, f"stale: {', '.join(changed)} changed since profiles/{summary} ({meta.get('tag')})"
    if sha != now:
        return None, f"stale: profiles/{summary} was collected on kernel sources {sha}, these are {now}"
    return d.get(kernel, {}).get(field), \
        f"profiles/{summary} ({meta.get('tag')}, kernel sources {sha})"


def cpu_orb_baseline(args, budget_s, okw=None):
    from mageslam_amd import synth
    from oracle import oracle as O

    s = O.default_settings(args.features, **(okw or {}))
    _, _, prev = O.orb_detect(synth.frame(0, args.width, args.height), s)  # untimed warm-up
    n_timed, el = 0, 0.0
    while el < budget_s or n_timed < 2:
        img = synth.frame(n_timed + 1, args.width, args.height)  # frame synthesis is not timed
        t0 = time.perf_counter()
        _, _, d = O.orb_detect(img, s)
        O.match(d, prev, max_distance=30, min_difference=1)
        el += time.perf_counter() - t0
        prev = d
        n_timed += 1
    return {"value": n_timed / el, "unit": "frames/s", "cores": 1, "kind": "port", "build": ORACLE_BUILD[0],
            "sample": f"{n_timed} consecutive {args.width}x{args.height} synthetic frames, oracle "
                      f"extract ({args.features} features{', ' + str(okw) if okw else ''}) + match vs previous "
                      f"frame, single thread, {el:.1f} s"}


def host_info() -> dict:
    """The host the CPU baselines ran on (record nproc and the CPU model)."""
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"cpu_model": model, "nproc": os.cpu_count(), "usable_cores": len(os.sched_getaffinity(0))}


def median_of(fn, budget_s, k=5):
    """the median of k samples of a CPU baseline leg, each with budget_s / k."""
    runs = [fn(budget_s / k) for _ in range(k)]
    vals = [r["value"] for r in runs]
    med = sorted(range(k), key=lambda i: vals[i])[k // 2]
    return dict(runs[med], statistic=f"median of {k} samples", samples=vals, host=host_info(), build=ORACLE_BUILD[0])


def host_threads(cap: int = 16) -> int:
    """The host cores the all-cores CPU legs use: the box's CPU share for one GPU, 16 (the GPU
    pool's rule for one-GPU boxes: worker pools sized to 16, OMP_NUM_THREADS=16), or fewer when
    the affinity mask allows fewer.  nproc / usable cores are recorded beside it (host_info).
    cap = 32 gives the second figure the legs report: one GPU's share of a 256-core 8-GPU node."""
    return max(1, min(cap, len(os.sched_getaffinity(0))))


NODE_SHARE_THREADS = 32  # 256 host cores / 8 GPUs


# the oracle build the CPU legs time (bench.py switches to the -march=native + SSE2-FAST build
# before the first CPU leg: SURVEY.md §8(d), and the reference's x64 build runs SSE2 FAST)
ORACLE_BUILD = ["portable"]


def use_native_oracle():
    from oracle import oracle as O

    ORACLE_BUILD[0] = O.use_native_build()


def _per_thread(fn, n):
    """Run fn(worker) on n threads (the oracle's ctypes calls release the GIL); returns the list
    of (units, timed seconds).  The aggregate rate is the sum of the per-thread rates, each
    measured while all n threads run."""
    from concurrent.futures import ThreadPoolExecutor

    with ThreadPoolExecutor(n) as ex:
        return list(ex.map(fn, range(n)))


def cpu_orb_baseline_all(args, budget_s, n=None):
    """the oracle on all host cores, frames in parallel (one detector per thread,
    each matching against its own previous frame)."""
    from mageslam_amd import synth
    from oracle import oracle as O

    n = n or host_threads()
    s = O.default_settings(args.features)
    frames = [synth.frame(i, args.width, args.height) for i in range(n + 1)]  # not timed

    def work(w):
        _, _, prev = O.orb_detect(frames[w], s)
        k, el, i = 0, 0.0, 1
        while el < budget_s or k < 2:
            t0 = time.perf_counter()
            _, _, d = O.orb_detect(frames[w + i], s)
            O.match(d, prev, max_distance=30, min_difference=1)
            el += time.perf_counter() - t0
            prev, i, k = d, 1 - i, k + 1
        return k, el

    res = _per_thread(work, n)
    return {"value": sum(k / el for k, el in res), "unit": "frames/s", "cores": n, "kind": "port",
            "build": ORACLE_BUILD[0],
            "sample": f"{n} threads, each alternating two consecutive {args.width}x{args.height} synthetic frames "
                      f"(extract + match vs its previous frame) for ~{budget_s:.0f} s; {sum(k for k, _ in res)} "
                      f"frames in total; sum of per-thread rates"}


# rBRIEF-31 variant (OpenCVModified.cpp:833, 867-871): 4 pyramid levels,
# 31x31 patches, intensity-centroid orientation
RBRIEF31 = dict(nlevels=4, patchSize=31, useOrientation=True)
RBRIEF31_ORACLE = dict(nlevels=4, patch_size=31, use_orientation=1)


def pyramid_level_bytes(w, h, levels, scale=1.5):
    """Bytes of pyramid levels 1.. (OpenCVModified.cpp:785-842: size = cvRound(W / scale^l))."""
    return sum(int(round(w / scale ** l)) * int(round(h / scale ** l)) for l in range(1, levels))


ROOF_KERNEL = "orb.fast_nms"  # the ORB step's dominant kernel (C2 and rBRIEF-31), priced by the roofline


def verify_orb_batch(args, batch_frames, ring, b, out, variant):
    """Frames 1..k of the last timed batch (gated FAST, B frames per launch) against the oracle:
    keypoints (28-byte records), descriptors and the two-way matches against frame j - 1, byte
    for byte.  Runs after the timed region on the results the timed launches left in the ring."""
    import numpy as np

    from oracle import oracle as O

    k = min(args.batch_parity, args.batch - 1)
    N = args.features
    s = O.default_settings(N, **(RBRIEF31_ORACLE if variant == "rbrief31" else {}))
    fr = batch_frames[:k + 1].cpu().numpy()
    kp = ring["kp"][b + 1:b + k + 2].cpu().numpy()
    de = ring["desc"][b + 1:b + k + 2].cpu().numpy()
    cn = ring["cnt"][b + 1:b + k + 2].cpu().numpy()
    mt, nm = out["mt"][:k + 1].cpu().numpy(), out["nm"][:k + 1].cpu().numpy()
    ores = [O.orb_detect(fr[j], s) for j in range(k + 1)]
    kp_ok = de_ok = m_ok = True
    for j in range(1, k + 1):
        _, okp, od = ores[j]
        n = int(cn[j])
        kp_ok &= n == len(okp) and np.array_equal(kp[j, :28 * n], okp.view(np.uint8).reshape(-1))
        de_ok &= np.array_equal(de[j, :n], od)
        om = O.match(od, ores[j - 1][2], max_distance=30, min_difference=1)
        m_ok &= int(nm[j]) == len(om) and np.array_equal(mt[j, :16 * int(nm[j])], om.view(np.uint8).reshape(-1))
    return {"frames": k, "batch": args.batch, "keypoints_identical": bool(kp_ok),
            "descriptors_identical": bool(de_ok), "matches_identical": bool(m_ok),
            "what": f"frames 1..{k} of the last timed {args.batch}-frame batch (gated FAST) vs the CPU oracle, "
                    f"byte for byte; matches against frame j - 1 of the same batch"}


def run_orb(args, rank, world, local_rank, torch, dist, variant=None):
    from mageslam_amd import _lib, matcher, multigpu, orb, synth

    W, H, N, B = args.width, args.height, args.features, args.batch
    F = max(B, (args.frames // B) * B)
    dev = torch.device("cuda", local_rank)
    stream = torch.cuda.current_stream(dev).cuda_stream
    # batches are pipelined over NSTR HIP streams (one detector each: its scratch is per detector):
    # batch s+1's FAST pass overlaps batch s's latency-bound select / describe / match kernels.
    NSTR = max(1, args.streams)
    det_kw = RBRIEF31 if variant == "rbrief31" else {}
    dets = [orb.OrbDetector(nfeatures=N, device=local_rank, **det_kw) for _ in range(NSTR)]
    det = dets[0]
    frames = torch.empty((F, H, W), dtype=torch.uint8, device=dev)
    orb.synth_frames_device(frames, F, W, H, 0, multigpu.sequence_seed(synth.FRAME_SEED, rank), stream=stream)
    torch.cuda.synchronize(dev)
    # The features live in one ring of RING batches (+ one slot): batch s in slots [b + 1, b + B]
    # with b = (s % RING) * B, so slot b holds the previous batch's last frame and the match reads
    # it in place; only when the ring wraps does that frame move to slot 0 (one copy per RING
    # batches instead of three per batch).  With several streams the only cross-stream waits are
    # batch s-1's extraction (its last frame) and the reuse of the ring slots (batches s-RING,
    # s-RING+1 matched).
    RING = 8
    ring = dict(kp=torch.zeros((RING * B + 1, N * 28), dtype=torch.uint8, device=dev),
                desc=torch.zeros((RING * B + 1, N, 32), dtype=torch.uint8, device=dev),
                cnt=torch.zeros(RING * B + 1, dtype=torch.int32, device=dev))
    outs = [dict(mt=torch.zeros((B, N * 16), dtype=torch.uint8, device=dev),
                 nm=torch.zeros(B, dtype=torch.int32, device=dev)) for _ in range(NSTR)]
    streams = [torch.cuda.current_stream(dev)] if NSTR == 1 else [torch.cuda.Stream(dev) for _ in range(NSTR)]
    ev_x = [torch.cuda.Event() for _ in range(RING)]  # extraction of the batch at ring index i done
    ev_m = [torch.cuda.Event() for _ in range(RING)]  # match of the batch at ring index i done

    def step(s):
        start = (s * B) % F
        fr = frames[start:start + B]
        st = streams[s % NSTR]
        d = dets[s % NSTR]
        O = outs[s % NSTR]
        b = (s % RING) * B  # ring base: slot b = the previous batch's last frame
        K, D, Cn = ring["kp"], ring["desc"], ring["cnt"]
        with torch.cuda.stream(st):
            if NSTR > 1:
                for q in (s - RING, s - RING + 1):  # the slots this batch overwrites are read
                    if q >= 0:
                        st.wait_event(ev_m[q % RING])
            d.detect_and_compute_batch_device(fr, W, H, K[b + 1:b + B + 1], D[b + 1:b + B + 1], Cn[b + 1:b + B + 1], N,
                                              stream=st.cuda_stream)
            ev_x[s % RING].record(st)
            if NSTR > 1 and s > 0:
                st.wait_event(ev_x[(s - 1) % RING])  # the previous batch's last frame is extracted
            if b == 0 and s > 0:  # the ring wrapped: the previous batch's last frame to slot 0
                K[0].copy_(K[RING * B])
                D[0].copy_(D[RING * B])
                Cn[0:1].copy_(Cn[RING * B:RING * B + 1])
            matcher.match_batch_device(D[b + 1:b + B + 1], N * 32, Cn[b + 1:b + B + 1], D[b:b + B], N * 32, Cn[b:b + B],
                                       B, 30, 1, O["mt"], N, O["nm"], stream=st.cuda_stream)
            ev_m[s % RING].record(st)

    for s in range(args.warmup):
        step(s)
    torch.cuda.synchronize(dev)
    for d in dets:
        d.device_status()
    lib = _lib.load()
    # the timed region times only the roofline kernel's launches (dispatch timestamps: an event
    # pair on every launch of the step cost ~3 % of the step); the per-kernel breakdown comes from
    # one more pass of the same steps after it
    if args.profile:
        lib.mage_profile_reset()
        lib.mage_profile_filter(ROOF_KERNEL.encode())
        lib.mage_profile_enable(1)
    multigpu.barrier(dist)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for s in range(args.warmup, args.warmup + args.steps):
        step(s)
    torch.cuda.synchronize(dev)
    multigpu.barrier(dist)
    el = time.perf_counter() - t0
    lib.mage_profile_enable(0)
    kern_timed = _lib.profile_report() if args.profile else {}
    lib.mage_profile_filter(None)
    for d in dets:
        d.device_status()
    s_last = args.warmup + args.steps - 1
    b_last = (s_last % RING) * B
    cnt, nm = ring["cnt"][b_last:b_last + B + 1], outs[s_last % NSTR]["nm"]
    # the last timed batch itself against the oracle: its first frames'
    # keypoints, descriptors and matches, byte for byte (test infrastructure: the check runs after
    # the timed region on copies of the results)
    parity = verify_orb_batch(args, frames[(s_last * B) % F:(s_last * B) % F + B], ring, b_last,
                              outs[s_last % NSTR], variant) if rank == 0 and args.batch_parity > 0 else None
    el_max = multigpu.max_over_ranks(el, dev, dist)
    # end-of-run exchange (RCCL over xGMI): per-frame (keypoints, matches) of the last batch
    summary = torch.stack([cnt[1:].to(torch.int64), nm.to(torch.int64)], 1)
    gathered = multigpu.gather_rows(summary, dist)
    kern = {}
    if args.profile:
        lib.mage_profile_reset()
        lib.mage_profile_enable(1)
        for s in range(args.warmup + args.steps, args.warmup + 2 * args.steps):
            step(s)
        torch.cuda.synchronize(dev)
        lib.mage_profile_enable(0)
        kern = _lib.profile_report()
    frames_total = world * args.steps * B
    res = {
        "value": frames_total / el_max,
        "ms_per_step": 1000.0 * el_max / args.steps,
        "frames_per_step": B,
        "kernels": {k: {"launches": c, "avg_ms": ms / max(c, 1)} for k, (c, ms) in kern.items()},
        "kernel_timing": "dispatch timestamps of one more pass of the same steps after the timed region "
                         "(the timed region times the roofline kernel only)",
        "mean_keypoints": float(torch.cat(gathered)[:, 0].float().mean().item()),
        "mean_matches": float(torch.cat(gathered)[:, 1].float().mean().item()),
    }
    if parity is not None:
        res["parity"] = parity
    orb_k = {k: {"launches": c, "avg_ms": ms / max(c, 1)} for k, (c, ms) in kern_timed.items()}
    if orb_k:
        dom = ROOF_KERNEL
        per_frame = orb_bytes_per_frame(W, H, N)
        if variant == "rbrief31":
            # + each pyramid level read once by FAST (the levels are written by resize_band_kernel,
            # whose bytes are not charged to fast_nms)
            per_frame += pyramid_level_bytes(W, H, RBRIEF31["nlevels"])
        # the kernel's time per step: one launch at C2, one per pyramid level for rBRIEF-31 (the
        # path's algorithmic bytes, SURVEY.md §8(d), priced on all of its launches: `frac` is a
        # single-kernel attribution; `frac_step` prices the same bytes on the whole step)
        per_step = max(1, round(orb_k[dom]["launches"] / max(args.steps, 1)))
        avg_s = orb_k[dom]["avg_ms"] * per_step / 1000.0
        achieved = per_frame * B / avg_s / 1e9
        # traffic: 2 x FETCH_SIZE + WRITE_SIZE (the guide's gfx950 correction of the wide-stream
        # read counter), per steady-state launch of the committed profile of these kernel sources
        psum = "pmc_summary_rbrief31.json" if variant == "rbrief31" else "pmc_summary.json"
        traffic, traffic_source = load_pmc(dom, "hbm_bytes_per_launch_fetch_x2", psum)
        traffic_raw, _ = load_pmc(dom, "hbm_bytes_per_launch", psum)
        valu, _ = load_pmc(dom, "valu_busy", psum)
        prof_us, _ = load_pmc(dom, "avg_us_steady", psum)
        step_s = el_max / args.steps
        frac_rocprof = None if prof_us is None else per_frame * B / (per_step * prof_us * 1e-6) / 1e9 / HBM_PEAK_GBS
        res["roofline"] = {"bound": "hbm", "kernel": dom, "achieved": achieved, "peak": HBM_PEAK_GBS,
                           "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                           # the same fraction priced on the committed rocprofv3 trace's steady-state
                           # average, and on the whole step (top-level scalars: see "rocprof" / "step")
                           "frac_rocprof": frac_rocprof,
                           "frac_step": per_frame * B / step_s / 1e9 / HBM_PEAK_GBS,
                           "valu_busy": valu,
                           "traffic_raw_fetch": traffic_raw,
                           "traffic_source": traffic_source + " (2 x FETCH_SIZE + WRITE_SIZE)",
                           "algorithmic_bytes_per_launch": per_frame * B,
                           "avg_launch_ms": orb_k[dom]["avg_ms"],
                           "launches_per_step": per_step,
                           "avg_launch_source": "dispatch timestamps (hipExtLaunchKernel events) on the launch stream, "
                                                "timed region only",
                           # the same figure priced on the committed rocprofv3 kernel trace (launches after
                           # the warm-up), so frac can be recomputed from profiles/
                           "rocprof": None if prof_us is None else {
                               "avg_launch_ms": prof_us / 1000.0,
                               "frac": frac_rocprof,
                               "source": traffic_source.split(" (")[0] + ", avg_us_steady"},
                           # whole step (extract + match of B frames) against the same bytes
                           "step": {"algorithmic_bytes": per_frame * B, "ms": 1000 * step_s,
                                    "frac": per_frame * B / step_s / 1e9 / HBM_PEAK_GBS},
                           # what actually binds the kernel: the SIMDs' VALU issue
                           # occupancy, (SQ_INSTS_VALU - SQ_ACTIVE_INST_VALU2) quad-cycles over the
                           # launch's GRBM_GUI_ACTIVE cycles (peak 1.0; pure-VALU probe loops read
                           # 0.93-0.95, profiles/r5_valu_probe_pmc.md), same PMC run
                           "binding": {"resource": "VALU issue", "frac": valu, "peak": 1.0,
                                       "calibration": "tools/valu_probe.hip loops: 0.93-0.95",
                                       "source": "SQ_INSTS_VALU / SQ_ACTIVE_INST_VALU2 / GRBM_GUI_ACTIVE pass of the same profile"
                                       if valu is not None else traffic_source}}
    return res


BA_ROUND_STEPS = 10  # timed LM steps per BA round (the C3 problem converges in ~15)


def ba_round(b, g, me, steps, timer):
    """One local-BA invocation in the reference's shape (BundleAdjust.cpp): load the graph, a first
    StepBundleAdjustment that removes the planted outliers (untimed), then `steps` timed steps.
    Rounds keep every timed step a real LM iteration: run past convergence, g2o's schedule
    rejects every trial (rho == 0) and lambda doubles up to inf, which is not BA work."""
    b.set_graph(g)
    b.step([1.8], me)
    timer.sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        b.step([1.8], me)
    timer.sync()
    return time.perf_counter() - t0


REF_WINDOW_STEPS = 10  # StepBundleAdjustment calls per local-BA window on the reference schedule
MIN_LAMBDA = 1e-3      # MappingSettings::MinLambda (MageSettings.h:260)
REF_DECAY = np.float32(0.95) * np.float32(0.95)  # MaxOutlierErrorSquared *= 0.95^2 per call (BundleAdjust.cpp:396)


def ba_reference_window(b, g, lam, steps, set_lambda, get_lambda, removed=None):
    """One local BA in the reference's invocation shape, all of it timed by the caller:
    BuildDataForG2O (graph load), the lambda persisted from the previous window
    (MappingWorker.cpp:272-293, PersistLambda), then `steps` x BundleAdjustTask::Impl::Iterate
    (BundleAdjust.cpp:380-404): StepBundleAdjustment at MaxOutlierErrorSquared, which starts at the
    NON-squared MaxOutlierError (:375) and is multiplied by 0.95^2 after every call (:396), and
    UpdateData's GetPose / GetPoint (:195-226).  Returns the next window's lambda
    (max(GetCurrentLambda, MinLambda), MappingWorker.cpp:293)."""
    b.set_graph(g)
    if lam is not None:
        set_lambda(lam)
    me = 7.25
    for _ in range(steps):
        _, out = b.step([1.8], me)
        if removed is not None:
            removed.append(len(out))
        b.poses()
        b.points()
        me *= REF_DECAY
    return max(get_lambda(), MIN_LAMBDA)


def run_ba_reference_schedule(b, g, budget_s, set_lambda, get_lambda, sync, steps=REF_WINDOW_STEPS):
    """Windows on the reference schedule for ~budget_s (at least 2), each timed whole (graph load,
    steps, readbacks).  The first window (lambda from computeLambdaInit) is untimed warm-up."""
    lam = ba_reference_window(b, g, None, steps, set_lambda, get_lambda)
    sync()
    el, n, removed = 0.0, 0, []
    s0 = b.stats()
    while el < budget_s or n < 2:
        t0 = time.perf_counter()
        lam = ba_reference_window(b, g, lam, steps, set_lambda, get_lambda, removed)
        sync()
        el += time.perf_counter() - t0
        n += 1
    s1 = b.stats()
    return {"value": n * steps / el, "unit": "iters/s", "windows": n, "steps_per_window": steps, "seconds": el,
            "trials_per_iteration": (s1["trials"] - s0["trials"]) / max(s1["iterations"] - s0["iterations"], 1),
            "outliers_per_call": float(np.mean(removed)), "calls_removing_edges": float(np.mean(np.array(removed) > 0)),
            "final_lambda": lam}


def run_ba(args, local_rank, torch):
    from mageslam_amd import _lib, bundler, synth

    class _Sync:
        @staticmethod
        def sync():
            torch.cuda.synchronize()

    g = synth.ba_graph()
    b = bundler.BundlerLib(device=local_rank)
    # maxErrorSquare held at MaxOutlierError (7.25, BundleAdjust.cpp:375) on GPU and CPU alike
    me = 7.25
    for _ in range(max(1, args.ba_warmup // 3)):
        ba_round(b, g, me, BA_ROUND_STEPS, _Sync)
    rounds = max(1, args.ba_iters // BA_ROUND_STEPS)
    lib = _lib.load()
    # timed steps without per-launch events (the BA trial is ~12 short launches, where even
    # dispatch-packet timestamps cost ~14%); the per-kernel breakdown comes from one more,
    # separately profiled round
    el, iters, trials = 0.0, 0, 0
    for _ in range(rounds):
        s0 = b.stats()
        el += ba_round(b, g, me, BA_ROUND_STEPS, _Sync)
        s1 = b.stats()
        iters += s1["iterations"] - s0["iterations"] - 1  # minus the untimed first pass
        trials += s1["trials"] - s0["trials"]
    steps = rounds * BA_ROUND_STEPS
    kern = {}
    if args.profile:
        b.set_graph(g)
        b.step([1.8], me)
        lib.mage_profile_reset()
        lib.mage_profile_enable(1)
        for _ in range(BA_ROUND_STEPS):
            b.step([1.8], me)
        torch.cuda.synchronize()
        lib.mage_profile_enable(0)
        kern = _lib.profile_report()
    # trials of the untimed first passes are one each (fresh lambda, accepted): excluded
    trials_per_iter = (trials - rounds) / max(iters, 1)
    res = {"metric": "local-BA iters/sec (50 KF, 5k pts)", "value": steps / el, "unit": "iters/s",
           "lm_iterations": iters, "trials_per_iteration": trials_per_iter, "dtype": "f64",
           "config": {"workload": "C3: 50 keyframes (10 fixed) x 5000 points x 20 obs = 100k observations",
                      "iteration": "BundlerLib::StepBundleAdjustment with one LM step + outlier pass",
                      "schedule": f"{rounds} rounds x (load graph + outlier-removing first step, untimed; "
                                  f"{BA_ROUND_STEPS} timed steps)"},
           "kernels": {k: {"launches": c, "avg_ms": ms / max(c, 1), "total_ms": ms} for k, (c, ms) in kern.items()},
           "kernel_timing": "dispatch timestamps (hipExtLaunchKernel events) of one more round, outside the "
                            "timed region"}
    # the reference's invocation shape (BundleAdjustTask::Iterate per call, lambda persisted across
    # windows): decaying outlier thresholds remove edges on most calls
    res["reference_schedule"] = dict(
        run_ba_reference_schedule(b, g, 3.0, b.SetCurrentLambda, b.GetCurrentLambda, torch.cuda.synchronize),
        schedule=f"windows of (BuildDataForG2O + SetCurrentLambda(persisted) + {REF_WINDOW_STEPS} x "
                 f"[StepBundleAdjustment(huber 1.8, maxErrSq 7.25 x 0.9025^k) + GetPose/GetPoint]), all timed")
    flops_iter = ba_flops(g, trials_per_iter)
    achieved = flops_iter * res["value"] / 1e12
    dom = max(kern, key=lambda k: kern[k][1]) if kern else None
    # HBM bytes per LM iteration from the committed counters of the same kernel sources: each
    # kernel's 2 x FETCH_SIZE + WRITE_SIZE per launch x its launches per iteration (profiled round)
    traffic, tsrc = 0.0, None
    for k, (c, _) in kern.items():
        v, tsrc = load_pmc(k, "hbm_bytes_per_launch_fetch_x2", "pmc_summary_ba.json")
        if v is None:
            traffic = None
            break
        traffic += v * c / BA_ROUND_STEPS
    res["roofline"] = {"bound": "mfma", "achieved": achieved, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                       "frac": achieved / FP64_PEAK_TFLOPS, "traffic": traffic if kern else None,
                       "traffic_unit": "HBM bytes per LM iteration (2 x FETCH_SIZE + WRITE_SIZE over the BA kernels)",
                       "traffic_source": tsrc, "flops_per_iteration": flops_iter, "dominant_kernel": dom}
    return res, g


POSE_STEPS, POSE_HUBER, POSE_MAXE = 3, 4.0, 36.0  # TrackLocalMap's first OptimizeCameraPose (MageSettings.h:184-189)


def run_pose(args, rank, world, local_rank, torch, dist):
    """Batched pose-only BA: TrackLocalMap::OptimizeCameraPose for a batch of
    frames per launch (mage_ba_pose_batch_device), inputs resident in HBM; with several ranks each
    solves its own batch (seed + rank), no collective."""
    from mageslam_amd import _lib, bundler, multigpu, synth

    pb = synth.pose_batch(problems=args.pose_problems, obs=600, seed=multigpu.sequence_seed(synth.BA_SEED + 1, rank))
    K = args.pose_problems
    E = int(pb.obs_start[-1])
    dev = f"cuda:{local_rank}"
    T = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a, dt)).to(dev)  # noqa: E731
    pos, r9, intr = T(pb.pos, np.float32), T(pb.r9, np.float32), T(pb.intr, np.float32)
    ost, pts, uv, info = T(pb.obs_start.astype(np.int32), np.int32), T(pb.points, np.float32), T(pb.uv, np.float32), \
        T(pb.info, np.float32)
    pos_o = torch.empty((K, 3), dtype=torch.float32, device=dev)
    r9_o = torch.empty((K, 9), dtype=torch.float32, device=dev)
    qt_o = torch.empty((K, 7), dtype=torch.float64, device=dev)
    outl = torch.empty(E, dtype=torch.uint8, device=dev)
    ms = torch.empty(K, dtype=torch.float32, device=dev)
    stats = torch.empty((K, 2), dtype=torch.int32, device=dev)

    def once():
        bundler.pose_batch_device(K, pos, r9, intr, ost, pts, uv, info, POSE_STEPS, POSE_HUBER, POSE_MAXE, pos_o,
                                  r9_o, qt_o, outl, ms, stats)

    for _ in range(3):
        once()
    torch.cuda.synchronize()
    n = args.pose_iters
    multigpu.barrier(dist)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        once()
    torch.cuda.synchronize()
    multigpu.barrier(dist)
    el = multigpu.max_over_ranks(time.perf_counter() - t0, dev, dist)
    lib = _lib.load()
    lib.mage_profile_reset()
    lib.mage_profile_enable(1)
    for _ in range(3):
        once()
    torch.cuda.synchronize()
    lib.mage_profile_enable(0)
    kern = _lib.profile_report()
    st = stats.cpu().numpy()
    res = {"metric": "pose-only BA problems/sec (OptimizeCameraPose: 1 camera, ~600 fixed points, 3 LM steps)",
           "value": world * n * K / el, "unit": "problems/s", "dtype": "f64", "problems_per_launch": K,
           "observations": E, "lm_iterations_per_problem": float(st[:, 0].mean()),
           "trials_per_problem": float(st[:, 1].mean()),
           "config": {"workload": f"{K} synthetic 720p frames x {E / K:.0f} observations, huber {POSE_HUBER}, "
                                  f"maxErrorSquare {POSE_MAXE}, {POSE_STEPS} steps (TrackLocalMap.cpp:96-107)"},
           "kernels": {k: {"launches": c, "avg_ms": v / max(c, 1)} for k, (c, v) in kern.items()}}
    if "ba.pose_batch" in kern:
        c, v = kern["ba.pose_batch"]
        avg_s = v / c / 1000.0
        # compulsory bytes per launch: observations (point 12 + uv 8 + info 4 + flag 1) and per-problem
        # pose in/out (12 + 36 + 16 in, 12 + 36 + 56 + 4 + 8 out)
        byts = E * 25 + K * (64 + 116)
        # counters from the per-row profile (tools/bench_rows.py pose leg: this launch alone)
        traffic, tsrc = load_pmc("pose.ba", "hbm_bytes_per_launch_fetch_x2", "pmc_summary_rows.json")
        res["roofline"] = {"bound": "hbm", "kernel": "ba.pose_batch", "achieved": byts / avg_s / 1e9,
                           "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": byts / avg_s / 1e9 / HBM_PEAK_GBS,
                           "traffic": traffic, "traffic_source": tsrc + " (2 x FETCH_SIZE + WRITE_SIZE)",
                           "algorithmic_bytes_per_launch": byts, "avg_launch_ms": v / c}
    return res, pb


def cpu_pose_baseline(pb, budget_s):
    from oracle import oracle as O

    K = len(pb.pos)
    el, n = 0.0, 0
    chunk = 32
    import dataclasses

    while el < budget_s or n == 0:
        k0 = (n * chunk) % K
        k1 = min(k0 + chunk, K)
        s0, s1 = int(pb.obs_start[k0]), int(pb.obs_start[k1])
        sub = dataclasses.replace(pb, pos=pb.pos[k0:k1], r9=pb.r9[k0:k1], intr=pb.intr[k0:k1],
                                  obs_start=(pb.obs_start[k0:k1 + 1] - pb.obs_start[k0]).astype(np.uint32),
                                  points=pb.points[s0:s1], uv=pb.uv[s0:s1], info=pb.info[s0:s1])
        t0 = time.perf_counter()
        O.pose_batch(sub, POSE_STEPS, POSE_HUBER, POSE_MAXE)
        el += time.perf_counter() - t0
        n += 1
    return {"value": n * chunk / el, "unit": "problems/s", "cores": 1, "kind": "port",
            "sample": f"{n * chunk} problems of the same batch, oracle (fresh BundlerLib per frame), single thread, "
                      f"{el:.1f} s"}


def c5_exchange(res, rank, dist, device, csv_path=""):
    """C5's one exchange step: every rank's tracked trajectory as 68-byte records
    (tracked flag + view matrix per frame, GetTrackingResultsForFrames, MAGESlam.cpp:410-428) is
    all-gathered (RCCL over xGMI; gloo in the CPU rehearsal); rank 0 writes them in rank order as
    ExportFossilCsv does (console.cpp:15-54).  Returns the gathered (T, 17) arrays, rank-ordered."""
    import torch

    from mageslam_amd import trajectory

    T = len(res.poses)
    tracked = np.array([f == 0 or res.inliers[f] > 0 for f in range(T)])
    rows = trajectory.records_from_poses(res.rotations(), res.translations(), tracked)
    gathered = [g.cpu().numpy() for g in trajectory.gather_trajectories(torch.from_numpy(rows).to(device), dist)]
    if rank == 0 and csv_path:
        trajectory.export_fossil_csv(csv_path, np.concatenate(gathered))
    return gathered, rows


TRACK_STEP = 0.03  # camera travel per frame on the plane: ~5.4 px at 720p, a keyframe every ~60 frames


def run_tracking(args, rank, world, local_rank, torch, dist):
    """C4 (BASELINE.json configs[3]) and, with several ranks, C5 (configs[4]): the tracking loop
    (mageslam_amd.tracking) over a synthetic hand-held 720p sequence of a textured plane, frames
    rendered into HBM first, composed with the local BA MappingWorker runs after every new keyframe
    (tracking.local_bundle_adjust).  A step is the whole sequence: batched ORB extraction of every
    frame, then the device-resident loop (RadiusMatch + two pose-only BundlerLib passes + the
    local-map search per frame, sequential: each frame's prediction needs the previous pose; a
    BundlerLib step between frames at every keyframe).  Every rank tracks its own sequence (texture
    seed + rank, camera path from synth.rank_origin); after the timed region the tracked trajectories
    are all-gathered (c5_exchange)."""
    from mageslam_amd import _lib, multigpu, orb, synth, tracking

    T = args.track_frames
    seq = synth.scene_sequence(T, args.width, args.height, step=TRACK_STEP, origin=synth.rank_origin(rank))
    seed = multigpu.sequence_seed(synth.FRAME_SEED, rank)
    dev = f"cuda:{local_rank}"
    cams = torch.from_numpy(seq.cams()).to(dev)
    frames = torch.empty((T, args.height, args.width), dtype=torch.uint8, device=dev)
    _lib.check(_lib.load().mage_synth_scene_device(_lib.ptr(frames), T, args.width, args.height,
                                                   args.width * args.height, _lib.ptr(cams), seq.fx, seq.fy, seq.cx,
                                                   seq.cy, synth.SCENE_PLANE_Z, synth.SCENE_TEXEL_SCALE,
                                                   synth.SCENE_TEXEL_OFFSET, seed, None))
    torch.cuda.synchronize()
    K = (seq.fx, seq.fy, seq.cx, seq.cy)
    p0 = tracking.Pose(seq.R[0], seq.t[0])
    ts = tracking.TrackerSettings(width=args.width, height=args.height, local_ba=not args.no_local_ba)
    N = args.features
    det = orb.OrbDetector(nfeatures=N, device=local_rank)
    d_kp = torch.zeros((T, N * 28), dtype=torch.uint8, device=dev)
    d_desc = torch.zeros((T, N, 32), dtype=torch.uint8, device=dev)
    d_n = torch.zeros(T, dtype=torch.int32, device=dev)

    def extract_device(n):  # batched extraction into the device layout the device loop reads
        for b0 in range(0, n, 64):
            b1 = min(n, b0 + 64)
            det.detect_and_compute_batch_device(frames[b0:b1], args.width, args.height, d_kp[b0:b1],
                                                d_desc[b0:b1], d_n[b0:b1], N)

    W = max(2, min(args.track_warmup, T))
    extract_device(W)  # warm-up: the first frames, extraction + loop, untimed
    tracking.track_native_device(d_kp, d_desc, N, d_n, W, K, p0, synth.SCENE_PLANE_Z, settings=ts)
    torch.cuda.synchronize()
    # the timed loop: device-resident extraction + mage_track_sequence_device
    multigpu.barrier(dist)
    t0 = time.perf_counter()
    extract_device(T)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    res = tracking.track_native_device(d_kp, d_desc, N, d_n, T, K, p0, synth.SCENE_PLANE_Z, settings=ts)
    t2 = time.perf_counter()
    multigpu.barrier(dist)
    el_max = multigpu.max_over_ranks(t2 - t0, dev, dist)
    per_rank = [float(x[0]) for x in multigpu.gather_rows(
        torch.tensor([T / (t2 - t0)], dtype=torch.float64, device=dev), dist)]
    gathered, own = c5_exchange(res, rank, dist, dev, args.trajectory_csv)
    gt = tracking.TrackResult(poses=[tracking.Pose(seq.R[i], seq.t[i]) for i in range(T)])
    out = {"metric": "tracking-loop frames/sec @720p (extract + RadiusMatch + 2x OptimizeCameraPose + local map"
                     + (" + local BA per keyframe" if ts.local_ba else "") + ")",
           "value": world * T / el_max, "unit": "frames/s", "frames": T, "warmup_frames": W, "dtype": "u8 / f64",
           "extract_ms_per_frame": 1000 * (t1 - t0) / T, "track_ms_per_frame": 1000 * (t2 - t1) / T,
           "loop": "device-resident (mage_track_sequence_device: per-frame decisions on the GPU; with the local BA "
                   "the host runs BundlerLib between frames at each keyframe)",
           "mean_matches": float(np.mean(res.matches[1:])), "mean_inliers": float(np.mean(res.inliers[1:])),
           "keyframes": len(res.keyframes), "local_ba_windows": len(res.ba_outliers),
           "local_ba_outliers": int(sum(n for _, n in res.ba_outliers)),
           "pose_rmse_vs_ground_truth": tracking.pose_rmse(res, gt),
           "local_map": f"TrackLocalMap local-map search over the last {ts.local_map_keyframes} keyframes",
           "local_ba": ("one StepBundleAdjustment per new keyframe over the covisibility window of the local map's "
                        "keyframes (GetMapPointsAndDistantKeyframes: the new keyframe and those sharing >= theta points "
                        "free, other observers fixed, theta retuned to 1500-2000 associations, ThreadSafeMap.cpp:888-957), "
                        "persisted lambda and theta (MappingWorker.cpp:228-371)") if ts.local_ba else "off",
           "config": {"workload": f"C4: {T}-frame {args.width}x{args.height} hand-held pan over a textured plane "
                                  f"(synthetic, {TRACK_STEP} units per frame), {args.features} features/frame"
                                  + (f"; C5: {world} independent sequences (seed + rank), one per GPU, RCCL "
                                     f"all-gather of the tracked trajectories" if world > 1 else "")}}
    if world > 1:
        out["per_gpu_fps"] = per_rank
        out["scaling"] = "weak"
    out["trajectory_frames_gathered"] = int(sum(len(g) for g in gathered))
    out["trajectory_gather_consistent"] = bool(np.array_equal(gathered[rank], own))
    if world > 1:
        return out, None
    # one GPU: the same loop driven from Python over the GPU kernels must give the identical result;
    # the host-driven native loop (mage_track_sequence, no local BA) equals the device loop without it
    be = tracking.GpuBackend(args.features, device=local_rank, batch=64)
    feats = be.extract(frames)
    torch.cuda.synchronize()

    def same(a, b):
        return a.matches == b.matches and a.inliers == b.inliers and a.keyframes == b.keyframes and all(
            np.array_equal(x.t, y.t) and np.array_equal(x.R, y.R) for x, y in zip(a.poses, b.poses))

    t3 = time.perf_counter()
    py = tracking.track(feats, K, p0, synth.SCENE_PLANE_Z, be, ts)
    t4 = time.perf_counter()
    nb = tracking.TrackerSettings(width=args.width, height=args.height)
    dev_nb = tracking.track_native_device(d_kp, d_desc, N, d_n, T, K, p0, synth.SCENE_PLANE_Z, settings=nb)
    t5 = time.perf_counter()
    host = tracking.track_native(feats, K, p0, synth.SCENE_PLANE_Z, settings=nb, device=local_rank)
    t6 = time.perf_counter()
    out.update(python_loop_track_ms_per_frame=1000 * (t4 - t3) / T,
               python_loop_identical=bool(same(py, res) and py.ba_outliers == res.ba_outliers),
               without_local_ba={"track_ms_per_frame": 1000 * (t5 - t4) / T, "keyframes": len(dev_nb.keyframes),
                                 "pose_rmse_vs_ground_truth": tracking.pose_rmse(dev_nb, gt)},
               host_loop_track_ms_per_frame=1000 * (t6 - t5) / T, host_loop_identical=bool(same(host, dev_nb)))
    # The regime the local BA exists for: new map points carry the depth error a triangulated point
    # has (NewMapPointsCreation.cpp:254) instead of the plane back-projection's exact depth; the
    # same frames and features, with and without the local BA (oracle parity in cpu_tracking_baseline)
    dctx = None
    if args.track_depth_noise > 0:
        import dataclasses

        tsd = dataclasses.replace(ts, local_ba=True, map_point_depth_noise=args.track_depth_noise)
        t7 = time.perf_counter()
        rd = tracking.track_native_device(d_kp, d_desc, N, d_n, T, K, p0, synth.SCENE_PLANE_Z, settings=tsd)
        t8 = time.perf_counter()
        rd_nb = tracking.track_native_device(d_kp, d_desc, N, d_n, T, K, p0, synth.SCENE_PLANE_Z,
                                             settings=dataclasses.replace(tsd, local_ba=False))
        out["depth_error"] = {
            "map_point_depth_noise": tsd.map_point_depth_noise,
            "what": "new map points' depth x (1 + sigma g), g a seeded unit-variance variate per (keyframe, keypoint) "
                    "(tracking.depth_noise_factor): a triangulated point's depth error; the same frames and features",
            "value": T / (t8 - t7 + (t1 - t0)), "unit": "frames/s (extraction of the main leg + this loop)",
            "track_ms_per_frame": 1000 * (t8 - t7) / T, "keyframes": len(rd.keyframes),
            "local_ba_windows": len(rd.ba_outliers), "local_ba_outliers": int(sum(n for _, n in rd.ba_outliers)),
            "local_ba": "covisibility window (GetMapPointsAndDistantKeyframes, ThreadSafeMap.cpp:888-957)",
            "pose_rmse_vs_ground_truth": tracking.pose_rmse(rd, gt),
            "without_local_ba": {"keyframes": len(rd_nb.keyframes),
                                 "pose_rmse_vs_ground_truth": tracking.pose_rmse(rd_nb, gt)}}
        out["depth_error"]["local_ba_reduces_error"] = bool(
            out["depth_error"]["pose_rmse_vs_ground_truth"][0] < out["depth_error"]["without_local_ba"]["pose_rmse_vs_ground_truth"][0])
        dctx = (rd, tsd)
    return out, (seq, frames, res, feats, ts, dctx)


def cpu_tracking_baseline(args, ctx, budget_s):
    """The identical loop (local BA included) on the CPU oracle over the first
    --track-parity-frames frames of the same sequence: its rate, and the GPU-vs-CPU parity of those
    frames (north star: pose RMSE <= 1e-4; identical matches, keyframes and BA outliers)."""
    from oracle.tracking_backend import OracleBackend

    from mageslam_amd import synth, tracking

    seq, frames, gres, gfeats, ts, dctx = ctx
    n = min(args.track_parity_frames, len(gres.poses))
    ob = OracleBackend(args.features)
    host = frames[:n].cpu().numpy()
    t0 = time.perf_counter()
    feats = ob.extract(host)
    K = (seq.fx, seq.fy, seq.cx, seq.cy)
    p0 = tracking.Pose(seq.R[0], seq.t[0])
    ores = tracking.track(feats, K, p0, synth.SCENE_PLANE_Z, ob, ts)
    el = time.perf_counter() - t0
    same = all(np.array_equal(a[0].view(np.uint8), b[0].view(np.uint8)) for a, b in zip(gfeats[:n], feats))
    def parity(g, o):
        gba = [x for x in g.ba_outliers if x[0] < n]
        return {"frames": n, "keypoints_identical": bool(same),
                "pose_rmse_gpu_vs_cpu": tracking.pose_rmse(tracking.TrackResult(poses=g.poses[:n]), o),
                "matches_identical": g.matches[:n] == o.matches, "inliers_identical": g.inliers[:n] == o.inliers,
                "keyframes_identical": [k for k in g.keyframes if k < n] == o.keyframes,
                "ba_outliers_identical": gba == o.ba_outliers, "local_ba_windows": len(o.ba_outliers),
                "local_ba_outliers": int(sum(c for _, c in o.ba_outliers))}

    par = parity(gres, ores)
    if dctx is not None:  # the depth-error leg: the same oracle features, its settings
        rd, tsd = dctx
        par["depth_error"] = parity(rd, tracking.track(feats, K, p0, synth.SCENE_PLANE_Z, ob, tsd))
    return {"value": n / el, "unit": "frames/s", "cores": 1, "kind": "port", "build": ORACLE_BUILD[0],
            "sample": f"first {n} frames of the same sequence, oracle extract + RadiusMatch + pose BA + local map + "
                      f"local BA, single thread, {el:.1f} s"}, par


def cpu_ba_baseline(g, budget_s):
    from oracle import oracle as O

    class _NoSync:
        @staticmethod
        def sync():
            pass

    b = O.BundlerOracle()
    me = 7.25  # same schedule as the GPU leg (run_ba)
    el, n = 0.0, 0
    while el < budget_s or n == 0:
        el += ba_round(b, g, me, BA_ROUND_STEPS, _NoSync)
        n += BA_ROUND_STEPS
    return {"value": n / el, "unit": "iters/s", "cores": 1, "kind": "port",
            "sample": f"{n // BA_ROUND_STEPS} rounds x {BA_ROUND_STEPS} timed StepBundleAdjustment iterations of "
                      f"the C3 graph (same schedule as the GPU leg), oracle, single thread, {el:.1f} s"}


def cpu_ba_reference_baseline(g, budget_s):
    """The oracle on the reference schedule (run_ba_reference_schedule), single thread."""
    from oracle import oracle as O

    b = O.BundlerOracle()
    r = run_ba_reference_schedule(b, g, budget_s, b.set_lambda, b.get_lambda, lambda: None)
    return dict(r, cores=1, kind="port",
                sample=f"{r['windows']} windows x {r['steps_per_window']} calls of the C3 graph on the reference "
                       f"schedule (same as the GPU leg), oracle, single thread, {r['seconds']:.1f} s")


def lockstep_rounds(windows, g, budget_s, sync=lambda: None):
    """Concurrent C3 windows on the fixed schedule, measured in lock-step: every thread loads its
    graph and takes the untimed outlier-removing first step, all meet at a barrier, then all run
    BA_ROUND_STEPS timed steps; a round's time is from the barrier to the last thread's end.  The
    aggregate is all timed steps over the summed round times — the graph loads of one thread never
    overlap another's timed steps (a per-thread rate summed over threads would credit that
    overlap)."""
    import threading
    from concurrent.futures import ThreadPoolExecutor

    n = len(windows)
    bar = threading.Barrier(n, timeout=300)
    marks = {}
    state = {"stop": False}

    def work(w):
        b, r = windows[w], 0
        while True:
            b.set_graph(g)
            b.step([1.8], 7.25)
            sync()
            bar.wait()
            if state["stop"]:
                return
            t0 = time.perf_counter()
            for _ in range(BA_ROUND_STEPS):
                b.step([1.8], 7.25)
            sync()
            marks[(r, w)] = (t0, time.perf_counter())
            bar.wait()
            if w == 0:  # decide for everyone before the next barrier
                rounds = r + 1
                total = sum(max(marks[(q, i)][1] for i in range(n)) - min(marks[(q, i)][0] for i in range(n))
                            for q in range(rounds))
                state["stop"] = total >= budget_s
            bar.wait()
            r += 1

    with ThreadPoolExecutor(n) as ex:
        list(ex.map(work, range(n)))
    rounds = max(r for r, _ in marks) + 1
    wall = sum(max(marks[(q, i)][1] for i in range(n)) - min(marks[(q, i)][0] for i in range(n)) for q in range(rounds))
    return n * rounds * BA_ROUND_STEPS / wall, rounds, wall


def concurrent_reference_windows(objs, g, budget_s, setter, getter):
    """Concurrent window sequences on the reference schedule (ba_reference_window, everything of a
    window timed): one untimed warm-up window per thread, then all threads start together at a
    barrier and run windows until a shared deadline; the aggregate is every thread's calls over the
    common wall time (start to the last thread's end), so no thread's idle time is credited."""
    import threading
    from concurrent.futures import ThreadPoolExecutor

    n = len(objs)
    bar = threading.Barrier(n, timeout=300)
    calls, ends, start = [0] * n, [0.0] * n, {}

    def work(w):
        b = objs[w]
        lam = ba_reference_window(b, g, None, REF_WINDOW_STEPS, setter(b), getter(b))
        bar.wait()
        if w == 0:
            start["t"] = time.perf_counter()
        bar.wait()
        t0 = start["t"]
        while time.perf_counter() - t0 < budget_s:
            lam = ba_reference_window(b, g, lam, REF_WINDOW_STEPS, setter(b), getter(b))
            calls[w] += REF_WINDOW_STEPS
        ends[w] = time.perf_counter()

    with ThreadPoolExecutor(n) as ex:
        list(ex.map(work, range(n)))
    wall = max(ends) - start["t"]
    return sum(calls) / wall, sum(calls) // REF_WINDOW_STEPS, wall


def run_ba_many(args, local_rank, g, budget_s):
    """Many independent C3 windows at once (one window per sequence): `host_threads()`
    BundlerLib instances, each with its own HIP stream, driven from as many host threads on the
    GPU leg's schedule — the GPU counterpart of cpu_ba_baseline_all (sum of per-thread rates)."""
    from mageslam_amd import bundler

    class _Blocking:  # StepBundleAdjustment returns after its last readback
        @staticmethod
        def sync():
            pass

    n = host_threads()
    libs = [bundler.BundlerLib(device=local_rank) for _ in range(n)]
    for b in libs:  # warm-up (allocations)
        ba_round(b, g, 7.25, 1, _Blocking)
    rate, rounds, wall = lockstep_rounds(libs, g, budget_s)

    ref, nwin, rwall = concurrent_reference_windows(libs, g, budget_s, lambda b: b.SetCurrentLambda,
                                                    lambda b: b.GetCurrentLambda)
    return {"value": rate, "unit": "iters/s", "windows": n,
            "config": f"{n} concurrent copies of the C3 window (one BundlerLib + HIP stream + host thread each) in "
                      f"lock-step rounds ({rounds} rounds, {wall:.1f} s of timed steps; lockstep_rounds)",
            "reference_schedule": {"value": ref, "unit": "iters/s", "windows": n,
                                   "config": f"{n} concurrent window sequences on the reference schedule (graph load + "
                                             f"{REF_WINDOW_STEPS} decaying-threshold calls with GetPose/GetPoint, "
                                             f"lambda persisted): {nwin} windows in {rwall:.1f} s of common wall time "
                                             f"(concurrent_reference_windows)"}}


def run_ba_many_child(local_rank):
    """run_ba_many in a child process (its own GPU context): the multi-threaded leg cannot take
    the headline run down with it."""
    import subprocess

    # the child sees exactly this rank's GPU: entry local_rank of the parent's visible list
    visible = os.environ.get("HIP_VISIBLE_DEVICES")
    dev = visible.split(",")[local_rank] if visible else str(local_rank)
    env = dict(os.environ, HIP_VISIBLE_DEVICES=dev, PYTHONFAULTHANDLER="1")
    try:
        r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--ba-many-child"], capture_output=True, text=True,
                           timeout=180, env=env, cwd=str(ROOT))
        lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
        if r.returncode == 0 and lines:
            return dict(json.loads(lines[-1]), status="ok")
        fail = {"status": "failed", "error": f"child exited with {r.returncode}", "stderr_tail": r.stderr[-1500:]}
    except subprocess.TimeoutExpired:
        fail = {"status": "failed", "error": "child timed out (180 s)"}
    print(f"bench: many-windows BA leg FAILED: {fail}", file=sys.stderr, flush=True)
    return fail


def cpu_ba_baseline_all(g, budget_s, n=None):
    """Independent copies of the C3 window on all host cores (one oracle BundlerLib per thread,
    the GPU leg's schedule) — the many-windows throughput of SURVEY.md §8(e)."""
    from oracle import oracle as O

    n = n or host_threads()
    rate, rounds, wall = lockstep_rounds([O.BundlerOracle() for _ in range(n)], g, budget_s)
    return {"value": rate, "unit": "iters/s", "cores": n, "kind": "port",
            "sample": f"{n} threads, each its own copy of the C3 window on the GPU leg's schedule, in lock-step rounds "
                      f"({rounds} rounds, {wall:.1f} s of timed steps; lockstep_rounds)", "host": host_info()}


def cpu_ba_reference_baseline_all(g, budget_s, n=None):
    """The reference schedule on all host cores: one oracle window sequence per thread."""
    from oracle import oracle as O

    n = n or host_threads()
    val, nwin, wall = concurrent_reference_windows([O.BundlerOracle() for _ in range(n)], g, budget_s,
                                                   lambda b: b.set_lambda, lambda b: b.get_lambda)
    return {"value": val, "unit": "iters/s", "cores": n, "kind": "port",
            "sample": f"{n} threads, each its own window sequence on the reference schedule: {nwin} windows in "
                      f"{wall:.1f} s of common wall time (concurrent_reference_windows)", "host": host_info()}


def run_dry(args, rank, world, dist):
    """CPU rehearsal of the multi-rank control flow (gloo): per-rank sequences, timed loop,
    max-reduce and the end-of-run gather, with the GPU kernels replaced by frame synthesis."""
    import torch

    from mageslam_amd import multigpu, synth

    seed = multigpu.sequence_seed(synth.FRAME_SEED, rank)
    w, h, B = 64, 48, 4
    multigpu.barrier(dist)
    t0 = time.perf_counter()
    sums = []
    for s in range(args.steps):
        fr = synth.frames(s * B, B, w, h, seed)
        sums.append(fr.reshape(B, -1).sum(1))
    el = time.perf_counter() - t0
    el_max = multigpu.max_over_ranks(el, "cpu", dist)
    summary = torch.tensor(np.stack([np.full(B, rank), sums[-1]], 1), dtype=torch.int64)
    gathered = multigpu.gather_rows(summary, dist)
    # C5's trajectory exchange with stand-in tracking results: the ground-truth poses of this rank's
    # scene sequence in place of the device loop's (which needs the GPU)
    from mageslam_amd import tracking

    T = min(args.track_frames, 16)
    seq = synth.scene_sequence(T, args.width, args.height, origin=synth.rank_origin(rank))
    res = tracking.TrackResult(poses=[tracking.Pose(seq.R[i], seq.t[i]) for i in range(T)], inliers=[1] * T)
    traj, _ = c5_exchange(res, rank, dist, "cpu", args.trajectory_csv)
    return {"trajectory_frames_gathered": int(sum(len(t) for t in traj)),"value": world * args.steps * B / el_max, "ms_per_step": 1000 * el_max / args.steps, "kernels": {},
            "mean_keypoints": 0.0, "mean_matches": 0.0, "frames_per_step": B,
            "gathered_ranks": [int(g[0, 0]) for g in gathered],
            "gathered_checksums": [int(g[:, 1].sum()) for g in gathered]}


def main():
    args = parse()
    from mageslam_amd import multigpu

    rank, world, local_rank = multigpu.rank_env()
    import torch

    if args.ba_many_child:  # see run_ba_many_child: one visible device
        from mageslam_amd import synth

        torch.cuda.set_device(0)
        print(json.dumps(run_ba_many(args, 0, synth.ba_graph(), 3.0)), flush=True)
        return

    if args.cpu_dry_run:
        dist = multigpu.init("gloo", local_rank)
        res = run_dry(args, rank, world, dist)
        if rank == 0:
            print(json.dumps({"metric": METRIC, "value": res["value"], "unit": "frames/s", "n_gpus": world,
                              "steps": args.steps, "warmup": args.warmup, "ms_per_step": res["ms_per_step"],
                              "dry_run": True, "scaling": "weak", "gathered_ranks": res["gathered_ranks"],
                              "gathered_checksums": res["gathered_checksums"],
                              "trajectory_frames_gathered": res["trajectory_frames_gathered"]}))
        if dist is not None:
            dist.destroy_process_group()
        return

    if args.rehearse_one_gpu:
        local_rank = 0  # every rank on the one GPU; RCCL refuses duplicate devices, so gloo
    torch.cuda.set_device(local_rank)
    dist = multigpu.init("gloo" if args.rehearse_one_gpu else "nccl", local_rank)

    orb_res = run_orb(args, rank, world, local_rank, torch, dist,
                      variant=None if args.orb_variant == "c2" else args.orb_variant)
    r31_res = None
    if world == 1 and not args.no_rbrief31 and args.orb_variant == "c2":
        import copy

        ra = copy.copy(args)
        ra.steps, ra.streams = args.rbrief31_steps, 1
        r31_res = run_orb(ra, rank, world, local_rank, torch, dist, variant="rbrief31")
    pipe_res = None
    if world == 1 and args.pipelined_streams > 1 and args.streams == 1:
        import copy

        pa = copy.copy(args)
        pa.streams, pa.profile, pa.batch_parity = args.pipelined_streams, False, 0
        pr = run_orb(pa, rank, world, local_rank, torch, dist)
        pipe_res = {"value": pr["value"], "unit": "frames/s", "ms_per_step": pr["ms_per_step"],
                    "hip_streams": pa.streams, "mean_matches": pr["mean_matches"],
                    "same_last_batch_as_single_stream": pr["mean_matches"] == orb_res["mean_matches"]
                    and pr["mean_keypoints"] == orb_res["mean_keypoints"],
                    "note": "the same workload with batch s+1's extraction overlapping batch s's select / describe "
                            "/ match on another stream (not the headline: overlapping batches stretch the "
                            "per-kernel durations the roofline is priced on)"}
    ba_res, g = (None, None) if args.no_ba else run_ba(args, local_rank, torch)
    if ba_res is not None and world == 1 and not args.no_all_cores:
        ba_res["many_windows"] = run_ba_many_child(local_rank)
    pose_res, pb = (None, None) if args.no_pose else run_pose(args, rank, world, local_rank, torch, dist)
    track_res, tctx = (None, None) if args.no_tracking else run_tracking(args, rank, world, local_rank, torch, dist)
    if world > 1:
        dist.barrier()

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": orb_res["value"],
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": orb_res["ms_per_step"],
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic",
            "config": {"workload": f"C2: {args.width}x{args.height} synthetic pan sequence, {args.features} "
                                   f"features/frame, ORB extract + two-way match vs previous frame"
                                   + (f"; C5: {world} independent sequences, one per GPU" if world > 1 else ""),
                       "frames_per_step": args.batch, "hip_streams": args.streams, "resident_frames_per_rank": max(args.batch, (args.frames // args.batch) * args.batch),
                       "parallelism": f"sequence-sharded x{world}"},
            "roofline": orb_res.get("roofline"),
            "kernels": orb_res["kernels"],
            "mean_keypoints": orb_res["mean_keypoints"],
            "mean_matches": orb_res["mean_matches"],
            "parity": orb_res.get("parity"),
        }
        if args.rehearse_one_gpu and world > 1:
            out["rehearsal"] = (f"{world} ranks sharing cuda:0 with gloo collectives (bench.py --rehearse-one-gpu): "
                                "the C5 flow, not a scaling measurement")
        failed = [k for k, v in (("ba.many_windows", (ba_res or {}).get("many_windows")),) if v and v.get("status") == "failed"]
        if failed:
            out["failed_legs"] = failed
        if pipe_res is not None:
            out["pipelined"] = pipe_res
        if r31_res is not None:
            out["rbrief31"] = {
                "metric": "frames/sec ORB extract+match @720p, rBRIEF-31 variant (4 levels x 1.5, 31x31 patch, "
                          "orientation)", "value": r31_res["value"], "unit": "frames/s",
                "ms_per_step": r31_res["ms_per_step"], "steps": args.rbrief31_steps,
                "config": {"workload": f"C2 frames ({args.width}x{args.height}, {args.features} features/frame) with "
                                       "NumLevels 4, PatchSize 31, UseOrientation (OpenCVModified.cpp:833, 867-871)",
                           "frames_per_step": args.batch},
                "roofline": r31_res.get("roofline"), "kernels": r31_res["kernels"],
                "mean_keypoints": r31_res["mean_keypoints"], "mean_matches": r31_res["mean_matches"],
                "parity": r31_res.get("parity")}
        if ba_res is not None:
            out["ba"] = ba_res
        if pose_res is not None:
            out["pose_ba"] = pose_res
        if track_res is not None:
            out["tracking"] = track_res
        if world == 1 and not args.no_cpu_baseline:
            use_native_oracle()
            out["cpu_baseline"] = median_of(lambda b: cpu_orb_baseline(args, b), args.cpu_sample_s)
            if r31_res is not None:
                c31 = median_of(lambda b: cpu_orb_baseline(args, b, RBRIEF31_ORACLE), args.cpu_sample_s / 2)
                out["rbrief31"]["cpu_baseline"] = c31
                out["rbrief31"]["vs_cpu"] = out["rbrief31"]["value"] / c31["value"]
            n32 = host_threads(NODE_SHARE_THREADS)
            share32 = not args.no_all_cores and n32 > host_threads()
            if not args.no_all_cores:
                out["cpu_baseline_all_cores"] = cpu_orb_baseline_all(args, args.cpu_sample_s / 2)
                out["vs_cpu_all_cores"] = out["value"] / out["cpu_baseline_all_cores"]["value"]
            if share32:  # one GPU's share of a 256-core 8-GPU node
                out["cpu_baseline_node_share"] = cpu_orb_baseline_all(args, args.cpu_sample_s / 2, n32)
                out["vs_cpu_node_share"] = out["value"] / out["cpu_baseline_node_share"]["value"]
            if ba_res is not None:
                cb = median_of(lambda b: cpu_ba_baseline(g, b), args.cpu_sample_s)
                ba_res["cpu_baseline"] = cb
                rs = ba_res["reference_schedule"]
                rs["cpu_baseline"] = median_of(lambda b: cpu_ba_reference_baseline(g, b), args.cpu_sample_s)
                rs["vs_cpu"] = rs["value"] / rs["cpu_baseline"]["value"]
                if not args.no_all_cores:
                    ca = cpu_ba_baseline_all(g, args.cpu_sample_s / 2)
                    ba_res["cpu_baseline_all_cores"] = ca
                    ba_res["vs_cpu_all_cores"] = ba_res["value"] / ca["value"]
                    if "many_windows" in ba_res:
                        ba_res["many_windows"]["vs_cpu_all_cores"] = ba_res["many_windows"]["value"] / ca["value"]
                    rca = cpu_ba_reference_baseline_all(g, args.cpu_sample_s / 2)
                    rs["cpu_baseline_all_cores"] = rca
                    rs["vs_cpu_all_cores"] = rs["value"] / rca["value"]
                    mref = (ba_res.get("many_windows") or {}).get("reference_schedule")
                    if mref:
                        mref["vs_cpu_all_cores"] = mref["value"] / rca["value"]
                if share32:
                    c32 = cpu_ba_baseline_all(g, args.cpu_sample_s / 2, n32)
                    ba_res["cpu_baseline_node_share"] = c32
                    ba_res["vs_cpu_node_share"] = ba_res["value"] / c32["value"]
                    r32 = cpu_ba_reference_baseline_all(g, args.cpu_sample_s / 2, n32)
                    rs["cpu_baseline_node_share"] = r32
                    rs["vs_cpu_node_share"] = rs["value"] / r32["value"]
                ba_res["vs_cpu"] = ba_res["value"] / cb["value"]
            if track_res is not None:
                ct, parity = cpu_tracking_baseline(args, tctx, args.cpu_sample_s)
                track_res["cpu_baseline"] = ct
                track_res["vs_cpu"] = track_res["value"] / ct["value"]
                track_res["parity"] = parity
                if "depth_error" in parity and "depth_error" in track_res:
                    track_res["depth_error"]["parity"] = parity.pop("depth_error")
            if pose_res is not None:
                cp = median_of(lambda b: cpu_pose_baseline(pb, b), min(args.cpu_sample_s, 6.0))
                pose_res["cpu_baseline"] = cp
                pose_res["vs_cpu"] = pose_res["value"] / cp["value"]
            out["vs_cpu"] = out["value"] / out["cpu_baseline"]["value"]
            out["cpu_baseline_build"] = ORACLE_BUILD[0]
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
