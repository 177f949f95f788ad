#!/usr/bin/env python3
"""VO frames/sec (extract + match + pose) at 1241x376, 2000 keypoints/frame.

Workload: S = 8 synthetic KITTI-shape scene
sequences (camera +1.0 m/frame along z, 0.1 deg/frame yaw; seed = splitmix64(0xACE0 ^ seq<<32 ^
frame)), --frames frames each.  Sequence s runs on rank s mod G (config 5's partition: at G < 8
a GPU runs 8/G sequences as one frame stream on its context, vo_set_sequence_starts resetting
the trajectory at each sequence's first frame).  One step = every sequence of the rank through the
full per-frame path (blur -> response -> NMS/top-N -> orientation/descriptor ->
Hamming match -> 8-point RANSAC -> refit -> getPose -> trajectory update), from vo_reset, with the
frames already resident in HBM (uploaded before the timed region).  value = all ranks' frames /
the slowest rank's time.

Multi-GPU (python -m torch.distributed.run --nproc-per-node N bench.py --gpus N): one process
per GPU, no data-path collective; RCCL ("nccl") carries the barrier, the max-over-ranks time and
one all-reduce that assembles every sequence's poses on every rank, after which rank 0 runs each
sequence alone on its own GPU (one vo_reset + call per sequence, as the reference's one run() per
sequence) and checks the gathered rows bit for bit.

Also on the JSON line:
  roofline      the kernel with the largest per-frame time (the stencil: the extract queue it runs
                on is the critical path, busy ~89 % of a step; the pose queue overlaps it):
                SURVEY 8(d)'s algorithmic bytes per launch / its average launch time (HIP events on
                its stream inside the timed region) against 8 TB/s; traffic = PMC HBM bytes per
                launch from the committed profile; valu = VALU issue from the PMC profile
  kernels       every kernel's per-frame time, algorithmic bytes and VALU issue fraction
  variants      (N = 1) the 0.05 m/frame and low-inlier (0.12 m/frame) sequences, the 0.12 m/frame
                regime in the headline's shape (8 sequences as one stream), extract only
                (config 2), host-frame streaming from pinned memory (H2D inside the timing), the
                per-frame vo_process_frame rate, and 1920x1080 / N=4096 (config 4) with the 32-test
                and the 512-test matcher
  cpu_baseline  the CPU oracle (plain-C restatement of the reference path) on the host's cores,
                timed by rank 0 at every world size before the GPU is touched: one process per
                usable core (the affinity set, capped by the box's CPU share when OMP_NUM_THREADS /
                VO_CPU_SHARE states one; logical and physical counts on the line) over the same
                sequence, plus one process alone; its rows of sequence 0 are checked against the GPU's
"""
from __future__ import annotations

import argparse
import json
import multiprocessing as mp
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

METRIC = "VO frames/sec (extract+match+pose), 1241×376 mono, 2000 kpts/frame"
HBM_PEAK_GBS = 8000.0
# VALU issue peak: 256 CUs x 4 SIMDs, a wave64 VALU instruction every 4 cycles per SIMD
# (profiles/r2_valu_calibration.md: tools/valu_rate.hip measures 4-4.5 cycles for f32, int, f64, DPP)
VALU_CYCLES = 4
VALU_SIMDS = 1024
KERNELS = ["stencil", "select", "describe", "match", "ransac", "refit", "triangulate", "finalize", "trajectory"]
POSE_QUEUE = ["match", "ransac", "refit", "triangulate", "finalize"]     # the trajectory queue overlaps them
ROCPROF_NAME = {"stencil": "k_stencil", "select": "k_select", "describe": "k_describe", "match": "k_match",
                "ransac": "k_ransac_hyp", "refit": "k_refit", "triangulate": "k_triangulate",
                "finalize": "k_finalize", "trajectory": "k_traj"}
# committed rocprofv3 summaries (tools/profile.sh -> tools/rocprof_summary.py --json): kernel
# durations, PMC HBM bytes and VALU counters per launch
# (tools/gpu_evidence.sh writes them on the GPU box before the bench runs, from the same build;
# PROFILE_ROUND names the round whose files are read)
PROFILE_ROUND = os.environ.get("VO_PROFILE_ROUND", "r6")
PROFILES = {(1241, 376, 32): f"{PROFILE_ROUND}_kitti_kernels.json", (1920, 1080, 32): f"{PROFILE_ROUND}_1080_kernels.json",
            (1920, 1080, 512): f"{PROFILE_ROUND}_1080_512_kernels.json",
            (1241, 376, 32, 0.12): f"{PROFILE_ROUND}_kitti_012_kernels.json"}


def algorithmic_bytes(kernel: str, W: int, H: int, info: np.ndarray) -> float:
    """SURVEY 8(d)'s algorithmic HBM bytes per frame, B = W*H + 80n + 24M + 96, split by the
    kernel that moves each term (n = keypoints, M = matches, I = inliers, averaged over info):
    the image read (stencil), 8n keypoints written (select), 64n descriptors written (describe),
    8n prefixes read + 8M matches written (match), 16M match coordinates read (RANSAC), 96 B of
    R, t (the trajectory kernel, which writes the pose row).  Refit and triangulate have no term of their own in 8(d); they are given
    their 16I inlier coordinates read."""
    n = float(info[:, 0].mean())
    M = float(info[:, 1].mean())
    I = float(info[:, 2].mean())
    return {"stencil": W * H, "select": 8 * n, "describe": 64 * n, "match": 8 * n + 8 * M, "ransac": 16 * M,
            "refit": 16 * I, "triangulate": 16 * I, "finalize": 0.0, "trajectory": 96.0,
            "path": W * H + 80 * n + 24 * M + 96}[kernel]


def load_profile(W: int, H: int, bits: int, motion: float = 1.0):
    """The committed profile of this workload: PROFILE_ROUND's, else the newest earlier round's
    (profile_row then refuses its rows if they are of another kernel form than this run's)."""
    name = PROFILES.get((W, H, bits)) if motion == 1.0 else PROFILES.get((W, H, bits, motion))
    if not name:
        return None, None
    rounds = sorted({f.split("_")[0] for f in os.listdir(os.path.join(ROOT, "profiles")) if f[:1] == "r"},
                    key=lambda r: int(r[1:]) if r[1:].isdigit() else -1, reverse=True)
    for r in [PROFILE_ROUND] + [r for r in rounds if r != PROFILE_ROUND]:
        path = os.path.join(ROOT, "profiles", name.replace(PROFILE_ROUND + "_", r + "_", 1))
        try:
            return json.load(open(path))["kernels"], os.path.relpath(path, ROOT)
        except (OSError, KeyError, ValueError):
            continue
    return None, None


def profile_row(prof, kernel: str, forms: dict):
    """The profile's per-launch figures of `kernel`, a launch as the live timing counts it: one
    pose pass launches k_ransac_hyp twice (hypothesis chunks), so the pose-queue kernels are
    normalised by the passes (matcher calls) and the extract kernels by the batches (k_stencil).
    forms = Context.kernel_forms(): the exact kernel symbols each stage launched in this run, so a
    profile of another matcher or select form is never read as this one's (None then)."""
    if not prof:
        return None
    names = set(forms[kernel])
    rows = [r for k, r in prof.items() if k.split("<")[0] in names]
    if len({k.split("<")[0] for k in prof if k.split("<")[0] in names}) != len(names):
        return None                                  # the profile ran another form of this stage
    ref = set(forms["match"]) if kernel in POSE_QUEUE or kernel == "trajectory" else {"k_stencil"}
    ref_calls = [r["calls"] for k, r in prof.items() if k.split("<")[0] in ref]
    launches = max(ref_calls) if ref_calls else max(r["calls"] for r in rows)

    def per(key):
        if any(r.get(key) is None for r in rows):
            return None
        return sum(r[key] * r["calls"] for r in rows) / launches
    vi, gc = per("valu_insts"), per("grbm_cycles")
    return {"avg_us": per("avg_us"), "hbm_bytes": per("hbm_bytes_per_launch"), "valu_insts": vi,
            "valu_issue_frac": vi * VALU_CYCLES / (VALU_SIMDS * gc / 8) if vi is not None and gc else None,
            "symbols": sorted({k for k in prof if k.split("<")[0] in names})}


EXTRACT_QUEUE = ["stencil", "select", "describe"]
POSE_ONLY = ["match", "ransac"]                  # the pose queue itself (refit .. finalize run on the fit queue)


def dominant_kernel(per_frame: dict) -> str:
    """The roofline kernel: the largest per-frame kernel of the queue with the most per-frame time --
    the step's critical path (tools/step_timeline.py on a kernel trace: the extract queue ~87 %
    busy, the pose queue ~72 %), not merely the largest kernel of any queue."""
    ext = sum(per_frame.get(k, 0.0) for k in EXTRACT_QUEUE)
    # the pose queue runs the matcher and a pass's first RANSAC chunk ("ransac_pose"); "ransac" also
    # times the later chunks, which run on the trajectory queue
    pose = per_frame.get("match", 0.0) + per_frame.get("ransac_pose", per_frame.get("ransac", 0.0))
    queue = EXTRACT_QUEUE if ext >= pose else POSE_ONLY
    return max(queue, key=lambda k: per_frame.get(k, 0.0))


def roofline_entry(kernel: str, live: list, info: np.ndarray, W: int, H: int, prof, psrc, forms: dict) -> dict:
    """roofline object of `kernel`: SURVEY 8(d)'s algorithmic bytes per launch over its average
    launch time, the launches timed live with HIP events on its own stream (`live`: kernel_stats()
    of the timed calls); traffic and VALU issue from the committed PMC profile."""
    ms = [b[kernel][0] for b in live if kernel in b]
    fpl = [b[kernel][1] for b in live if kernel in b]
    dom_ms = float(np.mean(ms)) if ms else float("nan")
    dom_fpl = float(np.mean(fpl)) if fpl else float("nan")
    abytes = algorithmic_bytes(kernel, W, H, info) * dom_fpl
    achieved = abytes / (dom_ms * 1e-3) / 1e9
    prow = profile_row(prof, kernel, forms)
    return {"bound": "hbm", "kernel": kernel, "symbols": forms[kernel], "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": prow["hbm_bytes"] if prow else None, "traffic_source": psrc,
            "avg_launch_ms": dom_ms, "frames_per_launch": dom_fpl, "algorithmic_bytes_per_launch": abytes,
            "rocprof_avg_launch_us": prow["avg_us"] if prow else None,
            "choice": "largest per-frame kernel of the queue with the most per-frame time (the critical path)",
            "valu": None if not prow else {
                "insts_per_launch": prow["valu_insts"], "issue_frac": prow["valu_issue_frac"],
                "peak": f"{VALU_SIMDS} SIMDs x 1 wave64 VALU instruction / {VALU_CYCLES} cycles (PMC: SQ_INSTS_VALU, "
                        f"GRBM_GUI_ACTIVE)"}}


# -- multi-GPU harness (config 5) --------------------------------------------------------
def rank_sequences(n_seq: int, rank: int, world: int, scaling: str = "strong"):
    """The sequences rank `rank` runs.  strong (config 5): n_seq sequences in all, sequence s on
    rank s mod G; weak: n_seq sequences per rank, rank r owning r*n_seq .. r*n_seq+n_seq-1
    (every rank runs the N = 1 workload on sequences of its own seeds)."""
    if scaling == "weak":
        return [rank * n_seq + i for i in range(n_seq)]
    return [s for s in range(n_seq) if s % world == rank]


def dist_init(world: int, local: int, backend: str = "nccl"):
    """One process per GPU; RCCL ("nccl") carries the barrier, the max-time reduction and the
    pose gather (replicas: no data-path collective).  gloo is used by the CPU tests."""
    if world <= 1:
        return None
    import torch
    import torch.distributed as dist
    if backend == "nccl":
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        dist.init_process_group(backend)
    return dist


def aggregate(dist, dt: float, frames_per_rank: int, world: int, backend: str = "nccl", local: int = 0):
    """Whole-job throughput: all ranks' frames / the slowest rank's time."""
    if dist is not None:
        import torch
        dev = f"cuda:{local}" if backend == "nccl" else "cpu"
        tt = torch.tensor([dt, float(frames_per_rank)], dtype=torch.float64, device=dev)
        t_max = tt[:1].clone()
        dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
        f_sum = tt[1:].clone()
        dist.all_reduce(f_sum, op=dist.ReduceOp.SUM)
        return float(t_max.item()), float(f_sum.item()) / float(t_max.item())
    return dt, frames_per_rank * world / dt


def gather_poses(dist, local_rows: dict, owners: list, nframes: int, backend: str = "nccl", local: int = 0):
    """Every sequence's (nframes, 13) rows -- 12 pose values and the status -- on every rank, by
    sequence id: owners[r] lists rank r's sequences.  Each rank packs its rows into a (k, nframes,
    13) block, viewed as int64 so the collective moves raw bits (a SUM all-reduce turned -0.0 into
    +0.0), and one all_gather assembles the blocks."""
    n_seq = 1 + max(s for o in owners for s in o)
    out = np.zeros((n_seq, nframes, 13))
    rank = dist.get_rank() if dist is not None else 0
    kmax = max(len(o) for o in owners)
    buf = np.zeros((kmax, nframes, 13))
    for i, s in enumerate(owners[rank]):
        buf[i] = local_rows[s]
    if dist is None:
        for i, s in enumerate(owners[0]):
            out[s] = buf[i]
        return out
    import torch
    dev = f"cuda:{local}" if backend == "nccl" else "cpu"
    t = torch.from_numpy(buf.view(np.int64).copy()).to(dev)
    parts = [torch.empty_like(t) for _ in owners]
    dist.all_gather(parts, t)
    for r, o in enumerate(owners):
        blk = parts[r].cpu().numpy().view(np.float64)
        for i, s in enumerate(o):
            out[s] = blk[i]
    return out


# -- CPU baseline ------------------------------------------------------------------------
_CPU = {}


def _cpu_worker(budget_s: float, keep_rows: bool = False):
    """The oracle over the sequence, restarted at frame 0 after each pass, for ~budget_s.
    keep_rows: also return the first complete pass's rows (pose, status) -- the bench checks the
    GPU's rows of the same sequence against them."""
    import oracle as O
    frames, W, H, K, gt, N = (_CPU[k] for k in ("frames", "W", "H", "K", "gt", "N"))
    cfg = O.config(W, H, K=K.reshape(9), max_kpts=N)
    O.stage_reset()
    t0 = time.perf_counter()
    done = 0
    rows = None
    while True:
        vo = O.VO(cfg, gt=gt)
        pas = []
        for f in range(frames.shape[0]):
            p, st, _ = vo.process(frames[f])
            pas.append((p, st))
            done += 1
            if time.perf_counter() - t0 > budget_s and done >= 2:
                break
        vo.close()
        if keep_rows and rows is None and len(pas) == frames.shape[0]:
            rows = pas
        if time.perf_counter() - t0 > budget_s and (rows is not None or not keep_rows):
            break
    dt = time.perf_counter() - t0
    stages = O.stage_times()
    return (done, dt, rows, stages) if keep_rows else (done, dt, stages)


def stage_ms(stages, frames: int):
    """The oracle's stage timers (VisualOdometry.cpp:85-178) as ms per frame of the run, and the
    calls behind each (match / RANSAC / pose run only on frames that reach them)."""
    return {k: {"ms_per_frame": round(1e3 * sec / max(frames, 1), 4), "calls": n} for k, (sec, n) in stages.items()}


def cpu_share() -> dict:
    """The host cores the CPU baseline may use: the process's affinity set (logical CPUs), capped
    by the CPU share the box states (VO_CPU_SHARE, else OMP_NUM_THREADS: a gpurun box shows the whole
    machine's CPUs but gives one GPU's job 16), with the physical cores behind those logical CPUs
    (distinct (package, core) pairs in /proc/cpuinfo)."""
    aff = sorted(os.sched_getaffinity(0))
    share, src = None, None
    for k in ("VO_CPU_SHARE", "OMP_NUM_THREADS"):
        v = os.environ.get(k, "")
        if v.isdigit() and int(v) > 0:
            share, src = int(v), k
            break
    cores = {}
    try:
        cpu = pkg = None
        for line in open("/proc/cpuinfo"):
            key, _, val = line.partition(":")
            key, val = key.strip(), val.strip()
            if key == "processor":
                cpu, pkg = int(val), None
            elif key == "physical id":
                pkg = val
            elif key == "core id" and cpu is not None:
                cores[cpu] = (pkg, val)
    except (OSError, ValueError):
        pass
    phys = len({cores[c] for c in aff if c in cores}) or None
    workers = min(len(aff), share) if share else len(aff)
    return {"workers": workers, "affinity_logical_cpus": len(aff), "affinity_physical_cores": phys,
            "host_logical_cpus": os.cpu_count(), "share": share, "share_source": src}


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(frames, seq, budget_s: float, max_kpts: int, share: dict):
    """The CPU oracle over the bench sequence (restarted at frame 0 after each pass) for about
    budget_s seconds: share["workers"] forked processes, one per usable logical CPU (cpu_share),
    each running the sequence (throughput = all frames / the slowest process), and one process
    alone.  Runs before the process touches the GPU.  Returns (the JSON object, the single
    process's first complete pass as [(pose 3x4, status)] -- the oracle's rows of the sequence,
    checked against the GPU's)."""
    procs = share["workers"]
    _CPU.update(frames=frames, W=seq.W, H=seq.H, K=seq.K, gt=seq.gt(), N=max_kpts)
    one_done, one_dt, rows, one_st = _cpu_worker(budget_s, keep_rows=True)
    single = {"value": one_done / one_dt, "unit": "frames/s", "cores": 1, "kind": "port",
              "sample": f"{one_done} frames of the {frames.shape[0]}-frame sequence (restarted at frame 0 after "
                        f"each pass), oracle/vo_oracle.c in one process, {one_dt:.1f} s",
              "stages": stage_ms(one_st, one_done)}
    if procs <= 1:
        return dict(single, cpu_model=cpu_model(), host=share), rows
    pool = mp.get_context("fork").Pool(procs)
    try:
        res = pool.map(_cpu_worker, [budget_s] * procs)
    finally:
        pool.close()                       # workers exit normally (no terminate / SIGTERM)
        pool.join()
    done = sum(r[0] for r in res)
    dt = max(r[1] for r in res)
    tot = {k: (sum(r[2][k][0] for r in res), sum(r[2][k][1] for r in res)) for k in res[0][2]}
    lim = (f"capped at the box's CPU share {share['share_source']}={share['share']}" if share["share"]
           and share["share"] < share["affinity_logical_cpus"] else "the whole affinity set")
    return {"value": done / dt, "unit": "frames/s", "cores": procs, "kind": "port",
            "cores_note": f"{procs} logical CPUs used ({lim}; affinity set {share['affinity_logical_cpus']} logical "
                          f"CPUs on {share['affinity_physical_cores']} physical cores, host "
                          f"{share['host_logical_cpus']} logical CPUs)",
            "sample": f"{procs} processes (one per usable logical CPU), each running oracle/vo_oracle.c over the "
                      f"same {frames.shape[0]}-frame sequence for ~{budget_s:.0f} s: {done} frames in {dt:.1f} s",
            "stages": stage_ms(tot, done),
            "cpu_model": cpu_model(), "host": share, "host_cpus": os.cpu_count(), "single_thread": single}, rows


# -- GPU measurement helpers ---------------------------------------------------------------
def timed_rate(fn, frames_per_call: int, steps: int, warmup: int = 1) -> float:
    for _ in range(warmup):
        fn()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    return frames_per_call * steps / (time.perf_counter() - t0)


def breakdown(ctx, call) -> dict:
    """{kernel: (ms per launch, frames per launch)} of one call with every launch timed."""
    call(1)
    return ctx.kernel_stats()


def run_variants(args, ctx, W, H, frames0, gt0, extra, Context) -> dict:
    """Secondary lines (N = 1): other motions, extract only, host streaming, per-frame calls,
    and config 4 at 1920x1080."""
    out = {}
    steps = max(3, args.steps // 2)
    for tag, (fr, seq) in extra.items():
        if tag in ("x1080", "stream") or tag.startswith("li8_"):
            continue
        df = ctx.device_frames(fr)
        ctx.set_ground_truth(seq.gt())

        def go(timing=0, df=df):
            ctx.reset()
            return ctx.process_frames_device(df, timing=timing)
        rate = timed_rate(go, fr.shape[0], steps)
        _, st, info = go()
        ks = breakdown(ctx, go)
        out[tag] = {"fps": rate, "motion_m_per_frame": seq.step, "frames": fr.shape[0],
                    "mean_hypotheses": float(info[1:, 4].mean()), "mean_matches": float(info[1:, 1].mean()),
                    "mean_inliers": float(info[1:, 2].mean()), "fitted_fraction": float(info[1:, 5].mean()),
                    "frames_ok": int((st == 0).sum()),
                    "kernels_us_per_frame": {k: round(v[0] / v[1] * 1e3, 3) for k, v in ks.items() if v[1] > 0}}
        if tag.startswith("low_inlier"):
            # its own roofline entry, chosen as the headline's (here the pose queue, RANSAC running
            # hundreds of hypotheses per frame), timed live over `steps` calls like the headline's
            per_frame = {k: v[0] / v[1] for k, v in ks.items() if v[1] > 0}
            dom = dominant_kernel(per_frame)
            live = []
            for _ in range(steps):
                go(timing=100 + KERNELS.index(dom))
                live.append(ctx.kernel_stats())
            prof, psrc = load_profile(W, H, 32, motion=seq.step)
            out[tag]["roofline"] = roofline_entry(dom, live, info, W, H, prof, psrc, ctx.kernel_forms())
        df.free()
    # the tracking regime in the headline's shape: 8 sequences at 0.12 m/frame as one stream (the
    # one-sequence variant above is dominated by its pipeline fill and drain: 4 batches)
    li8 = sorted((t for t in extra if t.startswith("li8_")), key=lambda t: int(t[4:]))
    if li8:
        seqs8 = [extra[t][1] for t in li8]
        df = ctx.device_frames(np.concatenate([extra[t][0] for t in li8]))
        gt8 = np.concatenate([q.gt() for q in seqs8])
        F8 = extra[li8[0]][0].shape[0]
        st8 = [F8 * i for i in range(1, len(li8))]

        def go8(timing=0, df=df):
            ctx.reset()
            ctx.set_ground_truth(gt8)
            ctx.set_sequence_starts(st8)
            return ctx.process_frames_device(df, timing=timing)
        rate = timed_rate(go8, F8 * len(li8), steps)
        _, st, info = go8()
        ks = breakdown(ctx, go8)
        ctx.set_sequence_starts([])
        out["low_inlier_0.12_8seq"] = {
            "fps": rate, "motion_m_per_frame": seqs8[0].step, "frames": F8 * len(li8), "sequences": len(li8),
            "mean_hypotheses": float(info[:, 4].mean()), "mean_matches": float(info[:, 1].mean()),
            "mean_inliers": float(info[:, 2].mean()), "frames_ok": int((st == 0).sum()),
            "kernels_us_per_frame": {k: round(v[0] / v[1] * 1e3, 3) for k, v in ks.items() if v[1] > 0}}
        df.free()
    # extract only (config 2), device-resident frames of sequence 0
    df = ctx.device_frames(frames0)
    rate = timed_rate(lambda: ctx.extract_frames_device(df), frames0.shape[0], steps)
    ks = breakdown(ctx, lambda t: ctx.extract_frames_device(df, timing=t))
    out["extract_only"] = {"fps": rate, "frames": frames0.shape[0], "config": "2: extract only, device-resident",
                           "kernels_us_per_frame": {k: round(v[0] / v[1] * 1e3, 3) for k, v in ks.items()
                                                    if v[1] > 0},
                           "roofline_stencil_frac": None}
    if "stencil" in ks:
        ms, fpl = ks["stencil"]
        out["extract_only"]["roofline_stencil_frac"] = W * H * fpl / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS
    df.free()
    # host-frame streaming from pinned memory (H2D inside the timed region) against the same
    # frames device-resident: one 1000-frame sequence, so the per-call pipeline fill (the first
    # batch's copy) and drain (the last batch's extract and pass) are amortised as in a KITTI run
    if "stream" in extra:
        fr, seq = extra["stream"]
        ctx.set_ground_truth(seq.gt())
        dl = ctx.device_frames(fr)

        def dev(dl=dl):
            ctx.reset()
            return ctx.process_frames_device(dl)
        dev_rate = timed_rate(dev, fr.shape[0], 3)
        ref = dev()
        dl.free()
        hf = ctx.host_frames(fr)

        def host():
            ctx.reset()
            return ctx.process_frames_host(hf)
        host_rate = timed_rate(host, fr.shape[0], 3)
        got = host()
        same = bool(np.array_equal(got[0], ref[0]) and np.array_equal(got[1], ref[1]))
        out["host_stream"] = {"fps": host_rate, "device_resident_fps": dev_rate, "ratio": host_rate / dev_rate,
                              "h2d_GBs": host_rate * W * H / 1e9, "rows_equal_device_path": same,
                              "frames": fr.shape[0], "motion_m_per_frame": seq.step,
                              "source": "pinned host memory (vo_host_alloc), vo_process_frames_host, one call per "
                                        "sequence pass"}
        hf.free()
    # per-frame calls (vo_process_frame: host frame in, pose out, one frame per call)
    nf = min(100, frames0.shape[0])

    def per_frame():
        ctx.reset()
        for f in range(nf):
            ctx.process_frame(frames0[f])
    out["process_frame"] = {"fps": timed_rate(per_frame, nf, 2), "frames": nf,
                            "note": "one vo_process_frame call per frame from pageable numpy frames (staging copy "
                                    "+ extract + pose + pose row back, host sync)"}
    hpf = ctx.host_frames(frames0[:nf])

    def per_frame_pinned():
        ctx.reset()
        for f in range(nf):
            ctx.process_frame(hpf.array[f])
    out["process_frame"]["pinned_source_fps"] = timed_rate(per_frame_pinned, nf, 2)
    out["process_frame"]["pinned_source_note"] = ("the same calls with the frames in pinned host memory "
                                                  "(vo_host_alloc): the stencil reads each frame over PCIe "
                                                  "where it lies, no staging copy")
    hpf.free()
    # config 4: 1920x1080, N = 4096, 32-test and 512-test matching
    if "x1080" in extra:
        fr, seq = extra["x1080"]
        for bits in (32, 512):
            cx = Context(seq.W, seq.H, K=seq.K, max_kpts=4096, match_bits=bits)
            cx.set_ground_truth(seq.gt())
            dx = cx.device_frames(fr)

            def g(timing=0, cx=cx, dx=dx):
                cx.reset()
                return cx.process_frames_device(dx, timing=timing)
            rate = timed_rate(g, fr.shape[0], steps)
            _, st, info = g()
            ks = breakdown(cx, g)
            prof, src = load_profile(seq.W, seq.H, bits)
            prow = profile_row(prof, "match", cx.kernel_forms())
            out[f"x1080_{bits}bit"] = {
                "fps": rate, "frames": fr.shape[0], "match_bits": bits, "motion_m_per_frame": seq.step,
                "frames_ok": int((st == 0).sum()), "mean_matches": float(info[1:, 1].mean()),
                "match_us_per_launch": ks.get("match", (float("nan"), 0))[0] * 1e3,
                "match_frames_per_launch": ks.get("match", (0, 0))[1],
                "match_kernel": cx.kernel_forms()["match"],
                "match_rocprof_avg_us": prow["avg_us"] if prow else None,
                "match_valu_issue_frac": prow["valu_issue_frac"] if prow else None, "profile": src,
                "kernels_us_per_frame": {k: round(v[0] / v[1] * 1e3, 3) for k, v in ks.items() if v[1] > 0}}
            dx.free()
            cx.close()
    return out


def context_class():
    """The engine: the HIP library's Context (no other; tests/test_multirank.py substitutes a stand-in
    here to run the N > 1 harness end to end on CPU-only machines)."""
    from acs_visual_odometry_amd import Context
    return Context


def render_workers(world: int) -> int:
    """Forked processes rendering the synthetic frames: the rank's part of the CPU share."""
    return max(1, min(16, cpu_share()["workers"]) // max(world, 1))


def shard_main(args, world: int, rank: int, local: int):
    """--shard-sequence: ONE sequence of sequences x frames frames split into G contiguous shards
    (acs_visual_odometry_amd/shard.py).  Each rank holds the frames up to the end of
    its shard in HBM, runs its halo stream, the flag exchange, a second run where needed and the
    T_curr hand-over (RCCL send/recv of 16 doubles).  value = the sequence's frames / the slowest
    rank's time; rank 0 checks the gathered rows against the unsplit run on its own GPU."""
    from acs_visual_odometry_amd import shard
    from acs_visual_odometry_amd.synth import SceneSequence, render_sequences
    W, H = args.width, args.height
    F = args.frames * args.sequences
    a, b = shard.partition(F, world)[rank]
    workers = render_workers(world)
    seq = SceneSequence(W, H, nframes=F, seq=0, step=args.motion)
    need = F if rank == 0 else b                      # rank 0 also runs the unsplit check
    frames = render_sequences([(W, H, F, 0, args.motion)], workers)[0][:need]
    dev = local if args.device < 0 else args.device
    dist = dist_init(world, dev, backend=args.backend)
    Context = context_class()
    ctx = Context(W, H, K=seq.K, max_kpts=args.max_kpts, device=dev, frame_batch=args.batch,
                  match_bits=args.match_bits)
    dall = ctx.device_frames(frames)
    gt = seq.gt()
    eng = shard.ContextEngine(ctx, dall, gt)

    class One:
        rank, world = 0, 1

    comm = (shard.TorchComm(dist, device=f"cuda:{dev}" if args.backend == "nccl" else "cpu") if dist is not None
            else One())

    def step():
        return shard.run_shard(eng, comm, F) if dist is not None else shard.run_local([eng], F)[0]

    def barrier():
        if dist is not None:
            dist.barrier()

    for _ in range(max(args.warmup, 1)):
        res = step()
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res = step()
    dt = time.perf_counter() - t0
    barrier()
    dt, _ = aggregate(dist, dt, 0, world, backend=args.backend, local=dev)
    value = F * args.steps / dt
    rows = np.concatenate([res.poses.reshape(-1, 12), res.status.reshape(-1, 1).astype(np.float64)], axis=1)
    if dist is not None:
        allrows = [None] * world
        dist.all_gather_object(allrows, (rows, res.runs, res.a - res.start))
    else:
        allrows = [(rows, res.runs, res.a - res.start)]
    if rank == 0:
        ctx.reset()
        ctx.set_sequence_starts([])
        ctx.set_frame_origin(0)
        ctx.set_ground_truth(gt)
        p, st, info = ctx.process_frames_device(dall)
        unsplit = np.concatenate([p.reshape(F, 12), st.reshape(F, 1).astype(np.float64)], axis=1)
        ok = bool(np.array_equal(np.concatenate([r[0] for r in allrows]), unsplit))
        line = {
            "metric": METRIC, "value": value, "unit": "frames/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": dt / args.steps * 1e3, "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "u8/f32/u32/f64", "data": "synthetic",
            "config": {"workload": f"{W}x{H}_{args.max_kpts}kpts_one_sequence_sharded", "frames": F,
                       "width": W, "height": H, "max_kpts": args.max_kpts, "match_bits": args.match_bits,
                       "motion": f"+{args.motion} m/frame along z, 0.1 deg/frame yaw",
                       "parallelism": f"one sequence in {world} contiguous shards, halo {shard.DEFAULT_HALO} frames, "
                                      f"T_curr handed over rank to rank",
                       "inputs": "device-resident (HBM) before timing", "shard_runs": [r[1] for r in allrows],
                       "halo_frames": [r[2] for r in allrows]},
            "determinism": {"shard_rows_equal_unsplit_run": ok},
        }
        print(json.dumps(line))
    dall.free()
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--frames", type=int, default=200, help="frames per sequence")
    ap.add_argument("--sequences", type=int, default=8,
                    help="sequences per rank (--scaling weak) or of the whole job (strong; config 5: 8)")
    ap.add_argument("--scaling", choices=("weak", "strong"), default="weak",
                    help="weak: every rank runs --sequences sequences of its own (the N = 1 workload per GPU); "
                         "strong: --sequences sequences in all, sequence s on rank s mod G (config 5)")
    ap.add_argument("--width", type=int, default=1241)
    ap.add_argument("--height", type=int, default=376)
    ap.add_argument("--max-kpts", type=int, default=2000)
    ap.add_argument("--match-bits", type=int, default=32)
    ap.add_argument("--motion", type=float, default=1.0, help="metres per frame of the synthetic camera")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--batch", type=int, default=0, help="frames per extract batch / pose window (0: default)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-variants", action="store_true")
    ap.add_argument("--no-check", action="store_true",
                    help="skip the per-sequence separate runs after timing (profiles: every launch is then a bench launch)")
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend (nccl = RCCL; gloo for CPU/one-GPU rehearsal)")
    ap.add_argument("--device", type=int, default=-1, help="GPU of every rank (default: LOCAL_RANK; one-GPU rehearsal: 0)")
    ap.add_argument("--shard-sequence", action="store_true",
                    help="one sequence (sequences x frames frames) split over the ranks (within-sequence sharding)")
    ap.add_argument("--breakdown", action="store_true", help="print the per-kernel table to stderr")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    if world != args.gpus:
        print(f"[bench] --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)
    if args.shard_sequence:
        return shard_main(args, world, rank, local)
    W, H, F = args.width, args.height, args.frames
    S = args.sequences if args.scaling == "weak" else max(args.sequences, world)   # strong: >= 1 per rank
    my_seqs = rank_sequences(S, rank, world, args.scaling)
    owners = [rank_sequences(S, r, world, args.scaling) for r in range(world)]
    n_total = sum(len(o) for o in owners)
    lead = rank == 0 and world == 1                      # the N = 1 variants
    # the CPU baseline and its oracle-row check run on rank 0 at every world size (north_star: the
    # reference CPU path timed on the same box in the same run)

    # -- host-side preparation, before anything touches the GPU (forked workers) --
    from acs_visual_odometry_amd.synth import SceneSequence, render_sequences
    workers = render_workers(world)
    # N > 1 with weak scaling: config 5 literally as well (8 sequences in all, sequence s on GPU s mod G),
    # timed after the weak-scaling line's run and reported beside it (config5_strong)
    c5_seqs = rank_sequences(8, rank, world, "strong") if world > 1 and args.scaling == "weak" else []
    specs = [(W, H, F, s, args.motion) for s in my_seqs] + [(W, H, F, s, args.motion) for s in c5_seqs
                                                            if s not in my_seqs]
    extra_specs = {}
    if lead and not args.no_variants:
        extra_specs = {"motion_0.05": (W, H, F, 0, 0.05), "low_inlier_0.12": (W, H, F, 0, 0.12),
                       "x1080": (1920, 1080, 64, 0, args.motion), "stream": (W, H, 1000, 0, args.motion)}
        extra_specs.update({f"li8_{s}": (W, H, F, s, 0.12) for s in range(8)})
    rendered = render_sequences(specs + list(extra_specs.values()), workers)
    seqs = {sp[3]: (SceneSequence(W, H, nframes=F, seq=sp[3], step=args.motion), rendered[i])
            for i, sp in enumerate(specs)}
    n_mine = len(specs)
    extra = {tag: (rendered[n_mine + i], SceneSequence(sp[0], sp[1], nframes=sp[2], seq=sp[3], step=sp[4]))
             for i, (tag, sp) in enumerate(extra_specs.items())}
    cpu, oracle_rows = None, None
    if rank == 0 and not args.no_cpu:
        s0, fr0 = seqs[my_seqs[0]]
        cpu, oracle_rows = cpu_baseline(fr0, s0, args.cpu_seconds, args.max_kpts, cpu_share())

    dev = local if args.device < 0 else args.device     # (--device 0 --backend gloo: ranks sharing one GPU)
    if world > 1:
        # the context's four queues plus RCCL's streams: room for all of them on hardware queues of
        # their own (HIP's default is 4 per process; a stream past them shares one and serialises
        # behind its kernels).  Measured neutral at N = 1 (gpurun_out r5g); set before HIP starts.
        os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")
    dist = dist_init(world, dev, backend=args.backend)
    Context = context_class()

    ctx = Context(W, H, K=seqs[my_seqs[0]][0].K, max_kpts=args.max_kpts, device=dev, frame_batch=args.batch,
                  match_bits=args.match_bits)
    # the rank's sequences as one frame stream: frames and GT rows concatenated, each sequence's
    # first frame marked (vo_set_sequence_starts), so the next sequence's extract overlaps the
    # previous one's last pose passes; rows are split back per sequence
    dall = ctx.device_frames(np.concatenate([seqs[s][1] for s in my_seqs]))
    gts = {s: seqs[s][0].gt() for s in my_seqs}
    gt_all = np.concatenate([gts[s] for s in my_seqs])
    starts = [F * i for i in range(1, len(my_seqs))]
    last = {}

    def step(timing=0, stats=None):
        ctx.reset()
        ctx.set_ground_truth(gt_all)
        ctx.set_sequence_starts(starts)
        poses, st, info = ctx.process_frames_device(dall, timing=timing)
        for i, s in enumerate(my_seqs):
            last[s] = (poses[i * F:(i + 1) * F], st[i * F:(i + 1) * F], info[i * F:(i + 1) * F])
        if stats is not None:
            stats.append(ctx.kernel_stats())

    def separate(s, frames):
        """Sequence s alone (its own stream: the reference's one run() per sequence)."""
        df = ctx.device_frames(frames)
        ctx.reset()
        ctx.set_sequence_starts([])
        ctx.set_ground_truth(seqs[s][0].gt())
        p, st, _ = ctx.process_frames_device(df)
        df.free()
        return np.concatenate([p.reshape(F, 12), st.reshape(F, 1).astype(np.float64)], axis=1)

    def barrier():
        if dist is not None:
            dist.barrier()

    for _ in range(max(args.warmup, 1)):
        step()
    warm = {s: (last[s][0].copy(), last[s][1].copy()) for s in my_seqs}
    # per-kernel breakdown (untimed): every launch bracketed by events
    bd = []
    step(timing=1, stats=bd)
    ks = {k: (float(np.mean([b[k][0] for b in bd if k in b])), float(np.mean([b[k][1] for b in bd if k in b])))
          for k in KERNELS + ["ransac_pose"] if any(k in b for b in bd)}
    info_all = np.concatenate([last[s][2] for s in my_seqs])
    per_frame = {k: ks[k][0] / ks[k][1] if k in ks and ks[k][1] > 0 else 0.0 for k in KERNELS + ["ransac_pose"]}
    dominant = dominant_kernel(per_frame)
    kidx = KERNELS.index(dominant)

    barrier()
    live = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(timing=100 + kidx, stats=live)          # two events around every 4th dominant launch
    t1 = time.perf_counter()
    barrier()
    dt = t1 - t0
    frames_rank = args.steps * F * len(my_seqs)
    dt, value = aggregate(dist, dt, frames_rank, world, backend=args.backend, local=dev)
    repeat_equal = all(np.array_equal(warm[s][0], last[s][0]) and np.array_equal(warm[s][1], last[s][1])
                       for s in my_seqs)
    rows = {s: np.concatenate([last[s][0].reshape(F, 12), last[s][1].reshape(F, 1).astype(np.float64)], axis=1)
            for s in my_seqs}
    gathered = gather_poses(dist, rows, owners, F, backend=args.backend, local=dev)
    # every rank runs each of its sequences alone, as the reference would (one run() each); those
    # rows are gathered too and rank 0 checks every sequence's stream rows against them bit for bit
    gather_ok = None
    if not args.no_check:
        sep = gather_poses(dist, {s: separate(s, seqs[s][1]) for s in my_seqs}, owners, F, backend=args.backend,
                           local=dev)
        gather_ok = bool(np.array_equal(sep.view(np.int64), gathered.view(np.int64)))
    # the CPU oracle's rows of the first sequence (the cpu_baseline leg's first complete pass)
    # against the GPU's rows of that sequence in the timed stream, bit for bit
    oracle_ok = None
    if oracle_rows is not None:
        s0 = my_seqs[0]
        oracle_ok = bool(len(oracle_rows) == F and
                         all(np.array_equal(last[s0][0][f], oracle_rows[f][0]) and int(last[s0][1][f]) == oracle_rows[f][1]
                             for f in range(F)))

    # config 5 literally (N > 1, weak-scaling line): 8 sequences in all, sequence s on GPU s mod G, each
    # rank's sequences as one stream; the same barrier / max-over-ranks timing
    c5 = None
    if c5_seqs:
        d5 = ctx.device_frames(np.concatenate([seqs[s][1] for s in c5_seqs]))
        gt5 = np.concatenate([seqs[s][0].gt() for s in c5_seqs])
        st5 = [F * i for i in range(1, len(c5_seqs))]

        res5 = {}

        def step5(timing=0, stats=None):
            ctx.reset()
            ctx.set_ground_truth(gt5)
            ctx.set_sequence_starts(st5)
            res5["out"] = ctx.process_frames_device(d5, timing=timing)
            if stats is not None:
                stats.append(ctx.kernel_stats())

        for _ in range(max(args.warmup, 1)):
            step5()
        # its own critical-path kernel (one untimed call with every launch timed), then timed live
        # inside the timed region as the headline's is
        bd5 = []
        step5(timing=1, stats=bd5)
        ks5 = {k: (float(np.mean([b[k][0] for b in bd5 if k in b])), float(np.mean([b[k][1] for b in bd5 if k in b])))
               for k in KERNELS + ["ransac_pose"] if any(k in b for b in bd5)}
        dom5 = dominant_kernel({k: ks5[k][0] / ks5[k][1] if k in ks5 and ks5[k][1] > 0 else 0.0
                                for k in KERNELS + ["ransac_pose"]})
        live5 = []
        barrier()
        t5 = time.perf_counter()
        for _ in range(args.steps):
            step5(timing=100 + KERNELS.index(dom5), stats=live5)
        t5 = time.perf_counter() - t5
        barrier()
        t5, v5 = aggregate(dist, t5, args.steps * F * len(c5_seqs), world, backend=args.backend, local=dev)
        info5 = res5["out"][2]
        c5 = {"value": v5, "unit": "frames/s", "ms_per_step": t5 / args.steps * 1e3, "sequences": 8,
              "sequences_per_gpu": [len(rank_sequences(8, r, world, "strong")) for r in range(world)],
              "scaling": "strong", "parallelism": f"config 5: sequence s of 0..7 on GPU s mod {world}",
              "roofline": roofline_entry(dom5, live5, info5, W, H, *load_profile(W, H, args.match_bits),
                                         ctx.kernel_forms())}
        d5.free()
        ctx.set_sequence_starts([])

    dev_errors = ctx.device_errors()                 # select consistency failures (expected 0)
    variants = None
    if lead and not args.no_variants:
        s0 = my_seqs[0]
        ctx.set_sequence_starts([])
        variants = run_variants(args, ctx, W, H, seqs[s0][1], gts[s0], extra, Context)

    if rank == 0:
        prof, psrc = load_profile(W, H, args.match_bits)
        forms = ctx.kernel_forms()
        roof = roofline_entry(dominant, live, info_all, W, H, prof, psrc, forms)
        path_bytes = algorithmic_bytes("path", W, H, info_all)
        kern = {}
        for k in KERNELS:
            if k not in ks:
                continue
            r = profile_row(prof, k, forms)
            kern[k] = {"symbols": forms[k],"us_per_frame": round(per_frame[k] * 1e3, 4), "us_per_launch": round(ks[k][0] * 1e3, 2),
                       "frames_per_launch": round(ks[k][1], 2),
                       "algorithmic_bytes_per_frame": round(algorithmic_bytes(k, W, H, info_all), 1),
                       "queue": "pose" if k in POSE_QUEUE else ("trajectory" if k == "trajectory" else "extract"),
                       "pmc_hbm_bytes_per_launch": r["hbm_bytes"] if r else None,
                       "valu_issue_frac": r["valu_issue_frac"] if r else None}
        if "ransac_pose" in ks and ks["ransac_pose"][1] > 0:
            kern["ransac_pose"] = {"us_per_frame": round(per_frame["ransac_pose"] * 1e3, 4), "queue": "pose",
                                   "note": "the first RANSAC chunk of each pass (the pose queue's share of 'ransac')"}
        st_all = np.concatenate([last[s][1] for s in my_seqs])
        line = {
            "metric": METRIC, "value": value, "unit": "frames/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": dt / args.steps * 1e3, "higher_is_better": True,
            "scaling": args.scaling, "vs_baseline": None, "dtype": "u8/f32/u32/f64", "data": "synthetic",
            "config": {"workload": ("kitti_1241x376_2000kpts_full_path" if (W, H) == (1241, 376)
                                    else f"{W}x{H}_{args.max_kpts}kpts_full_path"),
                       "sequences": n_total, "frames_per_sequence": F, "sequences_per_gpu": len(my_seqs),
                       "width": W, "height": H, "max_kpts": args.max_kpts, "match_bits": args.match_bits,
                       "motion": f"+{args.motion} m/frame along z, 0.1 deg/frame yaw (SURVEY 8(d) scene generator)",
                       "parallelism": (f"{world} GPU(s) x {S} sequences each (weak scaling: sequences r*{S} .. "
                                       f"r*{S}+{S - 1} on GPU r), no data-path collective" if args.scaling == "weak"
                                       else f"config 5: sequence s on GPU s mod {world}, no data-path collective"),
                       "frame_batch": ctx.cfg.frame_batch or 64, "inputs": "device-resident (HBM) before timing",
                       "mean_kpts": float(info_all[:, 0].mean()), "mean_matches": float(info_all[:, 1].mean()),
                       "mean_inliers": float(info_all[:, 2].mean()),
                       "mean_hypotheses": float(info_all[:, 4].mean()),
                       "fitted_fraction": float(info_all[np.concatenate([last[s][1] for s in my_seqs]) != 1, 5].mean()),
                       "frames_ok": int((st_all == 0).sum()), "frames": int(st_all.size)},
            "roofline": roof,
            # SURVEY 8(d) times "from frame H2D to pose D2H": the same path with the frames streamed
            # from pinned host memory (a 1000-frame sequence, vo_process_frames_host); never `value`
            "h2d_inclusive": None if not variants or "host_stream" not in variants else {
                "value": variants["host_stream"]["fps"], "unit": "frames/s",
                "source": "variants.host_stream (pinned host frames, H2D on a copy queue inside the timing)"},
            "path_roofline": {"algorithmic_bytes_per_frame": path_bytes,
                              "achieved_GBs": path_bytes * value / world / 1e9,
                              "frac": path_bytes * value / world / 1e9 / HBM_PEAK_GBS},
            "kernels": kern,
            "determinism": {"timed_rows_equal_warmup_rows": bool(repeat_equal),
                            "device_errors": dev_errors,
                            "gathered_rows_equal_separate_runs": gather_ok,
                            "gather": "all_gather of raw int64 bits (stream rows and separate-run rows of every "
                                      "sequence)",
                            "oracle_rows_equal": oracle_ok,
                            "oracle_rows_checked": f"sequence {my_seqs[0]}: {F} frames (pose rows + statuses) against "
                                                   f"the CPU oracle's run in the cpu_baseline leg" if oracle_ok is not None
                            else None},
            "variants": variants,
            "cpu_baseline": cpu,
        }
        if c5 is not None:
            line["config5_strong"] = c5
        if args.breakdown:
            for k in KERNELS:
                if k in ks:
                    print(f"{k:14s} {per_frame[k] * 1e3:9.2f} us/frame  {ks[k][0] * 1e3:9.1f} us/launch  "
                          f"{ks[k][1]:5.1f} frames/launch", file=sys.stderr)
        print(json.dumps(line))
    dall.free()
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
