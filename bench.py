#!/usr/bin/env python3
"""VO frames/sec (extract + match + pose) at 1241x376, 2000 keypoints/frame.

One step = one pass of the full per-frame hot path (blur -> response -> NMS/top-N ->
orientation/descriptor -> Hamming match -> 8-point RANSAC -> refit -> getPose ->
trajectory update) over a synthetic KITTI-shape sequence of --frames frames that is
already resident in HBM (uploaded before the timed region).  Frames are enqueued back
to back on the ctx's HIP stream; the step ends with one stream synchronisation.

Multi-GPU (python -m torch.distributed.run --nproc-per-node N bench.py --gpus N):
replicas -- rank r processes its own sequence (seq = r) on GPU LOCAL_RANK with no
data-path collective; the barrier and the max-over-ranks step time go over RCCL
("nccl" backend).  value = frames processed by all ranks / max rank time (weak scaling).

Also reported, on the same JSON line:
  roofline      -- the dominant kernel's algorithmic bytes per launch / its average
                   launch time (HIP events on the ctx stream, inside the timed region)
                   against the MI355X HBM peak (8 TB/s)
  cpu_baseline  -- the CPU oracle (a plain-C restatement of the reference path, one host
                   core) timed on a bounded sample of the same sequence (rank 0, N=1)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

METRIC = "VO frames/sec (extract+match+pose), 1241×376 mono, 2000 kpts/frame"
# committed rocprofv3 FETCH_SIZE / WRITE_SIZE summaries of the two bench configs (tools/profile.sh
# -> tools/rocprof_summary.py --fetch-x2 --json): the source of roofline.traffic
PMC_PROFILES = {(1241, 376): "r1_batched_kitti_kernels.json", (1920, 1080): "r1_batched_1080_kernels.json"}
ROCPROF_NAME = {"stencil": "k_stencil", "select": "k_select", "describe": "k_describe", "match": "k_match",
                "ransac": "k_ransac_hyp", "refit": "k_refit", "triangulate": "k_triangulate",
                "finalize": "k_finalize"}
HBM_PEAK_GBS = 8000.0
KERNELS = ["stencil", "select", "describe", "match", "ransac", "refit", "triangulate", "finalize"]


def algorithmic_bytes(kernel: str, W: int, H: int, info: np.ndarray, N: int) -> float:
    """Algorithmic HBM bytes per frame of `kernel` (one launch, two for ransac), averaged
    over the frames in `info` (n_kps, n_matches, n_inliers, ...).  DESIGN.md section 4
    derives each figure; n = keypoints, M = matches, I = inliers."""
    n = float(info[:, 0].mean())
    M = float(info[:, 1].mean())
    I = float(info[:, 2].mean())
    if kernel == "stencil":
        return 2.0 * W * H + 4 * 8 * n                # frame in + blurred out + ~4n candidate keys
    if kernel == "select":
        return 4 * 8 * n + 8 * n                      # ~4n candidate keys in, n keypoints out
    if kernel == "describe":
        return (86 + 8 + 64 + 4) * n                  # 86 sampled px + kp in; descriptor + prefix out
    if kernel == "match":
        return 3 * 4 * n + 8 * M                      # two 32-bit prefix sets + best index; pairs out
    if kernel == "ransac":
        return 32 * M + 36 * 4                        # match coords once (L2 re-reads excluded)
    if kernel == "refit":
        return 32 * M + 4 * I + 72 + 16 * I           # coords + inlier ids; F + f32 inlier points out
    if kernel == "triangulate":
        return 16 * I + 96 + 96                       # f32 inlier points in; candidate counts out
    if kernel == "finalize":
        return 2 * 96 + 96 + 128                      # two GT rows + R, t in; the output row
    return float(W * H + 80 * n + 24 * M + 96)       # whole path


def pmc_traffic(kernel: str, W: int, H: int):
    """HBM bytes per launch of `kernel` from the committed PMC profile of this frame size (None
    if absent); the RANSAC launches of a pass count as one launch, as in the live timing."""
    if (W, H) not in PMC_PROFILES:
        return None, None
    PMC_PROFILE = os.path.join(ROOT, "profiles", PMC_PROFILES[(W, H)])
    try:
        prof = json.load(open(PMC_PROFILE))["kernels"]
        rows = [r for k, r in prof.items() if k.split("<")[0] == ROCPROF_NAME[kernel]]   # template instances
        total = sum(r["hbm_bytes_per_launch"] for r in rows)
        return (total if rows else None), os.path.relpath(PMC_PROFILE, ROOT)
    except (OSError, KeyError, TypeError, ZeroDivisionError, ValueError):
        return None, None


def dist_init(world: int, local: int, backend: str = "nccl"):
    """One process per GPU; RCCL ("nccl") carries only the barrier and the max-time
    reduction (replicas: no data-path collective).  gloo is used by the CPU tests."""
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
        tt = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    return dt, frames_per_rank * world / dt


def cpu_baseline(frames: np.ndarray, seq, budget_s: float, max_kpts: int) -> dict:
    """The CPU oracle over the same sequence, restarted from frame 0 after each pass, until
    the time budget is spent."""
    import oracle as O
    cfg = O.config(seq.W, seq.H, K=seq.K.reshape(9), max_kpts=max_kpts)
    t0 = time.perf_counter()
    done = passes = 0
    while True:
        vo = O.VO(cfg, gt=seq.gt())
        for f in range(frames.shape[0]):
            vo.process(frames[f])
            done += 1
            if time.perf_counter() - t0 > budget_s and done >= 2:
                break
        vo.close()
        passes += 1
        if time.perf_counter() - t0 > budget_s:
            break
    dt = time.perf_counter() - t0
    return {"value": done / dt, "unit": "frames/s", "cores": 1, "kind": "port",
            "sample": f"{done} frames ({passes} pass(es) over the {frames.shape[0]}-frame sequence, seq 0, "
                      f"{seq.W}x{seq.H}, N={max_kpts}), oracle/vo_oracle.c single thread, {dt:.1f} s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--frames", type=int, default=200, help="frames per step (one sequence pass)")
    ap.add_argument("--width", type=int, default=1241)
    ap.add_argument("--height", type=int, default=376)
    ap.add_argument("--max-kpts", type=int, default=2000)
    ap.add_argument("--motion", type=float, default=0.05, help="metres per frame of the synthetic camera")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--batch", type=int, default=0, help="frames per extract batch / pose window (0: default)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--breakdown", action="store_true", help="print the per-kernel table to stderr")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    if world != args.gpus:
        print(f"[bench] --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)

    dist = dist_init(world, local)

    from acs_visual_odometry_amd import Context
    from acs_visual_odometry_amd.synth import SceneSequence

    seq = SceneSequence(args.width, args.height, nframes=args.frames, seq=rank, step=args.motion)
    frames = seq.frames()
    ctx = Context(seq.W, seq.H, K=seq.K, max_kpts=args.max_kpts, device=local, frame_batch=args.batch)
    ctx.set_ground_truth(seq.gt())
    dframes = ctx.device_frames(frames)

    def step(timing=0):
        ctx.reset()
        return ctx.process_frames_device(dframes, timing=timing)

    def barrier():
        if dist is not None:
            dist.barrier()

    for _ in range(max(args.warmup, 1)):
        step()
    # per-kernel breakdown (untimed pass): every launch bracketed by events; a launch covers
    # frames_per_launch frames (an extract batch or a pose-pass window)
    _, st, info = step(timing=1)
    ks = ctx.kernel_stats()
    per_frame = {k: (ks[k][0] / ks[k][1] if k in ks and ks[k][1] > 0 else 0.0) for k in KERNELS}
    dominant = max(per_frame, key=lambda k: per_frame[k])
    kidx = KERNELS.index(dominant)

    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        poses, st, info = step(timing=100 + kidx)       # two events around the dominant kernel
    t1 = time.perf_counter()
    barrier()
    dt = t1 - t0
    dom_ms, dom_fpl = ctx.kernel_stats().get(dominant, (float("nan"), float("nan")))

    dt, value = aggregate(dist, dt, args.steps * args.frames, world, local=local)

    if rank == 0:
        abytes = algorithmic_bytes(dominant, seq.W, seq.H, info, args.max_kpts) * dom_fpl   # per launch
        achieved = abytes / (dom_ms * 1e-3) / 1e9
        traffic, tsrc = pmc_traffic(dominant, seq.W, seq.H)
        roof = {"bound": "hbm", "kernel": dominant, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": tsrc,
                "avg_launch_ms": dom_ms, "frames_per_launch": dom_fpl, "algorithmic_bytes_per_launch": abytes}
        path_bytes = algorithmic_bytes("path", seq.W, seq.H, info, args.max_kpts)
        cpu = None
        if not args.no_cpu and world == 1:
            cpu = cpu_baseline(frames, seq, args.cpu_seconds, args.max_kpts)
        ok = int((st == 0).sum())
        line = {
            "metric": METRIC, "value": value, "unit": "frames/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": dt / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8/f32/u32/f64", "data": "synthetic",
            "config": {"workload": "kitti_1241x376_2000kpts_full_path" if (seq.W, seq.H) == (1241, 376)
                       else f"{seq.W}x{seq.H}_{args.max_kpts}kpts_full_path",
                       "frames_per_step": args.frames, "width": seq.W, "height": seq.H,
                       "max_kpts": args.max_kpts, "sequence": f"scene seq=rank, {args.motion} m/frame",
                       "parallelism": f"replicas: 1 sequence per GPU x {world}",
                       "frame_batch": ctx.cfg.frame_batch or 64,
                       "mean_kpts": float(info[:, 0].mean()), "mean_matches": float(info[:, 1].mean()),
                       "mean_inliers": float(info[:, 2].mean()), "mean_hypotheses": float(info[:, 4].mean()),
                       "frames_ok": ok},
            "roofline": roof,
            "path_roofline": {"algorithmic_bytes_per_frame": path_bytes,
                              "achieved_GBs": path_bytes * value / world / 1e9,
                              "frac": path_bytes * value / world / 1e9 / HBM_PEAK_GBS},
            "kernels_ms_per_frame": {k: round(v, 5) for k, v in per_frame.items()},
            "kernels_ms_per_launch": {k: round(ks[k][0], 5) for k in KERNELS if k in ks},
            "cpu_baseline": cpu,
        }
        if args.breakdown:
            for k in KERNELS:
                if k in ks:
                    print(f"{k:14s} {per_frame[k] * 1e3:9.2f} us/frame  {ks[k][0] * 1e3:9.1f} us/launch  "
                          f"{ks[k][1]:5.1f} frames/launch", file=sys.stderr)
        print(json.dumps(line))
    dframes.free()
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
