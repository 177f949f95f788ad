#!/usr/bin/env python3
"""Host-frame streaming diagnostics on the GPU box: pinned H2D bandwidth by copy size (torch
pinned tensors, CUDA events), then vo_process_frames_host vs vo_process_frames_device on the same
sequence (frames/s, rows equal).  Environment knobs (VO_FIRST, ...) apply as usual."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402


def h2d_bandwidth():
    import torch
    out = {}
    for mb in (0.5, 3.7, 15, 30, 120):
        n = int(mb * 1e6)
        h = torch.empty(n, dtype=torch.uint8, pin_memory=True)
        d = torch.empty(n, dtype=torch.uint8, device="cuda")
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            for _ in range(3):
                d.copy_(h, non_blocking=True)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                d.copy_(h, non_blocking=True)
            e1.record()
        e1.synchronize()
        out[f"{mb}MB"] = round(n * 10 / (e0.elapsed_time(e1) * 1e-3) / 1e9, 1)
    # the same bytes split over two / four copy streams at once (several SDMA engines)
    for ns in (2, 4):
        n = int(30e6)
        h = torch.empty(n, dtype=torch.uint8, pin_memory=True)
        d = torch.empty(n, dtype=torch.uint8, device="cuda")
        ss = [torch.cuda.Stream() for _ in range(ns)]
        part = n // ns
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            for i, s in enumerate(ss):
                with torch.cuda.stream(s):
                    d[i * part:(i + 1) * part].copy_(h[i * part:(i + 1) * part], non_blocking=True)
        torch.cuda.synchronize()
        out[f"30MB_x{ns}streams"] = round(n * 10 / (time.perf_counter() - t0) / 1e9, 1)
    return out


def main():
    from acs_visual_odometry_amd import Context
    from acs_visual_odometry_amd.synth import render_sequences, SceneSequence
    frames = render_sequences([(1241, 376, 200, 0, 1.0)], workers=16)[0]
    seq = SceneSequence(nframes=200, step=1.0)
    res = {"h2d_GBs_by_size": h2d_bandwidth()}
    ctx = Context(seq.W, seq.H, K=seq.K)
    ctx.set_ground_truth(seq.gt())
    df = ctx.device_frames(frames)
    hf = ctx.host_frames(frames)

    def rate(fn, k=10):
        fn()
        t0 = time.perf_counter()
        for _ in range(k):
            fn()
        return 200 * k / (time.perf_counter() - t0)

    def dev():
        ctx.reset()
        return ctx.process_frames_device(df)

    def host():
        ctx.reset()
        return ctx.process_frames_host(hf)
    res["device_fps"] = rate(dev)
    res["host_fps"] = rate(host)
    a, b = dev(), host()
    res["rows_equal"] = bool(np.array_equal(a[0], b[0]))
    res["env"] = {k: v for k, v in os.environ.items() if k.startswith("VO_")}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
