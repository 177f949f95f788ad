"""Host-side mirror of the reference's per-frame interface, over the C ABI.

``Context`` wraps one ``vo_ctx`` (one GPU, one HIP stream, persistent HBM buffers).
``VisualOdometry`` mirrors the reference class (VisualOdometry.h:15-31): same method
names, same argument meaning, same error behaviour (``RuntimeError`` where the
reference throws ``std::runtime_error``).
"""
from __future__ import annotations

import ctypes as C
import math
import os
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _lib
from ._lib import check, load


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


class Context:
    """One vo_ctx: HIP device buffers + stream for a width x height stream."""

    def __init__(self, width: int, height: int, **cfg):
        self.lib = load()
        self.cfg = _lib.default_config(width, height, **cfg)
        h = C.c_void_p()
        check(self.lib.vo_create(C.byref(self.cfg), C.byref(h)), "vo_create")
        self.h = h
        self.W, self.H, self.N = width, height, self.cfg.max_kpts

    def close(self):
        if getattr(self, "h", None):
            self.lib.vo_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # -- stage calls --------------------------------------------------------
    def extract(self, gray: np.ndarray, want_blurred: bool = False):
        g = np.ascontiguousarray(gray, dtype=np.uint8)
        assert g.shape == (self.H, self.W), g.shape
        kps = np.empty((self.N, 2), np.int32)
        desc = np.empty((self.N, 8), np.uint64)
        bl = np.empty_like(g) if want_blurred else None
        n = C.c_int()
        check(self.lib.vo_extract(self.h, _p(g), self.W, _p(kps), _p(desc), C.byref(n), _p(bl)), "vo_extract")
        out = (kps[:n.value].copy(), desc[:n.value].copy())
        return out + (bl,) if want_blurred else out

    def response(self, gray: np.ndarray) -> np.ndarray:
        g = np.ascontiguousarray(gray, dtype=np.uint8)
        R = np.empty((self.H, self.W), np.float32)
        check(self.lib.vo_response(self.h, _p(g), self.W, _p(R)), "vo_response")
        return R

    def match(self, d_prev: np.ndarray, d_cur: np.ndarray) -> np.ndarray:
        a = np.ascontiguousarray(d_prev, dtype=np.uint64).reshape(-1, 8)
        b = np.ascontiguousarray(d_cur, dtype=np.uint64).reshape(-1, 8)
        out = np.empty((max(a.shape[0], 1), 2), np.int32)
        m = C.c_int()
        check(self.lib.vo_match(self.h, _p(a), a.shape[0], _p(b), b.shape[0], _p(out), C.byref(m)), "vo_match")
        return out[:m.value].copy()

    def ransac(self, pts: np.ndarray, seed: int):
        pts = np.ascontiguousarray(pts, dtype=np.float64).reshape(-1, 4)
        m = pts.shape[0]
        F = np.zeros(9)
        inl = np.zeros(max(m, 1), np.int32)
        counts = np.zeros(2000, np.int32)
        fitted, n_inl, best_k, n_eval = C.c_int(), C.c_int(), C.c_int(), C.c_int()
        check(self.lib.vo_ransac_F(self.h, _p(pts), m, seed, _p(F), C.byref(fitted), _p(inl), C.byref(n_inl),
                                   C.byref(best_k), C.byref(n_eval), _p(counts)), "vo_ransac_F")
        ne = n_eval.value
        return dict(F=F.reshape(3, 3), fitted=fitted.value, n_inl=n_inl.value, best_k=best_k.value,
                    n_evaluated=ne, counts=counts[:min(ne, 2000)].copy(),
                    inliers=inl[:n_inl.value].copy() if best_k.value >= 0 else np.zeros(0, np.int32))

    def ransac_run(self, pts: np.ndarray, probability: float = 0.99, sampson_thr: float = 1.0,
                   num_threads: int = 8, seed: int = 0):
        """Ransac::run with the call's own parameters (vo_ransac_run): F is None when the model was
        not refit (fewer than 8 inliers: the caller's previous model stays, quirk 9)."""
        pts = np.ascontiguousarray(pts, dtype=np.float64).reshape(-1, 4)
        m = pts.shape[0]
        F = np.zeros(9)
        inl = np.zeros(max(m, 1), np.int32)
        fitted, n_inl, n_eval = C.c_int(), C.c_int(), C.c_int()
        check(self.lib.vo_ransac_run(self.h, _p(pts), m, probability, sampson_thr, num_threads, seed, _p(F),
                                     C.byref(fitted), _p(inl), C.byref(n_inl), C.byref(n_eval)), "vo_ransac_run")
        return dict(F=F.reshape(3, 3) if fitted.value else None, fitted=fitted.value, n_inl=n_inl.value,
                    n_evaluated=n_eval.value, inliers=inl[:n_inl.value].copy())

    def fit_F(self, pts: np.ndarray) -> np.ndarray:
        """FundamentalMatrix::fit / computeFundamentalMatrix on all n >= 8 correspondences (vo_fit_F)."""
        pts = np.ascontiguousarray(pts, dtype=np.float64).reshape(-1, 4)
        F = np.zeros(9)
        check(self.lib.vo_fit_F(self.h, _p(pts), pts.shape[0], _p(F)), "vo_fit_F")
        return F.reshape(3, 3)

    def pose(self, F, p1, p2, scale: float = 1.0):
        F = np.ascontiguousarray(F, dtype=np.float64).reshape(9)
        p1 = np.ascontiguousarray(p1, dtype=np.float32).reshape(-1, 2)
        p2 = np.ascontiguousarray(p2, dtype=np.float32).reshape(-1, 2)
        R = np.zeros(9)
        t = np.zeros(3)
        cnt = np.zeros(4, np.int32)
        rc = self.lib.vo_pose(self.h, _p(F), _p(p1), _p(p2), p1.shape[0], scale, _p(R), _p(t), _p(cnt))
        check(rc, "vo_pose")
        return R.reshape(3, 3), t, cnt

    # -- trajectory ---------------------------------------------------------
    def set_ground_truth(self, gt: Optional[np.ndarray]):
        if gt is None:
            check(self.lib.vo_set_ground_truth(self.h, None, 0))
            return
        g = np.ascontiguousarray(gt, dtype=np.float64).reshape(-1, 12)
        check(self.lib.vo_set_ground_truth(self.h, _p(g), g.shape[0]), "vo_set_ground_truth")

    def set_sequence_starts(self, starts):
        """Frames (since reset) that begin a new independent sequence (vo_set_sequence_starts)."""
        a = np.ascontiguousarray(np.asarray(starts, dtype=np.int32).reshape(-1))
        check(self.lib.vo_set_sequence_starts(self.h, _p(a) if a.size else None, a.size), "vo_set_sequence_starts")

    def set_frame_origin(self, origin: int):
        """The stream's first frame is frame `origin` of its sequence (a sequence shard,
        vo_set_frame_origin): RANSAC draws the hypotheses of the unsplit run."""
        check(self.lib.vo_set_frame_origin(self.h, int(origin)), "vo_set_frame_origin")

    def trajectory_state(self) -> np.ndarray:
        """T_curr after the last committed frame (4x4)."""
        T = np.zeros(16)
        check(self.lib.vo_trajectory_state(self.h, _p(T)), "vo_trajectory_state")
        return T.reshape(4, 4)

    def rechain(self, T_in: np.ndarray, f0: int, n: int) -> np.ndarray:
        """Rows of committed frames [f0, f0 + n) chained from T_curr = T_in (vo_rechain)."""
        T = np.ascontiguousarray(T_in, dtype=np.float64).reshape(16)
        poses = np.zeros((max(n, 0), 12))
        check(self.lib.vo_rechain(self.h, _p(T), int(f0), int(n), _p(poses)), "vo_rechain")
        return poses.reshape(-1, 3, 4)

    def reset(self):
        check(self.lib.vo_reset(self.h), "vo_reset")

    def device_errors(self) -> int:
        """Frames that failed the select's consistency check since creation / the last reset
        (vo_device_error_count; VO_STATUS_INCONSISTENT).  Expected 0."""
        n = C.c_uint32()
        check(self.lib.vo_device_error_count(self.h, C.byref(n)), "vo_device_error_count")
        return n.value

    def ring_slots(self) -> int:
        """Frames whose keypoints, descriptors and trajectory records stay resident (vo_ring_slots)."""
        return check(self.lib.vo_ring_slots(self.h), "vo_ring_slots")

    def process_frame(self, gray: Optional[np.ndarray]):
        pose = np.zeros(12)
        st = C.c_int()
        info = np.zeros(8, np.int32)
        g = None if gray is None else np.ascontiguousarray(gray, dtype=np.uint8)
        rc = self.lib.vo_process_frame(self.h, _p(g), 0 if g is None else self.W, _p(pose), C.byref(st), _p(info))
        if rc < 0 and rc != _lib.VO_ERR_DEGENERATE_E:
            check(rc, "vo_process_frame")
        return pose.reshape(3, 4), st.value, info

    def device_frames(self, frames: np.ndarray) -> "DeviceFrames":
        return DeviceFrames(self, frames)

    def process_frames_device(self, dframes: "DeviceFrames", timing: int = 0):
        """timing: 0 off, 1 every kernel, 100+k only kernel k (see kernel_times())."""
        n = dframes.n
        poses = np.zeros((n, 12))
        st = np.zeros(n, np.int32)
        info = np.zeros((n, 8), np.int32)
        check(self.lib.vo_enable_kernel_timing(self.h, int(timing)))
        check(self.lib.vo_process_frames_device(self.h, dframes.ptr, dframes.frame_bytes, n, _p(poses), _p(st),
                                                _p(info)), "vo_process_frames_device")
        return poses.reshape(n, 3, 4), st, info

    def extract_frames_device(self, dframes: "DeviceFrames", timing: int = 0, outputs: bool = False):
        """Batched extract only (vo_extract_frames_device).  outputs=True returns the keypoints
        and descriptors of every frame (lists of arrays); otherwise only the counts.  Resets the
        trajectory state."""
        n = dframes.n
        nk = np.zeros(n, np.int32)
        kps = np.zeros((n, self.N, 2), np.int32) if outputs else None
        desc = np.zeros((n, self.N, 8), np.uint64) if outputs else None
        check(self.lib.vo_enable_kernel_timing(self.h, int(timing)))
        check(self.lib.vo_extract_frames_device(self.h, dframes.ptr, dframes.frame_bytes, n, _p(kps), _p(desc), _p(nk)),
              "vo_extract_frames_device")
        if not outputs:
            return nk
        return nk, [kps[f, :nk[f]] for f in range(n)], [desc[f, :nk[f]] for f in range(n)]

    def process_frames_host(self, frames, timing: int = 0):
        """Host-frame streaming (vo_process_frames_host): frames is an (n, H, W) u8 array in host
        memory -- a HostFrames buffer (pinned) or any numpy array (pageable: registered for the
        call).  Batch k+1's H2D copy overlaps the extract/pose work of earlier batches."""
        arr = frames.array if isinstance(frames, HostFrames) else np.ascontiguousarray(frames, dtype=np.uint8)
        assert arr.ndim == 3 and arr.shape[1:] == (self.H, self.W)
        n = arr.shape[0]
        poses = np.zeros((n, 12))
        st = np.zeros(n, np.int32)
        info = np.zeros((n, 8), np.int32)
        check(self.lib.vo_enable_kernel_timing(self.h, int(timing)))
        check(self.lib.vo_process_frames_host(self.h, _p(arr), self.W * self.H, n, _p(poses), _p(st), _p(info)),
              "vo_process_frames_host")
        return poses.reshape(n, 3, 4), st, info

    def host_frames(self, frames: np.ndarray) -> "HostFrames":
        return HostFrames(self, frames)

    def kernel_times(self):
        """Average ms per timed launch of each kernel in the last process_frames_device call."""
        return {k: v[0] for k, v in self.kernel_stats().items()}

    def kernel_stats(self):
        """{kernel: (ms per timed launch, frames per launch)} of the last process_frames_device call."""
        names = (C.c_char_p * 32)()
        ms = (C.c_float * 32)()
        fpl = (C.c_float * 32)()
        k = self.lib.vo_last_kernel_stats(self.h, names, ms, fpl, 32)
        return {names[i].decode(): (ms[i], fpl[i]) for i in range(k) if ms[i] >= 0}

    def kernel_forms(self):
        """{stage: [kernel symbols]} the batched path of this context launches (vo_kernel_form):
        which rows of a rocprofv3 summary belong to each stage."""
        stages = ["stencil", "select", "describe", "match", "ransac", "refit", "triangulate", "finalize", "trajectory"]
        return {k: self.lib.vo_kernel_form(self.h, i).decode().split(",") for i, k in enumerate(stages)}


class DeviceFrames:
    """A batch of frames resident in HBM (uploaded once)."""

    def __init__(self, ctx: Context, frames: np.ndarray):
        f = np.ascontiguousarray(frames, dtype=np.uint8)
        assert f.ndim == 3 and f.shape[1:] == (ctx.H, ctx.W)
        self.ctx, self.n = ctx, f.shape[0]
        self.frame_bytes = ctx.W * ctx.H
        p = C.c_void_p()
        check(ctx.lib.vo_device_alloc(ctx.h, f.nbytes, C.byref(p)), "vo_device_alloc")
        self.ptr = p
        check(ctx.lib.vo_device_upload(ctx.h, p, _p(f), f.nbytes), "vo_device_upload")

    def view(self, f0: int, f1: int) -> "DeviceFrameView":
        """Frames [f0, f1) of the batch, without a copy."""
        assert 0 <= f0 <= f1 <= self.n
        return DeviceFrameView(C.c_void_p(self.ptr.value + f0 * self.frame_bytes), f1 - f0, self.frame_bytes)

    def free(self):
        if self.ptr:
            self.ctx.lib.vo_device_free(self.ctx.h, self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class DeviceFrameView:
    """Frames of a DeviceFrames batch (process_frames_device accepts either)."""

    def __init__(self, ptr, n: int, frame_bytes: int):
        self.ptr, self.n, self.frame_bytes = ptr, n, frame_bytes

    def free(self):
        pass


class HostFrames:
    """A batch of frames in pinned host memory (vo_host_alloc): the DMA source of
    process_frames_host.  ``array`` is an (n, H, W) u8 numpy view of the pinned buffer."""

    def __init__(self, ctx: Context, frames: np.ndarray):
        f = np.ascontiguousarray(frames, dtype=np.uint8)
        assert f.ndim == 3 and f.shape[1:] == (ctx.H, ctx.W)
        self.ctx, self.n = ctx, f.shape[0]
        p = C.c_void_p()
        check(ctx.lib.vo_host_alloc(ctx.h, f.nbytes, C.byref(p)), "vo_host_alloc")
        self.ptr = p
        buf = (C.c_uint8 * f.nbytes).from_address(p.value)
        self.array = np.frombuffer(buf, np.uint8).reshape(f.shape)
        self.array[...] = f

    def free(self):
        if self.ptr:
            self.array = None
            self.ctx.lib.vo_host_free(self.ctx.h, self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def unpack_descriptor(words: np.ndarray) -> np.ndarray:
    """8 x u64 words -> 512 bytes in {0,1} (the reference's byte-per-test descriptor)."""
    w = np.ascontiguousarray(words, dtype=np.uint64).reshape(-1, 8)
    bits = np.unpackbits(w.view(np.uint8).reshape(-1, 64), axis=1, bitorder="little")
    return bits.astype(np.uint8)


def pack_descriptor(bytes512: np.ndarray) -> np.ndarray:
    b = np.ascontiguousarray(bytes512, dtype=np.uint8).reshape(-1, 512)
    return np.packbits(b, axis=1, bitorder="little").view(np.uint64).reshape(-1, 8)


class VisualOdometry:
    """Mirror of the reference class VisualOdometry (VisualOdometry.h:15-31).

    ``kernel_filename`` is accepted for signature compatibility (the reference loads an
    OpenCL binary, main_pipeline.cpp:32); the HIP code objects are embedded in
    libvo_mi355x.so.  ``num_threads`` keeps its one semantic effect on the results:
    the RANSAC chunk count (ransac.cpp:152-157).
    """

    def __init__(self, kernel_filename: str = "", num_threads: int = 8, width: int = 1241, height: int = 376,
                 **cfg):
        self.kernel_filename = kernel_filename
        self.number_of_threads = int(num_threads)
        cfg.setdefault("ransac_chunk_threads", max(self.number_of_threads, 1))
        self._cfg = cfg
        self.ctx = Context(width, height, **cfg)

    def compute_descriptor_with_key_points(self, image: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
        """-> (descriptors n x 512 u8 in {0,1}, keypoints n x 2 (x=col, y=row)), raster order."""
        kps, desc = self.ctx.extract(image)
        return unpack_descriptor(desc), kps

    def match_descriptors(self, desc1, desc2) -> List[Tuple[int, int]]:
        d1 = np.asarray(desc1)
        d2 = np.asarray(desc2)
        if d1.size == 0 or d2.size == 0:
            return []
        w1 = pack_descriptor(d1) if d1.shape[-1] == 512 else d1
        w2 = pack_descriptor(d2) if d2.shape[-1] == 512 else d2
        return [tuple(map(int, r)) for r in self.ctx.match(w1, w2)]

    RUN_BATCH = 256   # frames decoded and streamed per host batch

    def run(self, image_dir: str, num_images: int, pose_file: str, output_csv: str) -> None:
        """VisualOdometry::run (VisualOdometry.cpp:38-193): image_dir + "%06d.png" for frames
        0 .. num_images-1 (frame 0 always, as the reference reads it before its loop), GT from
        pose_file (one readGTLine per line), pose rows to output_csv.  Present frames go to the
        GPU in batches through process_frames_host; a missing image is one process_frame(None)
        (VisualOdometry.cpp:77-82).  The context takes frame 0's size."""
        import sys
        from .io import read_gray, read_kitti_poses, write_pose_csv
        try:
            gt = read_kitti_poses(pose_file)
        except OSError:
            print("Failed to open pose file.", file=sys.stderr)
            return
        total = max(int(num_images), 1)

        def path(i):
            return image_dir + f"{i:06d}.png"

        img0 = read_gray(path(0))
        if img0 is not None and img0.shape != (self.ctx.H, self.ctx.W):
            self.ctx.close()
            self.ctx = Context(img0.shape[1], img0.shape[0], **self._cfg)
        self.ctx.reset()
        self.ctx.set_ground_truth(gt)
        rows = []
        for i0 in range(0, total, self.RUN_BATCH):
            imgs = [read_gray(path(i)) for i in range(i0, min(total, i0 + self.RUN_BATCH))]
            z = 0
            while z < len(imgs):
                if imgs[z] is None:
                    if i0 + z > 0:
                        print(f"Failed to load image: {path(i0 + z)}", file=sys.stderr)
                    pose, _, _ = self.ctx.process_frame(None)
                    rows.append(pose)
                    z += 1
                    continue
                e = z
                while e < len(imgs) and imgs[e] is not None:
                    if imgs[e].shape != (self.ctx.H, self.ctx.W):
                        raise RuntimeError(f"image size differs from frame 0: {path(i0 + e)}")
                    e += 1
                poses, st, _ = self.ctx.process_frames_host(np.stack(imgs[z:e]))
                for k in np.flatnonzero(st == 3):          # VisualOdometry.cpp:108-109
                    print(f"Too few matches at frame {i0 + z + int(k)}", file=sys.stderr)
                if (st == 5).any():
                    raise RuntimeError("Degenerate essential matrix")
                rows.extend(poses)
                z = e
        write_pose_csv(output_csv, rows)
        print(f"Wrote estimated poses to: {output_csv}")
