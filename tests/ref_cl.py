"""Minimal ctypes OpenCL host (test infrastructure): runs the reference's own extract
kernels, compiled offline from their source by oracle/ref_kernels.mk into
oracle/_ref/*.co, through the ROCm OpenCL runtime (libOpenCL.so.1 -> libamdocl64.so).

Launch geometry follows the reference host code:
  gradient_convolution      offset (1,1), size (W-2, H-2)   corner_detection_parallel_GPU.cpp:69-72
  shitomasi_response        offset (2,2), size (W-4, H-4)   corner_detection_parallel_GPU.cpp:96-99
  compute_all_orientations  size (n, 903)                   FREAK_feature_descriptor_parallel_GPU.cpp:117
  merge_all_orientations    size (n)                        FREAK_feature_descriptor_parallel_GPU.cpp:139
  compute_all_descriptors   size (n, 512)                   FREAK_feature_descriptor_parallel_GPU.cpp:165
The reference does not initialise its J / O buffers (the O fill is commented out at
FREAK_feature_descriptor_parallel_GPU.cpp:91-92); here every buffer starts at zero, the
convention the oracle restates (zero border, orientation sums from 0).
"""
from __future__ import annotations

import ctypes as C
import os
import re

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_DIR = os.path.join(ROOT, "oracle", "_ref")

CL_DEVICE_TYPE_GPU = 1 << 2
CL_MEM_READ_WRITE = 1 << 0
CL_MEM_COPY_HOST_PTR = 1 << 5

P = C.c_void_p
SZ = C.c_size_t


REF_FREAK_HEADER = "/root/reference/feature_extraction_parallel_GPU/FREAK_feature_descriptor_parallel_GPU.h"


def parse_reference_freak_header(path: str = REF_FREAK_HEADER):
    """The reference header's tables, read as text: (43 points, 512 patch indices, the text of
    generate_tests) -- FREAK_feature_descriptor_parallel_GPU.h:47-56, :58-81, :87-123."""
    src = re.sub(r"//[^\n]*", "", open(path).read())
    blk = src.split("predefined_point_for_matching", 1)[1].split("}};", 1)[0]
    pts = [(int(a), int(b)) for a, b in re.findall(r"\{\s*(-?\d+)\s*,\s*(-?\d+)\s*\}", blk)]
    body = src.split("generate_tests()", 1)[1].split("return result;", 1)[0]
    pat = src.split("PATCH_DESCRIPTION_POINTS", 1)[1].split("};", 1)[0]
    patch = [int(v) for v in re.findall(r"\b(\d+)\b", pat.split("=", 1)[1])]
    return pts, patch, body


def freak_tables(source: str = "reference"):
    """(test_cases int32[903,4], patch uint64[512]): the reference header's own tables where the
    reference sources are mounted (the reference kernels then run on the reference's tables), else
    include/vo_freak_tables.h (tests/test_freak_tables.py pins the two equal)."""
    if source == "reference" and os.path.exists(REF_FREAK_HEADER):
        pts, patch, _ = parse_reference_freak_header(REF_FREAK_HEADER)
        tc = [(pts[i][0], pts[i][1], pts[j][0], pts[j][1]) for i in range(43) for j in range(i + 1, 43)]
        return np.array(tc, np.int32), np.array(patch, np.uint64)
    src = open(os.path.join(ROOT, "include", "vo_freak_tables.h")).read()
    pts_blk = src.split("#define VO_FREAK_POINTS_LIST")[1].split("#define")[0]
    pts = [(int(a), int(b)) for a, b in re.findall(r"\{\s*(-?\d+),\s*(-?\d+)\s*\}", pts_blk)]
    assert len(pts) == 43
    pat_blk = src.split("#define VO_FREAK_PATCH_LIST")[1].split("static const")[0]
    patch = [int(v) for v in re.findall(r"\b(\d+)\b", pat_blk)]
    assert len(patch) == 512
    tc = [(pts[i][0], pts[i][1], pts[j][0], pts[j][1]) for i in range(43) for j in range(i + 1, 43)]
    return np.array(tc, np.int32), np.array(patch, np.uint64)


class CLError(RuntimeError):
    pass


class RefKernels:
    """One OpenCL context/queue on GPU 0 with the reference program loaded from a binary."""

    def __init__(self, variant: str = "strict"):
        self.name = variant
        path = os.path.join(REF_DIR, f"fe_kernels_{variant}.co")
        if not os.path.exists(path):
            raise FileNotFoundError(path)
        self.cl = cl = C.CDLL("libOpenCL.so.1")
        for name, res in [("clCreateContext", P), ("clCreateCommandQueue", P), ("clCreateProgramWithBinary", P),
                          ("clCreateKernel", P), ("clCreateBuffer", P)]:
            getattr(cl, name).restype = res
        err = C.c_int()
        nplat = C.c_uint()
        self._ok(cl.clGetPlatformIDs(0, None, C.byref(nplat)), "clGetPlatformIDs")
        plats = (P * nplat.value)()
        self._ok(cl.clGetPlatformIDs(nplat.value, plats, None), "clGetPlatformIDs")
        dev = P()
        for p in plats:
            if cl.clGetDeviceIDs(P(p), C.c_uint64(CL_DEVICE_TYPE_GPU), 1, C.byref(dev), None) == 0:
                break
        else:
            raise CLError("no OpenCL GPU device")
        self.dev = dev
        self.ctx = P(cl.clCreateContext(None, 1, C.byref(dev), None, None, C.byref(err)))
        self._ok(err.value, "clCreateContext")
        cl.clCreateCommandQueue.argtypes = [P, P, C.c_uint64, C.POINTER(C.c_int)]
        self.q = P(cl.clCreateCommandQueue(self.ctx, dev, 0, C.byref(err)))
        self._ok(err.value, "clCreateCommandQueue")
        blob = open(path, "rb").read()
        buf = C.create_string_buffer(blob, len(blob))
        lens = (SZ * 1)(len(blob))
        bins = (P * 1)(C.cast(buf, P))
        status = C.c_int()
        cl.clCreateProgramWithBinary.argtypes = [P, C.c_uint, C.POINTER(P), C.POINTER(SZ), C.POINTER(P),
                                                 C.POINTER(C.c_int), C.POINTER(C.c_int)]
        self.prog = P(cl.clCreateProgramWithBinary(self.ctx, 1, C.byref(dev), lens, bins, C.byref(status),
                                                   C.byref(err)))
        self._ok(err.value, "clCreateProgramWithBinary")
        cl.clBuildProgram.argtypes = [P, C.c_uint, C.POINTER(P), C.c_char_p, P, P]
        self._ok(cl.clBuildProgram(self.prog, 1, C.byref(dev), b"", None, None), "clBuildProgram")
        cl.clCreateKernel.argtypes = [P, C.c_char_p, C.POINTER(C.c_int)]
        cl.clCreateBuffer.argtypes = [P, C.c_uint64, SZ, P, C.POINTER(C.c_int)]
        cl.clSetKernelArg.argtypes = [P, C.c_uint, SZ, P]
        cl.clEnqueueNDRangeKernel.argtypes = [P, P, C.c_uint, C.POINTER(SZ), C.POINTER(SZ), C.POINTER(SZ),
                                              C.c_uint, P, P]
        cl.clEnqueueReadBuffer.argtypes = [P, P, C.c_uint, SZ, SZ, P, C.c_uint, P, P]
        cl.clReleaseMemObject.argtypes = [P]
        cl.clReleaseKernel.argtypes = [P]
        cl.clFinish.argtypes = [P]
        self.kernels = {}
        self._bufs = []

    @staticmethod
    def _ok(rc, what):
        if rc != 0:
            raise CLError(f"{what} failed: {rc}")

    def kernel(self, name):
        if name not in self.kernels:
            err = C.c_int()
            k = P(self.cl.clCreateKernel(self.prog, name.encode(), C.byref(err)))
            self._ok(err.value, f"clCreateKernel({name})")
            self.kernels[name] = k
        return self.kernels[name]

    def buffer(self, arr: np.ndarray):
        arr = np.ascontiguousarray(arr)
        err = C.c_int()
        m = P(self.cl.clCreateBuffer(self.ctx, CL_MEM_READ_WRITE | CL_MEM_COPY_HOST_PTR, arr.nbytes,
                                     arr.ctypes.data_as(P), C.byref(err)))
        self._ok(err.value, "clCreateBuffer")
        self._bufs.append(m)
        return m

    def read(self, m, like: np.ndarray) -> np.ndarray:
        out = np.empty_like(like)
        self._ok(self.cl.clEnqueueReadBuffer(self.q, m, 1, 0, out.nbytes, out.ctypes.data_as(P), 0, None, None),
                 "clEnqueueReadBuffer")
        return out

    def run(self, name, args, gsize, offset=None):
        k = self.kernel(name)
        for i, a in enumerate(args):
            if isinstance(a, P):
                v = P(a.value)
                self._ok(self.cl.clSetKernelArg(k, i, C.sizeof(P), C.byref(v)), f"arg {i}")
            elif isinstance(a, np.generic):
                v = np.array(a)
                self._ok(self.cl.clSetKernelArg(k, i, v.nbytes, v.ctypes.data_as(P)), f"arg {i}")
            else:
                raise TypeError(type(a))
        dims = len(gsize)
        gs = (SZ * dims)(*gsize)
        off = (SZ * dims)(*offset) if offset is not None else None
        self._ok(self.cl.clEnqueueNDRangeKernel(self.q, k, dims, off, gs, None, 0, None, None), name)
        self._ok(self.cl.clFinish(self.q), "clFinish")

    def release(self):
        for m in self._bufs:
            self.cl.clReleaseMemObject(m)
        self._bufs = []

    # ---- the reference's extract stages ----
    def response(self, blurred: np.ndarray, thr: float = 20000.0):
        H, W = blurred.shape
        z = np.zeros((H, W), np.float32)
        img = self.buffer(blurred.astype(np.uint8))
        jx, jy, jxy, r = self.buffer(z), self.buffer(z), self.buffer(z), self.buffer(z)
        self.run("gradient_convolution", [img, jx, jy, jxy, np.int32(W)], (W - 2, H - 2), (1, 1))
        self.run("shitomasi_response", [r, jx, jy, jxy, np.int32(W), np.float32(thr)], (W - 4, H - 4), (2, 2))
        out = [self.read(m, z) for m in (jx, jy, jxy, r)]
        self.release()
        return out

    def orient_describe(self, blurred: np.ndarray, kps: np.ndarray, rot_in: np.ndarray | None = None):
        """Orientation sums, rotation matrices and the 512 descriptor bytes for kps (n x 2,
        x=col, y=row).  rot_in: feed these rotations to the descriptor kernel instead of the
        ones merge_all_orientations produced (isolates the descriptor arithmetic)."""
        H, W = blurred.shape
        n = kps.shape[0]
        tc, patch = freak_tables()
        img = self.buffer(blurred.astype(np.uint8))
        tcb = self.buffer(tc)
        pb = self.buffer(patch)
        kb = self.buffer(np.ascontiguousarray(kps, np.int32))
        zf = np.zeros(n, np.float32)
        ox, oy = self.buffer(zf), self.buffer(zf)
        rz = np.zeros((n, 4), np.float32)
        rot = self.buffer(rz)
        self.run("compute_all_orientations", [img, tcb, ox, oy, kb, np.int32(W)], (n, 903))
        self.run("merge_all_orientations", [ox, oy, rot], (n,))
        rot_cl = self.read(rot, rz)
        rot_use = self.buffer(np.ascontiguousarray(rot_in, np.float32)) if rot_in is not None else rot
        dz = np.zeros((n, 512), np.uint8)
        desc = self.buffer(dz)
        self.run("compute_all_descriptors", [desc, img, pb, kb, rot_use, tcb, np.int32(W)], (n, 512))
        out = (self.read(ox, zf), self.read(oy, zf), rot_cl, self.read(desc, dz))
        self.release()
        return out
