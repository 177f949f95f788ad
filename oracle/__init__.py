"""ctypes binding of the CPU oracle (oracle/build/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg.  The product package (acs_visual_odometry_amd) never imports it.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# VO_ORACLE_LIB: another build of the same sources (tests/test_sanitizers.py: the ASan/UBSan build)
_LIB = os.environ.get("VO_ORACLE_LIB") or os.path.join(_HERE, "build", "liboracle.so")
_lib = None


class VooConfig(C.Structure):
    _fields_ = [
        ("width", C.c_int), ("height", C.c_int), ("max_kpts", C.c_int), ("nms_k", C.c_int),
        ("resp_thr", C.c_float), ("border_row", C.c_int), ("border_col", C.c_int),
        ("ratio", C.c_float), ("match_bits", C.c_int), ("ransac_p", C.c_double),
        ("sampson_thr", C.c_double), ("ransac_chunk_threads", C.c_int), ("seed", C.c_uint64),
        ("K", C.c_double * 9), ("rng_mode", C.c_int),
    ]


class VooRansacResult(C.Structure):
    _fields_ = [("F", C.c_double * 9), ("fitted", C.c_int), ("best_k", C.c_int),
                ("best_count", C.c_int), ("n_evaluated", C.c_int), ("n_inl", C.c_int)]


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            build()
        L = C.CDLL(_LIB)
        P = C.c_void_p
        L.voo_det_atan2.restype = C.c_double
        L.voo_det_atan2.argtypes = [C.c_double, C.c_double]
        L.voo_det_sin.restype = C.c_double
        L.voo_det_sin.argtypes = [C.c_double]
        L.voo_det_cos.restype = C.c_double
        L.voo_det_cos.argtypes = [C.c_double]
        L.voo_mix64.restype = C.c_uint64
        L.voo_mix64.argtypes = [C.c_uint64]
        L.voo_frame_seed.restype = C.c_uint64
        L.voo_frame_seed.argtypes = [C.c_uint64, C.c_int64]
        L.voo_sample8.argtypes = [C.c_uint64, C.c_int, C.c_int, P]
        L.voo_ransac_maxit_update.argtypes = [C.c_int, C.c_int, C.c_double]
        L.voo_ransac_maxit_initial.argtypes = [C.c_double]
        L.voo_config_default.argtypes = [C.POINTER(VooConfig), C.c_int, C.c_int]
        L.voo_blur7.argtypes = [P, C.c_size_t, C.c_int, C.c_int, P]
        L.voo_gradients.argtypes = [P, C.c_int, C.c_int, P, P, P]
        L.voo_response.argtypes = [P, C.c_int, C.c_int, C.c_float, P]
        L.voo_nms_topn.argtypes = [P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, P]
        L.voo_nms_candidates.argtypes = [P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int]
        L.voo_orientation.argtypes = [P, C.c_int, C.c_int, C.c_int, P, P]
        L.voo_describe.argtypes = [P, C.c_int, C.c_int, P, C.c_int, P, P]
        L.voo_extract.argtypes = [C.POINTER(VooConfig), P, C.c_size_t, P, P, P]
        L.voo_match.argtypes = [P, C.c_int, P, C.c_int, C.c_int, C.c_float, P]
        L.voo_fit_F.argtypes = [P, P, C.c_int, P]
        L.voo_fit_F8.argtypes = [P, P, P]
        L.voo_ls_nullvec9.argtypes = [P, P, P]
        L.voo_refit_normal.argtypes = [P, P, C.c_int, P]
        L.voo_sampson.restype = C.c_double
        L.voo_sampson.argtypes = [P, P]
        L.voo_ransac.argtypes = [P, C.c_int, C.c_double, C.c_double, C.c_int, C.c_uint64, P, P,
                                 C.POINTER(VooRansacResult)]
        L.voo_ransac_ex.argtypes = [P, C.c_int, C.c_double, C.c_double, C.c_int, C.c_uint64, C.c_int, P, P, P]
        L.voo_mt_samples.argtypes = [C.c_uint32, C.c_int, C.c_int, P]
        L.voo_mt_samples.restype = None
        L.voo_pose.argtypes = [P, P, P, P, C.c_int, C.c_double, P, P, P]
        L.voo_vo_create.restype = P
        L.voo_vo_create.argtypes = [C.POINTER(VooConfig)]
        L.voo_vo_destroy.argtypes = [P]
        L.voo_stage_reset.argtypes = []
        L.voo_stage_reset.restype = None
        L.voo_stage_times.argtypes = [P, P]
        L.voo_stage_times.restype = None
        L.voo_vo_process.argtypes = [P, P, C.c_size_t, P, C.c_int, P, P, P]
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(C.c_void_p) if a is not None else None


def config(width, height, **kw):
    c = VooConfig()
    lib().voo_config_default(C.byref(c), width, height)
    for k, v in kw.items():
        if k == "K":
            for i in range(9):
                c.K[i] = float(v[i])
        else:
            setattr(c, k, v)
    return c


def blur7(img):
    img = np.ascontiguousarray(img, dtype=np.uint8)
    H, W = img.shape
    out = np.empty_like(img)
    lib().voo_blur7(_p(img), W, W, H, _p(out))
    return out


def response(blurred, thr=20000.0):
    b = np.ascontiguousarray(blurred, dtype=np.uint8)
    H, W = b.shape
    R = np.empty((H, W), np.float32)
    lib().voo_response(_p(b), W, H, thr, _p(R))
    return R


def gradients(blurred):
    b = np.ascontiguousarray(blurred, dtype=np.uint8)
    H, W = b.shape
    J = [np.empty((H, W), np.float32) for _ in range(3)]
    lib().voo_gradients(_p(b), W, H, _p(J[0]), _p(J[1]), _p(J[2]))
    return J


def nms_topn(R, k=3, N=2000, brow=35, bcol=37):
    R = np.ascontiguousarray(R, dtype=np.float32)
    H, W = R.shape
    kps = np.empty((N, 2), np.int32)
    n = lib().voo_nms_topn(_p(R), W, H, k, N, brow, bcol, _p(kps))
    return kps[:n].copy()


def nms_candidates(R, k=3, brow=35, bcol=37):
    R = np.ascontiguousarray(R, dtype=np.float32)
    H, W = R.shape
    return lib().voo_nms_candidates(_p(R), W, H, k, brow, bcol)


def describe(blurred, kps, with_rot=False):
    b = np.ascontiguousarray(blurred, dtype=np.uint8)
    H, W = b.shape
    kps = np.ascontiguousarray(kps, dtype=np.int32).reshape(-1, 2)
    n = kps.shape[0]
    desc = np.zeros((max(n, 1), 8), np.uint64)
    rot = np.zeros((max(n, 1), 4), np.float32)
    lib().voo_describe(_p(b), W, H, _p(kps), n, _p(desc), _p(rot))
    if with_rot:
        return desc[:n], rot[:n]
    return desc[:n]


def orientation(blurred, kx, ky):
    b = np.ascontiguousarray(blurred, dtype=np.uint8)
    ox = C.c_float()
    oy = C.c_float()
    lib().voo_orientation(_p(b), b.shape[1], kx, ky, C.byref(ox), C.byref(oy))
    return ox.value, oy.value


def extract(gray, cfg=None):
    g = np.ascontiguousarray(gray, dtype=np.uint8)
    H, W = g.shape
    cfg = cfg or config(W, H)
    N = cfg.max_kpts
    kps = np.empty((N, 2), np.int32)
    desc = np.zeros((N, 8), np.uint64)
    bl = np.empty_like(g)
    n = lib().voo_extract(C.byref(cfg), _p(g), W, _p(kps), _p(desc), _p(bl))
    return kps[:n].copy(), desc[:n].copy(), bl


def match(d1, d2, match_bits=32, ratio=0.75):
    d1 = np.ascontiguousarray(d1, dtype=np.uint64).reshape(-1, 8)
    d2 = np.ascontiguousarray(d2, dtype=np.uint64).reshape(-1, 8)
    out = np.empty((max(d1.shape[0], 1), 2), np.int32)
    m = lib().voo_match(_p(d1), d1.shape[0], _p(d2), d2.shape[0], match_bits, ratio, _p(out))
    return out[:m].copy()


def sample8(seed, k, m):
    out = np.empty(8, np.int32)
    lib().voo_sample8(seed, k, m, _p(out))
    return out


def fit_F8(pts, idx):
    pts = np.ascontiguousarray(pts, dtype=np.float64)
    idx = np.ascontiguousarray(idx, dtype=np.int32)
    F = np.empty(9)
    lib().voo_fit_F8(_p(pts), _p(idx), _p(F))
    return F.reshape(3, 3)


def fit_F(pts, idx):
    pts = np.ascontiguousarray(pts, dtype=np.float64)
    idx = np.ascontiguousarray(idx, dtype=np.int32)
    F = np.empty(9)
    rc = lib().voo_fit_F(_p(pts), _p(idx), len(idx), _p(F))
    assert rc == 0
    return F.reshape(3, 3)


def ls_nullvec9(S, x0):
    """The refit's null-vector solver on a 9x9 PSD S (oracle ls_nullvec9): (f, status), status 0
    converged, 1 certified in the null space after the 32-step cap, 2 cyclic-Jacobi fallback."""
    S = np.ascontiguousarray(S, dtype=np.float64).reshape(81)
    x0 = np.ascontiguousarray(x0, dtype=np.float64).reshape(9)
    f = np.empty(9)
    st = lib().voo_ls_nullvec9(_p(S), _p(x0), _p(f))
    return f, st


def refit_normal(pts):
    """The refit's normal matrix A^T A over all rows of pts (n x 4), in the refit's sum order."""
    pts = np.ascontiguousarray(pts, dtype=np.float64).reshape(-1, 4)
    idx = np.arange(pts.shape[0], dtype=np.int32)
    S = np.empty(81)
    assert lib().voo_refit_normal(_p(pts), _p(idx), pts.shape[0], _p(S)) == 0
    return S.reshape(9, 9)


def sampson(F, p):
    F = np.ascontiguousarray(F, dtype=np.float64).reshape(9)
    p = np.ascontiguousarray(p, dtype=np.float64).reshape(4)
    return lib().voo_sampson(_p(F), _p(p))


def ransac(pts, prob=0.99, thr=1.0, T=8, seed=1, rng_mode=0):
    """rng_mode 1: the reference's sampler (std::mt19937(low 32 bits of seed) + std::sample)."""
    pts = np.ascontiguousarray(pts, dtype=np.float64).reshape(-1, 4)
    m = pts.shape[0]
    counts = np.zeros(2000, np.int32)
    inl = np.zeros(max(m, 1), np.int32)
    res = VooRansacResult()
    rc = lib().voo_ransac_ex(_p(pts), m, prob, thr, T, seed, rng_mode, _p(counts), _p(inl), C.byref(res))
    return dict(rc=rc, F=np.array(res.F[:]).reshape(3, 3), fitted=res.fitted, best_k=res.best_k,
                best_count=res.best_count, n_evaluated=res.n_evaluated, n_inl=res.n_inl,
                counts=counts[:res.n_evaluated].copy(), inliers=inl[:res.n_inl].copy())


def pose(F, K, p1, p2, scale=1.0):
    F = np.ascontiguousarray(F, dtype=np.float64).reshape(9)
    K = np.ascontiguousarray(K, dtype=np.float64).reshape(9)
    p1 = np.ascontiguousarray(p1, dtype=np.float32).reshape(-1, 2)
    p2 = np.ascontiguousarray(p2, dtype=np.float32).reshape(-1, 2)
    R = np.empty(9)
    t = np.empty(3)
    cnt = np.zeros(4, np.int32)
    rc = lib().voo_pose(_p(F), _p(K), _p(p1), _p(p2), p1.shape[0], scale, _p(R), _p(t), _p(cnt))
    return rc, R.reshape(3, 3), t, cnt


class VO:
    """Trajectory loop of the oracle (VisualOdometry::run restated)."""

    def __init__(self, cfg, gt=None):
        self.cfg = cfg
        self.h = lib().voo_vo_create(C.byref(cfg))
        self.gt = None if gt is None else np.ascontiguousarray(gt, dtype=np.float64).reshape(-1, 12)

    def process(self, gray):
        pose = np.zeros(12)
        st = C.c_int()
        info = np.zeros(8, np.int32)
        g = None if gray is None else np.ascontiguousarray(gray, dtype=np.uint8)
        gtp = _p(self.gt) if self.gt is not None else None
        gtn = 0 if self.gt is None else self.gt.shape[0]
        lib().voo_vo_process(self.h, _p(g) if g is not None else None, 0 if g is None else g.shape[1],
                             gtp, gtn, _p(pose), C.byref(st), _p(info))
        return pose.reshape(3, 4), st.value, info

    def close(self):
        if self.h:
            lib().voo_vo_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()


STAGES = ("blur", "response", "nms", "describe", "match", "ransac", "pose")


def stage_reset():
    lib().voo_stage_reset()


def stage_times():
    """{stage: (seconds, calls)} since the last stage_reset (the oracle's stage timers)."""
    sec = np.zeros(len(STAGES))
    n = np.zeros(len(STAGES), np.int64)
    lib().voo_stage_times(_p(sec), _p(n))
    return {k: (float(sec[i]), int(n[i])) for i, k in enumerate(STAGES)}


def mt_samples(seed32, m, nhyp):
    """The reference's std::sample draws of std::mt19937(seed32): (nhyp, 8) indices."""
    out = np.zeros((max(nhyp, 1), 8), np.int32)
    lib().voo_mt_samples(seed32 & 0xFFFFFFFF, m, nhyp, _p(out))
    return out[:nhyp]
