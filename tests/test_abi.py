"""The C-ABI library loads and exports every symbol include/vo_mi355x.h declares (no GPU
calls), and it carries gfx950 code objects only."""
import ctypes as C
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "vo_mi355x.h")
LIB = os.path.join(ROOT, "acs_visual_odometry_amd", "libvo_mi355x.so")


def declared_symbols():
    src = open(HDR).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(vo_[A-Za-z0-9_]+)\s*\(", src)))


def test_header_declares_the_boundary():
    syms = declared_symbols()
    for s in ["vo_create", "vo_destroy", "vo_extract", "vo_match", "vo_ransac_F", "vo_pose", "vo_process_frame",
              "vo_process_frames_device", "vo_strerror"]:
        assert s in syms


def test_library_exports_every_declared_symbol():
    assert os.path.exists(LIB), "run __graft_entry__.build() first"
    lib = C.CDLL(LIB)
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing


def test_vo_config_layout_matches_the_binding(tmp_path):
    """sizeof / offsetof of the header's vo_config (gcc) equal the ctypes mirror's, so a binding of
    the wrong ABI version cannot silently under-allocate the struct (rng_mode grew it)."""
    from acs_visual_odometry_amd import _lib
    fields = [f for f, _ in _lib.VoConfig._fields_]
    src = tmp_path / "cfg.c"
    body = "".join(f'printf("%zu\\n", offsetof(vo_config, {f}));' for f in fields)
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "vo_mi355x.h"\n'
                   f'int main(void){{printf("%zu\\n", sizeof(vo_config));{body}return 0;}}\n')
    exe = tmp_path / "cfg"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()]
    assert got[0] == C.sizeof(_lib.VoConfig)
    assert got[1:] == [getattr(_lib.VoConfig, f).offset for f in fields]


def test_python_binding_lists_every_export():
    from acs_visual_odometry_amd import _lib
    assert sorted(_lib.EXPORTS) == declared_symbols()


def test_host_only_entry_points():
    """Entry points that need no device: strerror, config defaults, descriptor unpack."""
    from acs_visual_odometry_amd import _lib
    L = _lib.load()
    assert L.vo_abi_version() == 2 == _lib.VO_ABI_VERSION
    assert L.vo_strerror(-10) == b"Degenerate essential matrix"
    cfg = _lib.default_config(1241, 376)
    assert (cfg.max_kpts, cfg.nms_k, cfg.border_row, cfg.border_col, cfg.match_bits) == (2000, 3, 35, 37, 32)
    assert abs(cfg.resp_thr - 20000.0) < 1e-9 and abs(cfg.ratio - 0.75) < 1e-9
    assert cfg.ransac_p == 0.99 and cfg.sampson_thr == 1.0
    assert list(cfg.K) == [718.856, 0.0, 607.1928, 0.0, 718.856, 185.2157, 0.0, 0.0, 1.0]
    import numpy as np
    w = np.array([1, 0, 0, 0, 0, 0, 0, 1 << 63], np.uint64)
    b = np.zeros(512, np.uint8)
    L.vo_unpack_descriptor(w.ctypes.data_as(C.c_void_p), b.ctypes.data_as(C.c_void_p))
    assert b[0] == 1 and b[511] == 1 and b.sum() == 2
    from acs_visual_odometry_amd import pack_descriptor, unpack_descriptor
    assert np.array_equal(unpack_descriptor(w)[0], b)
    assert np.array_equal(pack_descriptor(b)[0], w)


def test_create_without_gpu_fails_loudly():
    if os.path.exists("/dev/kfd"):
        pytest.skip("GPU present")
    from acs_visual_odometry_amd import Context
    with pytest.raises(RuntimeError):
        Context(1241, 376)


def test_code_objects_are_gfx950():
    blob = open(LIB, "rb").read()
    targets = set(re.findall(rb"amdgcn-amd-amdhsa--(gfx[0-9a-z]+)", blob))
    assert targets == {b"gfx950"}, targets
