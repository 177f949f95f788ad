"""include/vo_freak_tables.h against the reference's own header, parsed at test time (VERDICT r5
Missing 2): the 43 retinal sample offsets (predefined_point_for_matching,
feature_extraction_parallel_GPU/FREAK_feature_descriptor_parallel_GPU.h:47-56), the pair order of
generate_tests (:58-81: i < j, row-major) and the 512 tested pair indices (PATCH_DESCRIPTION_POINTS,
:87-123).  The oracle, the HIP kernels and tests/ref_cl.py's reference-kernel driver all include or
parse our header, so a transcription error there would be invisible to every parity test; this is
the test that sees it.  Skipped where /root/reference is absent (the GPU box)."""
import os
import re

import numpy as np
import pytest

from ref_cl import REF_FREAK_HEADER, freak_tables, parse_reference_freak_header

pytestmark = pytest.mark.skipif(not os.path.exists(REF_FREAK_HEADER), reason="reference sources absent")


def test_points_and_patch_equal_the_reference_header():
    pts, patch, body = parse_reference_freak_header(REF_FREAK_HEADER)
    assert len(pts) == 43 and len(patch) == 512
    ours_tc, ours_patch = freak_tables(source="ours")
    # rows 0..41 are the pairs (0, 1) .. (0, 42)
    ours_pts = [tuple(int(v) for v in ours_tc[0, :2])] + [tuple(int(v) for v in ours_tc[k, 2:]) for k in range(42)]
    assert ours_pts == pts
    assert list(ours_patch.astype(int)) == patch
    # every tested pair exists; the tested set has no duplicate
    assert max(patch) < 903 and len(set(patch)) == 512


def test_pair_order_is_generate_tests():
    """generate_tests' loop nest (i outer, j = i + 1 .. inner, result[index++]) is the order our pair
    table t = 0..902 follows; checked on the reference's statements, then on the tables."""
    pts, _, body = parse_reference_freak_header(REF_FREAK_HEADER)
    loops = re.findall(r"for\s*\(\s*size_t\s+(\w+)\s*=\s*([^;]+);", body)
    assert [v for v, _ in loops[:2]] == ["i", "j"]
    assert loops[0][1].strip() == "0" and re.sub(r"\s", "", loops[1][1]) == "i+1"
    assert "result[index++]" in body
    tc, _ = freak_tables(source="ours")
    exp = [(*pts[i], *pts[j]) for i in range(43) for j in range(i + 1, 43)]
    assert [tuple(r) for r in tc] == exp
    assert tc.shape == (903, 4)


def test_ref_cl_reads_the_reference_header_where_present():
    a, pa = freak_tables()                 # the reference-kernel driver's tables
    b, pb = freak_tables(source="ours")
    assert np.array_equal(a, b) and np.array_equal(pa, pb)
