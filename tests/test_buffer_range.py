"""gfx950's buffer range check, pinned on the hardware (tests/hip/buffer_range_probe.hip).

k_stencil drops stores without a branch by giving them an out-of-range buffer offset: halo lanes
through voffset, the blurred rows past a segment (round 3) through soffset.  Whether soffset is part
of the raw-buffer range check was the open question of round 3's determinism finding (if it were
not, those stores would land 1 GiB past the blurred plane).  The probe answers it: the check covers
voffset + soffset, for stores, loads and atomics, and cuts a straddling access at num_records.  The stencil
now drops through voffset, which is covered either way."""
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROBE = os.path.join(ROOT, "acs_visual_odometry_amd", "bin", "buffer_range_probe")


def test_probe_is_built():
    assert os.access(PROBE, os.X_OK), "make -C acs_visual_odometry_amd/csrc builds the probe"


@pytest.mark.gpu
def test_buffer_range_check_covers_soffset_and_voffset():
    out = subprocess.run([PROBE], capture_output=True, text=True, timeout=60, check=True).stdout
    rows = {r["case"]: r for r in (json.loads(line) for line in out.splitlines() if line.startswith("{"))}
    assert set(rows) == {0, 1, 2, 3, 4, 5, 6}, out
    # 0: soffset = 1 GiB, 1: voffset = 1 GiB -- dropped, nothing lands in range or at +1 GiB
    for c in (0, 1):
        assert rows[c]["stores_in_range"] == 0 and rows[c]["stores_at_1gib"] == 0, rows[c]
    # 2 / 3: offset 4000 + 2 lane straddles num_records = 4096 through voffset / soffset: the
    # 48 lanes below 4096 store, the rest are dropped (so soffset is inside the check)
    for c in (2, 3):
        assert rows[c]["stores_in_range"] == 48, rows[c]
        assert (rows[c]["first_byte"], rows[c]["last_byte"]) == (4000, 4094), rows[c]
        assert rows[c]["stores_at_1gib"] == 0, rows[c]
    # 4: a load with soffset = 1 GiB returns 0, not the pattern stored there
    assert rows[4]["loads_of_1gib_pattern"] == 0 and rows[4]["loads_zero"] == 64, rows[4]
    # 5 / 6: buffer atomics obey the same check (out of range: dropped; in range: applied once each)
    assert rows[5]["stores_in_range"] == 0 and rows[5]["stores_at_1gib"] == 0, rows[5]
    assert rows[6]["atomics_in_range"] == 64, rows[6]
