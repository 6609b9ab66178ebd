"""Device numerics that the parity tests rely on but cannot cover input by input.

drt::rcp_rn (drt_device.hpp) replaces hipcc's correctly rounded `1.0f / a` in the triangle tests
(scene.cpp:56, f = 1.0/a) by v_rcp_f32 plus one FMA Newton step inside 2^-125 <= |a| <= 2^125.
tools/rcp_check.hip compares it with the IEEE division for all 2^32 float inputs on the GPU; any
mismatch would be a parity hole that random scenes are unlikely to hit, so it runs here.
"""
import json
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
RCP_CHECK = ROOT / "tools" / "bin" / "rcp_check"


@pytest.mark.gpu
def test_rcp_rn_equals_ieee_division_for_every_float():
    if not RCP_CHECK.exists():
        pytest.fail(f"{RCP_CHECK} missing: build it with `make -C distributionraytracer_amd/csrc`")
    out = subprocess.run([str(RCP_CHECK)], capture_output=True, text=True, timeout=120)
    res = json.loads(out.stdout.strip().splitlines()[-1])
    assert res["inputs"] == 2 ** 32
    assert res["mismatches"] == 0, res
    # the guard is what makes it exact: the unguarded short path does differ outside the range
    assert res["short_path_mismatches_in_range"] == 0 and res["short_path_mismatches_outside_range"] > 0
    assert out.returncode == 0
