"""Parity under the library's launch-time knobs (tests/knob_parity.py; each
setting needs a process of its own because the knobs are read once)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

KNOBS = [
    {"CFWS_EDGE_SPLIT": "1"},
    {"CFWS_EDGE_ORDER": "0", "CFWS_SMALL": "0"},
    {"CFWS_EDGE_ORDER": "1", "CFWS_OCC_FRAME_MAX": "0", "CFWS_PLAN_LDS": "8192"},
    {"CFWS_GRID": "300", "CFWS_XFORM_LDS": "0"},
    {"CFWS_PLAN_SINGLE": "0"},
    {"CFWS_SER_INREG": "0"},
    {"CFWS_H2_INREG": "1"},
    {"CFWS_FUSED_DESER": "0"},
    {"CFWS_H2_UNITS_MERGED": "0"},
    {"CFWS_SLOTS_WINDOW": "0"},
    {"CFWS_SLOT_GRID": "37"},
]


@pytest.mark.parametrize("knobs", KNOBS, ids=lambda k: ",".join(f"{a[5:]}={b}" for a, b in k.items()))
def test_parity_under_knob(knobs):
    env = {k: v for k, v in os.environ.items() if not k.startswith("CFWS_")}
    env.update(knobs)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "knob_parity.py")], env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "KNOB OK" in r.stdout, r.stdout[-3000:] + r.stderr[-3000:]
