"""examples/batch_roundtrip.c: the batch C ABI driven from plain C (no
Python in the process): serialize, index the wire as a receive buffer,
deserialize (packed, into fixed slots, and to per-frame offsets); the wire must equal the
drop-in's co_ws_frame_serialize appends for the same random() stream and
every payload must come back."""
import json
import os
import subprocess

import pytest

from conftest import gpu_present

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "build", "examples", "batch_roundtrip")


def test_example_built_and_fails_loudly_without_device():
    if not os.path.exists(EXE):
        pytest.skip("build/examples not built (make)")
    if gpu_present():
        pytest.skip("a device is present")
    r = subprocess.run([EXE, "16"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and "no HIP device" in r.stderr


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_present(), reason="needs the MI355X")
@pytest.mark.parametrize("n,maxlen", [(4096, 70000), (20000, 300)])
def test_example_roundtrip(n, maxlen):
    assert os.path.exists(EXE), "build/examples/batch_roundtrip not built"
    r = subprocess.run([EXE, str(n), str(maxlen)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["frames"] == n and out["indexed"] == n
    assert out["wire_equals_dropin"] and out["roundtrip"] and out["slots"] and out["scatter"] and out["uniform"]
