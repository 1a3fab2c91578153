"""CPU test of the drop-in's device policy (coldforce_amd/csrc/
cfws_devpolicy.h, used by cfws_frame.cpp): a thread following its current
device, a thread bound with cfws_bind_thread_device, threads that come and
go, and 16 threads switching devices at once. The header has no HIP types;
tests/native/devpolicy_test.cpp instantiates it with a fake resource."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_device_policy_native(tmp_path):
    exe = tmp_path / "devpolicy_test"
    subprocess.run(["g++", "-std=c++17", "-O1", "-pthread", "-Wall", "-Werror",
                    "-I", os.path.join(ROOT, "coldforce_amd", "csrc"),
                    os.path.join(ROOT, "tests", "native", "devpolicy_test.cpp"), "-o", str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout.startswith("OK ")


def test_bind_thread_device_abi_without_device():
    """The C-ABI half that runs without a GPU: argument checks and the
    no-device answer (a bound device must be a gfx950)."""
    from conftest import gpu_present
    if gpu_present():
        pytest.skip("checks the no-device behaviour")
    from coldforce_amd import cfws
    L = cfws.lib()
    assert L.cfws_bind_thread_device(-2) == -1          # CFWS_ERROR_INVALID_ARGUMENT
    assert L.cfws_bind_thread_device(64) == -1
    assert L.cfws_bind_thread_device(0) == -4           # CFWS_ERROR_NO_DEVICE
    assert L.cfws_bind_thread_device(-1) == 0
    assert L.cfws_init_device(0) == -4
