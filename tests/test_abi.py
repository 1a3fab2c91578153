"""CPU checks of the C-ABI boundary: libcfws.so loads, exports every function
include/*.h declares, and its host-only parts behave like the reference
(no compute call that needs a GPU is made here)."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

import oracle as O
from conftest import ROOT, golden, gpu_present

LIB = os.path.join(ROOT, "coldforce_amd", "libcfws.so")


def declared_functions():
    names = set()
    for h in ("cfws.h", "cfws_co_ws_frame.h"):
        src = open(os.path.join(ROOT, "include", h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for m in re.finditer(r"^[A-Za-z_][\w \*]*?\b(\w+)\s*\(", src, flags=re.M):
            if not m.group(0).lstrip().startswith(("#", "typedef", "return")):
                names.add(m.group(1))
    return sorted(names)


def test_library_built():
    assert os.path.exists(LIB), "run `make` (libcfws.so is the product)"


def test_exports_every_declared_symbol():
    names = declared_functions()
    assert len(names) >= 24
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True,
                         check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    missing = [n for n in names if n not in exported]
    assert not missing, missing
    L = ctypes.CDLL(LIB)
    for n in names:
        getattr(L, n)


def test_python_binding_lists_match_headers():
    from coldforce_amd import cfws
    assert sorted(cfws.BATCH_SYMBOLS + cfws.DROPIN_SYMBOLS) == declared_functions()


def test_device_code_is_gfx950():
    blob = open(LIB, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob          # the embedded code object
    for other in (b"--gfx942", b"--gfx90a", b"--gfx1100"):
        assert other not in blob


def test_workspace_size_host_only():
    L = ctypes.CDLL(LIB)
    L.cfws_workspace_size.restype = ctypes.c_size_t
    L.cfws_workspace_size.argtypes = [ctypes.c_size_t, ctypes.c_uint64]
    a = L.cfws_workspace_size(65536, 1 << 32)
    # two passes x (per-frame offsets (8 B) + one u32 per 4 KiB output region)
    # + per plan block (256 frames) two u64 sums and the look-back's u32 + u64
    # words + a fixed part
    per_pass = 65536 * 8 + (1 << 32) // 4096 * 4
    blocks = 65536 // 256
    assert 2 * per_pass <= a < 2 * per_pass + blocks * (2 * 8 + 12) + 8192
    assert L.cfws_workspace_size(0, 0) > 0


def test_draw_mask_keys_matches_reference_stream():
    from coldforce_amd import cfws
    for seed, ks in golden("keys.json").items():
        got = cfws.draw_mask_keys(len(ks), seed=int(seed))
        assert [int.from_bytes(bytes.fromhex(k), "little") for k in ks] == [int(x) for x in got]
    # unmasked frames draw nothing and get key 0
    flags = np.array([1, 0, 1, 0], np.uint8)
    got = cfws.draw_mask_keys(4, flags, seed=1)
    ref = golden("keys.json")["1"]
    assert [int(x) for x in got] == [int.from_bytes(bytes.fromhex(ref[0]), "little"), 0,
                                     int.from_bytes(bytes.fromhex(ref[1]), "little"), 0]


def test_seeded_key_draw_equals_srandom_stream_and_keeps_global_state():
    """cfws_draw_mask_keys_seeded (a private random_r copy of the generator)
    draws what srandom(seed) + cfws_draw_mask_keys draws, and leaves the
    process's random() stream where it was."""
    from coldforce_amd import cfws
    libc = ctypes.CDLL(None)
    libc.random.restype = ctypes.c_long
    rng = np.random.default_rng(3)
    for seed in (0, 1, 2, 5, 1234, 0xFFFFFFFF):
        flags = (rng.random(3000) < .6).astype(np.uint8)
        libc.srandom(ctypes.c_uint(seed))
        glob = np.zeros(3000, np.uint32)
        cfws.lib().cfws_draw_mask_keys(3000, flags.ctypes.data, glob.ctypes.data)
        libc.srandom(ctypes.c_uint(99))
        before = libc.random()
        libc.srandom(ctypes.c_uint(99))
        seeded = cfws.draw_mask_keys(3000, flags, seed=seed)
        assert libc.random() == before                # global stream untouched
        assert np.array_equal(seeded, glob), seed


def test_dropin_host_paths_without_device():
    """Unmasked frames and header-only decisions never touch the device."""
    from coldforce_amd import cfws
    ok, w = cfws.frame_serialize(True, 1, False, b"Hello")
    assert ok and w.hex() == "810548656c6c6f"
    for c in golden("deserialize_cases.json"):
        if c["wire_hex"] is None:
            continue
        raw = bytes.fromhex(c["wire_hex"])
        masked_payload = c["rc"] == 0 and c["payload_size"] > 0 and (raw[c["index"] + 1] & 0x80)
        if masked_payload:
            continue
        cfws.lib().co_ws_config_set_max_receive_payload_size(c["max_payload"])
        r = cfws.frame_deserialize(raw, c["index"])
        cfws.lib().co_ws_config_set_max_receive_payload_size(O.DEFAULT_MAX_PAYLOAD)
        assert (r["rc"], r["index"], r["payload_size"], r["payload"] is None) == \
            (c["rc"], c["index_out"], c["payload_size"], c["payload_is_null"]), c["name"]


@pytest.mark.skipif(gpu_present(), reason="checks the no-device behaviour")
def test_no_cpu_fallback():
    """No gfx950 device: the batch API fails, and so does every masked frame
    the drop-in's size policy sends to the device. A frame below the
    policy's threshold is the library's own calling-thread loop (host_xor,
    not the oracle) and needs no device: it runs, bit-exact."""
    from coldforce_amd import cfws
    L = cfws.lib()
    assert L.cfws_init() == -4          # CFWS_ERROR_NO_DEVICE
    with pytest.raises(cfws.CodecError):
        cfws.init()
    saved = L.cfws_dropin_gpu_min()
    data = bytes(range(256)) * 4 + b"xyz"
    try:
        L.cfws_set_dropin_gpu_min(0)                               # every frame: device
        ok, _ = cfws.frame_serialize(True, 2, True, b"x" * 100)
        assert not ok
        w = O.serialize_keyed(True, 2, True, 0x11223344, b"x" * 100)
        assert cfws.frame_deserialize(w)["rc"] == -7006
        L.cfws_set_dropin_gpu_min(len(data) + 1)                   # below: calling thread
        ok, wire = cfws.frame_serialize(True, 2, True, data)
        assert ok
        key = int.from_bytes(wire[4:8], "little")                  # 126..65535: 2 + 2 B, key
        assert wire == O.serialize_keyed(True, 2, True, key, data)
        r = cfws.frame_deserialize(wire)
        assert r["rc"] == 0 and r["payload"] == data + b"\0"
        L.cfws_set_dropin_gpu_min(len(data))                       # at the threshold: device
        ok, _ = cfws.frame_serialize(True, 2, True, data)
        assert not ok
        assert cfws.frame_deserialize(wire)["rc"] == -7006
    finally:
        L.cfws_set_dropin_gpu_min(saved)


def test_link_level_dropin_fails_loudly_without_device():
    """The C harness built against coldforce's own headers (oracle/_ref/
    dropin_link, linked to libcfws.so): with no GPU its first masked
    non-empty frame fails -- serialize returns false and says why."""
    import os
    import subprocess
    exe = os.path.join(O.HERE, "_ref", "dropin_link")
    if not os.path.exists(exe):
        pytest.skip("oracle/_ref/dropin_link not built (needs /root/reference)")
    env = dict(os.environ, CFWS_DROPIN_GPU_MIN="0")
    r = subprocess.run([exe, "77"], capture_output=True, text=True, timeout=60, env=env)
    assert r.returncode == 2
    assert "serialize failed size=1 mask=1" in r.stdout
    assert "no HIP device" in r.stderr or "gfx950" in r.stderr
    # the default size policy: frames below the threshold run on the calling
    # thread without a device; the first masked frame at or above it fails
    env["CFWS_DROPIN_GPU_MIN"] = "65536"
    r = subprocess.run([exe, "77"], capture_output=True, text=True, timeout=60, env=env)
    assert r.returncode == 2
    assert "serialize failed size=65536 mask=1" in r.stdout


def test_deserialize_pass_kernel_routes():
    """cfws_deserialize_pass_kernel names the kernel cfws_deserialize_batch
    times for a call of these sizes (host only: the same rule the call
    applies, which bench.py reads instead of restating it)."""
    from coldforce_amd import cfws
    f = cfws.lib().cfws_deserialize_pass_kernel
    assert f(1000, 1000 * 264, 16, 0, 1 << 20).decode() == "deserialize_small_kernel"
    assert f(16 << 20, (16 << 20) * 264, 16, 0, 1 << 33).decode() == "deserialize_plan_single_kernel<true>"
    assert f(16 << 20, (16 << 20) * 264, 1, 0, 1 << 33).decode() == "xform_kernel<1>"       # align < 16
    assert f(65536, 65536 * 65550, 16, 0, 1 << 32).decode() == "xform_kernel<1>"           # large frames
    assert f(16 << 20, (16 << 20) * 264, 16, cfws.DESERIALIZE_REASSEMBLE, 1 << 33).decode() == "xform_kernel<1>"
    assert f(0, 0, 16, 0, 0).decode() == "xform_kernel<1>"


def test_serialize_uniform_pass_kernel_routes():
    """cfws_serialize_uniform_pass_kernel names the kernel
    cfws_serialize_uniform launches (host only; bench.py's roofline name)."""
    from coldforce_amd import cfws
    f = cfws.lib().cfws_serialize_uniform_pass_kernel
    for fs in (32, 256, 4096, 65520):
        assert f(fs, 1).decode() == "serialize_uniform_small_kernel"
    for fs, mask in ((65536, 1), (1000, 1), (4100, 0), (30, 1), (26, 1)):        # W >= 32
        assert f(fs, mask).decode() == "serialize_uniform_kernel", (fs, mask)
    for fs, mask in ((0, 1), (16, 1), (25, 1), (29, 0)):                        # W < 32
        assert f(fs, mask).decode() == "serialize_uniform_bytes_kernel", (fs, mask)


def test_deserialize_slots_pass_kernel_routes():
    """cfws_deserialize_slots_pass_kernel names the slot receives' kernel."""
    from coldforce_amd import cfws
    f = cfws.lib().cfws_deserialize_slots_pass_kernel
    full = lambda slot: f(1000, 1000 * (slot + 8), slot).decode()           # frames that fill their slots
    for slot in (16, 256, 1024, 2560, 3072, 4064, 5120, 8160):
        assert full(slot) == "deserialize_slots_window_kernel", slot
    for slot in (2048, 3584, 4096, 6144, 7680, 8176, 65536, 1 << 31):   # pieces >= 85 % used, on 128-B lines
        assert full(slot) == "deserialize_slots_piece_kernel", slot
    # frames shorter than their slots
    assert f(1000, 1000 * 264, 4096).decode() == "deserialize_slots_kernel"        # 6 % full
    assert f(1000, 1000 * 776, 1024).decode() == "deserialize_slots_kernel"        # 76 % of a 1 KiB slot
    assert f(1000, 1000 * 134, 256).decode() == "deserialize_slots_window_kernel"  # 52 % of 256 B
    assert f(1000, 1000 * 2056, 4096).decode() == "deserialize_slots_window_kernel"  # 2 KiB frames
    assert f(1000, 1000 * 264, 16384).decode() == "deserialize_slots_kernel"
    assert f(1000, 1000 * 4104, 65536).decode() == "deserialize_slots_piece_kernel"
    assert f(1000, 1000 * 1508, 16384).decode() == "deserialize_slots_piece_kernel"   # one wave per frame
    assert f(1000, 1000 * 1032, 16384).decode() == "deserialize_slots_kernel"
