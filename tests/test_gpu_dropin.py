"""GPU parity of the drop-in per-frame ABI (co_ws_frame_* exported by
libcfws.so, include/cfws_co_ws_frame.h) against the reference's golden
vectors: same wire bytes for the same random() stream, same decode results,
same NUL-terminated payloads."""
import hashlib
import random

import pytest

import oracle as O
from conftest import golden

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from coldforce_amd import cfws  # noqa: E402


def sha(b):
    return hashlib.sha256(b).hexdigest()


@pytest.fixture(scope="module", autouse=True)
def device():
    cfws.init()


@pytest.fixture(autouse=True)
def device_policy(request):
    """Every masked frame to the device (CFWS_DROPIN_GPU_MIN = 0) unless a
    test asks for the size policy's default (marker `host_policy`)."""
    L = cfws.lib()
    saved = L.cfws_dropin_gpu_min()
    if request.node.get_closest_marker("host_policy") is None:
        L.cfws_set_dropin_gpu_min(0)
    yield
    L.cfws_set_dropin_gpu_min(saved)


def test_serialize_golden_cases():
    import ctypes
    libc = ctypes.CDLL(None)
    for c in golden("serialize_cases.json"):
        data = O.fill_splitmix(c["n"], c["payload_seed"], c["payload_byte_base"]).tobytes()
        libc.srandom(c["seed"])
        ok, w = cfws.frame_serialize(c["fin"], c["opcode"], c["mask"], data)
        assert ok
        assert len(w) == c["wire_len"] and sha(w) == c["wire_sha256"], (c["n"], c["mask"])


def test_serialize_appends_with_reference_growth():
    # Several frames appended to one byte array: same bytes as one frame after
    # another, capacity = the co_array doubling rule (co_array.c:83-112).
    import ctypes
    libc = ctypes.CDLL(None)
    buf = cfws.byte_array_create()
    libc.srandom(5)
    expect = b""
    sizes = [0, 10, 200, 70000, 3]
    for n in sizes:
        ok, _ = cfws.frame_serialize(True, 2, True, bytes(range(256)) * (n // 256) + bytes(n % 256), buf)
        assert ok
    out = cfws.byte_array_bytes(buf)
    oracle_lib = O.lib()
    O.srandom(oracle_lib, 5)
    for n in sizes:
        expect += O.ref_serialize(oracle_lib, True, 2, True, bytes(range(256)) * (n // 256) + bytes(n % 256))
    assert out == expect
    cap = 8
    while cap <= len(expect):
        cap *= 2
    assert buf.capacity == cap and buf.count == len(expect)
    cfws.byte_array_destroy(buf)


def test_deserialize_golden_cases():
    for c in golden("deserialize_cases.json"):
        if c["wire_hex"] is None:
            continue
        raw = bytes.fromhex(c["wire_hex"])
        cfws.lib().co_ws_config_set_max_receive_payload_size(c["max_payload"])
        r = cfws.frame_deserialize(raw, c["index"])
        cfws.lib().co_ws_config_set_max_receive_payload_size(O.DEFAULT_MAX_PAYLOAD)
        got = (r["rc"], r["index"], r["fin"], r["opcode"], r["payload_size"], r["payload"] is None)
        exp = (c["rc"], c["index_out"], c["fin"], c["opcode"], c["payload_size"], c["payload_is_null"])
        assert got == exp, c["name"]
        if c["payload_sha256"] is not None:
            assert sha(r["payload"]) == c["payload_sha256"], c["name"]


def test_rfc6455_golden():
    for c in golden("rfc6455_kat.json"):
        if c["wire"] is None:
            continue
        r = cfws.frame_deserialize(bytes.fromhex(c["wire"]))
        assert (r["rc"], r["index"], r["fin"], r["opcode"], r["payload_size"]) == \
            (c["rc"], c["index"], c["fin"], c["opcode"], c["payload_size"])
        assert sha(r["payload"]) == c["payload_sha256"]


def test_random_roundtrip_vs_oracle():
    import ctypes
    libc = ctypes.CDLL(None)
    rng = random.Random(4)
    L = O.lib()
    for trial in range(60):
        # up to 1 MiB: zero-copy path; above: the DMA path (cfws_frame.cpp)
        n = rng.choice([1, 2, 125, 126, 65535, 65536, 65537, rng.randrange(300000),
                        (1 << 20) + rng.randrange(1, 3 << 20)])
        data = rng.randbytes(n)
        libc.srandom(trial)
        ok, w = cfws.frame_serialize(rng.random() < .5, rng.randrange(16), True, data)
        assert ok
        O.srandom(L, trial)
        assert w == O.ref_serialize(L, bool(w[0] & 0x80), w[0] & 0x7F, True, data)
        assert cfws.frame_deserialize(w) == O.ref_deserialize(L, w)


def test_frame_object_api():
    L = cfws.lib()
    f = L.co_ws_frame_create()
    assert L.co_ws_frame_get_opcode(f) == 0xFF and not L.co_ws_frame_get_fin(f)
    assert L.co_ws_frame_get_payload_size(f) == 0 and not L.co_ws_frame_get_payload_data(f)
    L.co_ws_frame_destroy(f)


def _fnv1a(b: bytes) -> int:
    h = 0xcbf29ce484222325
    for x in b:
        h = ((h ^ x) * 0x100000001b3) & 0xFFFFFFFFFFFFFFFF
    return h


@pytest.mark.parametrize("zc_max", [None, "0", "1000", "service_off", "policy_default"])
def test_link_level_dropin_harness(zc_max):
    """oracle/_ref/dropin_link: a C program built against coldforce's own
    headers (co_ws_frame.h, co_ws_config.h, co_byte_array.h) and the
    reference's co_array.c, linked to libcfws.so in place of co_ws_frame.c.
    Its wire equals the oracle's for the same random() stream, every frame
    decodes back, and the error codes are the reference's -- on the
    zero-copy path (default), the DMA path (CFWS_DROPIN_ZC_MAX=0) and both
    mixed (frames over 1,000 B by DMA)."""
    import os
    import subprocess
    exe = os.path.join(O.HERE, "_ref", "dropin_link")
    if not os.path.exists(exe):
        pytest.skip("oracle/_ref/dropin_link not built (built where /root/reference exists)")
    env = dict(os.environ)
    env.pop("CFWS_DROPIN_ZC_MAX", None)
    env.pop("CFWS_DROPIN_SERVICE", None)
    env["CFWS_DROPIN_GPU_MIN"] = "0"
    if zc_max == "policy_default":
        env.pop("CFWS_DROPIN_GPU_MIN")            # < 64 KiB on the calling thread
    elif zc_max == "service_off":
        env["CFWS_DROPIN_SERVICE"] = "0"          # every frame through the launch path
    elif zc_max is not None:
        env["CFWS_DROPIN_ZC_MAX"] = zc_max
    r = subprocess.run([exe, "77"], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    lines = r.stdout.split("\n")
    L = O.lib()
    O.srandom(L, 77)
    wire = b""
    sizes = [0, 1, 125, 126, 1000, 65535, 65536, 70000]
    for n in sizes:
        data = bytes((i * 131 + n) & 0xff for i in range(n))
        for mask in (False, True):
            wire += O.ref_serialize(L, True, 2, mask, data)
    assert lines[0] == f"wire {len(wire)} {_fnv1a(wire):016x}"
    assert lines[1] == f"frames {2 * len(sizes)} ok"
    at = 0
    for n in sizes[:4]:
        at += 2 * n + O.header_size(n, False) + O.header_size(n, True)
    assert lines[2] == f"codes 1 -7001 -7005 index {at}"


def test_thread_churn_reuses_resources():
    """Short-lived threads, three at a time, each decoding masked frames
    through the drop-in: every thread borrows a stream and staging buffers
    on its first frame and hands them back at exit (cfws_frame.cpp), so
    later threads reuse them; a thread that releases its resources early
    (cfws_release_thread_resources) gets fresh ones on its next frame."""
    import threading
    L = O.lib()
    O.srandom(L, 77)
    frames = []
    for n in (1, 126, 4000, 70000, (1 << 20) + 5):
        data = random.Random(n).randbytes(n)
        frames.append((O.ref_serialize(L, True, 2, True, data), data))
    errors = []

    def run(k):
        try:
            for j, (w, data) in enumerate(frames):
                r = cfws.frame_deserialize(w)
                assert r["rc"] == 0 and r["payload"] == data + b"\0", (k, j)
                if k == 1 and j == 2:
                    cfws.lib().cfws_release_thread_resources()
        except Exception as e:          # reported from the main thread
            errors.append(e)

    for _ in range(6):
        ts = [threading.Thread(target=run, args=(k,)) for k in range(3)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
    assert not errors, errors


def test_device_policy_bind_and_follow():
    """cfws_bind_thread_device: a bound thread's frames go to that device
    whatever its current device; unbound threads follow hipGetDevice; an
    ordinal that is not a visible gfx950 is refused."""
    import threading
    L = cfws.lib()
    n_dev = torch.cuda.device_count()
    assert L.cfws_bind_thread_device(n_dev) == -4          # CFWS_ERROR_NO_DEVICE
    assert L.cfws_bind_thread_device(-2) == -1
    data = random.Random(3).randbytes(5000)
    Lo = O.lib()
    O.srandom(Lo, 11)
    w = O.ref_serialize(Lo, True, 2, True, data)
    errors = []

    def run(dev):
        try:
            assert L.cfws_bind_thread_device(dev) == 0
            assert L.cfws_thread_device() == dev
            for _ in range(20):
                r = cfws.frame_deserialize(w)
                assert r["rc"] == 0 and r["payload"] == data + b"\0"
            assert L.cfws_bind_thread_device(-1) == 0
            torch.cuda.set_device(0)
            assert L.cfws_thread_device() == 0
            assert cfws.frame_deserialize(w)["payload"] == data + b"\0"
        except Exception as e:
            errors.append(e)

    ts = [threading.Thread(target=run, args=(d % n_dev,)) for d in range(2 * n_dev)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors, errors


def test_device_policy_spreads_over_gpus():
    """One thread per GPU, each bound to its own device, masking and
    unmasking concurrently: every thread's frames are correct and run on its
    device (a multi-thread coldforce server, co_net_worker.c:240)."""
    import threading
    n_dev = torch.cuda.device_count()
    if n_dev < 2:
        pytest.skip("needs 2+ GPUs")
    L = cfws.lib()
    errors = []
    data = random.Random(5).randbytes(70000)

    def run(dev):
        try:
            assert L.cfws_bind_thread_device(dev) == 0
            for k in range(50):
                ok, w = cfws.frame_serialize(True, 2, True, data)
                assert ok and w[1] & 0x80
                r = cfws.frame_deserialize(w)
                assert r["rc"] == 0 and r["payload"] == data + b"\0", (dev, k)
            assert L.cfws_thread_device() == dev
        except Exception as e:
            errors.append(e)

    ts = [threading.Thread(target=run, args=(d,)) for d in range(n_dev)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors, errors


def test_frame_service_idle_relaunch_and_seq_wrap():
    """The frame service (frames <= 64 KiB, cfws_frame.cpp): frames spaced
    wider than the service's idle timeout each find the kernel gone and
    relaunch it; 70,000 back-to-back frames wrap the 16-bit request
    sequence; sizes around the 16-byte chunk and the 64 KiB limit."""
    import time
    L = O.lib()
    rng = random.Random(9)
    cases = []
    for n in (1, 15, 16, 17, 1023, 1024, 1025, 65535, 65536, 65537):
        data = rng.randbytes(n)
        O.srandom(L, n)
        cases.append((O.ref_serialize(L, True, 1, True, data), data))
    for w, data in cases:
        assert cfws.frame_deserialize(w)["payload"] == data + b"\0"
        time.sleep(0.006)                      # > CFWS_DROPIN_SERVICE_IDLE_US (2 ms)
    w, data = cases[1]
    for k in range(70_000):
        r = cfws.frame_deserialize(w)
        if k % 5000 == 0 or k > 65_530:
            assert r["payload"] == data + b"\0", k
    # and the serialize side, against the reference's wire for the same keys
    import ctypes
    libc = ctypes.CDLL(None)
    for w, data in cases[:6]:
        libc.srandom(77)
        ok, got = cfws.frame_serialize(True, 2, True, data)
        O.srandom(L, 77)
        assert ok and got == O.ref_serialize(L, True, 2, True, data)


@pytest.mark.host_policy
def test_size_policy_both_sides():
    """The drop-in's size policy (cfws_set_dropin_gpu_min): payloads below the
    threshold are XORed on the calling thread, at or above it on the device;
    the wire and the decoded payloads equal the reference's on both sides,
    at the default threshold (SIZE_MAX: the calling thread at every size,
    the measured winner on wall and CPU time) and at
    moved ones (0: all device; 1000 and 65,536: both sides), for sizes
    around the 16-byte step and the thresholds themselves."""
    import ctypes
    libc = ctypes.CDLL(None)
    L = cfws.lib()
    Lo = O.lib()
    default = L.cfws_dropin_gpu_min()
    assert default == (1 << 64) - 1          # SIZE_MAX: every frame on the calling thread
    rng = random.Random(12)
    for gmin in (default, 0, 1000, 65536):
        L.cfws_set_dropin_gpu_min(gmin)
        for n in (1, 3, 15, 16, 17, 999, 1000, 1001, 4096, 65535, 65536, 65537, 300000):
            data = rng.randbytes(n)
            libc.srandom(n + gmin % 1000)
            ok, w = cfws.frame_serialize(True, 2, True, data)
            assert ok
            O.srandom(Lo, n + gmin % 1000)
            assert w == O.ref_serialize(Lo, True, 2, True, data), (gmin, n)
            assert cfws.frame_deserialize(w) == O.ref_deserialize(Lo, w), (gmin, n)


def test_service_many_threads_streaming():
    """16 threads on one device each stream masked frames through the frame
    service for 300 ms (1 KiB and 16 KiB frames alternating, deserialize of
    oracle-built frames plus serialize checked against the oracle's
    serialization under the key it drew), while a 17th thread sends 100 KiB
    frames through the launch path: the service kernel never idles out, it
    ends at its lifetime (CFWS_DROPIN_SERVICE_LIFE_US, 10 ms) and is
    relaunched under load, every frame is correct, and no call waits
    anywhere near the 5 s timeout (the largest per-frame time is reported
    and bounded)."""
    import threading
    import time
    Lo = O.lib()
    frames = []
    for n in (1024, 16384, 100_000):
        data = random.Random(n).randbytes(n)
        O.srandom(Lo, n)
        frames.append((O.ref_serialize(Lo, True, 2, True, data), data))
    errors, counts, worst = [], {}, {}
    t_end = time.perf_counter() + 0.3

    def run(k):
        try:
            c, slow = 0, 0.0
            big = k == 16
            while time.perf_counter() < t_end:
                w, data = frames[2] if big else frames[c % 2]
                t0 = time.perf_counter()
                r = cfws.frame_deserialize(w)
                slow = max(slow, time.perf_counter() - t0)
                assert r["rc"] == 0 and r["payload"] == data + b"\0", (k, c)
                if not big:
                    ok, s = cfws.frame_serialize(True, 1, True, data)
                    assert ok
                    key = int.from_bytes(s[len(s) - len(data) - 4:len(s) - len(data)], "little")
                    assert s == O.serialize_keyed(True, 1, True, key, data), (k, c)
                c += 1
            counts[k], worst[k] = c, slow
        except Exception as e:          # reported from the main thread
            errors.append(e)

    ts = [threading.Thread(target=run, args=(k,)) for k in range(17)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors, errors
    print("frames per thread", counts, "worst per-frame s", {k: round(v, 4) for k, v in worst.items()})
    assert all(counts[k] > 20 for k in range(17)), counts
    assert max(worst.values()) < 1.0, worst


def test_service_idle_gap_keeps_random_stream():
    """Two masked frames serialized after one srandom(), with a pause longer
    than the service's idle timeout between them (the second frame finds the
    kernel gone and relaunches it): both wires equal the reference's for the
    same seed, so nothing on the relaunch path consumed random()."""
    import ctypes
    import time
    libc = ctypes.CDLL(None)
    Lo = O.lib()
    datas = [random.Random(k).randbytes(n) for k, n in enumerate((1024, 20000, 77))]
    cfws.frame_serialize(True, 2, True, b"warm")        # service set up outside the seeded run
    time.sleep(0.02)
    libc.srandom(4321)
    got = []
    for d in datas:
        ok, w = cfws.frame_serialize(True, 2, True, d)
        assert ok
        got.append(w)
        time.sleep(0.02)                                 # > CFWS_DROPIN_SERVICE_IDLE_US (2 ms)
    O.srandom(Lo, 4321)
    assert got == [O.ref_serialize(Lo, True, 2, True, d) for d in datas]


def test_service_retired_slots_come_back():
    """A thread whose service answer does not come within the timeout retires
    its slot (the request stays posted; a later kernel may still XOR that
    buffer) and sends the frame through the launch path. Once the request
    completes the slot returns to the pool (before, each such
    stall lost a slot for good, and after 64 every frame took the launch
    path). With a 1 us timeout nearly every service frame retires its slot:
    more than 64 retirements in one process can only happen if slots come
    back, and every frame still equals the reference's."""
    import os
    import subprocess
    import sys
    script = r"""
import ctypes, sys
sys.path.insert(0, sys.argv[1])
import oracle as O
from coldforce_amd import cfws
cfws.init()
L = cfws.lib(); L.cfws_set_dropin_gpu_min(0)
libc = ctypes.CDLL(None); Lo = O.lib()
data = bytes(range(256)) * 4
for k in range(400):
    libc.srandom(k)
    ok, w = cfws.frame_serialize(True, 2, True, data)
    O.srandom(Lo, k)
    assert ok and w == O.ref_serialize(Lo, True, 2, True, data), k
    r = cfws.frame_deserialize(w)
    assert r["rc"] == 0 and r["payload"] == data + b"\0", k
print("ok")
"""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, CFWS_DROPIN_SERVICE_TIMEOUT_US="1")
    r = subprocess.run([sys.executable, "-c", script, root], capture_output=True, text=True,
                       timeout=120, env=env)
    assert r.returncode == 0 and "ok" in r.stdout, (r.stdout[-2000:], r.stderr[-2000:])
    retired = r.stderr.count("retired")
    print("retirements", retired)
    assert retired > 64, r.stderr[-2000:]
