"""Config 1 (BASELINE.json configs[0]) and the WebSocket-over-HTTP/2 callers
on the reference's own code, with the drop-in underneath.

oracle/ws_echo.c is an echo pair modelled on examples/ws_client/main.c:107-167
and examples/ws_server/main.c:32-80,131-157 (plus the ws-over-h2 test
threads, test/test_http/test_ws_http2_client_thread.c and
test_http_server_http2_connection.c). Every frame travels through the
reference's unchanged callers: co_ws_send (co_ws_client.c:427-460), the
receive loops (co_ws_client.c:178-274, co_ws_server.c:85-173) with their
INVALID_FRAME -> HTTP fallback carrying the upgrade, and
co_http2_stream_send_ws_frame / co_http2_stream_receive_ws_frame
(co_ws_http2_extension.c:134-199) over the reference's own
co_http2_stream_send_data (co_http2_stream.c:933-1013).

CPU tests pin the stock build (reference codec) to the oracle: the client's
wire is the oracle's serialization of the frames under srandom(seed) keys.
GPU tests run the drop-in build (libcfws.so in place of co_ws_frame.c /
co_ws_config.c) on the same port and seed and require byte-identical wire
in both directions, and every echo correct.
"""
import base64
import json
import os

import pytest

import oracle as O
from echo_util import available, free_port, frame_text, h2_frames, run_echo, split_http

PAYLOAD = 1024


def _need(build):
    if not available(build):
        pytest.skip(f"oracle/_ref/ws_echo_{build} not built (needs /root/reference at build time)")


def _ok(r, frames):
    assert r["client_rc"] == 0, (r["client_err"], r["server_err"])
    assert r["client"] is not None and r["client"]["received"] == frames, r
    assert r["client"]["bad_echo"] == 0 and r["client"]["upgrade_ok"] == 1
    assert r["server"] is not None and r["server"]["echoed"] == frames, r


def _read(path):
    with open(path, "rb") as f:
        return f.read()


def _check_ws_wire(client_wire, server_wire, frames, seed):
    """The stock client's bytes = upgrade request (key: 16 random() draws,
    co_random via co_ws_http_extension.c) + the oracle's serialization of
    every TEXT frame masked with the next keys of srandom(seed)'s stream +
    the CLOSE 1000 that co_ws_client_destroy sends (co_ws_client.c:364),
    masked with the key after those."""
    head, body = split_http(client_wire)
    keys = O.keys(seed, frames + 5)
    key16 = b"".join(int(k).to_bytes(4, "little") for k in keys[:4])
    assert b"Sec-WebSocket-Key: " + base64.b64encode(key16) + b"\r\n" in head
    exp = b"".join(O.serialize_keyed(True, 1, True, int(keys[4 + k]), frame_text(k, PAYLOAD))
                   for k in range(frames))
    exp += O.serialize_keyed(True, 8, True, int(keys[4 + frames]), (1000).to_bytes(2, "big"))
    assert body == exp
    shead, sbody = split_http(server_wire)
    assert shead.startswith(b"HTTP/1.1 101 ")
    # the echoes, then co_ws_default_handler's reply to the CLOSE
    sexp = b"".join(O.serialize_keyed(True, 1, False, 0, frame_text(k, PAYLOAD)) for k in range(frames))
    assert sbody == sexp + O.serialize_keyed(True, 8, False, 0, (1000).to_bytes(2, "big"))


def _check_h2_wire(client_wire, frames, seed):
    """The stock client's DATA frames on stream 1: one WS frame each, with
    END_STREAM (co_ws_http2_extension.c:190-194), masked with srandom(seed)'s
    keys (the CONNECT request draws none)."""
    data = [f for f in h2_frames(client_wire, preface=True) if f[0] == 0]
    assert len(data) == frames
    keys = O.keys(seed, frames)
    for k, (t, fl, sid, pl) in enumerate(data):
        assert sid == 1 and fl & 1
        assert pl == O.serialize_keyed(True, 1, True, int(keys[k]), frame_text(k, PAYLOAD)), k


# ---------------------------------------------------------------------------
# CPU: the harness and the stock build, pinned to the oracle
# ---------------------------------------------------------------------------
def test_stock_ws_echo_matches_oracle(tmp_path):
    _need("stock")
    frames = 3000
    r = run_echo("stock", "ws", frames, PAYLOAD, window=16, seed=1, capture_dir=str(tmp_path))
    _ok(r, frames)
    _check_ws_wire(_read(r["capture"]["client"]), _read(r["capture"]["server"]), frames, 1)


def test_stock_h2_echo_matches_oracle(tmp_path):
    _need("stock")
    frames = 2000
    r = run_echo("stock", "h2", frames, PAYLOAD, window=16, seed=3, capture_dir=str(tmp_path))
    _ok(r, frames)
    _check_h2_wire(_read(r["capture"]["client"]), frames, 3)


def test_stock_wire_is_deterministic(tmp_path):
    """Same seed, same port, same window: same bytes both ways (what the GPU
    comparison below relies on)."""
    _need("stock")
    port = free_port()
    a = run_echo("stock", "ws", 500, PAYLOAD, window=8, seed=9, port=port, capture_dir=str(tmp_path / "a"))
    b = run_echo("stock", "ws", 500, PAYLOAD, window=8, seed=9, port=port, capture_dir=str(tmp_path / "b"))
    _ok(a, 500)
    _ok(b, 500)
    for side in ("client", "server"):
        assert _read(a["capture"][side]) == _read(b["capture"][side])


@pytest.mark.skipif(__import__("conftest").gpu_present(), reason="checks the no-device behaviour")
@pytest.mark.parametrize("gpu_min", ["0", None], ids=["device_policy", "default_policy"])
def test_dropin_build_without_device(gpu_min):
    """No GPU. With every masked frame sent to the device
    (CFWS_DROPIN_GPU_MIN=0) the drop-in build's first masked frame fails
    (co_ws_send ignores the false return, co_ws_client.c:445-449, so nothing
    is sent), the client never completes, and libcfws says why on stderr.
    Under the default size policy config 1's 1 KiB frames are below the
    threshold: the library's own calling-thread loop masks them with no
    device, and the echo completes."""
    _need("cfws")
    # run the client against a stock server so only the client uses the drop-in
    import os
    import subprocess
    from echo_util import BUILDS, _read_line
    env = dict(os.environ)
    env.pop("CFWS_DROPIN_GPU_MIN", None)
    if gpu_min is not None:
        env["CFWS_DROPIN_GPU_MIN"] = gpu_min
    port = free_port()
    srv = subprocess.Popen([BUILDS["stock"], "ws-server", str(port)], stdout=subprocess.PIPE,
                           stderr=subprocess.PIPE)
    try:
        assert '"listening"' in _read_line(srv, 30)
        try:
            cli = subprocess.run([BUILDS["cfws"], "ws-client", f"ws://127.0.0.1:{port}/", "4", "1024", "1", "1"],
                                 capture_output=True, text=True, timeout=5 if gpu_min else 30, env=env)
            out, err = cli.stdout, cli.stderr
        except subprocess.TimeoutExpired as e:
            out = (e.stdout or b"").decode() if isinstance(e.stdout, bytes) else (e.stdout or "")
            err = (e.stderr or b"").decode() if isinstance(e.stderr, bytes) else (e.stderr or "")
        if gpu_min is not None:
            assert '"received": 4' not in out
            assert "no HIP device" in err or "gfx950" in err or "usable device" in err
        else:
            assert '"received": 4' in out, (out, err)
    finally:
        srv.kill()
        srv.wait(timeout=10)


# ---------------------------------------------------------------------------
# GPU: the drop-in under the reference's callers
# ---------------------------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("policy", ["default", "device"])
@pytest.mark.parametrize("mode", ["ws", "h2"])
def test_dropin_echo_wire_identical_to_stock(mode, policy, tmp_path):
    """Config 1 (100 k masked 1 KiB TEXT frames after srandom(1)) through the
    reference's callers: the drop-in build's wire equals the stock build's
    byte for byte in both directions, and every echo checks. Under the
    default size policy the 1 KiB payloads are XORed on the calling thread;
    with CFWS_DROPIN_GPU_MIN=0 every one goes through the device (the frame
    service)."""
    _need("stock")
    _need("cfws")
    frames = 100_000
    port = free_port()
    out = {}
    for build in ("stock", "cfws"):
        r = run_echo(build, mode, frames, PAYLOAD, window=64, seed=1, port=port,
                     capture_dir=str(tmp_path / build), timeout=240,
                     env={"CFWS_DROPIN_GPU_MIN": "0"} if policy == "device" else None)
        _ok(r, frames)
        out[build] = r
    for side in ("client", "server"):
        a = _read(out["stock"]["capture"][side])
        b = _read(out["cfws"]["capture"][side])
        assert len(a) == len(b) and a == b, (mode, side)
    if mode == "ws":
        assert len(_read(out["cfws"]["capture"]["client"])) > frames * (PAYLOAD + 8)
    dst = os.environ.get("CFWS_CONFIG1_OUT")
    if dst:
        with open(dst, "a") as f:
            for build in ("stock", "cfws"):
                f.write(json.dumps({"test": "wire_identical", "build": build, "mode": mode,
                                    "policy": policy, **out[build]["client"]}) + "\n")


@pytest.mark.gpu
def test_dropin_echo_small_frames_and_binary_sizes(tmp_path):
    """Frame sizes around the header-length boundaries through the real
    callers (125/126 B, 65,535/65,536 B) are checked by every echo; the wire
    equals the stock build's. Under the default size policy
    (CFWS_DROPIN_GPU_MIN_DEFAULT = SIZE_MAX, include/cfws.h) every one of
    these frames is XORed on the calling thread; the device paths at these
    sizes are test_dropin_device_paths_wire_identical_to_stock's."""
    _need("stock")
    _need("cfws")
    for payload, frames in ((125, 2000), (126, 2000), (65535, 200), (65536, 200)):
        port = free_port()
        wires = []
        for build in ("stock", "cfws"):
            r = run_echo(build, "ws", frames, payload, window=8, seed=payload, port=port,
                         capture_dir=str(tmp_path / f"{build}_{payload}"), timeout=120)
            _ok(r, frames)
            wires.append((_read(r["capture"]["client"]), _read(r["capture"]["server"])))
        assert wires[0] == wires[1], payload


def _accept_pairs(tmp_path, seeds):
    """(Sec-WebSocket-Key the stock client sent, Sec-WebSocket-Accept the
    stock server answered) for each seed: the reference's own static
    co_ws_create_base64_accept_key (co_ws_http_extension.c:26-57), reached
    through co_http_response_create_ws_upgrade (:322-362)."""
    import re
    pairs = []
    for seed in seeds:
        r = run_echo("stock", "ws", 1, 16, window=1, seed=seed, capture_dir=str(tmp_path / str(seed)))
        _ok(r, 1)
        chead, _ = split_http(_read(r["capture"]["client"]))
        shead, _ = split_http(_read(r["capture"]["server"]))
        key = re.search(rb"Sec-WebSocket-Key: (\S+)\r\n", chead).group(1)
        acc = re.search(rb"Sec-WebSocket-Accept: (\S+)\r\n", shead).group(1)
        pairs.append((key, acc.decode()))
    return pairs


def test_stock_accept_key_matches_oracle(tmp_path):
    """The oracle's accept key equals the reference's static function's, as
    the stock server put it on the wire."""
    _need("stock")
    for key, acc in _accept_pairs(tmp_path, (1, 2, 3, 99, 12345)):
        assert O.ws_accept_key(key) == acc, key


@pytest.mark.gpu
def test_device_accept_key_matches_reference_server(tmp_path):
    """ws_accept_kernel (cfws_ws_accept_keys_batch) against the accept keys
    the reference's own server code computed for the same client keys."""
    _need("stock")
    from coldforce_amd import cfws
    cfws.init()
    pairs = _accept_pairs(tmp_path, (1, 2, 3, 99, 12345))
    got = cfws.ws_accept_keys([k for k, _ in pairs])
    assert got == [a for _, a in pairs]


@pytest.mark.gpu
@pytest.mark.parametrize("mode,payload,frames", [("ws", 65536, 200), ("ws", 2 << 20, 24),
                                                 ("h2", 16376, 64), ("h2", 16377, 64),
                                                 ("h2", 40000, 64), ("h2", 65536, 64)])
def test_dropin_device_paths_wire_identical_to_stock(mode, payload, frames, tmp_path):
    """The drop-in's device paths through the reference's callers, every
    masked frame sent to the device (CFWS_DROPIN_GPU_MIN=0): 65,536 B takes
    the per-frame launch on mapped staging, 2 MiB the DMA path (under the
    32 MiB receive limit), 16,376-40,000 B the frame service. The callers
    are co_ws_send (co_ws_client.c:427-460) and the receive loops
    (co_ws_server.c:85-173, co_ws_client.c:178-274); in h2 mode
    co_http2_stream_send_ws_frame / co_http2_stream_receive_ws_frame over
    the reference's co_http2_stream_send_data split into several DATA frames
    (co_http2_stream.c:933-1013) and the receiver's pooling (:550-608). The
    wire equals the stock build's byte for byte in both directions, and the
    h2 runs equal tests/golden/h2_echo_digests.json (the stock capture)."""
    _need("stock")
    _need("cfws")
    import hashlib
    from conftest import golden
    from echo_util import h2_data_frames
    window = 4 if payload >= (1 << 20) else 8
    seed = payload % 1000 + 1
    g = None
    if mode == "h2":
        g = next(c for c in golden("h2_echo_digests.json") if c["payload"] == payload)
        frames, window, seed = g["frames"], g["window"], g["seed"]
    port = free_port()
    caps = {}
    for build in ("stock", "cfws"):
        r = run_echo(build, mode, frames, payload, window=window, seed=seed, port=port,
                     capture_dir=str(tmp_path / build), timeout=240,
                     env={"CFWS_DROPIN_GPU_MIN": "0"} if build == "cfws" else None)
        _ok(r, frames)
        caps[build] = {side: _read(r["capture"][side]) for side in ("client", "server")}
    for side in ("client", "server"):
        assert caps["stock"][side] == caps["cfws"][side], (mode, payload, side)
        if g is not None:
            data = h2_data_frames(caps["cfws"][side], preface=side == "client")
            raw = b"".join(x for _, x in data)
            assert hashlib.sha256(raw).hexdigest() == g[side]["data_sha256"], side
