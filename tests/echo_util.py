"""TEST INFRASTRUCTURE ONLY -- runs oracle/ws_echo.c's echo pair (config 1,
BASELINE.json configs[0]) over 127.0.0.1.

Two builds of the same program exist under oracle/_ref/ (oracle/Makefile):
``stock`` links the reference's own co_ws_frame.c + co_ws_config.c, ``cfws``
links libcfws.so in their place; everything around the codec is the
reference's src/core, net, http, http2, ws and ws_http2 compiled in place.
"""
from __future__ import annotations

import json
import os
import select
import socket
import subprocess
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_DIR = os.path.join(ROOT, "oracle", "_ref")
BUILDS = {"stock": os.path.join(REF_DIR, "ws_echo_stock"),
          "cfws": os.path.join(REF_DIR, "ws_echo_cfws")}


def available(build: str) -> bool:
    return os.path.exists(BUILDS[build])


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _read_line(proc: subprocess.Popen, timeout: float) -> str:
    end = time.monotonic() + timeout
    buf = b""
    fd = proc.stdout.fileno()
    while not buf.endswith(b"\n"):
        left = end - time.monotonic()
        if left <= 0 or proc.poll() is not None and not select.select([fd], [], [], 0)[0]:
            break
        r, _, _ = select.select([fd], [], [], min(left, 0.5))
        if r:
            c = os.read(fd, 1)
            if not c:
                break
            buf += c
    return buf.decode(errors="replace")


def run_echo(build: str, mode: str, frames: int, payload: int = 1024, window: int = 64, seed: int = 1,
             port: int | None = None, capture_dir: str | None = None, timeout: float = 300.0,
             env: dict | None = None) -> dict:
    """One server process + one client process of `build` in `mode` ("ws" or
    "h2"). Returns the client's and server's JSON lines, return codes, stderr
    tails and, with capture_dir, the paths of each side's sent bytes."""
    exe = BUILDS[build]
    port = port or free_port()
    env_s = dict(os.environ, **(env or {}))
    env_c = dict(os.environ, **(env or {}))
    cap = {}
    if capture_dir:
        os.makedirs(capture_dir, exist_ok=True)
        cap = {"client": os.path.join(capture_dir, f"{build}_{mode}_client.bin"),
               "server": os.path.join(capture_dir, f"{build}_{mode}_server.bin")}
        env_s["CFWS_ECHO_CAPTURE"] = cap["server"]
        env_c["CFWS_ECHO_CAPTURE"] = cap["client"]
    srv = subprocess.Popen([exe, f"{mode}-server", str(port)], stdout=subprocess.PIPE,
                           stderr=subprocess.PIPE, env=env_s)
    try:
        first = _read_line(srv, 60.0)
        if '"listening"' not in first:
            srv.kill()
            out, err = srv.communicate(timeout=10)
            raise RuntimeError(f"{build} {mode} server did not start: {first!r} {err[-2000:]!r}")
        url = f"{'ws' if mode == 'ws' else 'http'}://127.0.0.1:{port}/"
        cli = subprocess.run([exe, f"{mode}-client", url, str(frames), str(payload), str(window), str(seed)],
                             capture_output=True, text=True, timeout=timeout, env=env_c)
        try:
            s_out, s_err = srv.communicate(timeout=30)
        except subprocess.TimeoutExpired:
            srv.kill()
            s_out, s_err = srv.communicate(timeout=10)
    finally:
        if srv.poll() is None:
            srv.kill()
            srv.wait(timeout=10)
    client = None
    for line in cli.stdout.splitlines():
        if line.startswith("{"):
            client = json.loads(line)
    server = None
    for line in s_out.decode(errors="replace").splitlines():
        if '"echoed"' in line:
            server = json.loads(line)
    return {"build": build, "mode": mode, "port": port, "client": client, "server": server,
            "client_rc": cli.returncode, "server_rc": srv.returncode,
            "client_err": cli.stderr[-2000:], "server_err": s_err.decode(errors="replace")[-2000:],
            "capture": cap}


def split_http(wire: bytes) -> tuple[bytes, bytes]:
    """HTTP/1.1 head (through CRLFCRLF) and what follows it."""
    k = wire.index(b"\r\n\r\n") + 4
    return wire[:k], wire[k:]


def h2_frames(stream: bytes, preface: bool):
    """(type, flags, stream_id, payload) of each HTTP/2 frame in a byte stream
    (co_http2_frame.c:33-72 layout)."""
    p = 24 if preface else 0
    out = []
    while p + 9 <= len(stream):
        n = int.from_bytes(stream[p:p + 3], "big")
        t, fl = stream[p + 3], stream[p + 4]
        sid = int.from_bytes(stream[p + 5:p + 9], "big") & 0x7FFFFFFF
        out.append((t, fl, sid, stream[p + 9:p + 9 + n]))
        p += 9 + n
    assert p == len(stream), "trailing partial HTTP/2 frame"
    return out


def h2_data_frames(stream: bytes, preface: bool) -> list[tuple[int, bytes]]:
    """(flags, raw frame bytes: 9-byte header + payload) of every DATA frame
    (type 0) in a captured HTTP/2 byte stream, in order."""
    p = 24 if preface else 0
    out = []
    while p + 9 <= len(stream):
        n = int.from_bytes(stream[p:p + 3], "big")
        if stream[p + 3] == 0:
            out.append((stream[p + 4], stream[p:p + 9 + n]))
        p += 9 + n
    assert p == len(stream), "trailing partial HTTP/2 frame"
    return out


def frame_text(k: int, payload: int) -> bytes:
    """Frame k's payload: byte j is 'a' + (j + k) % 26 (oracle/ws_echo.c)."""
    base = bytes(97 + i % 26 for i in range(payload + 26))
    return base[k % 26:k % 26 + payload]
