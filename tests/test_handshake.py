"""Handshake accept keys: cfws_ws_accept_keys_batch
against the reference's co_sha1.c + co_base64.c (tests/golden/
handshake_cases.json) and the oracle on a connection storm of random keys."""
import base64
import random

import pytest

import oracle as O
from conftest import golden, gpu_present

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not gpu_present(), reason="needs the MI355X")]

torch = pytest.importorskip("torch")

from coldforce_amd import cfws  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def device():
    cfws.init()


def test_accept_keys_reference_fixtures():
    cases = golden("handshake_cases.json")
    got = cfws.ws_accept_keys([bytes.fromhex(c["key_hex"]) for c in cases])
    assert got == [c["accept"] for c in cases]


def test_accept_keys_connection_storm():
    rng = random.Random(7)
    keys = [base64.b64encode(rng.randbytes(16)) for _ in range(20000)]
    keys += [rng.randbytes(rng.randrange(0, 260)) for _ in range(2000)]   # any bytes, any length
    got = cfws.ws_accept_keys(keys)
    assert got == [O.ws_accept_key(k) for k in keys]


@pytest.mark.parametrize("slot_shift", [0, 1])
def test_accept_keys_decreasing_offset_gives_empty_slot(slot_shift):
    """A key whose end offset lies below its start (a caller bug) gets an
    all-zero slot instead of a wrapped 2^64-byte length; its neighbours are
    computed as usual. slot_shift 1: the output is not 16-byte aligned (the
    byte-store form)."""
    import numpy as np
    keys = [b"dGhlIHNhbXBsZSBub25jZQ==", b"x" * 24, b"abc"]
    raw = np.frombuffer(b"".join(keys), np.uint8).copy()
    off = np.array([0, 24, 10, 51], dtype=np.int64)        # key 1: [24, 10)
    d_keys = torch.from_numpy(raw).cuda()
    d_off = torch.from_numpy(off).cuda()
    buf = torch.full((3 * cfws.WS_ACCEPT_SLOT + 16,), 0xEE, dtype=torch.uint8, device="cuda")
    out = buf[slot_shift:]
    assert cfws.lib().cfws_ws_accept_keys_batch(d_keys.data_ptr(), d_off.data_ptr(), 3,
                                                out.data_ptr(), None) == 0
    h = out[:3 * cfws.WS_ACCEPT_SLOT].cpu().numpy().reshape(3, -1)
    assert bytes(h[0, :28]).decode() == O.ws_accept_key(keys[0])
    assert h[0, 28] == 0
    assert not h[1].any()
    assert bytes(h[2, :28]).decode() == O.ws_accept_key(bytes(raw[10:51]))
