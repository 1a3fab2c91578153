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
