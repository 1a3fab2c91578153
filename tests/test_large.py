"""Maximum sizes on one MI355X (-m gpu):

* config 4's per-GPU shard: shard 0 of the 8 M x 64 KiB batch cut in 8
  (1,048,576 frames, 64 GiB payload + 64 GiB wire + 64 GiB unmasked copy
  resident at once), 1,024 sampled frames checked against the oracle
  (SURVEY.md 8(d) config 4), the round trip checked whole;
* one masked frame larger than 4 GiB (127 + 64-bit length, 32-bit
  overflow of every size and offset), with and without the receive limit.
"""
import numpy as np
import pytest

import oracle as O
from conftest import gpu_present

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not gpu_present(), reason="needs the MI355X")]

torch = pytest.importorskip("torch")

from coldforce_amd import cfws, shard  # noqa: E402
from coldforce_amd import workloads as W  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def device():
    cfws.init()


def test_config4_shard_64gib():
    F, fs, shards, rank = 1 << 20, 65536, 8, 0
    desc_np, byte_base = shard.uniform_shard(F, fs, 4, rank, shards)
    dev = torch.device("cuda")
    payload = torch.empty(F * fs, dtype=torch.uint8, device=dev)
    cfws.fill_splitmix(payload, 0x5EED0004, byte_base)
    offs, wire_total = W.wire_layout(desc_np)
    wire = torch.empty(W.round16(wire_total), dtype=torch.uint8, device=dev)
    d_t = cfws.desc_to_device(desc_np, dev)
    tot = cfws.serialize(payload, d_t, wire)
    torch.cuda.synchronize()
    assert int(tot.item()) == wire_total
    # 1,024 sampled frames vs the oracle
    rng = np.random.default_rng(4)
    for f in np.sort(rng.choice(F, 1024, replace=False)):
        p = payload[f * fs:(f + 1) * fs].cpu().numpy().tobytes()
        exp = O.serialize_keyed(True, 2, True, int(desc_np["mask_key"][f]), p)
        got = wire[int(offs[f]):int(offs[f]) + len(exp)].cpu().numpy().tobytes()
        assert got == exp, f
    # the whole round trip
    back = torch.empty(F * fs + 64, dtype=torch.uint8, device=dev)
    idx = torch.from_numpy(offs.astype(np.int64)).to(dev)
    desc_de, st, tot_de = cfws.deserialize(wire, wire_total, idx, back)
    torch.cuda.synchronize()
    assert int(tot_de.item()) == F * fs
    assert bool((st == 0).all().item())
    assert torch.equal(back[:F * fs], payload)


def test_single_masked_frame_over_4gib():
    n = (9 << 29) + 3                                 # 4.5 GiB + 3 B
    dev = torch.device("cuda")
    payload = torch.empty(n + 13, dtype=torch.uint8, device=dev)
    cfws.fill_splitmix(payload, 0x5EED4444, 0)
    key = 0x9A3F17C5
    d = np.zeros(1, dtype=cfws.DESC_DTYPE)
    d[0] = (0, 0, n, key, 1, 2, 1, 0)
    hs = O.header_size(n, True)
    assert hs == 14
    wire = torch.empty(W.round16(n + hs) + 16, dtype=torch.uint8, device=dev)
    d_t = cfws.desc_to_device(d, dev)
    assert int(cfws.serialize(payload, d_t, wire).item()) == n + hs
    exp_hdr = O.serialize_keyed(True, 2, True, key, b"")[:2]
    exp_hdr = bytes([exp_hdr[0], 0xFF]) + n.to_bytes(8, "big") + key.to_bytes(4, "little")
    assert wire[:hs].cpu().numpy().tobytes() == exp_hdr
    kb = torch.tensor(list(key.to_bytes(4, "little")), dtype=torch.uint8, device=dev)
    kb = kb.repeat(n // 4 + 1)[:n]
    assert torch.equal(wire[hs:hs + n], payload[:n] ^ kb)
    del kb
    # receive: over the default 32 MiB limit -> DATA_TOO_BIG, nothing copied
    back = torch.zeros(n + 64, dtype=torch.uint8, device=dev)
    idx = torch.zeros(1, dtype=torch.int64, device=dev)
    _, st, tot = cfws.deserialize(wire, n + hs, idx, back)
    torch.cuda.synchronize()
    assert int(st[0].item()) == -7005 and int(tot.item()) == 0
    # with the limit raised: the payload comes back
    _, st, tot = cfws.deserialize(wire, n + hs, idx, back, max_payload=1 << 40, align=1)
    torch.cuda.synchronize()
    assert int(st[0].item()) == 0 and int(tot.item()) == n
    assert torch.equal(back[:n], payload[:n])
