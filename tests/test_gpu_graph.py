"""HIP graphs of the batch codec (cfws_graph_*, coldforce_amd/csrc/cfws_graph.cpp):
a captured serialize / deserialize replayed over the same arenas equals the
oracle for whatever the descriptors and bytes hold at launch time -- new
payload bytes, new keys, new frame sizes, a new receive buffer."""
import random

import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from coldforce_amd import cfws  # noqa: E402
from coldforce_amd import workloads as W  # noqa: E402

PAYLOAD = 1 << 20


@pytest.fixture(scope="module", autouse=True)
def device():
    cfws.init()


def random_desc(rng, n):
    d = np.zeros(n, dtype=cfws.DESC_DTYPE)
    for i in range(n):
        sz = rng.choice([0, 1, 5, 125, 126, 1000, 4097, 20000, 65536])
        d[i] = (rng.randrange(0, PAYLOAD - sz), 0, sz, rng.getrandbits(32), rng.random() < .7,
                rng.choice([0, 1, 2, 9]), rng.random() < .6, 0)
    return d


def test_graph_serialize_replays_new_contents():
    rng = random.Random(5)
    n = 300
    pay = torch.empty(PAYLOAD, dtype=torch.uint8, device="cuda")
    d_t = torch.empty((n, 32), dtype=torch.uint8, device="cuda")
    cap = n * (65536 + 14) + 64
    wire = torch.empty(cap, dtype=torch.uint8, device="cuda")
    ws = cfws.workspace(n, cap)
    tot = torch.zeros(1, dtype=torch.int64, device="cuda")
    g = cfws.Graph.serialize(pay, d_t, wire, ws, tot)
    for it in range(3):                    # new bytes, keys, sizes, flags each launch
        payload = O.fill_splitmix(PAYLOAD, 100 + it, 0)
        d = random_desc(rng, n)
        pay.copy_(torch.from_numpy(payload))
        d_t.copy_(cfws.desc_to_device(d))
        g.launch()
        torch.cuda.synchronize()
        exp, exp_d = O.serialize_batch(payload, d.view(O.DESC_DTYPE))
        assert int(tot.item()) == len(exp)
        assert np.array_equal(wire[:len(exp)].cpu().numpy(), exp)
        got_d = cfws.desc_from_device(d_t)
        assert np.array_equal(got_d["wire_off"], exp_d["wire_off"])
        assert np.array_equal(got_d["header_size"], exp_d["header_size"])
    g.close()


def test_graph_deserialize_replays_new_buffer_on_another_stream():
    rng = random.Random(6)
    n = 400
    cap_w = n * (40000 + 14) + 64
    wire = torch.zeros(cap_w, dtype=torch.uint8, device="cuda")
    idx = torch.zeros(n, dtype=torch.int64, device="cuda")
    d_t = torch.empty((n, 32), dtype=torch.uint8, device="cuda")
    st_t = torch.empty(n, dtype=torch.int32, device="cuda")
    out = torch.empty(cap_w + 16 * n, dtype=torch.uint8, device="cuda")
    ws = cfws.workspace(n, out.numel())
    tot = torch.zeros(1, dtype=torch.int64, device="cuda")
    g = cfws.Graph.deserialize(wire, cap_w, idx, d_t, st_t, out, ws, tot, align=16)
    side = torch.cuda.Stream()
    for it in range(3):
        frames = [O.serialize_keyed(rng.random() < .7, rng.randrange(16), rng.random() < .6,
                                    rng.getrandbits(32),
                                    rng.randbytes(rng.choice([0, 7, 125, 126, 3000, 40000])))
                  for _ in range(n)]
        raw = np.frombuffer(b"".join(frames), np.uint8)
        starts, _ = O.index_frames(raw, n)
        # the captured wire size is the arena's; bytes past the frames are
        # zero and not indexed
        buf = np.zeros(cap_w, np.uint8)
        buf[:len(raw)] = raw
        wire.copy_(torch.from_numpy(buf))
        idx.copy_(torch.from_numpy(starts.astype(np.int64)))
        torch.cuda.synchronize()
        g.launch(stream=side)
        side.synchronize()
        e_out, e_d, e_st, e_tot = O.deserialize_batch(buf, starts, align=16, capacity=out.numel())
        assert int(tot.item()) == e_tot
        assert np.array_equal(st_t.cpu().numpy(), e_st)
        got = cfws.desc_from_device(d_t)
        for f in ("payload_off", "payload_size", "mask_key", "fin", "opcode", "mask", "header_size"):
            assert np.array_equal(got[f], e_d[f]), f
        assert np.array_equal(out[:e_tot].cpu().numpy(), e_out[:e_tot])
    g.close()


def test_graph_round_trip_config2_shape():
    """1,024 x 64 KiB: a serialize graph then a deserialize graph over the
    wire it wrote, replayed; the payload comes back bit-exact."""
    n, fs = 1024, 65536
    desc = W.uniform_batch(n, fs, 2)
    offs, wtotal = W.wire_layout(desc)
    pay = torch.empty(n * fs, dtype=torch.uint8, device="cuda")
    cfws.fill_splitmix(pay, 0x5EED0002)
    d_t = cfws.desc_to_device(desc)
    wire = torch.empty(W.round16(wtotal), dtype=torch.uint8, device="cuda")
    back = torch.empty(n * fs + 64, dtype=torch.uint8, device="cuda")
    idx = torch.from_numpy(offs.astype(np.int64)).cuda()
    dd = torch.empty((n, 32), dtype=torch.uint8, device="cuda")
    st_t = torch.empty(n, dtype=torch.int32, device="cuda")
    t1 = torch.zeros(1, dtype=torch.int64, device="cuda")
    t2 = torch.zeros(1, dtype=torch.int64, device="cuda")
    gs = cfws.Graph.serialize(pay, d_t, wire, cfws.workspace(n, wire.numel()), t1)
    gd = cfws.Graph.deserialize(wire, wtotal, idx, dd, st_t, back, cfws.workspace(n, back.numel()), t2)
    for _ in range(3):
        back.zero_()
        gs.launch()
        gd.launch()
        torch.cuda.synchronize()
        assert int(t1.item()) == wtotal and int(t2.item()) == n * fs
        assert bool((st_t == 0).all()) and torch.equal(back[:n * fs], pay)
    gs.close()
    gd.close()
