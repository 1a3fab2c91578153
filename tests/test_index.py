"""Receive-buffer frame indexing: the walk of
co_ws_server.c:107-169 over connection streams.

* host form (cfws_index_frames, pure host code) against the reference's own
  receive loop on the committed streams (tests/golden/index_cases.json);
* device form (cfws_index_frames_batch, -m gpu) on every golden stream at
  once -- one connection each in one arena -- and on a config-3 Zipf wire
  cut into thousands of connections, against the oracle, then fed to
  cfws_deserialize_batch.
"""
import numpy as np
import pytest

import oracle as O
from conftest import golden

from coldforce_amd import cfws


def _cases():
    g = golden("index_cases.json")
    blobs = {k: bytes.fromhex(v) for k, v in g["blobs"].items()}
    return [(c, blobs[c["blob"]][:c["size"]]) for c in g["cases"]]


def test_host_index_matches_reference_receive_loop():
    for c, data in _cases():
        st, consumed, stop = cfws.index_frames(np.frombuffer(data, np.uint8), c["begin"],
                                               len(data), c["max_payload"])
        assert [int(x) for x in st] == c["starts"], c["name"]
        assert (consumed, stop) == (c["consumed"], c["stop"]), c["name"]


def test_host_index_full_resumes():
    """A full `starts` stops before the next COMPLETE frame; resuming from
    *consumed walks the rest exactly as one uninterrupted walk."""
    c, data = next((c, d) for c, d in _cases() if c["name"] == "tiny frames")
    buf = np.frombuffer(data, np.uint8)
    got, pos = [], 0
    while True:
        st, pos2, stop = cfws.index_frames(buf, pos, len(data), max_starts=37)
        got += [int(x) for x in st]
        pos = pos2
        if stop != cfws.INDEX_FULL:
            break
        assert len(st) == 37
    assert got == c["starts"] and pos == c["consumed"] and stop == c["stop"]


def test_host_index_random_vs_oracle():
    rng = np.random.default_rng(5)
    for t in range(40):
        frames = [O.serialize_keyed(bool(rng.random() < .7), int(rng.integers(16)),
                                    bool(rng.random() < .5), int(rng.integers(1 << 32)),
                                    rng.bytes(int(rng.choice([0, 1, 125, 126, 300, 70000]))))
                  for _ in range(int(rng.integers(1, 30)))]
        w = b"".join(frames)
        w = w[:int(rng.integers(0, len(w) + 1))] if t % 2 else w
        if t % 5 == 4 and w:
            w = w[:len(w) // 2] + b"\x7f\x00" + w[len(w) // 2:]       # opcode 0x7f: -7001
        buf = np.frombuffer(w, np.uint8)
        exp = O.index_stream(buf, 0, len(w))
        got = cfws.index_frames(buf, 0, len(w))
        assert np.array_equal(got[0], exp[0]) and got[1:] == exp[1:]


# ---- device ------------------------------------------------------------------

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def device():
    cfws.init()
    return torch.device("cuda")


def _arena(streams, device):
    """Streams back to back in one device arena (connection c = its slice)."""
    offs = np.zeros(len(streams) + 1, dtype=np.int64)
    offs[1:] = np.cumsum([len(s) for s in streams])
    raw = np.frombuffer(b"".join(streams) or b"\0", np.uint8).copy()
    return torch.from_numpy(raw).to(device), offs


@pytest.mark.gpu
def test_device_index_golden_streams(device):
    cases = _cases()
    buf, offs = _arena([d for _, d in cases], device)
    begin = torch.tensor([offs[i] + c["begin"] for i, (c, _) in enumerate(cases)],
                         dtype=torch.int64, device=device)
    end = torch.tensor(offs[1:], dtype=torch.int64, device=device)
    mp = {c["max_payload"] for c, _ in cases}
    for max_payload in mp:   # one launch per payload limit (the limit is global, co_ws_config.c)
        sel = [i for i, (c, _) in enumerate(cases) if c["max_payload"] == max_payload]
        idx = torch.tensor(sel, dtype=torch.int64, device=device)
        starts, first, consumed, stop, total = cfws.index_frames_batch(
            buf, begin[idx], end[idx], max_payload)
        starts, first = starts.cpu().numpy(), first.cpu().numpy()
        consumed, stop = consumed.cpu().numpy(), stop.cpu().numpy()
        assert total == sum(len(cases[i][0]["starts"]) for i in sel)
        for j, i in enumerate(sel):
            c = cases[i][0]
            k = len(c["starts"])
            got = starts[first[j]:first[j] + k] - offs[i]
            assert [int(x) for x in got] == c["starts"], c["name"]
            assert consumed[j] - offs[i] == c["consumed"] and stop[j] == c["stop"], c["name"]


@pytest.mark.gpu
def test_device_index_zipf_connections_then_deserialize(device):
    """A config-3-shaped Zipf wire (8 MiB) cut into 3,000 connections at
    random byte positions (so most end mid-frame and some start mid-frame):
    indexing equals the oracle's per connection, and the indexed frames
    deserialize bit-exactly."""
    from coldforce_amd import workloads as W
    desc, msgs = W.zipf_batch(8 << 20, 0x5EED0033, 33, ping_every=3)
    payload = O.fill_splitmix(int(msgs["arena_bytes"]) + 16, 0x33, 0)
    wire, _ = O.serialize_batch(payload, desc.view(O.DESC_DTYPE))
    rng = np.random.default_rng(11)
    cuts = np.sort(rng.choice(len(wire), 2999, replace=False))
    bounds = np.concatenate([[0], cuts, [len(wire)]]).astype(np.int64)
    # connection c starts at a frame start when one lies inside it: the
    # receive index of a live connection is always a frame boundary
    fstarts = desc["wire_off"].astype(np.int64)
    k = np.searchsorted(fstarts, bounds[:-1])
    begin_np = np.where(k < len(fstarts), fstarts[np.minimum(k, len(fstarts) - 1)], bounds[1:])
    begin_np = np.minimum(begin_np, bounds[1:])
    end_np = bounds[1:]
    buf = torch.from_numpy(wire.copy()).to(device)
    starts, first, consumed, stop, total = cfws.index_frames_batch(
        buf, torch.from_numpy(begin_np).to(device), torch.from_numpy(end_np).to(device))
    starts, first = starts.cpu().numpy(), first.cpu().numpy()
    consumed, stop = consumed.cpu().numpy(), stop.cpu().numpy()
    all_exp = []
    for c in range(len(end_np)):
        e_st, e_con, e_stop = O.index_stream(wire, int(begin_np[c]), int(end_np[c]))
        n_c = len(e_st)
        assert np.array_equal(starts[first[c]:first[c] + n_c].astype(np.uint64), e_st), c
        assert consumed[c] == e_con and stop[c] == e_stop, c
        all_exp.append((e_st, int(end_np[c])))
    assert total == sum(len(s) for s, _ in all_exp)
    # the indexed frames through the batch deserializer (each is COMPLETE)
    idx = np.concatenate([s for s, _ in all_exp]).astype(np.uint64)
    exp_out, exp_d, exp_st, exp_tot = O.deserialize_batch(wire, idx, align=16)
    out = torch.zeros(exp_tot + 64, dtype=torch.uint8, device=device)
    d_t, st_t, tot_t = cfws.deserialize(buf, len(wire), torch.from_numpy(idx.astype(np.int64)).to(device),
                                        out, align=16)
    assert int(tot_t.item()) == exp_tot and (exp_st == 0).all()
    assert np.array_equal(st_t.cpu().numpy(), exp_st)
    assert np.array_equal(out[:exp_tot].cpu().numpy(), exp_out[:exp_tot])


@pytest.mark.gpu
@pytest.mark.parametrize("cap_cut", [False, True])
def test_device_index_long_connections(device, cap_cut):
    """Connections of 1, 63, 64, 65, 130 and 700 small frames (the device walk
    keeps 64 starts per connection and walks on past them only where there
    are more), some ending inside a frame or on an invalid one; with
    cap_cut the starts capacity ends inside a long connection's starts."""
    import random
    rng = random.Random(65)
    streams, expect = [], []
    for n in (1, 63, 64, 65, 130, 700, 64, 200):
        frames = [O.serialize_keyed(True, rng.choice([1, 2, 9]), rng.random() < .7, rng.getrandbits(32),
                                    rng.randbytes(rng.randrange(0, 40))) for _ in range(n)]
        s = b"".join(frames)
        tail = rng.choice([b"", b"\x82", b"\x82\xfe\x01", b"\xf2\x00"])   # cut frame / RSV junk
        streams.append(s + tail)
    buf, offs = _arena(streams, device)
    host = np.frombuffer(b"".join(streams), np.uint8)
    begin = torch.tensor(offs[:-1], dtype=torch.int64, device=device)
    end = torch.tensor(offs[1:], dtype=torch.int64, device=device)
    exp = [O.index_stream(host, int(offs[i]), int(offs[i + 1])) for i in range(len(streams))]
    n_all = sum(len(e[0]) for e in exp)
    cap = n_all - 100 if cap_cut else n_all + 8
    starts_t = torch.full((max(cap, 1),), -1, dtype=torch.int64, device=device)
    starts, first, consumed, stop, total = cfws.index_frames_batch(buf, begin, end, starts_t=starts_t)
    starts, first = starts.cpu().numpy(), first.cpu().numpy()
    consumed, stop = consumed.cpu().numpy(), stop.cpu().numpy()
    assert total == n_all
    allexp = np.concatenate([e[0] for e in exp]).astype(np.int64)
    assert np.array_equal(starts[:min(cap, n_all)], allexp[:min(cap, n_all)])
    for i, (e_st, e_con, e_stop) in enumerate(exp):
        assert consumed[i] == e_con and stop[i] == e_stop, i
        assert first[i] == sum(len(x[0]) for x in exp[:i])
