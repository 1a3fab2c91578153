"""Randomised parity sweep and API edge cases on the MI355X.

* 48 seeds of small mixed batches through serialize and deserialize: frame
  sizes from 0 B to 70 KB weighted to the sizes that hit the edge paths
  (0-20 B frames, several frames per 16-byte chunk, every header form),
  unaligned payload offsets, random fin/opcode/mask, random capacities,
  alignments and reassembly; deserialize indices include frame starts,
  mid-frame positions and positions past the end. Every result equals the
  oracle's.
* Empty batches and the error codes of the batch ABI.
"""
import random

import numpy as np
import pytest

import oracle as O
from conftest import gpu_present

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not gpu_present(), reason="needs the MI355X")]

torch = pytest.importorskip("torch")

from coldforce_amd import cfws  # noqa: E402
from test_gpu_batch import check_deserialize, check_serialize, random_desc  # noqa: E402

FUZZ_SIZES = [0, 0, 1, 2, 3, 5, 7, 11, 13, 14, 15, 16, 17, 20, 31, 33, 100, 125, 126, 127, 500,
              4095, 4096, 4097, 20000, 65535, 65536, 70000]


@pytest.fixture(scope="module", autouse=True)
def device():
    cfws.init()


@pytest.mark.parametrize("seed", range(48))
def test_fuzz_serialize_deserialize(seed):
    rng = random.Random(1000 + seed)
    payload = O.fill_splitmix(300000, seed, 0)
    n = rng.choice([1, 2, 3, 7, 64, 257, 1000, 2500])
    desc = random_desc(rng, n, payload.size, sizes=FUZZ_SIZES)
    slack = rng.choice([0, 16, 4096])
    wire, total = check_serialize(payload, desc, slack=slack, plan_execute=seed % 2 == 1)
    wire = wire[:total].copy()
    starts, _ = O.index_frames(wire, n + 1)
    idx = list(starts)
    for _ in range(rng.randrange(0, 20)):            # mid-frame and past-the-end indices
        idx.insert(rng.randrange(len(idx) + 1), rng.randrange(0, total + 40))
    idx = np.array(sorted(idx) if rng.random() < 0.5 else idx, dtype=np.uint64)
    align = rng.choice([1, 2, 16, 64, 4096])
    flags = O.DESERIALIZE_REASSEMBLE if rng.random() < 0.3 else 0
    full = int(total) + 4096 * (len(idx) + 1)
    cap = rng.choice([full, full, total // 2 + 1, 17])
    check_deserialize(wire, idx, align=align, capacity=cap, flags=flags,
                      max_payload=rng.choice([O.DEFAULT_MAX_PAYLOAD, 1000, 0]),
                      plan_execute=seed % 3 == 0)


def test_empty_batches():
    dev = torch.device("cuda")
    wire = torch.zeros(64, dtype=torch.uint8, device=dev)
    pay = torch.zeros(64, dtype=torch.uint8, device=dev)
    d = torch.zeros((0, 32), dtype=torch.uint8, device=dev)
    assert int(cfws.serialize(pay, d, wire).item()) == 0
    idx = torch.zeros(0, dtype=torch.int64, device=dev)
    _, st, tot = cfws.deserialize(wire, 64, idx, pay)
    assert int(tot.item()) == 0 and st.numel() == 0
    e = torch.zeros(0, dtype=torch.int64, device=dev)
    starts, first, consumed, stop, total = cfws.index_frames_batch(wire, e, e)
    assert total == 0
    assert cfws.ws_accept_keys([]) == []


def test_error_codes():
    L = cfws.lib()
    dev = torch.device("cuda")
    s = torch.cuda.current_stream().cuda_stream
    pay = torch.zeros(4096, dtype=torch.uint8, device=dev)
    wire = torch.zeros(4096, dtype=torch.uint8, device=dev)
    desc = cfws.desc_to_device(np.zeros(4, dtype=cfws.DESC_DTYPE), dev)
    tot = torch.zeros(1, dtype=torch.int64, device=dev)
    ws = cfws.workspace(4, 4096, dev)
    # workspace too small
    assert L.cfws_serialize_batch(pay.data_ptr(), desc.data_ptr(), 4, wire.data_ptr(), 4096,
                                  tot.data_ptr(), ws.data_ptr(), 8, s) == cfws.ERROR_WORKSPACE
    # alignment must be a power of two <= 4096; flags must be known
    idx = torch.zeros(4, dtype=torch.int64, device=dev)
    st = torch.zeros(4, dtype=torch.int32, device=dev)
    for align, flags in ((3, 0), (8192, 0), (16, 4)):
        rc = L.cfws_deserialize_batch(wire.data_ptr(), 4096, idx.data_ptr(), 4,
                                      O.DEFAULT_MAX_PAYLOAD, align, flags, desc.data_ptr(),
                                      st.data_ptr(), pay.data_ptr(), 4096, tot.data_ptr(),
                                      ws.data_ptr(), ws.numel(), s)
        assert rc == cfws.ERROR_INVALID_ARGUMENT, (align, flags)
    # execute on arenas that are not 16-byte aligned
    rc = L.cfws_serialize_execute(pay.data_ptr() + 1, desc.data_ptr(), 4, wire.data_ptr(), 4096,
                                  ws.data_ptr(), s)
    assert rc == cfws.ERROR_INVALID_ARGUMENT
    # HTTP/2 max_frame_size beyond 2^24 - 1
    h2 = torch.zeros(8192, dtype=torch.uint8, device=dev)
    wsh = torch.zeros(cfws.lib().cfws_h2_serialize_workspace_size(4, 4096, 8192, 1 << 24),
                      dtype=torch.uint8, device=dev)
    rc = L.cfws_h2_serialize_batch(pay.data_ptr(), desc.data_ptr(), 4, 1, 1 << 24, wire.data_ptr(),
                                   4096, h2.data_ptr(), 8192, tot.data_ptr(), wsh.data_ptr(),
                                   wsh.numel(), s)
    assert rc == cfws.ERROR_INVALID_ARGUMENT
    assert cfws.lib().cfws_last_error()
