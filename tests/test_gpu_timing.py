"""cfws_time_next_pass (include/cfws.h): the pair belongs to the calling
thread's NEXT public batch call. That call takes it on entry and records it
around its timed pass (the small single-launch paths included); an error
return, an empty batch or a call with no timed pass drops it, so it never
reaches a later call. bench.py's per-kernel times rest on this."""
import pytest

torch = pytest.importorskip("torch")

from coldforce_amd import cfws  # noqa: E402
from coldforce_amd import workloads as W  # noqa: E402

pytestmark = pytest.mark.gpu


def _batch(F, fs, seed=11):
    desc = W.uniform_batch(F, fs, seed)
    payload = torch.empty(W.round16(F * fs) + 16, dtype=torch.uint8, device="cuda")
    cfws.fill_splitmix(payload, 0x77, 0)
    _, wtotal = W.wire_layout(desc)
    wire = torch.empty(W.round16(wtotal) + 16, dtype=torch.uint8, device="cuda")
    return payload, cfws.desc_to_device(desc, "cuda"), wire


def _recorded(a, b) -> bool:
    try:
        a.elapsed_time(b)
        return True
    except cfws.CodecError:
        return False


def test_pair_recorded_by_the_small_path():
    payload, d, wire = _batch(16, 100)             # one launch (serialize_small_kernel)
    a, b = cfws.TimingEvent(), cfws.TimingEvent()
    cfws.time_next_pass(a, b)
    cfws.serialize(payload, d, wire)
    torch.cuda.synchronize()
    assert a.elapsed_time(b) >= 0.0


def test_pair_recorded_once_by_the_execute():
    payload, d, wire = _batch(4096, 4096)          # plan + execute
    a, b = cfws.TimingEvent(), cfws.TimingEvent()
    cfws.time_next_pass(a, b)
    cfws.serialize(payload, d, wire)
    torch.cuda.synchronize()
    t1 = a.elapsed_time(b)
    for _ in range(3):                             # later calls leave the pair alone
        cfws.serialize(payload, d, wire)
    torch.cuda.synchronize()
    assert a.elapsed_time(b) == t1


@pytest.mark.parametrize("how", ["error", "empty", "untimed"])
def test_pair_dropped_by_the_call_that_took_it(how):
    payload, d, wire = _batch(4096, 4096)
    a, b = cfws.TimingEvent(), cfws.TimingEvent()
    cfws.time_next_pass(a, b)
    if how == "error":                             # workspace too small: an error return
        tiny = torch.empty(16, dtype=torch.uint8, device="cuda")
        with pytest.raises(cfws.CodecError):
            cfws.serialize(payload, d, wire, ws_t=tiny)
    elif how == "empty":                           # n == 0: nothing launched
        cfws.serialize(payload, d[:0], wire)
    else:                                          # a call with no timed pass
        cfws.device_copy(payload, wire, 4096)
    cfws.serialize(payload, d, wire)               # would record a carried-over pair
    torch.cuda.synchronize()
    assert not _recorded(a, b)


def test_pair_around_the_fused_and_slot_receives():
    payload, d, wire = _batch(8192, 240)           # small frames: the fused plan + copy
    tot = cfws.serialize(payload, d, wire)
    torch.cuda.synchronize()
    import numpy as np
    desc = cfws.desc_from_device(d)
    idx = torch.from_numpy(desc["wire_off"].astype(np.int64)).to("cuda")
    back = torch.empty(8192 * 256 + 64, dtype=torch.uint8, device="cuda")
    for recv in ("fused", "slots"):
        a, b = cfws.TimingEvent(), cfws.TimingEvent()
        cfws.time_next_pass(a, b)
        if recv == "fused":
            _, st, _ = cfws.deserialize(wire, int(tot.item()), idx, back)
        else:
            _, st, _ = cfws.deserialize_slots(wire, int(tot.item()), idx, back, 256)
        torch.cuda.synchronize()
        assert a.elapsed_time(b) >= 0.0 and bool((st == 0).all())
