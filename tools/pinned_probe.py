"""Which host allocations the device can address directly: torch's pinned
tensors and hipHostMalloc memory, via hipHostGetDevicePointer /
hipHostGetFlags (queries only, no kernel touches the memory). Prints JSON."""
import ctypes as C
import json

import torch

torch.cuda.init()
hip = C.CDLL("libamdhip64.so")
hip.hipHostGetDevicePointer.argtypes = [C.POINTER(C.c_void_p), C.c_void_p, C.c_uint]
hip.hipHostGetFlags.argtypes = [C.POINTER(C.c_uint), C.c_void_p]
hip.hipHostMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t, C.c_uint]
hip.hipHostFree.argtypes = [C.c_void_p]


def query(ptr):
    dp = C.c_void_p()
    rc = hip.hipHostGetDevicePointer(C.byref(dp), C.c_void_p(ptr), 0)
    fl = C.c_uint()
    rc2 = hip.hipHostGetFlags(C.byref(fl), C.c_void_p(ptr))
    return {"ptr": hex(ptr), "devptr_rc": rc, "devptr": hex(dp.value or 0),
            "same": (dp.value or 0) == ptr, "flags_rc": rc2, "flags": fl.value}


out = {}
t = torch.empty(1 << 24, dtype=torch.uint8, pin_memory=True)
out["torch_pinned"] = query(t.data_ptr())
out["torch_pinned_offset"] = query(t.data_ptr() + 12345)
h = C.c_void_p()
print(hip.hipHostMalloc(C.byref(h), 1 << 24, 0x2))    # hipHostMallocMapped
out["hipHostMalloc_mapped"] = query(h.value)
out["hipHostMalloc_mapped_offset"] = query(h.value + 777)
print(json.dumps(out))
