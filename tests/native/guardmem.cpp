// TEST INFRASTRUCTURE ONLY -- device buffers with unmapped guard ranges.
//
// A buffer is placed inside an address range reserved with
// hipMemAddressReserve, with physical memory mapped only under the buffer's
// own granules: the granules before and after it are reserved but never
// mapped. A kernel that reads or writes one byte past the buffer's end (or
// before its start) then faults at once, wherever the caching allocator would
// otherwise have had another live block next to it. The round-4 fault
// (hipErrorIllegalAddress in the first form of the fused deserialize) showed
// only on arenas whose end fell on an unmapped page -- the bench's exact
// 4 GiB-class arenas -- and passed on the tests' padded ones; these buffers
// make every test arena such an arena (tests/test_gpu_guard.py).
//
// flush_end = 1: the buffer's round16(len) end is the last mapped byte (the
//                library reads whole aligned 16-byte blocks: its arenas are
//                16-aligned and readable up to round16(size));
// flush_end = 0: the buffer starts at the first mapped byte.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <unordered_map>

namespace {

struct Guarded {
    void* base;       // reservation
    size_t reserved;  // bytes reserved
    void* mapped;     // first mapped byte
    size_t mapped_n;  // bytes mapped
    hipMemGenericAllocationHandle_t h;
};

std::mutex g_mu;
std::unordered_map<uintptr_t, Guarded> g_live;
char g_err[256];

int fail(const char* what, hipError_t e)
{
    snprintf(g_err, sizeof g_err, "%s: %s", what, hipGetErrorString(e));
    return -1;
}

}  // namespace

extern "C" {

const char* guard_last_error() { return g_err; }

// 1 when the current device supports HIP virtual memory management
int guard_supported()
{
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeVirtualMemoryManagementSupported, dev) != hipSuccess)
        return 0;
    return v != 0;
}

// Returns the buffer's device address (0 on failure, guard_last_error()).
uint64_t guard_alloc(uint64_t len, int flush_end)
{
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return fail("hipGetDevice", e), 0;
    hipMemAllocationProp prop = {};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = dev;
    size_t gran = 0;
    e = hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityMinimum);
    if (e != hipSuccess || gran == 0) return fail("hipMemGetAllocationGranularity", e), 0;
    const uint64_t len16 = (len + 15) & ~uint64_t(15);
    const size_t mapped_n = len16 == 0 ? gran : (len16 + gran - 1) / gran * gran;
    // guards of at least 2 MiB on both sides (a large page either way)
    const size_t guard = gran >= (2u << 20) ? gran : (2u << 20) / gran * gran;
    Guarded g = {};
    g.reserved = mapped_n + 2 * guard;
    g.mapped_n = mapped_n;
    e = hipMemAddressReserve(&g.base, g.reserved, guard, nullptr, 0);
    if (e != hipSuccess) return fail("hipMemAddressReserve", e), 0;
    g.mapped = static_cast<char*>(g.base) + guard;
    e = hipMemCreate(&g.h, mapped_n, &prop, 0);
    if (e != hipSuccess) {
        (void)hipMemAddressFree(g.base, g.reserved);
        return fail("hipMemCreate", e), 0;
    }
    e = hipMemMap(g.mapped, mapped_n, 0, g.h, 0);
    if (e != hipSuccess) {
        (void)hipMemRelease(g.h);
        (void)hipMemAddressFree(g.base, g.reserved);
        return fail("hipMemMap", e), 0;
    }
    hipMemAccessDesc acc = {};
    acc.location = prop.location;
    acc.flags = hipMemAccessFlagsProtReadWrite;
    e = hipMemSetAccess(g.mapped, mapped_n, &acc, 1);
    if (e != hipSuccess) {
        (void)hipMemUnmap(g.mapped, mapped_n);
        (void)hipMemRelease(g.h);
        (void)hipMemAddressFree(g.base, g.reserved);
        return fail("hipMemSetAccess", e), 0;
    }
    char* p = static_cast<char*>(g.mapped) + (flush_end ? mapped_n - len16 : 0);
    std::lock_guard<std::mutex> lk(g_mu);
    g_live[reinterpret_cast<uintptr_t>(p)] = g;
    return reinterpret_cast<uint64_t>(p);
}

int guard_free(uint64_t ptr)
{
    Guarded g;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        auto it = g_live.find(static_cast<uintptr_t>(ptr));
        if (it == g_live.end()) return -1;
        g = it->second;
        g_live.erase(it);
    }
    hipError_t e = hipDeviceSynchronize();
    if (e != hipSuccess) return fail("hipDeviceSynchronize", e);
    if ((e = hipMemUnmap(g.mapped, g.mapped_n)) != hipSuccess) return fail("hipMemUnmap", e);
    if ((e = hipMemRelease(g.h)) != hipSuccess) return fail("hipMemRelease", e);
    // GUARD_FREE_RANGES=1: release the range too (round 6's re-check of the
    // finding below: tools/vmm_remap_probe.hip, profiles/r06/vmm/)
    static const bool free_ranges = [] {
        const char* v = getenv("GUARD_FREE_RANGES");
        return v && v[0] == '1';
    }();
    if (free_ranges && (e = hipMemAddressFree(g.base, g.reserved)) != hipSuccess)
        return fail("hipMemAddressFree", e);
    // By default the address range stays reserved for the rest of the
    // process: on this stack (ROCm 7.2, gfx950) new physical memory mapped at
    // an address that earlier mapped other, still-allocated memory is read
    // through the old translation, by kernels and by hipMemcpy. Round 6
    // reproduced it with a plain copy kernel and no library code
    // (tools/vmm_remap_probe.hip, profiles/r06/vmm/); with GUARD_FREE_RANGES=1
    // tests/test_gpu_guard.py fails on its second test. Never reusing a range
    // keeps every buffer's first kernel on fresh addresses.
    return 0;
}

// plain synchronous copies and fills, host <-> guarded device memory
int guard_copy(uint64_t dst, uint64_t src, uint64_t n)
{
    hipError_t e = hipMemcpy(reinterpret_cast<void*>(dst), reinterpret_cast<const void*>(src), n,
                             hipMemcpyDefault);
    return e == hipSuccess ? 0 : fail("hipMemcpy", e);
}

int guard_fill(uint64_t dst, int byte, uint64_t n)
{
    hipError_t e = hipMemset(reinterpret_cast<void*>(dst), byte, n);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    return e == hipSuccess ? 0 : fail("hipMemset", e);
}

}  // extern "C"
