// vmm_remap_probe.hip -- does a kernel see the new memory behind a virtual
// address range that was freed (hipMemAddressFree) and handed out again?
//
// Standalone (no libcfws): a plain 16-byte copy kernel over a buffer mapped
// with the HIP virtual-memory API, in the sequence the round-5 guard
// allocator used (tests/native/guardmem.cpp): reserve a range with 2 MiB
// guards, create + map physical memory under the middle, set access, fill it
// with hipMemcpy, run the kernel, then unmap + release + free the range. The
// next trial reserves again (the runtime usually returns the same range),
// maps NEW physical memory, fills it with a different pattern and runs the
// kernel again. Each trial prints a JSON line: whether the range was reused,
// how many bytes the kernel read wrong, and how many of those equal the
// previous trial's pattern (a stale translation) -- and the same check by
// hipMemcpy, which goes through the copy engines.
//
// --hold keeps each trial's physical allocation until the end of the run
// (released after the next trial has mapped its own), so the next trial's
// memory cannot be the same physical pages: a stale translation then reads
// the previous pattern instead of (by luck) the same pages.
//
//   hipcc --offload-arch=gfx950 -O2 -o build/vmm_remap_probe tools/vmm_remap_probe.hip
// --remap reserves ONE range for the whole run and maps each trial's new
// memory at the same address (unmap, then map the next handle): the pattern
// of an allocator that grows and shrinks inside one reservation (torch's
// expandable segments).
//
//   build/vmm_remap_probe [trials] [--keep] [--hold] [--remap]
//   (--keep: never free a range)
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CHECK(x)                                                                              \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) {                                                               \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(2);                                                                          \
        }                                                                                     \
    } while (0)

__global__ void copy16(const uint4* __restrict__ src, uint4* __restrict__ dst, uint64_t n16)
{
    for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n16; i += uint64_t(gridDim.x) * blockDim.x)
        dst[i] = src[i];
}

static uint8_t pattern(int trial, uint64_t i) { return (uint8_t)(i * 131u + trial * 17u + (i >> 11)); }

int main(int argc, char** argv)
{
    const int trials = argc > 1 ? atoi(argv[1]) : 8;
    bool keep = false, hold = false, remap = false;
    for (int i = 2; i < argc; ++i) {
        keep |= strcmp(argv[i], "--keep") == 0;
        hold |= strcmp(argv[i], "--hold") == 0;
        remap |= strcmp(argv[i], "--remap") == 0;
    }
    std::vector<hipMemGenericAllocationHandle_t> held;
    int dev = 0;
    CHECK(hipSetDevice(dev));
    hipMemAllocationProp prop = {};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = dev;
    size_t gran = 0;
    CHECK(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityMinimum));
    const size_t mapped_n = (2u << 20) > gran ? (2u << 20) / gran * gran : gran;
    const size_t guard = gran >= (2u << 20) ? gran : (2u << 20) / gran * gran;
    const size_t reserved = mapped_n + 2 * guard;
    const uint64_t n16 = mapped_n / 16;

    uint4* dst = nullptr;
    CHECK(hipMalloc(&dst, mapped_n));
    std::vector<uint8_t> host(mapped_n), got(mapped_n);
    void* prev_base = nullptr;
    void* one = nullptr;
    if (remap) CHECK(hipMemAddressReserve(&one, reserved, guard, nullptr, 0));
    for (int t = 0; t < trials; ++t) {
        void* base = one;
        if (!remap) CHECK(hipMemAddressReserve(&base, reserved, guard, nullptr, 0));
        char* mapped = static_cast<char*>(base) + guard;
        hipMemGenericAllocationHandle_t h;
        CHECK(hipMemCreate(&h, mapped_n, &prop, 0));
        CHECK(hipMemMap(mapped, mapped_n, 0, h, 0));
        hipMemAccessDesc acc = {};
        acc.location = prop.location;
        acc.flags = hipMemAccessFlagsProtReadWrite;
        CHECK(hipMemSetAccess(mapped, mapped_n, &acc, 1));
        for (uint64_t i = 0; i < mapped_n; ++i) host[i] = pattern(t, i);
        CHECK(hipMemcpy(mapped, host.data(), mapped_n, hipMemcpyHostToDevice));
        // the copy engines' view of the range
        CHECK(hipMemcpy(got.data(), mapped, mapped_n, hipMemcpyDeviceToHost));
        uint64_t dma_bad = 0;
        for (uint64_t i = 0; i < mapped_n; ++i) dma_bad += got[i] != host[i];
        // a kernel's view
        CHECK(hipMemset(dst, 0, mapped_n));
        copy16<<<1024, 256>>>(reinterpret_cast<const uint4*>(mapped), dst, n16);
        CHECK(hipGetLastError());
        CHECK(hipDeviceSynchronize());
        CHECK(hipMemcpy(got.data(), dst, mapped_n, hipMemcpyDeviceToHost));
        uint64_t bad = 0, stale = 0, first = ~uint64_t(0);
        for (uint64_t i = 0; i < mapped_n; ++i) {
            if (got[i] != host[i]) {
                ++bad;
                if (first == ~uint64_t(0)) first = i;
                if (t > 0 && got[i] == pattern(t - 1, i)) ++stale;
            }
        }
        printf("{\"trial\": %d, \"keep\": %s, \"hold\": %s, \"remap\": %s, \"range\": \"%p\", \"reused\": %s, "
               "\"kernel_bad_bytes\": %llu, \"stale_bytes\": %llu, \"first_bad\": %lld, \"dma_bad_bytes\": %llu}\n",
               t, keep ? "true" : "false", hold ? "true" : "false", remap ? "true" : "false", base,
               base == prev_base ? "true" : "false",
               (unsigned long long)bad,
               (unsigned long long)stale, first == ~uint64_t(0) ? -1LL : (long long)first,
               (unsigned long long)dma_bad);
        fflush(stdout);
        CHECK(hipDeviceSynchronize());
        CHECK(hipMemUnmap(mapped, mapped_n));
        if (hold)
            held.push_back(h);
        else
            CHECK(hipMemRelease(h));
        if (!keep && !remap) CHECK(hipMemAddressFree(base, reserved));
        prev_base = base;
    }
    if (remap) CHECK(hipMemAddressFree(one, reserved));
    for (auto& h : held) CHECK(hipMemRelease(h));
    CHECK(hipFree(dst));
    return 0;
}
