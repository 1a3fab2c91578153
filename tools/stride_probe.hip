// Header-fetch ceiling probe for gfx950: how fast can one 16-byte block per
// frame be read when frames lie `stride` bytes apart (the deserialize plan's
// access pattern: lane l of a wave reads frame f0 + l, so one wave touches
// 64 lines ~stride apart)? Standalone, not part of libcfws; used to decide
// whether the 1 KiB receive plan (216 us for 4 M headers) has headroom.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/stride_probe.hip -o build/stride_probe
//   build/stride_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// kItems frames per thread (all loads issued before any use), kTwo: the
// plan's two aligned blocks per header, kAux: cache-policy bits (nt = 2)
template <int kItems, bool kTwo, int kAux>
__global__ void __launch_bounds__(256) stride_read(const uint8_t* __restrict__ base, uint64_t stride,
                                                   uint64_t n, uint32_t* __restrict__ out)
{
    const uint64_t f0 = uint64_t(blockIdx.x) * 256 * kItems + (threadIdx.x >> 6) * 64 * kItems + (threadIdx.x & 63);
    u32x4 a[kItems], b[kItems];
#pragma unroll
    for (int k = 0; k < kItems; ++k) {
        uint64_t f = f0 + uint64_t(k) * 64;
        f = f < n ? f : n - 1;
        const uint64_t off = (f * stride) & ~uint64_t(15);
        a[k] = kAux ? __builtin_nontemporal_load((const u32x4*)(base + off)) : *(const u32x4*)(base + off);
        if (kTwo) b[k] = *(const u32x4*)(base + off + 16);
    }
    uint32_t x = 0;
#pragma unroll
    for (int k = 0; k < kItems; ++k) {
        x ^= a[k].x ^ a[k].w;
        if (kTwo) x ^= b[k].y;
    }
    out[blockIdx.x * 256 + threadIdx.x] = x;
}

template <int kItems, bool kTwo, int kAux>
float run(const uint8_t* base, uint64_t stride, uint64_t n, uint32_t* out)
{
    const uint64_t per = 256ull * kItems;
    const uint32_t grid = (uint32_t)((n + per - 1) / per);
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    stride_read<kItems, kTwo, kAux><<<grid, 256>>>(base, stride, n, out);
    CHECK(hipEventRecord(e0));
    const int reps = 10;
    for (int r = 0; r < reps; ++r) stride_read<kItems, kTwo, kAux><<<grid, 256>>>(base, stride, n, out);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    CHECK(hipEventDestroy(e0));
    CHECK(hipEventDestroy(e1));
    return ms * 1000.f / reps;
}

int main()
{
    const uint64_t span = 4ull << 30;   // 4 GiB of "wire", as the bench's batches
    uint8_t* base;
    uint32_t* out;
    CHECK(hipMalloc(&base, span + 4096));
    CHECK(hipMemset(base, 1, span + 4096));
    CHECK(hipMalloc(&out, (span / 64 + 256) * 4));
    const uint64_t strides[] = {1032, 264, 136, 128, 4104};
    for (uint64_t s : strides) {
        const uint64_t n = span / s;
        const double lines = (double)n * (s >= 128 ? 1.0 : (double)s / 128.0);
        auto line = [&](const char* form, float us) {
            printf("{\"stride\": %lu, \"frames\": %lu, \"form\": \"%s\", \"us\": %.1f, \"lines_per_us\": %.0f, "
                   "\"line_GBps\": %.0f}\n", (unsigned long)s, (unsigned long)n, form, us, lines / us,
                   lines * 128.0 / us / 1e3);
        };
        line("1blk_items4", run<4, false, 0>(base, s, n, out));
        line("1blk_items8", run<8, false, 0>(base, s, n, out));
        line("1blk_items16", run<16, false, 0>(base, s, n, out));
        line("2blk_items8", run<8, true, 0>(base, s, n, out));
        line("2blk_items16", run<16, true, 0>(base, s, n, out));
        line("1blk_nt_items8", run<8, false, 2>(base, s, n, out));
        fflush(stdout);
    }
    CHECK(hipFree(base));
    CHECK(hipFree(out));
    return 0;
}
