// Partial-segment write probe for gfx950: does a 64-byte output segment
// written by two different waves (one 16-byte chunk early, the other 48
// bytes later -- the codec's edge chunks against its region stores) cost
// more than the bytes say? TCC_EA0_WRREQ - TCC_EA0_WRREQ_64B counted
// 163 k such partial writes per config-5 send launch (0 on the receive).
//
// A 4 GiB stream copy shaped like xform_kernel (4 KiB per wave, 4 x 16 B per
// lane, 256-thread workgroups, `nt` loads default/stores nt). In mode
// "split", one segment in every P has its first chunk left out by the
// region wave and written instead by an "edge" workgroup dispatched first
// (as the codec's edge workgroups are); mode "whole" has the edge workgroup
// write all four chunks of those segments (the region wave skips them all):
// the same ownership change the codec would make, at the same edge count.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/partial_probe.hip -o build/partial_probe
//   build/partial_probe            -> one JSON line per (mode, P, store policy)
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr uint32_t kRegion = 4096;

// kMode 0 none, 1 split, 2 whole (one lane, four stores), 3 whole4 (four
// adjacent lanes, one store instruction per segment), 4 skip (the region
// wave leaves the chunk out and nobody writes it: the region side of the
// partial segments alone); kAux store policy of
// the region stores (0 = global nt)
template <int kMode, int kAux>
__global__ void __launch_bounds__(256) probe_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                    uint64_t bytes, uint32_t P, uint32_t edge_blocks)
{
    extern __shared__ uint8_t lds_pad[];
    (void)lds_pad;
    if (kMode == 3 && blockIdx.x < edge_blocks) {
        // four lanes per edge segment, one 16-byte chunk each
        const uint64_t t = uint64_t(blockIdx.x) * 256 + threadIdx.x;
        const uint64_t s = (t >> 2) * P;
        if (s * 64 >= bytes) return;
        const uint64_t off = s * 64 + (t & 3) * 16;
        u32x4 v = *reinterpret_cast<const u32x4*>(src + off);
        v ^= 0x9e3779b9u;
        __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(dst + off));
        return;
    }
    if (blockIdx.x < edge_blocks) {
        // one thread per edge segment (segments s with s % P == 0)
        const uint64_t e = uint64_t(blockIdx.x) * 256 + threadIdx.x;
        const uint64_t s = e * P;
        if (s * 64 >= bytes) return;
        const uint32_t nchunks = kMode == 2 ? 4u : 1u;
        for (uint32_t c = 0; c < nchunks; ++c) {
            const uint64_t off = s * 64 + c * 16;
            u32x4 v = *reinterpret_cast<const u32x4*>(src + off);
            v ^= 0x9e3779b9u;
            __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(dst + off));
        }
        return;
    }
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t base = (uint64_t(blockIdx.x - edge_blocks) * 4 + wave) * kRegion;
    if (base >= bytes) return;
    u32x4 a[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) a[u] = *reinterpret_cast<const u32x4*>(src + base + u * 1024 + lane * 16);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const uint64_t off = base + u * 1024 + lane * 16;
        const uint64_t s = off >> 6;
        const bool edge = kMode != 0 && (s % P) == 0 && ((kMode == 2 || kMode == 3) || (off & 63) == 0);
        if (edge) continue;
        a[u] ^= 0x9e3779b9u;
        if (kAux == 0) {
            __builtin_nontemporal_store(a[u], reinterpret_cast<u32x4*>(dst + off));
        } else {
            const auto r = __builtin_amdgcn_make_buffer_rsrc(dst + base, 0, (int)kRegion, 0x00020000);
            __builtin_amdgcn_raw_buffer_store_b128(a[u], r, (int)(u * 1024 + lane * 16), 0, kAux);
        }
    }
}

template <int kMode, int kAux>
double run(const uint8_t* src, uint8_t* dst, uint64_t bytes, uint32_t P, int lds)
{
    auto k = probe_kernel<kMode, kAux>;
    CHECK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    const uint64_t regions = bytes / kRegion;
    const uint32_t body_blocks = (uint32_t)((regions + 3) / 4);
    const uint64_t edges = (kMode && kMode != 4) ? (bytes / 64 + P - 1) / P * (kMode == 3 ? 4 : 1) : 0;
    const uint32_t edge_blocks = (uint32_t)((edges + 255) / 256);
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    k<<<edge_blocks + body_blocks, 256, lds>>>(src, dst, bytes, P, edge_blocks);
    CHECK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
        CHECK(hipEventRecord(a, 0));
        k<<<edge_blocks + body_blocks, 256, lds>>>(src, dst, bytes, P, edge_blocks);
        CHECK(hipEventRecord(b, 0));
        CHECK(hipEventSynchronize(b));
        float t = 0;
        CHECK(hipEventElapsedTime(&t, a, b));
        if (t < best) best = t;
    }
    CHECK(hipEventDestroy(a));
    CHECK(hipEventDestroy(b));
    return 2.0 * double(bytes) / (best * 1e-3) / 1e12;
}

int main(int argc, char** argv)
{
    const uint64_t bytes = uint64_t(argc > 1 ? atof(argv[1]) : 4.0) * (1ull << 30);
    uint8_t *src, *dst;
    CHECK(hipMalloc(&src, bytes + 4096));
    CHECK(hipMalloc(&dst, bytes + 4096));
    CHECK(hipMemset(src, 0x5a, bytes + 4096));
    CHECK(hipMemset(dst, 0, bytes + 4096));
    const int lds = 32000;                       // 5 WG/CU, the codec's default
    for (int rep = 0; rep < 2; ++rep) {
        printf("{\"mode\": \"none\", \"aux\": \"nt\", \"TBps\": %.3f}\n", run<0, 0>(src, dst, bytes, 1, lds));
        printf("{\"mode\": \"none\", \"aux\": \"wt\", \"TBps\": %.3f}\n", run<0, 19>(src, dst, bytes, 1, lds));
        for (uint32_t P : {1024u, 256u, 100u, 16u}) {
            printf("{\"mode\": \"split\", \"aux\": \"nt\", \"P\": %u, \"TBps\": %.3f}\n", P,
                   run<1, 0>(src, dst, bytes, P, lds));
            printf("{\"mode\": \"whole\", \"aux\": \"nt\", \"P\": %u, \"TBps\": %.3f}\n", P,
                   run<2, 0>(src, dst, bytes, P, lds));
            printf("{\"mode\": \"whole4\", \"aux\": \"nt\", \"P\": %u, \"TBps\": %.3f}\n", P,
                   run<3, 0>(src, dst, bytes, P, lds));
            printf("{\"mode\": \"whole4\", \"aux\": \"wt\", \"P\": %u, \"TBps\": %.3f}\n", P,
                   run<3, 19>(src, dst, bytes, P, lds));
            printf("{\"mode\": \"skip\", \"aux\": \"nt\", \"P\": %u, \"TBps\": %.3f}\n", P,
                   run<4, 0>(src, dst, bytes, P, lds));
            printf("{\"mode\": \"split\", \"aux\": \"wt\", \"P\": %u, \"TBps\": %.3f}\n", P,
                   run<1, 19>(src, dst, bytes, P, lds));
            printf("{\"mode\": \"whole\", \"aux\": \"wt\", \"P\": %u, \"TBps\": %.3f}\n", P,
                   run<2, 19>(src, dst, bytes, P, lds));
            fflush(stdout);
        }
    }
    CHECK(hipFree(src));
    CHECK(hipFree(dst));
    return 0;
}
