// PCIe probe for the host-memory pipeline: SDMA copies (hipMemcpyAsync) vs
// kernels that read / write device-mapped pinned host memory directly, one
// direction at a time and both directions at once. Decides whether the
// pipeline's D2H (or H2D) leg should be a kernel instead of a copy engine.
// Standalone, not part of libcfws.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/pcie_probe2.hip -o build/pcie_probe2
//   build/pcie_probe2 [MiB]
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(256) copy16(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                              uint64_t n16, int nt_store)
{
    const uint64_t stride = uint64_t(gridDim.x) * 256;
    for (uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x; i < n16; i += stride) {
        const u32x4 v = src[i];
        if (nt_store) __builtin_nontemporal_store(v, dst + i);
        else dst[i] = v;
    }
}

static double now()
{
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

template <typename F>
static double timed(F f, int reps = 5)
{
    f();
    CHECK(hipDeviceSynchronize());
    const double t = now();
    for (int i = 0; i < reps; ++i) f();
    CHECK(hipDeviceSynchronize());
    return (now() - t) / reps;
}

int main(int argc, char** argv)
{
    const uint64_t mib = argc > 1 ? strtoull(argv[1], nullptr, 10) : 512;
    const uint64_t n = mib << 20;
    void *h_in = nullptr, *h_out = nullptr, *h_out_nc = nullptr;
    CHECK(hipHostMalloc(&h_in, n, hipHostMallocMapped));
    CHECK(hipHostMalloc(&h_out, n, hipHostMallocMapped));
    CHECK(hipHostMalloc(&h_out_nc, n, hipHostMallocMapped | hipHostMallocNonCoherent));
    void *dh_in = nullptr, *dh_out = nullptr, *dh_out_nc = nullptr;
    CHECK(hipHostGetDevicePointer(&dh_in, h_in, 0));
    CHECK(hipHostGetDevicePointer(&dh_out, h_out, 0));
    CHECK(hipHostGetDevicePointer(&dh_out_nc, h_out_nc, 0));
    void *d_a = nullptr, *d_b = nullptr;
    CHECK(hipMalloc(&d_a, n));
    CHECK(hipMalloc(&d_b, n));
    for (uint64_t i = 0; i < n; i += 4096) static_cast<uint8_t*>(h_in)[i] = (uint8_t)i;
    CHECK(hipMemset(d_b, 3, n));
    hipStream_t s1, s2;
    CHECK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CHECK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    const uint64_t n16 = n / 16;
    const int grid = argc > 2 ? atoi(argv[2]) : 1024;

    auto sdma_h2d = [&] { CHECK(hipMemcpyAsync(d_a, h_in, n, hipMemcpyHostToDevice, s1)); };
    auto sdma_d2h = [&] { CHECK(hipMemcpyAsync(h_out, d_b, n, hipMemcpyDeviceToHost, s2)); };
    auto kern_h2d = [&] {
        copy16<<<grid, 256, 0, s1>>>(static_cast<const u32x4*>(dh_in), static_cast<u32x4*>(d_a), n16, 0);
    };
    auto kern_d2h = [&] {
        copy16<<<grid, 256, 0, s2>>>(static_cast<const u32x4*>(d_b), static_cast<u32x4*>(dh_out), n16, 0);
    };
    auto kern_d2h_nt = [&] {
        copy16<<<grid, 256, 0, s2>>>(static_cast<const u32x4*>(d_b), static_cast<u32x4*>(dh_out), n16, 1);
    };
    auto kern_d2h_nc = [&] {
        copy16<<<grid, 256, 0, s2>>>(static_cast<const u32x4*>(d_b), static_cast<u32x4*>(dh_out_nc), n16, 0);
    };
    const double gb = double(n) / 1e9;
    printf("{\"bytes\": %llu, \"grid\": %d", (unsigned long long)n, grid);
    printf(", \"sdma_h2d\": %.2f", gb / timed(sdma_h2d));
    printf(", \"sdma_d2h\": %.2f", gb / timed(sdma_d2h));
    printf(", \"sdma_both_each\": %.2f", gb / timed([&] { sdma_h2d(); sdma_d2h(); }));
    printf(", \"kern_h2d\": %.2f", gb / timed(kern_h2d));
    printf(", \"kern_d2h\": %.2f", gb / timed(kern_d2h));
    printf(", \"kern_d2h_nt\": %.2f", gb / timed(kern_d2h_nt));
    printf(", \"kern_d2h_noncoherent\": %.2f", gb / timed(kern_d2h_nc));
    printf(", \"sdma_h2d+kern_d2h_each\": %.2f", gb / timed([&] { sdma_h2d(); kern_d2h(); }));
    printf(", \"kern_h2d+sdma_d2h_each\": %.2f", gb / timed([&] { kern_h2d(); sdma_d2h(); }));
    printf(", \"kern_h2d+kern_d2h_each\": %.2f", gb / timed([&] { kern_h2d(); kern_d2h(); }));
    printf("}\n");
    CHECK(hipFree(d_a));
    CHECK(hipFree(d_b));
    CHECK(hipHostFree(h_in));
    CHECK(hipHostFree(h_out));
    CHECK(hipHostFree(h_out_nc));
    return 0;
}
