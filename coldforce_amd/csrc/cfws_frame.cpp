// cfws_frame.cpp -- the drop-in per-frame ABI (include/cfws_co_ws_frame.h).
//
// Same symbols, prototypes, struct layouts and return codes as coldforce's
// src/ws/co_ws_frame.c + src/ws/co_ws_config.c, so libco_ws's callers
// (co_ws_send, the receive loops, the ws_http2 extension) link against this
// library unchanged. The payload XOR of a masked frame -- the reference's
// scalar byte loops at co_ws_frame.c:93-97 and :234-242 -- runs on the
// MI355X through cfws_xor_mask() at or above the size policy's threshold
// (CFWS_DROPIN_GPU_MIN), and on the calling thread below it (the library's
// own vector loop, host_xor: the reference's per-frame loop, done faster).
// The 2-14 header bytes and the byte-array bookkeeping stay on the calling
// thread. Unmasked frames are plain copies in the reference too and stay
// plain copies here. A frame the policy sends to the device fails without a
// gfx950 device (serialize returns false, deserialize
// CO_WS_ERROR_OUT_OF_MEMORY) and the reason goes to stderr and
// cfws_last_error(); a frame below the threshold never touches HIP.
#include <hip/hip_runtime.h>

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <chrono>
#include <mutex>
#include <vector>

#include "cfws.h"
#include "cfws_co_ws_frame.h"
#include "cfws_devpolicy.h"
#include "cfws_internal.h"

namespace {

// co_ws_config.c:12-15 -- one process-wide, unsynchronised setting.
size_t g_max_receive_payload_size = 32u * 1024u * 1024u;

// Per calling thread and device: one stream, a pinned host staging buffer
// the device reads and writes in place (mapped into the GPU's address
// space), and a device staging buffer for frames above the zero-copy limit;
// all reused across frames (coldforce runs each connection on one co_thread).
struct ThreadDevice {
    int device = -1;               // the device the stream and buffers belong to
    hipStream_t stream = nullptr;
    void* buf = nullptr;           // device memory (DMA path)
    size_t cap = 0;
    uint8_t* host = nullptr;       // pinned host memory (zero-copy path)
    void* host_dev = nullptr;      // its device-side address
    size_t host_cap = 0;
    bool zc_warm = false;          // first zero-copy frame done
    bool dma_warm = false;         // first DMA-path frame done
    // the frame service (frames up to service_max()): this thread's slot in
    // its device's service, and the seq of its last request there
    int svc_slot = -1;
    uint32_t seq = 0;
    bool svc_warm = false;         // first service frame done
    bool holds() const { return stream || buf || host || svc_slot >= 0; }
};

// Device policy and per-device resource pool: cfws_devpolicy.h. The pool is
// never destroyed (no HIP call at exit; the runtime may be tearing down).
constexpr int kPoolDevices = 64;
using DevicePool = cfws_policy::DevicePool<ThreadDevice, kPoolDevices>;
using ThreadSlot = cfws_policy::ThreadSlot<ThreadDevice, DevicePool>;

DevicePool& device_pool()
{
    static DevicePool* pool = new DevicePool;
    return *pool;
}

thread_local ThreadSlot t_slot(device_pool());

int target_device()
{
    int dev = 0;
    if (t_slot.bound() >= 0) return t_slot.bound();
    if (hipGetDevice(&dev) != hipSuccess) return -1;
    return t_slot.target(dev);
}

ThreadDevice& tdev(int dev) { return t_slot.on(dev); }

// Runs HIP calls that act on the current device (stream creation,
// allocation) against `dev`, restoring the caller's device afterwards.
class CurrentDevice {
public:
    explicit CurrentDevice(int dev)
    {
        if (hipGetDevice(&saved_) == hipSuccess && saved_ != dev && hipSetDevice(dev) == hipSuccess) switched_ = true;
    }
    ~CurrentDevice()
    {
        if (switched_) (void)hipSetDevice(saved_);
    }
    CurrentDevice(const CurrentDevice&) = delete;
    CurrentDevice& operator=(const CurrentDevice&) = delete;

private:
    int saved_ = 0;
    bool switched_ = false;
};

// Frames up to this size take the zero-copy path: the payload is copied into
// the pinned buffer and the XOR kernel reads and writes it over PCIe, so a
// frame costs one launch + one synchronize instead of H2D + launch + D2H
// (profiles/r01_dropin_latency_*.json). Larger frames take the DMA path, whose
// copy engines move bulk bytes faster than a kernel's PCIe accesses.
// CFWS_DROPIN_ZC_MAX overrides (bytes; 0 = DMA path always).
size_t zero_copy_max()
{
    // read once: a function-local static's initialiser runs under the C++
    // runtime's guard, whichever thread calls first
    static const size_t v = [] {
        const char* s = getenv("CFWS_DROPIN_ZC_MAX");
        return s ? static_cast<size_t>(strtoull(s, nullptr, 10)) : (size_t(1) << 20);
    }();
    return v;
}

bool stream_ready(ThreadDevice& t_dev)
{
    if (t_dev.stream) return true;
    if (hipStreamCreateWithFlags(&t_dev.stream, hipStreamNonBlocking) != hipSuccess) {
        fprintf(stderr, "cfws: hipStreamCreate on device %d failed\n", t_dev.device);
        t_dev.stream = nullptr;
        return false;
    }
    return true;
}

bool device_stage(ThreadDevice& t_dev, size_t n)
{
    if (!stream_ready(t_dev)) return false;
    if (t_dev.cap < n) {
        size_t cap = 1u << 16;
        while (cap < n) cap <<= 1;
        if (t_dev.buf) (void)hipFree(t_dev.buf);
        t_dev.buf = nullptr;
        t_dev.cap = 0;
        if (hipMalloc(&t_dev.buf, cap) != hipSuccess) {
            fprintf(stderr, "cfws: hipMalloc(%zu) failed\n", cap);
            return false;
        }
        t_dev.cap = cap;
    }
    return true;
}

bool host_stage(ThreadDevice& t_dev, size_t n)
{
    if (!stream_ready(t_dev)) return false;
    if (t_dev.host_cap < n) {
        size_t cap = 1u << 16;
        while (cap < n) cap <<= 1;
        if (t_dev.host) (void)hipHostFree(t_dev.host);
        t_dev.host = nullptr;
        t_dev.host_dev = nullptr;
        t_dev.host_cap = 0;
        void* h = nullptr;
        if (hipHostMalloc(&h, cap, hipHostMallocMapped) != hipSuccess) {
            fprintf(stderr, "cfws: hipHostMalloc(%zu) failed\n", cap);
            return false;
        }
        void* d = nullptr;
        if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess || !d) {
            fprintf(stderr, "cfws: hipHostGetDevicePointer failed\n");
            (void)hipHostFree(h);
            return false;
        }
        t_dev.host = static_cast<uint8_t*>(h);
        t_dev.host_dev = d;
        t_dev.host_cap = cap;
    }
    return true;
}

// The mask keys are the process's random() stream (co_random.c:32-35), so
// the drop-in's device work must not consume it. The HIP/HSA runtime calls
// rand()/random() (glibc: one shared state) while it sets things up: its
// initialisation, a new stream's first work (profiles/
// r02_random_state_probe.jsonl), allocations. While a guard lives, random()
// runs on a private state and the caller's state is put back exactly where
// the reference would leave it. glibc's state pointer is process-wide, so
// guards never overlap (one process-wide mutex) and are taken only around
// set-up work: a thread's first frame on a device, a staging buffer that
// grows, each path's first frame. A steady-state frame swaps nothing, so
// another thread's random() is never redirected by it (INTEGRATION.md §1
// notes the set-up window).
std::mutex& random_guard_mutex()
{
    static std::mutex* mu = new std::mutex;
    return *mu;
}

class RandomStateGuard {
public:
    RandomStateGuard() : lock_(random_guard_mutex(), std::defer_lock) {}
    void engage()
    {
        if (lock_.owns_lock()) return;
        lock_.lock();
        saved_ = initstate(0x5eedu, reinterpret_cast<char*>(scratch_), sizeof scratch_);
    }
    ~RandomStateGuard()
    {
        if (lock_.owns_lock()) setstate(saved_);
    }
    RandomStateGuard(const RandomStateGuard&) = delete;
    RandomStateGuard& operator=(const RandomStateGuard&) = delete;

private:
    std::unique_lock<std::mutex> lock_;
    int32_t scratch_[32];          // glibc reads the state as int32_t words
    char* saved_ = nullptr;
};

// ---- the frame service ---------------------------------------------------
// A masked frame of at most service_max() bytes is XORed by a resident
// kernel (dropin_service_kernel, cfws_ops.hip) that serves every calling
// thread on its device: the thread copies the frame into its slot's mapped
// pinned buffer, posts one 64-bit request word (key, length, seq) and spins
// on its done word, which the kernel writes after its stores are released
// to system scope. No launch and no completion signal per frame (DESIGN.md
// section 6). One kernel per device, whatever the number of threads: with
// GPU_MAX_HW_QUEUES = 4 the process's streams share hardware queues, and a
// resident kernel per thread would queue other threads' launches behind
// itself. The kernel ends after an idle spell (CFWS_DROPIN_SERVICE_IDLE_US,
// default 2,000) or after CFWS_DROPIN_SERVICE_LIFE_US in all (default
// 10,000: the longest a launch sharing its queue waits); the next request,
// or a waiting thread that sees the exit word, launches it again. A thread
// beyond the 64 slots, or one whose slot was given up after a timeout, takes
// the launch path. CFWS_DROPIN_SERVICE=0 sends every frame there.
bool service_enabled()
{
    static const bool v = [] {
        const char* s = getenv("CFWS_DROPIN_SERVICE");
        return !(s && *s == '0');
    }();
    return v;
}

// Largest frame the service takes (CFWS_DROPIN_SERVICE_MAX, at most
// kCfwsServiceMax); larger frames take the launch path. Default 32 KiB: per
// serialize (or deserialize) the service took 6.2 us at 1 KiB and 8.1 us at
// 16 KiB against 13.8 / 14.9 us with a launch per frame, but 23 us at
// 64 KiB against 18 (profiles/r03_dropin_lat.jsonl).
size_t service_max()
{
    static const size_t v = [] {
        const char* s = getenv("CFWS_DROPIN_SERVICE_MAX");
        const size_t x = s && *s ? (size_t)strtoull(s, nullptr, 10) : (size_t)32768;
        return x < (size_t)kCfwsServiceMax ? x : (size_t)kCfwsServiceMax;
    }();
    return v;
}

double env_us(const char* name, double dflt, double lo)
{
    const char* s = getenv(name);
    const double us = s && *s ? strtod(s, nullptr) : dflt;
    return (us < lo ? lo : us) * 1e-6;
}

double service_idle_s()
{
    static const double v = env_us("CFWS_DROPIN_SERVICE_IDLE_US", 2000.0, 50.0);
    return v;
}

double service_life_s()
{
    static const double v = env_us("CFWS_DROPIN_SERVICE_LIFE_US", 10000.0, 200.0);
    return v;
}

// How long a thread waits for the service's answer before it retires its
// slot and takes the launch path (CFWS_DROPIN_SERVICE_TIMEOUT_US, default
// 5 s; tests shorten it to make retirements happen).
double service_timeout_s()
{
    static const double v = env_us("CFWS_DROPIN_SERVICE_TIMEOUT_US", 5e6, 1.0);
    return v;
}

double now_s()
{
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// One per device, created by the first thread that needs it, never freed
// (no HIP call at exit: the process-exit hook only sets the stop word).
struct ServiceDevice {
    std::mutex mu;                         // launches; slot allocation
    uint64_t* ctl = nullptr;               // control page, host address
    uint64_t* ctl_dev = nullptr;
    uint8_t* bufs = nullptr;               // kCfwsServiceSlots x kCfwsServiceMax
    uint8_t* bufs_dev = nullptr;
    hipStream_t stream = nullptr;
    uint64_t idle_ticks = 0, life_ticks = 0;
    std::atomic<uint64_t> launched{0};     // generation of the last launch
    uint64_t free_slots = ~0ull;           // under mu
    // given up after a timeout, under mu: a slot comes back once its done
    // word reaches the seq it was given up at (a later kernel did finish
    // that request, and nothing is posted on the slot after it)
    uint64_t lost_slots = 0;
    uint32_t lost_seq[kCfwsServiceSlots] = {};
    bool failed = false;                   // set-up failed: launch path only
};

std::mutex& services_mutex()
{
    static std::mutex* mu = new std::mutex;
    return *mu;
}

ServiceDevice* g_services[kPoolDevices];   // under services_mutex()

void stop_all_services()
{
    std::lock_guard<std::mutex> lock(services_mutex());
    for (ServiceDevice* sd : g_services)
        if (sd && sd->ctl) __atomic_store_n(&sd->ctl[kCfwsServiceStopWord], uint64_t(1), __ATOMIC_RELEASE);
}

// The device's service, set up on first use; nullptr when that failed.
ServiceDevice* service_device(int dev)
{
    std::lock_guard<std::mutex> lock(services_mutex());
    ServiceDevice*& sd = g_services[dev];
    if (sd) return sd->failed ? nullptr : sd;
    sd = new ServiceDevice;
    CurrentDevice on(dev);
    void* m = nullptr;
    void* b = nullptr;
    void* md = nullptr;
    void* bd = nullptr;
    if (hipHostMalloc(&m, kCfwsServiceCtlBytes, hipHostMallocMapped) != hipSuccess ||
        hipHostMalloc(&b, size_t(kCfwsServiceSlots) * kCfwsServiceMax, hipHostMallocMapped) != hipSuccess ||
        hipHostGetDevicePointer(&md, m, 0) != hipSuccess || hipHostGetDevicePointer(&bd, b, 0) != hipSuccess ||
        hipStreamCreateWithFlags(&sd->stream, hipStreamNonBlocking) != hipSuccess) {
        fprintf(stderr, "cfws: frame service set-up on device %d failed; frames take the launch path\n", dev);
        if (m) (void)hipHostFree(m);
        if (b) (void)hipHostFree(b);
        sd->failed = true;
        return nullptr;
    }
    memset(m, 0, kCfwsServiceCtlBytes);
    sd->ctl = static_cast<uint64_t*>(m);
    sd->ctl_dev = static_cast<uint64_t*>(md);
    sd->bufs = static_cast<uint8_t*>(b);
    sd->bufs_dev = static_cast<uint8_t*>(bd);
    int rate_khz = 0;
    if (hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess || rate_khz <= 0)
        rate_khz = 100000;
    sd->idle_ticks = (uint64_t)(service_idle_s() * 1e3 * (double)rate_khz);
    sd->life_ticks = (uint64_t)(service_life_s() * 1e3 * (double)rate_khz);
    static std::once_flag exit_hook;
    std::call_once(exit_hook, [] { atexit(stop_all_services); });
    return sd;
}

// Is the last launched kernel still serving? It has ended once it wrote its
// generation to the exit word (after that it touches no slot).
bool service_running(ServiceDevice& sd)
{
    const uint64_t g = sd.launched.load(std::memory_order_acquire);
    return g != 0 && __atomic_load_n(&sd.ctl[kCfwsServiceExitWord], __ATOMIC_ACQUIRE) != g;
}

// Launches the next generation unless one is serving. Any thread may call;
// one launches.
bool service_ensure_running(ServiceDevice& sd, int dev)
{
    if (service_running(sd)) return true;
    std::lock_guard<std::mutex> lock(sd.mu);
    if (service_running(sd)) return true;
    const uint64_t g = sd.launched.load(std::memory_order_relaxed) + 1;
    CurrentDevice on(dev);
    if (cfws_internal_service_launch(sd.ctl_dev, sd.bufs_dev, g, sd.idle_ticks, sd.life_ticks, sd.stream) != CFWS_OK) {
        fprintf(stderr, "cfws: frame service launch failed: %s\n", cfws_last_error());
        return false;
    }
    sd.launched.store(g, std::memory_order_release);
    return true;
}

// Lost slots whose request has since completed go back to the free list
// (under sd.mu). A kernel stalled behind other work on a shared hardware
// queue can answer after the 5 s wait: each such stall would otherwise cost
// a slot for the rest of the process.
void service_reclaim(ServiceDevice& sd)
{
    for (uint64_t m = sd.lost_slots; m; m &= m - 1) {
        const int s = __builtin_ctzll(m);
        const uint32_t done = (uint32_t)(__atomic_load_n(&sd.ctl[kCfwsServiceDoneWord + s], __ATOMIC_ACQUIRE) >> 48);
        if (done == sd.lost_seq[s]) {
            sd.lost_slots &= ~(1ull << s);
            sd.free_slots |= 1ull << s;
        }
    }
}

int service_take_slot(ServiceDevice& sd)
{
    std::lock_guard<std::mutex> lock(sd.mu);
    if (!sd.free_slots && sd.lost_slots) service_reclaim(sd);
    if (!sd.free_slots) return -1;
    const int s = __builtin_ctzll(sd.free_slots);
    sd.free_slots &= sd.free_slots - 1;
    return s;
}

void service_give_slot(int dev, int s)
{
    if (dev < 0 || dev >= kPoolDevices || s < 0) return;
    ServiceDevice* sd = nullptr;
    {
        std::lock_guard<std::mutex> lock(services_mutex());
        sd = g_services[dev];
    }
    if (!sd) return;
    std::lock_guard<std::mutex> lock(sd->mu);
    if (!(sd->lost_slots >> s & 1)) sd->free_slots |= 1ull << s;
}

// 1: done; 0: no slot or no service here (the caller takes the launch
// path); -1: failed.
int service_xor(ThreadDevice& t_dev, int dev, const uint8_t* src, uint8_t* dst, size_t n, uint32_t key)
{
    ServiceDevice* sd = service_device(dev);
    if (!sd) return 0;
    if (t_dev.svc_slot < 0) {
        t_dev.svc_slot = service_take_slot(*sd);
        if (t_dev.svc_slot < 0) return 0;
        t_dev.seq = (uint32_t)(__atomic_load_n(&sd->ctl[kCfwsServiceDoneWord + t_dev.svc_slot], __ATOMIC_ACQUIRE) >> 48);
    }
    const int s = t_dev.svc_slot;
    uint8_t* buf = sd->bufs + (size_t)s * kCfwsServiceMax;
    memcpy(buf, src, n);
    const uint32_t seq = (t_dev.seq + 1) & 0xffffu;
    const uint64_t word = (uint64_t)key | ((uint64_t)(n - 1) << 32) | ((uint64_t)seq << 48);
    __atomic_store_n(&sd->ctl[kCfwsServiceReqWord + s], word, __ATOMIC_RELEASE);
    t_dev.seq = seq;               // posted: never reused for another frame
    if (!service_ensure_running(*sd, dev)) return -1;
    const uint64_t* done = &sd->ctl[kCfwsServiceDoneWord + s];
    const double t0 = now_s();
    for (uint64_t spin = 1;; ++spin) {
        if ((uint32_t)(__atomic_load_n(done, __ATOMIC_ACQUIRE) >> 48) == seq) break;
        if ((spin & 255u) == 0) {
            // the kernel may have ended (idle or lifetime) without taking
            // the request: launch the next one
            if (!service_ensure_running(*sd, dev)) return -1;
            if (now_s() - t0 > service_timeout_s()) {
                // give the slot up until its request completes: the request
                // stays posted, and a later kernel may still XOR that buffer
                // (service_reclaim returns the slot after that)
                fprintf(stderr, "cfws: frame service: no answer in %.0f us (slot %d retired)\n",
                        service_timeout_s() * 1e6, s);
                {
                    std::lock_guard<std::mutex> lock(sd->mu);
                    sd->lost_slots |= 1ull << s;
                    sd->lost_seq[s] = seq;
                }
                t_dev.svc_slot = -1;
                return -1;
            }
        }
        __builtin_ia32_pause();
    }
    memcpy(dst, buf, n);
    return 1;
}

std::atomic<bool> g_runtime_up{false};   // the HIP runtime has been initialised by us

// ---- the size policy --------------------------------------------------------
// Below CFWS_DROPIN_GPU_MIN bytes (cfws_set_dropin_gpu_min at run time) a
// masked payload is XORed on the calling thread: a per-frame call is
// latency-bound, and the payload would cross PCIe twice.
// DESIGN.md section 6 has wall and CPU time per frame for every path: the
// calling thread wins both at every size measured (125 B - 4 MiB), so the
// default threshold is SIZE_MAX and the device paths below are opt-in. The
// host path is the library's own loop and needs no device: a frame below the
// threshold makes no HIP call. At or above it the device paths run, and
// without a gfx950 agent such a frame fails. The batch ABI (include/cfws.h)
// has no host path at any size.
std::atomic<size_t> g_gpu_min{[] {
    const char* s = getenv("CFWS_DROPIN_GPU_MIN");
    return s && *s ? (size_t)strtoull(s, nullptr, 10) : (size_t)CFWS_DROPIN_GPU_MIN_DEFAULT;
}()};

// dst[i] = src[i] ^ key[i % 4] (key byte j = bits 8j..8j+7), 16 bytes per
// step on two 64-bit words (the compiler keeps them in one SSE register).
void host_xor(const uint8_t* src, uint8_t* dst, size_t n, uint32_t key)
{
    const uint64_t k = (uint64_t)key | (uint64_t)key << 32;
    size_t i = 0;
    for (; i + 16 <= n; i += 16) {
        uint64_t a, b;
        memcpy(&a, src + i, 8);
        memcpy(&b, src + i + 8, 8);
        a ^= k;
        b ^= k;
        memcpy(dst + i, &a, 8);
        memcpy(dst + i + 8, &b, 8);
    }
    for (; i < n; ++i) dst[i] = (uint8_t)(src[i] ^ (key >> (8 * (i & 3u))));
}

bool device_xor(const uint8_t* src, uint8_t* dst, size_t n, uint32_t key);

bool payload_xor(const uint8_t* src, uint8_t* dst, size_t n, uint32_t key)
{
    if (n >= g_gpu_min.load(std::memory_order_relaxed)) return device_xor(src, dst, n, key);
    host_xor(src, dst, n, key);
    return true;
}



bool device_xor(const uint8_t* src, uint8_t* dst, size_t n, uint32_t key)
{
    RandomStateGuard keep_random_stream;
    // the first HIP call of the process (hipGetDevice included) initialises
    // the runtime
    if (!g_runtime_up.load(std::memory_order_acquire)) keep_random_stream.engage();
    const int dev = target_device();
    if ((dev < 0 ? cfws_init() : cfws_init_device(dev)) != CFWS_OK || dev < 0) {
        fprintf(stderr, "cfws: drop-in has no usable device (%s)\n", cfws_last_error());
        return false;
    }
    g_runtime_up.store(true, std::memory_order_release);
    ThreadDevice& t_dev = tdev(dev);
    if (service_enabled() && n <= service_max()) {
        if (!t_dev.svc_warm) keep_random_stream.engage();
        // a service that failed (launch error, or a request that timed out:
        // its slot is retired) leaves the frame to the launch path below
        const int r = service_xor(t_dev, dev, src, dst, n, key);
        if (r > 0) {
            t_dev.svc_warm = true;
            return true;
        }
    }
    const bool zero_copy = n <= zero_copy_max();
    if (!t_dev.stream || (zero_copy ? (!t_dev.zc_warm || t_dev.host_cap < n) : (!t_dev.dma_warm || t_dev.cap < n)))
        keep_random_stream.engage();
    CurrentDevice on(dev);         // held across the launch and the synchronize
    if (zero_copy ? !host_stage(t_dev, n) : !device_stage(t_dev, n)) return false;
    hipStream_t st = t_dev.stream;
    if (zero_copy) {
        memcpy(t_dev.host, src, n);
        if (cfws_xor_mask(t_dev.host_dev, t_dev.host_dev, n, key, 0, st) != CFWS_OK) return false;
    } else {
        if (hipMemcpyAsync(t_dev.buf, src, n, hipMemcpyHostToDevice, st) != hipSuccess) return false;
        if (cfws_xor_mask(t_dev.buf, t_dev.buf, n, key, 0, st) != CFWS_OK) return false;
        if (hipMemcpyAsync(dst, t_dev.buf, n, hipMemcpyDeviceToHost, st) != hipSuccess) return false;
    }
    // (a wait blocked on a hipEventBlockingSync event instead measured the
    // same calling-thread CPU time as this spin)
    hipError_t e = hipStreamSynchronize(st);
    if (e != hipSuccess) {
        fprintf(stderr, "cfws: device XOR failed: %s\n", hipGetErrorString(e));
        return false;
    }
    if (zero_copy) {
        memcpy(dst, t_dev.host, n);
        t_dev.zc_warm = true;
    } else {
        t_dev.dma_warm = true;
    }
    return true;
}

// co_array_set_count growth rule (src/core/co_array.c:83-112): capacity
// doubles until it exceeds the new count.
bool byte_array_reserve(co_byte_array_t* b, size_t count)
{
    if (b->capacity > count) return true;
    size_t cap = b->capacity * 2;
    while (cap <= count) cap *= 2;
    void* nb = realloc(b->buffer, b->element_size * cap);
    if (!nb) return false;
    b->buffer = static_cast<uint8_t*>(nb);
    b->capacity = cap;
    return true;
}

// Header encode, co_ws_frame.c:34-91. Returns its size (2..14).
uint32_t encode_header(bool fin, uint8_t opcode, bool mask, uint32_t key, uint64_t n, uint8_t* h)
{
    uint32_t k = 2;
    h[0] = static_cast<uint8_t>(opcode | (fin ? 0x80u : 0u));
    if (n <= 125u) {
        h[1] = static_cast<uint8_t>(n);
    } else if (n <= 0xffffu) {
        h[1] = 126;
        h[k++] = static_cast<uint8_t>(n >> 8);
        h[k++] = static_cast<uint8_t>(n);
    } else {
        h[1] = 127;
        for (int s = 56; s >= 0; s -= 8) h[k++] = static_cast<uint8_t>(n >> s);
    }
    if (mask) {
        h[1] = static_cast<uint8_t>(h[1] | 0x80u);
        for (int j = 0; j < 4; ++j) h[k++] = static_cast<uint8_t>(key >> (8 * j));
    }
    return k;
}

}  // namespace

extern "C" {

bool co_ws_frame_serialize(bool fin, uint8_t opcode, bool mask, const void* data, size_t n,
                           co_byte_array_t* buffer)
{
    const size_t start = buffer->count;
    const size_t hmax = 2 + (n > 0xffffu ? 8 : (n > 125u ? 2 : 0)) + (mask ? 4 : 0);
    // The reference's only failure is malloc(n) before any key draw
    // (co_ws_frame.c:74-80); reserving up front fails at the same point.
    if (!byte_array_reserve(buffer, start + hmax + n)) return false;
    uint32_t key = 0;
    if (mask) {
        // co_random(mask_key, 4): four (uint8_t)(random() % 256) draws.
        for (int j = 0; j < 4; ++j) key |= static_cast<uint32_t>(static_cast<uint8_t>(random() % 256)) << (8 * j);
    }
    uint8_t* out = buffer->buffer + start;
    const uint32_t hs = encode_header(fin, opcode, mask, key, n, out);
    if (n > 0) {
        if (mask) {
            if (!payload_xor(static_cast<const uint8_t*>(data), out + hs, n, key)) return false;
        } else {
            memcpy(out + hs, data, n);
        }
    }
    buffer->count = start + hs + n;
    return true;
}

int co_ws_frame_deserialize(co_ws_frame_t* frame, const uint8_t* data, const size_t data_size,
                            size_t* index)
{
    size_t p = *index;
    const uint8_t b0 = data[p++];
    frame->header.fin = (b0 & 0x80u) != 0;
    frame->header.opcode = static_cast<uint8_t>(b0 & 0x7fu);
    if (frame->header.opcode > 0x0f) return CO_WS_ERROR_INVALID_FRAME;   // :139-142
    frame->header.payload_size = 0;
    frame->payload_data = nullptr;

    const uint8_t b1 = data[p++];
    const bool mask = (b1 & 0x80u) != 0;
    const uint8_t l7 = static_cast<uint8_t>(b1 & 0x7fu);
    if (l7 <= 125) {
        frame->header.payload_size = l7;
    } else {
        const size_t ext = (l7 == 126) ? 2 : 8;
        if (data_size - p < ext) return CO_WS_PARSE_MORE_DATA;           // :161-164, :176-179
        uint64_t v = 0;
        for (size_t i = 0; i < ext; ++i) v = (v << 8) | data[p + i];
        frame->header.payload_size = v;
        p += ext;
    }
    uint32_t key = 0;
    if (mask) {
        if (data_size - p < 4) return CO_WS_PARSE_MORE_DATA;             // :194-197
        key = static_cast<uint32_t>(data[p]) | static_cast<uint32_t>(data[p + 1]) << 8 |
              static_cast<uint32_t>(data[p + 2]) << 16 | static_cast<uint32_t>(data[p + 3]) << 24;
        p += 4;
    }
    const uint64_t n = frame->header.payload_size;
    if (static_cast<uint64_t>(data_size - p) < n) return CO_WS_PARSE_MORE_DATA;   // :203-206
    if (n > g_max_receive_payload_size) return CO_WS_ERROR_DATA_TOO_BIG;         // :208-213
    if (n > 0) {
        uint8_t* payload = static_cast<uint8_t*>(malloc(static_cast<size_t>(n) + 1));
        if (!payload) return CO_WS_ERROR_OUT_OF_MEMORY;
        payload[n] = 0;
        if (mask) {
            if (!payload_xor(data + p, payload, static_cast<size_t>(n), key)) {
                free(payload);
                return CO_WS_ERROR_OUT_OF_MEMORY;
            }
        } else {
            memcpy(payload, data + p, static_cast<size_t>(n));
        }
        frame->payload_data = payload;
        p += static_cast<size_t>(n);
    }
    *index = p;
    return CO_WS_PARSE_COMPLETE;
}

co_ws_frame_t* co_ws_frame_create(void)
{
    co_ws_frame_t* f = static_cast<co_ws_frame_t*>(malloc(sizeof(co_ws_frame_t)));
    if (!f) return nullptr;
    f->header.fin = false;
    f->header.opcode = 0xff;
    f->header.payload_size = 0;
    f->payload_data = nullptr;
    return f;
}

void co_ws_frame_destroy(co_ws_frame_t* frame)
{
    if (!frame) return;
    free(frame->payload_data);
    free(frame);
}

bool co_ws_frame_get_fin(const co_ws_frame_t* frame) { return frame->header.fin; }
uint8_t co_ws_frame_get_opcode(const co_ws_frame_t* frame) { return frame->header.opcode; }
uint64_t co_ws_frame_get_payload_size(const co_ws_frame_t* frame) { return frame->header.payload_size; }
const uint8_t* co_ws_frame_get_payload_data(const co_ws_frame_t* frame) { return frame->payload_data; }

void co_ws_config_set_max_receive_payload_size(size_t v) { g_max_receive_payload_size = v; }
size_t co_ws_config_get_max_receive_payload_size(void) { return g_max_receive_payload_size; }

void cfws_draw_mask_keys(size_t n, const uint8_t* mask_flags, uint32_t* keys)
{
    for (size_t i = 0; i < n; ++i) {
        uint32_t k = 0;
        if (!mask_flags || mask_flags[i])
            for (int j = 0; j < 4; ++j) k |= static_cast<uint32_t>(static_cast<uint8_t>(random() % 256)) << (8 * j);
        keys[i] = k;
    }
}

// The same keys from srandom(seed)'s stream, drawn on a private state
// (glibc's reentrant random_r over a 128-byte TYPE_3 table: the generator
// and seeding srandom uses on the default state), so no other thread's
// rand()/random() call can interleave with the draws, and the process's
// random() state is left alone.
int cfws_draw_mask_keys_seeded(uint32_t seed, size_t n, const uint8_t* mask_flags, uint32_t* keys)
{
    int32_t table[32];             // glibc reads the state as int32_t words
    struct random_data rd;
    memset(&rd, 0, sizeof rd);
    memset(table, 0, sizeof table);
    if (initstate_r(seed, reinterpret_cast<char*>(table), sizeof table, &rd) != 0) return CFWS_ERROR_INVALID_ARGUMENT;
    for (size_t i = 0; i < n; ++i) {
        uint32_t k = 0;
        if (!mask_flags || mask_flags[i]) {
            for (int j = 0; j < 4; ++j) {
                int32_t r = 0;
                (void)random_r(&rd, &r);
                k |= static_cast<uint32_t>(static_cast<uint8_t>(r % 256)) << (8 * j);
            }
        }
        keys[i] = k;
    }
    return CFWS_OK;
}

// Frees the calling thread's staging buffers and stream now (optional: a
// thread that exits without calling it hands them back for reuse by later
// threads instead).
void cfws_release_thread_resources(void)
{
    ThreadDevice& t_dev = t_slot.current();
    if (t_dev.svc_slot >= 0) service_give_slot(t_dev.device, t_dev.svc_slot);
    if (t_dev.buf) (void)hipFree(t_dev.buf);
    if (t_dev.host) (void)hipHostFree(t_dev.host);
    if (t_dev.stream) (void)hipStreamDestroy(t_dev.stream);
    t_slot.forget();
}

int cfws_bind_thread_device(int device)
{
    if (device < -1 || device >= kPoolDevices) return CFWS_ERROR_INVALID_ARGUMENT;
    if (device >= 0) {
        if (int rc = cfws_init_device(device)) return rc;
    }
    t_slot.bind(device);
    return CFWS_OK;
}

int cfws_thread_device(void) { return target_device(); }

void cfws_set_dropin_gpu_min(size_t bytes) { g_gpu_min.store(bytes, std::memory_order_relaxed); }
size_t cfws_dropin_gpu_min(void) { return g_gpu_min.load(std::memory_order_relaxed); }

}  // extern "C"
