// cfws_frame.cpp -- the drop-in per-frame ABI (include/cfws_co_ws_frame.h).
//
// Same symbols, prototypes, struct layouts and return codes as coldforce's
// src/ws/co_ws_frame.c + src/ws/co_ws_config.c, so libco_ws's callers
// (co_ws_send, the receive loops, the ws_http2 extension) link against this
// library unchanged. The payload XOR of a masked frame -- the reference's
// scalar byte loops at co_ws_frame.c:93-97 and :234-242 -- runs on the
// MI355X through cfws_xor_mask(); the 2-14 header bytes and the byte-array
// bookkeeping stay on the calling thread. Unmasked frames are plain copies
// in the reference too and stay plain copies here. There is no CPU XOR
// path: without a gfx950 device a masked frame fails (serialize returns
// false, deserialize CO_WS_ERROR_OUT_OF_MEMORY) and the reason goes to
// stderr and cfws_last_error().
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
    // the frame service (frames up to kCfwsServiceMax): a resident kernel on
    // svc_stream polling the mailbox; both in mapped pinned host memory
    uint64_t* mbox = nullptr;      // host address (cfws_internal.h: request, done, stop)
    uint64_t* mbox_dev = nullptr;
    uint8_t* svc_buf = nullptr;    // kCfwsServiceMax bytes, the frame is XORed here in place
    uint8_t* svc_buf_dev = nullptr;
    hipStream_t svc_stream = nullptr;
    uint32_t seq = 0;              // last request the service finished
    bool svc_running = false;      // a service kernel was launched and may still run
    bool svc_warm = false;         // first service frame done
    double svc_last = 0;           // when the last request finished (steady clock, s)
    bool holds() const { return stream || buf || host || mbox; }
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

// dst[i] = src[i] ^ key[i % 4] for a host buffer, through the device.
// ---- the frame service ---------------------------------------------------
// A masked frame of at most kCfwsServiceMax bytes (64 KiB) is XORed by a
// resident kernel (dropin_service_kernel, cfws_ops.hip): the host copies
// the frame into a mapped pinned buffer, posts one 64-bit request word
// (key, length, seq) and spins on the done word, which the kernel writes
// after its stores are released to system scope. No launch, no completion
// signal per frame: config 1's 1 KiB frames go from a launch + synchronise
// round trip to a PCIe round trip. The kernel exits
// by itself after an idle spell (CFWS_DROPIN_SERVICE_IDLE_US, default 2000)
// and is relaunched on the next frame; it is only ever relaunched after
// hipStreamQuery has seen the previous one finish, so at most one kernel
// serves a mailbox. CFWS_DROPIN_SERVICE=0 sends every frame through the
// launch path instead.
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

double service_idle_s()
{
    static const double v = [] {
        const char* s = getenv("CFWS_DROPIN_SERVICE_IDLE_US");
        const double us = s && *s ? strtod(s, nullptr) : 2000.0;
        return (us < 50.0 ? 50.0 : us) * 1e-6;
    }();
    return v;
}

double now_s()
{
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// Every mailbox ever created, so that process exit can tell the kernels to
// stop (a plain host store each; no HIP call at exit).
struct MailboxRegistry {
    std::mutex mu;
    std::vector<uint64_t*> boxes;
};

MailboxRegistry& mailboxes()
{
    static MailboxRegistry* r = new MailboxRegistry;
    return *r;
}

void stop_all_services()
{
    MailboxRegistry& r = mailboxes();
    std::lock_guard<std::mutex> lock(r.mu);
    for (uint64_t* m : r.boxes) __atomic_store_n(&m[2], uint64_t(1), __ATOMIC_RELEASE);
}

bool service_setup(ThreadDevice& t_dev, int dev)
{
    if (t_dev.mbox) return true;
    CurrentDevice on(dev);
    void* m = nullptr;
    void* b = nullptr;
    if (hipHostMalloc(&m, 4096, hipHostMallocMapped) != hipSuccess ||
        hipHostMalloc(&b, kCfwsServiceMax, hipHostMallocMapped) != hipSuccess) {
        fprintf(stderr, "cfws: frame service: hipHostMalloc failed\n");
        if (m) (void)hipHostFree(m);
        if (b) (void)hipHostFree(b);
        return false;
    }
    void* md = nullptr;
    void* bd = nullptr;
    if (hipHostGetDevicePointer(&md, m, 0) != hipSuccess || hipHostGetDevicePointer(&bd, b, 0) != hipSuccess ||
        hipStreamCreateWithFlags(&t_dev.svc_stream, hipStreamNonBlocking) != hipSuccess) {
        fprintf(stderr, "cfws: frame service: mapping or stream failed\n");
        (void)hipHostFree(m);
        (void)hipHostFree(b);
        t_dev.svc_stream = nullptr;
        return false;
    }
    memset(m, 0, 4096);
    t_dev.mbox = static_cast<uint64_t*>(m);
    t_dev.mbox_dev = static_cast<uint64_t*>(md);
    t_dev.svc_buf = static_cast<uint8_t*>(b);
    t_dev.svc_buf_dev = static_cast<uint8_t*>(bd);
    t_dev.seq = 0;
    t_dev.svc_running = false;
    static std::once_flag exit_hook;
    std::call_once(exit_hook, [] { atexit(stop_all_services); });
    MailboxRegistry& r = mailboxes();
    std::lock_guard<std::mutex> lock(r.mu);
    r.boxes.push_back(t_dev.mbox);
    return true;
}

bool service_launch(ThreadDevice& t_dev, int dev)
{
    int rate_khz = 0;
    if (hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess || rate_khz <= 0)
        rate_khz = 100000;
    const uint64_t idle_ticks = (uint64_t)(service_idle_s() * 1e3 * (double)rate_khz);
    __atomic_store_n(&t_dev.mbox[2], uint64_t(0), __ATOMIC_RELEASE);
    CurrentDevice on(dev);
    if (cfws_internal_service_launch(t_dev.mbox_dev, t_dev.svc_buf_dev, idle_ticks, t_dev.seq, t_dev.svc_stream) !=
        CFWS_OK)
        return false;
    t_dev.svc_running = true;
    return true;
}

// Has the service kernel finished (idled out)? hipStreamQuery on its stream.
bool service_finished(ThreadDevice& t_dev)
{
    const hipError_t e = hipStreamQuery(t_dev.svc_stream);
    if (e == hipErrorNotReady) return false;
    if (e != hipSuccess) fprintf(stderr, "cfws: frame service: %s\n", hipGetErrorString(e));
    return true;
}

bool service_xor(ThreadDevice& t_dev, int dev, const uint8_t* src, uint8_t* dst, size_t n, uint32_t key)
{
    if (!service_setup(t_dev, dev)) return false;
    // the kernel idles out service_idle_s() after its last request: well
    // inside that, it is still polling; past half of it, ask the stream
    if (t_dev.svc_running && now_s() - t_dev.svc_last > 0.5 * service_idle_s() && service_finished(t_dev))
        t_dev.svc_running = false;
    memcpy(t_dev.svc_buf, src, n);
    uint32_t seq = (t_dev.seq + 1) & 0xffffu;
    const uint64_t word = (uint64_t)key | ((uint64_t)(n - 1) << 32) | ((uint64_t)seq << 48);
    __atomic_store_n(&t_dev.mbox[0], word, __ATOMIC_RELEASE);
    if (!t_dev.svc_running && !service_launch(t_dev, dev)) return false;
    const double t0 = now_s();
    for (uint64_t spin = 1;; ++spin) {
        if ((uint32_t)(__atomic_load_n(&t_dev.mbox[1], __ATOMIC_ACQUIRE) >> 48) == seq) break;
        if ((spin & 1023u) == 0) {
            const double dt = now_s() - t0;
            if (dt > 5.0) {
                fprintf(stderr, "cfws: frame service: no answer in 5 s\n");
                return false;
            }
            // an exit that raced the request: relaunch once the old kernel
            // has finished (never two kernels on one mailbox)
            if (dt > 20e-6 && service_finished(t_dev) &&
                (uint32_t)(__atomic_load_n(&t_dev.mbox[1], __ATOMIC_ACQUIRE) >> 48) != seq &&
                !service_launch(t_dev, dev))
                return false;
        }
        __builtin_ia32_pause();
    }
    t_dev.seq = seq;
    t_dev.svc_last = now_s();
    memcpy(dst, t_dev.svc_buf, n);
    return true;
}

std::atomic<bool> g_runtime_up{false};   // the HIP runtime has been initialised by us

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
        if (!service_xor(t_dev, dev, src, dst, n, key)) return false;
        t_dev.svc_warm = true;
        return true;
    }
    const bool zero_copy = n <= zero_copy_max();
    if (!t_dev.stream || (zero_copy ? (!t_dev.zc_warm || t_dev.host_cap < n) : (!t_dev.dma_warm || t_dev.cap < n)))
        keep_random_stream.engage();
    {
        CurrentDevice on(dev);
        if (zero_copy ? !host_stage(t_dev, n) : !device_stage(t_dev, n)) return false;
    }
    hipStream_t st = t_dev.stream;
    if (zero_copy) {
        memcpy(t_dev.host, src, n);
        if (cfws_xor_mask(t_dev.host_dev, t_dev.host_dev, n, key, 0, st) != CFWS_OK) return false;
    } else {
        if (hipMemcpyAsync(t_dev.buf, src, n, hipMemcpyHostToDevice, st) != hipSuccess) return false;
        if (cfws_xor_mask(t_dev.buf, t_dev.buf, n, key, 0, st) != CFWS_OK) return false;
        if (hipMemcpyAsync(dst, t_dev.buf, n, hipMemcpyDeviceToHost, st) != hipSuccess) return false;
    }
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
            if (!device_xor(static_cast<const uint8_t*>(data), out + hs, n, key)) return false;
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
            if (!device_xor(data + p, payload, static_cast<size_t>(n), key)) {
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
    if (t_dev.mbox) {
        __atomic_store_n(&t_dev.mbox[2], uint64_t(1), __ATOMIC_RELEASE);
        if (t_dev.svc_stream) (void)hipStreamSynchronize(t_dev.svc_stream);
        {
            MailboxRegistry& r = mailboxes();
            std::lock_guard<std::mutex> lock(r.mu);
            for (auto& m : r.boxes)
                if (m == t_dev.mbox) {
                    m = r.boxes.back();
                    r.boxes.pop_back();
                    break;
                }
        }
        (void)hipHostFree(t_dev.mbox);
        if (t_dev.svc_buf) (void)hipHostFree(t_dev.svc_buf);
        if (t_dev.svc_stream) (void)hipStreamDestroy(t_dev.svc_stream);
    }
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

}  // extern "C"
