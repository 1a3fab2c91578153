// cfws_pipeline.cpp -- host-memory batch codec (include/cfws.h, cfws_pipeline_*).
//
// coldforce's frames start and end in host memory: socket receive buffers
// (co_tcp_receive_all, src/net/co_tcp_client.c:695-721) and send buffers
// (co_ws_send -> module.send, src/ws/co_ws_client.c:427-460). This pipeline
// runs the device batch codec over host buffers: the batch is cut into
// chunks of frames, and `depth` slots, each with its own stream and device
// staging, overlap H2D copies, the plan + streaming kernels and D2H copies of
// consecutive chunks (the two DMA directions run concurrently). H2D copies go
// in chunk order on one copy stream of the pipeline's, each waiting only for
// its slot's previous execute (the input staging free), never for a D2H: on a
// slot's own stream the next chunk's H2D would queue behind the slot's D2H,
// and all slots then alternate between an H2D burst and a D2H burst (half
// duplex). D2H copies stay on the slot streams (one shared
// in-order D2H stream measured no faster). The host
// buffers should be pinned (hipHostMalloc / hipHostRegister) for full PCIe
// rate. All codec decisions (header encode/decode, layout, status codes) are
// the device plan's; the host only cuts chunks and rebases offsets.
#include <hip/hip_runtime.h>

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "cfws.h"
#include "cfws_internal.h"

namespace {

constexpr int kMaxDepth = 4;

struct Slot {
    hipStream_t st = nullptr;
    void* d_in = nullptr;              // chunk source (payload or wire)
    void* d_out = nullptr;             // chunk output
    cfws_frame_desc_t* d_desc = nullptr;
    int32_t* d_status = nullptr;
    uint64_t* d_index = nullptr;
    uint64_t* d_total = nullptr;
    void* d_ws = nullptr;
    size_t ws_size = 0;
    void* h_stage = nullptr;           // pinned: descriptors / index / status staging
    uint64_t* h_total = nullptr;       // pinned
    hipEvent_t ev_done = nullptr;      // slot free again (its last D2H finished)
    hipEvent_t ev_total = nullptr;     // the chunk's layout total is on the host
    hipEvent_t ev_in = nullptr;        // the chunk's H2D copies landed (host staging free)
    hipEvent_t ev_exec = nullptr;      // the chunk's kernels finished (d_in / d_index free)
    // HTTP/2 (cfws_pipeline_h2_*), allocated at first use: WS wire / pool
    // scratch, message statuses and the HTTP/2 workspace
    void* d_aux = nullptr;
    int32_t* d_status2 = nullptr;
    void* d_ws2 = nullptr;
    size_t ws2_size = 0;
};

uint32_t hdr_size(uint64_t n, bool mask)
{
    return 2u + (n > 65535u ? 8u : (n > 125u ? 2u : 0u)) + (mask ? 4u : 0u);
}

int fail(const char* what, hipError_t e = hipSuccess)
{
    fprintf(stderr, "cfws pipeline: %s%s%s\n", what, e == hipSuccess ? "" : ": ",
            e == hipSuccess ? "" : hipGetErrorString(e));
    return e == hipSuccess ? CFWS_ERROR_INVALID_ARGUMENT : CFWS_ERROR_HIP;
}

// Device address of the pipeline's host output when its D2H leg is a kernel
// (copy_out_kernel storing into mapped pinned memory), NULL for an SDMA copy.
// Measured per direction with the H2D copies on their own stream (config 2,
// host to host): serialize 40 GiB/s with the kernel against 22
// with SDMA; deserialize 44 GiB/s with SDMA against 35 with the kernel. So
// CFWS_PIPELINE_D2H_AUTO takes the kernel for serialize when its wire arena
// is mapped and always copies for deserialize.
uint8_t* kernel_d2h_target(int mode, void* h_out, bool serialize)
{
    if (mode == CFWS_PIPELINE_D2H_DMA || (mode == CFWS_PIPELINE_D2H_AUTO && !serialize)) return nullptr;
    return static_cast<uint8_t*>(cfws_mapped_device_pointer(h_out));
}

// The default mode: CFWS_PIPELINE_D2H=dma | kernel | auto (unset: auto).
int default_d2h_mode()
{
    const char* s = getenv("CFWS_PIPELINE_D2H");
    if (s && strcmp(s, "dma") == 0) return CFWS_PIPELINE_D2H_DMA;
    if (s && strcmp(s, "kernel") == 0) return CFWS_PIPELINE_D2H_KERNEL;
    return CFWS_PIPELINE_D2H_AUTO;
}

#define CFWS_HIP(call)                                   \
    do {                                                 \
        hipError_t e_ = (call);                          \
        if (e_ != hipSuccess) return fail(#call, e_);    \
    } while (0)

}  // namespace

struct cfws_pipeline {
    hipStream_t st_in = nullptr;       // every H2D copy, in chunk order
    int d2h_mode = CFWS_PIPELINE_D2H_AUTO;
    int depth = 0;
    uint64_t chunk = 0;        // staging bytes per slot and direction
    size_t max_frames = 0;     // frames per chunk
    Slot slot[kMaxDepth];
};

extern "C" {

int cfws_pipeline_create(uint64_t chunk_bytes, size_t max_frames, int depth, cfws_pipeline_t** out)
{
    if (int rc = cfws_init()) return rc;
    if (!out || depth < 1 || depth > kMaxDepth || chunk_bytes < 4096 || max_frames == 0)
        return fail("bad pipeline parameters");
    auto* p = new cfws_pipeline;
    p->depth = depth;
    p->chunk = (chunk_bytes + 255) & ~uint64_t(255);
    p->max_frames = max_frames;
    p->d2h_mode = default_d2h_mode();
    // The deserialize output of a chunk can exceed its wire bytes only by
    // the alignment padding; reserve one 4 KiB pad per frame at most.
    const uint64_t out_bytes = p->chunk + 64;
    if (hipStreamCreateWithFlags(&p->st_in, hipStreamNonBlocking) != hipSuccess) {
        cfws_pipeline_destroy(p);
        return fail("pipeline allocation failed");
    }
    for (int s = 0; s < depth; ++s) {
        Slot& S = p->slot[s];
        S.ws_size = cfws_workspace_size(max_frames, out_bytes);
        if (hipStreamCreateWithFlags(&S.st, hipStreamNonBlocking) != hipSuccess ||
            hipMalloc(&S.d_in, p->chunk + 64) != hipSuccess ||
            hipMalloc(&S.d_out, out_bytes) != hipSuccess ||
            hipMalloc(&S.d_desc, max_frames * sizeof(cfws_frame_desc_t)) != hipSuccess ||
            hipMalloc(&S.d_status, max_frames * sizeof(int32_t)) != hipSuccess ||
            hipMalloc(&S.d_index, max_frames * sizeof(uint64_t)) != hipSuccess ||
            hipMalloc(&S.d_total, 64) != hipSuccess ||
            hipMalloc(&S.d_ws, S.ws_size) != hipSuccess ||
            hipHostMalloc(&S.h_stage, max_frames * (sizeof(cfws_frame_desc_t) + 2 * sizeof(int32_t))) != hipSuccess ||
            hipHostMalloc(reinterpret_cast<void**>(&S.h_total), 64) != hipSuccess ||
            hipEventCreateWithFlags(&S.ev_done, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&S.ev_total, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&S.ev_in, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&S.ev_exec, hipEventDisableTiming) != hipSuccess) {
            cfws_pipeline_destroy(p);
            return fail("pipeline allocation failed");
        }
        (void)hipEventRecord(S.ev_done, S.st);
        (void)hipEventRecord(S.ev_exec, S.st);
        (void)hipEventRecord(S.ev_in, p->st_in);
    }
    *out = p;
    return CFWS_OK;
}

void cfws_pipeline_destroy(cfws_pipeline_t* p)
{
    if (!p) return;
    if (p->st_in) (void)hipStreamSynchronize(p->st_in);
    for (int s = 0; s < kMaxDepth; ++s) {
        Slot& S = p->slot[s];
        if (S.st) (void)hipStreamSynchronize(S.st);
        if (S.d_in) (void)hipFree(S.d_in);
        if (S.d_out) (void)hipFree(S.d_out);
        if (S.d_desc) (void)hipFree(S.d_desc);
        if (S.d_status) (void)hipFree(S.d_status);
        if (S.d_index) (void)hipFree(S.d_index);
        if (S.d_total) (void)hipFree(S.d_total);
        if (S.d_ws) (void)hipFree(S.d_ws);
        if (S.h_stage) (void)hipHostFree(S.h_stage);
        if (S.h_total) (void)hipHostFree(S.h_total);
        if (S.ev_done) (void)hipEventDestroy(S.ev_done);
        if (S.ev_total) (void)hipEventDestroy(S.ev_total);
        if (S.d_aux) (void)hipFree(S.d_aux);
        if (S.d_status2) (void)hipFree(S.d_status2);
        if (S.d_ws2) (void)hipFree(S.d_ws2);
        if (S.ev_in) (void)hipEventDestroy(S.ev_in);
        if (S.ev_exec) (void)hipEventDestroy(S.ev_exec);
        if (S.st) (void)hipStreamDestroy(S.st);
    }
    if (p->st_in) (void)hipStreamDestroy(p->st_in);
    delete p;
}

int cfws_pipeline_set_d2h(cfws_pipeline_t* p, int mode)
{
    if (!p || mode < CFWS_PIPELINE_D2H_AUTO || mode > CFWS_PIPELINE_D2H_KERNEL) return fail("bad D2H mode");
    p->d2h_mode = mode;
    return CFWS_OK;
}

// co_ws_frame_serialize over a host batch: host payload arena -> host wire
// arena. h_desc is updated like cfws_serialize_plan updates d_desc.
int cfws_pipeline_serialize(cfws_pipeline_t* p, const void* h_payload, cfws_frame_desc_t* h_desc,
                            size_t n, void* h_wire, uint64_t wire_capacity, uint64_t* wire_total)
{
    const CfwsPassScope pass_scope;
    (void)cfws_internal_take_pass();   // not timed (cfws_time_next_pass): the pair is dropped
    if (!p || (n && (!h_payload || !h_desc || !h_wire))) return fail("null argument");
    // Layout on the host copy of the descriptors (same rule as the device
    // plan) so that chunks can be cut by wire bytes.
    uint64_t off = 0;
    for (size_t i = 0; i < n; ++i) {
        h_desc[i].header_size = (uint8_t)hdr_size(h_desc[i].payload_size, h_desc[i].mask != 0);
        h_desc[i].wire_off = off;
        off += h_desc[i].header_size + h_desc[i].payload_size;
    }
    if (wire_total) *wire_total = off;
    const uint8_t* src = static_cast<const uint8_t*>(h_payload);
    uint8_t* dst = static_cast<uint8_t*>(h_wire);
    uint8_t* dst_dev = n ? kernel_d2h_target(p->d2h_mode, h_wire, true) : nullptr;
    size_t i = 0;
    int c = 0;
    while (i < n) {
        // chunk = frames [i, j): source span and wire bytes within the staging
        uint64_t lo = h_desc[i].payload_off, hi = lo + h_desc[i].payload_size;
        size_t j = i;
        while (j < n && j - i < p->max_frames) {
            const uint64_t a = std::min(lo, (uint64_t)h_desc[j].payload_off);
            const uint64_t b = std::max(hi, (uint64_t)(h_desc[j].payload_off + h_desc[j].payload_size));
            const uint64_t wire = h_desc[j].wire_off + h_desc[j].header_size + h_desc[j].payload_size -
                                  h_desc[i].wire_off;
            if (j > i && ((b - (a & ~uint64_t(15))) > p->chunk || wire > p->chunk)) break;
            lo = a;
            hi = b;
            ++j;
        }
        const uint64_t src_lo = lo & ~uint64_t(15);
        const uint64_t wire_lo = h_desc[i].wire_off;
        const uint64_t wire_bytes = h_desc[j - 1].wire_off + h_desc[j - 1].header_size +
                                    h_desc[j - 1].payload_size - wire_lo;
        if (hi - src_lo > p->chunk || wire_bytes > p->chunk)
            return fail("a frame is larger than the pipeline chunk");
        Slot& S = p->slot[c % p->depth];
        CFWS_HIP(hipEventSynchronize(S.ev_in));       // the slot's last H2D read the staging
        auto* stage = static_cast<cfws_frame_desc_t*>(S.h_stage);
        for (size_t k = i; k < j; ++k) {
            stage[k - i] = h_desc[k];
            stage[k - i].payload_off -= src_lo;
        }
        CFWS_HIP(hipStreamWaitEvent(p->st_in, S.ev_exec, 0));   // d_in, d_desc free
        CFWS_HIP(hipMemcpyAsync(S.d_in, src + src_lo, hi - src_lo, hipMemcpyHostToDevice, p->st_in));
        CFWS_HIP(hipMemcpyAsync(S.d_desc, stage, (j - i) * sizeof(cfws_frame_desc_t),
                                hipMemcpyHostToDevice, p->st_in));
        CFWS_HIP(hipEventRecord(S.ev_in, p->st_in));
        CFWS_HIP(hipStreamWaitEvent(S.st, S.ev_in, 0));
        if (int rc = cfws_serialize_batch(S.d_in, S.d_desc, j - i, S.d_out, p->chunk + 64, S.d_total,
                                          S.d_ws, S.ws_size, S.st))
            return rc;
        CFWS_HIP(hipEventRecord(S.ev_exec, S.st));
        if (wire_lo < wire_capacity) {
            const uint64_t m = std::min(wire_bytes, wire_capacity - wire_lo);
            if (dst_dev) {
                if (int rc = cfws_internal_copy_out(S.d_out, dst_dev + wire_lo, m, S.st)) return rc;
            } else {
                CFWS_HIP(hipMemcpyAsync(dst + wire_lo, S.d_out, m, hipMemcpyDeviceToHost, S.st));
            }
        }
        CFWS_HIP(hipEventRecord(S.ev_done, S.st));
        i = j;
        ++c;
    }
    CFWS_HIP(hipStreamSynchronize(p->st_in));
    for (int s = 0; s < p->depth; ++s) CFWS_HIP(hipStreamSynchronize(p->slot[s].st));
    return CFWS_OK;
}

// co_ws_frame_deserialize at every h_index[i] of a host wire buffer: header
// decode, status, copy + unmask into the host payload arena laid out as
// cfws_deserialize_plan lays it out (flags must be 0: the reassembly layout
// puts control frames after ALL data, which a chunked pass cannot know).
// Precondition (what a receive loop's index satisfies): h_index increasing
// and every frame ending at or before the next frame's start.
}  // extern "C"

namespace {

// The frame starts a chunked deserialize consumes: a caller's index, or the
// receive loop's walk (cfws_index_frames, co_ws_server.c:107-169) run in
// steps just ahead of the chunks, so the host walks chunk c + 1's frames
// while the device copies and decodes chunk c (the walk is a chain of
// dependent reads through host memory, ~100 ns per frame).
struct StartSource {
    const uint64_t* fixed = nullptr;     // a caller's index of n_fixed starts
    size_t n_fixed = 0;
    const void* buf = nullptr;           // or the walk over buf[pos, end)
    uint64_t end = 0, max_payload = 0, pos = 0;
    size_t cap = 0;                      // at most this many starts
    std::vector<uint64_t> walked;
    int32_t stop = CFWS_PARSE_COMPLETE;
    bool done = true;
    static constexpr size_t kStep = 2048;

    // Does start k exist? (walks on until it is known)
    bool has(size_t k)
    {
        if (fixed) return k < n_fixed;
        while (k >= walked.size() && !done) step();
        return k < walked.size();
    }
    uint64_t at(size_t k) const { return fixed ? fixed[k] : walked[k]; }
    // Where the last frame's bytes end (has() said there is no next start):
    // the walk's stop, so trailing incomplete bytes are never staged.
    uint64_t last_end(uint64_t wire_size) const { return fixed ? wire_size : std::min(pos, wire_size); }
    // Stepwise walks end as one walk over the whole buffer would:
    // CFWS_INDEX_FULL only when another COMPLETE frame follows.
    void step()
    {
        const size_t at0 = walked.size();
        const size_t room = std::min(kStep, cap - at0);
        walked.resize(at0 + room);
        uint64_t used = pos;
        int32_t why = CFWS_PARSE_COMPLETE;
        const size_t got = cfws_index_frames(buf, pos, end, max_payload, walked.data() + at0, room,
                                             &used, &why);
        walked.resize(at0 + got);
        pos = used;
        stop = why;
        if (why != CFWS_INDEX_FULL || walked.size() == cap) done = true;
    }
};

int pipeline_deserialize(cfws_pipeline_t* p, const void* h_wire, uint64_t wire_size, StartSource& idx,
                         uint64_t max_payload, uint32_t align, cfws_frame_desc_t* h_desc,
                         int32_t* h_status, void* h_payload, uint64_t payload_capacity,
                         uint64_t* payload_total)
{
    const uint8_t* src = static_cast<const uint8_t*>(h_wire);
    uint8_t* dst = static_cast<uint8_t*>(h_payload);
    uint8_t* dst_dev = idx.has(0) ? kernel_d2h_target(p->d2h_mode, h_payload, false) : nullptr;

    struct Chunk { size_t i, j; int slot; uint64_t wire_lo, base; };
    std::vector<Chunk> pend;         // launched; layout total not read yet
    std::vector<Chunk> landing;      // D2H enqueued; descriptors not rebased yet
    uint64_t base = 0;               // payload bytes laid out by earlier chunks
    uint64_t out_slot = p->chunk + 64;

    // Chunk k's layout total is known: enqueue the D2H of its payload,
    // descriptors and status, and move the payload base on. Does not wait
    // for the copies, so the next chunk's kernels overlap them.
    auto settle = [&](Chunk k) -> int {
        Slot& S = p->slot[k.slot];
        CFWS_HIP(hipEventSynchronize(S.ev_total));
        const uint64_t tot = *S.h_total;          // unclamped chunk layout bytes
        if (base < payload_capacity && tot) {
            const uint64_t m = std::min(tot, payload_capacity - base);
            if (dst_dev) {
                if (int rc = cfws_internal_copy_out(S.d_out, dst_dev + base, m, S.st)) return rc;
            } else {
                CFWS_HIP(hipMemcpyAsync(dst + base, S.d_out, m, hipMemcpyDeviceToHost, S.st));
            }
        }
        auto* sdesc = static_cast<cfws_frame_desc_t*>(S.h_stage);
        auto* sstat = reinterpret_cast<int32_t*>(sdesc + p->max_frames);
        CFWS_HIP(hipMemcpyAsync(sdesc, S.d_desc, (k.j - k.i) * sizeof(cfws_frame_desc_t),
                                hipMemcpyDeviceToHost, S.st));
        CFWS_HIP(hipMemcpyAsync(sstat, S.d_status, (k.j - k.i) * sizeof(int32_t),
                                hipMemcpyDeviceToHost, S.st));
        CFWS_HIP(hipEventRecord(S.ev_done, S.st));
        k.base = base;
        base += tot;
        landing.push_back(k);
        return CFWS_OK;
    };
    // Chunk k's copies have landed: rebase its descriptors into the caller's.
    auto finish = [&](const Chunk& k) -> int {
        Slot& S = p->slot[k.slot];
        CFWS_HIP(hipEventSynchronize(S.ev_done));
        const auto* sdesc = static_cast<const cfws_frame_desc_t*>(S.h_stage);
        const auto* sstat = reinterpret_cast<const int32_t*>(sdesc + p->max_frames);
        for (size_t f = k.i; f < k.j; ++f) {
            h_desc[f] = sdesc[f - k.i];
            h_desc[f].wire_off += k.wire_lo;
            h_desc[f].payload_off += k.base;
            h_status[f] = sstat[f - k.i];
        }
        return CFWS_OK;
    };
    auto settle_all = [&]() -> int {
        for (const Chunk& k : pend)
            if (int rc = settle(k)) return rc;
        pend.clear();
        return CFWS_OK;
    };

    size_t i = 0;
    int c = 0;
    while (idx.has(i)) {
        const uint64_t lo = std::min(idx.at(i), wire_size);
        // a frame's bytes end at the next frame's start (the index precondition)
        auto end_of = [&](size_t k) {
            return idx.has(k + 1) ? std::min(idx.at(k + 1), wire_size) : idx.last_end(wire_size);
        };
        // frames [i, j): their wire bytes plus the worst-case alignment
        // padding of their payloads must fit the slot's staging
        size_t j = i + 1;
        while (idx.has(j) && j - i < p->max_frames &&
               end_of(j) - (lo & ~uint64_t(15)) + (j + 1 - i) * uint64_t(align - 1) <= p->chunk)
            ++j;
        const uint64_t hi = end_of(j - 1);
        const uint64_t wire_lo = lo & ~uint64_t(15);
        if (hi - wire_lo + (j - i) * uint64_t(align - 1) > p->chunk)
            return fail("a frame is larger than the pipeline chunk");
        const int s = c % p->depth;
        Slot& S = p->slot[s];
        // slot reuse: its previous chunk must have landed (staging reused)
        for (size_t q = 0; q < pend.size(); ++q)
            if (pend[q].slot == s) {
                if (int rc = settle_all()) return rc;
                break;
            }
        for (size_t q = 0; q < landing.size(); ++q)
            if (landing[q].slot == s) {
                for (size_t r = 0; r <= q; ++r)
                    if (int rc = finish(landing[r])) return rc;
                landing.erase(landing.begin(), landing.begin() + q + 1);
                break;
            }
        // the staging's last reader, this slot's previous chunk, was finished above
        auto* sidx = static_cast<uint64_t*>(S.h_stage);
        for (size_t k = i; k < j; ++k) sidx[k - i] = idx.at(k) - wire_lo;
        CFWS_HIP(hipStreamWaitEvent(p->st_in, S.ev_exec, 0));   // d_in, d_index free
        CFWS_HIP(hipMemcpyAsync(S.d_in, src + wire_lo, hi - wire_lo, hipMemcpyHostToDevice, p->st_in));
        CFWS_HIP(hipMemcpyAsync(S.d_index, sidx, (j - i) * sizeof(uint64_t), hipMemcpyHostToDevice,
                                p->st_in));
        CFWS_HIP(hipEventRecord(S.ev_in, p->st_in));
        CFWS_HIP(hipStreamWaitEvent(S.st, S.ev_in, 0));
        // The capacity rule needs this chunk's payload base: everything laid
        // out before it must be known (settle all pending chunks first).
        if (int rc = settle_all()) return rc;
        const uint64_t cap = base >= payload_capacity ? 0 : std::min(out_slot, payload_capacity - base);
        // cap == 0 (capacity exhausted): the plan marks every non-empty
        // COMPLETE frame OUT_OF_MEMORY, exactly the batch rule.
        if (int rc = cfws_deserialize_batch(S.d_in, hi - wire_lo, S.d_index, j - i, max_payload,
                                            align, 0, S.d_desc, S.d_status, S.d_out, cap,
                                            S.d_total, S.d_ws, S.ws_size, S.st))
            return rc;
        CFWS_HIP(hipEventRecord(S.ev_exec, S.st));
        // the unclamped layout total: offsets keep counting past the capacity
        CFWS_HIP(hipMemcpyAsync(S.h_total,
                                static_cast<char*>(S.d_ws) + cfws_internal_grand_total_offset(), 8,
                                hipMemcpyDeviceToHost, S.st));
        CFWS_HIP(hipEventRecord(S.ev_total, S.st));
        pend.push_back(Chunk{i, j, s, wire_lo, 0});
        i = j;
        ++c;
    }
    if (int rc = settle_all()) return rc;
    for (const Chunk& k : landing)
        if (int rc = finish(k)) return rc;
    if (payload_total) *payload_total = std::min(base, payload_capacity);
    return CFWS_OK;
}

}  // namespace

extern "C" {

int cfws_pipeline_deserialize(cfws_pipeline_t* p, const void* h_wire, uint64_t wire_size,
                              const uint64_t* h_index, size_t n, uint64_t max_payload,
                              uint32_t align, uint32_t flags, cfws_frame_desc_t* h_desc,
                              int32_t* h_status, void* h_payload, uint64_t payload_capacity,
                              uint64_t* payload_total)
{
    const CfwsPassScope pass_scope;
    (void)cfws_internal_take_pass();   // not timed (cfws_time_next_pass): the pair is dropped
    if (!p || (n && (!h_wire || !h_index || !h_desc || !h_status || !h_payload)))
        return fail("null argument");
    if (flags != 0) return fail("the pipeline supports flags = 0 only");
    if (align == 0 || (align & (align - 1)) || align > 4096) return fail("bad align");
    for (size_t i = 1; i < n; ++i)
        if (h_index[i] < h_index[i - 1]) return fail("frame index must be increasing");
    StartSource idx;
    idx.fixed = h_index;
    idx.n_fixed = n;
    return pipeline_deserialize(p, h_wire, wire_size, idx, max_payload, align, h_desc, h_status,
                                h_payload, payload_capacity, payload_total);
}

int cfws_pipeline_receive(cfws_pipeline_t* p, const void* h_wire, uint64_t begin, uint64_t end,
                          uint64_t max_payload, uint32_t align, cfws_frame_desc_t* h_desc,
                          int32_t* h_status, size_t* n_frames, uint64_t* consumed, int32_t* stop,
                          void* h_payload, uint64_t payload_capacity, uint64_t* payload_total)
{
    const CfwsPassScope pass_scope;
    (void)cfws_internal_take_pass();   // not timed (cfws_time_next_pass): the pair is dropped
    if (!p || !n_frames || (end > begin && !h_wire)) return fail("null argument");
    if (*n_frames && (!h_desc || !h_status || !h_payload)) return fail("null argument");
    if (align == 0 || (align & (align - 1)) || align > 4096) return fail("bad align");
    // the receive loop's walk (co_ws_server.c:107-169) on the host, where the
    // bytes are, a step ahead of the chunked device deserialize it drives.
    // Every walked frame is COMPLETE inside [begin, consumed): the walk stops
    // before an incomplete or invalid frame, whose bytes are never staged.
    StartSource idx;
    idx.buf = h_wire;
    idx.pos = begin;
    idx.end = end;
    idx.max_payload = max_payload;
    idx.cap = *n_frames;
    idx.done = false;
    idx.walked.reserve(std::min(*n_frames, size_t(1) << 20));
    const int rc = pipeline_deserialize(p, h_wire, end, idx, max_payload, align, h_desc, h_status,
                                        h_payload, payload_capacity, payload_total);
    while (!idx.done) idx.step();       // an error above may leave the walk short
    *n_frames = idx.walked.size();
    if (consumed) *consumed = idx.pos;
    if (stop) *stop = idx.stop;
    return rc;
}

}  // extern "C"

// ---- WebSocket over HTTP/2 through host memory -----------------------------

namespace {

uint64_t data_frames(uint64_t W, uint64_t S) { return W <= S ? 1 : (W + S - 1) / S; }

// A slot's HTTP/2 resources, allocated at first use: WS wire / pool scratch,
// message statuses, and an HTTP/2 workspace of at least ws_bytes.
int h2_slot(cfws_pipeline* p, Slot& S, size_t ws_bytes)
{
    if (!S.d_aux && hipMalloc(&S.d_aux, p->chunk + 64) != hipSuccess)
        return fail("pipeline allocation failed");
    if (!S.d_status2 && hipMalloc(&S.d_status2, p->max_frames * sizeof(int32_t)) != hipSuccess)
        return fail("pipeline allocation failed");
    if (S.ws2_size < ws_bytes) {
        if (S.d_ws2) {
            (void)hipStreamSynchronize(S.st);
            (void)hipFree(S.d_ws2);
            S.d_ws2 = nullptr;
            S.ws2_size = 0;
        }
        if (hipMalloc(&S.d_ws2, ws_bytes) != hipSuccess) return fail("pipeline allocation failed");
        S.ws2_size = ws_bytes;
    }
    return CFWS_OK;
}

// The HTTP/2 frame at s of h2[0, size) as the device parse decides it
// (co_http2_frame.c:211-300: MORE_DATA under 9 bytes or a short payload,
// PARSE_ERROR over max_frame_size or bad padding, NOT_DATA for other types):
// restated here because the receive pipeline cuts its chunks where no
// message is open. *pooled = the DATA payload bytes it adds to the pool.
int32_t h2_frame_host(const uint8_t* h2, uint64_t size, uint64_t s, uint64_t max_frame,
                      uint64_t* pooled, bool* end_stream)
{
    *pooled = 0;
    *end_stream = false;
    if (s > size || size - s < 9) return CFWS_H2_PARSE_MORE_DATA;
    const uint64_t len = (uint64_t)h2[s] << 16 | (uint64_t)h2[s + 1] << 8 | h2[s + 2];
    if (len > max_frame) return CFWS_H2_PARSE_ERROR;
    if (size - s - 9 < len) return CFWS_H2_PARSE_MORE_DATA;
    const uint32_t type = h2[s + 3], flags = h2[s + 4];
    if (type != 0) return CFWS_H2_NOT_DATA;
    uint64_t pad = 0, hs = 9;
    if (flags & 0x8u) {                                   // PADDED
        if (len < 1) return CFWS_H2_PARSE_ERROR;
        pad = h2[s + 9];
        hs = 10;
        if (pad + 1 > len) return CFWS_H2_PARSE_ERROR;
    }
    *pooled = len - (hs - 9) - pad;
    *end_stream = (flags & 0x1u) != 0;
    return CFWS_H2_PARSE_COMPLETE;
}

}  // namespace

extern "C" {

// co_http2_stream_send_ws_frame over a host batch (cfws_h2_serialize_batch
// per chunk of WS frames): host payload arena -> host DATA-frame stream.
// h_desc gets header_size / wire_off as cfws_serialize_plan writes them.
int cfws_pipeline_h2_serialize(cfws_pipeline_t* p, const void* h_payload, cfws_frame_desc_t* h_desc,
                               size_t n, uint32_t stream_id, uint32_t max_frame_size, void* h_h2,
                               uint64_t h2_capacity, uint64_t* h2_total)
{
    const CfwsPassScope pass_scope;
    (void)cfws_internal_take_pass();   // not timed (cfws_time_next_pass): the pair is dropped
    if (!p || (n && (!h_payload || !h_desc || !h_h2))) return fail("null argument");
    const uint64_t mfs = max_frame_size ? max_frame_size : CFWS_H2_DEFAULT_MAX_FRAME_SIZE;
    // the WS layout (as cfws_serialize_plan) and each frame's DATA-stream bytes
    uint64_t woff = 0, total = 0;
    for (size_t f = 0; f < n; ++f) {
        const uint32_t hs = hdr_size(h_desc[f].payload_size, h_desc[f].mask != 0);
        h_desc[f].header_size = (uint8_t)hs;
        h_desc[f].wire_off = woff;
        const uint64_t W = hs + h_desc[f].payload_size;
        woff += W;
        total += W + 9 * data_frames(W, mfs);
    }
    if (h2_total) *h2_total = total;
    const size_t ws_bytes = cfws_h2_serialize_workspace_size(p->max_frames, p->chunk + 64, p->chunk + 64,
                                                             (uint32_t)mfs);
    const uint8_t* src = static_cast<const uint8_t*>(h_payload);
    uint8_t* dst = static_cast<uint8_t*>(h_h2);
    uint8_t* dst_dev = n ? kernel_d2h_target(p->d2h_mode, h_h2, true) : nullptr;
    size_t i = 0;
    int c = 0;
    uint64_t h2_lo = 0;
    while (i < n) {
        // chunk = WS frames [i, j): source span, WS wire bytes (the two-pass
        // form's scratch) and DATA-stream bytes within the staging
        uint64_t lo = h_desc[i].payload_off, hi = lo + h_desc[i].payload_size, wb = 0, hb = 0;
        size_t j = i;
        while (j < n && j - i < p->max_frames) {
            const uint64_t a = std::min(lo, (uint64_t)h_desc[j].payload_off);
            const uint64_t b = std::max(hi, (uint64_t)(h_desc[j].payload_off + h_desc[j].payload_size));
            const uint64_t W = h_desc[j].header_size + h_desc[j].payload_size;
            const uint64_t H = W + 9 * data_frames(W, mfs);
            if (j > i && ((b - (a & ~uint64_t(15))) > p->chunk || wb + W > p->chunk || hb + H > p->chunk)) break;
            lo = a;
            hi = b;
            wb += W;
            hb += H;
            ++j;
        }
        const uint64_t src_lo = lo & ~uint64_t(15);
        if (hi - src_lo > p->chunk || wb > p->chunk || hb > p->chunk)
            return fail("a frame is larger than the pipeline chunk");
        Slot& S = p->slot[c % p->depth];
        if (int rc = h2_slot(p, S, ws_bytes)) return rc;
        CFWS_HIP(hipEventSynchronize(S.ev_in));       // the slot's last H2D read the staging
        auto* stage = static_cast<cfws_frame_desc_t*>(S.h_stage);
        for (size_t k = i; k < j; ++k) {
            stage[k - i] = h_desc[k];
            stage[k - i].payload_off -= src_lo;
        }
        CFWS_HIP(hipStreamWaitEvent(p->st_in, S.ev_exec, 0));   // d_in, d_desc free
        CFWS_HIP(hipMemcpyAsync(S.d_in, src + src_lo, hi - src_lo, hipMemcpyHostToDevice, p->st_in));
        CFWS_HIP(hipMemcpyAsync(S.d_desc, stage, (j - i) * sizeof(cfws_frame_desc_t),
                                hipMemcpyHostToDevice, p->st_in));
        CFWS_HIP(hipEventRecord(S.ev_in, p->st_in));
        CFWS_HIP(hipStreamWaitEvent(S.st, S.ev_in, 0));
        if (int rc = cfws_h2_serialize_batch(S.d_in, S.d_desc, j - i, stream_id, (uint32_t)mfs, S.d_aux,
                                             p->chunk + 64, S.d_out, p->chunk + 64, S.d_total, S.d_ws2,
                                             S.ws2_size, S.st))
            return rc;
        CFWS_HIP(hipEventRecord(S.ev_exec, S.st));
        if (h2_lo < h2_capacity) {
            const uint64_t m = std::min(hb, h2_capacity - h2_lo);
            if (dst_dev) {
                if (int rc = cfws_internal_copy_out(S.d_out, dst_dev + h2_lo, m, S.st)) return rc;
            } else {
                CFWS_HIP(hipMemcpyAsync(dst + h2_lo, S.d_out, m, hipMemcpyDeviceToHost, S.st));
            }
        }
        CFWS_HIP(hipEventRecord(S.ev_done, S.st));
        h2_lo += hb;
        i = j;
        ++c;
    }
    CFWS_HIP(hipStreamSynchronize(p->st_in));
    for (int s = 0; s < p->depth; ++s) CFWS_HIP(hipStreamSynchronize(p->slot[s].st));
    return CFWS_OK;
}

// co_http2_stream_receive_ws_frame over a host DATA-frame stream
// (cfws_h2_deserialize_batch per chunk): the DATA frames at h_index[i] ->
// HTTP/2 statuses, pooled messages -> co_ws_frame_deserialize -> payloads in
// the host arena, laid out as the batch call lays them out. Chunks end where
// no message is open (after a COMPLETE END_STREAM frame, or where no pooled
// bytes wait), so every message is decoded whole; the next chunk's H2D is
// queued before each batch call, which synchronises for its message count.
// Same index precondition as cfws_pipeline_deserialize.
int cfws_pipeline_h2_deserialize(cfws_pipeline_t* p, const void* h_h2, uint64_t h2_size,
                                 const uint64_t* h_index, size_t n, uint32_t max_frame_size,
                                 uint64_t max_payload, uint32_t align, int32_t* h_h2_status,
                                 cfws_frame_desc_t* h_msg_desc, int32_t* h_msg_status,
                                 size_t* n_messages, void* h_payload, uint64_t payload_capacity,
                                 uint64_t* payload_total)
{
    const CfwsPassScope pass_scope;
    (void)cfws_internal_take_pass();   // not timed (cfws_time_next_pass): the pair is dropped
    if (!p || !n_messages ||
        (n && (!h_h2 || !h_index || !h_h2_status || !h_msg_desc || !h_msg_status || !h_payload)))
        return fail("null argument");
    if (align == 0 || (align & (align - 1)) || align > 4096) return fail("bad align");
    for (size_t i = 1; i < n; ++i)
        if (h_index[i] < h_index[i - 1]) return fail("frame index must be increasing");
    *n_messages = 0;
    if (payload_total) *payload_total = 0;
    if (n == 0) return CFWS_OK;
    const uint64_t mfs = max_frame_size ? max_frame_size : CFWS_H2_DEFAULT_MAX_FRAME_SIZE;
    const uint8_t* h2 = static_cast<const uint8_t*>(h_h2);
    uint8_t* dst = static_cast<uint8_t*>(h_payload);
    uint8_t* dst_dev = kernel_d2h_target(p->d2h_mode, h_payload, false);
    const uint64_t out_slot = p->chunk + 64, pool_cap = p->chunk + 64;
    const size_t ws_bytes = cfws_h2_deserialize_workspace_size(p->max_frames, pool_cap, out_slot);
    auto end_of = [&](size_t k) { return k + 1 < n ? std::min(h_index[k + 1], h2_size) : h2_size; };

    struct Cut { size_t i, j; uint64_t wire_lo, hi, pooled; };
    // frames [i, j) up to the last point where no message is open, with the
    // staged bytes and the payload layout (<= pooled bytes + padding) in the
    // staging; the stream's tail (an unterminated message) ends the last chunk
    auto next_cut = [&](size_t i, Cut& C) -> int {
        const uint64_t wire_lo = std::min(h_index[i], h2_size) & ~uint64_t(15);
        uint64_t open = 0, pooled = 0, best_pooled = 0;
        size_t j = i, best = i;
        while (j < n && j - i < p->max_frames &&
               end_of(j) - wire_lo + (j + 1 - i) * uint64_t(align - 1) <= p->chunk) {
            uint64_t pb = 0;
            bool es = false;
            if (h2_frame_host(h2, h2_size, h_index[j], mfs, &pb, &es) == CFWS_H2_PARSE_COMPLETE) {
                pooled += pb;
                open = es ? 0 : open + pb;
            }
            ++j;
            if (open == 0) {
                best = j;
                best_pooled = pooled;
            }
        }
        if (j == n) {
            best = n;
            best_pooled = pooled;
        }
        if (best == i) return fail("a message spans more bytes or DATA frames than a pipeline chunk holds");
        C = Cut{i, best, wire_lo, end_of(best - 1), best_pooled};
        return CFWS_OK;
    };

    struct Land { size_t i, j, m0, nm; int slot; uint64_t base, pool_base; };
    std::vector<Land> landing;       // D2H enqueued; outputs not rebased yet
    auto finish = [&](const Land& k) -> int {
        Slot& S = p->slot[k.slot];
        CFWS_HIP(hipEventSynchronize(S.ev_done));
        const auto* mdesc = static_cast<const cfws_frame_desc_t*>(S.h_stage);
        const auto* hst = reinterpret_cast<const int32_t*>(mdesc + p->max_frames);
        const int32_t* mst = hst + p->max_frames;
        for (size_t f = k.i; f < k.j; ++f) h_h2_status[f] = hst[f - k.i];
        for (size_t m = 0; m < k.nm; ++m) {
            h_msg_desc[k.m0 + m] = mdesc[m];
            h_msg_desc[k.m0 + m].payload_off += k.base;
            h_msg_desc[k.m0 + m].wire_off += k.pool_base;
            h_msg_status[k.m0 + m] = mst[m];
        }
        return CFWS_OK;
    };
    // the slot's staging is free once its last chunk's outputs are rebased
    auto free_slot = [&](int s) -> int {
        for (size_t q = 0; q < landing.size(); ++q)
            if (landing[q].slot == s) {
                for (size_t r = 0; r <= q; ++r)
                    if (int rc = finish(landing[r])) return rc;
                landing.erase(landing.begin(), landing.begin() + q + 1);
                break;
            }
        return CFWS_OK;
    };
    auto stage_in = [&](const Cut& C, int s) -> int {
        Slot& S = p->slot[s];
        if (int rc = free_slot(s)) return rc;
        if (int rc = h2_slot(p, S, ws_bytes)) return rc;
        auto* sidx = static_cast<uint64_t*>(S.h_stage);
        for (size_t k = C.i; k < C.j; ++k) sidx[k - C.i] = h_index[k] - C.wire_lo;
        CFWS_HIP(hipStreamWaitEvent(p->st_in, S.ev_exec, 0));   // d_in, d_index free
        CFWS_HIP(hipMemcpyAsync(S.d_in, h2 + C.wire_lo, C.hi - C.wire_lo, hipMemcpyHostToDevice, p->st_in));
        CFWS_HIP(hipMemcpyAsync(S.d_index, sidx, (C.j - C.i) * sizeof(uint64_t), hipMemcpyHostToDevice,
                                p->st_in));
        CFWS_HIP(hipEventRecord(S.ev_in, p->st_in));
        return CFWS_OK;
    };

    uint64_t base = 0, pool_base = 0;
    size_t m0 = 0;
    Cut cur, nxt;
    if (int rc = next_cut(0, cur)) return rc;
    if (int rc = stage_in(cur, 0)) return rc;
    for (int c = 0;; ++c) {
        const int s = c % p->depth;
        const bool more = cur.j < n;
        if (more) {
            if (int rc = next_cut(cur.j, nxt)) return rc;
            if (p->depth > 1)
                if (int rc = stage_in(nxt, (c + 1) % p->depth)) return rc;
        }
        Slot& S = p->slot[s];
        CFWS_HIP(hipStreamWaitEvent(S.st, S.ev_in, 0));
        const uint64_t cap = base >= payload_capacity ? 0 : std::min(out_slot, payload_capacity - base);
        size_t nm = 0;
        if (int rc = cfws_h2_deserialize_batch(S.d_in, cur.hi - cur.wire_lo, S.d_index, cur.j - cur.i,
                                               (uint32_t)mfs, S.d_status, S.d_aux, pool_cap, max_payload,
                                               align, S.d_desc, S.d_status2, S.d_out, cap, S.d_total,
                                               &nm, S.d_ws2, S.ws2_size, S.st))
            return rc;
        CFWS_HIP(hipEventRecord(S.ev_exec, S.st));
        // the unclamped payload layout total: offsets keep counting past the capacity
        CFWS_HIP(hipMemcpyAsync(S.h_total,
                                static_cast<char*>(S.d_ws2) +
                                    cfws_internal_h2_grand_total_offset(cur.j - cur.i, pool_cap, cap),
                                8, hipMemcpyDeviceToHost, S.st));
        CFWS_HIP(hipEventRecord(S.ev_total, S.st));
        CFWS_HIP(hipEventSynchronize(S.ev_total));
        const uint64_t tot = nm ? *S.h_total : 0;
        if (base < payload_capacity && tot) {
            const uint64_t m = std::min(tot, payload_capacity - base);
            if (dst_dev) {
                if (int rc = cfws_internal_copy_out(S.d_out, dst_dev + base, m, S.st)) return rc;
            } else {
                CFWS_HIP(hipMemcpyAsync(dst + base, S.d_out, m, hipMemcpyDeviceToHost, S.st));
            }
        }
        auto* mdesc = static_cast<cfws_frame_desc_t*>(S.h_stage);
        auto* hst = reinterpret_cast<int32_t*>(mdesc + p->max_frames);
        if (nm)
            CFWS_HIP(hipMemcpyAsync(mdesc, S.d_desc, nm * sizeof(cfws_frame_desc_t), hipMemcpyDeviceToHost,
                                    S.st));
        CFWS_HIP(hipMemcpyAsync(hst, S.d_status, (cur.j - cur.i) * sizeof(int32_t), hipMemcpyDeviceToHost,
                                S.st));
        if (nm)
            CFWS_HIP(hipMemcpyAsync(hst + p->max_frames, S.d_status2, nm * sizeof(int32_t),
                                    hipMemcpyDeviceToHost, S.st));
        CFWS_HIP(hipEventRecord(S.ev_done, S.st));
        landing.push_back(Land{cur.i, cur.j, m0, nm, s, base, pool_base});
        base += tot;
        m0 += nm;
        pool_base += cur.pooled;
        if (!more) break;
        if (p->depth == 1)
            if (int rc = stage_in(nxt, 0)) return rc;
        cur = nxt;
    }
    for (const Land& k : landing)
        if (int rc = finish(k)) return rc;
    *n_messages = m0;
    if (payload_total) *payload_total = std::min(base, payload_capacity);
    return CFWS_OK;
}

}  // extern "C"
