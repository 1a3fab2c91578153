// cfws_kernels.h -- device code and launch helpers shared by the codec's
// translation units (cfws_device.hip: WS plan / execute / batch ABI and the
// small-batch path; cfws_h2.hip: WebSocket over HTTP/2; cfws_ops.hip: split
// ops, handshake keys, device indexing, copies and fills). Everything here is
// internal to each unit (anonymous namespace); the error state and the
// deserialize plan, which the units share, are defined once in
// cfws_device.hip (namespace cfws_rt).
#ifndef CFWS_KERNELS_H
#define CFWS_KERNELS_H

#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "cfws.h"
#include "cfws_internal.h"

// Each unit uses part of what follows.
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Wunused-function"

namespace cfws_rt {
extern thread_local char g_err[512];
int set_err(int code, const char* what, hipError_t e);
int check_init();
int check_device(int dev);
int launch_check(const char* what);
// cfws_deserialize_plan's body; d_ends (optional) bounds each frame's data
// (the HTTP/2 receive passes each pooled message's end)
int deserialize_plan_impl(const void* d_wire, uint64_t wire_size, const uint64_t* d_index,
                          const uint64_t* d_ends, size_t n, uint64_t max_payload, uint32_t align,
                          uint32_t flags, cfws_frame_desc_t* d_desc, int32_t* d_status, uint64_t cap,
                          uint64_t* d_total, void* ws, size_t ws_size, void* stream);
}  // namespace cfws_rt

namespace {

using cfws_rt::check_init;
using cfws_rt::deserialize_plan_impl;
using cfws_rt::launch_check;
using cfws_rt::set_err;

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;
#ifndef CFWS_UNROLL
#define CFWS_UNROLL 4
#endif
constexpr int kUnroll = CFWS_UNROLL;                         // chunks per lane per region
constexpr uint64_t kChunk = 16;
constexpr uint64_t kSlice = 64 * kChunk;                     // one wave-instruction: 1 KiB
constexpr uint64_t kRegion = kSlice * kUnroll;               // one wave's region: 4 KiB
constexpr int kScanItems = 8;
constexpr uint64_t kScanBlock = uint64_t(kThreads) * kScanItems;
// Plan kernels: one frame per thread. Their per-frame work is a chain of
// dependent loads (descriptor or header bytes), so parallelism beats items
// per thread: 2,048-frame blocks left 224 of 256 CUs idle at 65,536 frames.
#ifndef CFWS_PLAN_ITEMS
#define CFWS_PLAN_ITEMS 1
#endif
constexpr int kPlanItems = CFWS_PLAN_ITEMS;
constexpr uint64_t kPlanBlock = uint64_t(kThreads) * kPlanItems;

// Frame classes a pass copies (deserialize): all, data only, control only.
enum : uint32_t { kClassAll = 0, kClassData = 1, kClassControl = 2 };

// What a streaming pass produces.
//   kModeSer:    WS serialize    -- header (2-14 B) + masked payload per frame
//   kModeDeser:  WS deserialize  -- unmasked payload per frame (or any
//                                   "strip a prefix, copy the body" pass:
//                                   HTTP/2 DATA unwrap uses it too)
//   kModeH2Wrap: HTTP/2 DATA wrap -- 9-byte DATA header + a slice of WS wire
//   kModeH2Ser:  WS serialize straight into HTTP/2 DATA frames -- per DATA
//                frame: 9-byte DATA header, the WS header when the slice
//                starts the WS frame, then the masked payload slice (one
//                pass: the WS wire bytes are never materialised)
enum : int { kModeSer = 0, kModeDeser = 1, kModeH2Wrap = 2, kModeH2Ser = 3 };
__host__ __device__ constexpr bool is_ser(int mode) { return mode != kModeDeser; }

// ---------------------------------------------------------------------------
// workspace layout (deterministic from n_frames and the output capacity)
// ---------------------------------------------------------------------------
// hdr[0] pass-0 total (clamped)   hdr[1] pass-1 total (clamped)
// hdr[2] pass-1 output base       hdr[3] pass-0 grand total   hdr[4] pass-1 grand
struct WsLayout {
    uint64_t hdr;
    uint64_t offs[2];      // u64[n] per pass: sizes, then exclusive offsets
    uint64_t partials[2];  // u64[scan blocks + 1] per pass
    uint64_t map[2];       // u32[regions + 2] per pass
    uint64_t look;         // u32[scan blocks + 1]: single-pass plans' ticket, then block flags
    uint64_t bytes;
    uint64_t regions;
    uint64_t scan_blocks;
};

inline uint64_t align_up(uint64_t x, uint64_t a) { return (x + a - 1) / a * a; }

// The single-pass plans' look area for sb blocks (plan_lookback): the u32
// ticket and flag words, then a u64 word per block from this u32 index.
__host__ __device__ inline uint64_t look_state_index(uint64_t sb) { return (sb + 3) & ~uint64_t(1); }
__host__ __device__ inline uint64_t look_bytes(uint64_t sb) { return 4 * look_state_index(sb) + 8 * (sb + 1); }

WsLayout ws_layout(uint64_t n, uint64_t capacity)
{
    WsLayout L;
    L.regions = (capacity + kRegion - 1) / kRegion;
    L.scan_blocks = (n + kPlanBlock - 1) / kPlanBlock;     // >= any run_scan's blocks
    uint64_t at = 0;
    L.hdr = at;
    at += 256;
    for (int p = 0; p < 2; ++p) { L.offs[p] = at; at = align_up(at + 8 * n, 256); }
    for (int p = 0; p < 2; ++p) { L.partials[p] = at; at = align_up(at + 8 * (L.scan_blocks + 1), 256); }
    for (int p = 0; p < 2; ++p) { L.map[p] = at; at = align_up(at + 4 * (L.regions + 2), 256); }
    L.look = at;
    at = align_up(at + look_bytes(L.scan_blocks), 256);
    L.bytes = at;
    return L;
}

// ---------------------------------------------------------------------------
// device helpers
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t header_size_of(uint64_t n, bool mask)
{
    return 2u + (n > 65535u ? 8u : (n > 125u ? 2u : 0u)) + (mask ? 4u : 0u);
}

__device__ __forceinline__ bool is_control(uint32_t opcode)
{
    return opcode <= 0x0fu && (opcode & 0x08u) != 0;       // co_ws_frame.h:32-34
}

__device__ __forceinline__ uint32_t rotr8(uint32_t key, uint32_t bytes)
{
    return __builtin_amdgcn_alignbyte(key, key, bytes & 3u);
}

// The descriptor is read as four 64-bit words so that a wave-uniform f
// becomes one s_load_dwordx8 (byte-field loads would be vector loads).
struct DescWords {
    uint64_t payload_off, wire_off, payload_size, w3;
    __device__ uint32_t key() const { return (uint32_t)w3; }
    __device__ uint32_t fin() const { return (uint32_t)(w3 >> 32) & 0xffu; }
    __device__ uint32_t opcode() const { return (uint32_t)(w3 >> 40) & 0xffu; }
    __device__ uint32_t mask() const { return (uint32_t)(w3 >> 48) & 0xffu; }
    __device__ uint32_t header_size() const { return (uint32_t)(w3 >> 56); }
};

__device__ __forceinline__ DescWords load_desc(const cfws_frame_desc_t* __restrict__ desc, uint32_t f)
{
    const uint64_t* q = reinterpret_cast<const uint64_t*>(desc) + 4 * uint64_t(f);
    return DescWords{q[0], q[1], q[2], q[3]};
}

// Arguments of one streaming pass.
struct Pass {
    const uint8_t* src;
    uint8_t* dst;                 // already offset by the pass base
    const cfws_frame_desc_t* desc;
    const int32_t* status;        // deserialize only
    const uint64_t* offs;         // per-frame output offsets of this pass
    uint64_t total;               // output bytes of this pass
    uint64_t capacity;            // writable bytes from dst
    uint32_t n_frames;
    uint32_t klass;
    uint32_t sid;                 // HTTP/2 stream id (kModeH2Wrap, kModeH2Ser)
    const cfws_frame_desc_t* parent;   // kModeH2Ser: the WS frames
};

// What one frame contributes to a pass's output.
//   [out_off, out_off + pre)              header bytes (serialize only)
//   [out_off + pre, + body_len)           src[src_off + k] ^ key[k % 4]
//   [.., next frame's out_off)            zero (deserialize alignment pad)
struct FrameView {
    uint64_t out_off;
    uint64_t body_start;
    uint64_t body_len;
    uint64_t src_off;
    uint32_t key;   // 0 when the frame is not masked: XOR becomes a copy
    uint32_t pre;
    uint32_t hb;    // serialize: header byte 0 | mask bit << 8; DATA: flags
    uint32_t whb;   // kModeH2Ser, a WS frame's first slice: its WS header byte 0 | mask bit << 8
    uint64_t wlen;  // kModeH2Ser, a WS frame's first slice: the WS payload size
};

// Byte r < pre of a serialize frame's header, from its view (co_ws_frame.c:34-91).
__device__ __forceinline__ uint32_t view_header_byte(const FrameView& v, uint32_t r)
{
    const uint64_t n = v.body_len;
    const uint32_t ext = n > 65535u ? 8u : (n > 125u ? 2u : 0u);
    const uint32_t l7 = ext == 8 ? 127u : (ext == 2 ? 126u : (uint32_t)n);
    const uint32_t key_b = (v.key >> (8 * ((r - 2 - ext) & 3u))) & 0xffu;
    const uint32_t len_b = (uint32_t)(n >> (8 * ((ext - 1 - (r - 2)) & 7u))) & 0xffu;
    return r == 0 ? (v.hb & 0xffu)
         : r == 1 ? ((l7 | ((v.hb >> 1) & 0x80u)) & 0xffu)
         : (r - 2 < ext) ? len_b : key_b;
}

template <int kMode>
__device__ __forceinline__ FrameView frame_view(const Pass& P, uint32_t f)
{
    const DescWords d = load_desc(P.desc, f);
    FrameView v;
    v.key = d.mask() ? d.key() : 0u;
    v.out_off = P.offs[f];
    v.hb = 0;
    v.whb = 0;
    v.wlen = 0;
    if (kMode == kModeH2Ser) {
        // one DATA frame as h2_ser_plan_apply_kernel laid it out: body
        // source offset and length, rotated key, 9 + h_in bytes before the
        // body (0: an unused slot), END_STREAM, and for a WS frame's first
        // slice (h_in > 0: the whole WS header, max_frame_size >= 64) the
        // WS header's fields: no load of the WS frame's descriptor
        v.pre = d.header_size();
        v.body_len = d.payload_size;
        v.src_off = d.payload_off;
        v.key = d.key();
        v.hb = d.fin() ? 0x1u : 0u;                      // DATA flags: END_STREAM
        v.whb = d.opcode() | (d.mask() ? 0x100u : 0u);
        v.wlen = d.wire_off;
    } else if (is_ser(kMode)) {
        v.pre = d.header_size();
        v.body_len = d.payload_size;
        v.src_off = d.payload_off;
        v.hb = kMode == kModeH2Wrap
                   ? (d.fin() ? 0x1u : 0u)                         // DATA flags: END_STREAM
                   : ((d.opcode() | (d.fin() ? 0x80u : 0u)) & 0xffu) | (d.mask() ? 0x100u : 0u);
    } else {
        const bool ctl = is_control(d.opcode());
        const bool take = P.klass == kClassAll || (P.klass == kClassControl) == ctl;
        v.pre = 0;
        v.body_len = (take && P.status[f] == CFWS_PARSE_COMPLETE) ? d.payload_size : 0;
        v.src_off = d.wire_off + d.header_size();
    }
    v.body_start = v.out_off + v.pre;
    return v;
}

// 16-byte global accesses of the streaming paths. Output is written once and
// never re-read by the kernel, so stores carry the `nt` bit (measured +2-3 %
// on config 2). Loads keep the default policy: every source byte is read by
// exactly one lane, once, yet `nt` loads measured -10 % with two loads per
// block and -3 % with the DPP path (6.37/6.49 TB/s plain vs 5.97/6.29 nt,
// profiles/r01_ab_dpp.json), although the bare copy probe
// (tools/copy_probe.hip) gains from them.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint4 ld16(const uint8_t* p)
{
    const u32x4 v = *reinterpret_cast<const u32x4*>(p);
    return make_uint4(v.x, v.y, v.z, v.w);
}

// Lane i receives lane i + 1's `v` (DPP wave_shl:1); lane 63, which has no
// right neighbour, keeps `last`.
__device__ __forceinline__ uint32_t from_next_lane(uint32_t v, uint32_t last)
{
    return __builtin_amdgcn_update_dpp(last, v, 0x130, 0xf, 0xf, false);
}

// lane i <- lane i + 1, lane 63 <- lane 0 (DPP wave_rol:1)
__device__ __forceinline__ uint4 from_next_lane_wrap(const uint4& v)
{
    return make_uint4(__builtin_amdgcn_update_dpp(0u, v.x, 0x134, 0xf, 0xf, false),
                      __builtin_amdgcn_update_dpp(0u, v.y, 0x134, 0xf, 0xf, false),
                      __builtin_amdgcn_update_dpp(0u, v.z, 0x134, 0xf, 0xf, false),
                      __builtin_amdgcn_update_dpp(0u, v.w, 0x134, 0xf, 0xf, false));
}

__device__ __forceinline__ uint4 from_next_lane(const uint4& v, const uint4& last)
{
    return make_uint4(from_next_lane(v.x, last.x), from_next_lane(v.y, last.y),
                      from_next_lane(v.z, last.z), from_next_lane(v.w, last.w));
}

__device__ __forceinline__ void st16(uint8_t* p, uint4 o)
{
    const u32x4 v = {o.x, o.y, o.z, o.w};
    __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p));
}

// Body stores of the streaming regions, at byte `off` of the wave's output
// region `rb` (wave-uniform), with a cache policy per mode. Policy bits
// (gfx940+): sc0 1, nt 2, sc1 16; 0 = the global `nt` store (st16).
// WS serialize and deserialize store write-through (`sc0 sc1 nt`, a buffer
// store over the region): deserialize 6.49 -> 6.52-6.60 TB/s on config 2;
// serialize gains only at 4 workgroups per CU (xform_lds_bytes), where it
// went from 6.34-6.37 to 6.44-6.48 TB/s (at 5 per CU it lost 1-2 %;
// profiles/r02_ab_store.txt, r02_ab_sendwt_lds.txt, r02_ab_fs.txt). The
// HTTP/2 send keeps `nt` (write-through measured no faster there).
// CFWS_STORE_AUX_SER / _RECV override at build time.
#ifndef CFWS_STORE_AUX_SER
#define CFWS_STORE_AUX_SER 19
#endif
#ifndef CFWS_STORE_AUX_RECV
#define CFWS_STORE_AUX_RECV 19
#endif
#ifndef CFWS_STORE_AUX_H2SER
#define CFWS_STORE_AUX_H2SER 0
#endif
template <int kMode>
__device__ __forceinline__ void st16_region(uint8_t* rb, uint32_t off, uint4 o)
{
    constexpr int aux = kMode == kModeDeser ? CFWS_STORE_AUX_RECV
                      : kMode == kModeSer ? CFWS_STORE_AUX_SER
                      : kMode == kModeH2Ser ? CFWS_STORE_AUX_H2SER : 0;
    if (aux == 0) {
        st16(rb + off, o);
    } else {
        const u32x4 v = {o.x, o.y, o.z, o.w};
        const auto r = __builtin_amdgcn_make_buffer_rsrc(rb, 0, (int)kRegion, 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b128(v, r, (int)off, 0, aux);
    }
}

// 16 output bytes starting `ph` bytes into the 32-byte window {A, B}.
__device__ __forceinline__ uint4 funnel16(uint4 A, uint4 B, uint32_t ph)
{
    const bool s8 = (ph & 8u) != 0;
    const bool s4 = (ph & 4u) != 0;
    const uint32_t r = ph & 3u;
    const uint32_t a0 = s8 ? A.z : A.x, a1 = s8 ? A.w : A.y, a2 = s8 ? B.x : A.z;
    const uint32_t a3 = s8 ? B.y : A.w, a4 = s8 ? B.z : B.x, a5 = s8 ? B.w : B.y;
    const uint32_t b0 = s4 ? a1 : a0, b1 = s4 ? a2 : a1, b2 = s4 ? a3 : a2;
    const uint32_t b3 = s4 ? a4 : a3, b4 = s4 ? a5 : a4;
    uint4 o;
    o.x = __builtin_amdgcn_alignbyte(b1, b0, r);
    o.y = __builtin_amdgcn_alignbyte(b2, b1, r);
    o.z = __builtin_amdgcn_alignbyte(b3, b2, r);
    o.w = __builtin_amdgcn_alignbyte(b4, b3, r);
    return o;
}

__device__ __forceinline__ void xor4(uint4& o, uint32_t k)
{
    o.x ^= k; o.y ^= k; o.z ^= k; o.w ^= k;
}

// Byte r of an HTTP/2 DATA frame header (co_http2_frame.c:33-72: 24-bit BE
// length, type 0, flags, 31-bit BE stream id).
__device__ __forceinline__ uint32_t h2_header_byte(uint32_t len, uint32_t flags, uint32_t sid,
                                                   uint32_t r)
{
    const uint32_t sidm = sid & 0x7fffffffu;
    return r == 0 ? (len >> 16) & 0xffu
         : r == 1 ? (len >> 8) & 0xffu
         : r == 2 ? len & 0xffu
         : r == 3 ? 0u
         : r == 4 ? (flags & 0xffu)
         : (sidm >> (8 * (8 - r))) & 0xffu;
}

template <int kMode>
__device__ __forceinline__ uint32_t header_byte_of(const Pass& P, const FrameView& v, uint32_t r)
{
    if (kMode == kModeH2Wrap) return h2_header_byte((uint32_t)v.body_len, v.hb, P.sid, r);
    if (kMode == kModeH2Ser) {
        if (r < 9) return h2_header_byte(v.pre - 9u + (uint32_t)v.body_len, v.hb, P.sid, r);
        // the WS frame's header (co_ws_frame.c:34-91), from the slice's fields
        FrameView wv;
        wv.body_len = v.wlen;
        wv.key = v.key;                                 // the first slice: rotated by 0
        wv.hb = v.whb;
        return view_header_byte(wv, r - 9u);
    }
    return view_header_byte(v, r);
}

// One chunk entirely inside v's body.
__device__ __forceinline__ uint4 body_chunk(const uint8_t* __restrict__ src, const FrameView& v,
                                            uint64_t D)
{
    const uint64_t k0 = D - v.body_start;
    const uint64_t s = v.src_off + k0;
    const uint8_t* sp = src + (s & ~uint64_t(15));
    const uint32_t ph = (uint32_t)(s & 15u);
    uint4 o = ld16(sp);
    // The aligned block holding the chunk's last byte: it contains a valid
    // source byte, so it never lies past the allocation's last page.
    if (ph != 0) o = funnel16(o, ld16(sp + 16), ph);
    xor4(o, rotr8(v.key, (uint32_t)(k0 & 3u)));
    return o;
}

// Chunks that hold more than two frames (runs of frames shorter than ~14
// bytes): byte by byte, walking frames forward from f. (Loading the views of
// four bytes at a time measured 30 % slower on config 3: the register cost
// dropped the edge kernels' occupancy more than the shorter chains saved.)
template <int kMode>
__device__ __forceinline__ uint4 edge_chunk_bytes(const Pass& P, uint32_t f, uint64_t D)
{
    FrameView v = frame_view<kMode>(P, f);
    uint64_t next = (f + 1 < P.n_frames) ? P.offs[f + 1] : ~uint64_t(0);
    uint32_t w0 = 0, w1 = 0, w2 = 0, w3 = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const uint64_t pos = D + j;
        uint32_t b = 0;
        if (pos < P.total) {
            while (pos >= next) {
                ++f;
                v = frame_view<kMode>(P, f);
                next = (f + 1 < P.n_frames) ? P.offs[f + 1] : ~uint64_t(0);
            }
            const uint64_t r = pos - v.out_off;
            if (r < v.pre) {
                b = header_byte_of<kMode>(P, v, (uint32_t)r);
            } else {
                const uint64_t k = r - v.pre;
                if (k < v.body_len) b = (P.src[v.src_off + k] ^ (v.key >> (8 * (k & 3u)))) & 0xffu;
            }
        }
        const uint32_t sh = 8 * (j & 3);
        if (j < 4) w0 |= b << sh;
        else if (j < 8) w1 |= b << sh;
        else if (j < 12) w2 |= b << sh;
        else w3 |= b << sh;
    }
    return make_uint4(w0, w1, w2, w3);
}

// Frame v's (masked) body bytes lined up with the output chunk at D: byte j
// of the result is the body byte at output position D + j, for every j
// whose position lies inside v's body (other bytes are don't-care). One or
// two aligned source blocks are read -- only blocks that hold a body byte
// of the chunk -- and shifted once with funnel16; the per-byte assembly in
// edge_chunk then indexes registers statically (a dynamic byte index into
// {A, B} is lowered through scratch memory).
__device__ __forceinline__ uint4 edge_body(const uint8_t* __restrict__ src, const FrameView& v,
                                           uint64_t D, uint64_t lim)
{
    const uint64_t be = v.body_start + v.body_len;
    const uint64_t lo = D > v.body_start ? D : v.body_start;
    const uint64_t hi = lim < be ? lim : be;
    uint4 W = make_uint4(0, 0, 0, 0);
    if (hi > lo) {
        const uint64_t s_first = v.src_off + (lo - v.body_start);
        const uint64_t s_last = v.src_off + (hi - 1 - v.body_start);
        const uint64_t abase = s_first & ~uint64_t(15);
        const uint4 A = ld16(src + abase);
        const uint4 B = ((s_last & ~uint64_t(15)) != abase) ? ld16(src + abase + 16) : A;
        // window byte ph holds the body byte at output position lo
        const uint32_t ph = (uint32_t)(s_first - abase);
        const uint32_t j0 = (uint32_t)(lo - D);                   // 0..15
        if (ph >= j0) {
            W = funnel16(A, B, ph - j0);
        } else {                                                   // body starts mid-chunk
            W = funnel16(make_uint4(0, 0, 0, 0), A, 16u - (j0 - ph));
        }
        xor4(W, rotr8(v.key, (uint32_t)(D - v.body_start) & 3u));
    }
    return W;
}

__device__ __forceinline__ uint32_t u4_byte(const uint4& w, int j)
{
    const uint32_t d = j < 4 ? w.x : (j < 8 ? w.y : (j < 12 ? w.z : w.w));
    return (d >> (8 * (j & 3))) & 0xffu;
}

// Bytes [a, b) of a 16-byte chunk as a mask (0 <= a, b <= 16).
__device__ __forceinline__ uint32_t low_bytes(int k)
{
    return k <= 0 ? 0u : (k >= 4 ? 0xffffffffu : (1u << (8 * k)) - 1u);
}

__device__ __forceinline__ uint4 byte_range(uint32_t a, uint32_t b)
{
    const int ia = (int)a, ib = (int)b;
    return make_uint4(low_bytes(ib) & ~low_bytes(ia), low_bytes(ib - 4) & ~low_bytes(ia - 4),
                      low_bytes(ib - 8) & ~low_bytes(ia - 8), low_bytes(ib - 12) & ~low_bytes(ia - 12));
}

__device__ __forceinline__ uint4 and4(uint4 a, uint4 b)
{
    return make_uint4(a.x & b.x, a.y & b.y, a.z & b.z, a.w & b.w);
}

__device__ __forceinline__ uint4 or4(uint4 a, uint4 b)
{
    return make_uint4(a.x | b.x, a.y | b.y, a.z | b.z, a.w | b.w);
}

// Output position x relative to chunk D, clamped to [0, 16].
__device__ __forceinline__ uint32_t chunk_rel(uint64_t x, uint64_t D)
{
    return x <= D ? 0u : (x - D >= 16 ? 16u : (uint32_t)(x - D));
}

// A WS frame's header (co_ws_frame.c:34-91) as little-endian words: byte 0,
// byte 1 (mask bit | 7-bit length), the 0/2/8-byte big-endian extended
// length, the key (hb: byte 0 | mask bit << 8; key 0 when unmasked).
__device__ __forceinline__ uint4 ws_header_words(uint64_t n, uint32_t hb, uint32_t k)
{
    const uint32_t ext = n > 65535u ? 8u : (n > 125u ? 2u : 0u);
    const uint32_t l7 = ext == 8 ? 127u : (ext == 2 ? 126u : (uint32_t)n);
    const uint32_t b01 = (hb & 0xffu) | ((l7 | ((hb >> 1) & 0x80u)) & 0xffu) << 8;
    if (ext == 0) return make_uint4(b01 | k << 16, k >> 16, 0u, 0u);
    if (ext == 2) return make_uint4(b01 | (uint32_t)__builtin_bswap16((uint16_t)n) << 16, k, 0u, 0u);
    const uint64_t be = __builtin_bswap64(n);
    return make_uint4(b01 | (uint32_t)(be & 0xffffu) << 16, (uint32_t)(be >> 16),
                      (uint32_t)(be >> 48) | k << 16, k >> 16);
}

// The bytes a frame writes before its body, as little-endian words (lo:
// bytes 0-15, hi: 16-31; bytes past `pre` are don't-care):
// * serialize: its WS header;
// * the two-pass HTTP/2 wrap: the 9-byte DATA header (co_http2_frame.c:33-72),
//   from constant byte indices;
// * the fused HTTP/2 send: the DATA header, then the WS header bytes the slice
//   carries from s0 on (h_in = pre - 9 of them; with max_frame_size >= 64 a
//   WS header lies whole in its frame's first slice).
struct HeaderWords {
    uint4 lo, hi;
};

template <int kMode>
__device__ __forceinline__ HeaderWords header_words(const Pass& P, const FrameView& v)
{
    const uint4 z = make_uint4(0, 0, 0, 0);
    if (kMode == kModeSer) return {ws_header_words(v.body_len, v.hb, v.key), z};
    if (kMode == kModeH2Ser) {
        const uint32_t len = v.pre - 9u + (uint32_t)v.body_len;
        const uint32_t sid = P.sid & 0x7fffffffu;
        uint4 w = z;
        if (v.pre > 9u) w = ws_header_words(v.wlen, v.whb, v.key);
        HeaderWords h;
        h.lo.x = (len >> 16 & 0xffu) | (len >> 8 & 0xffu) << 8 | (len & 0xffu) << 16;
        h.lo.y = (v.hb & 0xffu) | (sid >> 24 & 0xffu) << 8 | (sid >> 16 & 0xffu) << 16 |
                 (sid >> 8 & 0xffu) << 24;
        h.lo.z = (sid & 0xffu) | w.x << 8;
        h.lo.w = w.x >> 24 | w.y << 8;
        h.hi = make_uint4(w.y >> 24 | w.z << 8, w.z >> 24 | w.w << 8, 0u, 0u);
        return h;
    }
    uint32_t h[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (uint32_t r = 0; r < 16; ++r)
        if (r < v.pre) h[r >> 2] |= header_byte_of<kMode>(P, v, r) << (8u * (r & 3u));
    return {make_uint4(h[0], h[1], h[2], h[3]), z};
}

// Frame v's bytes in chunk D: its header (when the mode writes one), then its
// body (W: edge_body's lined-up body bytes), zero elsewhere.
template <int kMode>
__device__ __forceinline__ uint4 view_chunk(const Pass& P, const FrameView& v, uint64_t D, uint4 W)
{
    uint4 o = and4(W, byte_range(chunk_rel(v.body_start, D), chunk_rel(v.body_start + v.body_len, D)));
    if (kMode != kModeDeser && v.pre) {
        const HeaderWords H = header_words<kMode>(P, v);
        const uint4 z = make_uint4(0, 0, 0, 0);
        uint4 Hs;
        if (v.out_off >= D) {
            const uint64_t q = v.out_off - D;              // header byte 0 at chunk byte q
            Hs = q == 0 ? H.lo : (q >= 16 ? z : funnel16(z, H.lo, 16u - (uint32_t)q));
        } else {
            const uint64_t sft = D - v.out_off;            // chunk byte 0 is header byte sft
            Hs = sft < 16 ? funnel16(H.lo, H.hi, (uint32_t)sft)
                          : (sft < 32 ? funnel16(H.hi, z, (uint32_t)(sft - 16)) : z);
        }
        o = or4(o, and4(Hs, byte_range(chunk_rel(v.out_off, D), chunk_rel(v.out_off + v.pre, D))));
    }
    return o;
}

// A chunk that crosses a header, a frame boundary, padding or the end of
// the pass. With at most two frames in it (every boundary of frames larger
// than the chunk) all source blocks are loaded up front and the bytes are
// assembled in registers: one memory round trip instead of sixteen. Each
// frame's header and body words are shifted into place and masked to their
// byte ranges (word operations, not sixteen per-byte selects per frame).
template <int kMode>
__device__ __forceinline__ uint4 edge_chunk(const Pass& P, uint32_t f, uint64_t D,
                                            const FrameView& va, const FrameView& vb, uint64_t o1,
                                            uint64_t o2)
{
    const uint64_t lim = D + 16 < P.total ? D + 16 : P.total;
    if (o2 < lim) return edge_chunk_bytes<kMode>(P, f, D);
    const bool two = o1 < lim;
    const uint4 Wa = edge_body(P.src, va, D, lim);
    const uint4 Wb = two ? edge_body(P.src, vb, D, lim) : Wa;
    uint4 o = view_chunk<kMode>(P, va, D, Wa);
    if (two) o = or4(o, view_chunk<kMode>(P, vb, D, Wb));
    return and4(o, byte_range(0, chunk_rel(lim, D)));
}

__device__ __forceinline__ void store_chunk(const Pass& P, uint64_t D, uint4 o)
{
    if (D + 16 <= P.capacity) {
        st16(P.dst + D, o);
    } else {
        for (uint32_t j = 0; D + j < P.capacity; ++j) {
            const uint32_t w = j < 4 ? o.x : (j < 8 ? o.y : (j < 12 ? o.z : o.w));
            P.dst[D + j] = (uint8_t)(w >> (8 * (j & 3)));
        }
    }
}

// ---------------------------------------------------------------------------
// the streaming kernel
// ---------------------------------------------------------------------------

// A region inside one frame's body: frame, source phase and rotated key are
// wave-uniform (SGPRs); all kUnroll loads are in flight before the first
// store. Each lane loads the one aligned source block A that holds its
// chunk's first byte; when the source is misaligned against the output
// (phase != 0) the block B after it is the next lane's A, taken over DPP, so
// every source byte is loaded once (lane 63 loads its B itself).
template <int kMode>
__device__ __forceinline__ void fast_region(const Pass& P, const FrameView& v, uint64_t base,
                                            uint32_t lane)
{
    const uint64_t delta = v.src_off - v.body_start;           // src = out + delta
    const uint32_t ph = (uint32_t)(delta & 15u);
    const uint32_t kr = rotr8(v.key, (uint32_t)((0 - v.body_start) & 3u));
    const uint8_t* s0 = P.src + ((base + delta) & ~uint64_t(15)) + lane * kChunk;
    uint8_t* const rb = P.dst + base;
    const uint32_t l0 = lane * (uint32_t)kChunk;
    uint4 a[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) a[u] = ld16(s0 + u * kSlice);
    if (ph == 0) {
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            xor4(a[u], kr);
            st16_region<kMode>(rb, l0 + u * (uint32_t)kSlice, a[u]);
        }
    } else {
        // lane 63's B is the block after its A: it holds the chunk's last
        // byte, a body byte, so it lies inside the source allocation.
        uint4 e[kUnroll];
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) e[u] = make_uint4(0, 0, 0, 0);
        if (lane == 63) {
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) e[u] = ld16(s0 + u * kSlice + 16);
        }
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            uint4 o = funnel16(a[u], from_next_lane(a[u], e[u]), ph);
            xor4(o, kr);
            st16_region<kMode>(rb, l0 + u * (uint32_t)kSlice, o);
        }
    }
}

// A region crossed by exactly one frame boundary (the boundary case of large
// frames): both views are wave-uniform, each lane picks one by comparing its
// chunk with the boundary. Chunks not entirely inside a body are left to
// edge_kernel. As in fast_region, a lane's block B comes from the next lane
// over DPP when that lane loads it (same frame, chunk inside the body);
// otherwise (lane 63, the last chunk before a body end) the lane loads it.
//
// kEdges (the fused HTTP/2 send when its plan found every DATA frame but the
// last at least kRegion + 32 bytes long, h2_ser_plan_apply_kernel): the
// region's edge chunks too, assembled from registers and stored in the same
// instruction as their segment's body chunks, so no edge workgroup writes
// them and no 64-byte segment leaves L2 in two parts. With
// such frames a region holds at most one header, vb's (the frames are back
// to back: va's body ends where vb starts), and an edge chunk at r is
//   [va's body tail: bytes < q] [vb's header at q = vb.out_off - r]
//   [vb's body head from q + pre on]
// (va == vb: the header started at or before the region; no tail). The
// header words and the body's first 16 masked bytes are wave-uniform,
// computed once per region; the tail is the lane's own source blocks.
template <int kMode, bool kEdges = false>
__device__ __forceinline__ void two_frame_region(const Pass& P, const FrameView& va,
                                                 const FrameView& vb, uint64_t base, uint32_t lane)
{
    // Everything per frame is wave-uniform and taken relative to the region
    // base (offsets clamped into [0, kRegion + 32], enough for every compare
    // below), so a lane only selects between two sets of scalars: its chunk
    // r (a multiple of 16) is in frame B iff r >= ob; the source block, the
    // phase and the rotated key follow (phase and key rotation are the same
    // for every chunk of a frame, because r is a multiple of 16).
    auto rel = [base](uint64_t x) -> uint32_t {
        return x <= base ? 0u : (x - base >= kRegion + 32 ? (uint32_t)(kRegion + 32) : (uint32_t)(x - base));
    };
    const uint32_t ob = rel(vb.out_off);
    const uint32_t a_lo = rel(va.body_start), a_hi = rel(va.body_start + va.body_len);
    const uint32_t b_lo = rel(vb.body_start), b_hi = rel(vb.body_start + vb.body_len);
    const uint64_t sA = base + (va.src_off - va.body_start);
    const uint64_t sB = base + (vb.src_off - vb.body_start);
    const uint32_t phA = (uint32_t)(sA & 15u), phB = (uint32_t)(sB & 15u);
    const uint32_t krA = rotr8(va.key, (uint32_t)(base - va.body_start) & 3u);
    const uint32_t krB = rotr8(vb.key, (uint32_t)(base - vb.body_start) & 3u);
    const uint8_t* sp[kUnroll];
    bool fast[kUnroll], own[kUnroll], hi[kUnroll], tl[kUnroll];
    // kEdges: vb's header start relative to the region (va == vb: <= 0)
    const bool twof = kEdges && vb.out_off != va.out_off;
    const int64_t hs64 = (int64_t)vb.out_off - (int64_t)base;
    const int hs = hs64 < -64 ? -64 : (hs64 > (int64_t)kRegion ? (int)kRegion : (int)hs64);
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
        const uint32_t r = u * (uint32_t)kSlice + lane * (uint32_t)kChunk;
        hi[u] = r >= ob;
        const uint32_t lo_ = hi[u] ? b_lo : a_lo, hi_ = hi[u] ? b_hi : a_hi;
        fast[u] = r >= lo_ && r + 16 <= hi_;
        // the next lane's chunk loads block sp + 16 iff it is in the same
        // frame and inside the body
        const bool next_loads = lane != 63 && (r + 16 >= ob) == hi[u] && r + 32 <= hi_;
        // kEdges: the chunk holding va's body tail (and vb's header start)
        tl[u] = twof && !fast[u] && (int)r < hs;
        own[u] = (fast[u] && (hi[u] ? phB : phA) != 0 && !next_loads) ||
                 (tl[u] && phA + (uint32_t)(hs - (int)r) > 16u);
        sp[u] = P.src + (((hi[u] ? sB : sA) + r) & ~uint64_t(15));
    }
    uint4 a[kUnroll], e[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) a[u] = fast[u] || tl[u] ? ld16(sp[u]) : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) e[u] = own[u] ? ld16(sp[u] + 16) : make_uint4(0, 0, 0, 0);
    // kEdges: vb's header words and its body's first 16 bytes, masked
    // (every lane loads the same two blocks; a full 64-bit VGPR address, see
    // general_region_ser_edges)
    HeaderWords H = {};
    uint4 W0 = make_uint4(0, 0, 0, 0);
    if (kEdges) {
        H = header_words<kMode>(P, vb);
        uint64_t addr = reinterpret_cast<uint64_t>(P.src) + (vb.src_off & ~uint64_t(15));
        asm volatile("" : "+v"(addr));
        const uint8_t* p0 = reinterpret_cast<const uint8_t*>(addr);
        const uint32_t ph0 = (uint32_t)(vb.src_off & 15u);
        // only blocks that hold a body byte (the stream's last frame may be
        // short when the pass ends on a region boundary)
        if (vb.body_len > 0) W0 = ld16(p0);
        if (ph0) W0 = funnel16(W0, vb.body_len > 16 - ph0 ? ld16(p0 + 16) : make_uint4(0, 0, 0, 0), ph0);
        xor4(W0, vb.key);
    }
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
        const uint4 nb = from_next_lane(a[u], e[u]);     // every lane: DPP needs the full wave
        const uint32_t R = u * (uint32_t)kSlice + lane * (uint32_t)kChunk;
        if (kEdges && !fast[u]) {
            const uint4 z = make_uint4(0, 0, 0, 0);
            const int q = hs - (int)R;                   // vb's header byte 0 at chunk byte q
            const int pre = (int)vb.pre;
            uint4 o = z;
            if (tl[u]) {                                 // va's body tail: bytes [0, q)
                uint4 t = phA ? funnel16(a[u], e[u], phA) : a[u];
                xor4(t, krA);
                o = and4(t, byte_range(0, (uint32_t)(q < 16 ? q : 16)));
            }
            if (q < 16 && q + pre > 0) {                 // the header: bytes [q, q + pre)
                uint4 Hs;
                if (q >= 0) Hs = q == 0 ? H.lo : funnel16(z, H.lo, 16u - (uint32_t)q);
                else Hs = -q < 16 ? funnel16(H.lo, H.hi, (uint32_t)-q) : funnel16(H.hi, z, (uint32_t)(-q - 16));
                o = or4(o, and4(Hs, byte_range(q > 0 ? (uint32_t)q : 0u,
                                               q + pre < 16 ? (uint32_t)(q + pre) : 16u)));
            }
            const int s = q + pre;                       // vb's body head: bytes [s, 16)
            if (s > 0 && s < 16) o = or4(o, funnel16(z, W0, 16u - (uint32_t)s));
            st16_region<kMode>(P.dst + base, R, o);
            continue;
        }
        if (!fast[u]) continue;
        const uint32_t ph = hi[u] ? phB : phA;
        uint4 o = ph ? funnel16(a[u], own[u] ? e[u] : nb, ph) : a[u];
        xor4(o, hi[u] ? krB : krA);
        st16_region<kMode>(P.dst + base, R, o);
    }
}

// Any other region (small frames, padding, pass end) with more than 64
// frames: every lane finds the frame of each of its chunks by binary search
// over the region's frames and writes it when it lies inside that frame's
// body.
template <int kMode>
__device__ __forceinline__ void general_region_search(const Pass& P, uint32_t f0, uint32_t f1,
                                                      uint64_t base, uint32_t lane)
{
    uint32_t fr[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
        const uint64_t D = base + u * kSlice + lane * kChunk;
        uint32_t lo = f0, hi = f1;                  // largest f with offs[f] <= D
        while (lo < hi) {
            const uint32_t mid = (lo + hi + 1) >> 1;
            if (P.offs[mid] <= D) lo = mid; else hi = mid - 1;
        }
        fr[u] = lo;
    }
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
        const uint64_t D = base + u * kSlice + lane * kChunk;
        const FrameView v = frame_view<kMode>(P, fr[u]);
        if (D >= v.body_start && D + kChunk <= v.body_start + v.body_len)
            st16_region<kMode>(P.dst + base, (uint32_t)(D - base), body_chunk(P.src, v, D));
    }
}

// A region touched by 3..64 frames (runs of small frames): lane l loads what
// the chunks need of frame f0 + l, all lanes at once (one round of loads
// instead of a search and a view per chunk, each a chain of dependent
// loads), reduced to four words relative to the region base: the frame's
// output start, its body range, its source delta and its key rotated for
// 16-aligned chunks. Each chunk then finds its frame by a binary search over
// the lanes (shuffles) and loads only its source blocks. Up to
// CFWS_GENERAL_SCAN frames a count of the frame starts replaces the search:
// 8 -> 12 took 384 B and 512 B steps 1.3 % and 2.3 % faster (512 B send
// 1.523 -> 1.473 ms, receive 1.489 -> 1.461), 256 B and 768 B unchanged; 16
// and 64 cost the 256 B send 0.4-0.6 % (profiles/r05/general_scan_ab/)
#ifndef CFWS_GENERAL_SCAN
#define CFWS_GENERAL_SCAN 12
#endif
#ifndef CFWS_GENERAL_DIRECT
#define CFWS_GENERAL_DIRECT 1
#endif

// WS serialize, in-region edge chunks (`inreg`: the plan found every frame
// with an 80..3,584-byte payload at a 16-aligned source offset; see
// ser_inreg_frame_ok). Such frames are longer than a chunk, so a chunk that
// is not inside one body holds exactly one frame's header bytes (at most 8:
// 16-bit lengths), with frame j's body tail before them and the header
// frame's body head after them; and every region holding a header comes
// here (region_loop sends the one- and two-frame ones too). Each part comes from
// registers the region already holds: the header words from the frames'
// views, the body tail from the lane's own source blocks, the body head from
// the next chunk's first block (that chunk lies inside the same body, whose
// source is 16-aligned, so its block A is the body's first source block).
// The chunk is stored in the same instruction as its segment's body chunks:
// no edge workgroup touches it and no 64-byte segment is written in two
// parts. 1 KiB frames: send 1.77 -> 1.59 ms; 256 B: 2.71-2.89
// -> 1.83 ms (profiles/r03_inreg_ab/v2/). The first form, a full two-frame
// assembly per chunk (masks and funnels per part, six shuffles per slot),
// was slower than the edge workgroups (profiles/r03_inreg_ab/).
__device__ __forceinline__ uint4 readlane4(const uint4& v, int l)
{
    return make_uint4((uint32_t)__builtin_amdgcn_readlane((int)v.x, l), (uint32_t)__builtin_amdgcn_readlane((int)v.y, l),
                      (uint32_t)__builtin_amdgcn_readlane((int)v.z, l), (uint32_t)__builtin_amdgcn_readlane((int)v.w, l));
}

// The 128-bit value v shifted up by `sh` bytes (0 <= sh < 16), as two 64-bit halves.
__device__ __forceinline__ uint4 shl_bytes(uint64_t lo, uint64_t hi, uint32_t sh)
{
    const uint32_t b = 8u * (sh & 7u);
    const uint64_t l1 = b ? lo << b : lo;
    const uint64_t h1 = b ? (hi << b) | (lo >> (64u - b)) : hi;
    const uint64_t L = sh < 8 ? l1 : 0, H = sh < 8 ? h1 : l1;
    return make_uint4((uint32_t)L, (uint32_t)(L >> 32), (uint32_t)H, (uint32_t)(H >> 32));
}

// general_region's send with in-region edge chunks (see above): every chunk
// of the region, body or edge, in one store round. js/fast/ph/sp/key are the
// chunks' frame lanes, classification, source phase, source block and
// rotated key; the lane's frame (lane < nf): ro/rng/dlo/dhi as in
// general_region, its header as words (h0, h1: <= 8 bytes, zero past pre),
// hm = its header start relative to the region (16-bit signed) | pre << 16,
// tk its key. A non-fast chunk holds exactly one frame's header bytes: frame
// j's (the chunk starts before j's body) or j + 1's; it is
//   [j's body tail] [the header, at q = header start - chunk] [the body head,
//   the header's frame's first source block, at q + pre]
// each part a shift of words and none masked but the tail.
__device__ __forceinline__ void general_region_ser_edges(const Pass& P, uint64_t base, uint32_t lane, uint32_t nf,
                                                        const uint32_t (&js)[kUnroll], const bool (&fast)[kUnroll],
                                                        const uint32_t (&ph)[kUnroll],
                                                        const uint8_t* const (&sp)[kUnroll],
                                                        const uint32_t (&key)[kUnroll], uint32_t rng,
                                                        uint32_t dlo, uint32_t dhi, uint32_t h0, uint32_t h1,
                                                        uint32_t hm, uint32_t tk)
{
    const uint4 z = make_uint4(0, 0, 0, 0);
    auto hstart = [](uint32_t m) { return (int)(int16_t)(m & 0xffffu); };
    bool tl[kUnroll], ob[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
        const uint32_t r = u * (uint32_t)kSlice + lane * (uint32_t)kChunk;
        const uint32_t rg = (uint32_t)__shfl((int)rng, (int)js[u], 64);
        const uint32_t bs = rg & 0xffffu, be = rg >> 16;
        tl[u] = !fast[u] && r >= bs && r < be;                 // frame j's body tail
        const uint32_t cnt = be - r < 16u ? be - r : 16u;
        ob[u] = (fast[u] && ph[u]) || (tl[u] && ph[u] + cnt > 16u);
    }
    // The region's last chunk takes a body head from the next region's first
    // chunk: loaded here by lane 63.
    uint4 hx = z;
    {
        const int R = (int)(kRegion - kChunk);
        const uint32_t jl = (uint32_t)__builtin_amdgcn_readlane((int)js[kUnroll - 1], 63);
        const uint32_t ml = (uint32_t)__builtin_amdgcn_readlane((int)hm, (int)jl);
        const int bsl = hstart(ml) + (int)(ml >> 16);
        int h = -1, bsh = 0;
        if (R < bsl && bsl < R + 16) {
            h = (int)jl;
            bsh = bsl;
        } else if (jl + 1 < nf) {
            const uint32_t mn = (uint32_t)__builtin_amdgcn_readlane((int)hm, (int)jl + 1);
            const int bsn = hstart(mn) + (int)(mn >> 16);
            if (bsn < R + 16) {
                h = (int)jl + 1;
                bsh = bsn;
            }
        }
        // a vector load from a full 64-bit VGPR address (as a wave-uniform
        // address it became a scalar load with the delta's low word as a
        // 32-bit SOFFSET, which does not carry: the block came back wrong)
        if (h >= 0 && lane == 63) {
            const uint64_t d = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)dlo, h) |
                               (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)dhi, h) << 32;
            uint64_t addr = reinterpret_cast<uint64_t>(P.src) + base + (uint64_t)bsh + d;
            asm volatile("" : "+v"(addr));
            hx = ld16(reinterpret_cast<const uint8_t*>(addr));
        }
    }
    uint4 a[kUnroll], b[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) a[u] = fast[u] || tl[u] ? ld16(sp[u]) : z;
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) b[u] = ob[u] ? ld16(sp[u] + 16) : z;
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
        const int R = (int)(u * (uint32_t)kSlice + lane * (uint32_t)kChunk);
        const uint32_t j = js[u], jn = j + 1 < nf ? j + 1 : j;
        // the header's frame, and its values with every lane active
        const uint32_t rg = (uint32_t)__shfl((int)rng, (int)j, 64);
        const uint32_t hf = R < (int)(rg & 0xffffu) ? j : jn;
        const uint32_t mf = (uint32_t)__shfl((int)hm, (int)hf, 64);
        const uint32_t x0 = (uint32_t)__shfl((int)h0, (int)hf, 64);
        const uint32_t x1 = (uint32_t)__shfl((int)h1, (int)hf, 64);
        const uint32_t kf = (uint32_t)__shfl((int)tk, (int)hf, 64);
        const uint4 N = from_next_lane(a[u], u + 1 < kUnroll ? readlane4(a[u + 1 < kUnroll ? u + 1 : u], 0) : hx);
        uint4 o = ph[u] ? funnel16(a[u], b[u], ph[u]) : a[u];
        xor4(o, key[u]);
        if (!fast[u]) {
            const int q = hstart(mf) - R;                 // -7 .. 15
            const int s = q + (int)(mf >> 16);            // 1 .. 23
            const uint64_t Hv = (uint64_t)x0 | (uint64_t)x1 << 32;
            // the tail: bytes [0, q) of o
            const uint32_t t = q > 0 ? (uint32_t)q : 0u;
            const uint64_t ml = t >= 8 ? ~0ull : (t ? (1ull << (8 * t)) - 1 : 0ull);
            const uint64_t mh = t > 8 ? (1ull << (8 * (t - 8))) - 1 : 0ull;
            uint4 w = make_uint4(o.x & (uint32_t)ml, o.y & (uint32_t)(ml >> 32), o.z & (uint32_t)mh,
                                 o.w & (uint32_t)(mh >> 32));
            // the header at q
            const uint4 Hs = q >= 0 ? shl_bytes(Hv, 0, (uint32_t)q)
                                    : make_uint4((uint32_t)(Hv >> (8 * -q)), (uint32_t)(Hv >> (8 * -q) >> 32), 0u, 0u);
            w = or4(w, Hs);
            // the body head at s
            if (s < 16) {
                uint4 W = N;
                xor4(W, kf);
                w = or4(w, shl_bytes((uint64_t)W.x | (uint64_t)W.y << 32, (uint64_t)W.z | (uint64_t)W.w << 32,
                                     (uint32_t)s));
            }
            o = w;
        }
        st16_region<kModeSer>(P.dst + base, (uint32_t)R, o);
    }
}

template <int kMode>
__device__ __forceinline__ void general_region(const Pass& P, uint32_t f0, uint32_t f1, uint64_t base,
                                               uint32_t lane, bool inreg = false)
{
    const uint32_t nf = f1 - f0 + 1;
    if (nf > 64) {
        general_region_search<kMode>(P, f0, f1, base, lane);
        return;
    }
    auto rel = [base](uint64_t x, uint64_t hi) -> uint32_t {
        return x <= base ? 0u : (x - base >= hi ? (uint32_t)hi : (uint32_t)(x - base));
    };
    uint32_t ro = (uint32_t)kRegion, rng = 0, kr = 0, dlo = 0, dhi = 0, h0 = 0, h1 = 0, hm = 0, tk = 0;
    if (lane < nf) {
        const FrameView v = frame_view<kMode>(P, f0 + lane);
        ro = rel(v.out_off, kRegion);
        rng = rel(v.body_start + v.body_len, kRegion + kChunk) << 16 | rel(v.body_start, kRegion);
        const uint64_t delta = v.src_off - v.body_start;           // src = out + delta
        dlo = (uint32_t)delta;
        dhi = (uint32_t)(delta >> 32);
        kr = rotr8(v.key, (uint32_t)(base - v.body_start) & 3u);
        if (kMode == kModeSer && inreg) {
            const uint4 H = ws_header_words(v.body_len, v.hb, v.key);
            h0 = H.x;
            h1 = H.y;
            // the header start, clamped below (a long frame's header far
            // before the region is simply before it)
            const int64_t ho = (int64_t)v.out_off - (int64_t)base;
            hm = ((uint32_t)(ho < -64 ? -64 : (int)ho) & 0xffffu) | v.pre << 16;
            tk = v.key;
        }
    }
    const uint8_t* sp[kUnroll];
    uint32_t ph[kUnroll], key[kUnroll];
    bool fast[kUnroll];
    uint32_t js[kUnroll];
    if (nf <= CFWS_GENERAL_SCAN) {
        // few frames: count the frame starts <= r, each start read once into
        // an SGPR (no LDS round trips; 1 KiB frames: send 1.813 -> 1.765 ms,
        // receive 1.458 -> 1.437, profiles/r03_small_ab/)
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) js[u] = 0;
        for (uint32_t c = 1; c < nf; ++c) {
            const uint32_t oc = (uint32_t)__builtin_amdgcn_readlane((int)ro, (int)c);
#pragma unroll
            for (int u = 0; u < kUnroll; ++u)
                js[u] += oc <= u * (uint32_t)kSlice + lane * (uint32_t)kChunk ? 1u : 0u;
        }
    } else {
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            const uint32_t r = u * (uint32_t)kSlice + lane * (uint32_t)kChunk;
            uint32_t j = 0;                             // largest frame with start <= r
#pragma unroll
            for (uint32_t step = 32; step >= 1; step >>= 1) {
                const uint32_t c = j + step;
                const uint32_t oc = (uint32_t)__shfl((int)ro, (int)(c & 63u), 64);
                if (c < nf && oc <= r) j = c;
            }
            js[u] = j;
        }
    }
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
        const uint32_t r = u * (uint32_t)kSlice + lane * (uint32_t)kChunk;
        const uint32_t j = js[u];
        const uint32_t rg = (uint32_t)__shfl((int)rng, (int)j, 64);
        const uint64_t d = (uint64_t)(uint32_t)__shfl((int)dlo, (int)j, 64) |
                           (uint64_t)(uint32_t)__shfl((int)dhi, (int)j, 64) << 32;
        key[u] = (uint32_t)__shfl((int)kr, (int)j, 64);
        fast[u] = r >= (rg & 0xffffu) && r + kChunk <= (rg >> 16);
        const uint64_t s = base + r + d;
        ph[u] = (uint32_t)(s & 15u);
        sp[u] = P.src + (s & ~uint64_t(15));
    }
    if (kMode == kModeSer && inreg) {
        general_region_ser_edges(P, base, lane, nf, js, fast, ph, sp, key, rng, dlo, dhi, h0, h1, hm, tk);
        return;
    }
    uint4 a[kUnroll], b[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) a[u] = fast[u] ? ld16(sp[u]) : make_uint4(0, 0, 0, 0);
    // the block holding the chunk's last byte: a body byte, inside the source
    if (kMode == kModeDeser) {
        // ... loaded by this lane only when the next lane does not hold it
        // as its own block (the next chunk in the same frame's body): over
        // DPP. The receive only: 256 B frames 1.69 -> 1.57 ms, 1 KiB 1.40
        // -> 1.39; the send measured slower with it (1 KiB 1.76 -> 1.98 ms,
        // profiles/r03_small_ab/dpp/)
        bool own[kUnroll];
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            const uint32_t nj = from_next_lane(js[u], 0xffffffffu);
            const uint32_t nf_ = from_next_lane(fast[u] ? 1u : 0u, 0u);
            own[u] = fast[u] && ph[u] && !(nj == js[u] && nf_);
        }
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) b[u] = own[u] ? ld16(sp[u] + 16) : make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            const uint4 nb = from_next_lane(a[u], b[u]);    // every lane: DPP needs the full wave
            if (!fast[u]) continue;
            uint4 o = ph[u] ? funnel16(a[u], own[u] ? b[u] : nb, ph[u]) : a[u];
            xor4(o, key[u]);
            st16_region<kMode>(P.dst + base, u * (uint32_t)kSlice + lane * (uint32_t)kChunk, o);
        }
        return;
    }
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) b[u] = fast[u] && ph[u] ? ld16(sp[u] + 16) : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
        if (!fast[u]) continue;
        uint4 o = ph[u] ? funnel16(a[u], b[u], ph[u]) : a[u];
        xor4(o, key[u]);
        st16_region<kMode>(P.dst + base, u * (uint32_t)kSlice + lane * (uint32_t)kChunk, o);
    }
}

// The region holding the pass end when a capacity cut ends the pass inside a
// body: the body chunks below the end only, each store clipped at the
// capacity (the other region paths write whole bodies' chunks, which would
// run past a cut).
template <int kMode>
__device__ __forceinline__ void tail_region(const Pass& P, uint32_t f0, uint32_t f1, uint64_t base,
                                            uint32_t lane)
{
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
        const uint64_t D = base + u * kSlice + lane * kChunk;
        if (D >= P.total) continue;
        uint32_t lo = f0, hi = f1;                  // largest f with offs[f] <= D
        while (lo < hi) {
            const uint32_t mid = (lo + hi + 1) >> 1;
            if (P.offs[mid] <= D) lo = mid; else hi = mid - 1;
        }
        const FrameView v = frame_view<kMode>(P, lo);
        if (D >= v.body_start && D + kChunk <= v.body_start + v.body_len)
            store_chunk(P, D, body_chunk(P.src, v, D));
    }
}

// Two threads per frame (part 0: the chunks before the body -- headers;
// part 1: the chunks reaching past the body end -- the boundary into the
// next frame, padding, the pass end): the 16-byte chunks that START inside
// the frame's output range and do not lie entirely inside its body. The
// kernel is latency-bound (descriptor -> offsets -> source blocks -> store),
// so the work is spread thin: 64-thread blocks, edge_chunk inlined.
#ifndef CFWS_EDGE_THREADS
#define CFWS_EDGE_THREADS 64
#endif
constexpr uint32_t kEdgeThreads = CFWS_EDGE_THREADS;

// Edge thread t -> (frame, part): each 128 threads take 64 consecutive
// frames, lanes 0-63 part 0 and lanes 64-127 part 1, so a wave runs one part
// only. (Parts alternating by lane ran both parts' code in every wave: on
// 4 M x 1 KiB frames the serialize edge pass issued 892 VALU instructions
// per wave.) edge_threads(n) threads cover every frame's two parts.
__host__ __device__ constexpr uint64_t edge_threads(uint64_t n) { return (n + 63) / 64 * 128; }

__device__ __forceinline__ uint64_t edge_thread_frame(uint64_t t) { return (t >> 7) * 64 + (t & 63); }

__device__ __forceinline__ uint32_t edge_thread_part(uint64_t t) { return (uint32_t)(t >> 6) & 1u; }

// The edge chunks of frame f in pass P (part 0: before the body; part 1:
// reaching past the body end).
template <int kMode>
__device__ __forceinline__ void edge_frame(const Pass& P, uint64_t f, uint32_t part, uint64_t dmin = 0)
{
    // Everything the chunks need that depends on f alone is loaded up front
    // (frame f and f + 1's descriptors, statuses, offsets): one memory round
    // trip before the source blocks instead of a chain of six.
    const uint32_t n = P.n_frames;
    const uint32_t fa = (uint32_t)f, fb = fa + 1 < n ? fa + 1 : fa;
    const FrameView va = frame_view<kMode>(P, fa);
    const FrameView vb = frame_view<kMode>(P, fb);
    const uint64_t o2 = fa + 2 < n ? P.offs[fa + 2] : ~uint64_t(0);
    const uint64_t o1 = fa + 1 < n ? vb.out_off : ~uint64_t(0);
    const uint64_t lo = va.out_off;
    uint64_t hi = fa + 1 < n ? vb.out_off : P.total;
    if (hi > P.total) hi = P.total;
    if (lo >= hi) return;
    const FrameView& v = va;
    const uint64_t be = v.body_start + v.body_len;
    uint64_t first = (lo + 15) & ~uint64_t(15);
    if (first < dmin) first = dmin;                   // chunks below dmin: written in-region
    if (part == 0) {
        // chunks before the body (headers): D < body_start
        for (uint64_t D = first; D < hi && D < v.body_start; D += 16)
            store_chunk(P, D, edge_chunk<kMode>(P, fa, D, va, vb, o1, o2));
        return;
    }
    // chunks reaching past the body end (boundary, padding, pass end)
    uint64_t d0 = be >= 15 ? ((be - 15 + 15) & ~uint64_t(15)) : 0;  // first D with D + 16 > be
    if (d0 < first) d0 = first;
    if (d0 < v.body_start) d0 = (v.body_start + 15) & ~uint64_t(15);  // header chunks: part 0
    for (uint64_t D = d0; D < hi; D += 16) {
        if (D >= be && D + 16 <= hi)          // pure alignment padding / OOM body
            store_chunk(P, D, make_uint4(0, 0, 0, 0));
        else
            store_chunk(P, D, edge_chunk<kMode>(P, fa, D, va, vb, o1, o2));
    }
}

template <int kMode>
__global__ void __launch_bounds__(kEdgeThreads)
edge_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
            const cfws_frame_desc_t* __restrict__ desc, const int32_t* __restrict__ status,
            const uint64_t* __restrict__ offs, const uint64_t* __restrict__ total_p,
            const uint64_t* __restrict__ base_p, uint64_t capacity, uint32_t n_frames,
            uint32_t klass, uint32_t sid, const cfws_frame_desc_t* __restrict__ parent)
{
    const uint64_t t = uint64_t(blockIdx.x) * kEdgeThreads + threadIdx.x;
    const uint64_t f = edge_thread_frame(t);
    if (f >= n_frames) return;
    const uint64_t out_base = base_p ? *base_p : 0;
    Pass P;
    P.src = src;
    P.dst = dst + out_base;
    P.desc = desc;
    P.status = status;
    P.offs = offs;
    P.total = *total_p;
    P.capacity = capacity - out_base;
    P.n_frames = n_frames;
    P.klass = klass;
    P.sid = sid;
    P.parent = parent;
    edge_frame<kMode>(P, f, edge_thread_part(t));
}

// Deserialize with reassembly (CFWS_DESERIALIZE_REASSEMBLE): the edge chunks
// of frame f in the one pass that holds its bytes (data frames in pass 0,
// control frames in pass 1 from hdr[2]). Pass 0's stores stop at its data
// bytes: pass 1 starts there, at an unaligned address, and its edge chunks
// are written concurrently.
__device__ __forceinline__ void reasm_edge_frame(const uint8_t* __restrict__ src,
                                                 uint8_t* __restrict__ dst,
                                                 const cfws_frame_desc_t* __restrict__ desc,
                                                 const int32_t* __restrict__ status,
                                                 const uint64_t* __restrict__ offs0,
                                                 const uint64_t* __restrict__ offs1,
                                                 const uint64_t* __restrict__ hdr, uint64_t capacity,
                                                 uint32_t n_frames, uint64_t f, uint32_t part)
{
    const uint32_t p = is_control(desc[f].opcode) ? 1u : 0u;
    const uint64_t out_base = p ? hdr[2] : 0;
    Pass P;
    P.src = src;
    P.dst = dst + out_base;
    P.desc = desc;
    P.status = status;
    P.offs = p ? offs1 : offs0;
    P.total = hdr[p];
    P.capacity = p ? capacity - out_base : (hdr[0] < capacity ? hdr[0] : capacity);
    P.n_frames = n_frames;
    P.klass = p ? kClassControl : kClassData;
    P.sid = 0;
    P.parent = nullptr;
    edge_frame<kModeDeser>(P, f, part);
}

// The streaming regions of one launch (the waves of the non-edge
// workgroups, one 4 KiB region each per grid stride). kInreg: WS serialize
// with in-region edge chunks (general_region_ser_edges).
template <int kMode, bool kInreg>
__device__ __forceinline__ void region_loop(const Pass& P, const uint64_t* __restrict__ offs,
                                            const uint32_t* __restrict__ region_map, uint32_t n_frames,
                                            uint32_t edge_blocks, uint32_t sidx)
{
    const uint64_t n_regions = (P.total + kRegion - 1) / kRegion;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t stride = uint64_t(gridDim.x - edge_blocks) * kWaves;

    for (uint64_t r = uint64_t(sidx) * kWaves + wave; r < n_regions;
         r += stride) {
        const uint64_t base = r * kRegion;
        const uint64_t end = base + kRegion;
        // The plan writes every entry in [0, n_regions]; the clamps only keep
        // a corrupted workspace from turning into an out-of-bounds read.
        uint32_t f0 = region_map[r];
        uint32_t f1 = region_map[r + 1];
        if (f1 >= n_frames) f1 = n_frames - 1;
        if (f0 > f1) f0 = f1;
        if (end > P.total) {                  // the pass end (a capacity cut may fall in a body)
            tail_region<kMode>(P, f0, f1, base, lane);
            continue;
        }
#if CFWS_GENERAL_DIRECT
        // f0 + 1 and f0 + 2 start inside the region: a run of small frames,
        // straight to the per-lane views without the offset round trip below
        // (general_region ignores frames that start at or after the end).
        // The receive, and the in-region send: 1 KiB frames receive 1.437 ->
        // 1.385 ms, 256 B 1.758 -> 1.686; in-region send 1 KiB 1.58 -> 1.54,
        // 256 B 1.81-1.83 -> 1.69-1.70 (profiles/r03_inreg_ab/v3/); the send
        // with edge workgroups measured slower with it (256 B 2.74 -> 2.93
        // ms, profiles/r03_small_ab/)
        if ((kMode == kModeDeser || (kInreg && kMode == kModeSer)) && f1 >= f0 + 3) {
            general_region<kMode>(P, f0, f1, base, lane, kInreg);
            continue;
        }
#endif
        // region_map[r + 1] holds the NEXT region's first byte; frames that
        // start at or after this region's end do not touch it.
        if (f1 > f0 && offs[f0 + 1] >= end) f1 = f0;
        const FrameView va = frame_view<kMode>(P, f0);
        constexpr bool kEdges = kInreg && kMode == kModeH2Ser;   // edge chunks in-region
        // the in-region WS send: every region holding a header goes to
        // general_region, whose edge chunks need no frame-size bound
        // (payloads over 2,000 bytes, up to CFWS_SER_INREG_MAX, make such regions
        // one- or two-frame ones)
        constexpr bool kSerGen = kInreg && kMode == kModeSer;
        if (f0 == f1) {
            if (base >= va.body_start && end <= va.body_start + va.body_len)
                fast_region<kMode>(P, va, base, lane);
            else if (kSerGen)
                general_region<kMode>(P, f0, f0, base, lane, true);
            else
                two_frame_region<kMode, kEdges>(P, va, va, base, lane);   // partial body, one frame
        } else if (f1 == f0 + 1 || offs[f0 + 2] >= end) {
            if (kSerGen)
                general_region<kMode>(P, f0, f0 + 1, base, lane, true);
            else
                two_frame_region<kMode, kEdges>(P, va, frame_view<kMode>(P, f0 + 1), base, lane);
        } else {
            general_region<kMode>(P, f0, f1, base, lane, kInreg);
        }
    }
}

// WS serialize / deserialize and the fused WS-over-HTTP/2 send carry their
// edge chunks in the streaming launch. The send's edge code spills 12 bytes
// per lane there (96 VGPRs, 5 waves per SIMD, the residency the LDS
// reservation sets anyway); the spills sit in the edge branch only, none in
// the region loop. It still measured 12 us per config-5 step faster than its
// own launch (xform<3> 352 us against 338 + 26), and 1.5 % faster than 4
// workgroups per CU without spills (CFWS_H2SER_MIN_BLOCKS=4: 122 VGPRs). The
// two-pass wrap (max_frame_size < 64) keeps a separate edge launch.
__host__ __device__ constexpr bool has_edge_blocks(int mode)
{
    return mode == kModeSer || mode == kModeDeser || mode == kModeH2Ser;
}

// The streaming kernel: serialize (kSer) = header + (masked) payload into
// the wire arena; deserialize = copy + unmask into the payload arena.
// `edge_blocks` workgroups write the edge chunks (edge_frame: two threads
// per frame, one part per wave); the rest stream the regions, writing every
// 16-byte chunk that lies inside one frame's body. The two chunk sets are
// disjoint. The edge workgroups ride in the streaming launch -- the first
// ones dispatched, or every `edge_stride`-th when frames are small
// (edge_interleave) -- so their latency-bound chains run under the stream
// instead of as a launch of their own after it (which cost 17 us serialize /
// 4 us deserialize on config 2, plus a kernel boundary).
// The wave-per-EU floor keeps the merged kernel at <= 102 VGPRs, so the
// 5 workgroups per CU the LDS reservation allows stay resident.
// workgroups per CU the send's streaming kernel is compiled for (A/B knob)
#ifndef CFWS_H2SER_MIN_BLOCKS
#define CFWS_H2SER_MIN_BLOCKS 5
#endif
#ifndef CFWS_XFORM_MIN_BLOCKS
#define CFWS_XFORM_MIN_BLOCKS 5
#endif
template <int kMode>
__global__ void __launch_bounds__(kThreads, kMode == kModeH2Ser ? CFWS_H2SER_MIN_BLOCKS : CFWS_XFORM_MIN_BLOCKS)
xform_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
             const cfws_frame_desc_t* __restrict__ desc, const int32_t* __restrict__ status,
             const uint64_t* __restrict__ offs, const uint32_t* __restrict__ region_map,
             const uint64_t* __restrict__ total_p, const uint64_t* __restrict__ base_p,
             uint64_t capacity, uint32_t n_frames, uint32_t klass, uint32_t sid,
             const cfws_frame_desc_t* __restrict__ parent, uint32_t edge_blocks,
             const uint64_t* __restrict__ reasm_offs1, uint32_t edge_stride,
             const uint32_t* __restrict__ inreg_flag)
{
    // Which workgroups are edge workgroups: the first edge_blocks, or (edge
    // stride s > 0) every s-th one, spread through the grid
    uint32_t eidx = blockIdx.x, sidx = blockIdx.x - edge_blocks;
    bool is_edge = blockIdx.x < edge_blocks;
    if (edge_stride) {
        const uint32_t k = blockIdx.x / edge_stride;
        is_edge = blockIdx.x == k * edge_stride && k < edge_blocks;
        eidx = k;
        sidx = blockIdx.x - (k + 1 < edge_blocks ? k + 1 : edge_blocks);
    }
    if (kMode == kModeDeser && reasm_offs1 && is_edge) {
        // reassembly pass 0: the edge chunks of both passes (total_p = hdr)
        const uint64_t t = uint64_t(eidx) * kThreads + threadIdx.x;
        if (edge_thread_frame(t) < n_frames)
            reasm_edge_frame(src, dst, desc, status, offs, reasm_offs1, total_p, capacity, n_frames,
                             edge_thread_frame(t), edge_thread_part(t));
        return;
    }
    const uint64_t out_base = base_p ? *base_p : 0;
    Pass P;
    P.src = src;
    P.dst = dst + out_base;
    P.desc = desc;
    P.status = status;
    P.offs = offs;
    P.total = *total_p;                              // clamped by the plan
    P.capacity = capacity - out_base;
    P.n_frames = n_frames;
    P.klass = klass;
    P.sid = sid;
    P.parent = parent;
    // In-region edge chunks (the plan's flag word clear): WS serialize of
    // 80..3,584-byte frames (the general regions write them) and the fused
    // HTTP/2 send of DATA frames >= kRegion + 32 bytes (the two-frame
    // regions write them): every edge chunk below the tail region.
    const bool inreg = (kMode == kModeSer || kMode == kModeH2Ser) && inreg_flag && *inreg_flag == 0;
    if (has_edge_blocks(kMode) && is_edge) {
        const uint64_t t = uint64_t(eidx) * kThreads + threadIdx.x;
        const uint64_t f = edge_thread_frame(t);
        if (f >= n_frames) return;
        uint64_t dmin = 0;
        if (inreg) {
            // only the tail region's chunks are left (tail_region writes
            // body chunks only); the frames before its first have none
            dmin = P.total / kRegion * kRegion;
            if (dmin >= P.total || f < region_map[dmin / kRegion]) return;
        }
        edge_frame<kMode>(P, f, edge_thread_part(t), dmin);
        return;
    }
    // the region loop, instantiated apart for the in-region send so that the
    // other loops' code stays as it was (config 3's send lost 6 % when one
    // loop carried both)
    if ((kMode == kModeSer || kMode == kModeH2Ser) && inreg)
        region_loop<kMode, true>(P, offs, region_map, n_frames, edge_blocks, sidx);
    else
        region_loop<kMode, false>(P, offs, region_map, n_frames, edge_blocks, sidx);
}

// ---------------------------------------------------------------------------
// plan kernels
// ---------------------------------------------------------------------------
// WS header at s of data[0, size) (co_ws_frame.c:131-213), with the callers'
// two-byte precheck (co_ws_client.c:202-206): the reference's decisions in
// its order (MORE_DATA before DATA_TOO_BIG). d gets what the reference has
// written into the frame by the time it returns.
// `at(i)` returns byte i of the data (an arena, or header bytes held in
// registers: parse_ws_header_regs).
template <typename At>
__device__ __forceinline__ int32_t parse_ws_header_by(At at, uint64_t size, uint64_t s,
                                                      uint64_t max_payload, cfws_frame_desc_t& d)
{
    d.payload_off = 0;
    d.wire_off = s;
    d.payload_size = 0;
    d.mask_key = 0;
    d.fin = 0;
    d.opcode = 0;
    d.mask = 0;
    d.header_size = 0;
    if (s > size || size - s < 2) return CFWS_PARSE_MORE_DATA;
    const uint32_t b0 = at(s), b1 = at(s + 1);
    d.fin = (uint8_t)(b0 >> 7);
    d.opcode = (uint8_t)(b0 & 0x7fu);
    if (d.opcode > 0x0f) return CFWS_ERROR_INVALID_FRAME;
    d.mask = (uint8_t)(b1 >> 7);
    const uint32_t l7 = b1 & 0x7fu;
    uint64_t p = s + 2;
    if (l7 <= 125) {
        d.payload_size = l7;
    } else {
        const uint32_t ext = (l7 == 126) ? 2u : 8u;
        if (size - p < ext) return CFWS_PARSE_MORE_DATA;
        uint64_t len = 0;
        if (ext == 2) {
            len = (uint64_t)at(p) << 8 | at(p + 1);
        } else {
#pragma unroll
            for (uint32_t i = 0; i < 8; ++i) len = (len << 8) | at(p + i);
        }
        d.payload_size = len;
        p += ext;
    }
    if (d.mask) {
        if (size - p < 4) return CFWS_PARSE_MORE_DATA;
        d.mask_key = at(p) | at(p + 1) << 8 | at(p + 2) << 16 | at(p + 3) << 24;
        p += 4;
    }
    d.header_size = (uint8_t)(p - s);
    if (size - p < d.payload_size) return CFWS_PARSE_MORE_DATA;
    if (d.payload_size > max_payload) return CFWS_ERROR_DATA_TOO_BIG;
    return CFWS_PARSE_COMPLETE;
}

// The same parse over header bytes gathered into registers: w holds bytes
// 0-15 of the frame little-endian (a frame starts at 0, `size` bytes long).
// Byte selection is by compare + select, so w stays in VGPRs (an indexed
// byte array here was placed in LDS).
__device__ __forceinline__ int32_t parse_ws_header_regs(const uint32_t (&w)[4], uint64_t size,
                                                        uint64_t max_payload, cfws_frame_desc_t& d)
{
    const uint32_t w0 = w[0], w1 = w[1], w2 = w[2], w3 = w[3];
    return parse_ws_header_by(
        [=](uint64_t i) -> uint32_t {
            const uint32_t q = (uint32_t)(i >> 2);
            const uint32_t x = q == 0 ? w0 : q == 1 ? w1 : q == 2 ? w2 : w3;
            return (x >> (8u * (uint32_t)(i & 3u))) & 0xffu;
        },
        size, 0, max_payload, d);
}

// Bytes [b, b + k) of global memory, k <= 16, into w (little-endian; bytes
// past k are unspecified): the up to five aligned dwords that hold them,
// issued as independent loads, funnel-shifted by b's alignment. Only dwords
// holding at least one of the k bytes are read (no access past the span's
// last mapped dword).
__device__ __forceinline__ void load_span16(const uint8_t* b, uint32_t k, uint32_t (&w)[4])
{
    const uint32_t o = (uint32_t)(reinterpret_cast<uintptr_t>(b) & 3u);
    const uint32_t* p = reinterpret_cast<const uint32_t*>(b - o);
    const uint32_t nd = k ? (o + k + 3u) >> 2 : 0u;
    uint32_t x[5];
#pragma unroll
    for (uint32_t j = 0; j < 5; ++j) x[j] = j < nd ? p[j] : 0u;
#pragma unroll
    for (uint32_t t = 0; t < 4; ++t) w[t] = __builtin_amdgcn_alignbyte(x[t + 1], x[t], o);
}

// The header at s of wire[0, size): its up to 14 bytes in one round of
// independent dword loads (load_span16), parsed from registers. A byte-wise
// parse from memory takes up to 14 single-byte requests in three dependent
// rounds (first two bytes, the length, the key): with frames ~1 KiB apart
// every request is a line of its own. On 4 M x 1 KiB frames the plan's
// header pass went from 311 to 182-198 us (two aligned 16-byte loads instead
// of the dwords: no faster).
__device__ __forceinline__ int32_t parse_ws_header(const uint8_t* __restrict__ wire, uint64_t size,
                                                   uint64_t s, uint64_t max_payload,
                                                   cfws_frame_desc_t& d)
{
    const uint64_t avail = s <= size ? size - s : 0;
    uint32_t w[4];
    load_span16(wire + s, avail < 14 ? (uint32_t)avail : 14u, w);
    const int32_t st = parse_ws_header_regs(w, avail, max_payload, d);
    d.wire_off = s;
    return st;
}

// Exclusive block scan of one value per thread; *block_total gets the sum.
__device__ __forceinline__ uint64_t block_exclusive_scan(uint64_t x, uint64_t* s_wave,
                                                         uint64_t* block_total)
{
    const uint32_t lane = threadIdx.x & 63u, wid = threadIdx.x >> 6;
    uint64_t inc = x;
#pragma unroll
    for (uint32_t o = 1; o < 64; o <<= 1) {
        const uint64_t y = __shfl_up(inc, o, 64);
        if (lane >= o) inc += y;
    }
    __syncthreads();
    if (lane == 63) s_wave[wid] = inc;
    __syncthreads();
    uint64_t before = 0, all = 0;
#pragma unroll
    for (uint32_t w = 0; w < kWaves; ++w) {
        if (w < wid) before += s_wave[w];
        all += s_wave[w];
    }
    *block_total = all;
    return before + inc - x;
}

__global__ void __launch_bounds__(kThreads)
scan_reduce_kernel(const uint64_t* __restrict__ vals, uint64_t n, uint64_t* __restrict__ partials)
{
    __shared__ uint64_t s_wave[kWaves];
    const uint64_t b0 = uint64_t(blockIdx.x) * kScanBlock;
    uint64_t sum = 0;
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
        const uint64_t i = b0 + uint64_t(k) * kThreads + threadIdx.x;
        if (i < n) sum += vals[i];
    }
    uint64_t total;
    block_exclusive_scan(sum, s_wave, &total);
    if (threadIdx.x == 0) partials[blockIdx.x] = total;
}

// One workgroup's exclusive scan of nb block sums, in place; *grand gets the
// total. A step takes kThreads x kPartialItems sums, kPartialItems
// consecutive ones per thread with all their loads in flight: the 16,384
// sums of a 4 M-frame plan in one step, 19 us (one sum per thread per step:
// 64 dependent steps, 46 us; 16 per thread through LDS with coalesced loads
// and stores: 4 steps, 29-35 us -- each step's round trip costs more than
// the strided access).
constexpr int kPartialItems = 64;

__device__ __forceinline__ void scan_partials_block(uint64_t* __restrict__ partials, uint64_t nb,
                                                    uint64_t* __restrict__ grand, uint64_t* s_wave)
{
    uint64_t carry = 0;
    for (uint64_t b = 0; b < nb; b += uint64_t(kThreads) * kPartialItems) {
        const uint64_t i0 = b + uint64_t(threadIdx.x) * kPartialItems;
        uint64_t v[kPartialItems];
        uint64_t sum = 0;
#pragma unroll
        for (int k = 0; k < kPartialItems; ++k) {
            v[k] = i0 + k < nb ? partials[i0 + k] : 0;
            sum += v[k];
        }
        uint64_t tot;
        uint64_t run = block_exclusive_scan(sum, s_wave, &tot) + carry;
#pragma unroll
        for (int k = 0; k < kPartialItems; ++k) {
            if (i0 + k < nb) partials[i0 + k] = run;
            run += v[k];
        }
        carry += tot;
    }
    if (threadIdx.x == 0) *grand = carry;
}

__global__ void __launch_bounds__(kThreads)
scan_partials_kernel(uint64_t* __restrict__ partials, uint64_t nb, uint64_t* __restrict__ grand)
{
    __shared__ uint64_t s_wave[kWaves];
    scan_partials_block(partials, nb, grand, s_wave);
}

// scan_partials_kernel for up to two passes in one launch (block p: pass p).
__global__ void __launch_bounds__(kThreads)
scan_partials2_kernel(uint64_t* __restrict__ partials0, uint64_t* __restrict__ partials1, uint64_t nb,
                      uint64_t* __restrict__ grand0, uint64_t* __restrict__ grand1)
{
    __shared__ uint64_t s_wave[kWaves];
    scan_partials_block(blockIdx.x ? partials1 : partials0, nb, blockIdx.x ? grand1 : grand0, s_wave);
}

__global__ void __launch_bounds__(kThreads)
scan_apply_kernel(uint64_t* __restrict__ vals, uint64_t n, const uint64_t* __restrict__ partials)
{
    __shared__ uint64_t s_wave[kWaves];
    const uint64_t i0 = uint64_t(blockIdx.x) * kScanBlock + uint64_t(threadIdx.x) * kScanItems;
    uint64_t v[kScanItems];
    uint64_t sum = 0;
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
        v[k] = (i0 + k < n) ? vals[i0 + k] : 0;
        sum += v[k];
    }
    uint64_t tot;
    uint64_t run = block_exclusive_scan(sum, s_wave, &tot) + partials[blockIdx.x];
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
        if (i0 + k < n) vals[i0 + k] = run;
        run += v[k];
    }
}

// Fills the region -> first-frame map of one pass over [0, total).
__device__ __forceinline__ void map_regions(const uint64_t* __restrict__ offs, uint64_t f, uint64_t n,
                                            uint64_t grand, uint64_t total, uint32_t* __restrict__ map)
{
    const uint64_t lo = offs[f];
    const uint64_t hi = (f + 1 < n) ? offs[f + 1] : grand;
    const uint64_t a = lo < total ? lo : total;
    const uint64_t b = hi < total ? hi : total;
    if (b > a) {
        const uint64_t r1 = (b + kRegion - 1) / kRegion;
        for (uint64_t r = (a + kRegion - 1) / kRegion; r < r1; ++r) map[r] = (uint32_t)f;
    }
    if (f == n - 1) map[(total + kRegion - 1) / kRegion] = (uint32_t)(n - 1);
}

// Region-map entries of one frame's output bytes [lo, hi) of a pass over
// [0, total): every region whose first byte lies inside gets the frame.
__device__ __forceinline__ void map_range(uint64_t lo, uint64_t hi, uint64_t f, uint64_t total,
                                          uint32_t* __restrict__ map)
{
    const uint64_t a = lo < total ? lo : total;
    const uint64_t b = hi < total ? hi : total;
    if (b > a) {
        const uint64_t r1 = (b + kRegion - 1) / kRegion;
        for (uint64_t r = (a + kRegion - 1) / kRegion; r < r1; ++r) map[r] = (uint32_t)f;
    }
}

// This block's exclusive prefix and the grand total, straight from the
// per-block sums the reduce kernel wrote (plans of up to kSelfScanBlocks
// blocks: every apply block reads them all, <= 16 KiB from L2, instead of
// a scan launch between the two).
constexpr uint64_t kSelfScanBlocks = 2048;

__device__ __forceinline__ void prefix_from_partials(const uint64_t* __restrict__ partials, uint64_t nb,
                                                     uint64_t b, uint64_t* s_wave, uint64_t& before,
                                                     uint64_t& all)
{
    uint64_t xb = 0, xa = 0;
    for (uint64_t i = threadIdx.x; i < nb; i += kThreads) {
        const uint64_t v = partials[i];
        xa += v;
        if (i < b) xb += v;
    }
    block_exclusive_scan(xb, s_wave, &before);
    block_exclusive_scan(xa, s_wave, &all);
}

// ---- single-pass plans (more than kSelfScanBlocks blocks) --------------------
// A plan of many blocks scans its block sums with a decoupled look-back
// instead of a scan launch and a second pass over the frames: each block
// takes a ticket (so every lower ticket is already running), publishes its
// sum (flag 1), finds its exclusive prefix from the words of the blocks
// below it, 64 at a time, and publishes the inclusive prefix (flag 2). A
// block's flag and value are one 64-bit word (value << 2 | flag: sums below
// 2^62 bytes, far above any arena), stored and
// loaded whole by device-scope atomics (coherent across the XCDs' L2s by
// themselves), so a reader never sees a flag without its value and nothing
// has to be ordered: a publish is one store the block does not wait for, a
// poll one load. (The first form kept flags and values apart: each publish
// waited for its value's store before the flag's, and each poll loaded the
// value after the flag -- two more round trips per block, which under a
// saturated memory system bound the plans by look-back latency. Release /
// acquire fences would write back and invalidate the whole L2 at each
// publish and each poll: measured 2 ms per plan on 16 K blocks.)
//
// The words live in the workspace's look area after the u32 ticket (word
// 0), the u32 flag words 1..sb + 1 that some plans leave for their execute,
// and padding to 8 bytes (look_state_index, look_bytes); all of it is zeroed
// before the launch.

__device__ __forceinline__ uint64_t* look_states(uint32_t* look)
{
    return reinterpret_cast<uint64_t*>(look + look_state_index(gridDim.x));
}

__device__ __forceinline__ uint32_t plan_ticket(uint32_t* look, uint32_t* s_bid)
{
    if (threadIdx.x == 0) *s_bid = __hip_atomic_fetch_add(look, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    return *s_bid;
}

// Wave 0 of block b (every lane): b's exclusive prefix, after publishing
// `total` as b's sum; then b's inclusive prefix is published. Blocks below
// b that have not published yet (flag 0) hold a lower ticket, so they are
// running and publish without waiting on anyone.
__device__ __forceinline__ uint64_t plan_lookback(uint32_t b, uint64_t total, uint64_t* state)
{
    const uint32_t lane = threadIdx.x & 63u;
    if (b == 0) {
        if (lane == 0) __hip_atomic_store(&state[0], total << 2 | 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return 0;
    }
    if (lane == 0) __hip_atomic_store(&state[b], total << 2 | 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint64_t excl = 0;
    int64_t hi = (int64_t)b - 1;                      // window [hi - 63, hi], lane l: hi - l
    while (true) {
        const int64_t i = hi - (int64_t)lane;
        uint64_t w = 2u;                              // below block 0: an inclusive 0
        if (i >= 0) {
            do {
                w = __hip_atomic_load(&state[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if ((w & 3u) == 0u) __builtin_amdgcn_s_sleep(2);
            } while ((w & 3u) == 0u);
        }
        // the nearest inclusive prefix (lowest lane) ends the walk
        const uint64_t pm = __ballot((w & 3u) == 2u);
        const uint32_t stop = pm ? (uint32_t)__builtin_ctzll(pm) : 64u;
        uint64_t c = lane <= stop ? w >> 2 : 0;
#pragma unroll
        for (uint32_t o = 32; o >= 1; o >>= 1) c += __shfl_xor(c, o, 64);
        excl += c;
        if (pm) break;
        hi -= 64;
    }
    if (lane == 0) __hip_atomic_store(&state[b], (excl + total) << 2 | 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return excl;
}

// ---- plans: two launches each (three above kSelfScanBlocks blocks) ---------
// 1. per frame: sizes (serialize: header size, co_ws_frame.c:41-91;
//    deserialize: the header decode) + the block's sum;
// (2. scan_partials_kernel: the block sums, one block per pass -- only when
//    there are more than kSelfScanBlocks blocks; otherwise step 3 sums them);
// 3. per block: exclusive offsets of its frames, then everything the
//    offsets decide (descriptor offsets, capacity rule, region maps, totals).

// Offsets into the descriptors, the capacity rule (a COMPLETE frame with a
// payload that does not fit gets CFWS_ERROR_OUT_OF_MEMORY, like the
// reference's failed malloc, co_ws_frame.c:216-223), region maps, totals.
__global__ void __launch_bounds__(kThreads)
deserialize_plan_apply_kernel(cfws_frame_desc_t* __restrict__ desc, int32_t* __restrict__ status,
                              uint64_t* __restrict__ vals0, uint64_t* __restrict__ vals1, uint64_t n,
                              const uint64_t* __restrict__ partials0,
                              const uint64_t* __restrict__ partials1, uint64_t nb,
                              uint32_t self_scan, uint64_t* __restrict__ hdr,
                              uint64_t capacity, uint32_t reassemble, uint32_t* __restrict__ map0,
                              uint32_t* __restrict__ map1, uint64_t* __restrict__ user_total)
{
    __shared__ uint64_t s_wave[kWaves];
    uint64_t pre0, pre1 = 0, g0, g1 = 0;
    if (self_scan) {
        prefix_from_partials(partials0, nb, blockIdx.x, s_wave, pre0, g0);
        if (reassemble) prefix_from_partials(partials1, nb, blockIdx.x, s_wave, pre1, g1);
    } else {
        pre0 = partials0[blockIdx.x];
        g0 = hdr[3];
        if (reassemble) {
            pre1 = partials1[blockIdx.x];
            g1 = hdr[4];
        }
    }
    const uint64_t t0 = g0 < capacity ? g0 : capacity;
    const uint64_t room1 = capacity - t0;
    const uint64_t t1 = g1 < room1 ? g1 : room1;
    const uint64_t i0 = uint64_t(blockIdx.x) * kPlanBlock + uint64_t(threadIdx.x) * kPlanItems;
    uint64_t v0[kPlanItems], v1[kPlanItems];
    uint64_t s0 = 0, s1 = 0;
#pragma unroll
    for (int k = 0; k < kPlanItems; ++k) {
        v0[k] = (i0 + k < n) ? vals0[i0 + k] : 0;
        v1[k] = (reassemble && i0 + k < n) ? vals1[i0 + k] : 0;
        s0 += v0[k];
        s1 += v1[k];
    }
    uint64_t tot;
    uint64_t run0 = block_exclusive_scan(s0, s_wave, &tot) + pre0;
    uint64_t run1 = 0;
    if (reassemble) run1 = block_exclusive_scan(s1, s_wave, &tot) + pre1;
#pragma unroll
    for (int k = 0; k < kPlanItems; ++k) {
        const uint64_t f = i0 + k;
        if (f < n) {
            vals0[f] = run0;
            const bool ctl = reassemble && is_control(desc[f].opcode);
            const uint64_t off = ctl ? g0 + run1 : run0;
            desc[f].payload_off = off;
            const uint64_t len = desc[f].payload_size;
            if (status[f] == CFWS_PARSE_COMPLETE && len > 0 && off + len > capacity)
                status[f] = CFWS_ERROR_OUT_OF_MEMORY;
            map_range(run0, run0 + v0[k], f, t0, map0);
            if (reassemble) {
                vals1[f] = run1;
                map_range(run1, run1 + v1[k], f, t1, map1);
            }
            if (f == n - 1) {
                map0[(t0 + kRegion - 1) / kRegion] = (uint32_t)f;
                if (reassemble) map1[(t1 + kRegion - 1) / kRegion] = (uint32_t)f;
                hdr[0] = t0;
                hdr[1] = t1;
                hdr[2] = t0;
                if (self_scan) {
                    hdr[3] = g0;
                    if (reassemble) hdr[4] = g1;
                }
                if (user_total) *user_total = t0 + t1;
            }
        }
        run0 += v0[k];
        run1 += v1[k];
    }
}

// ---------------------------------------------------------------------------
// host-side launch helpers
// ---------------------------------------------------------------------------
inline uint32_t grid_for(uint64_t items, uint64_t per_block)
{
    const uint64_t g = (items + per_block - 1) / per_block;
    return (uint32_t)(g == 0 ? 1 : g);
}

// A numeric environment knob, or `dflt` when unset. Callers keep the value
// in a function-local static: its initialiser runs once, under the C++
// runtime's guard, whichever thread calls first.
inline int64_t env_knob(const char* name, int64_t dflt)
{
    const char* s = getenv(name);
    return s && *s ? (int64_t)strtoull(s, nullptr, 10) : dflt;
}

// One 4 KiB region per wave (measured fastest: no grid-stride loop, every
// wave's loads in flight at once); CFWS_GRID caps the workgroup count.
inline uint32_t stream_grid(uint64_t regions)
{
    static const uint64_t cap = [] {
        const int64_t v = env_knob("CFWS_GRID", 0);
        return v > 0 ? (uint64_t)v : 0x7fffffffull;
    }();
    uint64_t g = (regions + kWaves - 1) / kWaves;
    if (g > cap) g = cap;
    return (uint32_t)(g == 0 ? 1 : g);
}

template <typename T>
T* ws_ptr(const void* ws, uint64_t off)
{
    return reinterpret_cast<T*>(static_cast<char*>(const_cast<void*>(ws)) + off);
}

inline int run_scan(uint64_t* vals, uint64_t n, uint64_t* partials, uint64_t* grand, hipStream_t st)
{
    const uint32_t nb = grid_for(n, kScanBlock);
    scan_reduce_kernel<<<nb, kThreads, 0, st>>>(vals, n, partials);
    scan_partials_kernel<<<1, kThreads, 0, st>>>(partials, nb, grand);
    scan_apply_kernel<<<nb, kThreads, 0, st>>>(vals, n, partials);
    return launch_check("scan");
}

inline bool misaligned(const void* a, const void* b)
{
    return ((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b)) & 15u) != 0;
}

inline int zero_totals(const WsLayout& L, void* ws, uint64_t* d_total, hipStream_t st)
{
    (void)hipMemsetAsync(ws_ptr<uint64_t>(ws, L.hdr), 0, 64, st);
    if (d_total) (void)hipMemsetAsync(d_total, 0, 8, st);
    return launch_check("zero totals");
}

// Dynamic LDS the streaming kernel reserves per workgroup. It is never
// touched: it only caps residency at 5 workgroups (20 waves) per CU. More
// resident streams contend for HBM pages: at the register-limited 8 per CU
// the kernel ran 8-12 % slower, at 7 6 % slower; 5 measured best with the
// DPP body path (config 2: 6.44/6.46 TB/s vs 6.44/6.40 at 6 and 6.41/6.42 at
// 4; profiles/r01_ab_dpp.json, tools/ab.sh). The WS serialize kernel (96
// VGPRs) is register-limited to 5 per CU already, and there the reservation
// only cost: config 3 serialize 6.20 TB/s without it against 6.02-6.10 with
// (config 2 6.27 vs 6.29; the 78-80-VGPR modes reach 6 per CU without it and
// lose 8 % on config 2 deserialize). With its write-through stores (round 2)
// serialize runs best at 4 per CU (CFWS_SER_LDS = 40000): 6.44-6.48 TB/s on
// config 2, and ahead at every uniform frame size from 16 KiB to 1 MiB
// (6.35-6.46 against 6.00-6.37); config 3 holds its rate since the
// small-frame regions load their frames in one round (general_region).
// CFWS_XFORM_LDS overrides for every mode (0 = none).
constexpr uint32_t kXformLdsDefault = 32000;     // 5 x fits 160 KiB, 6 x does not

#ifndef CFWS_SER_LDS
#define CFWS_SER_LDS 40000                       // 4 x fits 160 KiB, 5 x does not
#endif
#ifndef CFWS_H2SER_LDS
#define CFWS_H2SER_LDS kXformLdsDefault
#endif
// Batches of small frames (on average at most the mode's threshold of output
// bytes per frame: cap / n at launch) run at the residency the registers
// allow: their regions are latency-bound (a frame view, then the source
// blocks, per region; edge chunks every frame), and more resident waves hide
// that. Serialize: 512 B frames 3.47 -> 3.90 TB/s, 1 KiB 4.25 -> 4.84,
// 2 KiB 4.44 -> 5.01, 4 KiB unchanged, 8 KiB and up slower. Deserialize:
// 512 B 4.88 -> 5.36, 1 KiB 5.35 -> 5.82, but 2 KiB 6.46 -> 5.96 and slower
// from there (profiles/r02_ab_occupancy_by_frame.txt). CFWS_OCC_FRAME_MAX
// overrides both thresholds (0: never).
#ifndef CFWS_OCC_FRAME_MAX_SER
#define CFWS_OCC_FRAME_MAX_SER 4096
#endif
#ifndef CFWS_OCC_FRAME_MAX_RECV
#define CFWS_OCC_FRAME_MAX_RECV 1536
#endif
inline uint64_t occ_frame_max(int mode)
{
    static const int64_t v = env_knob("CFWS_OCC_FRAME_MAX", -1);
    if (v >= 0) return (uint64_t)v;
    if (mode == kModeSer) return CFWS_OCC_FRAME_MAX_SER;
    if (mode == kModeDeser) return CFWS_OCC_FRAME_MAX_RECV;
    return 0;
}

inline uint32_t xform_lds_bytes(int mode = -1, uint64_t frame_bytes = ~uint64_t(0))
{
    static const int64_t v = [] {                 // -1: no override
        const int64_t x = env_knob("CFWS_XFORM_LDS", -1);
        return x > 65536 ? 65536 : x;
    }();
    if (v >= 0) return (uint32_t)v;
    if (frame_bytes <= occ_frame_max(mode)) return 0;
    if (mode == kModeSer) return CFWS_SER_LDS;
    if (mode == kModeH2Ser) return CFWS_H2SER_LDS;
    return kXformLdsDefault;
}

// One pass: the streaming kernel with its edge workgroups in front
// (CFWS_EDGE_SPLIT=1: the edge chunks as a launch of their own after it, the
// previous layout, kept for A/B).
inline bool edge_split()
{
    static const bool v = env_knob("CFWS_EDGE_SPLIT", 0) == 1;
    return v;
}

// Where the edge workgroups go: first (their chains run beside the first
// streaming waves), or spread through the grid, one every `stride`
// workgroups, so that they never hold every slot at once. Spread pays when
// frames are small -- one edge workgroup (128 frames) per <= 128 streaming
// workgroups (2 MiB), i.e. frames averaging <= 16 KiB of output: config 3
// +1.1 %, 4 KiB frames +2.3 % -- and costs 64 KiB frames 3 % of serialize
// (configs 2 and 4), where it lands each edge workgroup beside the regions of
// its own frames (profiles/r02_ab_edge_order.txt). CFWS_EDGE_ORDER=0 / 1
// forces first / spread.
#ifndef CFWS_EDGE_SPREAD_MAX_STRIDE
#define CFWS_EDGE_SPREAD_MAX_STRIDE 128
#endif
inline bool edge_interleave(uint32_t stride)
{
    static const int64_t v = env_knob("CFWS_EDGE_ORDER", -1);
    return v < 0 ? stride <= CFWS_EDGE_SPREAD_MAX_STRIDE : v == 1;
}

template <int kMode>
void launch_streaming(const void* src, void* dst, const cfws_frame_desc_t* desc,
                      const int32_t* status, const uint64_t* offs, const uint32_t* map,
                      const uint64_t* total_p, const uint64_t* base_p, uint64_t regions,
                      uint64_t cap, size_t n, uint32_t klass, uint32_t sid, hipStream_t st,
                      const cfws_frame_desc_t* parent = nullptr, bool edges = true,
                      const uint64_t* reasm_offs1 = nullptr, const uint32_t* inreg_flag = nullptr)
{
    const bool split = edges && (edge_split() || !has_edge_blocks(kMode));
    const uint32_t eb = (edges && !split) ? grid_for(edge_threads(n), kThreads) : 0;
    const uint32_t sg = stream_grid(regions);
    // edge workgroups first, or spread evenly through the grid (edge_interleave)
    const uint32_t spread = eb ? (eb + sg) / eb : 0;
    const uint32_t stride = (eb && edge_interleave(spread)) ? spread : 0;
    // The residency choice takes cap / n as the average output per frame: the
    // output size itself is only known on the device. Callers whose capacity
    // is far above their output (an oversized arena; the HTTP/2 receive passes
    // len(h2) + 16 n) may get the large-frame residency for small frames --
    // a speed effect only, the bytes written are the same.
    const CfwsPassTimer timer(st);
    xform_kernel<kMode><<<eb + sg, kThreads, xform_lds_bytes(kMode, n ? cap / n : cap), st>>>(
        static_cast<const uint8_t*>(src), static_cast<uint8_t*>(dst), desc, status, offs, map,
        total_p, base_p, cap, (uint32_t)n, klass, sid, parent, eb, eb ? reasm_offs1 : nullptr,
        stride, split ? nullptr : inreg_flag);
    // (a separate edge launch on a second stream, overlapping the streaming
    // kernel, measured no faster on config 5: the stream slowed by what the
    // overlap saved)
    if (split) edge_kernel<kMode><<<grid_for(edge_threads(n), kEdgeThreads), kEdgeThreads, 0, st>>>(
        static_cast<const uint8_t*>(src), static_cast<uint8_t*>(dst), desc, status, offs,
        total_p, base_p, cap, (uint32_t)n, klass, sid, parent);
}

template <int kMode>
void launch_pass(const WsLayout& L, int p, const void* src, void* dst, const cfws_frame_desc_t* desc,
                 const int32_t* status, const void* ws, uint64_t cap, size_t n, uint32_t klass,
                 hipStream_t st, uint32_t sid = 0, bool edges = true, bool reasm_edges = false,
                 const uint32_t* inreg_flag = nullptr)
{
    const uint64_t* hdr = ws_ptr<const uint64_t>(ws, L.hdr);
    // Pass 1 (reassembly: control frames, <= 125-byte payloads each) is
    // usually tiny or empty, and its size is only known on the device: a
    // capped grid (the kernel strides over the regions) instead of one
    // workgroup per 16 KiB of capacity, which cost ~20 us of empty dispatch.
    const uint64_t regions = p == 1 ? (L.regions < 4096 ? L.regions : 4096) : L.regions;
    launch_streaming<kMode>(src, dst, desc, status, ws_ptr<const uint64_t>(ws, L.offs[p]),
                            ws_ptr<const uint32_t>(ws, L.map[p]), hdr + p,
                            p == 1 ? hdr + 2 : nullptr, regions, cap, n, klass, sid, st, nullptr,
                            edges, reasm_edges ? ws_ptr<const uint64_t>(ws, L.offs[1]) : nullptr,
                            inreg_flag);
}

}  // namespace

#pragma clang diagnostic pop

#endif
