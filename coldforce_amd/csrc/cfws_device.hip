// cfws_device.hip -- MI355X (gfx950) kernels and batch C ABI of the
// WebSocket frame codec (include/cfws.h).
//
// Reference behaviour restated on the device:
//   header encode        co_ws_frame.c:34-68, :70-91
//   payload mask         co_ws_frame.c:93-97    out[i] = in[i] ^ key[i % 4]
//   header decode        co_ws_frame.c:131-213 (MORE_DATA before TOO_BIG)
//   payload copy+unmask  co_ws_frame.c:214-242
//
// Design (DESIGN.md §3 has the full story):
//   * The output arena (wire arena for serialize, payload arena for
//     deserialize) is cut into 4 KiB regions, one per wave; every 16-byte
//     chunk is produced by exactly one lane and written with one 16-byte
//     store, so frame boundaries never need byte stores or read-modify-write.
//   * A plan (prefix sum of frame sizes + a region -> first-frame map) lets a
//     wave find its frames with two scalar loads; a region inside one frame
//     runs with the frame's descriptor, key and alignment phase in SGPRs.
//   * Source and destination are misaligned against each other (a masked
//     64 KiB frame is 65,550 B on the wire); a lane funnel-shifts the two
//     aligned 16-byte source blocks covering its chunk (v_alignbyte_b32) and
//     XORs with the key pre-rotated once per frame.
//   * Pure HBM streaming: 2 bytes of traffic per payload byte, no LDS on the
//     fast path, no MFMA.
//   * A pass writes output bytes [base, base + total) from per-frame output
//     offsets `offs` (monotone). Deserialize with CFWS_DESERIALIZE_REASSEMBLE
//     runs two passes: data frames packed (messages contiguous), then control
//     frames after them.
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "cfws.h"
#include "cfws_internal.h"

namespace {

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
constexpr int kPlanItems = 1;
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
    uint64_t bytes;
    uint64_t regions;
    uint64_t scan_blocks;
};

inline uint64_t align_up(uint64_t x, uint64_t a) { return (x + a - 1) / a * a; }

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
    uint32_t aux;   // kModeH2Ser: the parent WS frame
    uint32_t s0;    // kModeH2Ser: the slice's first byte within the WS frame
    uint64_t ws_len;  // kModeH2Ser: the WS frame's payload size, key and
    uint32_t ws_key;  //   header byte 0 | mask bit << 8 (its header bytes
    uint32_t ws_hb;   //   are generated from these)
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
    v.aux = 0;
    v.ws_len = 0;
    v.ws_key = 0;
    v.ws_hb = 0;
    v.s0 = 0;
    if (kMode == kModeH2Ser) {
        // d: one DATA frame = a slice [payload_off, + payload_size) of the
        // virtual WS wire arena; key field = its WS frame w
        const uint32_t wf = d.key();
        const DescWords w = load_desc(P.parent, wf);
        const uint64_t s0 = d.payload_off - w.wire_off;
        const uint64_t hs = w.header_size();
        const uint64_t h_in = s0 < hs ? (hs - s0 < d.payload_size ? hs - s0 : d.payload_size) : 0;
        const uint64_t q = s0 + h_in - hs;             // payload index of the body start
        v.pre = d.payload_size ? 9u + (uint32_t)h_in : 0u;   // unused slots: empty
        v.body_len = d.payload_size - h_in;
        v.src_off = w.payload_off + q;
        v.key = w.mask() ? rotr8(w.key(), (uint32_t)(q & 3u)) : 0u;
        v.hb = d.fin() ? 0x1u : 0u;                      // DATA flags: END_STREAM
        v.aux = wf;
        v.s0 = (uint32_t)s0;                           // only read when h_in > 0 (s0 < 14)
        v.ws_len = w.payload_size;
        v.ws_key = w.mask() ? w.key() : 0u;
        v.ws_hb = ((w.opcode() | (w.fin() ? 0x80u : 0u)) & 0xffu) | (w.mask() ? 0x100u : 0u);
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
// on config 2; -DCFWS_PLAIN_STORE turns it off). `nt` loads measured -10 %
// and stay off unless -DCFWS_NT_LOAD.
#ifndef CFWS_PLAIN_STORE
#define CFWS_NT_STORE 1
#endif
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint4 ld16(const uint8_t* p)
{
#ifdef CFWS_NT_LOAD
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
#else
    const u32x4 v = *reinterpret_cast<const u32x4*>(p);
#endif
    return make_uint4(v.x, v.y, v.z, v.w);
}

// The streaming kernel's body loads. Every source byte is read by exactly one
// lane, once, yet `nt` measured slower here (config 2: 6.37/6.49 TB/s plain
// vs 5.97/6.29 nt, profiles/r01_ab_dpp.json), although the bare copy probe
// (tools/copy_probe.hip) gains from it; -DCFWS_STREAM_NT turns it on.
__device__ __forceinline__ uint4 ld16_stream(const uint8_t* p)
{
#ifdef CFWS_STREAM_NT
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
#else
    return ld16(p);
#endif
}

// Lane i receives lane i + 1's `v` (DPP wave_shl:1); lane 63, which has no
// right neighbour, keeps `last`.
__device__ __forceinline__ uint32_t from_next_lane(uint32_t v, uint32_t last)
{
    return __builtin_amdgcn_update_dpp(last, v, 0x130, 0xf, 0xf, false);
}

__device__ __forceinline__ uint4 from_next_lane(const uint4& v, const uint4& last)
{
    return make_uint4(from_next_lane(v.x, last.x), from_next_lane(v.y, last.y),
                      from_next_lane(v.z, last.z), from_next_lane(v.w, last.w));
}

__device__ __forceinline__ void st16(uint8_t* p, uint4 o)
{
    const u32x4 v = {o.x, o.y, o.z, o.w};
#ifdef CFWS_NT_STORE
    __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p));
#else
    *reinterpret_cast<u32x4*>(p) = v;
#endif
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
        // the WS frame's header (co_ws_frame.c:34-91)
        FrameView wv;
        wv.body_len = v.ws_len;
        wv.key = v.ws_key;
        wv.hb = v.ws_hb;
        return view_header_byte(wv, r - 9u + v.s0);
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

// Byte at output position pos of frame v (pos inside v's output range),
// given v's body bytes lined up with the chunk (edge_body).
template <int kMode>
__device__ __forceinline__ uint32_t edge_byte(const Pass& P, const FrameView& v, uint64_t pos,
                                              const uint4& W, int j)
{
    const uint64_t r = pos - v.out_off;
    if (r < v.pre) return header_byte_of<kMode>(P, v, (uint32_t)r);
    return (r - v.pre < v.body_len) ? u4_byte(W, j) : 0u;
}

// A chunk that crosses a header, a frame boundary, padding or the end of
// the pass. With at most two frames in it (every boundary of frames larger
// than the chunk) all source blocks are loaded up front and the bytes are
// assembled in registers: one memory round trip instead of sixteen.
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
    uint32_t w0 = 0, w1 = 0, w2 = 0, w3 = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const uint64_t pos = D + j;
        uint32_t b = 0;
        if (pos < lim)
            b = (two && pos >= o1) ? edge_byte<kMode>(P, vb, pos, Wb, j)
                                   : edge_byte<kMode>(P, va, pos, Wa, j);
        const uint32_t sh = 8 * (j & 3);
        if (j < 4) w0 |= b << sh;
        else if (j < 8) w1 |= b << sh;
        else if (j < 12) w2 |= b << sh;
        else w3 |= b << sh;
    }
    return make_uint4(w0, w1, w2, w3);
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
__device__ __forceinline__ void fast_region(const Pass& P, const FrameView& v, uint64_t base,
                                            uint32_t lane)
{
    const uint64_t delta = v.src_off - v.body_start;           // src = out + delta
    const uint32_t ph = (uint32_t)(delta & 15u);
    const uint32_t kr = rotr8(v.key, (uint32_t)((0 - v.body_start) & 3u));
    const uint8_t* s0 = P.src + ((base + delta) & ~uint64_t(15)) + lane * kChunk;
    uint8_t* d0 = P.dst + base + lane * kChunk;
    uint4 a[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) a[u] = ld16_stream(s0 + u * kSlice);
    if (ph == 0) {
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            xor4(a[u], kr);
            st16(d0 + u * kSlice, a[u]);
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
            st16(d0 + u * kSlice, o);
        }
    }
}

// A region crossed by exactly one frame boundary (the boundary case of large
// frames): both views are wave-uniform, each lane picks one by comparing its
// chunk with the boundary. Chunks not entirely inside a body are left to
// edge_kernel. As in fast_region, a lane's block B comes from the next lane
// over DPP when that lane loads it (same frame, chunk inside the body);
// otherwise (lane 63, the last chunk before a body end) the lane loads it.
template <int kMode>
__device__ __forceinline__ void two_frame_region(const Pass& P, const FrameView& va,
                                                 const FrameView& vb, uint64_t base, uint32_t lane)
{
    uint4 a[kUnroll], e[kUnroll];
    bool fast[kUnroll];
    uint32_t own_b = 0;
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
        const uint64_t D = base + u * kSlice + lane * kChunk;
        const bool hi = D >= vb.out_off;
        const uint64_t bs = hi ? vb.body_start : va.body_start;
        const uint64_t be = bs + (hi ? vb.body_len : va.body_len);
        const uint64_t s = (hi ? vb.src_off : va.src_off) + (D - bs);
        const uint8_t* sp = P.src + (s & ~uint64_t(15));
        fast[u] = D >= bs && D + kChunk <= be;
        a[u] = make_uint4(0, 0, 0, 0);
        e[u] = make_uint4(0, 0, 0, 0);
        if (fast[u]) {
            a[u] = ld16_stream(sp);
            // the next lane's chunk D + 16 loads block sp + 16 iff it is in
            // the same frame and inside the body
            const bool next_loads = lane != 63 && (D + kChunk >= vb.out_off) == hi &&
                                    D + 2 * kChunk <= be;
            if ((s & 15u) && !next_loads) {
                e[u] = ld16(sp + 16);
                own_b |= 1u << u;
            }
        }
    }
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
        const uint4 nb = from_next_lane(a[u], e[u]);     // every lane: DPP needs the full wave
        if (!fast[u]) continue;
        const uint64_t D = base + u * kSlice + lane * kChunk;
        const bool hi = D >= vb.out_off;
        const uint64_t k0 = D - (hi ? vb.body_start : va.body_start);
        const uint32_t ph = (uint32_t)(((hi ? vb.src_off : va.src_off) + k0) & 15u);
        uint4 o = ph ? funnel16(a[u], (own_b >> u) & 1u ? e[u] : nb, ph) : a[u];
        xor4(o, rotr8(hi ? vb.key : va.key, (uint32_t)(k0 & 3u)));
        st16(P.dst + D, o);
    }
}

// Any other region (small frames, padding, pass end): every lane finds the
// frame of each of its chunks by binary search over the region's frames and
// writes it when it lies inside that frame's body.
template <int kMode>
__device__ __forceinline__ void general_region(const Pass& P, uint32_t f0, uint32_t f1,
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
            st16(P.dst + D, body_chunk(P.src, v, D));
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

// The edge chunks of frame f in pass P (part 0: before the body; part 1:
// reaching past the body end).
template <int kMode>
__device__ __forceinline__ void edge_frame(const Pass& P, uint64_t f, uint32_t part)
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
    const uint64_t first = (lo + 15) & ~uint64_t(15);
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
    const uint64_t f = t >> 1;
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
    edge_frame<kMode>(P, f, (uint32_t)(t & 1u));
}

// WS serialize / deserialize carry their edge chunks in the streaming
// launch; the HTTP/2 modes keep a separate edge launch (their edge code
// needs more registers than the merged kernel's 5-waves-per-EU budget).
__host__ __device__ constexpr bool has_edge_blocks(int mode)
{
    return mode == kModeSer || mode == kModeDeser;
}

// The streaming kernel: serialize (kSer) = header + (masked) payload into
// the wire arena; deserialize = copy + unmask into the payload arena.
// The first `edge_blocks` workgroups write the edge chunks (edge_frame: two
// threads per frame); the rest stream the regions, writing every 16-byte
// chunk that lies inside one frame's body. The two chunk sets are disjoint.
// Edge workgroups are dispatched first, so their latency-bound chains run
// under the stream instead of as a launch of their own after it (which cost
// 17 us serialize / 4 us deserialize on config 2, plus a kernel boundary).
// The wave-per-EU floor keeps the merged kernel at <= 102 VGPRs, so the
// 5 workgroups per CU the LDS reservation allows stay resident.
template <int kMode>
__global__ void __launch_bounds__(kThreads, 5)
xform_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
             const cfws_frame_desc_t* __restrict__ desc, const int32_t* __restrict__ status,
             const uint64_t* __restrict__ offs, const uint32_t* __restrict__ region_map,
             const uint64_t* __restrict__ total_p, const uint64_t* __restrict__ base_p,
             uint64_t capacity, uint32_t n_frames, uint32_t klass, uint32_t sid,
             const cfws_frame_desc_t* __restrict__ parent, uint32_t edge_blocks)
{
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
    if (has_edge_blocks(kMode) && blockIdx.x < edge_blocks) {
        const uint64_t t = uint64_t(blockIdx.x) * kThreads + threadIdx.x;
        if ((t >> 1) < n_frames) edge_frame<kMode>(P, t >> 1, (uint32_t)(t & 1u));
        return;
    }
    const uint64_t n_regions = (P.total + kRegion - 1) / kRegion;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t stride = uint64_t(gridDim.x - edge_blocks) * kWaves;

    for (uint64_t r = uint64_t(blockIdx.x - edge_blocks) * kWaves + wave; r < n_regions;
         r += stride) {
        const uint64_t base = r * kRegion;
        const uint64_t end = base + kRegion;
        // The plan writes every entry in [0, n_regions]; the clamps only keep
        // a corrupted workspace from turning into an out-of-bounds read.
        uint32_t f0 = region_map[r];
        uint32_t f1 = region_map[r + 1];
        if (f1 >= n_frames) f1 = n_frames - 1;
        if (f0 > f1) f0 = f1;
        // region_map[r + 1] holds the NEXT region's first byte; frames that
        // start at or after this region's end do not touch it.
        if (f1 > f0 && offs[f0 + 1] >= end) f1 = f0;
        if (end > P.total) {                  // the pass end (a capacity cut may fall in a body)
            tail_region<kMode>(P, f0, f1, base, lane);
            continue;
        }
        const FrameView va = frame_view<kMode>(P, f0);
        if (f0 == f1) {
            if (base >= va.body_start && end <= va.body_start + va.body_len)
                fast_region(P, va, base, lane);
            else
                two_frame_region<kMode>(P, va, va, base, lane);   // partial body, one frame
        } else if (f1 == f0 + 1 || offs[f0 + 2] >= end) {
            two_frame_region<kMode>(P, va, frame_view<kMode>(P, f0 + 1), base, lane);
        } else {
            general_region<kMode>(P, f0, f1, base, lane);
        }
    }
}

// Both reassembly passes in one launch: a frame has bytes in exactly one of
// them (data frames in pass 0, control frames in pass 1), so each thread
// serves its frame's pass only.
__global__ void __launch_bounds__(kEdgeThreads)
edge_reasm_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                  const cfws_frame_desc_t* __restrict__ desc, const int32_t* __restrict__ status,
                  const uint64_t* __restrict__ offs0, const uint64_t* __restrict__ offs1,
                  const uint64_t* __restrict__ hdr, uint64_t capacity, uint32_t n_frames)
{
    const uint64_t t = uint64_t(blockIdx.x) * kEdgeThreads + threadIdx.x;
    const uint64_t f = t >> 1;
    if (f >= n_frames) return;
    const uint32_t p = is_control(desc[f].opcode) ? 1u : 0u;
    const uint64_t out_base = p ? hdr[2] : 0;
    Pass P;
    P.src = src;
    P.dst = dst + out_base;
    P.desc = desc;
    P.status = status;
    P.offs = p ? offs1 : offs0;
    P.total = hdr[p];
    // pass 0's last chunk must not write past the data bytes: pass 1 starts
    // there (at an unaligned address) and runs concurrently in this launch
    P.capacity = p ? capacity - out_base : (hdr[0] < capacity ? hdr[0] : capacity);
    P.n_frames = n_frames;
    P.klass = p ? kClassControl : kClassData;
    P.sid = 0;
    P.parent = nullptr;
    edge_frame<kModeDeser>(P, f, (uint32_t)(t & 1u));
}

// ---------------------------------------------------------------------------
// plan kernels
// ---------------------------------------------------------------------------
// WS header at s of data[0, size) (co_ws_frame.c:131-213), with the callers'
// two-byte precheck (co_ws_client.c:202-206): the reference's decisions in
// its order (MORE_DATA before DATA_TOO_BIG). d gets what the reference has
// written into the frame by the time it returns.
__device__ __forceinline__ int32_t parse_ws_header(const uint8_t* __restrict__ wire, uint64_t size,
                                                   uint64_t s, uint64_t max_payload,
                                                   cfws_frame_desc_t& d)
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
    const uint32_t b0 = wire[s], b1 = wire[s + 1];
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
        for (uint32_t i = 0; i < ext; ++i) len = (len << 8) | wire[p + i];
        d.payload_size = len;
        p += ext;
    }
    if (d.mask) {
        if (size - p < 4) return CFWS_PARSE_MORE_DATA;
        d.mask_key = (uint32_t)wire[p] | (uint32_t)wire[p + 1] << 8 |
                     (uint32_t)wire[p + 2] << 16 | (uint32_t)wire[p + 3] << 24;
        p += 4;
    }
    d.header_size = (uint8_t)(p - s);
    if (size - p < d.payload_size) return CFWS_PARSE_MORE_DATA;
    if (d.payload_size > max_payload) return CFWS_ERROR_DATA_TOO_BIG;
    return CFWS_PARSE_COMPLETE;
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

__global__ void __launch_bounds__(kThreads)
scan_partials_kernel(uint64_t* __restrict__ partials, uint64_t nb, uint64_t* __restrict__ grand)
{
    __shared__ uint64_t s_wave[kWaves];
    uint64_t carry = 0;
    for (uint64_t b = 0; b < nb; b += kThreads) {
        const uint64_t i = b + threadIdx.x;
        const uint64_t x = i < nb ? partials[i] : 0;
        uint64_t tot;
        const uint64_t ex = block_exclusive_scan(x, s_wave, &tot);
        if (i < nb) partials[i] = carry + ex;
        carry += tot;
    }
    if (threadIdx.x == 0) *grand = carry;
}

// scan_partials_kernel for up to two passes in one launch (block p: pass p).
__global__ void __launch_bounds__(kThreads)
scan_partials2_kernel(uint64_t* __restrict__ partials0, uint64_t* __restrict__ partials1, uint64_t nb,
                      uint64_t* __restrict__ grand0, uint64_t* __restrict__ grand1)
{
    __shared__ uint64_t s_wave[kWaves];
    uint64_t* partials = blockIdx.x ? partials1 : partials0;
    uint64_t carry = 0;
    for (uint64_t b = 0; b < nb; b += kThreads) {
        const uint64_t i = b + threadIdx.x;
        const uint64_t x = i < nb ? partials[i] : 0;
        uint64_t tot;
        const uint64_t ex = block_exclusive_scan(x, s_wave, &tot);
        if (i < nb) partials[i] = carry + ex;
        carry += tot;
    }
    if (threadIdx.x == 0) *(blockIdx.x ? grand1 : grand0) = carry;
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

// ---- plans: two launches each (three above kSelfScanBlocks blocks) ---------
// 1. per frame: sizes (serialize: header size, co_ws_frame.c:41-91;
//    deserialize: the header decode) + the block's sum;
// (2. scan_partials_kernel: the block sums, one block per pass -- only when
//    there are more than kSelfScanBlocks blocks; otherwise step 3 sums them);
// 3. per block: exclusive offsets of its frames, then everything the
//    offsets decide (descriptor offsets, capacity rule, region maps, totals).

__global__ void __launch_bounds__(kThreads)
serialize_plan_reduce_kernel(cfws_frame_desc_t* __restrict__ desc, uint64_t* __restrict__ vals,
                             uint64_t n, uint64_t* __restrict__ partials)
{
    __shared__ uint64_t s_wave[kWaves];
    const uint64_t b0 = uint64_t(blockIdx.x) * kPlanBlock;
    uint64_t sum = 0;
#pragma unroll
    for (int k = 0; k < kPlanItems; ++k) {
        const uint64_t f = b0 + uint64_t(k) * kThreads + threadIdx.x;
        if (f < n) {
            const uint64_t len = desc[f].payload_size;
            const uint32_t hs = header_size_of(len, desc[f].mask != 0);
            desc[f].header_size = (uint8_t)hs;
            vals[f] = hs + len;
            sum += hs + len;
        }
    }
    uint64_t total;
    block_exclusive_scan(sum, s_wave, &total);
    if (threadIdx.x == 0) partials[blockIdx.x] = total;
}

__global__ void __launch_bounds__(kThreads)
serialize_plan_apply_kernel(cfws_frame_desc_t* __restrict__ desc, uint64_t* __restrict__ vals,
                            uint64_t n, const uint64_t* __restrict__ partials, uint64_t nb,
                            uint32_t self_scan, uint64_t* __restrict__ hdr, uint64_t capacity,
                            uint32_t* __restrict__ map, uint64_t* __restrict__ user_total)
{
    __shared__ uint64_t s_wave[kWaves];
    uint64_t prefix, g;
    if (self_scan) {
        prefix_from_partials(partials, nb, blockIdx.x, s_wave, prefix, g);
    } else {
        prefix = partials[blockIdx.x];
        g = hdr[3];
    }
    const uint64_t total = g < capacity ? g : capacity;
    const uint64_t i0 = uint64_t(blockIdx.x) * kPlanBlock + uint64_t(threadIdx.x) * kPlanItems;
    uint64_t v[kPlanItems];
    uint64_t sum = 0;
#pragma unroll
    for (int k = 0; k < kPlanItems; ++k) {
        v[k] = (i0 + k < n) ? vals[i0 + k] : 0;
        sum += v[k];
    }
    uint64_t tot;
    uint64_t run = block_exclusive_scan(sum, s_wave, &tot) + prefix;
#pragma unroll
    for (int k = 0; k < kPlanItems; ++k) {
        const uint64_t f = i0 + k;
        if (f < n) {
            vals[f] = run;
            desc[f].wire_off = run;
            map_range(run, run + v[k], f, total, map);
            if (f == n - 1) {
                map[(total + kRegion - 1) / kRegion] = (uint32_t)f;
                hdr[0] = total;
                if (self_scan) hdr[3] = g;
                if (user_total) *user_total = g;
            }
        }
        run += v[k];
    }
}

// Header decode at index[f] against its data size (the whole buffer, or the
// frame's own message: co_http2_stream_receive_ws_frame passes the pooled
// DATA, co_ws_http2_extension.c:144-146). Layout sizes: vals0 = data (or
// every frame without reassembly), vals1 = control frames when reassembling.
__global__ void __launch_bounds__(kThreads)
deserialize_plan_reduce_kernel(const uint8_t* __restrict__ wire, uint64_t wire_size_all,
                               const uint64_t* __restrict__ index, const uint64_t* __restrict__ ends,
                               uint64_t n, uint64_t max_payload, uint64_t align, uint32_t reassemble,
                               cfws_frame_desc_t* __restrict__ desc, int32_t* __restrict__ status,
                               uint64_t* __restrict__ vals0, uint64_t* __restrict__ vals1,
                               uint64_t* __restrict__ partials0, uint64_t* __restrict__ partials1)
{
    __shared__ uint64_t s_wave[kWaves];
    const uint64_t b0 = uint64_t(blockIdx.x) * kPlanBlock;
    uint64_t sum0 = 0, sum1 = 0;
#pragma unroll
    for (int k = 0; k < kPlanItems; ++k) {
        const uint64_t f = b0 + uint64_t(k) * kThreads + threadIdx.x;
        if (f >= n) continue;
        const uint64_t wire_size = ends && ends[f] < wire_size_all ? ends[f] : wire_size_all;
        cfws_frame_desc_t d;
        const int32_t st = parse_ws_header(wire, wire_size, index[f], max_payload, d);
        desc[f] = d;
        status[f] = st;
        const uint64_t len = (st == CFWS_PARSE_COMPLETE) ? d.payload_size : 0;
        if (reassemble) {
            const bool ctl = is_control(d.opcode);
            vals0[f] = ctl ? 0 : len;
            vals1[f] = ctl ? len : 0;
            sum0 += ctl ? 0 : len;
            sum1 += ctl ? len : 0;
        } else {
            const uint64_t v = (len + align - 1) & ~(align - 1);
            vals0[f] = v;
            sum0 += v;
        }
    }
    uint64_t total;
    block_exclusive_scan(sum0, s_wave, &total);
    if (threadIdx.x == 0) partials0[blockIdx.x] = total;
    if (reassemble) {
        block_exclusive_scan(sum1, s_wave, &total);
        if (threadIdx.x == 0) partials1[blockIdx.x] = total;
    }
}

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

// Offsets into the descriptors, the capacity rule (a COMPLETE frame with a
// payload that does not fit gets CFWS_ERROR_OUT_OF_MEMORY, like the
// reference's failed malloc, co_ws_frame.c:216-223), region maps.
__global__ void __launch_bounds__(kThreads)
deserialize_finalize_kernel(cfws_frame_desc_t* __restrict__ desc, int32_t* __restrict__ status,
                            const uint64_t* __restrict__ offs0, const uint64_t* __restrict__ offs1,
                            uint64_t* __restrict__ hdr, uint64_t n, uint64_t capacity,
                            uint32_t reassemble, uint32_t* __restrict__ map0,
                            uint32_t* __restrict__ map1, uint64_t* __restrict__ user_total)
{
    const uint64_t f = uint64_t(blockIdx.x) * kThreads + threadIdx.x;
    if (f >= n) return;
    const uint64_t g0 = hdr[3];
    const uint64_t g1 = reassemble ? hdr[4] : 0;
    const uint64_t t0 = g0 < capacity ? g0 : capacity;
    const uint64_t room1 = capacity - t0;
    const uint64_t t1 = g1 < room1 ? g1 : room1;
    const bool ctl = reassemble && is_control(desc[f].opcode);
    const uint64_t off = ctl ? g0 + offs1[f] : offs0[f];
    desc[f].payload_off = off;
    const uint64_t len = desc[f].payload_size;
    if (status[f] == CFWS_PARSE_COMPLETE && len > 0 && off + len > capacity)
        status[f] = CFWS_ERROR_OUT_OF_MEMORY;
    map_regions(offs0, f, n, g0, t0, map0);
    if (reassemble) map_regions(offs1, f, n, g1, t1, map1);
    if (f == n - 1) {
        hdr[0] = t0;
        hdr[1] = t1;
        hdr[2] = t0;
        if (user_total) *user_total = t0 + t1;
    }
}

// ---------------------------------------------------------------------------
// small batches: plan and stream in one launch per direction
// ---------------------------------------------------------------------------
// A batch of up to kSmallFrames frames into at most kSmallBytes of output is
// bound by launch latency, not HBM: plan (two launches) + execute (one) per
// direction. Here every workgroup computes the batch's layout itself into
// LDS (a 1,024-entry scan: a few microseconds, all reads from L2 after the
// first workgroup), workgroup 0 writes the descriptors, statuses and totals
// the plan would, and all workgroups then write their 16-byte output chunks:
// a chunk inside one body takes body_chunk (two aligned loads + funnel), any
// other chunk (headers, frame boundaries, padding) is assembled byte by byte.
// Outputs are the normal path's, byte for byte, including the zeros the last
// chunk writes past the total within the capacity.
constexpr uint32_t kSmallFrames = 1024;
constexpr uint64_t kSmallBytes = 4ull << 20;
constexpr int kSmallItems = kSmallFrames / kThreads;
#ifndef CFWS_SMALL_CPT
#define CFWS_SMALL_CPT 1
#endif
constexpr uint32_t kSmallChunksPerThread = CFWS_SMALL_CPT;   // output chunks per thread

// Frame k * kThreads + tid of a small batch is thread tid's k-th: every
// thread loads (and parses) at most kSmallItems frames, all independent, and
// a batch of up to kThreads frames keeps every thread busy.
__device__ __forceinline__ uint32_t small_frame(int k) { return k * kThreads + threadIdx.x; }

// s_off[f] = exclusive prefix of w over the frames (w[k]: frame
// small_frame(k)), one block scan per slice of kThreads frames; s_off[n] =
// the grand total (returned). Ends with a barrier.
__device__ __forceinline__ uint64_t small_scan(const uint64_t (&w)[kSmallItems], uint32_t n,
                                               uint64_t* s_off, uint64_t* s_wave)
{
    uint64_t carry = 0;
#pragma unroll
    for (int k = 0; k < kSmallItems; ++k) {
        if (uint32_t(k) * kThreads >= n) break;          // uniform: the slice is empty
        uint64_t tot;
        const uint64_t ex = block_exclusive_scan(w[k], s_wave, &tot);
        const uint32_t f = small_frame(k);
        if (f < n) s_off[f] = carry + ex;
        carry += tot;
    }
    if (threadIdx.x == 0) s_off[n] = carry;
    __syncthreads();
    return carry;
}

// Largest f < n with s_off[f] <= D (s_off[0] = 0 <= D).
__device__ __forceinline__ uint32_t small_frame_of(const uint64_t* s_off, uint32_t n, uint64_t D)
{
    uint32_t lo = 0, hi = n - 1;
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (s_off[mid] <= D) lo = mid; else hi = mid - 1;
    }
    return lo;
}

__device__ __forceinline__ void small_store(uint8_t* dst, uint64_t cap, uint64_t D, uint4 o)
{
    if (D + 16 <= cap) {
        st16(dst + D, o);
    } else {
        for (uint32_t j = 0; D + j < cap; ++j) dst[D + j] = (uint8_t)(u4_byte(o, (int)j));
    }
}

// A serialize frame's view from the LDS copy of its descriptor.
__device__ __forceinline__ FrameView small_ser_view(const uint64_t* s_off, const uint64_t* s_src,
                                                    const uint64_t* s_len, const uint32_t* s_key,
                                                    const uint32_t* s_hb, uint32_t f)
{
    FrameView v = {};
    v.out_off = s_off[f];
    v.pre = s_hb[f] >> 16;
    v.body_start = v.out_off + v.pre;
    v.body_len = s_len[f];
    v.src_off = s_src[f];
    v.key = s_key[f];
    v.hb = s_hb[f] & 0xffffu;
    return v;
}

// co_ws_frame_serialize for every frame (co_ws_frame.c:34-97), frames back
// to back from wire offset 0; as cfws_serialize_plan + cfws_serialize_execute.
__global__ void __launch_bounds__(kThreads)
serialize_small_kernel(const uint8_t* __restrict__ src, cfws_frame_desc_t* __restrict__ desc,
                       uint32_t n, uint8_t* __restrict__ dst, uint64_t cap,
                       uint64_t* __restrict__ ws_hdr, uint64_t* __restrict__ user_total)
{
    __shared__ uint64_t s_off[kSmallFrames + 1];
    __shared__ uint64_t s_src[kSmallFrames];        // payload offset
    __shared__ uint64_t s_len[kSmallFrames];        // payload size
    __shared__ uint32_t s_key[kSmallFrames];        // mask key (0: unmasked)
    __shared__ uint32_t s_hb[kSmallFrames];         // header byte 0 | mask bit << 8 | header size << 16
    __shared__ uint64_t s_wave[kWaves];
    uint64_t w[kSmallItems];
#pragma unroll
    for (int k = 0; k < kSmallItems; ++k) {
        const uint32_t f = small_frame(k);
        w[k] = 0;
        if (f < n) {
            const DescWords d = load_desc(desc, f);
            const uint32_t hs = header_size_of(d.payload_size, d.mask() != 0);
            w[k] = hs + d.payload_size;
            s_src[f] = d.payload_off;
            s_len[f] = d.payload_size;
            s_key[f] = d.mask() ? d.key() : 0u;
            s_hb[f] = ((d.opcode() | (d.fin() ? 0x80u : 0u)) & 0xffu) | (d.mask() ? 0x100u : 0u) | hs << 16;
        }
    }
    const uint64_t g = small_scan(w, n, s_off, s_wave);      // (its barrier publishes the views)
    const uint64_t total = g < cap ? g : cap;
    if (blockIdx.x == 0) {
        // the plan's outputs
        for (uint32_t f = threadIdx.x; f < n; f += kThreads) {
            desc[f].header_size = (uint8_t)(s_hb[f] >> 16);
            desc[f].wire_off = s_off[f];
        }
        if (threadIdx.x == 0) {
            ws_hdr[0] = total;
            ws_hdr[3] = g;
            if (user_total) *user_total = g;
        }
    }
    const uint64_t n_chunks = (total + 15) / 16;
    for (uint64_t c = uint64_t(blockIdx.x) * kThreads + threadIdx.x; c < n_chunks;
         c += uint64_t(gridDim.x) * kThreads) {
        const uint64_t D = c * 16;
        uint32_t f = small_frame_of(s_off, n, D);
        FrameView v = small_ser_view(s_off, s_src, s_len, s_key, s_hb, f);
        uint4 o;
        const uint64_t lim = D + 16 < total ? D + 16 : total;
        const uint64_t o1 = f + 1 < n ? s_off[f + 1] : ~uint64_t(0);
        const uint64_t o2 = f + 2 < n ? s_off[f + 2] : ~uint64_t(0);
        if (D >= v.body_start && D + 16 <= v.body_start + v.body_len) {
            o = body_chunk(src, v, D);
        } else if (o2 >= lim) {
            // at most two frames in the chunk: their body bytes lined up in
            // registers (edge_chunk), headers generated
            const FrameView vb = f + 1 < n ? small_ser_view(s_off, s_src, s_len, s_key, s_hb, f + 1) : v;
            Pass P = {};
            P.src = src;
            P.total = total;
            o = edge_chunk<kModeSer>(P, f, D, v, vb, o1, o2);
        } else {
            uint32_t b[16];
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const uint64_t pos = D + j;
                b[j] = 0;
                if (pos >= total) continue;
                while (pos >= s_off[f + 1]) v = small_ser_view(s_off, s_src, s_len, s_key, s_hb, ++f);
                const uint64_t r = pos - v.out_off;
                if (r < v.pre) {
                    b[j] = view_header_byte(v, (uint32_t)r);
                } else {
                    const uint64_t k = r - v.pre;
                    b[j] = (src[v.src_off + k] ^ (v.key >> (8 * (k & 3u)))) & 0xffu;
                }
            }
            o = make_uint4(b[0] | b[1] << 8 | b[2] << 16 | b[3] << 24,
                           b[4] | b[5] << 8 | b[6] << 16 | b[7] << 24,
                           b[8] | b[9] << 8 | b[10] << 16 | b[11] << 24,
                           b[12] | b[13] << 8 | b[14] << 16 | b[15] << 24);
        }
        small_store(dst, cap, D, o);
    }
}

// A deserialize frame's view from LDS: no header in the output, the body
// copied + unmasked, then zeros to the next frame (alignment padding).
__device__ __forceinline__ FrameView small_de_view(const uint64_t* s_off, const uint64_t* s_src,
                                                   const uint64_t* s_len, const uint32_t* s_key,
                                                   uint32_t f)
{
    FrameView v = {};
    v.out_off = s_off[f];
    v.body_start = v.out_off;
    v.body_len = s_len[f];
    v.src_off = s_src[f];
    v.key = s_key[f];
    return v;
}

// co_ws_frame_deserialize at every index (co_ws_frame.c:121-247), payloads
// laid out as cfws_deserialize_plan lays them out without reassembly;
// as cfws_deserialize_plan + cfws_deserialize_execute (flags 0).
__global__ void __launch_bounds__(kThreads)
deserialize_small_kernel(const uint8_t* __restrict__ wire, uint64_t wire_size,
                         const uint64_t* __restrict__ index, uint32_t n, uint64_t max_payload,
                         uint64_t align, cfws_frame_desc_t* __restrict__ desc,
                         int32_t* __restrict__ status, uint8_t* __restrict__ dst, uint64_t cap,
                         uint64_t* __restrict__ ws_hdr, uint64_t* __restrict__ user_total)
{
    __shared__ uint64_t s_off[kSmallFrames + 1];
    __shared__ uint64_t s_src[kSmallFrames];        // body source: wire offset + header size
    __shared__ uint64_t s_len[kSmallFrames];        // body bytes copied (COMPLETE, fits)
    __shared__ uint32_t s_key[kSmallFrames];
    __shared__ uint64_t s_wave[kWaves];
    cfws_frame_desc_t d[kSmallItems];
    int32_t st[kSmallItems];
    uint64_t w[kSmallItems];
#pragma unroll
    for (int k = 0; k < kSmallItems; ++k) {
        const uint32_t f = small_frame(k);
        w[k] = 0;
        st[k] = CFWS_PARSE_COMPLETE;
        if (f < n) {
            st[k] = parse_ws_header(wire, wire_size, index[f], max_payload, d[k]);
            const uint64_t len = st[k] == CFWS_PARSE_COMPLETE ? d[k].payload_size : 0;
            w[k] = (len + align - 1) & ~(align - 1);
        }
    }
    const uint64_t g = small_scan(w, n, s_off, s_wave);
    const uint64_t total = g < cap ? g : cap;
#pragma unroll
    for (int k = 0; k < kSmallItems; ++k) {
        const uint32_t f = small_frame(k);
        if (f >= n) continue;
        d[k].payload_off = s_off[f];
        // the capacity rule: a COMPLETE payload that does not fit is OOM
        // (the reference's failed malloc, co_ws_frame.c:216-223)
        if (st[k] == CFWS_PARSE_COMPLETE && d[k].payload_size > 0 && s_off[f] + d[k].payload_size > cap)
            st[k] = CFWS_ERROR_OUT_OF_MEMORY;
        s_src[f] = d[k].wire_off + d[k].header_size;
        s_len[f] = st[k] == CFWS_PARSE_COMPLETE ? d[k].payload_size : 0;
        s_key[f] = d[k].mask ? d[k].mask_key : 0u;
        if (blockIdx.x == 0) {
            desc[f] = d[k];
            status[f] = st[k];
        }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        ws_hdr[0] = total;
        ws_hdr[1] = 0;
        ws_hdr[2] = total;
        ws_hdr[3] = g;
        if (user_total) *user_total = total;
    }
    __syncthreads();
    const uint64_t n_chunks = (total + 15) / 16;
    for (uint64_t c = uint64_t(blockIdx.x) * kThreads + threadIdx.x; c < n_chunks;
         c += uint64_t(gridDim.x) * kThreads) {
        const uint64_t D = c * 16;
        uint32_t f = small_frame_of(s_off, n, D);
        uint4 o;
        const uint64_t lim = D + 16 < total ? D + 16 : total;
        const uint64_t o1 = f + 1 < n ? s_off[f + 1] : ~uint64_t(0);
        const uint64_t o2 = f + 2 < n ? s_off[f + 2] : ~uint64_t(0);
        if (D + 16 <= s_off[f] + s_len[f]) {          // D >= s_off[f] by the search
            o = body_chunk(wire, small_de_view(s_off, s_src, s_len, s_key, f), D);
        } else if (o2 >= lim) {
            // at most two frames: bodies lined up in registers, padding zero
            const FrameView va = small_de_view(s_off, s_src, s_len, s_key, f);
            const FrameView vb = f + 1 < n ? small_de_view(s_off, s_src, s_len, s_key, f + 1) : va;
            Pass P = {};
            P.src = wire;
            P.total = total;
            o = edge_chunk<kModeDeser>(P, f, D, va, vb, o1, o2);
        } else {
            uint32_t b[16];
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const uint64_t pos = D + j;
                b[j] = 0;
                if (pos >= total) continue;
                while (pos >= s_off[f + 1]) ++f;
                const uint64_t r = pos - s_off[f];
                if (r < s_len[f]) b[j] = (wire[s_src[f] + r] ^ (s_key[f] >> (8 * (r & 3u)))) & 0xffu;
            }
            o = make_uint4(b[0] | b[1] << 8 | b[2] << 16 | b[3] << 24,
                           b[4] | b[5] << 8 | b[6] << 16 | b[7] << 24,
                           b[8] | b[9] << 8 | b[10] << 16 | b[11] << 24,
                           b[12] | b[13] << 8 | b[14] << 16 | b[15] << 24);
        }
        small_store(dst, cap, D, o);
    }
}

// ---- split ops: header and payload passes over caller-laid-out frames -----

// co_ws_frame.c:34-91 for every frame: its 2-14 header bytes at wire_off,
// one thread per frame; bytes at or past cap are not written.
__global__ void __launch_bounds__(kThreads)
encode_headers_kernel(cfws_frame_desc_t* __restrict__ desc, uint64_t n, uint8_t* __restrict__ wire,
                      uint64_t cap)
{
    const uint64_t f = uint64_t(blockIdx.x) * kThreads + threadIdx.x;
    if (f >= n) return;
    const DescWords d = load_desc(desc, (uint32_t)f);
    const uint32_t hs = header_size_of(d.payload_size, d.mask() != 0);
    FrameView v;
    v.body_len = d.payload_size;
    v.key = d.mask() ? d.key() : 0u;
    v.hb = ((d.opcode() | (d.fin() ? 0x80u : 0u)) & 0xffu) | (d.mask() ? 0x100u : 0u);
#pragma unroll
    for (uint32_t r = 0; r < 14; ++r)
        if (r < hs && d.wire_off + r < cap) wire[d.wire_off + r] = (uint8_t)view_header_byte(v, r);
    desc[f].header_size = (uint8_t)hs;
}

// co_ws_frame.c:131-213 (+ the callers' 2-byte precheck) at every frame
// start, one thread per frame: cfws_deserialize_plan's decode without the
// payload layout.
__global__ void __launch_bounds__(kThreads)
parse_headers_kernel(const uint8_t* __restrict__ wire, uint64_t size, const uint64_t* __restrict__ index,
                     uint64_t n, uint64_t max_payload, cfws_frame_desc_t* __restrict__ desc,
                     int32_t* __restrict__ status)
{
    const uint64_t f = uint64_t(blockIdx.x) * kThreads + threadIdx.x;
    if (f >= n) return;
    cfws_frame_desc_t d;
    status[f] = parse_ws_header(wire, size, index[f], max_payload, d);
    desc[f] = d;
}

// The payload loops (mask: co_ws_frame.c:93-97, unmask: :232-242) of every
// frame, each frame from its own source to its own destination. Work unit
// (frame, piece): a workgroup writes the 16-byte destination chunks of one
// frame, 1,024 per pass (4 per lane, loads in flight before the stores),
// striding by `pieces` passes. Chunks inside the frame are one 16-byte store
// (source funnel-shifted into place); the frame's first and last chunk, which
// it may share with its neighbours, are written byte by byte.
constexpr uint32_t kPieceChunks = 4 * kThreads;

template <bool kUnmask>
__global__ void __launch_bounds__(kThreads)
payload_xor_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                   const cfws_frame_desc_t* __restrict__ desc, const int32_t* __restrict__ status,
                   uint64_t n, uint32_t pieces, uint64_t cap)
{
    const uint64_t f = blockIdx.x / pieces;
    const uint32_t p = blockIdx.x % pieces;
    if (f >= n) return;
    if (kUnmask && status && status[f] != CFWS_PARSE_COMPLETE) return;
    const DescWords d = load_desc(desc, (uint32_t)f);
    const uint64_t len = d.payload_size;
    const uint64_t so = kUnmask ? d.wire_off + d.header_size() : d.payload_off;
    const uint64_t dof = kUnmask ? d.payload_off : d.wire_off + header_size_of(len, d.mask() != 0);
    const uint32_t key = d.mask() ? d.key() : 0u;
    if (len == 0 || dof >= cap) return;
    const uint64_t dend = len < cap - dof ? dof + len : cap;
    const uint64_t c0 = dof & ~uint64_t(15);
    const uint64_t nchunks = (dend - c0 + 15) >> 4;
    // source phase against the 16-byte destination chunks: one per frame
    const uint32_t ph = (uint32_t)((so - dof) & 15u);
    const uint32_t lane = threadIdx.x & 63u;
    for (uint64_t base = uint64_t(p) * kPieceChunks; base < nchunks;
         base += uint64_t(pieces) * kPieceChunks) {
        // a lane's block B is the next lane's A (DPP) when that lane's chunk
        // is full too; lane 63 and the last full chunk load their own
        uint4 a[4], e[4];
        bool full[4];
        uint32_t own_b = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint64_t A = c0 + 16 * (base + uint64_t(k) * kThreads + threadIdx.x);
            full[k] = A >= dof && A + 16 <= dend;
            a[k] = make_uint4(0, 0, 0, 0);
            e[k] = make_uint4(0, 0, 0, 0);
            if (full[k]) {
                const uint8_t* sp = src + ((so + (A - dof)) & ~uint64_t(15));
                a[k] = ld16(sp);
                // the block holding the chunk's last source byte: a payload byte
                if (ph && (lane == 63 || A + 32 > dend)) {
                    e[k] = ld16(sp + 16);
                    own_b |= 1u << k;
                }
            }
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint4 nb = from_next_lane(a[k], e[k]);     // every lane: DPP needs the full wave
            const uint64_t c = base + uint64_t(k) * kThreads + threadIdx.x;
            const uint64_t A = c0 + 16 * c;
            if (full[k]) {
                uint4 o = ph ? funnel16(a[k], (own_b >> k) & 1u ? e[k] : nb, ph) : a[k];
                xor4(o, rotr8(key, (uint32_t)((A - dof) & 3u)));
                st16(dst + A, o);
            } else if (c < nchunks) {
                for (uint32_t j = 0; j < 16; ++j) {
                    const uint64_t x = A + j;
                    if (x < dof || x >= dend) continue;
                    const uint64_t kk = x - dof;
                    dst[x] = (uint8_t)(src[so + kk] ^ (key >> (8 * (kk & 3u))));
                }
            }
        }
    }
}

// Device -> host copy by a kernel (cfws_copy_to_host): 16-byte stores into
// device-mapped pinned host memory, any alignment on either side. Running the
// D2H leg this way beside an SDMA H2D measured 43 GB/s each way against 28
// for two SDMA copies (tools/pcie_probe2.hip). Each lane writes whole
// destination-aligned 16-byte chunks (source funnel-shifted into place); the
// first and last chunk, which the destination may share with other data,
// byte by byte. The chunk grid starts on a kCopyOutAlign boundary of the
// destination, so each wave's 64 x 16 B of stores is one aligned 1 KiB span
// of PCIe writes wherever the caller's destination starts.
#ifndef CFWS_COPY_OUT_ALIGN
#define CFWS_COPY_OUT_ALIGN 1024
#endif
constexpr uintptr_t kCopyOutAlign = CFWS_COPY_OUT_ALIGN;

__global__ void __launch_bounds__(kThreads)
copy_out_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, uint64_t n)
{
    const uintptr_t d0 = reinterpret_cast<uintptr_t>(dst);
    const uintptr_t c0 = d0 & ~(kCopyOutAlign - 1);
    const uint64_t nchunks = (d0 + n - c0 + 15) >> 4;
    const uint32_t ph = (uint32_t)((reinterpret_cast<uintptr_t>(src) - d0) & 15u);
    const uint64_t stride = uint64_t(gridDim.x) * kThreads;
    for (uint64_t c = uint64_t(blockIdx.x) * kThreads + threadIdx.x; c < nchunks; c += stride) {
        const uintptr_t A = c0 + 16 * c;
        if (A >= d0 && A + 16 <= d0 + n) {
            const uint8_t* sp = reinterpret_cast<const uint8_t*>(
                (reinterpret_cast<uintptr_t>(src) + (A - d0)) & ~uintptr_t(15));
            uint4 o = ld16(sp);
            if (ph) o = funnel16(o, ld16(sp + 16), ph);    // holds the chunk's last source byte
            *reinterpret_cast<u32x4*>(A) = u32x4{o.x, o.y, o.z, o.w};
        } else {
            for (uint32_t j = 0; j < 16; ++j) {
                const uintptr_t x = A + j;
                if (x >= d0 && x < d0 + n) *reinterpret_cast<uint8_t*>(x) = src[x - d0];
            }
        }
    }
}

__global__ void __launch_bounds__(kThreads)
xor_mask_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, uint64_t n,
                uint32_t key, uint32_t phase)
{
    const uint64_t stride = uint64_t(gridDim.x) * kThreads;
    const uint64_t nv = n / 16;
    const uint32_t kr = rotr8(key, phase);
    const bool aligned = ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15u) == 0;
    const uint64_t tid = uint64_t(blockIdx.x) * kThreads + threadIdx.x;
    if (aligned) {
        for (uint64_t i = tid; i < nv; i += stride) {
            uint4 v = reinterpret_cast<const uint4*>(src)[i];
            xor4(v, kr);
            reinterpret_cast<uint4*>(dst)[i] = v;
        }
        for (uint64_t i = nv * 16 + tid; i < n; i += stride)
            dst[i] = src[i] ^ (uint8_t)(kr >> (8 * (i & 3)));
    } else {
        for (uint64_t i = tid; i < n; i += stride)
            dst[i] = src[i] ^ (uint8_t)(kr >> (8 * (i & 3)));
    }
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t seed, uint64_t i)
{
    uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ void __launch_bounds__(kThreads)
fill_splitmix_kernel(uint8_t* __restrict__ dst, uint64_t n, uint64_t seed, uint64_t word_base)
{
    const uint64_t stride = uint64_t(gridDim.x) * kThreads;
    const uint64_t nv = n / 16;
    for (uint64_t i = uint64_t(blockIdx.x) * kThreads + threadIdx.x; i < nv; i += stride) {
        const uint64_t a = splitmix64(seed, word_base + 2 * i);
        const uint64_t b = splitmix64(seed, word_base + 2 * i + 1);
        reinterpret_cast<uint4*>(dst)[i] =
            make_uint4((uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32));
    }
    const uint64_t t = uint64_t(blockIdx.x) * kThreads + threadIdx.x;
    if (t < (n & 15u)) {
        const uint64_t o = nv * 16 + t;
        dst[o] = (uint8_t)(splitmix64(seed, word_base + o / 8) >> (8 * (o & 7)));
    }
}

// ---------------------------------------------------------------------------
// WebSocket over HTTP/2 (src/ws_http2): DATA-frame wrap and unwrap
// ---------------------------------------------------------------------------

// DATA frames a serialized WS frame becomes: co_http2_stream_send_data splits
// its bytes into frames of at most max_frame_size (co_http2_stream.c:964-1010).
__global__ void __launch_bounds__(kThreads)
h2_count_kernel(const cfws_frame_desc_t* __restrict__ desc, uint64_t n, uint64_t S,
                uint64_t* __restrict__ vals)
{
    const uint64_t f = uint64_t(blockIdx.x) * kThreads + threadIdx.x;
    if (f >= n) return;
    const uint64_t W = desc[f].header_size + desc[f].payload_size;
    vals[f] = W <= S ? 1 : (W + S - 1) / S;
}

// One DATA-frame descriptor per slice: payload_off = slice start in the WS
// wire arena, payload_size = slice length, fin = END_STREAM (last slice;
// co_ws_http2_extension.c:190-194 sends every WS frame with end_stream).
// Output offset of DATA frame d = 9 d + its wire offset.
__global__ void __launch_bounds__(kThreads)
h2_expand_kernel(const cfws_frame_desc_t* __restrict__ desc, const uint64_t* __restrict__ first,
                 uint64_t n, uint64_t S, uint64_t n_max, cfws_frame_desc_t* __restrict__ ddesc,
                 uint64_t* __restrict__ doffs)
{
    const uint64_t f = uint64_t(blockIdx.x) * kThreads + threadIdx.x;
    if (f >= n) return;
    const uint64_t W = desc[f].header_size + desc[f].payload_size;
    const uint64_t w0 = desc[f].wire_off;
    const uint64_t k = W <= S ? 1 : (W + S - 1) / S;
    for (uint64_t j = 0; j < k; ++j) {
        const uint64_t d = first[f] + j;
        if (d >= n_max) break;
        cfws_frame_desc_t e;
        e.payload_off = w0 + j * S;
        e.wire_off = 9 * d + e.payload_off;
        e.payload_size = (j + 1 < k) ? S : W - j * S;
        e.mask_key = (uint32_t)f;                    // the WS frame (kModeH2Ser)
        e.fin = (j + 1 == k) ? 1 : 0;
        e.opcode = 0;
        e.mask = 0;
        e.header_size = 9;
        ddesc[d] = e;
        doffs[d] = e.wire_off;
    }
}

// Unused descriptor slots past the real DATA-frame count become empty frames
// at the end; then the region map of the wrapped arena.
__global__ void __launch_bounds__(kThreads)
h2_finalize_kernel(cfws_frame_desc_t* __restrict__ ddesc, uint64_t* __restrict__ doffs,
                   uint64_t n_max, const uint64_t* __restrict__ n_data_p,
                   const uint64_t* __restrict__ wire_total_p, uint64_t capacity,
                   uint32_t* __restrict__ map, uint64_t* __restrict__ hdr,
                   uint64_t* __restrict__ user_total)
{
    const uint64_t d = uint64_t(blockIdx.x) * kThreads + threadIdx.x;
    if (d >= n_max) return;
    const uint64_t nd = *n_data_p;
    const uint64_t T = *wire_total_p + 9 * nd;
    const uint64_t total = T < capacity ? T : capacity;
    if (d >= nd) {
        cfws_frame_desc_t e = {};
        e.payload_off = 0;
        e.wire_off = T;
        ddesc[d] = e;
        doffs[d] = T;
    }
    const uint64_t lo = d < nd ? doffs[d] : T;
    const uint64_t hi = d + 1 < nd ? doffs[d + 1] : T;
    const uint64_t a = lo < total ? lo : total, b = hi < total ? hi : total;
    if (b > a) {
        const uint64_t r1 = (b + kRegion - 1) / kRegion;
        for (uint64_t r = (a + kRegion - 1) / kRegion; r < r1; ++r) map[r] = (uint32_t)d;
    }
    if (d == n_max - 1) {
        map[(total + kRegion - 1) / kRegion] = (uint32_t)(n_max - 1);
        hdr[0] = total;
        if (user_total) *user_total = T;
    }
}

// ---- HTTP/2 send plan in two launches --------------------------------------
// The WS layout (header sizes, wire offsets: as serialize_plan_*) and the
// DATA frames each WS frame becomes (co_http2_stream.c:964-1010) from two
// sums per block, wire bytes W and DATA-frame count K. The apply kernel scans
// both, writes the WS descriptors' offsets, expands its frames' DATA
// descriptors, maps their regions and fills the unused descriptor slots: the
// work of serialize_plan + h2_count + a scan + h2_expand + h2_finalize (seven
// launches) in two.
__device__ __forceinline__ uint64_t data_frames_of(uint64_t W, uint64_t S)
{
    return W <= S ? 1 : (W + S - 1) / S;
}

__global__ void __launch_bounds__(kThreads)
h2_ser_plan_reduce_kernel(cfws_frame_desc_t* __restrict__ desc, uint64_t n, uint64_t S,
                          uint64_t* __restrict__ partials_w, uint64_t* __restrict__ partials_k)
{
    __shared__ uint64_t s_wave[kWaves];
    const uint64_t f = uint64_t(blockIdx.x) * kThreads + threadIdx.x;
    uint64_t w = 0, k = 0;
    if (f < n) {
        const uint64_t len = desc[f].payload_size;
        const uint32_t hs = header_size_of(len, desc[f].mask != 0);
        desc[f].header_size = (uint8_t)hs;
        w = hs + len;
        k = data_frames_of(w, S);
    }
    uint64_t tw, tk;
    block_exclusive_scan(w, s_wave, &tw);
    block_exclusive_scan(k, s_wave, &tk);
    if (threadIdx.x == 0) {
        partials_w[blockIdx.x] = tw;
        partials_k[blockIdx.x] = tk;
    }
}

// hdr[0] = DATA-stream bytes clamped by the capacity, hdr[3] = DATA frames;
// hdr[4] / hdr[5] = the grand sums when a scan launch made them (more than
// kSelfScanBlocks blocks). DATA frame d of WS frame f: a slice of its wire
// bytes at 9 d + wire offset (h2_expand_kernel's layout).
__global__ void __launch_bounds__(kThreads)
h2_ser_plan_apply_kernel(cfws_frame_desc_t* __restrict__ desc, uint64_t n, uint64_t S,
                         const uint64_t* __restrict__ partials_w, const uint64_t* __restrict__ partials_k,
                         uint64_t nb, uint32_t self_scan, uint64_t* __restrict__ hdr, uint64_t capacity,
                         uint64_t n_max, cfws_frame_desc_t* __restrict__ ddesc,
                         uint64_t* __restrict__ doffs, uint32_t* __restrict__ map,
                         uint64_t* __restrict__ user_total)
{
    __shared__ uint64_t s_wave[kWaves];
    uint64_t pre_w, pre_k, gw, gk;
    if (self_scan) {
        prefix_from_partials(partials_w, nb, blockIdx.x, s_wave, pre_w, gw);
        prefix_from_partials(partials_k, nb, blockIdx.x, s_wave, pre_k, gk);
    } else {
        pre_w = partials_w[blockIdx.x];
        pre_k = partials_k[blockIdx.x];
        gw = hdr[4];
        gk = hdr[5];
    }
    const uint64_t T = gw + 9 * gk;                      // DATA-stream bytes, unclamped
    const uint64_t total = T < capacity ? T : capacity;
    const uint64_t f = uint64_t(blockIdx.x) * kThreads + threadIdx.x;
    uint64_t w = 0, k = 0;
    if (f < n) {
        w = desc[f].header_size + desc[f].payload_size;
        k = data_frames_of(w, S);
    }
    uint64_t tot;
    const uint64_t w0 = block_exclusive_scan(w, s_wave, &tot) + pre_w;
    const uint64_t d0 = block_exclusive_scan(k, s_wave, &tot) + pre_k;
    if (f < n) {
        desc[f].wire_off = w0;
        for (uint64_t j = 0; j < k; ++j) {
            const uint64_t d = d0 + j;
            if (d >= n_max) break;
            cfws_frame_desc_t e;
            e.payload_off = w0 + j * S;
            e.wire_off = 9 * d + e.payload_off;
            e.payload_size = (j + 1 < k) ? S : w - j * S;
            e.mask_key = (uint32_t)f;                    // the WS frame (kModeH2Ser)
            e.fin = (j + 1 == k) ? 1 : 0;
            e.opcode = 0;
            e.mask = 0;
            e.header_size = 9;
            ddesc[d] = e;
            doffs[d] = e.wire_off;
            // DATA frames lie back to back: this one ends where d + 1 starts
            map_range(e.wire_off, e.wire_off + 9 + e.payload_size, d, total, map);
        }
    }
    // descriptor slots past the DATA frames: empty frames at the end
    for (uint64_t d = gk + f; d < n_max; d += uint64_t(gridDim.x) * kThreads) {
        cfws_frame_desc_t e = {};
        e.wire_off = T;
        ddesc[d] = e;
        doffs[d] = T;
    }
    if (f == 0) {
        map[(total + kRegion - 1) / kRegion] = (uint32_t)(n_max - 1);
        hdr[0] = total;
        hdr[3] = gk;
        if (user_total) *user_total = T;
    }
}

// HTTP/2 frame header at index[i] (co_http2_frame.c:211-300): MORE_DATA under
// 9 bytes, PARSE_ERROR when length > max_frame_size, MORE_DATA when the
// payload is incomplete; DATA payload after the optional pad length byte and
// without the padding. Non-DATA frames are CFWS_H2_NOT_DATA (no bytes).
__device__ __forceinline__ int32_t parse_h2_frame(const uint8_t* __restrict__ h2, uint64_t size,
                                                  uint64_t s, uint64_t max_frame, cfws_frame_desc_t& d)
{
    d = {};
    d.wire_off = s;
    int32_t st = CFWS_H2_PARSE_COMPLETE;
    do {
        if (s > size || size - s < 9) { st = CFWS_H2_PARSE_MORE_DATA; break; }
        const uint64_t len = (uint64_t)h2[s] << 16 | (uint64_t)h2[s + 1] << 8 | h2[s + 2];
        if (len > max_frame) { st = CFWS_H2_PARSE_ERROR; break; }
        if (size - s - 9 < len) { st = CFWS_H2_PARSE_MORE_DATA; break; }
        const uint32_t type = h2[s + 3], flags = h2[s + 4];
        d.opcode = (uint8_t)type;
        d.fin = (uint8_t)(flags & 0x1u);
        if (type != 0) { st = CFWS_H2_NOT_DATA; break; }
        uint64_t pad = 0, hs = 9;
        if (flags & 0x8u) {                               // PADDED
            if (len < 1) { st = CFWS_H2_PARSE_ERROR; break; }
            pad = h2[s + 9];
            hs = 10;
            if (pad + 1 > len) { st = CFWS_H2_PARSE_ERROR; break; }
        }
        d.header_size = (uint8_t)hs;
        d.payload_size = len - (hs - 9) - pad;
    } while (0);
    return st;
}

// ---- HTTP/2 receive plan, fast form: two launches --------------------------
// Valid when the pool capacity holds every DATA payload (then no frame is
// OUT_OF_MEMORY and every COMPLETE END_STREAM frame closes a message); the
// host checks the pooled total afterwards and otherwise runs the general
// form (h2_parse + scans + finalize + message kernels). Reduce: the DATA
// headers (co_http2_frame.c:211-300) and per-block sums of pooled bytes and
// END_STREAM frames.
__global__ void __launch_bounds__(kThreads)
h2_de_plan_reduce_kernel(const uint8_t* __restrict__ h2, uint64_t size, const uint64_t* __restrict__ index,
                         uint64_t n, uint64_t max_frame, cfws_frame_desc_t* __restrict__ desc,
                         int32_t* __restrict__ status, uint64_t* __restrict__ partials_p,
                         uint64_t* __restrict__ partials_e)
{
    __shared__ uint64_t s_wave[kWaves];
    const uint64_t i = uint64_t(blockIdx.x) * kThreads + threadIdx.x;
    uint64_t v = 0, e = 0;
    if (i < n) {
        cfws_frame_desc_t d;
        const int32_t st = parse_h2_frame(h2, size, index[i], max_frame, d);
        desc[i] = d;
        status[i] = st;
        if (st == CFWS_H2_PARSE_COMPLETE) {
            v = d.payload_size;
            e = d.fin;
        }
    }
    uint64_t tp, te;
    block_exclusive_scan(v, s_wave, &tp);
    block_exclusive_scan(e, s_wave, &te);
    if (threadIdx.x == 0) {
        partials_p[blockIdx.x] = tp;
        partials_e[blockIdx.x] = te;
    }
}

// Apply: pool offsets (poffs, desc payload_off), message ids (END_STREAM
// frames before, co_http2_stream.c:550-608), and per message its pooled
// span [starts, ends) and first DATA frame. phdr[3] = pooled bytes,
// *n_msg_p = messages (made by scan_partials2_kernel above kSelfScanBlocks).
__global__ void __launch_bounds__(kThreads)
h2_de_plan_apply_kernel(cfws_frame_desc_t* __restrict__ desc, const int32_t* __restrict__ status,
                        uint64_t n, const uint64_t* __restrict__ partials_p,
                        const uint64_t* __restrict__ partials_e, uint64_t nb, uint32_t self_scan,
                        uint64_t* __restrict__ phdr, uint64_t* __restrict__ poffs,
                        uint64_t* __restrict__ msg_id, uint64_t* __restrict__ n_msg_p,
                        uint64_t* __restrict__ starts, uint64_t* __restrict__ ends,
                        uint64_t* __restrict__ first)
{
    __shared__ uint64_t s_wave[kWaves];
    uint64_t pre_p, pre_e, gp, ge;
    if (self_scan) {
        prefix_from_partials(partials_p, nb, blockIdx.x, s_wave, pre_p, gp);
        prefix_from_partials(partials_e, nb, blockIdx.x, s_wave, pre_e, ge);
    } else {
        pre_p = partials_p[blockIdx.x];
        pre_e = partials_e[blockIdx.x];
        gp = phdr[3];
        ge = *n_msg_p;
    }
    const uint64_t i = uint64_t(blockIdx.x) * kThreads + threadIdx.x;
    uint64_t v = 0, e = 0;
    if (i < n && status[i] == CFWS_H2_PARSE_COMPLETE) {
        v = desc[i].payload_size;
        e = desc[i].fin;
    }
    uint64_t tot;
    const uint64_t off = block_exclusive_scan(v, s_wave, &tot) + pre_p;
    const uint64_t m = block_exclusive_scan(e, s_wave, &tot) + pre_e;
    if (i < n) {
        poffs[i] = off;
        desc[i].payload_off = off;
        msg_id[i] = m;
        if (e) {                      // closes message m; m + 1 starts after it
            ends[m] = off + v;
            if (m + 1 < n) {
                starts[m + 1] = off + v;
                first[m + 1] = i + 1;
            }
        }
    }
    if (i == 0) {
        starts[0] = 0;
        first[0] = 0;
        phdr[3] = gp;
        *n_msg_p = ge;
    }
}

// A WS message = the pooled payloads of DATA frames up to and including one
// with END_STREAM (co_http2_stream.c:550-608). es[i] = 1 for those frames.
__global__ void __launch_bounds__(kThreads)
h2_end_flags_kernel(const cfws_frame_desc_t* __restrict__ desc, const int32_t* __restrict__ status,
                    uint64_t n, uint64_t* __restrict__ es)
{
    const uint64_t i = uint64_t(blockIdx.x) * kThreads + threadIdx.x;
    if (i >= n) return;
    es[i] = (status[i] == CFWS_H2_PARSE_COMPLETE && desc[i].fin) ? 1 : 0;
}

// Message m ends after its END_STREAM frame's data; it starts where message
// m - 1 ended (pooled offsets are monotone, failed frames add no bytes).
__global__ void __launch_bounds__(kThreads)
h2_messages_kernel(const cfws_frame_desc_t* __restrict__ desc, const int32_t* __restrict__ status,
                   const uint64_t* __restrict__ msg_id, uint64_t n, uint64_t* __restrict__ ends)
{
    const uint64_t i = uint64_t(blockIdx.x) * kThreads + threadIdx.x;
    if (i >= n) return;
    if (status[i] == CFWS_H2_PARSE_COMPLETE && desc[i].fin)
        ends[msg_id[i]] = desc[i].payload_off + desc[i].payload_size;
}

__global__ void __launch_bounds__(kThreads)
h2_starts_kernel(const uint64_t* __restrict__ ends, const uint64_t* __restrict__ n_msg_p,
                 uint64_t n, uint64_t* __restrict__ starts)
{
    const uint64_t m = uint64_t(blockIdx.x) * kThreads + threadIdx.x;
    if (m >= n || m >= *n_msg_p) return;
    starts[m] = m == 0 ? 0 : ends[m - 1];
}

// ---- fused receive: WS frames read straight out of the DATA frames --------
// With every DATA payload inside the pool capacity the pool is only a
// concatenation: pool byte p lives in the DATA frame d with
// poff[d] <= p < poff[d] + len[d]. The message plan gathers each message's
// 2-14 WS header bytes through that map, and the payload pass copies +
// unmasks each DATA frame's slice of its message's WS payload directly from
// the HTTP/2 arena (one streaming pass instead of pool + deserialize).

// co_ws_frame_deserialize on each pooled message [starts[m], ends[m])
// (co_ws_http2_extension.c:134-164), header bytes gathered from the DATA
// frames; same outputs as deserialize_parse_kernel on the pool.
// first[m]: message m's first DATA frame (h2_de_plan_apply_kernel: the
// frame after the previous END_STREAM). partials: per-block sums of vals for
// deserialize_plan_apply_kernel (plan blocks).
__global__ void __launch_bounds__(kThreads)
h2_msg_parse_kernel(const uint8_t* __restrict__ h2, const cfws_frame_desc_t* __restrict__ pdesc,
                    const int32_t* __restrict__ h2_status, const uint64_t* __restrict__ poff,
                    uint64_t n_h2, const uint64_t* __restrict__ starts,
                    const uint64_t* __restrict__ ends, uint64_t n_msg, uint64_t max_payload,
                    uint64_t align, cfws_frame_desc_t* __restrict__ mdesc,
                    int32_t* __restrict__ mstatus, uint64_t* __restrict__ vals,
                    const uint64_t* __restrict__ first, uint64_t* __restrict__ partials)
{
    __shared__ uint64_t s_wave[kWaves];
    const uint64_t m = uint64_t(blockIdx.x) * kThreads + threadIdx.x;
    uint64_t v = 0;
    if (m < n_msg) {
        const uint64_t s = starts[m], len = ends[m] - s;
        uint8_t hb[16];
        const uint32_t k = len < 14 ? (uint32_t)len : 14u;
        uint64_t d = first[m];
        const uint64_t l0 = h2_status[d] == CFWS_H2_PARSE_COMPLETE ? pdesc[d].payload_size : 0;
        if (s + k <= poff[d] + l0) {
            // the whole header in the first DATA frame (every frame of >= 14
            // bytes): one base, independent byte loads
            const uint8_t* b = h2 + pdesc[d].wire_off + pdesc[d].header_size + (s - poff[d]);
            for (uint32_t i = 0; i < k; ++i) hb[i] = b[i];
        } else {
            for (uint32_t i = 0; i < k; ++i) {
                const uint64_t p = s + i;
                while (p >= poff[d] + (h2_status[d] == CFWS_H2_PARSE_COMPLETE ? pdesc[d].payload_size : 0))
                    ++d;
                hb[i] = h2[pdesc[d].wire_off + pdesc[d].header_size + (p - poff[d])];
            }
        }
        cfws_frame_desc_t dd;
        const int32_t st = parse_ws_header(hb, len, 0, max_payload, dd);
        dd.wire_off = s;
        mdesc[m] = dd;
        mstatus[m] = st;
        const uint64_t pl = st == CFWS_PARSE_COMPLETE ? dd.payload_size : 0;
        v = (pl + align - 1) & ~(align - 1);
        vals[m] = v;
    }
    uint64_t tot;
    block_exclusive_scan(v, s_wave, &tot);
    if (threadIdx.x == 0) partials[blockIdx.x] = tot;
}

// One unit per DATA frame: the part of its pooled bytes that is WS payload
// of its message's frame, as a deserialize-mode frame of the payload pass
// (source = that slice in the HTTP/2 arena, key rotated to the slice's
// payload index, output = message payload offset + index). Frames outside
// any message, or of a message whose frame did not parse COMPLETE, are
// empty units at the matching layout position (offsets stay monotone and
// the pass zero-fills what the layout does not cover).
__device__ __forceinline__ uint64_t h2_unit(const cfws_frame_desc_t* __restrict__ pdesc,
                                            const int32_t* __restrict__ h2_status,
                                            const uint64_t* __restrict__ poff,
                                            const uint64_t* __restrict__ msg_id, uint64_t d,
                                            uint64_t n_msg, const uint64_t* __restrict__ starts,
                                            const cfws_frame_desc_t* __restrict__ mdesc,
                                            const int32_t* __restrict__ mstatus,
                                            const uint64_t* __restrict__ hdr, cfws_frame_desc_t& u)
{
    const uint64_t m = msg_id[d];
    u = {};
    uint64_t out = hdr[3];                             // past the last message
    if (m < n_msg) {
        const cfws_frame_desc_t M = mdesc[m];
        const int32_t ms = mstatus[m];
        const uint64_t hs = M.header_size;
        // the message's layout span: payload_size when it parsed (an OOM
        // frame keeps its layout), else nothing
        const uint64_t span = (ms == CFWS_PARSE_COMPLETE || ms == CFWS_ERROR_OUT_OF_MEMORY)
                                  ? M.payload_size : 0;
        const uint64_t a = poff[d] - starts[m];
        const uint64_t dl = h2_status[d] == CFWS_H2_PARSE_COMPLETE ? pdesc[d].payload_size : 0;
        const uint64_t b = a + dl;
        const uint64_t qa = a > hs ? (a - hs < span ? a - hs : span) : 0;
        const uint64_t qb = b > hs ? (b - hs < span ? b - hs : span) : 0;
        out = M.payload_off + qa;
        if (ms == CFWS_PARSE_COMPLETE && qb > qa) {
            u.wire_off = pdesc[d].wire_off + pdesc[d].header_size + (hs + qa - a);
            u.payload_size = qb - qa;
            u.mask = M.mask;
            u.mask_key = M.mask ? __builtin_amdgcn_alignbyte(M.mask_key, M.mask_key,
                                                             (uint32_t)(qa & 3u)) : 0u;
        }
    }
    return out;
}

// One thread per DATA frame: its unit, and the region map of the payload
// pass (a unit ends where unit d + 1 starts, computed here too, so no
// second launch reads uoffs).
__global__ void __launch_bounds__(kThreads)
h2_units_kernel(const cfws_frame_desc_t* __restrict__ pdesc, const int32_t* __restrict__ h2_status,
                const uint64_t* __restrict__ poff, const uint64_t* __restrict__ msg_id, uint64_t n,
                uint64_t n_msg, const uint64_t* __restrict__ starts,
                const cfws_frame_desc_t* __restrict__ mdesc, const int32_t* __restrict__ mstatus,
                const uint64_t* __restrict__ hdr, cfws_frame_desc_t* __restrict__ udesc,
                int32_t* __restrict__ ustatus, uint64_t* __restrict__ uoffs, uint32_t* __restrict__ map)
{
    const uint64_t d = uint64_t(blockIdx.x) * kThreads + threadIdx.x;
    if (d >= n) return;
    cfws_frame_desc_t u, u1;
    const uint64_t lo = h2_unit(pdesc, h2_status, poff, msg_id, d, n_msg, starts, mdesc, mstatus, hdr, u);
    const uint64_t hi = d + 1 < n ? h2_unit(pdesc, h2_status, poff, msg_id, d + 1, n_msg, starts, mdesc,
                                            mstatus, hdr, u1)
                                  : hdr[3];
    udesc[d] = u;
    ustatus[d] = CFWS_PARSE_COMPLETE;
    uoffs[d] = lo;
    const uint64_t total = hdr[0];
    map_range(lo, hi, d, total, map);
    if (d == n - 1) map[(total + kRegion - 1) / kRegion] = (uint32_t)(n - 1);
}


// ---------------------------------------------------------------------------
// handshake accept keys (co_ws_create_base64_accept_key,
// co_ws_http_extension.c:26-57): base64(SHA-1(key || GUID))
// ---------------------------------------------------------------------------
__constant__ char kWsGuid[37] = "258EAFA5-E914-47DA-95CA-C5AB0DC85B11";
__constant__ char kB64[65] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";

// Byte i of the SHA-1 input key || GUID || 0x80 || 0... || bit length (BE64)
// over `blocks` 64-byte blocks.
__device__ __forceinline__ uint32_t accept_msg_byte(const uint8_t* __restrict__ key, uint64_t L,
                                                    uint64_t blocks, uint64_t i)
{
    const uint64_t m = L + 36;
    if (i < L) return key[i];
    if (i < m) return (uint8_t)kWsGuid[i - L];
    if (i == m) return 0x80u;
    const uint64_t end = blocks * 64;
    if (i >= end - 8) return (uint32_t)((m * 8) >> (8 * (end - 1 - i))) & 0xffu;
    return 0;
}

__device__ __forceinline__ uint32_t rol32(uint32_t v, int b) { return (v << b) | (v >> (32 - b)); }

// One thread per connection: a connection storm's accept keys at once.
__global__ void __launch_bounds__(kThreads)
ws_accept_kernel(const uint8_t* __restrict__ keys, const uint64_t* __restrict__ key_off, uint64_t n,
                 char* __restrict__ out)
{
    const uint64_t c = uint64_t(blockIdx.x) * kThreads + threadIdx.x;
    if (c >= n) return;
    const uint8_t* key = keys + key_off[c];
    const uint64_t L = key_off[c + 1] - key_off[c];
    const uint64_t blocks = (L + 36 + 9 + 63) / 64;
    uint32_t st[5] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u, 0xc3d2e1f0u};
    for (uint64_t b = 0; b < blocks; ++b) {
        uint32_t w[16];
#pragma unroll
        for (int t = 0; t < 16; ++t) {
            const uint64_t i = b * 64 + 4 * t;
            w[t] = accept_msg_byte(key, L, blocks, i) << 24 | accept_msg_byte(key, L, blocks, i + 1) << 16 |
                   accept_msg_byte(key, L, blocks, i + 2) << 8 | accept_msg_byte(key, L, blocks, i + 3);
        }
        uint32_t a = st[0], bb = st[1], cc = st[2], d = st[3], e = st[4];
#pragma unroll
        for (int r = 0; r < 80; ++r) {
            if (r >= 16)
                w[r & 15] = rol32(w[(r + 13) & 15] ^ w[(r + 8) & 15] ^ w[(r + 2) & 15] ^ w[r & 15], 1);
            const uint32_t f = r < 20 ? ((bb & cc) | (~bb & d))
                             : r < 40 ? (bb ^ cc ^ d)
                             : r < 60 ? ((bb & cc) | (bb & d) | (cc & d)) : (bb ^ cc ^ d);
            const uint32_t k = r < 20 ? 0x5a827999u : r < 40 ? 0x6ed9eba1u : r < 60 ? 0x8f1bbcdcu : 0xca62c1d6u;
            const uint32_t t = rol32(a, 5) + f + e + k + w[r & 15];
            e = d; d = cc; cc = rol32(bb, 30); bb = a; a = t;
        }
        st[0] += a; st[1] += bb; st[2] += cc; st[3] += d; st[4] += e;
    }
    // base64 of the 20 hash bytes: 6 full groups + 2 bytes -> 3 chars + '='
    char* o = out + CFWS_WS_ACCEPT_SLOT * c;
#pragma unroll
    for (int g = 0; g < 7; ++g) {
        uint32_t v = 0;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const int idx = 3 * g + j;
            const uint32_t byte = idx < 20 ? (st[idx >> 2] >> (8 * (3 - (idx & 3)))) & 0xffu : 0u;
            v = v << 8 | byte;
        }
        o[4 * g] = kB64[(v >> 18) & 63];
        o[4 * g + 1] = kB64[(v >> 12) & 63];
        o[4 * g + 2] = kB64[(v >> 6) & 63];
        o[4 * g + 3] = g < 6 ? kB64[v & 63] : '=';
    }
    o[28] = 0;
}

// ---------------------------------------------------------------------------
// receive-buffer frame indexing (co_ws_server.c:107-169)
// ---------------------------------------------------------------------------

// One connection per thread: the receive loop's walk over buf[begin, end).
// The walk is a chain of dependent header reads, so a connection is one
// thread and the parallelism is across connections (a server's event loop
// tick holds the receive buffers of many). Pass 1 (kWrite = false) counts
// and records consumed / stop; pass 2 walks again and writes the starts at
// the scanned offsets.
template <bool kWrite>
__global__ void __launch_bounds__(kThreads)
index_walk_kernel(const uint8_t* __restrict__ buf, const uint64_t* __restrict__ begin,
                  const uint64_t* __restrict__ end, uint64_t n, uint64_t max_payload,
                  uint64_t* __restrict__ first, uint64_t* __restrict__ consumed,
                  int32_t* __restrict__ stop, uint64_t* __restrict__ starts, uint64_t cap)
{
    const uint64_t c = uint64_t(blockIdx.x) * kThreads + threadIdx.x;
    if (c >= n) return;
    const uint64_t e = end[c];
    uint64_t p = begin[c];
    uint64_t k = kWrite ? first[c] : 0;
    int32_t st = CFWS_PARSE_COMPLETE;
    while (e > p) {
        if (e - p < 2) { st = CFWS_PARSE_MORE_DATA; break; }
        cfws_frame_desc_t d;
        st = parse_ws_header(buf, e, p, max_payload, d);
        if (st != CFWS_PARSE_COMPLETE) break;
        if (kWrite && k < cap) starts[k] = p;
        ++k;
        p += d.header_size + d.payload_size;
    }
    if (!kWrite) {
        first[c] = k;
        consumed[c] = p;
        stop[c] = st;
    }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
thread_local char g_err[512] = "";
int g_init_state = 0;   // 0 unknown, 1 ok, <0 error code

int set_err(int code, const char* what, hipError_t e)
{
    snprintf(g_err, sizeof g_err, "%s%s%s", what, e == hipSuccess ? "" : ": ",
             e == hipSuccess ? "" : hipGetErrorString(e));
    fprintf(stderr, "cfws: %s\n", g_err);
    return code;
}

int check_init()
{
    if (g_init_state == 1) return CFWS_OK;
    if (g_init_state < 0) return g_init_state;
    int count = 0;
    hipError_t e = hipGetDeviceCount(&count);
    if (e != hipSuccess || count == 0) {
        g_init_state = CFWS_ERROR_NO_DEVICE;
        return set_err(CFWS_ERROR_NO_DEVICE, "no HIP device", e);
    }
    int dev = 0;
    (void)hipGetDevice(&dev);
    hipDeviceProp_t prop;
    e = hipGetDeviceProperties(&prop, dev);
    if (e != hipSuccess) return set_err(CFWS_ERROR_NO_DEVICE, "hipGetDeviceProperties", e);
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        g_init_state = CFWS_ERROR_NO_DEVICE;
        snprintf(g_err, sizeof g_err, "device arch %s is not gfx950", prop.gcnArchName);
        fprintf(stderr, "cfws: %s\n", g_err);
        return CFWS_ERROR_NO_DEVICE;
    }
    g_init_state = 1;
    return CFWS_OK;
}

int launch_check(const char* what)
{
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? CFWS_OK : set_err(CFWS_ERROR_HIP, what, e);
}

uint32_t grid_for(uint64_t items, uint64_t per_block)
{
    const uint64_t g = (items + per_block - 1) / per_block;
    return (uint32_t)(g == 0 ? 1 : g);
}

// The single-launch small-batch path (CFWS_SMALL=0 turns it off: plan +
// execute for every batch, for A/B and for tests of both paths).
bool small_path()
{
    static int v = -1;
    if (v < 0) {
        const char* s = getenv("CFWS_SMALL");
        v = (s && *s == '0') ? 0 : 1;
    }
    return v == 1;
}

// Workgroups of a small-batch launch: kSmallChunksPerThread output chunks
// per thread at the capacity's size.
uint32_t small_grid(uint64_t cap)
{
    const uint64_t per = uint64_t(kThreads) * kSmallChunksPerThread * 16;
    return grid_for(cap, per);
}

// One 4 KiB region per wave (measured fastest: no grid-stride loop, every
// wave's loads in flight at once); CFWS_GRID caps the workgroup count.
uint32_t stream_grid(uint64_t regions)
{
    static uint64_t cap = 0;
    if (cap == 0) {
        const char* s = getenv("CFWS_GRID");
        cap = s ? strtoull(s, nullptr, 10) : 0;
        if (cap == 0) cap = 0x7fffffffull;
    }
    uint64_t g = (regions + kWaves - 1) / kWaves;
    if (g > cap) g = cap;
    return (uint32_t)(g == 0 ? 1 : g);
}

template <typename T>
T* ws_ptr(const void* ws, uint64_t off)
{
    return reinterpret_cast<T*>(static_cast<char*>(const_cast<void*>(ws)) + off);
}

int run_scan(uint64_t* vals, uint64_t n, uint64_t* partials, uint64_t* grand, hipStream_t st)
{
    const uint32_t nb = grid_for(n, kScanBlock);
    scan_reduce_kernel<<<nb, kThreads, 0, st>>>(vals, n, partials);
    scan_partials_kernel<<<1, kThreads, 0, st>>>(partials, nb, grand);
    scan_apply_kernel<<<nb, kThreads, 0, st>>>(vals, n, partials);
    return launch_check("scan");
}

bool misaligned(const void* a, const void* b)
{
    return ((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b)) & 15u) != 0;
}

int zero_totals(const WsLayout& L, void* ws, uint64_t* d_total, hipStream_t st)
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
// 4; profiles/r01_ab_dpp.json, tools/ab.sh). CFWS_XFORM_LDS overrides (0 = none).
constexpr uint32_t kXformLdsDefault = 32000;     // 5 x fits 160 KiB, 6 x does not

uint32_t xform_lds_bytes()
{
    static int64_t v = -1;
    if (v < 0) {
        const char* s = getenv("CFWS_XFORM_LDS");
        v = s ? (int64_t)strtoull(s, nullptr, 10) : kXformLdsDefault;
        if (v > 65536) v = 65536;
    }
    return (uint32_t)v;
}

// One pass: the streaming kernel with its edge workgroups in front
// (CFWS_EDGE_SPLIT=1: the edge chunks as a launch of their own after it, the
// previous layout, kept for A/B).
bool edge_split()
{
    static int v = -1;
    if (v < 0) {
        const char* s = getenv("CFWS_EDGE_SPLIT");
        v = (s && *s == '1') ? 1 : 0;
    }
    return v == 1;
}

template <int kMode>
void launch_streaming(const void* src, void* dst, const cfws_frame_desc_t* desc,
                      const int32_t* status, const uint64_t* offs, const uint32_t* map,
                      const uint64_t* total_p, const uint64_t* base_p, uint64_t regions,
                      uint64_t cap, size_t n, uint32_t klass, uint32_t sid, hipStream_t st,
                      const cfws_frame_desc_t* parent = nullptr, bool edges = true)
{
    const bool split = edges && (edge_split() || !has_edge_blocks(kMode));
    const uint32_t eb = (edges && !split) ? grid_for(2 * (uint64_t)n, kThreads) : 0;
    xform_kernel<kMode><<<eb + stream_grid(regions), kThreads, xform_lds_bytes(), st>>>(
        static_cast<const uint8_t*>(src), static_cast<uint8_t*>(dst), desc, status, offs, map,
        total_p, base_p, cap, (uint32_t)n, klass, sid, parent, eb);
    // (a separate edge launch on a second stream, overlapping the streaming
    // kernel, measured no faster on config 5: the stream slowed by what the
    // overlap saved)
    if (split) edge_kernel<kMode><<<grid_for(2 * (uint64_t)n, kEdgeThreads), kEdgeThreads, 0, st>>>(
        static_cast<const uint8_t*>(src), static_cast<uint8_t*>(dst), desc, status, offs,
        total_p, base_p, cap, (uint32_t)n, klass, sid, parent);
}

template <int kMode>
void launch_pass(const WsLayout& L, int p, const void* src, void* dst, const cfws_frame_desc_t* desc,
                 const int32_t* status, const void* ws, uint64_t cap, size_t n, uint32_t klass,
                 hipStream_t st, uint32_t sid = 0, bool edges = true)
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
                            edges);
}

}  // namespace

int cfws_internal_copy_out(const void* d_src, void* dev_dst, uint64_t n, void* stream)
{
    if (n == 0) return CFWS_OK;
    const uint64_t chunks = (n + kCopyOutAlign) / 16 + 1;
    const uint64_t blocks = (chunks + kThreads - 1) / kThreads;
    copy_out_kernel<<<(uint32_t)(blocks < 1024 ? blocks : 1024), kThreads, 0,
                      static_cast<hipStream_t>(stream)>>>(static_cast<const uint8_t*>(d_src),
                                                          static_cast<uint8_t*>(dev_dst), n);
    return launch_check("copy_to_host");
}

uint64_t cfws_internal_grand_total_offset() { return ws_layout(0, 0).hdr + 3 * sizeof(uint64_t); }

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
extern "C" {

int cfws_init(void) { return check_init(); }
const char* cfws_last_error(void) { return g_err; }
const char* cfws_version(void) { return "cfws 0.2 gfx950"; }

size_t cfws_workspace_size(size_t n_frames, uint64_t out_capacity)
{
    return (size_t)ws_layout(n_frames, out_capacity).bytes;
}

int cfws_serialize_plan(cfws_frame_desc_t* d_desc, size_t n, uint64_t cap, uint64_t* d_total,
                        void* ws, size_t ws_size, void* stream)
{
    if (int rc = check_init()) return rc;
    const WsLayout L = ws_layout(n, cap);
    if (!ws || ws_size < L.bytes) return set_err(CFWS_ERROR_WORKSPACE, "workspace too small", hipSuccess);
    if (n > 0xffffffffull) return set_err(CFWS_ERROR_INVALID_ARGUMENT, "too many frames", hipSuccess);
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (n == 0) return zero_totals(L, ws, d_total, st);
    if (!d_desc) return set_err(CFWS_ERROR_INVALID_ARGUMENT, "null descriptor table", hipSuccess);
    uint64_t* hdr = ws_ptr<uint64_t>(ws, L.hdr);
    uint64_t* offs = ws_ptr<uint64_t>(ws, L.offs[0]);
    uint64_t* partials = ws_ptr<uint64_t>(ws, L.partials[0]);
    const uint32_t nb = grid_for(n, kPlanBlock);
    const uint32_t self_scan = nb <= kSelfScanBlocks ? 1u : 0u;
    serialize_plan_reduce_kernel<<<nb, kThreads, 0, st>>>(d_desc, offs, n, partials);
    if (!self_scan) scan_partials_kernel<<<1, kThreads, 0, st>>>(partials, nb, hdr + 3);
    serialize_plan_apply_kernel<<<nb, kThreads, 0, st>>>(d_desc, offs, n, partials, nb, self_scan,
                                                        hdr, cap, ws_ptr<uint32_t>(ws, L.map[0]),
                                                        d_total);
    return launch_check("serialize_plan");
}

int cfws_serialize_execute(const void* d_payload, const cfws_frame_desc_t* d_desc, size_t n,
                           void* d_wire, uint64_t cap, const void* ws, void* stream)
{
    if (int rc = check_init()) return rc;
    if (n == 0 || cap == 0) return CFWS_OK;
    if (!d_payload || !d_desc || !d_wire || !ws)
        return set_err(CFWS_ERROR_INVALID_ARGUMENT, "null pointer", hipSuccess);
    if (misaligned(d_payload, d_wire))
        return set_err(CFWS_ERROR_INVALID_ARGUMENT, "arenas must be 16-byte aligned", hipSuccess);
    const WsLayout L = ws_layout(n, cap);
    launch_pass<kModeSer>(L, 0, d_payload, d_wire, d_desc, nullptr, ws, cap, n, kClassAll,
                      static_cast<hipStream_t>(stream));
    return launch_check("serialize_execute");
}

int cfws_serialize_batch(const void* d_payload, cfws_frame_desc_t* d_desc, size_t n, void* d_wire,
                         uint64_t cap, uint64_t* d_total, void* ws, size_t ws_size, void* stream)
{
    // small batch, every argument valid: one launch (serialize_small_kernel)
    if (small_path() && n > 0 && n <= kSmallFrames && cap <= kSmallBytes && check_init() == CFWS_OK &&
        d_desc && ws && ws_size >= ws_layout(n, cap).bytes &&
        (cap == 0 || (d_payload && d_wire && !misaligned(d_payload, d_wire)))) {
        serialize_small_kernel<<<small_grid(cap), kThreads, 0, static_cast<hipStream_t>(stream)>>>(
            static_cast<const uint8_t*>(d_payload), d_desc, (uint32_t)n, static_cast<uint8_t*>(d_wire),
            cap, ws_ptr<uint64_t>(ws, ws_layout(n, cap).hdr), d_total);
        return launch_check("serialize_batch(small)");
    }
    if (int rc = cfws_serialize_plan(d_desc, n, cap, d_total, ws, ws_size, stream)) return rc;
    return cfws_serialize_execute(d_payload, d_desc, n, d_wire, cap, ws, stream);
}

static int deserialize_plan_impl(const void* d_wire, uint64_t wire_size, const uint64_t* d_index,
                                 const uint64_t* d_ends, size_t n, uint64_t max_payload, uint32_t align, uint32_t flags,
                          cfws_frame_desc_t* d_desc, int32_t* d_status, uint64_t cap,
                          uint64_t* d_total, void* ws, size_t ws_size, void* stream)
{
    if (int rc = check_init()) return rc;
    if (align == 0 || (align & (align - 1)) || align > 4096)
        return set_err(CFWS_ERROR_INVALID_ARGUMENT, "align must be a power of two <= 4096", hipSuccess);
    if (flags & ~CFWS_DESERIALIZE_REASSEMBLE)
        return set_err(CFWS_ERROR_INVALID_ARGUMENT, "unknown flags", hipSuccess);
    const WsLayout L = ws_layout(n, cap);
    if (!ws || ws_size < L.bytes) return set_err(CFWS_ERROR_WORKSPACE, "workspace too small", hipSuccess);
    if (n > 0xffffffffull) return set_err(CFWS_ERROR_INVALID_ARGUMENT, "too many frames", hipSuccess);
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (n == 0) return zero_totals(L, ws, d_total, st);
    if (!d_wire || !d_index || !d_desc || !d_status)
        return set_err(CFWS_ERROR_INVALID_ARGUMENT, "null pointer", hipSuccess);
    const uint32_t reasm = (flags & CFWS_DESERIALIZE_REASSEMBLE) ? 1u : 0u;
    uint64_t* hdr = ws_ptr<uint64_t>(ws, L.hdr);
    uint64_t* offs0 = ws_ptr<uint64_t>(ws, L.offs[0]);
    uint64_t* offs1 = ws_ptr<uint64_t>(ws, L.offs[1]);
    uint64_t* part0 = ws_ptr<uint64_t>(ws, L.partials[0]);
    uint64_t* part1 = ws_ptr<uint64_t>(ws, L.partials[1]);
    const uint32_t nb = grid_for(n, kPlanBlock);
    deserialize_plan_reduce_kernel<<<nb, kThreads, 0, st>>>(
        static_cast<const uint8_t*>(d_wire), wire_size, d_index, d_ends, n, max_payload, align, reasm,
        d_desc, d_status, offs0, offs1, part0, part1);
    const uint32_t self_scan = nb <= kSelfScanBlocks ? 1u : 0u;
    if (!self_scan)
        scan_partials2_kernel<<<reasm ? 2 : 1, kThreads, 0, st>>>(part0, part1, nb, hdr + 3, hdr + 4);
    deserialize_plan_apply_kernel<<<nb, kThreads, 0, st>>>(
        d_desc, d_status, offs0, offs1, n, part0, part1, nb, self_scan, hdr, cap, reasm,
        ws_ptr<uint32_t>(ws, L.map[0]), ws_ptr<uint32_t>(ws, L.map[1]), d_total);
    return launch_check("deserialize_plan");
}

int cfws_deserialize_plan(const void* d_wire, uint64_t wire_size, const uint64_t* d_index,
                          size_t n, uint64_t max_payload, uint32_t align, uint32_t flags,
                          cfws_frame_desc_t* d_desc, int32_t* d_status, uint64_t cap,
                          uint64_t* d_total, void* ws, size_t ws_size, void* stream)
{
    return deserialize_plan_impl(d_wire, wire_size, d_index, nullptr, n, max_payload, align, flags,
                                 d_desc, d_status, cap, d_total, ws, ws_size, stream);
}

int cfws_deserialize_execute(const void* d_wire, const cfws_frame_desc_t* d_desc,
                             const int32_t* d_status, size_t n, uint32_t flags, void* d_payload,
                             uint64_t cap, const void* ws, void* stream)
{
    if (int rc = check_init()) return rc;
    if (n == 0 || cap == 0) return CFWS_OK;
    if (!d_wire || !d_desc || !d_status || !d_payload || !ws)
        return set_err(CFWS_ERROR_INVALID_ARGUMENT, "null pointer", hipSuccess);
    if (misaligned(d_payload, d_wire))
        return set_err(CFWS_ERROR_INVALID_ARGUMENT, "arenas must be 16-byte aligned", hipSuccess);
    const WsLayout L = ws_layout(n, cap);
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (flags & CFWS_DESERIALIZE_REASSEMBLE) {
        launch_pass<kModeDeser>(L, 0, d_wire, d_payload, d_desc, d_status, ws, cap, n, kClassData, st,
                                0, false);
        launch_pass<kModeDeser>(L, 1, d_wire, d_payload, d_desc, d_status, ws, cap, n, kClassControl,
                                st, 0, false);
        edge_reasm_kernel<<<grid_for(2 * (uint64_t)n, kEdgeThreads), kEdgeThreads, 0, st>>>(
            static_cast<const uint8_t*>(d_wire), static_cast<uint8_t*>(d_payload), d_desc, d_status,
            ws_ptr<const uint64_t>(ws, L.offs[0]), ws_ptr<const uint64_t>(ws, L.offs[1]),
            ws_ptr<const uint64_t>(ws, L.hdr), cap, (uint32_t)n);
    } else {
        launch_pass<kModeDeser>(L, 0, d_wire, d_payload, d_desc, d_status, ws, cap, n, kClassAll, st);
    }
    return launch_check("deserialize_execute");
}

int cfws_deserialize_batch(const void* d_wire, uint64_t wire_size, const uint64_t* d_index,
                           size_t n, uint64_t max_payload, uint32_t align, uint32_t flags,
                           cfws_frame_desc_t* d_desc, int32_t* d_status, void* d_payload,
                           uint64_t cap, uint64_t* d_total, void* ws, size_t ws_size,
                           void* stream)
{
    // small batch without reassembly, every argument valid: one launch
    if (small_path() && n > 0 && n <= kSmallFrames && cap <= kSmallBytes && flags == 0 && align != 0 &&
        (align & (align - 1)) == 0 && align <= 4096 && check_init() == CFWS_OK && d_wire && d_index &&
        d_desc && d_status && ws && ws_size >= ws_layout(n, cap).bytes &&
        (cap == 0 || (d_payload && !misaligned(d_payload, d_wire)))) {
        deserialize_small_kernel<<<small_grid(cap), kThreads, 0, static_cast<hipStream_t>(stream)>>>(
            static_cast<const uint8_t*>(d_wire), wire_size, d_index, (uint32_t)n, max_payload, align,
            d_desc, d_status, static_cast<uint8_t*>(d_payload), cap,
            ws_ptr<uint64_t>(ws, ws_layout(n, cap).hdr), d_total);
        return launch_check("deserialize_batch(small)");
    }
    if (int rc = cfws_deserialize_plan(d_wire, wire_size, d_index, n, max_payload, align, flags,
                                       d_desc, d_status, cap, d_total, ws, ws_size, stream))
        return rc;
    return cfws_deserialize_execute(d_wire, d_desc, d_status, n, flags, d_payload, cap, ws, stream);
}

// ---- WebSocket over HTTP/2 -------------------------------------------------

namespace {

struct H2SerLayout {
    uint64_t ser;        // WS serialize workspace
    uint64_t hdr;        // [0] wrapped total (clamped) [3] DATA-frame count
    uint64_t vals;       // u64[n]: DATA frames per WS frame -> first DATA frame
    uint64_t partials;
    uint64_t ddesc;      // cfws_frame_desc_t[n_max]
    uint64_t doffs;      // u64[n_max]
    uint64_t map;        // u32[regions + 2]
    uint64_t bytes, n_max, regions;
};

H2SerLayout h2_ser_layout(uint64_t n, uint64_t wire_cap, uint64_t h2_cap, uint64_t S)
{
    H2SerLayout L;
    L.n_max = n + wire_cap / S + 1;
    L.regions = (h2_cap + kRegion - 1) / kRegion;
    uint64_t at = align_up(ws_layout(n, wire_cap).bytes, 256);
    L.ser = 0;
    L.hdr = at; at += 256;
    L.vals = at; at = align_up(at + 8 * n, 256);
    L.partials = at; at = align_up(at + 8 * ((n + kScanBlock - 1) / kScanBlock + 1), 256);
    L.ddesc = at; at = align_up(at + sizeof(cfws_frame_desc_t) * L.n_max, 256);
    L.doffs = at; at = align_up(at + 8 * L.n_max, 256);
    L.map = at; at = align_up(at + 4 * (L.regions + 2), 256);
    L.bytes = at;
    return L;
}

struct H2DeLayout {
    uint64_t pool;       // pool pass (DATA unwrap): a WsLayout over n_h2 frames
    uint64_t pdesc;      // cfws_frame_desc_t[n_h2]
    uint64_t es;         // u64[n_h2]: END_STREAM flags -> message ids
    uint64_t es_part;
    uint64_t es_total;   // u64: message count
    uint64_t starts, ends;   // u64[n_h2]
    uint64_t first;      // u64[n_h2]: a message's first DATA frame
    uint64_t wsd;        // WS deserialize workspace
    uint64_t udesc;      // cfws_frame_desc_t[n_h2]: fused payload-pass units
    uint64_t ustatus;    // int32[n_h2]
    uint64_t bytes;
};

H2DeLayout h2_de_layout(uint64_t n, uint64_t pool_cap, uint64_t payload_cap)
{
    H2DeLayout L;
    uint64_t at = 0;
    L.pool = at; at = align_up(at + ws_layout(n, pool_cap).bytes, 256);
    L.pdesc = at; at = align_up(at + sizeof(cfws_frame_desc_t) * n, 256);
    L.es = at; at = align_up(at + 8 * n, 256);
    L.es_part = at; at = align_up(at + 8 * ((n + kScanBlock - 1) / kScanBlock + 1), 256);
    L.es_total = at; at += 256;
    L.starts = at; at = align_up(at + 8 * n, 256);
    L.ends = at; at = align_up(at + 8 * n, 256);
    L.first = at; at = align_up(at + 8 * n, 256);
    L.wsd = at; at = align_up(at + ws_layout(n, payload_cap).bytes, 256);
    L.udesc = at; at = align_up(at + sizeof(cfws_frame_desc_t) * n, 256);
    L.ustatus = at; at = align_up(at + 4 * n, 256);
    L.bytes = at;
    return L;
}

}  // namespace

size_t cfws_h2_serialize_workspace_size(size_t n, uint64_t wire_cap, uint64_t h2_cap, uint32_t S)
{
    return (size_t)h2_ser_layout(n, wire_cap, h2_cap, S ? S : CFWS_H2_DEFAULT_MAX_FRAME_SIZE).bytes;
}

size_t cfws_h2_deserialize_workspace_size(size_t n_h2, uint64_t pool_cap, uint64_t payload_cap)
{
    return (size_t)h2_de_layout(n_h2, pool_cap, payload_cap).bytes;
}

int cfws_h2_serialize_batch(const void* d_payload, cfws_frame_desc_t* d_desc, size_t n,
                            uint32_t stream_id, uint32_t S, void* d_wire, uint64_t wire_cap,
                            void* d_h2, uint64_t h2_cap, uint64_t* d_h2_total, void* ws,
                            size_t ws_size, void* stream)
{
    if (int rc = check_init()) return rc;
    if (S == 0) S = CFWS_H2_DEFAULT_MAX_FRAME_SIZE;
    if (S > 0xffffff) return set_err(CFWS_ERROR_INVALID_ARGUMENT, "max_frame_size > 2^24-1", hipSuccess);
    const H2SerLayout L = h2_ser_layout(n, wire_cap, h2_cap, S);
    if (!ws || ws_size < L.bytes) return set_err(CFWS_ERROR_WORKSPACE, "workspace too small", hipSuccess);
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (n == 0) {
        if (d_h2_total) (void)hipMemsetAsync(d_h2_total, 0, 8, st);
        return launch_check("h2_serialize(empty)");
    }
    // 1. the WS frames' layout, exactly as cfws_serialize_batch lays them
    //    out (header sizes, wire offsets into d_desc). With max_frame_size
    //    >= 64 every WS header lies in its first DATA frame and the WS bytes
    //    go straight into the DATA frames (kModeH2Ser, one streaming pass);
    //    smaller limits write the WS wire first and wrap it (two passes).
    const bool fused = S >= 64;
    const WsLayout WL = ws_layout(n, wire_cap);
    uint64_t* hdr = ws_ptr<uint64_t>(ws, L.hdr);
    cfws_frame_desc_t* ddesc = ws_ptr<cfws_frame_desc_t>(ws, L.ddesc);
    uint64_t* doffs = ws_ptr<uint64_t>(ws, L.doffs);
    uint32_t* map = ws_ptr<uint32_t>(ws, L.map);
    if (fused) {
        // WS layout + DATA frames + region map in two launches (three above
        // kSelfScanBlocks blocks)
        const uint32_t nb = grid_for(n, kPlanBlock);
        const uint32_t self_scan = nb <= kSelfScanBlocks ? 1u : 0u;
        uint64_t* pw = ws_ptr<uint64_t>(ws, WL.partials[0]);
        uint64_t* pk = ws_ptr<uint64_t>(ws, WL.partials[1]);
        h2_ser_plan_reduce_kernel<<<nb, kThreads, 0, st>>>(d_desc, n, S, pw, pk);
        if (!self_scan) scan_partials2_kernel<<<2, kThreads, 0, st>>>(pw, pk, nb, hdr + 4, hdr + 5);
        h2_ser_plan_apply_kernel<<<nb, kThreads, 0, st>>>(d_desc, n, S, pw, pk, nb, self_scan, hdr,
                                                         h2_cap, L.n_max, ddesc, doffs, map, d_h2_total);
    } else {
        if (int rc = cfws_serialize_batch(d_payload, d_desc, n, d_wire, wire_cap, nullptr, ws, WL.bytes,
                                          stream))
            return rc;
        // 2. their DATA frames
        uint64_t* vals = ws_ptr<uint64_t>(ws, L.vals);
        h2_count_kernel<<<grid_for(n, kThreads), kThreads, 0, st>>>(d_desc, n, S, vals);
        if (int rc = run_scan(vals, n, ws_ptr<uint64_t>(ws, L.partials), hdr + 3, st)) return rc;
        h2_expand_kernel<<<grid_for(n, kThreads), kThreads, 0, st>>>(d_desc, vals, n, S, L.n_max, ddesc,
                                                                      doffs);
        h2_finalize_kernel<<<grid_for(L.n_max, kThreads), kThreads, 0, st>>>(
            ddesc, doffs, L.n_max, hdr + 3, ws_ptr<const uint64_t>(ws, WL.hdr + 24), h2_cap, map, hdr,
            d_h2_total);
    }
    // 3. the DATA frames: 9-byte header + slice, one streaming pass
    if (h2_cap && fused)
        launch_streaming<kModeH2Ser>(d_payload, d_h2, ddesc, nullptr, doffs, map, hdr, nullptr,
                                     L.regions, h2_cap, L.n_max, kClassAll, stream_id, st, d_desc);
    else if (h2_cap)
        launch_streaming<kModeH2Wrap>(d_wire, d_h2, ddesc, nullptr, doffs, map, hdr, nullptr,
                                      L.regions, h2_cap, L.n_max, kClassAll, stream_id, st);
    return launch_check("h2_serialize");
}

int cfws_h2_deserialize_batch(const void* d_h2, uint64_t h2_size, const uint64_t* d_h2_index,
                              size_t n, uint32_t S, int32_t* d_h2_status, void* d_pool,
                              uint64_t pool_cap, uint64_t max_payload, uint32_t align,
                              cfws_frame_desc_t* d_msg_desc, int32_t* d_msg_status,
                              void* d_payload, uint64_t payload_cap, uint64_t* d_payload_total,
                              size_t* n_messages, void* ws, size_t ws_size, void* stream)
{
    if (int rc = check_init()) return rc;
    if (S == 0) S = CFWS_H2_DEFAULT_MAX_FRAME_SIZE;
    const H2DeLayout L = h2_de_layout(n, pool_cap, payload_cap);
    if (!ws || ws_size < L.bytes) return set_err(CFWS_ERROR_WORKSPACE, "workspace too small", hipSuccess);
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (n_messages) *n_messages = 0;
    if (n == 0) {
        if (d_payload_total) (void)hipMemsetAsync(d_payload_total, 0, 8, st);
        return launch_check("h2_deserialize(empty)");
    }
    if (!d_h2 || !d_h2_index || !d_h2_status || !d_pool || !d_msg_desc || !d_msg_status || !d_payload)
        return set_err(CFWS_ERROR_INVALID_ARGUMENT, "null pointer", hipSuccess);
    // 1. unwrap: DATA payloads pooled back to back (a prefix-strip pass).
    //    The plan's fast form assumes the pool capacity holds them all.
    const WsLayout PL = ws_layout(n, pool_cap);
    void* pws = ws_ptr<void>(ws, L.pool);
    uint64_t* phdr = ws_ptr<uint64_t>(pws, PL.hdr);
    uint64_t* poffs = ws_ptr<uint64_t>(pws, PL.offs[0]);
    cfws_frame_desc_t* pdesc = ws_ptr<cfws_frame_desc_t>(ws, L.pdesc);
    uint64_t* es = ws_ptr<uint64_t>(ws, L.es);
    uint64_t* n_msg_d = ws_ptr<uint64_t>(ws, L.es_total);
    uint64_t* starts = ws_ptr<uint64_t>(ws, L.starts);
    uint64_t* ends = ws_ptr<uint64_t>(ws, L.ends);
    uint64_t* first = ws_ptr<uint64_t>(ws, L.first);
    const uint8_t* h2 = static_cast<const uint8_t*>(d_h2);
    {
        const uint32_t nb = grid_for(n, kPlanBlock);
        const uint32_t self_scan = nb <= kSelfScanBlocks ? 1u : 0u;
        uint64_t* pp = ws_ptr<uint64_t>(pws, PL.partials[0]);
        uint64_t* pe = ws_ptr<uint64_t>(pws, PL.partials[1]);
        h2_de_plan_reduce_kernel<<<nb, kThreads, 0, st>>>(h2, h2_size, d_h2_index, n, S, pdesc,
                                                          d_h2_status, pp, pe);
        if (!self_scan) scan_partials2_kernel<<<2, kThreads, 0, st>>>(pp, pe, nb, phdr + 3, n_msg_d);
        h2_de_plan_apply_kernel<<<nb, kThreads, 0, st>>>(pdesc, d_h2_status, n, pp, pe, nb, self_scan,
                                                         phdr, poffs, es, n_msg_d, starts, ends, first);
    }
    uint64_t counts[2] = {0, 0};       // messages, pooled bytes
    auto read_counts = [&]() -> int {
        hipError_t e = hipMemcpyAsync(&counts[0], n_msg_d, 8, hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipMemcpyAsync(&counts[1], phdr + 3, 8, hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e != hipSuccess) return set_err(CFWS_ERROR_HIP, "h2_deserialize message count", e);
        return CFWS_OK;
    };
    if (int rc = read_counts()) return rc;
    void* wsd = ws_ptr<void>(ws, L.wsd);
    const WsLayout WL = ws_layout(n, payload_cap);
    if (counts[1] > pool_cap) {
        // 2'. general form: the pool capacity cuts DATA payloads, and a frame
        //     past it is OUT_OF_MEMORY and closes no message. Pool offsets
        //     and the grand total stand; the capacity rule, END_STREAM flags
        //     and messages are redone (co_http2_stream.c:550-608).
        deserialize_finalize_kernel<<<grid_for(n, kThreads), kThreads, 0, st>>>(
            pdesc, d_h2_status, poffs, poffs, phdr, n, pool_cap, 0, ws_ptr<uint32_t>(pws, PL.map[0]),
            ws_ptr<uint32_t>(pws, PL.map[1]), nullptr);
        h2_end_flags_kernel<<<grid_for(n, kThreads), kThreads, 0, st>>>(pdesc, d_h2_status, n, es);
        if (int rc = run_scan(es, n, ws_ptr<uint64_t>(ws, L.es_part), n_msg_d, st)) return rc;
        h2_messages_kernel<<<grid_for(n, kThreads), kThreads, 0, st>>>(pdesc, d_h2_status, es, n, ends);
        h2_starts_kernel<<<grid_for(n, kThreads), kThreads, 0, st>>>(ends, n_msg_d, n, starts);
        if (int rc = read_counts()) return rc;
        if (n_messages) *n_messages = (size_t)counts[0];
        // 3'. each pooled message through co_ws_frame_deserialize against
        //     its own size (co_ws_http2_extension.c:134-164), from the
        //     materialised pool (layout-first OOM rule)
        if (pool_cap)
            launch_pass<kModeDeser>(PL, 0, d_h2, d_pool, pdesc, d_h2_status, pws, pool_cap, n,
                                    kClassAll, st);
        if (int rc = deserialize_plan_impl(d_pool, pool_cap, starts, ends, counts[0], max_payload, align,
                                           0, d_msg_desc, d_msg_status, payload_cap,
                                           d_payload_total, wsd, WL.bytes, stream))
            return rc;
        return cfws_deserialize_execute(d_pool, d_msg_desc, d_msg_status, counts[0], 0, d_payload,
                                        payload_cap, wsd, stream);
    }
    const uint64_t n_msg = counts[0];
    if (n_messages) *n_messages = (size_t)n_msg;
    // 2. fused: the pool is never written. Each message's WS header is
    //    gathered from its DATA frames and parsed against the message's own
    //    size (co_ws_http2_extension.c:134-164); then its layout.
    if (align == 0 || (align & (align - 1)) || align > 4096)
        return set_err(CFWS_ERROR_INVALID_ARGUMENT, "align must be a power of two <= 4096", hipSuccess);
    uint64_t* hdr = ws_ptr<uint64_t>(wsd, WL.hdr);
    if (n_msg == 0) return zero_totals(WL, wsd, d_payload_total, st);
    uint64_t* offs0 = ws_ptr<uint64_t>(wsd, WL.offs[0]);
    uint64_t* part0 = ws_ptr<uint64_t>(wsd, WL.partials[0]);
    const uint32_t mb = grid_for(n_msg, kPlanBlock);
    const uint32_t m_self = mb <= kSelfScanBlocks ? 1u : 0u;
    h2_msg_parse_kernel<<<mb, kThreads, 0, st>>>(h2, pdesc, d_h2_status, poffs, n, starts, ends, n_msg,
                                                max_payload, align, d_msg_desc, d_msg_status, offs0,
                                                first, part0);
    if (!m_self) scan_partials_kernel<<<1, kThreads, 0, st>>>(part0, mb, hdr + 3);
    deserialize_plan_apply_kernel<<<mb, kThreads, 0, st>>>(
        d_msg_desc, d_msg_status, offs0, ws_ptr<uint64_t>(wsd, WL.offs[1]), n_msg, part0,
        ws_ptr<uint64_t>(wsd, WL.partials[1]), mb, m_self, hdr, payload_cap, 0,
        ws_ptr<uint32_t>(wsd, WL.map[0]), ws_ptr<uint32_t>(wsd, WL.map[1]), d_payload_total);
    // 3. one payload-pass unit per DATA frame, and the pass's region map
    cfws_frame_desc_t* udesc = ws_ptr<cfws_frame_desc_t>(ws, L.udesc);
    int32_t* ustatus = ws_ptr<int32_t>(ws, L.ustatus);
    uint64_t* uoffs = ws_ptr<uint64_t>(wsd, WL.offs[1]);
    uint32_t* umap = ws_ptr<uint32_t>(wsd, WL.map[1]);
    h2_units_kernel<<<grid_for(n, kThreads), kThreads, 0, st>>>(
        pdesc, d_h2_status, poffs, es, n, n_msg, starts, d_msg_desc, d_msg_status, hdr, udesc,
        ustatus, uoffs, umap);
    if (payload_cap)
        launch_streaming<kModeDeser>(d_h2, d_payload, udesc, ustatus, uoffs, umap, hdr, nullptr,
                                     WL.regions, payload_cap, n, kClassAll, 0, st);
    return launch_check("h2_deserialize");
}

size_t cfws_index_workspace_size(size_t n_conns)
{
    return 64 + sizeof(uint64_t) * (size_t)grid_for(n_conns, kScanBlock);
}

int cfws_index_frames_batch(const void* d_buf, const uint64_t* d_begin, const uint64_t* d_end,
                            size_t n, uint64_t max_payload, uint64_t* d_starts, uint64_t cap,
                            uint64_t* d_first, uint64_t* d_consumed, int32_t* d_stop,
                            uint64_t* d_total, void* ws, size_t ws_size, void* stream)
{
    if (int rc = check_init()) return rc;
    if (ws_size < cfws_index_workspace_size(n))
        return set_err(CFWS_ERROR_WORKSPACE, "index workspace too small", hipSuccess);
    if ((n && (!d_buf || !d_begin || !d_end || !d_first || !d_consumed || !d_stop)) ||
        (cap && !d_starts) || !d_total || !ws)
        return set_err(CFWS_ERROR_INVALID_ARGUMENT, "index: null pointer", hipSuccess);
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (n == 0) {
        (void)hipMemsetAsync(d_total, 0, 8, st);
        return launch_check("index");
    }
    const uint8_t* buf = static_cast<const uint8_t*>(d_buf);
    uint64_t* partials = ws_ptr<uint64_t>(ws, 64);
    const uint32_t g = grid_for(n, kThreads);
    index_walk_kernel<false><<<g, kThreads, 0, st>>>(buf, d_begin, d_end, n, max_payload, d_first,
                                                     d_consumed, d_stop, nullptr, 0);
    if (int rc = run_scan(d_first, n, partials, d_total, st)) return rc;
    index_walk_kernel<true><<<g, kThreads, 0, st>>>(buf, d_begin, d_end, n, max_payload, d_first,
                                                    nullptr, nullptr, d_starts, cap);
    return launch_check("index");
}

int cfws_ws_accept_keys_batch(const void* d_keys, const uint64_t* d_key_off, size_t n,
                              char* d_accept, void* stream)
{
    if (int rc = check_init()) return rc;
    if (n == 0) return CFWS_OK;
    if (!d_keys || !d_key_off || !d_accept)
        return set_err(CFWS_ERROR_INVALID_ARGUMENT, "accept keys: null pointer", hipSuccess);
    ws_accept_kernel<<<grid_for(n, kThreads), kThreads, 0, static_cast<hipStream_t>(stream)>>>(
        static_cast<const uint8_t*>(d_keys), d_key_off, n, d_accept);
    return launch_check("ws_accept_keys");
}

void* cfws_mapped_device_pointer(const void* h_ptr)
{
    if (check_init() != CFWS_OK || !h_ptr) return nullptr;
    unsigned flags = 0;
    void* d = nullptr;
    if (hipHostGetFlags(&flags, const_cast<void*>(h_ptr)) != hipSuccess || !(flags & hipHostMallocMapped) ||
        hipHostGetDevicePointer(&d, const_cast<void*>(h_ptr), 0) != hipSuccess) {
        (void)hipGetLastError();     // not a mapped HIP host allocation: no sticky error
        return nullptr;
    }
    return d;
}

int cfws_copy_to_host(const void* d_src, void* h_dst, uint64_t n, void* stream)
{
    if (int rc = check_init()) return rc;
    if (n == 0) return CFWS_OK;
    if (!d_src || !h_dst) return set_err(CFWS_ERROR_INVALID_ARGUMENT, "null pointer", hipSuccess);
    void* d = cfws_mapped_device_pointer(h_dst);
    if (!d) return set_err(CFWS_ERROR_INVALID_ARGUMENT, "destination is not mapped pinned host memory",
                           hipSuccess);
    return cfws_internal_copy_out(d_src, d, n, stream);
}

int cfws_encode_headers(cfws_frame_desc_t* d_desc, size_t n, void* d_wire, uint64_t wire_capacity,
                        void* stream)
{
    if (int rc = check_init()) return rc;
    if (n == 0) return CFWS_OK;
    if (!d_desc || !d_wire) return set_err(CFWS_ERROR_INVALID_ARGUMENT, "null pointer", hipSuccess);
    if (n > 0xffffffffull) return set_err(CFWS_ERROR_INVALID_ARGUMENT, "too many frames", hipSuccess);
    encode_headers_kernel<<<grid_for(n, kThreads), kThreads, 0, static_cast<hipStream_t>(stream)>>>(
        d_desc, n, static_cast<uint8_t*>(d_wire), wire_capacity);
    return launch_check("encode_headers");
}

int cfws_parse_headers(const void* d_wire, uint64_t wire_size, const uint64_t* d_frame_index, size_t n,
                       uint64_t max_payload, cfws_frame_desc_t* d_desc, int32_t* d_status,
                       void* stream)
{
    if (int rc = check_init()) return rc;
    if (n == 0) return CFWS_OK;
    if (!d_wire || !d_frame_index || !d_desc || !d_status)
        return set_err(CFWS_ERROR_INVALID_ARGUMENT, "null pointer", hipSuccess);
    parse_headers_kernel<<<grid_for(n, kThreads), kThreads, 0, static_cast<hipStream_t>(stream)>>>(
        static_cast<const uint8_t*>(d_wire), wire_size, d_frame_index, n, max_payload, d_desc,
        d_status);
    return launch_check("parse_headers");
}

}  // extern "C"

namespace {

// Pieces per frame for the split payload ops: enough workgroups to cover the
// largest frame in one pass, capped so the grid stays under 2^31 blocks.
uint32_t payload_pieces(size_t n, uint64_t max_payload_size)
{
    const uint64_t chunks = max_payload_size / 16 + 2;
    uint64_t pieces = (chunks + kPieceChunks - 1) / kPieceChunks;
    if (pieces > 65536) pieces = 65536;
    while (pieces > 1 && pieces * n > 0x7fffffffull) pieces >>= 1;
    return (uint32_t)pieces;
}

template <bool kUnmask>
int launch_payload_xor(const void* src, void* dst, const cfws_frame_desc_t* d_desc,
                       const int32_t* d_status, size_t n, uint64_t max_payload_size, uint64_t cap,
                       void* stream, const char* what)
{
    if (int rc = check_init()) return rc;
    if (n == 0 || cap == 0) return CFWS_OK;
    if (!src || !dst || !d_desc) return set_err(CFWS_ERROR_INVALID_ARGUMENT, "null pointer", hipSuccess);
    if (misaligned(src, dst))
        return set_err(CFWS_ERROR_INVALID_ARGUMENT, "arenas must be 16-byte aligned", hipSuccess);
    if (n > 0x7fffffffull) return set_err(CFWS_ERROR_INVALID_ARGUMENT, "too many frames", hipSuccess);
    const uint32_t pieces = payload_pieces(n, max_payload_size);
    payload_xor_kernel<kUnmask><<<(uint32_t)(n * pieces), kThreads, xform_lds_bytes(),
                                  static_cast<hipStream_t>(stream)>>>(
        static_cast<const uint8_t*>(src), static_cast<uint8_t*>(dst), d_desc, d_status, n, pieces, cap);
    return launch_check(what);
}

}  // namespace

extern "C" {

int cfws_mask_batch(const void* d_payload, const cfws_frame_desc_t* d_desc, size_t n,
                    uint64_t max_payload_size, void* d_wire, uint64_t wire_capacity, void* stream)
{
    return launch_payload_xor<false>(d_payload, d_wire, d_desc, nullptr, n, max_payload_size,
                                     wire_capacity, stream, "mask_batch");
}

int cfws_unmask_batch(const void* d_wire, const cfws_frame_desc_t* d_desc, const int32_t* d_status,
                      size_t n, uint64_t max_payload_size, void* d_payload,
                      uint64_t payload_capacity, void* stream)
{
    return launch_payload_xor<true>(d_wire, d_payload, d_desc, d_status, n, max_payload_size,
                                    payload_capacity, stream, "unmask_batch");
}

int cfws_xor_mask(const void* d_src, void* d_dst, uint64_t n, uint32_t key, uint32_t phase,
                  void* stream)
{
    if (int rc = check_init()) return rc;
    if (n == 0) return CFWS_OK;
    const uint64_t blocks = (n / 16 + kThreads - 1) / kThreads;
    const uint32_t g = (uint32_t)(blocks == 0 ? 1 : (blocks < 4096 ? blocks : 4096));
    xor_mask_kernel<<<g, kThreads, 0, static_cast<hipStream_t>(stream)>>>(
        static_cast<const uint8_t*>(d_src), static_cast<uint8_t*>(d_dst), n, key, phase & 3u);
    return launch_check("xor_mask");
}

int cfws_fill_splitmix(void* d_dst, uint64_t n, uint64_t seed, uint64_t byte_base, void* stream)
{
    if (int rc = check_init()) return rc;
    if (byte_base & 7u) return set_err(CFWS_ERROR_INVALID_ARGUMENT, "byte_base % 8 != 0", hipSuccess);
    if (reinterpret_cast<uintptr_t>(d_dst) & 15u)
        return set_err(CFWS_ERROR_INVALID_ARGUMENT, "destination must be 16-byte aligned", hipSuccess);
    if (n == 0) return CFWS_OK;
    const uint64_t blocks = (n / 16 + kThreads - 1) / kThreads;
    const uint32_t g = (uint32_t)(blocks == 0 ? 1 : (blocks < 8192 ? blocks : 8192));
    fill_splitmix_kernel<<<g, kThreads, 0, static_cast<hipStream_t>(stream)>>>(
        static_cast<uint8_t*>(d_dst), n, seed, byte_base / 8);
    return launch_check("fill_splitmix");
}

}  // extern "C"

uint64_t cfws_internal_h2_grand_total_offset(uint64_t n_h2, uint64_t pool_cap, uint64_t payload_cap)
{
    return h2_de_layout(n_h2, pool_cap, payload_cap).wsd + ws_layout(n_h2, payload_cap).hdr +
           3 * sizeof(uint64_t);
}
