// cfws_uniform.hip -- the compact send of a uniform batch
// (cfws_serialize_uniform, include/cfws.h).
//
// Every frame of the batch has the same payload size, fin, opcode and mask:
// n sequential co_ws_frame_serialize calls (src/ws/co_ws_frame.c:21-119)
// appending fixed-size messages to one co_byte_array. Frame i's wire bytes
// are then [i W, (i + 1) W), W = header size + payload size, its payload
// source [i fs, (i + 1) fs): no layout depends on another frame, so there is
// no plan and no descriptor table. Per frame the pass reads the payload and a
// 4-byte key and writes the frame -- the descriptor form reads a 32-byte
// descriptor per frame in its plan and again in its execute (14 % more read
// traffic at 256 B) and writes wire_off back into it.
//
// Each wave owns a span of wire (4 KiB in the small kernel, 2 KiB in the
// general one; aligned 16-byte chunks, every wire byte written once); a chunk's frame comes from a multiply by a 32-bit
// reciprocal of W (host-computed) and one correction, relative to the wave's
// first frame. Three kernels, by frame size (uniform_route):
//  * serialize_uniform_small_kernel, payloads of 32-65,535 bytes that are
//    multiples of 16 (headers of at most 8 bytes, every payload 16-aligned in
//    the source): every chunk of the span -- body or header -- in one store
//    round, a header chunk assembled in registers from its own source blocks,
//    the frame's key and the next chunk's first block (over DPP); every load
//    issued before any computes (comment at the kernel).
//  * serialize_uniform_kernel, any other frame of at least 32 wire bytes, in
//    two phases: body chunks (one or two aligned source loads, a funnel shift
//    and the key XOR), then the chunks the body phase skipped -- exactly the
//    chunks that hold header bytes, one or two per frame -- handed out one
//    per lane (frame fr of the span to lanes 2 fr and 2 fr + 1), each the end
//    of one payload, a header and the start of the next payload.
//  * serialize_uniform_bytes_kernel, frames of under 32 wire bytes (payloads
//    up to 17-29 bytes): byte by byte.
#include "cfws_kernels.h"

namespace {

// serialize_uniform_small_kernel<kU> spans kU KiB of wire per wave (4 or 2,
// small_span); serialize_uniform_kernel 2 KiB (4,100 B frames 1.70 -> 1.51
// ms, 1,000 B 1.83 -> 1.75, 64 KiB 1.455 -> 1.44 against 4 KiB;
// profiles/r06/compact/uniform_general/spans.txt)
#ifndef CFWS_UNIFORM_GEN_UNROLL
#define CFWS_UNIFORM_GEN_UNROLL 2
#endif
constexpr int kGenUnroll = CFWS_UNIFORM_GEN_UNROLL;
constexpr uint32_t kGenSpan = 64u * 16u * kGenUnroll;
#ifndef CFWS_UNIFORM_STORE_AUX
#define CFWS_UNIFORM_STORE_AUX 19                                 // write-through, as the WS send (st16_region)
#endif

// Uniform frame parameters (all wave-uniform).
struct UniformFrames {
    const uint8_t* src;
    const uint32_t* keys;      // null: unmasked
    uint64_t n;                // frames
    uint64_t fs;               // payload bytes per frame (< 2^30)
    uint32_t hs;               // header bytes (2..14)
    uint32_t W;                // wire bytes per frame: hs + fs
    uint32_t M;                // ceil(2^32 / W): r / W = mulhi(r, M) or one less, r < 2^31
    uint32_t hb;               // header byte 0 | mask << 8 (ws_header_words)
    uint64_t total;            // n W
    double invW;               // 1 / W, for the wave's first frame
};

__device__ __forceinline__ uint32_t div_w(const UniformFrames& U, uint32_t r)
{
    uint32_t q = __umulhi(r, U.M);
    if (q * U.W > r) --q;
    return q;
}

// A chunk of the wave's span: D0 the span's start (wave-uniform, the base of
// the buffer resource `rs`), D the chunk's. Past the capacity byte by byte.
template <typename Rsrc>
__device__ __forceinline__ void uniform_store(uint8_t* __restrict__ out, Rsrc rs, uint64_t D0, uint64_t D,
                                              uint64_t cap, uint4 o)
{
    if (D + 16 <= cap) {
        if (CFWS_UNIFORM_STORE_AUX == 0) {
            st16(out + D, o);
        } else {
            const u32x4 v = {o.x, o.y, o.z, o.w};
            __builtin_amdgcn_raw_buffer_store_b128(v, rs, (int)(D - D0), 0, CFWS_UNIFORM_STORE_AUX);
        }
    } else {
        for (uint32_t j = 0; D + j < cap; ++j) out[D + j] = (uint8_t)(u4_byte(o, (int)j));
    }
}

// Source blocks through a buffer resource whose base is the wave's first
// frame's payload: a block that is not wanted gets an offset past the
// resource's range and reads as zeros without a memory access, so every load
// of the span is issued unconditionally. With a branch around a load, the
// join made the compiler wait for all loads in flight after each round
// (s_waitcnt vmcnt(0) for a register copy), serialising the rounds.
constexpr uint32_t kNoLoad = 0x7ffffff0u;
__device__ __forceinline__ uint4 src_ld16(__amdgpu_buffer_rsrc_t rs, uint32_t off)
{
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)off, 0, 0);
    return make_uint4(v[0], v[1], v[2], v[3]);
}

// A header chunk: chunk byte 0 is byte `off` of frame f (f + 1 may start in
// the chunk at byte t = W - off). Loads issued by header_prep, bytes by
// header_finish.
struct HeaderChunk {
    uint4 A, B;
    uint32_t k0, k1;
    uint32_t ph, j_lo;
};

__device__ __forceinline__ void header_prep(const UniformFrames& U, uint64_t f, uint32_t off, HeaderChunk& h)
{
    const uint32_t t = U.W - off;
    const uint32_t a = off < U.hs ? U.hs - off : 0u, b = t < 16u ? t : 16u;
    const bool hasF = b > a;
    const bool next = t < 16u && f + 1 < U.n;
    const bool hasN = next && t + U.hs < 16u;
    uint64_t s_lo = 0;
    uint32_t npay = 0;
    h.j_lo = 0;
    if (hasF) {
        s_lo = f * U.fs + (off + a - U.hs);
        h.j_lo = a;
        npay = (b - a) + (hasN ? 16u - (t + U.hs) : 0u);
    } else if (hasN) {
        s_lo = (f + 1) * U.fs;
        h.j_lo = t + U.hs;
        npay = 16u - h.j_lo;
    }
    const uint4 z = make_uint4(0, 0, 0, 0);
    h.A = h.B = z;
    h.ph = (uint32_t)(s_lo & 15u);
    if (npay) {
        const uint8_t* sp = U.src + (s_lo & ~uint64_t(15));
        h.A = ld16(sp);
        if (h.ph + npay > 16u) h.B = ld16(sp + 16);       // the block holds payload bytes of the chunk
    }
    h.k0 = U.keys ? U.keys[f] : 0u;
    h.k1 = U.keys && next ? U.keys[f + 1] : 0u;
}

__device__ __forceinline__ uint4 header_finish(const UniformFrames& U, uint64_t f, uint32_t off, const HeaderChunk& h)
{
    const uint4 z = make_uint4(0, 0, 0, 0);
    const uint32_t t = U.W - off;
    const uint32_t a = off < U.hs ? U.hs - off : 0u, b = t < 16u ? t : 16u;
    const bool hasF = b > a;
    const bool next = t < 16u && f + 1 < U.n;
    const uint32_t he = t + U.hs < 16u ? t + U.hs : 16u;
    const bool hasN = next && he < 16u;
    // Y[k] = source byte s_lo + (k - j_lo)
    const uint4 Y = h.ph >= h.j_lo ? funnel16(h.A, h.B, h.ph - h.j_lo) : funnel16(z, h.A, 16u - (h.j_lo - h.ph));
    uint4 o = z;
    if (off < U.hs)                                           // f's header from its byte off
        o = and4(funnel16(ws_header_words(U.fs, U.hb, h.k0), z, off), byte_range(0, U.hs - off));
    if (hasF) {                                               // the end of f's payload
        uint4 X = Y;
        xor4(X, rotr8(h.k0, off + 16u - U.hs));
        o = or4(o, and4(X, byte_range(a, b)));
    }
    if (next)                                                 // f + 1's header from chunk byte t
        o = or4(o, and4(funnel16(z, ws_header_words(U.fs, U.hb, h.k1), 16u - t), byte_range(t, he)));
    if (hasN) {                                               // the start of f + 1's payload
        uint4 X = hasF ? funnel16(z, Y, 16u - U.hs) : Y;      // contiguous after f's: hs bytes on
        xor4(X, rotr8(h.k1, 16u - (he & 3u)));
        o = or4(o, and4(X, byte_range(he, 16u)));
    }
    return o;
}

// The body chunk at D (round u of `lane`, frame byte `off`) is followed by a
// body chunk of the same frame that this wave loads (lane + 1, or lane 0 of
// round u + 1): its first source block is this chunk's second.
__device__ __forceinline__ bool body_next_of(uint32_t hs, uint32_t W, int u, uint32_t lane, uint32_t off, uint64_t D,
                                             uint64_t lim)
{
    return off + 32u <= W && off + 16u >= hs && D + 16 < lim && !(lane == 63 && u == kGenUnroll - 1);
}

__global__ void __launch_bounds__(kThreads)
serialize_uniform_kernel(UniformFrames U, uint8_t* __restrict__ out, uint64_t cap, uint64_t* __restrict__ user_total)
{
    const uint32_t lane = threadIdx.x & 63u;
    // wave-uniform values in scalar registers
    const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const uint64_t wave = uint64_t(blockIdx.x) * kWaves + wv;
    const uint64_t D0 = wave * kGenSpan;
    const uint64_t lim = U.total < cap ? U.total : cap;
    if (wave == 0 && lane == 0 && user_total) *user_total = U.total;
    if (D0 >= lim) return;
    // the wave's first frame: D0 / W in double (D0 < 2^40), corrected
    uint64_t F0 = (uint64_t)((double)D0 * U.invW);
    if (F0 * U.W > D0) --F0;
    else if ((F0 + 1) * U.W <= D0) ++F0;
    F0 = (uint64_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)F0) |
         (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(F0 >> 32)) << 32;
    const uint64_t base = F0 * U.W;                           // <= D0
    const uint32_t rel0 = (uint32_t)(D0 - base);              // < W
    const uint64_t src0 = F0 * U.fs;
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(out + D0, 0, (int)kGenSpan, 0x00020000);

    // frames whose header meets the span: fa .. fb (fb may be n: the chunk
    // holding the batch's end past the last payload is handled as frame n's)
    auto body_next = [&](int u, uint32_t ln, uint32_t o, uint64_t D, uint64_t lm) {
        return body_next_of(U.hs, U.W, u, ln, o, D, lm);
    };
    const uint64_t fa = (base + U.hs > D0) ? F0 : F0 + 1;
    uint64_t fb = F0 + div_w(U, rel0 + kGenSpan - 1);
    if (fb > U.n) fb = U.n;
    const uint32_t n_hdr = fa <= fb ? 2u * (uint32_t)(fb - fa + 1) : 0u;

    // ---- issue every load: body chunks, then the first 64 header chunks
    uint32_t q[kGenUnroll], off[kGenUnroll], key[kGenUnroll];
    bool body[kGenUnroll];
    uint4 A[kGenUnroll], B[kGenUnroll];
#pragma unroll
    for (int u = 0; u < kGenUnroll; ++u) {
        const uint32_t r = rel0 + 16u * (64u * u + lane);
        q[u] = div_w(U, r);
        off[u] = r - q[u] * U.W;
        body[u] = D0 + 16ull * (64u * u + lane) < lim && off[u] >= U.hs && off[u] + 16u <= U.W;
        A[u] = B[u] = make_uint4(0, 0, 0, 0);
        key[u] = 0;
        if (body[u]) {
            const uint64_t s = src0 + uint64_t(q[u]) * U.fs + (off[u] - U.hs);
            const uint8_t* sp = U.src + (s & ~uint64_t(15));
            A[u] = ld16(sp);
            // the second block: the next chunk's own first block (over DPP)
            // when that chunk is a body chunk of the same frame
            if ((s & 15u) && !body_next(u, lane, off[u], D0 + 16ull * (64u * u + lane), lim)) B[u] = ld16(sp + 16);
            key[u] = U.keys ? U.keys[F0 + q[u]] : 0u;
        }
    }
    uint4 N[kGenUnroll];
#pragma unroll
    for (int u = 0; u < kGenUnroll; ++u)          // every lane: DPP needs the full wave
        N[u] = from_next_lane(A[u], u + 1 < kGenUnroll ? readlane4(A[u + 1 < kGenUnroll ? u + 1 : u], 0)
                                                           : make_uint4(0, 0, 0, 0));
    HeaderChunk h;
    uint64_t hD = 0, hf = 0;
    uint32_t hoff = 0;
    bool hown = false;
    auto header_lane = [&](uint32_t idx) {
        // lane idx of the header pass: frame fa + idx / 2, its first or second header chunk
        hown = false;
        if (idx >= n_hdr) return;
        const uint64_t fr = fa + idx / 2;
        const uint64_t hstart = fr * U.W;
        const uint64_t c1 = hstart >> 4, c2 = (hstart + U.hs - 1) >> 4;
        if ((idx & 1u) && c2 == c1) return;
        hD = ((idx & 1u) ? c2 : c1) << 4;
        if (hD < D0 || hD >= D0 + kGenSpan || hD >= lim) return;
        hf = hD >= hstart ? fr : fr - 1;
        hoff = (uint32_t)(hD - hf * U.W);
        hown = true;
        header_prep(U, hf, hoff, h);
    };
    header_lane(lane);

    // ---- body chunks
#pragma unroll
    for (int u = 0; u < kGenUnroll; ++u) {
        if (!body[u]) continue;
        const uint32_t ph = (uint32_t)((src0 + uint64_t(q[u]) * U.fs + (off[u] - U.hs)) & 15u);
        const bool nb = body_next(u, lane, off[u], D0 + 16ull * (64u * u + lane), lim);
        uint4 o = ph ? funnel16(A[u], nb ? N[u] : B[u], ph) : A[u];
        xor4(o, rotr8(key[u], off[u] - U.hs));
        uniform_store(out, rs, D0, D0 + 16ull * (64u * u + lane), cap, o);
    }
    // ---- header chunks, 64 at a time
    for (uint32_t g = 0; g < n_hdr; g += 64) {
        if (g) header_lane(g + lane);
        if (hown) uniform_store(out, rs, D0, hD, cap, header_finish(U, hf, hoff, h));
    }
}

// The 128-bit value (lo, hi) shifted up by `sh` bytes (0 <= sh < 16): byte j
// moves to j + sh, zeros below.
__device__ __forceinline__ uint4 shl16(uint4 v, uint32_t sh)
{
    const uint64_t lo = (uint64_t)v.x | (uint64_t)v.y << 32, hi = (uint64_t)v.z | (uint64_t)v.w << 32;
    const uint32_t b = 8u * (sh & 7u);
    const uint64_t l1 = b ? lo << b : lo;
    const uint64_t h1 = b ? (hi << b) | (lo >> (64u - b)) : hi;
    const uint64_t L = sh < 8 ? l1 : 0, H = sh < 8 ? h1 : l1;
    return make_uint4((uint32_t)L, (uint32_t)(L >> 32), (uint32_t)H, (uint32_t)(H >> 32));
}

// Frames of 32 <= fs <= 65,535 payload bytes, fs a multiple of 16, masked or
// not (headers of at most 8 bytes, payload starts 16-aligned in the source):
// every chunk of the span, body or header, in one store round, so no 32-byte
// sector of the wire is written in two parts. A header chunk is
//   [f's body tail: bytes < q] [a header at q] [that frame's body head at q + hs]
// (q = header start - chunk start, -7..15): the tail is the chunk's own
// funnel of its source blocks (as a body chunk's), the header 8 bytes from
// the frame's key, the head the NEXT chunk's first source block (that chunk
// lies in the same body, whose source starts 16-aligned), taken over DPP --
// the shape of general_region_ser_edges in cfws_kernels.h, with the frames
// computed instead of read from a plan. The span's keys are read once (lane
// j: frame F0 + j and F0 + 64 + j) and handed to chunks by ds_bpermute.
#ifndef CFWS_UNIFORM_OCC
#define CFWS_UNIFORM_OCC 1                 // __launch_bounds__ workgroups per CU (A/B knob)
#endif
#ifndef CFWS_UNIFORM_DPP_B
#define CFWS_UNIFORM_DPP_B 1               // a body chunk's second block from the next lane: 256 B send 1.57 -> 1.53 ms (A/B knob)
#endif
template <int kU>
__global__ void __launch_bounds__(kThreads, CFWS_UNIFORM_OCC)
serialize_uniform_small_kernel(UniformFrames U, uint8_t* __restrict__ out, uint64_t cap,
                               uint64_t* __restrict__ user_total)
{
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const uint64_t wave = uint64_t(blockIdx.x) * kWaves + wv;
    const uint64_t D0 = wave * (64u * 16u * kU);
    const uint64_t lim = U.total < cap ? U.total : cap;
    if (wave == 0 && lane == 0 && user_total) *user_total = U.total;
    if (D0 >= lim) return;
    uint64_t F0 = (uint64_t)((double)D0 * U.invW);
    if (F0 * U.W > D0) --F0;
    else if ((F0 + 1) * U.W <= D0) ++F0;
    F0 = (uint64_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)F0) |
         (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(F0 >> 32)) << 32;
    const uint32_t rel0 = (uint32_t)(D0 - F0 * U.W);
    const uint64_t src0 = F0 * U.fs;
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(out + D0, 0, (int)(64u * 16u * kU), 0x00020000);
    // payload source from frame F0's first byte (16-aligned: fs % 16 == 0)
    const auto srs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(U.src + src0), 0, (int)kNoLoad,
                                                       0x00020000);
    const uint32_t hs = U.hs, W = U.W;
    uint32_t q[kU], off[kU], ph[kU];
    bool fast[kU], tail[kU], live[kU];
    uint4 A[kU], B[kU];
    const uint4 z = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int u = 0; u < kU; ++u) {
        const uint32_t r = rel0 + 16u * (64u * u + lane);
        q[u] = div_w(U, r);
        off[u] = r - q[u] * W;
        // chunks past the batch end are not written; their neighbours may need
        // their block as a body head (a capacity cut inside the batch)
        live[u] = D0 + 16ull * (64u * u + lane) < U.total;
        fast[u] = off[u] >= hs && off[u] + 16u <= W;
        tail[u] = !fast[u] && off[u] >= hs;                  // f's body, then f + 1's header
        ph[u] = (off[u] - hs) & 15u;
        const bool ld = live[u] && (fast[u] || tail[u]);
        const uint32_t so = (q[u] * (uint32_t)U.fs + (off[u] - hs)) & ~15u;   // < W + 4 KiB
        A[u] = src_ld16(srs, ld ? so : kNoLoad);
        // the second block when the chunk's own bytes reach into it (with
        // CFWS_UNIFORM_DPP_B, a body chunk followed by a chunk of the same
        // body takes it from that chunk's lane instead)
        const bool from_next = CFWS_UNIFORM_DPP_B && fast[u] && off[u] + 16u < W &&
                               !(lane == 63 && u == kU - 1);
        const bool needB = ld && ph[u] && !from_next && (fast[u] || ph[u] + (W - off[u]) > 16u);
        B[u] = src_ld16(srs, needB ? so + 16u : kNoLoad);
    }
    // lane 63's last chunk takes a body head from the next span's first
    // chunk: loaded here (the first block of that frame's payload)
    uint4 hx;
    {
        constexpr int u = kU - 1;
        const bool head = live[u] && !fast[u] && (off[u] < hs ? 16u > hs - off[u] : W - off[u] + hs < 16u) &&
                          (off[u] < hs || F0 + q[u] + 1 < U.n);
        hx = src_ld16(srs, lane == 63 && head ? (q[u] + (off[u] < hs ? 0u : 1u)) * (uint32_t)U.fs : kNoLoad);
    }
    // the span's keys, after the payload loads: frames F0 .. F0 + 127 (W >=
    // 38: at most 110 frames meet a 4 KiB span); keys null: a resource of no
    // bytes, zeros
    const auto krs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(U.keys ? U.keys + F0 : U.keys), 0,
                                                       U.keys ? (int)(U.n - F0 < 128 ? 4 * (U.n - F0) : 512) : 0,
                                                       0x00020000);
    const uint32_t kl0 = __builtin_amdgcn_raw_buffer_load_b32(krs, (int)(4 * lane), 0, 0);
    const uint32_t kl1 = __builtin_amdgcn_raw_buffer_load_b32(krs, (int)(4 * (64 + lane)), 0, 0);
    auto key_of = [&](uint32_t j) {          // frame F0 + j's key, j < 128 (every lane active)
        const uint32_t a = (uint32_t)__shfl((int)kl0, (int)(j & 63u), 64);
        const uint32_t b = (uint32_t)__shfl((int)kl1, (int)(j & 63u), 64);
        return j < 64 ? a : b;
    };
#pragma unroll
    for (int u = 0; u < kU; ++u) {
        const uint4 nextA = u + 1 < kU ? readlane4(A[u + 1 < kU ? u + 1 : u], 0) : hx;
        const uint4 N = from_next_lane(A[u], nextA);        // every lane: DPP needs the full wave
        const uint32_t kf = key_of(q[u]);
        const uint32_t kn = key_of(q[u] + 1);
        const uint64_t D = D0 + 16ull * (64u * u + lane);
        if (D >= lim) continue;
        const bool from_next = CFWS_UNIFORM_DPP_B && fast[u] && off[u] + 16u < W &&
                               !(lane == 63 && u == kU - 1);
        uint4 o = ph[u] ? funnel16(A[u], from_next ? N : B[u], ph[u]) : A[u];
        xor4(o, rotr8(kf, off[u] - hs));
        if (!fast[u]) {
            // the header in the chunk: f's (the chunk starts inside it) or f + 1's
            const bool own_hdr = off[u] < hs;
            const bool has_hdr = own_hdr || F0 + q[u] + 1 < U.n;
            const int qh = own_hdr ? -(int)off[u] : (int)(W - off[u]);          // -7 .. 15
            const uint32_t kh = own_hdr ? kf : kn;
            uint4 w = z;
            if (!own_hdr) w = and4(o, byte_range(0, W - off[u]));              // f's body tail
            if (has_hdr) {
                const uint4 H = ws_header_words(U.fs, U.hb, kh);                   // hs <= 8 bytes
                const uint64_t Hv = (uint64_t)H.x | (uint64_t)H.y << 32;
                const uint4 Hs = qh >= 0 ? shl16(make_uint4(H.x, H.y, 0u, 0u), (uint32_t)qh)
                                         : make_uint4((uint32_t)(Hv >> (8 * -qh)), (uint32_t)(Hv >> (8 * -qh) >> 32),
                                                      0u, 0u);
                w = or4(w, Hs);
                const int sh = qh + (int)hs;                                       // its body head
                if (sh < 16) {
                    uint4 X = N;
                    xor4(X, kh);
                    w = or4(w, shl16(X, (uint32_t)sh));
                }
            }
            o = w;
        }
        uniform_store(out, rs, D0, D, cap, o);
    }
}

// W < 32: frames shorter than two chunks; every chunk byte by byte.
__global__ void __launch_bounds__(kThreads)
serialize_uniform_bytes_kernel(UniformFrames U, uint8_t* __restrict__ out, uint64_t cap,
                               uint64_t* __restrict__ user_total)
{
    const uint64_t c = uint64_t(blockIdx.x) * kThreads + threadIdx.x;
    const uint64_t lim = U.total < cap ? U.total : cap;
    if (c == 0 && user_total) *user_total = U.total;
    const uint64_t D = c * 16;
    if (D >= lim) return;
    uint64_t f = D / U.W;
    uint32_t off = (uint32_t)(D - f * U.W);
    uint32_t w[4] = {0, 0, 0, 0};
    uint32_t k = U.keys ? U.keys[f] : 0u;
    uint4 H = ws_header_words(U.fs, U.hb, k);
    for (int j = 0; j < 16; ++j) {
        if (D + j >= U.total) break;
        if (off == U.W) {
            ++f;
            off = 0;
            k = U.keys ? U.keys[f] : 0u;
            H = ws_header_words(U.fs, U.hb, k);
        }
        uint32_t b;
        if (off < U.hs) {
            b = u4_byte(H, (int)off);
        } else {
            const uint32_t p = off - U.hs;
            b = (U.src[f * U.fs + p] ^ (k >> (8 * (p & 3u)))) & 0xffu;
        }
        w[j >> 2] |= b << (8 * (j & 3));
        ++off;
    }
    const uint4 o = make_uint4(w[0], w[1], w[2], w[3]);
    if (D + 16 <= cap)
        st16(out + D, o);
    else
        for (uint32_t j = 0; D + j < cap; ++j) out[D + j] = (uint8_t)(u4_byte(o, (int)j));
}

__global__ void uniform_total_kernel(uint64_t* __restrict__ user_total, uint64_t total)
{
    if (threadIdx.x == 0) *user_total = total;
}

}  // namespace

namespace {

// the kernel a uniform batch takes (cfws_serialize_uniform and
// cfws_serialize_uniform_pass_kernel)
enum UniformRoute { kUniformSmall, kUniformGeneral, kUniformBytes };
UniformRoute uniform_route(uint64_t fs, uint64_t W)
{
    if (fs >= 32 && fs <= 65535 && fs % 16 == 0) return kUniformSmall;
    return W >= 32 ? kUniformGeneral : kUniformBytes;
}

// the small kernel's span per wave: 2 KiB from CFWS_UNIFORM_SPAN2_MIN-byte
// payloads (1 / 4 KiB frames 2 / 4.5 % faster than at 4 KiB; 256 B 0.5 %
// slower), 4 KiB below
uint64_t small_span(uint64_t fs)
{
    static const uint64_t min2 = (uint64_t)env_knob("CFWS_UNIFORM_SPAN2_MIN", 1024);   // A/B knob
    return fs >= min2 ? 2048 : 4096;
}

uint32_t uniform_header_size(uint64_t fs, bool mask)
{
    return 2u + (fs > 65535u ? 8u : (fs > 125u ? 2u : 0u)) + (mask ? 4u : 0u);
}

}  // namespace

extern "C" const char* cfws_serialize_uniform_pass_kernel(uint64_t fs, uint8_t mask)
{
    switch (uniform_route(fs, uniform_header_size(fs, mask) + fs)) {
    case kUniformSmall: return "serialize_uniform_small_kernel";
    case kUniformGeneral: return "serialize_uniform_kernel";
    default: return "serialize_uniform_bytes_kernel";
    }
}

extern "C" int cfws_serialize_uniform(const void* d_payload, const uint32_t* d_keys, size_t n, uint64_t fs,
                                      uint8_t fin, uint8_t opcode, uint8_t mask, void* d_wire, uint64_t cap,
                                      uint64_t* d_total, void* stream)
{
    const CfwsPassScope pass_scope;
    if (int rc = check_init()) return rc;
    if (fs > (1ull << 30)) return set_err(CFWS_ERROR_INVALID_ARGUMENT, "payload_size > 2^30", hipSuccess);
    const uint32_t hs = uniform_header_size(fs, mask);
    const uint64_t W = hs + fs;
    if (n > (uint64_t(1) << 40) / W) return set_err(CFWS_ERROR_INVALID_ARGUMENT, "batch over 2^40 wire bytes",
                                                    hipSuccess);
    hipStream_t st = static_cast<hipStream_t>(stream);
    const uint64_t total = n * W;
    if (n == 0 || cap == 0) {
        // nothing to write but the total: one thread stores it (no host
        // copy, so nothing waits on the stream)
        if (d_total) uniform_total_kernel<<<1, 64, 0, st>>>(d_total, total);
        return launch_check("serialize_uniform");
    }
    if (!d_wire || (fs && !d_payload) || (mask && !d_keys))
        return set_err(CFWS_ERROR_INVALID_ARGUMENT, "null pointer", hipSuccess);
    if (misaligned(fs ? d_payload : d_wire, d_wire))
        return set_err(CFWS_ERROR_INVALID_ARGUMENT, "arenas must be 16-byte aligned", hipSuccess);
    UniformFrames U;
    U.src = static_cast<const uint8_t*>(d_payload);
    U.keys = mask ? d_keys : nullptr;
    U.n = n;
    U.fs = fs;
    U.hs = hs;
    U.W = (uint32_t)W;
    U.M = (uint32_t)(((uint64_t(1) << 32) + W - 1) / W);
    U.hb = (uint32_t)(opcode | (fin ? 0x80u : 0u)) | (mask ? 0x100u : 0u);
    U.total = total;
    U.invW = 1.0 / (double)W;
    const uint64_t lim = total < cap ? total : cap;
    const CfwsPassTimer timer(st);
    const UniformRoute route = uniform_route(fs, W);
    if (route == kUniformSmall) {
        const uint64_t span = small_span(fs);
        const uint64_t waves = (lim + span - 1) / span;
        const uint64_t blocks = (waves + kWaves - 1) / kWaves;
        if (blocks > 0x7fffffffull) return set_err(CFWS_ERROR_INVALID_ARGUMENT, "batch too large", hipSuccess);
        static const uint32_t lds = (uint32_t)env_knob("CFWS_UNIFORM_LDS", 0);   // residency cap (A/B knob)
        if (small_span(fs) == 2048)
            serialize_uniform_small_kernel<2><<<(uint32_t)blocks, kThreads, lds, st>>>(
                U, static_cast<uint8_t*>(d_wire), cap, d_total);
        else
            serialize_uniform_small_kernel<4><<<(uint32_t)blocks, kThreads, lds, st>>>(
                U, static_cast<uint8_t*>(d_wire), cap, d_total);
    } else if (route == kUniformGeneral) {
        const uint64_t waves = (lim + kGenSpan - 1) / kGenSpan;
        const uint64_t blocks = (waves + kWaves - 1) / kWaves;
        if (blocks > 0x7fffffffull) return set_err(CFWS_ERROR_INVALID_ARGUMENT, "batch too large", hipSuccess);
        // dynamic LDS per workgroup, a residency cap: frames of 32 KiB and
        // more run at 5 workgroups per CU (64 / 128 KiB 1.44 -> 1.39 ms; 4 per
        // CU 1.50; 16 KiB level; 1,000 / 4,100 B 21-30 % slower capped,
        // profiles/r06/compact/uniform_general/lds.txt). CFWS_UNIFORM_LDS
        // overrides (A/B knob; 0 = none).
        static const int64_t lds_knob = env_knob("CFWS_UNIFORM_LDS", -1);
        const uint32_t lds = lds_knob >= 0 ? (uint32_t)lds_knob : W >= 32768 ? 32000u : 0u;
        serialize_uniform_kernel<<<(uint32_t)blocks, kThreads, lds, st>>>(U, static_cast<uint8_t*>(d_wire), cap,
                                                                        d_total);
    } else {
        const uint64_t chunks = (lim + 15) / 16;
        serialize_uniform_bytes_kernel<<<grid_for(chunks, kThreads), kThreads, 0, st>>>(
            U, static_cast<uint8_t*>(d_wire), cap, d_total);
    }
    return launch_check("serialize_uniform");
}
