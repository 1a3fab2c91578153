// cfws_ops.hip -- the codec's smaller device operations and their C ABI
// (include/cfws.h): split header / payload passes over caller-laid-out frames
// (cfws_encode_headers, cfws_parse_headers, cfws_mask_batch,
// cfws_unmask_batch), handshake accept keys, the multi-connection receive
// walk, the single-buffer XOR of the per-frame drop-in, the D2H copy into
// mapped host memory, and the synthetic fill.
#include "cfws_kernels.h"

namespace {

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
// frame, each frame from its own source to its own destination. A wave
// writes one 1 KiB-aligned span of the destination per store instruction
// (64 lanes x 16 B), as the streaming kernel's regions do, so interior
// 64-byte segments are always written whole by one instruction (a span
// grid starting at the frame's first chunk left every instruction's first
// and last segment half-written: 5.6 / 5.9 TB/s against the streaming
// kernel's 6.5). Work unit (frame, piece): the frame's spans are split
// evenly over the fewest pieces of at most 20 spans, each wave taking a
// contiguous run of up to 5 (every load in flight before the first store),
// so a 64 KiB frame is 4 equal workgroups at any alignment. Stores are
// write-through (+0.6 % over `nt` stores and interleaved spans,
// tools/split_ab.sh) and both run at 4 workgroups per CU (the unmask ran
// at 5 until the round-3 rewrite; at 4 since, 1.377 -> 1.349 ms). A run is
// straight-line buffer loads and stores over descriptors clipped to it
// (xor_run); the frame's first and last chunk, which it may share with its
// neighbours, are written byte by byte by payload_edge_kernel after the
// stream. Round 3 took the per-lane bounds and per-store descriptor work out
// of the slots: 1.59 / 1.42 ms -> 1.47 / 1.38 ms (mask / unmask, config 2
// layout, profiles/r03_split_ab/).
#ifndef CFWS_MASK_LDS
#define CFWS_MASK_LDS 40000
#endif
#ifndef CFWS_UNMASK_LDS
#define CFWS_UNMASK_LDS 40000
#endif
constexpr uint32_t kPieceK = 5;
constexpr uint32_t kSpanChunks = 64;
constexpr uint32_t kPieceSpans = kPieceK * kWaves;

// One wave's run of up to kPieceK 1 KiB spans of a frame: every lane of every
// slot loads and stores; buffer descriptors clipped to the run and to the
// frame's whole chunks make the loads outside them return zeros and the
// stores outside them drop, so there is no branch. Lane l of slot k reads
// the aligned source block at offset sd + 1024 k + 16 l of rs
// (funnel-shifted with the next lane's block over DPP; the block after slot
// k < 4 is lane 0 of slot k + 1, rotated into lane 63) and writes the chunk
// at offset dd + 1024 k + 16 l of rd. kEdge: the run holds the frame's first
// span and starts below a descriptor's base (sd or dd negative), so offsets
// go out of range explicitly, never by 32-bit wrap-around. Without it
// (every other run) the offsets are plain: a per-slot edge test cost the
// unmask 7 % (1.46 against 1.37 ms).
// A packed mask's boundary chunks (cfws_mask_batch_packed): the chunks from
// the one holding frame f's header start up to its first whole payload
// chunk, [c0, c0 + 16 nbc), hold frame f - 1's payload tail, f's header,
// then f's payload head. The tail and the header are wave-uniform words
// (T.lo, T.hi: bytes [0, 32) from c0; zero from pre = dof - c0 on); the
// payload head is the lane's own chunk, which is right from dof on.
struct PackedHead {
    uint64_t c0 = 0, dof = 0;
    uint4 lo = {0, 0, 0, 0}, hi = {0, 0, 0, 0};
};

template <bool kEdge, bool kPacked = false>
__device__ __forceinline__ void xor_run(__amdgpu_buffer_rsrc_t rs, __amdgpu_buffer_rsrc_t rd, int32_t sd, int32_t dd,
                                        uint32_t ph, uint32_t kr, uint64_t wbase = 0, const PackedHead* ph_ = nullptr)
{
    constexpr uint64_t kSpan = kSpanChunks * 16;
    const uint32_t lane = threadIdx.x & 63u;
    auto off = [](int32_t o) { return kEdge ? (o < 0 ? 0x7fffffff : o) : o; };
    u32x4 a[kPieceK], ex = {0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < (int)kPieceK; ++k)
        a[k] = __builtin_amdgcn_raw_buffer_load_b128(rs, off(sd + (int32_t)(lane * 16 + k * kSpan)), 0, 0);
    if (ph && lane == 63) ex = __builtin_amdgcn_raw_buffer_load_b128(rs, off(sd + (int32_t)(kPieceK * kSpan)), 0, 0);
    auto slot = [&](const int k) {
        const uint4 A4 = make_uint4(a[k][0], a[k][1], a[k][2], a[k][3]);
        uint4 o = A4;
        if (ph) {
            const uint4 L = k + 1 < (int)kPieceK
                                ? from_next_lane_wrap(make_uint4(a[k + 1][0], a[k + 1][1], a[k + 1][2], a[k + 1][3]))
                                : make_uint4(ex[0], ex[1], ex[2], ex[3]);
            o = funnel16(A4, from_next_lane(A4, L), ph);
        }
        xor4(o, kr);
        if (kPacked) {
            const uint64_t D = wbase + (uint64_t)k * kSpan + lane * 16;
            if (D >= ph_->c0 && D < ph_->dof) {
                const uint32_t q = (uint32_t)(ph_->dof - D < 16 ? ph_->dof - D : 16);   // bytes before the payload
                const uint4 T = D == ph_->c0 ? ph_->lo : ph_->hi;
                o = or4(and4(o, byte_range(q, 16)), and4(T, byte_range(0, q)));
            }
        }
        // write-through, as the streaming kernel's regions (sc0 sc1 nt)
        const u32x4 v = {o.x, o.y, o.z, o.w};
        __builtin_amdgcn_raw_buffer_store_b128(v, rd, off(dd + (int32_t)(lane * 16 + k * kSpan)), 0, 19);
    };
#pragma unroll
    for (int k = 0; k < (int)kPieceK; ++k) slot(k);
}

// cfws_mask_batch_packed: frame g's boundary chunks (PackedHead) are written
// whole by g's first run when g - 1's payload ends exactly where g's header
// starts (checked here, not trusted), g's payload has at least 16 bytes and
// g - 1's at least 16 (so a boundary chunk holds one tail and one header),
// and the chunks end inside the capacity; otherwise payload_edge_kernel
// writes g's head bytes and g - 1's tail bytes one by one, as unpacked.
__device__ __forceinline__ bool packed_inrun(const cfws_frame_desc_t* __restrict__ desc, uint64_t g, uint64_t n,
                                             uint64_t cap)
{
    if (g == 0 || g >= n) return false;
    const DescWords a = load_desc(desc, (uint32_t)(g - 1)), b = load_desc(desc, (uint32_t)g);
    const uint64_t aend = a.wire_off + header_size_of(a.payload_size, a.mask() != 0) + a.payload_size;
    const uint64_t bdof = b.wire_off + header_size_of(b.payload_size, b.mask() != 0);
    return aend == b.wire_off && a.payload_size >= 16 && b.payload_size >= 16 &&
           ((bdof + 15) & ~uint64_t(15)) <= cap;
}

template <bool kUnmask>
__global__ void __launch_bounds__(kThreads)
payload_xor_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                   const cfws_frame_desc_t* __restrict__ desc, const int32_t* __restrict__ status,
                   uint64_t n, uint32_t pieces, uint64_t cap, uint32_t packed)
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
    // the packed mask: this frame's boundary chunks in its first run
    PackedHead H;
    const bool inrun = !kUnmask && packed && packed_inrun(desc, f, n, cap);
    if (inrun) {
        const DescWords a = load_desc(desc, (uint32_t)(f - 1));
        H.c0 = d.wire_off & ~uint64_t(15);
        H.dof = dof;
        const uint32_t t = (uint32_t)(d.wire_off - H.c0);             // f - 1's tail bytes
        const uint4 z = make_uint4(0, 0, 0, 0);
        // the header (co_ws_frame.c:34-91) at byte t of the 32-byte window
        const uint32_t hb = ((d.opcode() | (d.fin() ? 0x80u : 0u)) & 0xffu) | (d.mask() ? 0x100u : 0u);
        const uint4 Hd = ws_header_words(len, hb, key);
        H.lo = t ? funnel16(z, Hd, 16u - t) : Hd;
        H.hi = t ? funnel16(Hd, z, 16u - t) : z;
        if (t) {
            // f - 1's last t payload bytes, masked with its key
            const uint64_t ts = a.payload_off + a.payload_size - t;       // their source
            uint64_t addr = reinterpret_cast<uint64_t>(src) + (ts & ~uint64_t(15));
            asm volatile("" : "+v"(addr));
            const uint8_t* sp = reinterpret_cast<const uint8_t*>(addr);
            const uint32_t tph = (uint32_t)(ts & 15u);
            uint4 T = ld16(sp);
            if (tph + t > 16) T = funnel16(T, ld16(sp + 16), tph);
            else if (tph) T = funnel16(T, z, tph);
            xor4(T, a.mask() ? rotr8(a.key(), (uint32_t)((a.payload_size - t) & 3u)) : 0u);
            H.lo = or4(H.lo, and4(T, byte_range(0, t)));
        }
    }
    const uint64_t dend = len < cap - dof ? dof + len : cap;
    // 1 KiB spans of the destination arena (dst is 16-byte aligned; spans
    // count from it) holding the frame
    const uint64_t s0 = (inrun ? H.c0 : dof) / (16 * kSpanChunks), s1 = (dend - 1) / (16 * kSpanChunks) + 1;
    const uint64_t ns = s1 - s0;
    const uint64_t used = (ns + kPieceSpans - 1) / kPieceSpans;
    // source phase against the 16-byte destination chunks: one per frame
    const uint32_t ph = (uint32_t)((so - dof) & 15u);
    // wave-uniform, so the span bases and buffer descriptors stay scalar (a
    // descriptor the compiler cannot prove uniform costs a readfirstlane loop
    // per store)
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // the key rotation of every 16-byte destination chunk: A - dof = -dof mod 4
    const uint32_t kr = rotr8(key, (uint32_t)((0u - (uint32_t)dof) & 3u));
    constexpr uint64_t kSpan = kSpanChunks * 16;
    // the aligned source blocks holding the frame's bytes, [xs0, xs1), and
    // the destination chunks the frame fills whole, [xd0, xd1)
    const int64_t xs0 = (int64_t)(so & ~uint64_t(15)), xs1 = (int64_t)((so + (dend - dof) + 15) & ~uint64_t(15));
    const uint64_t xd0 = inrun ? H.c0 : (dof + 15) & ~uint64_t(15), xd1 = dend & ~uint64_t(15);
    // virtual pieces p, p + pieces, ...: a frame larger than the caller's
    // max_payload_size (or a grid capped below 2^31 blocks) still gets every
    // chunk written
    for (uint64_t vp = p; vp < used; vp += pieces) {
        const uint64_t sb = s0 + ns * vp / used, se_piece = s0 + ns * (vp + 1) / used;
        // wave w streams a contiguous run of the piece's spans, [wb, se)
        const uint64_t m = se_piece - sb;
        const uint64_t wb = sb + m * wave / kWaves, se = sb + m * (wave + 1) / kWaves;
        const uint32_t cnt = (uint32_t)(se - wb);
        // descriptors over the run's source blocks and whole destination
        // chunks, clipped to the frame's (xor_run); lane l of span wb + k
        // reads the aligned source block at vb + 1024 k + 16 l
        const int64_t vb = (int64_t)so + (int64_t)(wb * kSpan) - (int64_t)dof - (int64_t)ph;
        const int64_t ve = vb + (int64_t)(cnt * kSpan) + 16;
        const int64_t ls = vb > xs0 ? vb : xs0, le = ve < xs1 ? ve : xs1;
        const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(src) + (le > ls ? ls : 0), 0,
                                                          le > ls ? (int)(le - ls) : 0, 0x00020000);
        const int32_t sd = (int32_t)(vb - ls);
        const uint64_t ds = wb * kSpan > xd0 ? wb * kSpan : xd0, de = se * kSpan < xd1 ? se * kSpan : xd1;
        const auto rd = __builtin_amdgcn_make_buffer_rsrc(dst + (de > ds ? ds : 0), 0,
                                                          de > ds ? (int)(de - ds) : 0, 0x00020000);
        const int32_t ddl = (int32_t)((int64_t)(wb * kSpan) - (int64_t)ds);
        if (inrun && wb * kSpan < ((dof + 15) & ~uint64_t(15)))
            xor_run<true, true>(rs, rd, sd, ddl, ph, kr, wb * kSpan, &H);
        else if (sd < 0 || ddl < 0)
            xor_run<true>(rs, rd, sd, ddl, ph, kr);
        else
            xor_run<false>(rs, rd, sd, ddl, ph, kr);
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

// A plain streaming device-to-device copy: the practical HBM ceiling the
// bench reports the codec against (copy_ceiling). The best bare-copy shape of
// tools/copy_probe.hip (profiles/r01_copy_probe.jsonl): `nt` loads and
// stores, 2 KiB per wave (2 x 16 B per lane), 4 workgroups per CU (an LDS
// reservation of 40,000 B), one chunk per lane per slot, no grid-stride.
constexpr uint32_t kCopyU = 2;

__global__ void __launch_bounds__(kThreads)
stream_copy_kernel(const u32x4* __restrict__ src, u32x4* __restrict__ dst, uint64_t n16)
{
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t base = (uint64_t(blockIdx.x) * kWaves + wave) * (kCopyU * 64) + (threadIdx.x & 63u);
    u32x4 a[kCopyU];
#pragma unroll
    for (uint32_t u = 0; u < kCopyU; ++u)
        if (base + u * 64 < n16) a[u] = __builtin_nontemporal_load(src + base + u * 64);
#pragma unroll
    for (uint32_t u = 0; u < kCopyU; ++u)
        if (base + u * 64 < n16) __builtin_nontemporal_store(a[u], dst + base + u * 64);
}

// The drop-in's frame service (cfws_internal.h): the XOR of a masked frame
// (co_ws_frame.c:93-97 / :234-242) without a launch per frame, for every
// calling thread of a process on one device. One workgroup of 16 waves:
//   * wave 0 dispatches: lane s polls slot s's request word with one
//     coalesced system-scope load per round (all 64 slots' words in 512
//     contiguous bytes of mapped host memory, s_sleep between rounds),
//     cuts each new frame into 4 KiB pieces and hands the pieces to idle
//     worker waves through LDS;
//   * waves 1-15 serve: a worker XORs its piece of its slot's buffer in
//     place (4 chunks per lane, all loads in flight at once, each a PCIe
//     round trip) and releases its stores at system scope; the worker that
//     finishes a frame's last piece writes the slot's done word. A 64 KiB
//     frame is 16 pieces on 15 workers; frames of several threads share
//     them.
// The kernel ends (a) when the stop word is set, (b) after idle_ticks of the
// wall clock without a request, or (c) after life_ticks in all, so that a
// stream sharing its hardware queue never waits behind it for longer
// (GPU_MAX_HW_QUEUES = 4: streams share queues); requests not yet taken stay
// posted for the next launch. After every wave has left the loop, thread 0
// writes the launch's generation to the exit word: from then on this kernel
// touches no slot, and the host may launch the next one.
constexpr uint32_t kServiceThreads = 1024;
constexpr uint32_t kServiceWorkers = kServiceThreads / 64 - 1;     // 15
constexpr uint32_t kServicePiece = 4096;           // bytes per piece: 4 chunks per lane
static_assert(kCfwsServiceSlots == 64, "wave 0's lanes poll the slots");

__device__ __forceinline__ uint64_t sys_load(const uint64_t* p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ void sys_store(uint64_t* p, uint64_t v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Piece p of a frame of n bytes at buf, XORed in place by one wave (chunk c
// at 16c: key phase 0 for every chunk); the frame's 0-15 tail bytes by the
// wave of its last piece.
__device__ __forceinline__ void service_xor_piece(uint8_t* buf, uint32_t n, uint32_t key, uint32_t p, uint32_t lane)
{
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");      // the frame's bytes, written by the host
    constexpr uint32_t kPer = kServicePiece / 16 / 64;
    const uint32_t nv = n / 16, c0 = p * (kServicePiece / 16);
    u32x4* b = reinterpret_cast<u32x4*>(buf);
    u32x4 v[kPer];
#pragma unroll
    for (uint32_t k = 0; k < kPer; ++k) {
        const uint32_t c = c0 + k * 64 + lane;
        if (c < nv) v[k] = b[c];
    }
#pragma unroll
    for (uint32_t k = 0; k < kPer; ++k) {
        const uint32_t c = c0 + k * 64 + lane;
        if (c < nv) b[c] = v[k] ^ key;
    }
    if ((n - 1) / kServicePiece == p && lane < n - nv * 16) {
        const uint32_t i = nv * 16 + lane;
        buf[i] = (uint8_t)(buf[i] ^ (key >> (8 * (i & 3u))));
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");      // the stores, before the piece counts as done
}

__global__ void __launch_bounds__(kServiceThreads)
dropin_service_kernel(uint64_t* ctl, uint8_t* bufs, uint64_t gen, uint64_t idle_ticks, uint64_t life_ticks)
{
    // per worker: its job (slot + 1 | piece << 8; 0 = idle), written by the
    // dispatcher, cleared by the worker; per slot: its request word and the
    // pieces not yet finished (the worker that takes it to 0 writes done)
    __shared__ uint32_t s_job[kServiceWorkers];
    __shared__ uint64_t s_word[kCfwsServiceSlots];
    __shared__ uint32_t s_left[kCfwsServiceSlots];
    __shared__ uint32_t s_exit;
    const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    if (threadIdx.x < kServiceWorkers) s_job[threadIdx.x] = 0;
    if (threadIdx.x == 0) s_exit = 0;
    __syncthreads();
    uint64_t* req = ctl + kCfwsServiceReqWord;
    uint64_t* done = ctl + kCfwsServiceDoneWord;
    if (wv == 0) {
        // lane s: the seq last taken for slot s (its done word at launch:
        // every earlier request of the slot was finished), and the pieces of
        // the slot's current frame still to hand out: [next, npieces)
        uint32_t handed = (uint32_t)(sys_load(&done[lane]) >> 48);
        uint32_t next = 0, npieces = 0;
        const uint64_t t_start = (uint64_t)wall_clock64();
        uint64_t t_last = t_start;
        for (;;) {
            const uint64_t now = (uint64_t)wall_clock64();
            const bool retiring = sys_load(&ctl[kCfwsServiceStopWord]) != 0 || now - t_start > life_ticks;
            // a slot takes a new request only when its frame is all handed
            // out; a retiring kernel takes none
            if (!retiring && next == npieces) {
                const uint64_t w = sys_load(&req[lane]);
                if ((uint32_t)(w >> 48) != handed) {
                    // its previous frame is finished: the host posts the next
                    // request only after that frame's done word
                    const uint32_t n = (uint32_t)((w >> 32) & 0xffffu) + 1u;
                    handed = (uint32_t)(w >> 48);
                    next = 0;
                    npieces = (n + kServicePiece - 1) / kServicePiece;
                    s_word[lane] = w;
                    s_left[lane] = npieces;
                    t_last = now;
                }
            }
            // hand out pieces, lowest slot first, to idle workers
            for (uint32_t k = 0; k < kServiceWorkers; ++k) {
                uint64_t want = __ballot(next < npieces);
                if (!want) break;
                if (__hip_atomic_load(&s_job[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != 0) continue;
                const uint32_t s = (uint32_t)__builtin_ctzll(want);
                const uint32_t p = (uint32_t)__shfl((int)next, (int)s);
                if (lane == 0)
                    __hip_atomic_store(&s_job[k], (s + 1) | p << 8, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                if (lane == s) ++next;
            }
            bool busy = __ballot(next < npieces) != 0;
            for (uint32_t k = 0; k < kServiceWorkers; ++k)
                busy |= __hip_atomic_load(&s_job[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != 0;
            // the workers finish the pieces they hold, and every handed-out
            // frame is completed, before the kernel ends
            if (!busy && (retiring || now - t_last > idle_ticks)) break;
            __builtin_amdgcn_s_sleep(2);
        }
        if (lane == 0) __hip_atomic_store(&s_exit, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    } else {
        const uint32_t me = wv - 1;
        for (;;) {
            const uint32_t j = __hip_atomic_load(&s_job[me], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (j == 0) {
                if (__hip_atomic_load(&s_exit, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)) break;
                __builtin_amdgcn_s_sleep(1);
                continue;
            }
            const uint32_t s = (j & 0xffu) - 1, p = j >> 8;
            const uint64_t w = s_word[s];
            const uint32_t n = (uint32_t)((w >> 32) & 0xffffu) + 1u;
            service_xor_piece(bufs + (uint64_t)s * kCfwsServiceMax, n, (uint32_t)w, p, lane);
            if (lane == 0) {
                // the last piece of the frame: its done word
                if (__hip_atomic_fetch_sub(&s_left[s], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP) == 1u)
                    sys_store(&done[s], w & 0xffff000000000000ull);
                __hip_atomic_store(&s_job[me], 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) sys_store(&ctl[kCfwsServiceExitWord], gen);
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
// handshake accept keys (co_ws_create_base64_accept_key,
// co_ws_http_extension.c:26-57): base64(SHA-1(key || GUID))
// ---------------------------------------------------------------------------
__constant__ char kWsGuid[37] = "258EAFA5-E914-47DA-95CA-C5AB0DC85B11";
__constant__ char kB64[65] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";

// A base64 character (RFC 4648 4, co_base64.c's table). The table lookup
// measured 10 % faster than computing the character by compares.
__device__ __forceinline__ uint32_t b64_char(uint32_t x) { return (uint8_t)kB64[x]; }

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

// One SHA-1 block (80 rounds over a 16-word schedule kept in registers).
// When w is a compile-time constant (the second block of a 24-byte key's
// message), the whole schedule folds into constants.
__device__ __forceinline__ void sha1_block(uint32_t (&st)[5], uint32_t (&w)[16])
{
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

// The GUID's bytes as big-endian words (it follows a 24-byte key at word 6).
__device__ __forceinline__ uint32_t guid_word(int j)
{
    constexpr char g[] = "258EAFA5-E914-47DA-95CA-C5AB0DC85B11";
    return (uint32_t)(uint8_t)g[4 * j] << 24 | (uint32_t)(uint8_t)g[4 * j + 1] << 16 |
           (uint32_t)(uint8_t)g[4 * j + 2] << 8 | (uint32_t)(uint8_t)g[4 * j + 3];
}

// One thread per connection: a connection storm's accept keys at once.
// A key of 24 bytes (every RFC 6455 client key: base64 of 16 bytes) takes
// the fast form: its SHA-1 input is 6 key words + 9 GUID words + the 0x80
// pad in block 0, and a constant block 1 (zeros and the 480-bit length).
// Any other length builds the message byte by byte.
#ifndef CFWS_ACCEPT_MIN_BLOCKS
#define CFWS_ACCEPT_MIN_BLOCKS 1
#endif
__global__ void __launch_bounds__(kThreads, CFWS_ACCEPT_MIN_BLOCKS)
ws_accept_kernel(const uint8_t* __restrict__ keys, const uint64_t* __restrict__ key_off, uint64_t n,
                 char* __restrict__ out)
{
    const uint64_t c = uint64_t(blockIdx.x) * kThreads + threadIdx.x;
    if (c >= n) return;
    const uint8_t* key = keys + key_off[c];
    char* o = out + CFWS_WS_ACCEPT_SLOT * c;
    if (key_off[c + 1] < key_off[c]) {
        // offsets out of order: no key, an empty slot (a wrapped length would
        // walk ~2^58 SHA-1 blocks)
        for (int b = 0; b < CFWS_WS_ACCEPT_SLOT; ++b) o[b] = 0;
        return;
    }
    const uint64_t L = key_off[c + 1] - key_off[c];
    uint32_t st[5] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u, 0xc3d2e1f0u};
    if (L == 24) {
        uint32_t w[16];
        if ((reinterpret_cast<uintptr_t>(key) & 7u) == 0) {
            // three 8-byte loads (keys packed 24 bytes apart stay aligned)
            const uint2* k8 = reinterpret_cast<const uint2*>(key);
#pragma unroll
            for (int t = 0; t < 3; ++t) {
                const uint2 v = k8[t];
                w[2 * t] = __builtin_bswap32(v.x);
                w[2 * t + 1] = __builtin_bswap32(v.y);
            }
        } else {
#pragma unroll
            for (int t = 0; t < 6; ++t)
                w[t] = (uint32_t)key[4 * t] << 24 | (uint32_t)key[4 * t + 1] << 16 |
                       (uint32_t)key[4 * t + 2] << 8 | (uint32_t)key[4 * t + 3];
        }
#pragma unroll
        for (int t = 6; t < 15; ++t) w[t] = guid_word(t - 6);
        w[15] = 0x80000000u;
        sha1_block(st, w);
        uint32_t w2[16];
#pragma unroll
        for (int t = 0; t < 15; ++t) w2[t] = 0;
        w2[15] = 60u * 8u;
        sha1_block(st, w2);
    } else {
        const uint64_t blocks = (L + 36 + 9 + 63) / 64;
        for (uint64_t b = 0; b < blocks; ++b) {
            uint32_t w[16];
#pragma unroll
            for (int t = 0; t < 16; ++t) {
                const uint64_t i = b * 64 + 4 * t;
                w[t] = accept_msg_byte(key, L, blocks, i) << 24 | accept_msg_byte(key, L, blocks, i + 1) << 16 |
                       accept_msg_byte(key, L, blocks, i + 2) << 8 | accept_msg_byte(key, L, blocks, i + 3);
            }
            sha1_block(st, w);
        }
    }
    // base64 of the 20 hash bytes: 6 full groups + 2 bytes -> 3 chars + '=';
    // the 32-byte slot written as words: 28 characters, the NUL, 3 zeros
    uint32_t ow[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
#pragma unroll
    for (int g = 0; g < 7; ++g) {
        uint32_t v = 0;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const int idx = 3 * g + j;
            const uint32_t byte = idx < 20 ? (st[idx >> 2] >> (8 * (3 - (idx & 3)))) & 0xffu : 0u;
            v = v << 8 | byte;
        }
        const uint32_t c3 = g < 6 ? b64_char(v & 63) : (uint32_t)'=';
        ow[g] = b64_char((v >> 18) & 63) | b64_char((v >> 12) & 63) << 8 | b64_char((v >> 6) & 63) << 16 |
                c3 << 24;
    }
    if ((reinterpret_cast<uintptr_t>(o) & 15u) == 0) {
        uint4* o16 = reinterpret_cast<uint4*>(o);
        o16[0] = make_uint4(ow[0], ow[1], ow[2], ow[3]);
        o16[1] = make_uint4(ow[4], ow[5], ow[6], ow[7]);
    } else {
#pragma unroll
        for (int b = 0; b < 29; ++b) o[b] = (char)(ow[b >> 2] >> (8 * (b & 3)));
    }
}

// ---------------------------------------------------------------------------
// receive-buffer frame indexing (co_ws_server.c:107-169)
// ---------------------------------------------------------------------------

// One connection per thread: the receive loop's walk over buf[begin, end).
// The walk is a chain of dependent header reads (one memory round trip per
// frame), so a connection is one thread and the parallelism is across
// connections (a server's event loop tick holds the receive buffers of
// many). The walk runs once: it counts, records consumed / stop, and keeps
// the first kIndexSlots starts in the connection's workspace slots (where
// they wait for the scan that places them) and where frame kIndexSlots
// starts. After the scan, index_place_kernel copies the kept starts to
// their places, and only connections with more frames than slots walk on
// from there (index_rest_kernel).
constexpr uint32_t kIndexSlots = 64;

__global__ void __launch_bounds__(kThreads)
index_walk_kernel(const uint8_t* __restrict__ buf, const uint64_t* __restrict__ begin,
                  const uint64_t* __restrict__ end, uint64_t n, uint64_t max_payload,
                  uint64_t* __restrict__ first, uint64_t* __restrict__ consumed,
                  int32_t* __restrict__ stop, uint64_t* __restrict__ slots, uint64_t* __restrict__ resume)
{
    const uint64_t c = uint64_t(blockIdx.x) * kThreads + threadIdx.x;
    if (c >= n) return;
    const uint64_t e = end[c];
    uint64_t p = begin[c];
    uint64_t k = 0, r = e;
    uint64_t* my = slots + c * kIndexSlots;
    int32_t st = CFWS_PARSE_COMPLETE;
    while (e > p) {
        if (e - p < 2) { st = CFWS_PARSE_MORE_DATA; break; }
        // the header's bytes (up to 14) in one round of independent loads,
        // parsed from registers: one memory round trip per hop, where a
        // byte-by-byte parse takes two (the length code, then the rest)
        uint32_t w[4];
        load_span16(buf + p, e - p < 14 ? (uint32_t)(e - p) : 14u, w);
        cfws_frame_desc_t d;
        st = parse_ws_header_regs(w, e - p, max_payload, d);
        if (st != CFWS_PARSE_COMPLETE) break;
        if (k < kIndexSlots) my[k] = p;
        else if (k == kIndexSlots) r = p;
        ++k;
        p += d.header_size + d.payload_size;
    }
    first[c] = k;
    consumed[c] = p;
    stop[c] = st;
    resume[c] = r;
}

// The kept starts to their places: thread (c, j) copies connection c's j-th
// start (j < kIndexSlots), after the scan turned the counts into firsts.
__global__ void __launch_bounds__(kThreads)
index_place_kernel(const uint64_t* __restrict__ first, const uint64_t* __restrict__ slots,
                   const uint64_t* __restrict__ total, uint64_t n, uint64_t* __restrict__ starts,
                   uint64_t cap)
{
    const uint64_t t = uint64_t(blockIdx.x) * kThreads + threadIdx.x;
    const uint64_t c = t / kIndexSlots, j = t % kIndexSlots;
    if (c >= n) return;
    const uint64_t next = c + 1 < n ? first[c + 1] : *total;
    const uint64_t k = next - first[c];
    if (j < k && first[c] + j < cap) starts[first[c] + j] = slots[t];
}

// Connections with more than kIndexSlots frames: the walk on from frame
// kIndexSlots, writing the rest of their starts in place.
__global__ void __launch_bounds__(kThreads)
index_rest_kernel(const uint8_t* __restrict__ buf, const uint64_t* __restrict__ end, uint64_t n,
                  uint64_t max_payload, const uint64_t* __restrict__ first,
                  const uint64_t* __restrict__ total, const uint64_t* __restrict__ resume,
                  uint64_t* __restrict__ starts, uint64_t cap)
{
    const uint64_t c = uint64_t(blockIdx.x) * kThreads + threadIdx.x;
    if (c >= n) return;
    const uint64_t next = c + 1 < n ? first[c + 1] : *total;
    if (next - first[c] <= kIndexSlots) return;
    const uint64_t e = end[c];
    uint64_t p = resume[c];
    for (uint64_t k = first[c] + kIndexSlots; k < next; ++k) {
        uint32_t w[4];
        load_span16(buf + p, e - p < 14 ? (uint32_t)(e - p) : 14u, w);
        cfws_frame_desc_t d;
        (void)parse_ws_header_regs(w, e - p, max_payload, d);   // COMPLETE: the first walk's frames
        if (k < cap) starts[k] = p;
        p += d.header_size + d.payload_size;
    }
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

extern "C" {

// [0, 64): header; then the scan partials, each connection's kIndexSlots
// kept starts and its resume position.
struct IndexLayout {
    uint64_t partials, slots, resume, bytes;
};

static IndexLayout index_layout(uint64_t n)
{
    IndexLayout L;
    uint64_t at = 64;
    L.partials = at; at = align_up(at + sizeof(uint64_t) * grid_for(n, kScanBlock), 256);
    L.slots = at; at = align_up(at + sizeof(uint64_t) * kIndexSlots * n, 256);
    L.resume = at; at = align_up(at + sizeof(uint64_t) * n, 256);
    L.bytes = at;
    return L;
}

size_t cfws_index_workspace_size(size_t n_conns)
{
    return (size_t)index_layout(n_conns).bytes;
}

int cfws_index_frames_batch(const void* d_buf, const uint64_t* d_begin, const uint64_t* d_end,
                            size_t n, uint64_t max_payload, uint64_t* d_starts, uint64_t cap,
                            uint64_t* d_first, uint64_t* d_consumed, int32_t* d_stop,
                            uint64_t* d_total, void* ws, size_t ws_size, void* stream)
{
    const CfwsPassScope pass_scope;
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
    const IndexLayout L = index_layout(n);
    uint64_t* slots = ws_ptr<uint64_t>(ws, L.slots);
    uint64_t* resume = ws_ptr<uint64_t>(ws, L.resume);
    const uint32_t g = grid_for(n, kThreads);
    index_walk_kernel<<<g, kThreads, 0, st>>>(buf, d_begin, d_end, n, max_payload, d_first, d_consumed,
                                              d_stop, slots, resume);
    if (int rc = run_scan(d_first, n, ws_ptr<uint64_t>(ws, L.partials), d_total, st)) return rc;
    if (cap) {
        index_place_kernel<<<grid_for(n * kIndexSlots, kThreads), kThreads, 0, st>>>(
            d_first, slots, d_total, n, d_starts, cap);
        index_rest_kernel<<<g, kThreads, 0, st>>>(buf, d_end, n, max_payload, d_first, d_total, resume,
                                                  d_starts, cap);
    }
    return launch_check("index");
}

int cfws_ws_accept_keys_batch(const void* d_keys, const uint64_t* d_key_off, size_t n,
                              char* d_accept, void* stream)
{
    const CfwsPassScope pass_scope;
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
    const CfwsPassScope pass_scope;
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
    const CfwsPassScope pass_scope;
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
    const CfwsPassScope pass_scope;
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

// The frames' partial first and last chunks: one thread per frame writes
// the frame's bytes of the (at most two) 16-byte destination chunks it
// shares with its neighbours, byte by byte, in a launch after the stream.
// (In the stream, the edge runs' byte stores held their workgroups' slots:
// mask 1.482 ms there against 1.404 + 0.012 here, profiles/r03_split_ab/
// edge_kernel/.)
template <bool kUnmask>
__global__ void __launch_bounds__(kThreads)
payload_edge_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                    const cfws_frame_desc_t* __restrict__ desc, const int32_t* __restrict__ status,
                    uint64_t n, uint64_t cap, uint32_t packed)
{
    const uint64_t f = uint64_t(blockIdx.x) * kThreads + threadIdx.x;
    if (f >= n) return;
    if (kUnmask && status && status[f] != CFWS_PARSE_COMPLETE) return;
    // the packed mask: bytes a boundary chunk written in-run carries are done
    const bool head_done = !kUnmask && packed && packed_inrun(desc, f, n, cap);
    const bool tail_done = !kUnmask && packed && packed_inrun(desc, f + 1, n, cap);
    const DescWords d = load_desc(desc, (uint32_t)f);
    const uint64_t len = d.payload_size;
    const uint64_t so = kUnmask ? d.wire_off + d.header_size() : d.payload_off;
    const uint64_t dof = kUnmask ? d.payload_off : d.wire_off + header_size_of(len, d.mask() != 0);
    const uint32_t key = d.mask() ? d.key() : 0u;
    if (len == 0 || dof >= cap) return;
    const uint64_t dend = len < cap - dof ? dof + len : cap;
    // [dof, first whole chunk) and [last whole chunk's end, dend)
    const uint64_t h1 = (dof + 15) & ~uint64_t(15), t0 = dend & ~uint64_t(15);
    const uint64_t ha = dof, hb = h1 < dend ? h1 : dend;
    const uint64_t ta = t0 > hb ? t0 : hb, tb = dend;
    if (!head_done)
        for (uint64_t x = ha; x < hb; ++x)
            dst[x] = src[so + (x - dof)] ^ (uint8_t)(key >> (8 * ((x - dof) & 3u)));
    if (!tail_done)
        for (uint64_t x = ta; x < tb; ++x)
            dst[x] = src[so + (x - dof)] ^ (uint8_t)(key >> (8 * ((x - dof) & 3u)));
}

// Pieces per frame for the split payload ops: enough workgroups to cover the
// largest frame (max_payload_size, at any alignment) in pieces of at most
// kPieceSpans 1 KiB spans, capped so the grid stays under 2^31 blocks (the
// kernel then strides over a frame's pieces).
uint32_t payload_pieces(size_t n, uint64_t max_payload_size)
{
    const uint64_t spans = max_payload_size / (16 * kSpanChunks) + 2;
    uint64_t pieces = (spans + kPieceSpans - 1) / kPieceSpans;
    if (pieces > 65536) pieces = 65536;
    while (pieces > 1 && pieces * n > 0x7fffffffull) pieces >>= 1;
    return (uint32_t)pieces;
}

template <bool kUnmask>
int launch_payload_xor(const void* src, void* dst, const cfws_frame_desc_t* d_desc,
                       const int32_t* d_status, size_t n, uint64_t max_payload_size, uint64_t cap,
                       void* stream, const char* what, uint32_t packed = 0)
{
    if (int rc = check_init()) return rc;
    if (n == 0 || cap == 0) return CFWS_OK;
    if (!src || !dst || !d_desc) return set_err(CFWS_ERROR_INVALID_ARGUMENT, "null pointer", hipSuccess);
    if (misaligned(src, dst))
        return set_err(CFWS_ERROR_INVALID_ARGUMENT, "arenas must be 16-byte aligned", hipSuccess);
    if (n > 0x7fffffffull) return set_err(CFWS_ERROR_INVALID_ARGUMENT, "too many frames", hipSuccess);
    const uint32_t pieces = payload_pieces(n, max_payload_size);
    payload_xor_kernel<kUnmask><<<(uint32_t)(n * pieces), kThreads, kUnmask ? CFWS_UNMASK_LDS : CFWS_MASK_LDS,
                                  static_cast<hipStream_t>(stream)>>>(
        static_cast<const uint8_t*>(src), static_cast<uint8_t*>(dst), d_desc, d_status, n, pieces, cap, packed);
    payload_edge_kernel<kUnmask><<<grid_for(n, kThreads), kThreads, 0, static_cast<hipStream_t>(stream)>>>(
        static_cast<const uint8_t*>(src), static_cast<uint8_t*>(dst), d_desc, d_status, n, cap, packed);
    return launch_check(what);
}

}  // namespace

CfwsPassEvents& cfws_internal_pass_events()
{
    thread_local CfwsPassEvents e = {nullptr, nullptr};
    return e;
}

namespace {
thread_local CfwsPassEvents t_call_pass = {nullptr, nullptr};   // the open call's pair
thread_local int t_pass_depth = 0;                               // open public calls
}  // namespace

CfwsPassScope::CfwsPassScope()
{
    if (t_pass_depth++ == 0) {
        CfwsPassEvents& pe = cfws_internal_pass_events();
        t_call_pass = pe;
        pe = {nullptr, nullptr};
    }
}

CfwsPassScope::~CfwsPassScope()
{
    if (--t_pass_depth == 0) t_call_pass = {nullptr, nullptr};
}

CfwsPassEvents cfws_internal_take_pass()
{
    const CfwsPassEvents e = t_call_pass;
    t_call_pass = {nullptr, nullptr};
    return e;
}

CfwsPassTimer::CfwsPassTimer(void* s) : e(cfws_internal_take_pass()), stream(s)
{
    if (e.start) (void)hipEventRecord(static_cast<hipEvent_t>(e.start), static_cast<hipStream_t>(stream));
}

CfwsPassTimer::~CfwsPassTimer()
{
    if (e.stop) (void)hipEventRecord(static_cast<hipEvent_t>(e.stop), static_cast<hipStream_t>(stream));
}

extern "C" {

int cfws_mask_batch(const void* d_payload, const cfws_frame_desc_t* d_desc, size_t n,
                    uint64_t max_payload_size, void* d_wire, uint64_t wire_capacity, void* stream)
{
    const CfwsPassScope pass_scope;
    return launch_payload_xor<false>(d_payload, d_wire, d_desc, nullptr, n, max_payload_size,
                                     wire_capacity, stream, "mask_batch");
}

int cfws_mask_batch_packed(const void* d_payload, const cfws_frame_desc_t* d_desc, size_t n,
                           uint64_t max_payload_size, void* d_wire, uint64_t wire_capacity, void* stream)
{
    const CfwsPassScope pass_scope;
    return launch_payload_xor<false>(d_payload, d_wire, d_desc, nullptr, n, max_payload_size,
                                     wire_capacity, stream, "mask_batch_packed", 1u);
}

int cfws_unmask_batch(const void* d_wire, const cfws_frame_desc_t* d_desc, const int32_t* d_status,
                      size_t n, uint64_t max_payload_size, void* d_payload,
                      uint64_t payload_capacity, void* stream)
{
    const CfwsPassScope pass_scope;
    return launch_payload_xor<true>(d_wire, d_payload, d_desc, d_status, n, max_payload_size,
                                    payload_capacity, stream, "unmask_batch");
}

int cfws_xor_mask(const void* d_src, void* d_dst, uint64_t n, uint32_t key, uint32_t phase,
                  void* stream)
{
    const CfwsPassScope pass_scope;
    if (int rc = check_init()) return rc;
    if (n == 0) return CFWS_OK;
    const uint64_t blocks = (n / 16 + kThreads - 1) / kThreads;
    const uint32_t g = (uint32_t)(blocks == 0 ? 1 : (blocks < 4096 ? blocks : 4096));
    xor_mask_kernel<<<g, kThreads, 0, static_cast<hipStream_t>(stream)>>>(
        static_cast<const uint8_t*>(d_src), static_cast<uint8_t*>(d_dst), n, key, phase & 3u);
    return launch_check("xor_mask");
}

int cfws_internal_service_launch(uint64_t* dev_ctl, uint8_t* dev_bufs, uint64_t gen, uint64_t idle_ticks,
                                 uint64_t life_ticks, void* stream)
{
    dropin_service_kernel<<<1, kServiceThreads, 0, static_cast<hipStream_t>(stream)>>>(dev_ctl, dev_bufs, gen,
                                                                                     idle_ticks, life_ticks);
    return launch_check("dropin_service");
}

int cfws_time_next_pass(void* start, void* stop)
{
    if ((start == nullptr) != (stop == nullptr))
        return set_err(CFWS_ERROR_INVALID_ARGUMENT, "start and stop events go together", hipSuccess);
    cfws_internal_pass_events() = {start, stop};
    return CFWS_OK;
}

int cfws_device_copy(const void* d_src, void* d_dst, uint64_t n, void* stream)
{
    const CfwsPassScope pass_scope;
    if (int rc = check_init()) return rc;
    if (n == 0) return CFWS_OK;
    if (misaligned(d_src, d_dst) || (n & 15u))
        return set_err(CFWS_ERROR_INVALID_ARGUMENT, "copy needs 16-byte aligned pointers and size",
                       hipSuccess);
    const uint64_t n16 = n / 16;
    const uint64_t per_block = uint64_t(kWaves) * kCopyU * 64;
    const uint64_t blocks = (n16 + per_block - 1) / per_block;
    if (blocks > 0x7fffffffull) return set_err(CFWS_ERROR_INVALID_ARGUMENT, "copy too large", hipSuccess);
    stream_copy_kernel<<<(uint32_t)blocks, kThreads, 40000, static_cast<hipStream_t>(stream)>>>(
        static_cast<const u32x4*>(d_src), static_cast<u32x4*>(d_dst), n16);
    return launch_check("device_copy");
}

int cfws_fill_splitmix(void* d_dst, uint64_t n, uint64_t seed, uint64_t byte_base, void* stream)
{
    const CfwsPassScope pass_scope;
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

