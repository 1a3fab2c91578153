// cfws_device.hip -- MI355X (gfx950) WebSocket frame codec: the batch C ABI
// (include/cfws.h: serialize / deserialize plan, execute, batch), its plan
// kernels and the single-launch small-batch kernels, and the library's
// error state. The streaming kernel and the device code the units share are
// in cfws_kernels.h; HTTP/2 in cfws_h2.hip; the smaller ops in cfws_ops.hip.
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
#include "cfws_kernels.h"

#include <mutex>

namespace cfws_rt {

thread_local char g_err[512] = "";

int set_err(int code, const char* what, hipError_t e)
{
    snprintf(g_err, sizeof g_err, "%s%s%s", what, e == hipSuccess ? "" : ": ",
             e == hipSuccess ? "" : hipGetErrorString(e));
    fprintf(stderr, "cfws: %s\n", g_err);
    return code;
}

// Every visible device is probed once, by whichever thread gets here first
// (std::call_once); afterwards the checks only read what the probe wrote.
// A call runs on the caller's current device, which must be a gfx950.
namespace {
std::once_flag g_probe_once;
int g_probe_rc = CFWS_OK;
int g_dev_count = 0;
uint64_t g_gfx950_mask = 0;        // bit d: device d is a gfx950 (d < 64)
char g_probe_msg[256] = "";

void probe_devices()
{
    int count = 0;
    hipError_t e = hipGetDeviceCount(&count);
    if (e != hipSuccess || count <= 0) {
        g_probe_rc = set_err(CFWS_ERROR_NO_DEVICE, "no HIP device", e);
        snprintf(g_probe_msg, sizeof g_probe_msg, "%s", g_err);
        return;
    }
    g_dev_count = count;
    char first_arch[64] = "";
    for (int d = 0; d < count && d < 64; ++d) {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, d) != hipSuccess) continue;
        if (d == 0) snprintf(first_arch, sizeof first_arch, "%s", prop.gcnArchName);
        if (strncmp(prop.gcnArchName, "gfx950", 6) == 0) g_gfx950_mask |= uint64_t(1) << d;
    }
    if (g_gfx950_mask == 0) {
        snprintf(g_probe_msg, sizeof g_probe_msg, "no gfx950 device (device 0 is %s)", first_arch);
        g_probe_rc = set_err(CFWS_ERROR_NO_DEVICE, g_probe_msg, hipSuccess);
    }
}
}  // namespace

int check_device(int dev)
{
    std::call_once(g_probe_once, probe_devices);
    if (g_probe_rc != CFWS_OK) {
        snprintf(g_err, sizeof g_err, "%s", g_probe_msg);
        return g_probe_rc;
    }
    if (dev < 0 || dev >= g_dev_count || dev >= 64 || !((g_gfx950_mask >> dev) & 1)) {
        snprintf(g_err, sizeof g_err, "device %d is not a usable gfx950 device (%d visible)", dev, g_dev_count);
        return CFWS_ERROR_NO_DEVICE;
    }
    return CFWS_OK;
}

int check_init()
{
    std::call_once(g_probe_once, probe_devices);
    if (g_probe_rc != CFWS_OK) return check_device(0);
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return set_err(CFWS_ERROR_NO_DEVICE, "hipGetDevice", e);
    return check_device(dev);
}

int launch_check(const char* what)
{
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? CFWS_OK : set_err(CFWS_ERROR_HIP, what, e);
}

}  // namespace cfws_rt

namespace {

using cfws_rt::g_err;

// A/B knob: dynamic LDS the WS plan kernels reserve (CFWS_PLAN_LDS; default 0)
uint32_t plan_lds_bytes()
{
    static const int64_t v = env_knob("CFWS_PLAN_LDS", 0);
    return (uint32_t)(v > 65536 ? 65536 : v);
}

// Both reassembly passes' edge chunks in one launch of their own (the
// CFWS_EDGE_SPLIT=1 form; by default pass 0's streaming launch carries them).
__global__ void __launch_bounds__(kEdgeThreads)
edge_reasm_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                  const cfws_frame_desc_t* __restrict__ desc, const int32_t* __restrict__ status,
                  const uint64_t* __restrict__ offs0, const uint64_t* __restrict__ offs1,
                  const uint64_t* __restrict__ hdr, uint64_t capacity, uint32_t n_frames)
{
    const uint64_t t = uint64_t(blockIdx.x) * kEdgeThreads + threadIdx.x;
    if (edge_thread_frame(t) >= n_frames) return;
    reasm_edge_frame(src, dst, desc, status, offs0, offs1, hdr, capacity, n_frames, edge_thread_frame(t),
                     edge_thread_part(t));
}

// ---------------------------------------------------------------------------
// WS plan kernels
// ---------------------------------------------------------------------------
// WS serialize's in-region edge chunks (general_region_ser_edges) need every
// frame's payload at 80..2,000 bytes and 16-aligned in the payload arena.
__device__ __forceinline__ bool ser_inreg_frame_ok(uint64_t len, uint32_t payload_off_lo)
{
    return len >= 80 && len <= 2000 && (payload_off_lo & 15u) == 0;
}

__global__ void __launch_bounds__(kThreads)
serialize_plan_reduce_kernel(cfws_frame_desc_t* __restrict__ desc, uint64_t* __restrict__ vals,
                             uint64_t n, uint64_t* __restrict__ partials, uint32_t* __restrict__ inreg_flag)
{
    __shared__ uint64_t s_wave[kWaves];
    if (blockIdx.x == 0 && threadIdx.x == 0) *inreg_flag = 0u;    // the apply kernel ORs into it
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
                            uint32_t* __restrict__ map, uint64_t* __restrict__ user_total,
                            uint32_t* __restrict__ inreg_flag)
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
    bool bad = false;
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
            bad |= !ser_inreg_frame_ok(desc[f].payload_size, (uint32_t)desc[f].payload_off);
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
    if (__syncthreads_or(bad) && threadIdx.x == 0) atomicOr(inreg_flag, 1u);
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

// Single-pass plans (plan_lookback): the reduce and apply kernels above in
// one launch, for plans of more than kSelfScanBlocks blocks (no scan launch,
// no second read of the sizes). A block takes kThreads x kSingleItems frames,
// each wave a contiguous kSingleItems x 64 of them (item k, lane l: frame k * 64 + l of
// the wave's run, so every load is coalesced): the look-back's cost is a
// device-scope round trip per 64 blocks, and 16 K blocks of 256 frames spent
// 232 us on it for 4 M frames. With a capacity cut the region map clips at
// the capacity itself: a frame's range ends at or below the grand total, so
// that is the same clip as at min(total, capacity).
#ifndef CFWS_SINGLE_ITEMS_SER
#define CFWS_SINGLE_ITEMS_SER 16
#endif
#ifndef CFWS_SINGLE_ITEMS_DESER
#define CFWS_SINGLE_ITEMS_DESER 8
#endif
constexpr int kSingleItemsSer = CFWS_SINGLE_ITEMS_SER;
constexpr int kSingleItemsDeser = CFWS_SINGLE_ITEMS_DESER;

// The flag word the serialize plan leaves for the execute: 0 = in-region
// edges (the single-pass plan found every frame qualifying), else not. It
// sits after the single-pass plan's ticket and block flags, inside the
// look area (>= 64 words, and >= n / 256 + 1).
uint32_t* ser_inreg_flag(const WsLayout& L, const void* ws, uint64_t n)
{
    return ws_ptr<uint32_t>(ws, L.look) + grid_for(n, uint64_t(kThreads) * kSingleItemsSer) + 1;
}

// CFWS_SER_INREG=0: the edge workgroups write every serialize edge chunk
// (A/B knob).
bool ser_inreg()
{
    static const bool v = env_knob("CFWS_SER_INREG", 1) != 0;
    return v;
}

// The wave-exclusive prefixes of v[k] in frame order (k-major), and the
// wave's total.
template <int kSingleItems>
__device__ __forceinline__ uint64_t wave_scan_items(const uint64_t (&v)[kSingleItems], uint64_t (&ex)[kSingleItems])
{
    const uint32_t lane = threadIdx.x & 63u;
    uint64_t run = 0;
#pragma unroll
    for (int k = 0; k < kSingleItems; ++k) {
        uint64_t inc = v[k];
#pragma unroll
        for (uint32_t o = 1; o < 64; o <<= 1) {
            const uint64_t y = __shfl_up(inc, o, 64);
            if (lane >= o) inc += y;
        }
        ex[k] = run + inc - v[k];
        run += __shfl(inc, 63, 64);
    }
    return run;
}

// This block's exclusive prefix from the look-back, plus each wave's offset
// within the block (s_wave: the waves' totals).
__device__ __forceinline__ uint64_t single_block_prefix(uint32_t b, uint64_t wave_total, uint64_t* s_wave,
                                                        uint64_t* s_prefix, uint32_t* look, uint64_t* agg,
                                                        uint64_t* incl)
{
    const uint32_t wid = threadIdx.x >> 6;
    if ((threadIdx.x & 63u) == 0) s_wave[wid] = wave_total;
    __syncthreads();
    uint64_t before = 0, all = 0;
#pragma unroll
    for (uint32_t w = 0; w < kWaves; ++w) {
        if (w < wid) before += s_wave[w];
        all += s_wave[w];
    }
    if (wid == 0) {
        const uint64_t pre = plan_lookback(b, all, look + 1, agg, incl);
        if (threadIdx.x == 0) *s_prefix = pre;
    }
    __syncthreads();
    return *s_prefix + before;
}

__global__ void __launch_bounds__(kThreads)
serialize_plan_single_kernel(cfws_frame_desc_t* __restrict__ desc, uint64_t* __restrict__ offs, uint64_t n,
                             uint32_t* __restrict__ look, uint64_t* __restrict__ agg,
                             uint64_t* __restrict__ incl, uint64_t* __restrict__ hdr, uint64_t capacity,
                             uint32_t* __restrict__ map, uint64_t* __restrict__ user_total)
{
    __shared__ uint64_t s_wave[kWaves];
    __shared__ uint64_t s_prefix;
    __shared__ uint32_t s_bid;
    constexpr int kSingleItems = kSingleItemsSer;
    static_assert(kSingleItems <= 16, "4-bit header sizes in one word");
    constexpr uint64_t kSingleFrames = uint64_t(kThreads) * kSingleItems;
    const uint32_t b = plan_ticket(look, &s_bid);
    const uint64_t f0 = uint64_t(b) * kSingleFrames + uint64_t(threadIdx.x >> 6) * (64 * kSingleItems) +
                        (threadIdx.x & 63u);
    uint64_t v[kSingleItems], ex[kSingleItems];
    uint64_t hsp = 0;                                  // 4 bits per item: header sizes (2..14)
    // every item's loads in one round (frames past n read frame n - 1's:
    // a branch per item made it a round trip per item)
    uint64_t len[kSingleItems];
    uint32_t msk[kSingleItems];
#pragma unroll
    for (int k = 0; k < kSingleItems; ++k) {
        const uint64_t f = f0 + uint64_t(k) * 64, fc = f < n ? f : n - 1;
        len[k] = desc[fc].payload_size;
        msk[k] = desc[fc].mask;
    }
    bool bad = false;                                  // a frame outside ser_inreg_frame_ok
#pragma unroll
    for (int k = 0; k < kSingleItems; ++k) {
        const uint64_t f = f0 + uint64_t(k) * 64;
        const uint32_t hs = header_size_of(len[k], msk[k] != 0);
        hsp |= uint64_t(hs) << (4 * k);
        v[k] = f < n ? hs + len[k] : 0;
    }
    const uint64_t pre = single_block_prefix(b, wave_scan_items(v, ex), s_wave, &s_prefix, look, agg, incl);
#pragma unroll
    for (int k = 0; k < kSingleItems; ++k) {
        const uint64_t f = f0 + uint64_t(k) * 64;
        if (f >= n) continue;
        const uint64_t run = pre + ex[k];
        offs[f] = run;
        const uint32_t hs = (uint32_t)((hsp >> (4 * k)) & 15u);
        // (the payload offset read here, not with the sizes: 276 VGPRs there)
        bad |= !ser_inreg_frame_ok(v[k] - hs, (uint32_t)desc[f].payload_off);
        // both descriptor fields at once, so the line is written back once
        desc[f].wire_off = run;
        desc[f].header_size = (uint8_t)hs;
        map_range(run, run + v[k], f, capacity, map);
        if (f == n - 1) {
            const uint64_t g = run + v[k], t = g < capacity ? g : capacity;
            map[(t + kRegion - 1) / kRegion] = (uint32_t)f;
            hdr[0] = t;
            hdr[3] = g;
            if (user_total) *user_total = g;
        }
    }
    // in-region edges only when every frame qualifies (look[gridDim.x + 1],
    // zeroed with the tickets)
    if (__syncthreads_or(bad) && threadIdx.x == 0) atomicOr(look + gridDim.x + 1, 1u);
}

// deserialize_plan_reduce_kernel + deserialize_plan_apply_kernel in one
// launch, without reassembly (its control-frame pass starts at the data
// pass's grand total, which no block knows before the last one). The
// descriptors are written as parsed, their payload offsets (and the
// capacity rule's status) once the offsets are known.
__global__ void __launch_bounds__(kThreads)
deserialize_plan_single_kernel(const uint8_t* __restrict__ wire, uint64_t wire_size_all,
                               const uint64_t* __restrict__ index, const uint64_t* __restrict__ ends,
                               uint64_t n, uint64_t max_payload, uint64_t align,
                               cfws_frame_desc_t* __restrict__ desc, int32_t* __restrict__ status,
                               uint64_t* __restrict__ offs, uint32_t* __restrict__ look,
                               uint64_t* __restrict__ agg, uint64_t* __restrict__ incl,
                               uint64_t* __restrict__ hdr, uint64_t capacity, uint32_t* __restrict__ map,
                               uint64_t* __restrict__ user_total)
{
    __shared__ uint64_t s_wave[kWaves];
    __shared__ uint64_t s_prefix;
    __shared__ uint32_t s_bid;
    constexpr int kSingleItems = kSingleItemsDeser;
    constexpr uint64_t kSingleFrames = uint64_t(kThreads) * kSingleItems;
    const uint32_t b = plan_ticket(look, &s_bid);
    const uint64_t f0 = uint64_t(b) * kSingleFrames + uint64_t(threadIdx.x >> 6) * (64 * kSingleItems) +
                        (threadIdx.x & 63u);
    // each descriptor is written once, whole, with its offset: the parsed
    // fields wait in registers (wire_off, payload_size, the last word)
    uint64_t v[kSingleItems], ex[kSingleItems], wo[kSingleItems], ps[kSingleItems], w3[kSingleItems];
    int32_t sts[kSingleItems];
    // the loads of all items first, in two rounds (starts and ends, then
    // every header's two blocks, clamped to the buffer's last whole block
    // instead of branching on the bytes available), then the parses: a
    // header per round trip serialized the wave (24 round trips for 8
    // items). Frames past n load frame n - 1's entries: no branch in a round.
    uint64_t sx[kSingleItems], sz[kSingleItems];
#pragma unroll
    for (int k = 0; k < kSingleItems; ++k) {
        const uint64_t f = f0 + uint64_t(k) * 64, fc = f < n ? f : n - 1;
        sx[k] = index[fc];
        sz[k] = wire_size_all;
    }
    if (ends) {
#pragma unroll
        for (int k = 0; k < kSingleItems; ++k) {
            const uint64_t f = f0 + uint64_t(k) * 64, fc = f < n ? f : n - 1;
            const uint64_t e = ends[fc];
            sz[k] = e < wire_size_all ? e : wire_size_all;
        }
    }
    // a 16-byte-aligned buffer: every header from the two aligned 16-byte
    // blocks that hold it (2 loads per header instead of 5 dwords); a header
    // whose second block is not a whole block of the buffer (the last 32
    // bytes) is parsed by the loads of parse_ws_header instead
    const bool b16 = ((uintptr_t)wire & 15u) == 0 && wire_size_all >= 32;
    const uint64_t lastb = (wire_size_all - 16) & ~uint64_t(15);
    uint4 hb0[kSingleItems], hb1[kSingleItems];
    if (b16) {
#pragma unroll
        for (int k = 0; k < kSingleItems; ++k) {
            const uint64_t a = sx[k] & ~uint64_t(15);
            hb0[k] = ld16(wire + (a < lastb ? a : lastb));
            hb1[k] = ld16(wire + (a + 16 < lastb ? a + 16 : lastb));
        }
    }
#pragma unroll
    for (int k = 0; k < kSingleItems; ++k) {
        const uint64_t f = f0 + uint64_t(k) * 64;
        v[k] = 0;
        if (f < n) {
            const uint64_t wire_size = sz[k];
            cfws_frame_desc_t d;
            const uint64_t s0 = sx[k], a = s0 & ~uint64_t(15);
            if (b16 && a + 16 <= lastb) {
                const uint64_t avail = s0 <= wire_size ? wire_size - s0 : 0;
                const uint4 W = funnel16(hb0[k], hb1[k], (uint32_t)(s0 - a));
                const uint32_t w[4] = {W.x, W.y, W.z, W.w};
                sts[k] = parse_ws_header_regs(w, avail, max_payload, d);
                d.wire_off = s0;
            } else {
                sts[k] = parse_ws_header(wire, wire_size, s0, max_payload, d);
            }
            wo[k] = d.wire_off;
            ps[k] = d.payload_size;
            w3[k] = (uint64_t)d.mask_key | (uint64_t)d.fin << 32 | (uint64_t)d.opcode << 40 |
                    (uint64_t)d.mask << 48 | (uint64_t)d.header_size << 56;
            const uint64_t len = (sts[k] == CFWS_PARSE_COMPLETE) ? d.payload_size : 0;
            v[k] = (len + align - 1) & ~(align - 1);
        }
    }
    const uint64_t pre = single_block_prefix(b, wave_scan_items(v, ex), s_wave, &s_prefix, look, agg, incl);
#pragma unroll
    for (int k = 0; k < kSingleItems; ++k) {
        const uint64_t f = f0 + uint64_t(k) * 64;
        if (f >= n) continue;
        const uint64_t run = pre + ex[k];
        offs[f] = run;
        uint64_t* q = reinterpret_cast<uint64_t*>(desc) + 4 * f;
        q[0] = run;
        q[1] = wo[k];
        q[2] = ps[k];
        q[3] = w3[k];
        // the capacity rule (co_ws_frame.c:216-223), as deserialize_plan_apply_kernel
        int32_t st = sts[k];
        if (st == CFWS_PARSE_COMPLETE && ps[k] > 0 && run + ps[k] > capacity) st = CFWS_ERROR_OUT_OF_MEMORY;
        status[f] = st;
        map_range(run, run + v[k], f, capacity, map);
        if (f == n - 1) {
            const uint64_t g = run + v[k], t = g < capacity ? g : capacity;
            map[(t + kRegion - 1) / kRegion] = (uint32_t)f;
            hdr[0] = t;
            hdr[1] = 0;
            hdr[2] = t;
            hdr[3] = g;
            if (user_total) *user_total = t;
        }
    }
}

// Single-pass plans above kSelfScanBlocks blocks (CFWS_PLAN_SINGLE=0: the
// reduce / scan / apply launches everywhere; A/B knob).
bool plan_single()
{
    static const bool v = env_knob("CFWS_PLAN_SINGLE", 1) != 0;
    return v;
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

// The single-launch small-batch path (CFWS_SMALL=0 turns it off: plan +
// execute for every batch, for A/B and for tests of both paths).
bool small_path()
{
    static const bool v = env_knob("CFWS_SMALL", 1) != 0;
    return v;
}

// Workgroups of a small-batch launch: kSmallChunksPerThread output chunks
// per thread at the capacity's size.
uint32_t small_grid(uint64_t cap)
{
    const uint64_t per = uint64_t(kThreads) * kSmallChunksPerThread * 16;
    return grid_for(cap, per);
}

}  // namespace

namespace cfws_rt {

int deserialize_plan_impl(const void* d_wire, uint64_t wire_size, const uint64_t* d_index,
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
    if (!reasm && nb > kSelfScanBlocks && plan_single()) {
        uint32_t* look = ws_ptr<uint32_t>(ws, L.look);
        const uint32_t sb = grid_for(n, uint64_t(kThreads) * kSingleItemsDeser);
        if (hipMemsetAsync(look, 0, 4 * (uint64_t(sb) + 1), st) != hipSuccess)
            return launch_check("deserialize_plan");
        deserialize_plan_single_kernel<<<sb, kThreads, 0, st>>>(
            static_cast<const uint8_t*>(d_wire), wire_size, d_index, d_ends, n, max_payload, align, d_desc,
            d_status, offs0, look, part0, part1, hdr, cap, ws_ptr<uint32_t>(ws, L.map[0]), d_total);
        return launch_check("deserialize_plan");
    }
    deserialize_plan_reduce_kernel<<<nb, kThreads, plan_lds_bytes(), st>>>(
        static_cast<const uint8_t*>(d_wire), wire_size, d_index, d_ends, n, max_payload, align, reasm,
        d_desc, d_status, offs0, offs1, part0, part1);
    const uint32_t self_scan = nb <= kSelfScanBlocks ? 1u : 0u;
    if (!self_scan)
        scan_partials2_kernel<<<reasm ? 2 : 1, kThreads, 0, st>>>(part0, part1, nb, hdr + 3, hdr + 4);
    deserialize_plan_apply_kernel<<<nb, kThreads, plan_lds_bytes(), st>>>(
        d_desc, d_status, offs0, offs1, n, part0, part1, nb, self_scan, hdr, cap, reasm,
        ws_ptr<uint32_t>(ws, L.map[0]), ws_ptr<uint32_t>(ws, L.map[1]), d_total);
    return launch_check("deserialize_plan");
}

}  // namespace cfws_rt

uint64_t cfws_internal_grand_total_offset() { return ws_layout(0, 0).hdr + 3 * sizeof(uint64_t); }

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
extern "C" {

int cfws_init(void) { return check_init(); }
int cfws_init_device(int device) { return cfws_rt::check_device(device); }
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
    if (!self_scan && plan_single()) {
        uint32_t* look = ws_ptr<uint32_t>(ws, L.look);
        const uint32_t sb = grid_for(n, uint64_t(kThreads) * kSingleItemsSer);
        if (hipMemsetAsync(look, 0, 4 * (uint64_t(sb) + 2), st) != hipSuccess)
            return launch_check("serialize_plan");
        serialize_plan_single_kernel<<<sb, kThreads, 0, st>>>(d_desc, offs, n, look, partials,
                                                              ws_ptr<uint64_t>(ws, L.partials[1]), hdr, cap,
                                                              ws_ptr<uint32_t>(ws, L.map[0]), d_total);
        return launch_check("serialize_plan");
    }
    serialize_plan_reduce_kernel<<<nb, kThreads, plan_lds_bytes(), st>>>(d_desc, offs, n, partials,
                                                                         ser_inreg_flag(L, ws, n));
    if (!self_scan) scan_partials_kernel<<<1, kThreads, 0, st>>>(partials, nb, hdr + 3);
    serialize_plan_apply_kernel<<<nb, kThreads, plan_lds_bytes(), st>>>(d_desc, offs, n, partials, nb, self_scan,
                                                        hdr, cap, ws_ptr<uint32_t>(ws, L.map[0]),
                                                        d_total, ser_inreg_flag(L, ws, n));
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
                          static_cast<hipStream_t>(stream), 0, true, false,
                          ser_inreg() ? ser_inreg_flag(L, ws, n) : nullptr);
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
        // every edge chunk of both passes is disjoint from the body chunks
        // either streaming pass writes, so pass 0's launch carries them all
        const bool split = edge_split();
        launch_pass<kModeDeser>(L, 0, d_wire, d_payload, d_desc, d_status, ws, cap, n, kClassData, st,
                                0, !split, !split);
        launch_pass<kModeDeser>(L, 1, d_wire, d_payload, d_desc, d_status, ws, cap, n, kClassControl,
                                st, 0, false);
        if (split)
            edge_reasm_kernel<<<grid_for(edge_threads(n), kEdgeThreads), kEdgeThreads, 0, st>>>(
                static_cast<const uint8_t*>(d_wire), static_cast<uint8_t*>(d_payload), d_desc,
                d_status, ws_ptr<const uint64_t>(ws, L.offs[0]), ws_ptr<const uint64_t>(ws, L.offs[1]),
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

}  // extern "C"
