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
#include <type_traits>

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
// frame's payload at 80..CFWS_SER_INREG_MAX bytes and 16-aligned in the payload
// arena (3,584: 2 to 3.5 KiB frames 1.5-8 % faster in-region, 4 KiB 5 % slower;
// profiles/r04/inreg_bound_ab/).
#ifndef CFWS_SER_INREG_MAX
#define CFWS_SER_INREG_MAX 3584
#endif
// general_region_ser_edges carries a header as two words: 16-bit lengths
static_assert(CFWS_SER_INREG_MAX <= 65535, "in-region headers are at most 8 bytes");
__device__ __forceinline__ bool ser_inreg_frame_ok(uint64_t len, uint32_t payload_off_lo)
{
    return len >= 80 && len <= CFWS_SER_INREG_MAX && (payload_off_lo & 15u) == 0;
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
// The serialize plan reads every descriptor whole and writes it back whole
// (8 frames per thread for the registers): a descriptor line then leaves L2
// fully written, and the payload offset is not fetched a second time. The
// round-4 A/B against reading the sizes first and writing two fields after
// the look-back (16 frames per thread): at 16 M x 256 B 0.54 GB read per plan
// instead of 1.08, the same 0.68 GB written, the same time (328 against
// 331 us; profiles/r04/plan_ab.json); with the packed look-back, the two-field
// form at 4, 8 or 16 frames per thread (down to 122 VGPRs, 4 waves per SIMD)
// was 0.2-1.9 % slower per step at 256 B and 1 KiB (profiles/r04/plan_lite_ab.json).
#ifndef CFWS_SINGLE_ITEMS_SER
#define CFWS_SINGLE_ITEMS_SER 8
#endif
#ifndef CFWS_SINGLE_ITEMS_DESER
#define CFWS_SINGLE_ITEMS_DESER 8
#endif
constexpr int kSingleItemsSer = CFWS_SINGLE_ITEMS_SER;
constexpr int kSingleItemsDeser = CFWS_SINGLE_ITEMS_DESER;
// Threads per block of the single-pass plans (serialize, deserialize) and
// of the fused deserialize. A block's look-back waits on the inclusive
// frontier, which advances 64 blocks per poll round trip (about 2.3 us
// under load: tools/plan_trace.py timed the serialize plan's blocks at
// 5.2 us of loads, 6.6 us of look-back, 4.0 us of stores, 465 resident),
// so a block of more frames moves the frontier further per round trip. On
// 16 M x 256 B: serialize plan 305 -> 274 us at 512 threads (1,024: 128
// VGPRs, spills); fused receive 1.95 -> 1.79 ms at 1,024 threads (512:
// 1.87); step 3.84-3.87 -> 3.65-3.66 ms. 1 KiB and 3 KiB unchanged, and the
// receive plan at 512 / 1,024 threads too (profiles/r05/plan_blocks_ab/).
#ifndef CFWS_SER_PLAN_THREADS
#define CFWS_SER_PLAN_THREADS 512
#endif
#ifndef CFWS_DE_PLAN_THREADS
#define CFWS_DE_PLAN_THREADS 256
#endif
#ifndef CFWS_FUSED_THREADS
#define CFWS_FUSED_THREADS 1024
#endif
constexpr int kSerPlanThreads = CFWS_SER_PLAN_THREADS;
constexpr int kDePlanThreads = CFWS_DE_PLAN_THREADS;
constexpr int kFusedThreads = CFWS_FUSED_THREADS;

// The flag word the serialize plan leaves for the execute: 0 = in-region
// edges (the single-pass plan found every frame qualifying), else not. It
// sits after the single-pass plan's ticket and block flags, inside the
// look area (>= 64 words, and >= n / 256 + 1).
uint32_t* ser_inreg_flag(const WsLayout& L, const void* ws, uint64_t n)
{
    return ws_ptr<uint32_t>(ws, L.look) + grid_for(n, uint64_t(kSerPlanThreads) * kSingleItemsSer) + 1;
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
template <int kNW = kWaves>
__device__ __forceinline__ uint64_t single_block_prefix(uint32_t b, uint64_t wave_total, uint64_t* s_wave,
                                                        uint64_t* s_prefix, uint32_t* look)
{
    const uint32_t wid = threadIdx.x >> 6;
    if ((threadIdx.x & 63u) == 0) s_wave[wid] = wave_total;
    __syncthreads();
    uint64_t before = 0, all = 0;
#pragma unroll
    for (uint32_t w = 0; w < (uint32_t)kNW; ++w) {
        if (w < wid) before += s_wave[w];
        all += s_wave[w];
    }
    if (wid == 0) {
        const uint64_t pre = plan_lookback(b, all, look_states(look));
        if (threadIdx.x == 0) *s_prefix = pre;
    }
    __syncthreads();
    return *s_prefix + before;
}

// CFWS_PLAN_TRACE builds (tools/plan_trace.py; never the shipped library):
// per block ticket, wall-clock stamps at the ticket, after the loads and
// the block scan, after the look-back, at the end.
#ifndef CFWS_PLAN_TRACE
#define CFWS_PLAN_TRACE 0
#endif
#if CFWS_PLAN_TRACE
constexpr uint32_t kTraceBlocks = 1u << 16;
__device__ uint64_t g_plan_trace[kTraceBlocks][4];
#define PLAN_STAMP(b, i)                                                                       \
    do {                                                                                       \
        if (threadIdx.x == 0 && (b) < kTraceBlocks) g_plan_trace[(b)][(i)] = wall_clock64();   \
    } while (0)
#else
#define PLAN_STAMP(b, i) do {} while (0)
#endif

template <int kBT>
__global__ void __launch_bounds__(kBT)
serialize_plan_single_kernel(cfws_frame_desc_t* __restrict__ desc, uint64_t* __restrict__ offs, uint64_t n,
                             uint32_t* __restrict__ look, uint64_t* __restrict__ hdr, uint64_t capacity,
                             uint32_t* __restrict__ map, uint64_t* __restrict__ user_total)
{
    __shared__ uint64_t s_wave[kBT / 64];
    __shared__ uint64_t s_prefix;
    __shared__ uint32_t s_bid;
    constexpr int kSingleItems = kSingleItemsSer;
    static_assert(kSingleItems <= 16, "4-bit header sizes in one word");
    constexpr uint64_t kSingleFrames = uint64_t(kBT) * kSingleItems;
    const uint32_t b = plan_ticket(look, &s_bid);
    PLAN_STAMP(b, 0);
    const uint64_t f0 = uint64_t(b) * kSingleFrames + uint64_t(threadIdx.x >> 6) * (64 * kSingleItems) +
                        (threadIdx.x & 63u);
    uint64_t v[kSingleItems], ex[kSingleItems];
    uint64_t hsp = 0;                                  // 4 bits per item: header sizes (2..14)
    // every item's loads in one round (frames past n read frame n - 1's:
    // a branch per item made it a round trip per item)
    uint64_t len[kSingleItems];
    uint32_t msk[kSingleItems];
    bool bad = false;                                  // a frame outside ser_inreg_frame_ok
    uint64_t poff[kSingleItems], w3[kSingleItems];
#pragma unroll
    for (int k = 0; k < kSingleItems; ++k) {
        const uint64_t f = f0 + uint64_t(k) * 64, fc = f < n ? f : n - 1;
        const DescWords d = load_desc(desc, (uint32_t)fc);
        poff[k] = d.payload_off;
        len[k] = d.payload_size;
        w3[k] = d.w3;
        msk[k] = d.mask();
    }
#pragma unroll
    for (int k = 0; k < kSingleItems; ++k)
        bad |= f0 + uint64_t(k) * 64 < n && !ser_inreg_frame_ok(len[k], (uint32_t)poff[k]);
#pragma unroll
    for (int k = 0; k < kSingleItems; ++k) {
        const uint64_t f = f0 + uint64_t(k) * 64;
        const uint32_t hs = header_size_of(len[k], msk[k] != 0);
        hsp |= uint64_t(hs) << (4 * k);
        v[k] = f < n ? hs + len[k] : 0;
    }
    const uint64_t wt = wave_scan_items(v, ex);
    PLAN_STAMP(b, 1);
    const uint64_t pre = single_block_prefix<kBT / 64>(b, wt, s_wave, &s_prefix, look);
    PLAN_STAMP(b, 2);
#pragma unroll
    for (int k = 0; k < kSingleItems; ++k) {
        const uint64_t f = f0 + uint64_t(k) * 64;
        if (f >= n) continue;
        const uint64_t run = pre + ex[k];
        offs[f] = run;
        const uint32_t hs = (uint32_t)((hsp >> (4 * k)) & 15u);
        // the whole descriptor: the line leaves L2 fully written
        uint64_t* q = reinterpret_cast<uint64_t*>(desc) + 4 * f;
        q[0] = poff[k];
        q[1] = run;
        q[2] = len[k];
        q[3] = (w3[k] & ~(uint64_t(0xff) << 56)) | uint64_t(hs) << 56;
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
    PLAN_STAMP(b, 3);
}

// ---- the fused deserialize: plan and copy in one pass ------------------------
// For batches of small frames at 16-byte slots (cfws_deserialize_batch),
// each block of the single-pass plan copies its own frames once their
// offsets are known, so the header lines the plan reads are the lines the
// copy streams next (one pass over the wire instead of two: the plan alone
// re-read 0.5 GB of 128-byte lines for 4 M x 1 KiB frames, 2.2 GB for
// 16 M x 256 B). Wave w copies the frames it parsed (item k, lane l: frame
// k * 64 + l of its run). Per item, the wave's largest slot sets how many
// frames share one wave-instruction: groups of G lanes (G x 16 bytes >= the
// slot), one frame per group; items with a slot over 1 KiB go frame by
// frame, 1 KiB per instruction. A lane's chunk is its frame's source block
// funnel-shifted with the next lane's block over DPP (the lane loads the
// next block itself at its group's end), XORed with the key (each chunk
// starts at a payload index that is a multiple of 16, so the key needs no
// rotation) and masked past the payload: every slot byte below the pass
// total is written once, payload or zero, as the plan + execute write it.
#ifndef CFWS_FUSED_UNROLL
#define CFWS_FUSED_UNROLL 4
#endif
// The fused kernel's occupancy hint, stated as what it is: workgroups of
// kFusedThreads per CU (__launch_bounds__' second argument). 1 at 1024
// threads = 16 waves per CU, 4 per SIMD: the register budget every fused
// measurement in DESIGN.md ran with (the hint used to be written as
// 5 * 256 / kBT, which truncated to this same 1).
#ifndef CFWS_FUSED_MIN_BLOCKS_PER_CU
#define CFWS_FUSED_MIN_BLOCKS_PER_CU 1
#endif
constexpr int kFusedMinBlocksPerCU = CFWS_FUSED_MIN_BLOCKS_PER_CU;
static_assert(kFusedMinBlocksPerCU >= 1, "the fused kernel's occupancy hint must be at least 1");
constexpr int kFusedUnroll = CFWS_FUSED_UNROLL;   // rounds of loads in flight per wave

__device__ __forceinline__ void fused_store(uint8_t* __restrict__ out, uint64_t D, uint64_t total, uint4 o)
{
    if (D + 16 <= total) {
        st16(out + D, o);
    } else {
        for (uint32_t j = 0; D + j < total; ++j) {
            const uint32_t w = j < 4 ? o.x : (j < 8 ? o.y : (j < 12 ? o.z : o.w));
            out[D + j] = (uint8_t)(w >> (8 * (j & 3)));
        }
    }
}

// One lane's chunk in a round: its destination D and source s, the bytes
// of the slot it writes (nbytes) and of those the payload (need), the key.
struct FusedChunk {
    uint64_t D, s;
    uint32_t need, nbytes, key;
};

template <int kUnroll = kFusedUnroll>
__device__ __forceinline__ void fused_item(const uint8_t* __restrict__ wire, uint8_t* __restrict__ out,
                                           uint64_t total, uint64_t run, uint64_t src, uint32_t len,
                                           uint32_t nb, uint32_t key, uint32_t lane)
{
    // wave-wide largest slot
    uint32_t m = nb;
#pragma unroll
    for (uint32_t o = 32; o >= 1; o >>= 1) {
        const uint32_t y = (uint32_t)__shfl_xor((int)m, o, 64);
        m = y > m ? y : m;
    }
    const uint4 z = make_uint4(0, 0, 0, 0);
    if (m == 0) return;
    if (m <= 1024) {
        // G lanes per frame (G x 16 >= m), P = 64 / G frames per round
        uint32_t G = 1;
        while (G * 16 < m) G <<= 1;
        const uint32_t P = 64 / G, g = lane / G, c = lane % G;
        for (uint32_t r0 = 0; r0 < G; r0 += kUnroll) {
            uint4 A[kUnroll], E[kUnroll];
            FusedChunk q[kUnroll];
            bool nl[kUnroll];
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) {
                const uint32_t r = r0 + u;
                const int fl = (int)((r < G ? r : 0) * P + g);
                const uint64_t runj = __shfl(run, fl, 64), srcj = __shfl(src, fl, 64);
                const uint32_t lenj = (uint32_t)__shfl((int)len, fl, 64);
                const uint32_t nbj = r < G ? (uint32_t)__shfl((int)nb, fl, 64) : 0u;
                q[u].key = (uint32_t)__shfl((int)key, fl, 64);
                q[u].D = runj + 16 * c;
                q[u].s = srcj + 16 * c;
                q[u].nbytes = 16 * c < nbj ? (uint32_t)(nbj - 16 * c < 16 ? nbj - 16 * c : 16) : 0u;
                q[u].need = q[u].nbytes && 16 * c < lenj ? (uint32_t)(lenj - 16 * c < 16 ? lenj - 16 * c : 16) : 0u;
                nl[u] = c + 1 < G && 16 * (c + 1) < lenj;          // the next lane loads the next block
                const uint32_t ph = (uint32_t)(q[u].s & 15u);
                A[u] = q[u].need ? ld16(wire + (q[u].s & ~uint64_t(15))) : z;
                E[u] = q[u].need && ph && !nl[u] && ph + q[u].need > 16
                           ? ld16(wire + (q[u].s & ~uint64_t(15)) + 16) : z;
            }
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) {
                const uint4 nb4 = from_next_lane(A[u], E[u]);      // every lane: DPP needs the full wave
                if (!q[u].nbytes) continue;
                const uint32_t ph = (uint32_t)(q[u].s & 15u);
                uint4 o = z;
                if (q[u].need) {
                    o = ph ? funnel16(A[u], nl[u] ? nb4 : E[u], ph) : A[u];
                    xor4(o, q[u].key);
                    if (q[u].need < 16) o = and4(o, byte_range(0, q[u].need));
                }
                fused_store(out, q[u].D, total, o);
            }
        }
        return;
    }
    // items with a slot over 1 KiB: frame by frame, wave-uniform
    for (int j = 0; j < 64; ++j) {
        const uint64_t nbj = (uint32_t)__builtin_amdgcn_readlane((int)nb, j);
        if (nbj == 0) continue;
        const uint64_t runj = __shfl(run, j, 64), srcj = __shfl(src, j, 64);
        const uint64_t lenj = (uint32_t)__builtin_amdgcn_readlane((int)len, j);
        const uint32_t kj = (uint32_t)__shfl((int)key, j, 64);
        const uint32_t ph = (uint32_t)(srcj & 15u);
        for (uint64_t c0 = 0; c0 < nbj; c0 += 64 * 16 * kUnroll) {
            uint4 A[kUnroll], E[kUnroll];
            uint32_t need[kUnroll];
            bool nl[kUnroll];
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) {
                const uint64_t k0 = c0 + (uint64_t)u * 1024 + 16 * lane;
                need[u] = k0 < lenj ? (uint32_t)(lenj - k0 < 16 ? lenj - k0 : 16) : 0u;
                nl[u] = lane != 63 && k0 + 16 < lenj;
                const uint64_t s = srcj + k0;
                A[u] = need[u] ? ld16(wire + (s & ~uint64_t(15))) : z;
                E[u] = need[u] && ph && !nl[u] && ph + need[u] > 16 ? ld16(wire + (s & ~uint64_t(15)) + 16) : z;
            }
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) {
                const uint4 nb4 = from_next_lane(A[u], E[u]);
                const uint64_t k0 = c0 + (uint64_t)u * 1024 + 16 * lane;
                if (k0 >= nbj) continue;
                uint4 o = z;
                if (need[u]) {
                    o = ph ? funnel16(A[u], nl[u] ? nb4 : E[u], ph) : A[u];
                    xor4(o, kj);
                    if (need[u] < 16) o = and4(o, byte_range(0, need[u]));
                }
                fused_store(out, runj + k0, total, o);
            }
        }
    }
}

// deserialize_plan_reduce_kernel + deserialize_plan_apply_kernel in one
// launch, without reassembly (its control-frame pass starts at the data
// pass's grand total, which no block knows before the last one). The
// descriptors are written as parsed, their payload offsets (and the
// capacity rule's status) once the offsets are known. kCopy: the fused
// deserialize (above): each block then copies its frames into `out`; no
// offsets or region map are written (no execute follows).
// One unaligned 16-byte load (the part's unaligned access mode): the
// receive plan's header loads.
__device__ __forceinline__ uint4 ld16u(const uint8_t* p)
{
    typedef uint32_t u32x4u __attribute__((ext_vector_type(4), aligned(1)));
    const u32x4u v = *reinterpret_cast<const u32x4u*>(p);
    return make_uint4(v.x, v.y, v.z, v.w);
}

#ifndef CFWS_FUSED_ITEMS
#define CFWS_FUSED_ITEMS 2
#endif
constexpr int kFusedItems = CFWS_FUSED_ITEMS;   // frames per thread in the fused form (registers)

template <bool kCopy, int kBT>
__global__ void __launch_bounds__(kBT, kCopy ? kFusedMinBlocksPerCU : 1)
deserialize_plan_single_kernel(const uint8_t* __restrict__ wire, uint64_t wire_size_all,
                               const uint64_t* __restrict__ index, const uint64_t* __restrict__ ends,
                               uint64_t n, uint64_t max_payload, uint64_t align,
                               cfws_frame_desc_t* __restrict__ desc, int32_t* __restrict__ status,
                               uint64_t* __restrict__ offs, uint32_t* __restrict__ look,
                               uint64_t* __restrict__ hdr, uint64_t capacity, uint32_t* __restrict__ map,
                               uint64_t* __restrict__ user_total, uint8_t* __restrict__ out = nullptr)
{
    __shared__ uint64_t s_wave[kBT / 64];
    __shared__ uint64_t s_prefix;
    __shared__ uint32_t s_bid;
    constexpr int kSingleItems = kCopy ? kFusedItems : kSingleItemsDeser;
    constexpr uint64_t kSingleFrames = uint64_t(kBT) * kSingleItems;
    const uint32_t b = plan_ticket(look, &s_bid);
    PLAN_STAMP(b, 0);
    const uint64_t f0 = uint64_t(b) * kSingleFrames + uint64_t(threadIdx.x >> 6) * (64 * kSingleItems) +
                        (threadIdx.x & 63u);
    // each descriptor is written once, whole, with its offset: the parsed
    // fields wait in registers (wire_off, payload_size, the last word)
    uint64_t v[kSingleItems], ex[kSingleItems], wo[kSingleItems], ps[kSingleItems], w3[kSingleItems];
    int32_t sts[kSingleItems];
    // the loads of all items first, in two rounds (starts and ends, then
    // every header's 16 bytes, below), then the parses: a
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
    // every header from one 16-byte load at its first byte (unaligned: the
    // part's unaligned access mode; one request, or two when the 16 bytes
    // cross a line), clamped to the buffer's last 16 bytes instead of
    // branching on the bytes available; a header with fewer than 16 bytes
    // after it in the buffer is parsed by the loads of parse_ws_header
    const bool b16 = wire_size_all >= 16;
    const uint64_t lastu = wire_size_all - 16;
    uint4 hw[kSingleItems];
    if (b16) {
#pragma unroll
        for (int k = 0; k < kSingleItems; ++k) hw[k] = ld16u(wire + (sx[k] < lastu ? sx[k] : lastu));
    }
#pragma unroll
    for (int k = 0; k < kSingleItems; ++k) {
        const uint64_t f = f0 + uint64_t(k) * 64;
        v[k] = 0;
        if (f < n) {
            const uint64_t wire_size = sz[k];
            cfws_frame_desc_t d;
            const uint64_t s0 = sx[k];
            if (b16 && s0 <= lastu) {
                const uint64_t avail = s0 <= wire_size ? wire_size - s0 : 0;
                const uint4 W = hw[k];
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
    const uint64_t wt = wave_scan_items(v, ex);
    PLAN_STAMP(b, 1);
    const uint64_t pre = single_block_prefix<kBT / 64>(b, wt, s_wave, &s_prefix, look);
    PLAN_STAMP(b, 2);
    // kCopy: what the copy needs per item, compact (the parse's arrays die here)
    uint64_t c_run[kSingleItems], c_src[kSingleItems];
    uint32_t c_len[kSingleItems], c_nb[kSingleItems], c_key[kSingleItems];
#pragma unroll
    for (int k = 0; k < kSingleItems; ++k) {
        const uint64_t f = f0 + uint64_t(k) * 64;
        c_run[k] = c_src[k] = 0;
        c_len[k] = c_nb[k] = c_key[k] = 0;
        if (f >= n) continue;
        const uint64_t run = pre + ex[k];
        if (!kCopy) offs[f] = run;
        uint64_t* q = reinterpret_cast<uint64_t*>(desc) + 4 * f;
        q[0] = run;
        q[1] = wo[k];
        q[2] = ps[k];
        q[3] = w3[k];
        // the capacity rule (co_ws_frame.c:216-223), as deserialize_plan_apply_kernel
        int32_t st = sts[k];
        if (st == CFWS_PARSE_COMPLETE && ps[k] > 0 && run + ps[k] > capacity) st = CFWS_ERROR_OUT_OF_MEMORY;
        status[f] = st;
        if (kCopy) {
            // slot bytes below the capacity (every slot ends at or below the
            // grand total, so that is the pass total's cut); the payload
            // only for a frame still COMPLETE, zeros otherwise
            const uint64_t end = run + v[k] < capacity ? run + v[k] : capacity;
            const uint64_t nbk = end > run ? end - run : 0;
            c_run[k] = run;
            c_src[k] = wo[k] + (w3[k] >> 56);
            c_nb[k] = nbk < 0xffffffffull ? (uint32_t)nbk : 0xffffffffu;
            c_len[k] = st == CFWS_PARSE_COMPLETE ? (uint32_t)(ps[k] < nbk ? ps[k] : nbk) : 0u;
            c_key[k] = (w3[k] >> 48) & 0xffu ? (uint32_t)w3[k] : 0u;
        } else {
            map_range(run, run + v[k], f, capacity, map);
        }
        if (f == n - 1) {
            const uint64_t g = run + v[k], t = g < capacity ? g : capacity;
            if (!kCopy) map[(t + kRegion - 1) / kRegion] = (uint32_t)f;
            hdr[0] = t;
            hdr[1] = 0;
            hdr[2] = t;
            hdr[3] = g;
            if (user_total) *user_total = t;
        }
    }
    if (!kCopy) {
#if CFWS_PLAN_TRACE
        __syncthreads();
        PLAN_STAMP(b, 3);
#endif
        return;
    }
    // the copy: every slot byte below the pass total min(grand total,
    // capacity), cut at the capacity itself (above)
    const uint32_t lane = threadIdx.x & 63u;
#pragma unroll
    for (int k = 0; k < kSingleItems; ++k)
        fused_item(wire, out, capacity, c_run[k], c_src[k], c_len[k], c_nb[k], c_key[k], lane);
#if CFWS_PLAN_TRACE
    __syncthreads();
    PLAN_STAMP(b, 3);
#endif
}

// The fused deserialize (deserialize_plan_single_kernel<true>) for batches
// of more than kSmallFrames frames averaging at most fused_avg_max() wire
// bytes (CFWS_FUSED_DESER=0: plan + execute; CFWS_FUSED_AVG_MAX: the
// average, 512 by default; A/B knobs). A block copies its own frames, so a
// batch mixing a few huge frames into small ones would leave those to
// single waves: the average keeps such batches on the region stream.
bool fused_deser()
{
    static const bool v = env_knob("CFWS_FUSED_DESER", 1) != 0;
    return v;
}

uint64_t fused_avg_max()
{
    static const uint64_t v = (uint64_t)env_knob("CFWS_FUSED_AVG_MAX", 512);
    return v;
}

// ---------------------------------------------------------------------------
// fixed payload slots (cfws_deserialize_slots)
// ---------------------------------------------------------------------------
// Frame i's payload goes to slot i (payload_off = i * slot): no prefix, so
// no look-back, and the pass reads each wire line once. The packed receive
// cannot: a frame's destination needs every earlier header, so its header
// line is fetched by the parse and again by the copy (§9: 6.86 GB per
// 16 M x 256 B launch against 4.43 GB of wire).
//
// Slots of at most kSlotWindow8Max bytes (deserialize_slots_window_kernel):
// a frame's window is the 16-byte block holding its first byte and the
// G - 1 after it, G = slot / 16 + 2 (block phase <= 15 plus header <= 14 plus
// payload <= slot bytes), one block per virtual lane. S sub-windows of 64
// lanes give 64 S virtual lanes (S = 1 up to 992 B -- 2 for 496-640 B, three
// frames to a pair --, 2 up to 2,016 B, 4 up to 4,064 B, 8 up to 8,160 B),
// so P = 64 S / G frames share a wave-round. A wave takes R rounds (R P <=
// 64 frames) per iteration: lane l loads frame l's index, every round's
// window blocks are issued at once together with each frame's 16 header
// bytes (one unaligned load, lane = frame: the same lines as the windows, in
// flight together, so HBM sees them once), each lane parses its frame and
// writes its descriptor and status (consecutive lanes, consecutive
// entries), and each round then takes its frames' (length, phase + header,
// key) from the parsing lanes. A virtual lane's 16 payload bytes start
// (phase + header) bytes into its own block: blocks c and c + 1, or c + 1
// and c + 2 past 16 (DPP shifts by one lane, no LDS; a sub-window's last two
// lanes take the next sub-window's first two blocks), funnelled and
// unmasked (each chunk starts at a payload index that is a multiple of 16:
// no key rotation). Blocks at or past the wire's end are not loaded. The
// first form parsed in every lane of every round (480 instructions per 3
// frames at 256 B) and ran at 5.2 TB/s.
constexpr uint64_t kSlotWindow8Max = 512 * 16 - 32;   // eight blocks per lane up to 8,160 B
// Rounds per iteration (their loads in flight together): 8 for one frame per
// round (slots over 480 B), 4 for more (16 M x 256 B receive 1.686 -> 1.620
// ms; 12 or 16 rounds: 3.3 ms; 8 M x 512 B at 4 rounds 1.59 -> 1.76 ms).
#ifndef CFWS_SLOT_ROUNDS
#define CFWS_SLOT_ROUNDS 8
#endif
#ifndef CFWS_SLOT_ROUNDS_MULTI
#define CFWS_SLOT_ROUNDS_MULTI 4
#endif
#ifndef CFWS_SLOT_ROUNDS2
#define CFWS_SLOT_ROUNDS2 4      // two blocks per lane (1,008-2,016 B): 2,016 B 2 / 4 / 6 -> 1.61-1.62 / 1.61 / 1.63 ms
#endif
#ifndef CFWS_SLOT_ROUNDS8
#define CFWS_SLOT_ROUNDS8 1      // eight blocks per lane (4,080-8,160 B)
#endif
#ifndef CFWS_SLOT_ROUNDS4
#define CFWS_SLOT_ROUNDS4 1      // four blocks per lane (2,032-4,064 B): 3 KiB 1 / 2 / 4 -> 1.48 / 1.55 / 1.59 ms
#endif

__device__ __forceinline__ uint4 shfl16(uint4 v, int src)
{
    return make_uint4((uint32_t)__shfl((int)v.x, src, 64), (uint32_t)__shfl((int)v.y, src, 64),
                      (uint32_t)__shfl((int)v.z, src, 64), (uint32_t)__shfl((int)v.w, src, 64));
}

__device__ __forceinline__ uint64_t shfl64(uint64_t v, int src)
{
    return (uint64_t)__shfl((long long)v, src, 64);
}

// The slot rule: a COMPLETE frame whose non-empty payload is longer than the
// slot, or ends past the capacity, gets CFWS_ERROR_OUT_OF_MEMORY (the
// reference's failed allocation, co_ws_frame.c:216-223); its slot is not
// written.
__device__ __forceinline__ int32_t slot_rule(int32_t st, uint64_t run, uint64_t ps, uint64_t slot, uint64_t cap)
{
    return st == CFWS_PARSE_COMPLETE && ps > 0 && (ps > slot || run > cap || ps > cap - run)
               ? CFWS_ERROR_OUT_OF_MEMORY : st;
}

// The scatter form (cfws_deserialize_scatter): frame i's payload at the
// caller's dst[i] instead of i * slot, which must be a multiple of 16 (the
// copy stores whole aligned blocks); a frame whose offset is not does not
// fit either.
__device__ __forceinline__ int32_t scatter_rule(int32_t st, uint64_t run, uint64_t ps, uint64_t slot, uint64_t cap)
{
    st = slot_rule(st, run, ps, slot, cap);
    return st == CFWS_PARSE_COMPLETE && ps > 0 && (run & 15u) ? CFWS_ERROR_OUT_OF_MEMORY : st;
}

__device__ __forceinline__ void slot_desc(cfws_frame_desc_t* desc, int32_t* status, uint64_t f, uint64_t run,
                                          const cfws_frame_desc_t& d, int32_t st)
{
    uint4* q = reinterpret_cast<uint4*>(desc + f);
    const uint64_t w3 = (uint64_t)d.mask_key | (uint64_t)d.fin << 32 | (uint64_t)d.opcode << 40 |
                        (uint64_t)d.mask << 48 | (uint64_t)d.header_size << 56;
    q[0] = make_uint4((uint32_t)run, (uint32_t)(run >> 32), (uint32_t)d.wire_off, (uint32_t)(d.wire_off >> 32));
    q[1] = make_uint4((uint32_t)d.payload_size, (uint32_t)(d.payload_size >> 32), (uint32_t)w3,
                      (uint32_t)(w3 >> 32));
    status[f] = st;
}

// The compact per-frame output (cfws_deserialize_slots_info /
// _scatter_info): the reference frame's header fields and the status in 8
// bytes, one u64 store per frame (consecutive lanes, consecutive entries).
__device__ __forceinline__ void slot_info(cfws_frame_info_t* info, uint64_t f, const cfws_frame_desc_t& d, int32_t st)
{
    const uint32_t ps = d.payload_size > 0xffffffffull ? 0xffffffffu : (uint32_t)d.payload_size;
    const uint32_t w1 = (uint32_t)d.fin | (uint32_t)d.opcode << 8 | ((uint32_t)st & 0xffffu) << 16;
    reinterpret_cast<uint2*>(info)[f] = make_uint2(ps, w1);
}

// the uniform receive's check: lanes whose frame is not a COMPLETE frame of
// exactly `stride` wire bytes, one atomic per wave that has any
__device__ __forceinline__ void count_mismatch(uint32_t* mismatch, bool odd, uint32_t lane)
{
    const uint64_t b = __ballot(odd);
    if (b && lane == 0) atomicAdd(mismatch, (uint32_t)__popcll(b));
}

// kInfo: write cfws_frame_info_t entries to `info` instead of descriptors
// and statuses; index null: frame i starts at i * stride and `mismatch`
// (when not null) counts the frames that are not uniform frames
template <int kSlotRounds, int kSub, bool kScatter, bool kInfo>
__global__ void __launch_bounds__(kThreads)
deserialize_slots_window_kernel(const uint8_t* __restrict__ wire, uint64_t wire_size,
                                const uint64_t* __restrict__ index, uint64_t n, uint64_t max_payload,
                                uint64_t slot, uint32_t G, cfws_frame_desc_t* __restrict__ desc,
                                int32_t* __restrict__ status, uint8_t* __restrict__ out, uint64_t capacity,
                                uint64_t* __restrict__ user_total, const uint64_t* __restrict__ dst,
                                cfws_frame_info_t* __restrict__ infos, uint64_t stride,
                                uint32_t* __restrict__ mismatch)
{
    const uint32_t lane = threadIdx.x & 63u;
    // kSub sub-windows of 64 lanes make 64 kSub virtual lanes, v = 64 sw +
    // lane; frame g of a round takes virtual lanes [g G, g G + G), P = 64 kSub
    // / G frames, so lane `lane` of sub-window sw holds block c[sw] of the
    // round's frame g[sw]
    const uint32_t P = 64u * kSub / G;
    uint32_t g[kSub], c[kSub];
#pragma unroll
    for (int sw = 0; sw < kSub; ++sw) {
        g[sw] = (64u * sw + lane) / G;
        c[sw] = 64u * sw + lane - g[sw] * G;
    }
    const uint32_t R = P * kSlotRounds <= 64 ? (uint32_t)kSlotRounds : 64u / P;
    const uint64_t FI = uint64_t(R) * P;                 // frames per wave-iteration
    const uint64_t grid_frames = uint64_t(gridDim.x) * kWaves * FI;
    const uint4 z = make_uint4(0, 0, 0, 0);
    const bool b16 = wire_size >= 16;
    const uint64_t lastu = wire_size - 16;
    for (uint64_t f0 = (uint64_t(blockIdx.x) * kWaves + (threadIdx.x >> 6)) * FI; f0 < n; f0 += grid_frames) {
        const uint64_t fl = f0 + lane;
        const bool mine = lane < FI && fl < n;
        // the frame's start: the index, or frame i at i * stride (the uniform
        // receive: its window loads need no index load before them)
        const uint64_t wl = !mine ? ~uint64_t(0) : index ? index[fl] : fl * stride;
        // the frame's payload offset: its slot, or the caller's (scatter)
        const uint64_t runl = !mine ? 0 : kScatter ? dst[fl] : fl * slot;
        // every round's window block, then each frame's header bytes
        uint4 A[kSlotRounds][kSub];
#pragma unroll
        for (int u = 0; u < kSlotRounds; ++u) {
#pragma unroll
            for (int sw = 0; sw < kSub; ++sw) {
                const uint32_t src = (uint32_t)u * P + g[sw];
                const uint64_t wo = shfl64(wl, (int)(src < 64 ? src : 63));
                const uint64_t blk = (wo & ~uint64_t(15)) + 16ull * c[sw];   // block c of the window
                A[u][sw] = (uint32_t)u < R && g[sw] < P && wo < wire_size && blk < wire_size
                               ? ld16(wire + blk) : z;
            }
        }
        const uint4 hw = mine && b16 && wl <= lastu ? ld16u(wire + wl) : z;
        // lane l parses frame f0 + l; its round info: payload length (<= slot
        // < 2^16) | (phase + header size) << 16, zero when not copied
        uint32_t info = 0, key = 0;
        bool odd = false;   // not a uniform frame at its place (mismatch count)
        if (mine) {
            cfws_frame_desc_t d;
            int32_t st;
            if (b16 && wl <= lastu) {
                const uint32_t w[4] = {hw.x, hw.y, hw.z, hw.w};
                st = parse_ws_header_regs(w, wire_size - wl, max_payload, d);
                d.wire_off = wl;
            } else {
                st = parse_ws_header(wire, wire_size, wl, max_payload, d);
            }
            const uint64_t run = runl;
            st = kScatter ? scatter_rule(st, run, d.payload_size, slot, capacity)
                          : slot_rule(st, run, d.payload_size, slot, capacity);
            if constexpr (kInfo)
                slot_info(infos, fl, d, st);
            else
                slot_desc(desc, status, fl, run, d, st);
            if (fl == n - 1 && user_total) {
                const uint64_t t = n * slot;
                *user_total = t < capacity ? t : capacity;
            }
            if (st == CFWS_PARSE_COMPLETE && d.payload_size > 0)
                info = (uint32_t)d.payload_size | ((uint32_t)(wl & 15u) + d.header_size) << 16;
            key = d.mask ? d.mask_key : 0u;
            odd = st != CFWS_PARSE_COMPLETE || d.header_size + d.payload_size != stride;
        }
        if (mismatch) count_mismatch(mismatch, odd, lane);
#pragma unroll
        for (int u = 0; u < kSlotRounds; ++u) {
            if ((uint32_t)u >= R) break;   // wave-uniform
#pragma unroll
            for (int sw = 0; sw < kSub; ++sw) {
                const uint32_t src = (uint32_t)u * P + g[sw];
                const int s = (int)(src < 64 ? src : 63);
                const uint32_t inf = (uint32_t)__shfl((int)info, s, 64);
                const uint32_t k = (uint32_t)__shfl((int)key, s, 64);
                const uint32_t len = inf & 0xffffu, off = inf >> 16;
                const uint64_t runf = kScatter ? shfl64(runl, s) : (f0 + src) * slot;
                // blocks c + 1 and c + 2 of this sub-window, by DPP (every
                // lane); lanes 62 and 63 of a sub-window take the next one's
                // first two blocks
                const uint4 l0 = sw + 1 < kSub ? shfl16(A[u][sw + 1 < kSub ? sw + 1 : sw], 0) : z;
                const uint4 l1 = sw + 1 < kSub ? shfl16(A[u][sw + 1 < kSub ? sw + 1 : sw], 1) : z;
                const uint4 n1 = from_next_lane(A[u][sw], l0);
                const uint4 n2 = from_next_lane(n1, l1);
                const uint32_t q = c[sw];          // payload chunk
                if (g[sw] < P && 16u * q < len) {
                    const bool k1 = off >= 16;
                    const uint4 B0 = k1 ? n1 : A[u][sw], B1 = k1 ? n2 : n1;
                    const uint32_t sh = off & 15u;
                    uint4 o = sh ? funnel16(B0, B1, sh) : B0;
                    xor4(o, k);
                    if (len - 16u * q < 16u) o = and4(o, byte_range(0, len - 16u * q));
                    fused_store(out, runf + 16ull * q, capacity, o);
                }
            }
        }
    }
}

#ifndef CFWS_SLOT_UNROLL
#define CFWS_SLOT_UNROLL 16      // slots over 8,160 B: 64 K x 64 KiB receive 2.04 / 1.76 / 1.71 ms at 4 / 8 / 16 rounds, 8 KiB 1.72 at each
#endif
constexpr int kSlotUnroll = CFWS_SLOT_UNROLL;   // deserialize_slots_kernel: rounds of loads in flight

// Slots over kSlotWindow8Max: one frame per thread parsed (its header line
// fetched twice, a small share of a frame this long), the payloads copied
// by fused_item.
template <bool kScatter, bool kInfo>
__global__ void __launch_bounds__(kThreads)
deserialize_slots_kernel(const uint8_t* __restrict__ wire, uint64_t wire_size, const uint64_t* __restrict__ index,
                         uint64_t n, uint64_t max_payload, uint64_t slot, cfws_frame_desc_t* __restrict__ desc,
                         int32_t* __restrict__ status, uint8_t* __restrict__ out, uint64_t capacity,
                         uint64_t* __restrict__ user_total, const uint64_t* __restrict__ dst,
                         cfws_frame_info_t* __restrict__ info, uint64_t stride, uint32_t* __restrict__ mismatch)
{
    const uint64_t f = uint64_t(blockIdx.x) * kThreads + threadIdx.x;
    uint64_t run = 0, src = 0;
    uint32_t len = 0, nb = 0, key = 0;
    bool odd = false;
    if (f < n) {
        cfws_frame_desc_t d;
        const uint64_t s0 = index ? index[f] : f * stride;
        run = kScatter ? dst[f] : f * slot;
        const int32_t p = parse_ws_header(wire, wire_size, s0, max_payload, d);
        const int32_t st = kScatter ? scatter_rule(p, run, d.payload_size, slot, capacity)
                                    : slot_rule(p, run, d.payload_size, slot, capacity);
        if constexpr (kInfo)
            slot_info(info, f, d, st);
        else
            slot_desc(desc, status, f, run, d, st);
        if (st == CFWS_PARSE_COMPLETE) {
            len = (uint32_t)d.payload_size;   // <= slot < 2^31
            nb = (len + 15u) & ~15u;
            src = s0 + d.header_size;
            key = d.mask ? d.mask_key : 0u;
        }
        odd = st != CFWS_PARSE_COMPLETE || d.header_size + d.payload_size != stride;
        if (f == n - 1 && user_total) {
            const uint64_t t = n * slot;
            *user_total = t < capacity ? t : capacity;
        }
    }
    if (mismatch) count_mismatch(mismatch, odd, threadIdx.x & 63u);
    fused_item<kSlotUnroll>(wire, out, capacity, run, src, len, nb, key, threadIdx.x & 63u);
}

// Slots over kSlotWindow8Max, piece by piece: wave w copies piece w % P of
// frame w / P (kSlotPiece bytes of slot), so a 64 KiB frame is 32 waves'
// work and a launch has n x P waves. P is the slot's piece count; when the
// batch's frames are shorter on average (wire bytes / frames) P is that
// average's piece count and each wave takes pieces w % P, w % P + P, ...
// (kLoop), so a large slot holding short payloads does not cost a wave per
// piece of the slot. Batches averaging under one piece per frame take the
// per-frame kernel, which packs short frames into shared wave-instructions
// (slots_route; tools/slot_sparse_probe.py: 1 M x 256 B in 16 KiB slots
// 0.13 ms there against 0.59 one wave per frame). The per-frame kernel above
// gives each wave the 64 frames its lanes parsed, one after another: 1,024
// waves for 64 K frames, one per SIMD. Every wave of a frame parses its
// header (one line, the same address in every lane); piece 0's lane 0 writes
// the frame's descriptor + status or info entry and counts a mismatch.
// 64 K x 64 KiB receive (profiles/r06/compact/slot_pieces/): per-frame
// kernel 1.59-1.64 ms; pieces of 8 / 4 / 2 / 1 KiB 1.51-1.60 / 1.42-1.49 /
// 1.35-1.36 / 2.13 ms; 2 KiB with write-through stores 1.31-1.32 (8 KiB
// frames 1.38, against 1.51-1.64).
#ifndef CFWS_SLOT_PIECE_AUX
#define CFWS_SLOT_PIECE_AUX 19        // write-through (sc0 sc1 nt), as the WS receive; 0: the global nt store
#endif
#ifndef CFWS_SLOT_PIECE_UNROLL
#define CFWS_SLOT_PIECE_UNROLL 2
#endif
constexpr int kSlotPieceUnroll = CFWS_SLOT_PIECE_UNROLL;            // rounds of loads in flight per wave
constexpr uint64_t kSlotPiece = 64ull * 16 * kSlotPieceUnroll;     // 2 KiB
template <bool kScatter, bool kInfo, bool kLoop>
__global__ void __launch_bounds__(kThreads)
deserialize_slots_piece_kernel(const uint8_t* __restrict__ wire, uint64_t wire_size,
                               const uint64_t* __restrict__ index, uint64_t n, uint64_t max_payload, uint64_t slot,
                               cfws_frame_desc_t* __restrict__ desc, int32_t* __restrict__ status,
                               uint8_t* __restrict__ out, uint64_t capacity, uint64_t* __restrict__ user_total,
                               const uint64_t* __restrict__ dst, cfws_frame_info_t* __restrict__ info,
                               uint64_t stride, uint32_t* __restrict__ mismatch, uint64_t pieces)
{
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const uint4 z = make_uint4(0, 0, 0, 0);
    const uint64_t waves = n * pieces;
    for (uint64_t w = uint64_t(blockIdx.x) * kWaves + wv; w < waves; w += uint64_t(gridDim.x) * kWaves) {
        const uint64_t f = w / pieces, piece = w - f * pieces;
        cfws_frame_desc_t d;
        const uint64_t s0 = index ? index[f] : f * stride;
        const uint64_t run = kScatter ? dst[f] : f * slot;
        const int32_t p = parse_ws_header(wire, wire_size, s0, max_payload, d);
        const int32_t st = kScatter ? scatter_rule(p, run, d.payload_size, slot, capacity)
                                    : slot_rule(p, run, d.payload_size, slot, capacity);
        if (piece == 0 && lane == 0) {
            if constexpr (kInfo)
                slot_info(info, f, d, st);
            else
                slot_desc(desc, status, f, run, d, st);
            if (f == n - 1 && user_total) {
                const uint64_t t = n * slot;
                *user_total = t < capacity ? t : capacity;
            }
            if (mismatch && (st != CFWS_PARSE_COMPLETE || d.header_size + d.payload_size != stride))
                atomicAdd(mismatch, 1u);
        }
        if (st != CFWS_PARSE_COMPLETE) continue;             // wave-uniform: every lane parsed the same frame
        const uint64_t len = d.payload_size;                 // <= slot <= 2^31
        const uint64_t nb = (len + 15) & ~uint64_t(15);
        const uint64_t src = s0 + d.header_size;
        const uint32_t key = d.mask ? d.mask_key : 0u;
        const uint32_t ph = (uint32_t)(src & 15u);
        // this wave's piece of the frame (kLoop: pieces piece, piece + P, ...;
        // without, the loop body once: the straight-line form measured 7 %
        // faster when every frame fills its slot)
        for (uint64_t c0 = piece * kSlotPiece; c0 < nb; c0 += pieces * kSlotPiece) {
            const auto prs = __builtin_amdgcn_make_buffer_rsrc(out + run + c0, 0, (int)kSlotPiece, 0x00020000);
            uint4 A[kSlotPieceUnroll], E[kSlotPieceUnroll];
            uint32_t need[kSlotPieceUnroll];
            bool nl[kSlotPieceUnroll];
#pragma unroll
            for (int u = 0; u < kSlotPieceUnroll; ++u) {
                const uint64_t k0 = c0 + (uint64_t)u * 1024 + 16 * lane;
                need[u] = k0 < len ? (uint32_t)(len - k0 < 16 ? len - k0 : 16) : 0u;
                nl[u] = lane != 63 && k0 + 16 < len;                 // the next lane loads the next block
                const uint64_t s = src + k0;
                A[u] = need[u] ? ld16(wire + (s & ~uint64_t(15))) : z;
                E[u] = need[u] && ph && !nl[u] && ph + need[u] > 16 ? ld16(wire + (s & ~uint64_t(15)) + 16) : z;
            }
#pragma unroll
            for (int u = 0; u < kSlotPieceUnroll; ++u) {
                const uint4 nb4 = from_next_lane(A[u], E[u]);       // every lane: DPP needs the full wave
                const uint64_t k0 = c0 + (uint64_t)u * 1024 + 16 * lane;
                if (k0 >= nb) continue;
                uint4 o = z;
                if (need[u]) {
                    o = ph ? funnel16(A[u], nl[u] ? nb4 : E[u], ph) : A[u];
                    xor4(o, key);
                    if (need[u] < 16) o = and4(o, byte_range(0, need[u]));
                }
                if (CFWS_SLOT_PIECE_AUX != 0 && run + k0 + 16 <= capacity) {
                    // a buffer store over the wave's piece (cache policy CFWS_SLOT_PIECE_AUX)
                    const u32x4 v = {o.x, o.y, o.z, o.w};
                    __builtin_amdgcn_raw_buffer_store_b128(v, prs, (int)(k0 - c0), 0, CFWS_SLOT_PIECE_AUX);
                } else {
                    fused_store(out, run + k0, capacity, o);
                }
            }
            if (!kLoop) break;
        }
    }
}

// Frames of at least CFWS_SLOT_SUB2_G lanes (default 33: slots of 496
// bytes and more) that fit three to a 128-lane pair of sub-windows (up to
// 42 lanes: slots up to 640 bytes) pack two sub-windows per round instead of
// one frame per round. Receive, two sub-windows against one: 512 B 1.535 ->
// 1.498 ms; 768 B (two frames per pair) 1.447 -> 1.490; 256 B and 384 B
// (already 2-3 frames per sub-window) 1.508 -> 1.552, 1.473 -> 1.506
// (profiles/r05/slots/sub2_ab/). A/B knob; 65 turns the packing off.
uint32_t slot_sub2_g()
{
    static const uint32_t v = (uint32_t)env_knob("CFWS_SLOT_SUB2_G", 33);
    return v;
}

// The receive without an index (cfws_deserialize_slots_uniform) keeps one
// frame per round there: with no index load ahead of the window loads, 8 M
// x 512 B takes 1.50 ms at one sub-window against 1.62 at two
// (profiles/r06/compact/implicit/). A/B knob.
uint32_t slot_sub2_g_implicit()
{
    static const uint32_t v = (uint32_t)env_knob("CFWS_SLOT_SUB2_G_IMPLICIT", 65);
    return v;
}

// The same for four sub-windows: frames of CFWS_SLOT_SUB4_G (default 129:
// off) to 85 lanes, three to 256 virtual lanes (A/B knob)
uint32_t slot_sub4_g()
{
    static const uint32_t v = (uint32_t)env_knob("CFWS_SLOT_SUB4_G", 129);
    return v;
}

bool slots_window()
{
    static const bool v = env_knob("CFWS_SLOTS_WINDOW", 1) != 0;
    return v;
}

bool slots_piece()
{
    static const bool v = env_knob("CFWS_SLOTS_PIECE", 1) != 0;
    return v;
}

// the kernel a slot / scatter receive takes (slots_impl and
// cfws_deserialize_slots_pass_kernel): windows up to kSlotWindow8Max-byte
// slots, pieces past that (A/B knobs: CFWS_SLOTS_WINDOW=0, CFWS_SLOTS_PIECE=0
// fall back to the per-frame kernel)
enum SlotsRoute { kSlotsWindow, kSlotsPiece, kSlotsPerFrame };
// Slots of 2 KiB up to kSlotWindow8Max take pieces too where the pieces'
// lanes are at least 85 % used and every piece starts on a 128-byte line.
// Receive without / with an index (profiles/r06/compact/slot_pieces/):
// 2 / 4 / 6 / 7.5 KiB 1.41 / 1.38 / 1.36 / 1.45 and 1.47 / 1.43 / 1.40 /
// 1.47 ms against the windows' 1.59 / 1.58 / 1.54 / 1.57 and 1.84 / 1.62 /
// 1.52 / 1.51; 5 KiB (83 % used) 1.47 / 1.56 against 1.52 / 1.53; 2.5 / 3 KiB
// (63 / 75 %) 1.90 / 1.62 against 1.52 / 1.48; 8,160 B (off the 128-byte
// lines) 1.86 against 1.69.
bool piece_pays(uint64_t slot)
{
    const uint64_t pieces = (slot + kSlotPiece - 1) / kSlotPiece;
    return slot % 128 == 0 && 20 * slot >= 17 * pieces * kSlotPiece;
}

SlotsRoute slots_route(uint64_t slot, uint64_t n, uint64_t wire_size)
{
    static const uint64_t piece_min = (uint64_t)env_knob("CFWS_SLOTS_PIECE_MIN", 2048);   // A/B knob
    // the batch's average frame (wire bytes): pieces pay for frames that
    // fill them, not for short frames in large slots
    const uint64_t avg = n ? wire_size / n : 0;
    const bool piece = slots_piece() && slot >= piece_min &&
                       (slot > kSlotWindow8Max ? avg > 1040 : piece_pays(slot) && 20 * avg >= 17 * slot);
    // a window spans the whole slot, whatever the frame: frames of up to
    // 1 KiB filling under half their slot (under 80 % of a slot of 1 KiB or
    // more) take the per-frame kernel, which packs them into shared
    // wave-instructions (tools/slot_sparse_probe.py: 256 B frames in 4 KiB
    // slots 0.14 against 1.15 ms, 512 B in 1 KiB 0.91 against 1.25, 768 B in
    // 1 KiB 1.30 against 1.41; 128 B in 256 B slots stay on the windows,
    // 0.67 against 0.71)
    const bool sparse = avg <= 1040 && (2 * avg < slot || (slot >= 1024 && 5 * avg < 4 * slot));
    if (slot <= kSlotWindow8Max && slots_window() && !piece && !sparse) return kSlotsWindow;
    return piece ? kSlotsPiece : kSlotsPerFrame;
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
        const uint32_t sb = grid_for(n, uint64_t(kDePlanThreads) * kSingleItemsDeser);
        if (hipMemsetAsync(look, 0, look_bytes(sb), st) != hipSuccess)
            return launch_check("deserialize_plan");
        deserialize_plan_single_kernel<false, kDePlanThreads><<<sb, kDePlanThreads, 0, st>>>(
            static_cast<const uint8_t*>(d_wire), wire_size, d_index, d_ends, n, max_payload, align, d_desc,
            d_status, offs0, look, hdr, cap, ws_ptr<uint32_t>(ws, L.map[0]), d_total);
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
    const CfwsPassScope pass_scope;
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
        const uint32_t sb = grid_for(n, uint64_t(kSerPlanThreads) * kSingleItemsSer);
        if (hipMemsetAsync(look, 0, look_bytes(sb), st) != hipSuccess)
            return launch_check("serialize_plan");
        serialize_plan_single_kernel<kSerPlanThreads><<<sb, kSerPlanThreads, 0, st>>>(d_desc, offs, n, look, hdr, cap,
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
    const CfwsPassScope pass_scope;
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
    const CfwsPassScope pass_scope;
    // small batch, every argument valid: one launch (serialize_small_kernel)
    if (small_path() && n > 0 && n <= kSmallFrames && cap <= kSmallBytes && check_init() == CFWS_OK &&
        d_desc && ws && ws_size >= ws_layout(n, cap).bytes &&
        (cap == 0 || (d_payload && d_wire && !misaligned(d_payload, d_wire)))) {
        const CfwsPassTimer timer(stream);
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
    const CfwsPassScope pass_scope;
    return deserialize_plan_impl(d_wire, wire_size, d_index, nullptr, n, max_payload, align, flags,
                                 d_desc, d_status, cap, d_total, ws, ws_size, stream);
}

int cfws_deserialize_execute(const void* d_wire, const cfws_frame_desc_t* d_desc,
                             const int32_t* d_status, size_t n, uint32_t flags, void* d_payload,
                             uint64_t cap, const void* ws, void* stream)
{
    const CfwsPassScope pass_scope;
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
        const CfwsPassTimer timer(st);      // both passes: one timed span
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

}  // extern "C"

namespace {

// Which form of cfws_deserialize_batch a call with these sizes takes, its
// other arguments valid (cfws_deserialize_pass_kernel reports the same
// choice): the one-launch small batch, the fused plan + copy of batches of
// small frames, or plan + execute.
enum DeserRoute { kDeserSmall, kDeserFused, kDeserPlanExecute };

DeserRoute deser_route(size_t n, uint64_t wire_size, uint32_t align, uint32_t flags, uint64_t cap)
{
    const bool align_ok = align != 0 && (align & (align - 1)) == 0 && align <= 4096;
    if (small_path() && n > 0 && n <= kSmallFrames && cap <= kSmallBytes && flags == 0 && align_ok)
        return kDeserSmall;
    if (fused_deser() && flags == 0 && align >= 16 && align_ok && n > kSmallFrames && n <= 0xffffffffull &&
        wire_size / n <= fused_avg_max())
        return kDeserFused;
    return kDeserPlanExecute;
}

}  // namespace

extern "C" {

const char* cfws_deserialize_pass_kernel(size_t n, uint64_t wire_size, uint32_t align, uint32_t flags,
                                         uint64_t payload_capacity)
{
    switch (deser_route(n, wire_size, align, flags, payload_capacity)) {
    case kDeserSmall: return "deserialize_small_kernel";
    case kDeserFused: return "deserialize_plan_single_kernel<true>";
    default: return "xform_kernel<1>";
    }
}

int cfws_deserialize_batch(const void* d_wire, uint64_t wire_size, const uint64_t* d_index,
                           size_t n, uint64_t max_payload, uint32_t align, uint32_t flags,
                           cfws_frame_desc_t* d_desc, int32_t* d_status, void* d_payload,
                           uint64_t cap, uint64_t* d_total, void* ws, size_t ws_size,
                           void* stream)
{
    const CfwsPassScope pass_scope;
    const DeserRoute route = deser_route(n, wire_size, align, flags, cap);
    // small batch without reassembly, every argument valid: one launch
    if (route == kDeserSmall && check_init() == CFWS_OK && d_wire && d_index &&
        d_desc && d_status && ws && ws_size >= ws_layout(n, cap).bytes &&
        (cap == 0 || (d_payload && !misaligned(d_payload, d_wire)))) {
        const CfwsPassTimer timer(stream);
        deserialize_small_kernel<<<small_grid(cap), kThreads, 0, static_cast<hipStream_t>(stream)>>>(
            static_cast<const uint8_t*>(d_wire), wire_size, d_index, (uint32_t)n, max_payload, align,
            d_desc, d_status, static_cast<uint8_t*>(d_payload), cap,
            ws_ptr<uint64_t>(ws, ws_layout(n, cap).hdr), d_total);
        return launch_check("deserialize_batch(small)");
    }
    // small frames at 16-byte (or wider) slots: the fused plan + copy
    if (route == kDeserFused && check_init() == CFWS_OK &&
        d_wire && d_index && d_desc && d_status && ws && ws_size >= ws_layout(n, cap).bytes &&
        (cap == 0 || (d_payload && !misaligned(d_payload, d_wire)))) {
        const WsLayout L = ws_layout(n, cap);
        hipStream_t st = static_cast<hipStream_t>(stream);
        uint32_t* look = ws_ptr<uint32_t>(ws, L.look);
        const uint32_t sb = grid_for(n, uint64_t(kFusedThreads) * kFusedItems);
        if (hipMemsetAsync(look, 0, look_bytes(sb), st) != hipSuccess)
            return launch_check("deserialize_batch(fused)");
        const CfwsPassTimer timer(st);
        deserialize_plan_single_kernel<true, kFusedThreads><<<sb, kFusedThreads, 0, st>>>(
            static_cast<const uint8_t*>(d_wire), wire_size, d_index, nullptr, n, max_payload, align, d_desc,
            d_status, nullptr, look, ws_ptr<uint64_t>(ws, L.hdr), cap, nullptr, d_total,
            static_cast<uint8_t*>(d_payload));
        return launch_check("deserialize_batch(fused)");
    }
    if (int rc = cfws_deserialize_plan(d_wire, wire_size, d_index, n, max_payload, align, flags,
                                       d_desc, d_status, cap, d_total, ws, ws_size, stream))
        return rc;
    return cfws_deserialize_execute(d_wire, d_desc, d_status, n, flags, d_payload, cap, ws, stream);
}

}  // extern "C"

namespace {

// cfws_deserialize_slots (dst null: frame i at i * slot) and
// cfws_deserialize_scatter (frame i at dst[i], slot = the largest payload
// a frame may have)
int slots_impl(const void* d_wire, uint64_t wire_size, const uint64_t* d_index, const uint64_t* dst, size_t n,
               uint64_t max_payload, uint64_t slot, cfws_frame_desc_t* d_desc, int32_t* d_status,
               void* d_payload, uint64_t cap, uint64_t* d_total, void* stream, bool scatter, const char* what,
               cfws_frame_info_t* d_info = nullptr, uint64_t stride = 0, uint32_t* d_mismatch = nullptr)
{
    if (int rc = check_init()) return rc;
    if (slot < 16 || (slot & 15) || slot > (1ull << 31))
        return set_err(CFWS_ERROR_INVALID_ARGUMENT, "slot bytes must be a multiple of 16 in [16, 2^31]",
                       hipSuccess);
    if (n > 0xffffffffull) return set_err(CFWS_ERROR_INVALID_ARGUMENT, "too many frames", hipSuccess);
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (n == 0) {
        if (d_total && hipMemsetAsync(d_total, 0, sizeof(uint64_t), st) != hipSuccess)
            return launch_check(what);
        return CFWS_OK;
    }
    const bool info = d_info != nullptr;
    if (!d_wire || (!d_index && !stride) || (!info && (!d_desc || !d_status)) || (cap && !d_payload) ||
        (scatter && !dst))
        return set_err(CFWS_ERROR_INVALID_ARGUMENT, "null pointer", hipSuccess);
    if (misaligned(d_payload, d_wire))
        return set_err(CFWS_ERROR_INVALID_ARGUMENT, "arenas must be 16-byte aligned", hipSuccess);
    const uint8_t* w = static_cast<const uint8_t*>(d_wire);
    uint8_t* out = static_cast<uint8_t*>(d_payload);
    const CfwsPassTimer timer(st);
    const SlotsRoute route = slots_route(slot, n, wire_size);
    if (route == kSlotsWindow) {
        // one wave-iteration of R P frames per wave (CFWS_SLOT_GRID caps the
        // workgroups: a grid-stride loop; A/B knob)
        const uint32_t G = (uint32_t)(slot / 16 + 2);
        const uint32_t sub2 = d_index ? slot_sub2_g() : slot_sub2_g_implicit();
        const uint32_t S = G > 256 ? 8
                           : G > 128 || (G >= slot_sub4_g() && 256 / G >= 3) ? 4
                           : G > 64 || (G >= sub2 && 128 / G >= 3) ? 2 : 1;   // sub-windows
        const uint32_t P = 64 * S / G;
        const uint64_t RK = S == 8 ? CFWS_SLOT_ROUNDS8 : S == 4 ? CFWS_SLOT_ROUNDS4 : S == 2 ? CFWS_SLOT_ROUNDS2
                            : P > 1 ? CFWS_SLOT_ROUNDS_MULTI : CFWS_SLOT_ROUNDS;
        const uint64_t R = P * RK <= 64 ? RK : 64 / P;
        const uint64_t per_block = uint64_t(kWaves) * R * P;
        static const uint64_t cap_blocks = [] {
            const int64_t v = env_knob("CFWS_SLOT_GRID", 0);   // 0: one iteration per wave
            return v > 0 ? (uint64_t)v : 0x7fffffffull;
        }();
        const uint64_t want = (n + per_block - 1) / per_block;
        const uint32_t grid = (uint32_t)(want < cap_blocks ? want : cap_blocks);
        auto window = [&](auto scatter, auto compact) {
            constexpr bool kSc = decltype(scatter)::value;
            constexpr bool kIn = decltype(compact)::value;
            if (S == 8)
                deserialize_slots_window_kernel<CFWS_SLOT_ROUNDS8, 8, kSc, kIn><<<grid, kThreads, 0, st>>>(
                    w, wire_size, d_index, n, max_payload, slot, G, d_desc, d_status, out, cap, d_total, dst, d_info,
                    stride, d_mismatch);
            else if (S == 4)
                deserialize_slots_window_kernel<CFWS_SLOT_ROUNDS4, 4, kSc, kIn><<<grid, kThreads, 0, st>>>(
                    w, wire_size, d_index, n, max_payload, slot, G, d_desc, d_status, out, cap, d_total, dst, d_info,
                    stride, d_mismatch);
            else if (S == 2)
                deserialize_slots_window_kernel<CFWS_SLOT_ROUNDS2, 2, kSc, kIn><<<grid, kThreads, 0, st>>>(
                    w, wire_size, d_index, n, max_payload, slot, G, d_desc, d_status, out, cap, d_total, dst, d_info,
                    stride, d_mismatch);
            else if (P > 1)
                deserialize_slots_window_kernel<CFWS_SLOT_ROUNDS_MULTI, 1, kSc, kIn><<<grid, kThreads, 0, st>>>(
                    w, wire_size, d_index, n, max_payload, slot, G, d_desc, d_status, out, cap, d_total, dst, d_info,
                    stride, d_mismatch);
            else
                deserialize_slots_window_kernel<CFWS_SLOT_ROUNDS, 1, kSc, kIn><<<grid, kThreads, 0, st>>>(
                    w, wire_size, d_index, n, max_payload, slot, G, d_desc, d_status, out, cap, d_total, dst, d_info,
                    stride, d_mismatch);
        };
        // the scatter form as its own instantiation: its per-round offset
        // shuffle, as a run-time branch in one kernel, cost the 1 KiB slot
        // receive 11 % (1.525 -> 1.70 ms)
        if (scatter && info)
            window(std::true_type{}, std::true_type{});
        else if (scatter)
            window(std::true_type{}, std::false_type{});
        else if (info)
            window(std::false_type{}, std::true_type{});
        else
            window(std::false_type{}, std::false_type{});
    } else if (route == kSlotsPiece) {
        // waves per frame: the slot's pieces, at most the pieces of the
        // batch's average frame (its wire bytes; at least one)
        const uint64_t slot_pieces = (slot + kSlotPiece - 1) / kSlotPiece;
        const uint64_t avg_pieces = (wire_size / n + kSlotPiece - 1) / kSlotPiece;
        const uint64_t pieces = avg_pieces < 1 ? 1 : avg_pieces < slot_pieces ? avg_pieces : slot_pieces;
        const bool loop = pieces < slot_pieces;
        const uint64_t waves = n * pieces;
        const uint64_t want = (waves + kWaves - 1) / kWaves;
        const uint32_t grid = (uint32_t)(want < (1u << 22) ? want : (1u << 22));   // a grid-stride loop past that
        auto piecewise = [&](auto scatter, auto compact) {
            constexpr bool kSc = decltype(scatter)::value, kIn = decltype(compact)::value;
            if (loop)
                deserialize_slots_piece_kernel<kSc, kIn, true><<<grid, kThreads, 0, st>>>(
                    w, wire_size, d_index, n, max_payload, slot, d_desc, d_status, out, cap, d_total, dst, d_info,
                    stride, d_mismatch, pieces);
            else
                deserialize_slots_piece_kernel<kSc, kIn, false><<<grid, kThreads, 0, st>>>(
                    w, wire_size, d_index, n, max_payload, slot, d_desc, d_status, out, cap, d_total, dst, d_info,
                    stride, d_mismatch, pieces);
        };
        if (scatter && info)
            piecewise(std::true_type{}, std::true_type{});
        else if (scatter)
            piecewise(std::true_type{}, std::false_type{});
        else if (info)
            piecewise(std::false_type{}, std::true_type{});
        else
            piecewise(std::false_type{}, std::false_type{});
    } else {
        auto one = [&](auto scatter, auto compact) {
            deserialize_slots_kernel<decltype(scatter)::value, decltype(compact)::value>
                <<<grid_for(n, kThreads), kThreads, 0, st>>>(w, wire_size, d_index, n, max_payload, slot, d_desc,
                                                             d_status, out, cap, d_total, dst, d_info, stride,
                                                             d_mismatch);
        };
        if (scatter && info)
            one(std::true_type{}, std::true_type{});
        else if (scatter)
            one(std::true_type{}, std::false_type{});
        else if (info)
            one(std::false_type{}, std::true_type{});
        else
            one(std::false_type{}, std::false_type{});
    }
    return launch_check(what);
}

}  // namespace

extern "C" {

int cfws_deserialize_slots(const void* d_wire, uint64_t wire_size, const uint64_t* d_index, size_t n,
                           uint64_t max_payload, uint64_t slot, cfws_frame_desc_t* d_desc, int32_t* d_status,
                           void* d_payload, uint64_t cap, uint64_t* d_total, void* stream)
{
    const CfwsPassScope pass_scope;
    return slots_impl(d_wire, wire_size, d_index, nullptr, n, max_payload, slot, d_desc, d_status, d_payload, cap,
                      d_total, stream, false, "deserialize_slots");
}

int cfws_deserialize_scatter(const void* d_wire, uint64_t wire_size, const uint64_t* d_index,
                             const uint64_t* d_payload_off, size_t n, uint64_t max_payload, uint64_t max_slot,
                             cfws_frame_desc_t* d_desc, int32_t* d_status, void* d_payload, uint64_t cap,
                             void* stream)
{
    const CfwsPassScope pass_scope;
    return slots_impl(d_wire, wire_size, d_index, d_payload_off, n, max_payload, max_slot, d_desc, d_status,
                      d_payload, cap, nullptr, stream, true, "deserialize_scatter");
}

int cfws_deserialize_slots_info(const void* d_wire, uint64_t wire_size, const uint64_t* d_index, size_t n,
                                uint64_t max_payload, uint64_t slot, cfws_frame_info_t* d_info, void* d_payload,
                                uint64_t cap, uint64_t* d_total, void* stream)
{
    const CfwsPassScope pass_scope;
    if (!d_info && n) return set_err(CFWS_ERROR_INVALID_ARGUMENT, "null pointer", hipSuccess);
    return slots_impl(d_wire, wire_size, d_index, nullptr, n, max_payload, slot, nullptr, nullptr, d_payload, cap,
                      d_total, stream, false, "deserialize_slots_info", d_info);
}

int cfws_deserialize_scatter_info(const void* d_wire, uint64_t wire_size, const uint64_t* d_index,
                                  const uint64_t* d_payload_off, size_t n, uint64_t max_payload, uint64_t max_slot,
                                  cfws_frame_info_t* d_info, void* d_payload, uint64_t cap, void* stream)
{
    const CfwsPassScope pass_scope;
    if (!d_info && n) return set_err(CFWS_ERROR_INVALID_ARGUMENT, "null pointer", hipSuccess);
    return slots_impl(d_wire, wire_size, d_index, d_payload_off, n, max_payload, max_slot, nullptr, nullptr,
                      d_payload, cap, nullptr, stream, true, "deserialize_scatter_info", d_info);
}

int cfws_deserialize_slots_uniform(const void* d_wire, uint64_t wire_size, size_t n, uint64_t stride,
                                   uint64_t max_payload, uint64_t slot, cfws_frame_info_t* d_info, void* d_payload,
                                   uint64_t cap, uint64_t* d_total, uint32_t* d_mismatch, void* stream)
{
    const CfwsPassScope pass_scope;
    if (int rc = check_init()) return rc;
    if (stride < 2 || (n && stride > (1ull << 63) / n))
        return set_err(CFWS_ERROR_INVALID_ARGUMENT, "frame stride must be >= 2 and n * stride < 2^63", hipSuccess);
    if (!d_info && n) return set_err(CFWS_ERROR_INVALID_ARGUMENT, "null pointer", hipSuccess);
    if (d_mismatch && hipMemsetAsync(d_mismatch, 0, sizeof(uint32_t), static_cast<hipStream_t>(stream)) != hipSuccess)
        return launch_check("deserialize_slots_uniform");
    return slots_impl(d_wire, wire_size, nullptr, nullptr, n, max_payload, slot, nullptr, nullptr, d_payload, cap,
                      d_total, stream, false, "deserialize_slots_uniform", d_info, stride, d_mismatch);
}

const char* cfws_deserialize_slots_pass_kernel(size_t n, uint64_t wire_size, uint64_t slot)
{
    switch (slots_route(slot, n, wire_size)) {
    case kSlotsWindow: return "deserialize_slots_window_kernel";
    case kSlotsPiece: return "deserialize_slots_piece_kernel";
    default: return "deserialize_slots_kernel";
    }
}

#if CFWS_PLAN_TRACE
// tools/plan_trace.py: the last traced launch's stamps, blocks [0, n)
int cfws_debug_plan_trace(void* out, size_t n)
{
    if (n > kTraceBlocks) n = kTraceBlocks;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_plan_trace), n * 4 * sizeof(uint64_t)) == hipSuccess ? 0 : -1;
}
#endif

}  // extern "C"
