// cfws_h2.hip -- WebSocket over HTTP/2 (src/ws_http2) on the device: DATA-frame
// wrap of serialized WS frames (co_http2_stream_send_ws_frame ->
// co_http2_stream_send_data, co_http2_frame.c:33-72) and the receive side's
// DATA parse, pooling and per-message WS deserialize
// (co_http2_stream_receive_ws_frame, co_ws_http2_extension.c:134-164);
// batch C ABI cfws_h2_* (include/cfws.h). DESIGN.md section 3.4.
#include "cfws_kernels.h"

#include <mutex>
#include <vector>

namespace {

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
                          uint64_t* __restrict__ partials_w, uint64_t* __restrict__ partials_k,
                          uint32_t* __restrict__ inreg_flag)
{
    __shared__ uint64_t s_wave[kWaves];
    const uint64_t f = uint64_t(blockIdx.x) * kThreads + threadIdx.x;
    if (f == 0) *inreg_flag = 0;                         // the apply kernel ORs misses in
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
// bytes at 9 d + wire offset (h2_expand_kernel's output layout); its
// descriptor holds what the send pass reads per region (see the loop).
__global__ void __launch_bounds__(kThreads)
h2_ser_plan_apply_kernel(cfws_frame_desc_t* __restrict__ desc, uint64_t n, uint64_t S,
                         const uint64_t* __restrict__ partials_w, const uint64_t* __restrict__ partials_k,
                         uint64_t nb, uint32_t self_scan, uint64_t* __restrict__ hdr, uint64_t capacity,
                         uint64_t n_max, cfws_frame_desc_t* __restrict__ ddesc,
                         uint64_t* __restrict__ doffs, uint32_t* __restrict__ map,
                         uint64_t* __restrict__ user_total, uint32_t* __restrict__ inreg_flag)
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
    DescWords wd = {};
    if (f < n) {
        wd = load_desc(desc, (uint32_t)f);
        w = wd.header_size() + wd.payload_size;
        k = data_frames_of(w, S);
    }
    uint64_t tot;
    const uint64_t w0 = block_exclusive_scan(w, s_wave, &tot) + pre_w;
    const uint64_t d0 = block_exclusive_scan(k, s_wave, &tot) + pre_k;
    if (f < n) {
        desc[f].wire_off = w0;
        const uint64_t hs = wd.header_size();
        for (uint64_t j = 0; j < k; ++j) {
            const uint64_t d = d0 + j;
            if (d >= n_max) break;
            // DATA frame d: slice [s0, s0 + len) of WS frame f's wire bytes,
            // h_in of them header; stored as the send pass reads it
            // (frame_view<kModeH2Ser>): body source offset and length, key
            // rotated to the body's first payload index, bytes before the
            // body (9 + h_in), END_STREAM; for the first slice (h_in > 0:
            // with S >= 64 the whole WS header, s0 = 0) the WS header's
            // fields: payload size in wire_off, byte 0 in opcode, the mask
            // bit (the output offset is doffs[d])
            const uint64_t s0 = j * S;
            const uint64_t len = (j + 1 < k) ? S : w - s0;
            const uint64_t h_in = s0 < hs ? (hs - s0 < len ? hs - s0 : len) : 0;
            const uint64_t q = s0 + h_in - hs;           // payload index of the body start
            cfws_frame_desc_t e;
            e.payload_off = wd.payload_off + q;
            e.wire_off = h_in ? wd.payload_size : 0;
            e.payload_size = len - h_in;
            e.mask_key = wd.mask() ? rotr8(wd.key(), (uint32_t)(q & 3u)) : 0u;
            e.fin = (j + 1 == k) ? 1 : 0;
            e.opcode = h_in ? (uint8_t)((wd.opcode() | (wd.fin() ? 0x80u : 0u)) & 0xffu) : 0;
            e.mask = h_in && wd.mask() ? 1 : 0;
            e.header_size = (uint8_t)(9 + h_in);
            ddesc[d] = e;
            const uint64_t out = 9 * d + w0 + s0;
            doffs[d] = out;
            // the send's in-region edge chunks need every DATA frame but the
            // stream's last to span a region and more (two_frame_region)
            if (9 + len < kRegion + 32 && d + 1 < gk) atomicOr(inreg_flag, 1u);
            // DATA frames lie back to back: this one ends where d + 1 starts
            map_range(out, out + 9 + len, d, total, map);
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
                        uint64_t* __restrict__ first, uint64_t* __restrict__ host_counts)
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
    // message count and pooled total straight to the caller thread's mapped
    // host words (read after one stream synchronize)
    if (host_counts && blockIdx.x == 0 && threadIdx.x == 0) {
        host_counts[0] = ge;
        host_counts[1] = gp;
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
                    const uint64_t* __restrict__ ends, const uint64_t* __restrict__ n_msg_p,
                    uint64_t max_payload,
                    uint64_t align, cfws_frame_desc_t* __restrict__ mdesc,
                    int32_t* __restrict__ mstatus, uint64_t* __restrict__ vals,
                    const uint64_t* __restrict__ first, uint64_t* __restrict__ partials)
{
    __shared__ uint64_t s_wave[kWaves];
    const uint64_t m = uint64_t(blockIdx.x) * kThreads + threadIdx.x;
    const uint64_t n_msg = *n_msg_p;
    uint64_t v = 0;
    if (m >= n_msg && m < n_h2) {
        // rows past the message count (the grid is sized before the host
        // knows it): empty entries, no payload, so the layout over n_h2 rows
        // equals the layout over the messages
        cfws_frame_desc_t e = {};
        mdesc[m] = e;
        mstatus[m] = CFWS_PARSE_MORE_DATA;
        vals[m] = 0;
    }
    if (m < n_msg) {
        const uint64_t s = starts[m], len = ends[m] - s;
        const uint32_t k = len < 14 ? (uint32_t)len : 14u;
        uint64_t d = first[m];
        const uint64_t l0 = h2_status[d] == CFWS_H2_PARSE_COMPLETE ? pdesc[d].payload_size : 0;
        uint32_t w[4] = {0u, 0u, 0u, 0u};
        if (s + k <= poff[d] + l0) {
            // the whole header in the first DATA frame (every frame of >= 14
            // bytes): the aligned dwords holding [b, b + k), issued together
            // (a byte loop here compiled to one memory round trip per byte)
            load_span16(h2 + pdesc[d].wire_off + pdesc[d].header_size + (s - poff[d]), k, w);
        } else {
            // the header straddles DATA frames: walk them byte by byte
#pragma unroll
            for (uint32_t i = 0; i < 14; ++i) {
                if (i >= k) break;
                const uint64_t p = s + i;
                while (p >= poff[d] + (h2_status[d] == CFWS_H2_PARSE_COMPLETE ? pdesc[d].payload_size : 0))
                    ++d;
                w[i >> 2] |= (uint32_t)h2[pdesc[d].wire_off + pdesc[d].header_size + (p - poff[d])]
                             << (8u * (i & 3u));
            }
        }
        cfws_frame_desc_t dd;
        const int32_t st = parse_ws_header_regs(w, len, max_payload, dd);
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
// DATA frame d of message m (descriptor M, status ms, pooled start s_m);
// `past`: the layout's end, the output offset of a frame in no message.
__device__ __forceinline__ uint64_t h2_unit_of(const cfws_frame_desc_t* __restrict__ pdesc,
                                               const int32_t* __restrict__ h2_status,
                                               const uint64_t* __restrict__ poff, uint64_t d, bool in_msg,
                                               uint64_t s_m, const cfws_frame_desc_t& M, int32_t ms,
                                               uint64_t past, cfws_frame_desc_t& u)
{
    u = {};
    uint64_t out = past;
    if (in_msg) {
        const uint64_t hs = M.header_size;
        // the message's layout span: payload_size when it parsed (an OOM
        // frame keeps its layout), else nothing
        const uint64_t span = (ms == CFWS_PARSE_COMPLETE || ms == CFWS_ERROR_OUT_OF_MEMORY)
                                  ? M.payload_size : 0;
        const uint64_t a = poff[d] - s_m;
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
    const bool in_msg = m < n_msg;
    cfws_frame_desc_t M = {};
    int32_t ms = CFWS_PARSE_MORE_DATA;
    uint64_t s_m = 0;
    if (in_msg) {
        M = mdesc[m];
        ms = mstatus[m];
        s_m = starts[m];
    }
    return h2_unit_of(pdesc, h2_status, poff, d, in_msg, s_m, M, ms, hdr[3], u);
}

// One thread per DATA frame: its unit, and the region map of the payload
// pass (a unit ends where unit d + 1 starts, computed here too, so no
// second launch reads uoffs). *pass_total: the payload pass's total, or 0
// (the pass then stores nothing) when the pooled bytes exceed the pool
// capacity and the general form redoes the call.
__global__ void __launch_bounds__(kThreads)
h2_units_kernel(const cfws_frame_desc_t* __restrict__ pdesc, const int32_t* __restrict__ h2_status,
                const uint64_t* __restrict__ poff, const uint64_t* __restrict__ msg_id, uint64_t n,
                const uint64_t* __restrict__ n_msg_p, const uint64_t* __restrict__ starts,
                const cfws_frame_desc_t* __restrict__ mdesc, const int32_t* __restrict__ mstatus,
                const uint64_t* __restrict__ hdr, cfws_frame_desc_t* __restrict__ udesc,
                int32_t* __restrict__ ustatus, uint64_t* __restrict__ uoffs, uint32_t* __restrict__ map,
                const uint64_t* __restrict__ pooled_p, uint64_t pool_cap, uint64_t* __restrict__ pass_total)
{
    const uint64_t d = uint64_t(blockIdx.x) * kThreads + threadIdx.x;
    if (d == 0) *pass_total = *pooled_p <= pool_cap ? hdr[0] : 0;
    if (d >= n) return;
    const uint64_t n_msg = *n_msg_p;
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


// Messages of at most this many DATA frames in a wave are walked by their own
// thread; a wave holding a longer one deals its frames out over its lanes.
constexpr uint64_t kUnitsPerThread = 8;

// deserialize_plan_apply_kernel (one message per thread, no reassembly) and
// h2_units_kernel in one launch (CFWS_H2_UNITS_MERGED, default): the
// thread of message m lays it out (payload offset, the capacity rule, the
// message map, the totals), then writes the units of m's DATA frames
// [first[m], first[m + 1]) -- all from values it holds: a frame's unit
// needs only its message's descriptor, and the last frame's unit ends
// where message m + 1's layout starts, m's offset + its aligned size. The
// frames after the last END_STREAM (in no message) go to the threads in
// turn. One launch less on the receive (config 5: 7 plan kernels -> 6).
__global__ void __launch_bounds__(kThreads)
h2_msg_apply_units_kernel(cfws_frame_desc_t* __restrict__ mdesc, int32_t* __restrict__ mstatus,
                          uint64_t* __restrict__ vals, uint64_t n, const uint64_t* __restrict__ partials,
                          uint64_t nb, uint32_t self_scan, uint64_t* __restrict__ hdr, uint64_t capacity,
                          uint32_t* __restrict__ mmap, uint64_t* __restrict__ user_total,
                          const cfws_frame_desc_t* __restrict__ pdesc, const int32_t* __restrict__ h2_status,
                          const uint64_t* __restrict__ poff, const uint64_t* __restrict__ n_msg_p,
                          const uint64_t* __restrict__ starts, const uint64_t* __restrict__ first,
                          cfws_frame_desc_t* __restrict__ udesc, int32_t* __restrict__ ustatus,
                          uint64_t* __restrict__ uoffs, uint32_t* __restrict__ umap,
                          const uint64_t* __restrict__ pooled_p, uint64_t pool_cap,
                          uint64_t* __restrict__ pass_total)
{
    static_assert(kPlanItems == 1, "one message per thread");
    __shared__ uint64_t s_wave[kWaves];
    uint64_t pre, g;
    if (self_scan) {
        prefix_from_partials(partials, nb, blockIdx.x, s_wave, pre, g);
    } else {
        pre = partials[blockIdx.x];
        g = hdr[3];
    }
    const uint64_t t = g < capacity ? g : capacity;
    const uint64_t m = uint64_t(blockIdx.x) * kThreads + threadIdx.x;
    const uint64_t v = m < n ? vals[m] : 0;
    uint64_t tot;
    const uint64_t run = block_exclusive_scan(v, s_wave, &tot) + pre;
    const uint64_t n_msg = *n_msg_p;
    cfws_frame_desc_t M = {};
    int32_t ms = CFWS_PARSE_MORE_DATA;
    if (m < n) {
        // deserialize_plan_apply_kernel's row m
        vals[m] = run;
        M = mdesc[m];
        M.payload_off = run;
        mdesc[m].payload_off = run;
        ms = mstatus[m];
        if (ms == CFWS_PARSE_COMPLETE && M.payload_size > 0 && run + M.payload_size > capacity) {
            ms = CFWS_ERROR_OUT_OF_MEMORY;
            mstatus[m] = ms;
        }
        map_range(run, run + v, m, t, mmap);
        if (m == n - 1) {
            mmap[(t + kRegion - 1) / kRegion] = (uint32_t)m;
            hdr[0] = t;
            hdr[1] = 0;
            hdr[2] = t;
            if (self_scan) hdr[3] = g;
            if (user_total) *user_total = t;
        }
    }
    if (m == 0) *pass_total = *pooled_p <= pool_cap ? t : 0;
    // the units of message m's DATA frames [d0, d1)
    uint64_t d0 = 0, d1 = 0, s_m = 0, next = 0;
    if (m < n_msg) {
        d0 = first[m];
        d1 = m + 1 < n_msg ? first[m + 1] : (n_msg < n ? first[n_msg] : n);
        s_m = starts[m];
        next = m + 1 < n_msg ? run + v : g;                   // where the next unit starts
    }
    const uint64_t cnt = d1 - d0;
    uint64_t wmax = cnt;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        const uint64_t y = __shfl_xor(wmax, o, 64);
        wmax = y > wmax ? y : wmax;
    }
    if (wmax <= kUnitsPerThread) {
        // short messages (config 5: one or two DATA frames each): each
        // thread walks its own, one unit computed per frame
        if (cnt) {
            cfws_frame_desc_t u, u1;
            uint64_t lo = h2_unit_of(pdesc, h2_status, poff, d0, true, s_m, M, ms, g, u);
            for (uint64_t d = d0; d < d1; ++d) {
                const uint64_t hi = d + 1 < d1 ? h2_unit_of(pdesc, h2_status, poff, d + 1, true, s_m, M, ms, g, u1)
                                               : next;
                udesc[d] = u;
                ustatus[d] = CFWS_PARSE_COMPLETE;
                uoffs[d] = lo;
                map_range(lo, hi, d, t, umap);
                lo = hi;
                u = u1;
            }
        }
    } else {
        // a long message in the wave (a multi-MiB message is hundreds to
        // thousands of DATA frames): the wave's frames are dealt out 64 at a
        // time over all its lanes, each lane finding its frame's message by a
        // binary search over the lanes' inclusive counts, that message's
        // fields over shuffles (one lane walking thousands of
        // frames serialized the kernel on it)
        const uint32_t lane = threadIdx.x & 63u;
        uint64_t inc = cnt;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint64_t y = __shfl_up(inc, o, 64);
            if (lane >= (uint32_t)o) inc += y;
        }
        const uint64_t total = __shfl(inc, 63, 64);
        const uint64_t exc = inc - cnt;
        for (uint64_t base = 0; base < total; base += 64) {
            const uint64_t i = base + lane;
            int o = 0;
#pragma unroll
            for (int step = 32; step >= 1; step >>= 1) {
                const uint64_t x = __shfl(inc, o + step - 1, 64);
                if (x <= i) o += step;
            }
            // the owner's message, every lane taking part in the shuffles
            cfws_frame_desc_t Mo = {};
            Mo.payload_off = __shfl(M.payload_off, o, 64);
            Mo.payload_size = __shfl(M.payload_size, o, 64);
            Mo.header_size = (uint8_t)__shfl((int)M.header_size, o, 64);
            Mo.mask = (uint8_t)__shfl((int)M.mask, o, 64);
            Mo.mask_key = (uint32_t)__shfl((int)M.mask_key, o, 64);
            const int32_t mso = __shfl(ms, o, 64);
            const uint64_t s_o = __shfl(s_m, o, 64), d0o = __shfl(d0, o, 64), d1o = __shfl(d1, o, 64);
            const uint64_t exo = __shfl(exc, o, 64), nexto = __shfl(next, o, 64);
            if (i >= total) continue;
            const uint64_t d = d0o + (i - exo);
            cfws_frame_desc_t u, u1;
            const uint64_t lo = h2_unit_of(pdesc, h2_status, poff, d, true, s_o, Mo, mso, g, u);
            const uint64_t hi = d + 1 < d1o ? h2_unit_of(pdesc, h2_status, poff, d + 1, true, s_o, Mo, mso, g, u1)
                                            : nexto;
            udesc[d] = u;
            ustatus[d] = CFWS_PARSE_COMPLETE;
            uoffs[d] = lo;
            map_range(lo, hi, d, t, umap);
        }
    }
    // frames in no message: empty units at the layout's end
    const uint64_t tail0 = n_msg < n ? first[n_msg] : n;
    for (uint64_t d = tail0 + m; d < n; d += uint64_t(gridDim.x) * kThreads) {
        cfws_frame_desc_t e = {};
        udesc[d] = e;
        ustatus[d] = CFWS_PARSE_COMPLETE;
        uoffs[d] = g;
        map_range(g, g, d, t, umap);
    }
    if (m == 0 && n > 0) umap[(t + kRegion - 1) / kRegion] = (uint32_t)(n - 1);
}

}  // namespace

namespace {

// The receive-plan handoff: two mapped host words for the message count and
// pooled total (h2_de_plan_apply_kernel writes them) and an event recorded
// after the plan. The host waits on that event alone while the rest of the
// call runs on. One entry per device of the call's STREAM (an event and the
// words' device pointer belong to the device the kernels run on, which need
// not be the thread's current device).
struct CountWords {
    uint64_t* h = nullptr;
    uint64_t* d = nullptr;
    hipEvent_t ev = nullptr;
};

// Devices past kCountDevices, and any entry that cannot be made, use the
// copies (read_counts).
constexpr int kCountDevices = 16;

// Entries are made once and never freed: a host thread borrows one per device
// on its first call and its thread_local holder hands it back at thread exit
// (no HIP call at exit, so the runtime's own teardown order does not matter).
// A server whose worker threads come and go reuses the same few entries: the
// process holds at most one per device per thread alive at once.
struct CountPool {
    std::mutex mu;
    std::vector<CountWords*> free_list[kCountDevices];
};

CountPool& count_pool()
{
    static CountPool* pool = new CountPool;   // outlives every thread's holder
    return *pool;
}

struct CountHolder {
    CountWords* w[kCountDevices] = {};
    bool tried[kCountDevices] = {};
    ~CountHolder()
    {
        CountPool& pool = count_pool();
        std::lock_guard<std::mutex> lock(pool.mu);
        for (int i = 0; i < kCountDevices; ++i)
            if (w[i]) pool.free_list[i].push_back(w[i]);
    }
};

CountWords* make_count_words(int dev)
{
    int cur = -1;
    if (hipGetDevice(&cur) != hipSuccess) return nullptr;
    if (cur != dev && hipSetDevice(dev) != hipSuccess) return nullptr;
    CountWords* cw = nullptr;
    void* p = nullptr;
    void* q = nullptr;
    hipEvent_t ev = nullptr;
    if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) == hipSuccess) {
        if (hipHostMalloc(&p, 64, hipHostMallocMapped | hipHostMallocPortable) == hipSuccess) {
            if (hipHostGetDevicePointer(&q, p, 0) == hipSuccess && q) {
                cw = new CountWords;
                cw->h = static_cast<uint64_t*>(p);
                cw->d = static_cast<uint64_t*>(q);
                cw->ev = ev;
            } else {
                (void)hipHostFree(p);
            }
        }
        if (!cw) (void)hipEventDestroy(ev);
    }
    if (cur != dev) (void)hipSetDevice(cur);
    (void)hipGetLastError();                 // a failure here only means: use the copies
    return cw;
}

// The calling thread's entry for device `dev`, or null (use the copies).
CountWords* count_words(int dev)
{
    thread_local CountHolder holder;
    if (dev < 0 || dev >= kCountDevices) return nullptr;
    if (holder.w[dev] || holder.tried[dev]) return holder.w[dev];
    holder.tried[dev] = true;
    {
        CountPool& pool = count_pool();
        std::lock_guard<std::mutex> lock(pool.mu);
        if (!pool.free_list[dev].empty()) {
            holder.w[dev] = pool.free_list[dev].back();
            pool.free_list[dev].pop_back();
            return holder.w[dev];
        }
    }
    holder.w[dev] = make_count_words(dev);
    return holder.w[dev];
}

// The device the stream's work runs on (the null stream: the current device).
int stream_device(hipStream_t st)
{
    hipDevice_t dev = -1;
    if (hipStreamGetDevice(st, &dev) != hipSuccess) {
        (void)hipGetLastError();
        return -1;
    }
    return dev;
}

}  // namespace

extern "C" {

// ---- WebSocket over HTTP/2 -------------------------------------------------

namespace {

// CFWS_H2_INREG=1: the fused send's two-frame regions write the edge chunks
// of a batch whose DATA frames (all but the last) span more than a region
// (two_frame_region<kModeH2Ser, true>). Off by default: on config 5 it cut
// the sub-64-byte write requests from 160 K to 47 K per launch and the
// wave-cycles by 8.6 %, yet the step ran 0.5-1.5 % slower on the same box
// (profiles/r04/h2_inreg_ab/). Parity-tested both ways.
// CFWS_H2_UNITS_MERGED=0: the receive's message layout and its payload-pass
// units as two launches (A/B knob)
bool h2_units_merged()
{
    static const bool v = env_knob("CFWS_H2_UNITS_MERGED", 1) != 0;
    return v;
}

bool h2_inreg()
{
    static const bool v = env_knob("CFWS_H2_INREG", 0) != 0;
    return v;
}

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

static H2SerLayout h2_ser_layout(uint64_t n, uint64_t wire_cap, uint64_t h2_cap, uint64_t S)
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
    uint64_t pass_total; // u64: the fused payload pass's total (0: the pool overflowed)
    uint64_t starts, ends;   // u64[n_h2]
    uint64_t first;      // u64[n_h2]: a message's first DATA frame
    uint64_t wsd;        // WS deserialize workspace
    uint64_t udesc;      // cfws_frame_desc_t[n_h2]: fused payload-pass units
    uint64_t ustatus;    // int32[n_h2]
    uint64_t bytes;
};

static H2DeLayout h2_de_layout(uint64_t n, uint64_t pool_cap, uint64_t payload_cap)
{
    H2DeLayout L;
    uint64_t at = 0;
    L.pool = at; at = align_up(at + ws_layout(n, pool_cap).bytes, 256);
    L.pdesc = at; at = align_up(at + sizeof(cfws_frame_desc_t) * n, 256);
    L.es = at; at = align_up(at + 8 * n, 256);
    L.es_part = at; at = align_up(at + 8 * ((n + kScanBlock - 1) / kScanBlock + 1), 256);
    L.es_total = at; at += 256;
    L.pass_total = at; at += 256;
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
    const CfwsPassScope pass_scope;
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
    // clear: every DATA frame but the last spans more than a region, and
    // the send's two-frame regions write the edge chunks (kEdges)
    uint32_t* inreg = reinterpret_cast<uint32_t*>(hdr + 8);
    if (fused) {
        // WS layout + DATA frames + region map in two launches (three above
        // kSelfScanBlocks blocks)
        const uint32_t nb = grid_for(n, kPlanBlock);
        const uint32_t self_scan = nb <= kSelfScanBlocks ? 1u : 0u;
        uint64_t* pw = ws_ptr<uint64_t>(ws, WL.partials[0]);
        uint64_t* pk = ws_ptr<uint64_t>(ws, WL.partials[1]);
        h2_ser_plan_reduce_kernel<<<nb, kThreads, 0, st>>>(d_desc, n, S, pw, pk, inreg);
        if (!self_scan) scan_partials2_kernel<<<2, kThreads, 0, st>>>(pw, pk, nb, hdr + 4, hdr + 5);
        h2_ser_plan_apply_kernel<<<nb, kThreads, 0, st>>>(d_desc, n, S, pw, pk, nb, self_scan, hdr,
                                                         h2_cap, L.n_max, ddesc, doffs, map, d_h2_total,
                                                         inreg);
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
                                     L.regions, h2_cap, L.n_max, kClassAll, stream_id, st, d_desc, true,
                                     nullptr, h2_inreg() ? inreg : nullptr);
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
    const CfwsPassScope pass_scope;
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
    if (align == 0 || (align & (align - 1)) || align > 4096)
        return set_err(CFWS_ERROR_INVALID_ARGUMENT, "align must be a power of two <= 4096", hipSuccess);
    uint64_t counts[2] = {0, 0};       // messages, pooled bytes
    CountWords* cw = count_words(stream_device(st));
    {
        const uint32_t nb = grid_for(n, kPlanBlock);
        const uint32_t self_scan = nb <= kSelfScanBlocks ? 1u : 0u;
        uint64_t* pp = ws_ptr<uint64_t>(pws, PL.partials[0]);
        uint64_t* pe = ws_ptr<uint64_t>(pws, PL.partials[1]);
        h2_de_plan_reduce_kernel<<<nb, kThreads, 0, st>>>(h2, h2_size, d_h2_index, n, S, pdesc,
                                                          d_h2_status, pp, pe);
        if (!self_scan) scan_partials2_kernel<<<2, kThreads, 0, st>>>(pp, pe, nb, phdr + 3, n_msg_d);
        h2_de_plan_apply_kernel<<<nb, kThreads, 0, st>>>(pdesc, d_h2_status, n, pp, pe, nb, self_scan,
                                                         phdr, poffs, es, n_msg_d, starts, ends, first,
                                                         cw ? cw->d : nullptr);
    }
    // the plan's event; if it cannot be recorded, the copies below read the
    // counts instead (the words are still written, and nothing reads them)
    bool plan_event = false;
    if (cw) {
        plan_event = hipEventRecord(cw->ev, st) == hipSuccess;
        if (!plan_event) (void)hipGetLastError();
    }
    // an early return below still lets the plan finish first: the words are
    // the thread's, and a later call must not see this call's counts land
    auto fail = [&](int rc) {
        if (plan_event) (void)hipEventSynchronize(cw->ev);
        return rc;
    };
    void* wsd = ws_ptr<void>(ws, L.wsd);
    const WsLayout WL = ws_layout(n, payload_cap);
    uint64_t* hdr = ws_ptr<uint64_t>(wsd, WL.hdr);
    // 2. fused, queued before the host knows the message count (rows past it
    //    are empty): the pool is never written. Each message's WS header is
    //    gathered from its DATA frames and parsed against the message's own
    //    size (co_ws_http2_extension.c:134-164); then its layout. Valid when
    //    every DATA payload fits the pool capacity; otherwise the general
    //    form below rewrites every output after it, in stream order (the
    //    fused kernels store only inside the payload capacity).
    uint64_t* offs0 = ws_ptr<uint64_t>(wsd, WL.offs[0]);
    uint64_t* part0 = ws_ptr<uint64_t>(wsd, WL.partials[0]);
    const uint32_t mb = grid_for(n, kPlanBlock);
    const uint32_t m_self = mb <= kSelfScanBlocks ? 1u : 0u;
    h2_msg_parse_kernel<<<mb, kThreads, 0, st>>>(h2, pdesc, d_h2_status, poffs, n, starts, ends, n_msg_d,
                                                max_payload, align, d_msg_desc, d_msg_status, offs0,
                                                first, part0);
    if (!m_self) scan_partials_kernel<<<1, kThreads, 0, st>>>(part0, mb, hdr + 3);
    // 3. one payload-pass unit per DATA frame, and the pass's region map
    cfws_frame_desc_t* udesc = ws_ptr<cfws_frame_desc_t>(ws, L.udesc);
    int32_t* ustatus = ws_ptr<int32_t>(ws, L.ustatus);
    uint64_t* uoffs = ws_ptr<uint64_t>(wsd, WL.offs[1]);
    uint32_t* umap = ws_ptr<uint32_t>(wsd, WL.map[1]);
    // the pass's total, or 0 when the pool overflows (it then stores nothing;
    // the general form below does the call's work once)
    uint64_t* pass_total = ws_ptr<uint64_t>(ws, L.pass_total);
    if (h2_units_merged()) {
        h2_msg_apply_units_kernel<<<mb, kThreads, 0, st>>>(
            d_msg_desc, d_msg_status, offs0, n, part0, mb, m_self, hdr, payload_cap,
            ws_ptr<uint32_t>(wsd, WL.map[0]), d_payload_total, pdesc, d_h2_status, poffs, n_msg_d, starts,
            first, udesc, ustatus, uoffs, umap, phdr + 3, pool_cap, pass_total);
    } else {
        deserialize_plan_apply_kernel<<<mb, kThreads, 0, st>>>(
            d_msg_desc, d_msg_status, offs0, ws_ptr<uint64_t>(wsd, WL.offs[1]), n, part0,
            ws_ptr<uint64_t>(wsd, WL.partials[1]), mb, m_self, hdr, payload_cap, 0,
            ws_ptr<uint32_t>(wsd, WL.map[0]), ws_ptr<uint32_t>(wsd, WL.map[1]), d_payload_total);
        h2_units_kernel<<<grid_for(n, kThreads), kThreads, 0, st>>>(
            pdesc, d_h2_status, poffs, es, n, n_msg_d, starts, d_msg_desc, d_msg_status, hdr, udesc,
            ustatus, uoffs, umap, phdr + 3, pool_cap, pass_total);
    }
    // the call's timed pass (cfws_time_next_pass): this fused pass, or, when
    // the pool overflows and it stores nothing, the general form's passes
    // below (the pair is recorded again around them)
    const CfwsPassEvents timed = cfws_internal_take_pass();
    if (timed.start) (void)hipEventRecord(static_cast<hipEvent_t>(timed.start), st);
    if (payload_cap)
        launch_streaming<kModeDeser>(d_h2, d_payload, udesc, ustatus, uoffs, umap, pass_total, nullptr,
                                     WL.regions, payload_cap, n, kClassAll, 0, st);
    if (timed.stop) (void)hipEventRecord(static_cast<hipEvent_t>(timed.stop), st);
    if (int rc = launch_check("h2_deserialize")) return fail(rc);
    auto read_counts = [&]() -> int {
        hipError_t e = hipMemcpyAsync(&counts[0], n_msg_d, 8, hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipMemcpyAsync(&counts[1], phdr + 3, 8, hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e != hipSuccess) return set_err(CFWS_ERROR_HIP, "h2_deserialize message count", e);
        return CFWS_OK;
    };
    if (plan_event) {
        // the plan's event only: the kernels above keep the device busy while
        // the host reads the counts (a stream synchronize here left it idle
        // 25-46 us per call on config 5)
        const hipError_t e = hipEventSynchronize(cw->ev);
        if (e != hipSuccess) return set_err(CFWS_ERROR_HIP, "h2_deserialize message count", e);
        const volatile uint64_t* hw = cw->h;
        counts[0] = hw[0];
        counts[1] = hw[1];
    } else if (int rc = read_counts()) {
        return rc;
    }
    if (counts[1] <= pool_cap) {
        if (n_messages) *n_messages = (size_t)counts[0];
        return CFWS_OK;
    }
    // 2'. general form: the pool capacity cuts DATA payloads, and a frame
    //     past it is OUT_OF_MEMORY and closes no message. Pool offsets and
    //     the grand total stand; the capacity rule, END_STREAM flags and
    //     messages are redone (co_http2_stream.c:550-608).
    deserialize_finalize_kernel<<<grid_for(n, kThreads), kThreads, 0, st>>>(
        pdesc, d_h2_status, poffs, poffs, phdr, n, pool_cap, 0, ws_ptr<uint32_t>(pws, PL.map[0]),
        ws_ptr<uint32_t>(pws, PL.map[1]), nullptr);
    h2_end_flags_kernel<<<grid_for(n, kThreads), kThreads, 0, st>>>(pdesc, d_h2_status, n, es);
    if (int rc = run_scan(es, n, ws_ptr<uint64_t>(ws, L.es_part), n_msg_d, st)) return rc;
    h2_messages_kernel<<<grid_for(n, kThreads), kThreads, 0, st>>>(pdesc, d_h2_status, es, n, ends);
    h2_starts_kernel<<<grid_for(n, kThreads), kThreads, 0, st>>>(ends, n_msg_d, n, starts);
    if (int rc = read_counts()) return rc;
    if (n_messages) *n_messages = (size_t)counts[0];
    // rows past the message count are empty entries, as in the fused form
    // (which wrote its own, longer, parse into some of them)
    if (counts[0] < n) {
        hipError_t e = hipMemsetAsync(d_msg_desc + counts[0], 0, sizeof(cfws_frame_desc_t) * (n - counts[0]), st);
        if (e == hipSuccess)
            e = hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(d_msg_status + counts[0]),
                                  CFWS_PARSE_MORE_DATA, n - counts[0], st);
        if (e != hipSuccess) return set_err(CFWS_ERROR_HIP, "h2_deserialize empty rows", e);
    }
    // 3'. each pooled message through co_ws_frame_deserialize against its
    //     own size (co_ws_http2_extension.c:134-164), from the materialised
    //     pool (layout-first OOM rule)
    if (timed.start) (void)hipEventRecord(static_cast<hipEvent_t>(timed.start), st);
    struct StopAtExit {
        const CfwsPassEvents& e;
        hipStream_t st;
        ~StopAtExit() { if (e.stop) (void)hipEventRecord(static_cast<hipEvent_t>(e.stop), st); }
    } stop_at_exit{timed, st};
    if (pool_cap)
        launch_pass<kModeDeser>(PL, 0, d_h2, d_pool, pdesc, d_h2_status, pws, pool_cap, n, kClassAll, st);
    if (int rc = deserialize_plan_impl(d_pool, pool_cap, starts, ends, counts[0], max_payload, align, 0,
                                       d_msg_desc, d_msg_status, payload_cap, d_payload_total, wsd,
                                       WL.bytes, stream))
        return rc;
    return cfws_deserialize_execute(d_pool, d_msg_desc, d_msg_status, counts[0], 0, d_payload,
                                    payload_cap, wsd, stream);
}

}  // extern "C"

uint64_t cfws_internal_h2_grand_total_offset(uint64_t n_h2, uint64_t pool_cap, uint64_t payload_cap)
{
    return h2_de_layout(n_h2, pool_cap, payload_cap).wsd + ws_layout(n_h2, payload_cap).hdr +
           3 * sizeof(uint64_t);
}
