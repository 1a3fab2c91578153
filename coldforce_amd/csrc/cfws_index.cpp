// cfws_index.cpp -- receive-buffer frame indexing on the host (SURVEY §8 f#2).
//
// The frame walk of coldforce's receive loops, co_ws_server_on_tcp_receive_ready
// (src/ws/co_ws_server.c:107-169) and co_ws_client_on_tcp_receive_ready
// (src/ws/co_ws_client.c:200-270), without the per-frame payload copy: it
// only decodes the 2-14 header bytes of each frame (co_ws_frame.c:131-213)
// to find where the next one starts. The payloads are then copied + unmasked
// on the GPU by cfws_deserialize_* / cfws_pipeline_*. This is the host half
// of a receive loop whose bytes are in host memory (socket buffers); the
// device-resident form is cfws_index_frames_batch (cfws_ops.hip).
#include <cstdint>
#include <cstring>

#include "cfws.h"

namespace {

// Header at p of data[0, size) (size - p >= 2): COMPLETE and the frame's
// total length, or the code co_ws_frame_deserialize returns for it.
int32_t header_walk(const uint8_t* d, uint64_t size, uint64_t p, uint64_t max_payload,
                    uint64_t* frame_len)
{
    const uint64_t s = p;
    const uint32_t b0 = d[p], b1 = d[p + 1];
    p += 2;
    if ((b0 & 0x7fu) > 0x0f) return CFWS_ERROR_INVALID_FRAME;      // co_ws_frame.c:136-142
    uint64_t len = b1 & 0x7fu;
    if (len > 125) {                                                // :147-188
        const uint32_t ext = len == 126 ? 2u : 8u;
        if (size - p < ext) return CFWS_PARSE_MORE_DATA;
        len = 0;
        for (uint32_t i = 0; i < ext; ++i) len = (len << 8) | d[p + i];
        p += ext;
    }
    if (b1 & 0x80u) {                                               // :190-201
        if (size - p < 4) return CFWS_PARSE_MORE_DATA;
        p += 4;
    }
    if (size - p < len) return CFWS_PARSE_MORE_DATA;                // :203-206
    if (len > max_payload) return CFWS_ERROR_DATA_TOO_BIG;          // :208-213
    *frame_len = (p - s) + len;
    return CFWS_PARSE_COMPLETE;
}

}  // namespace

extern "C" {

size_t cfws_index_frames(const void* h_buf, uint64_t begin, uint64_t end, uint64_t max_payload,
                         uint64_t* starts, size_t max_starts, uint64_t* consumed, int32_t* stop)
{
    const uint8_t* d = static_cast<const uint8_t*>(h_buf);
    uint64_t p = begin;
    size_t k = 0;
    int32_t st = CFWS_PARSE_COMPLETE;
    while (end > p) {                                               // co_ws_server.c:107
        if (end - p < 2) { st = CFWS_PARSE_MORE_DATA; break; }      // :109-113
        uint64_t len = 0;
        st = header_walk(d, end, p, max_payload, &len);
        if (st != CFWS_PARSE_COMPLETE) break;                       // :144-166
        if (k == max_starts) { st = CFWS_INDEX_FULL; break; }       // resume at *consumed
        starts[k++] = p;
        p += len;                                                   // co_ws_frame.c:244
    }
    if (consumed) *consumed = p;
    if (stop) *stop = st;
    return k;
}

}  // extern "C"
