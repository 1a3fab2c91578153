/*
 * cfws_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of coldforce's WebSocket frame codec
 * (/root/reference/src/ws/co_ws_frame.c), used as the parity checker for the
 * MI355X batch codec in coldforce_amd/.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load this library; the product path
 * (libcfws.so) never links or calls it.
 *
 * Parity pinning: checked against (1) RFC 6455 section 5.7 known answers and
 * (2) golden vectors produced by the reference codec itself, compiled from
 * /root/reference by oracle/Makefile into oracle/_ref/ (tests/golden/).
 */
#ifndef CFWS_ORACLE_H
#define CFWS_ORACLE_H

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Reference return codes: inc/coldforce/ws/co_ws.h:25-39 */
#define ORC_PARSE_COMPLETE        0
#define ORC_PARSE_MORE_DATA       1
#define ORC_ERROR_INVALID_FRAME   (-7001)
#define ORC_ERROR_DATA_TOO_BIG    (-7005)
#define ORC_ERROR_OUT_OF_MEMORY   (-7006)

/* Frame object, same layout as co_ws_frame_t (co_ws_frame.h:36-49). */
typedef struct {
    bool fin;
    uint8_t opcode;
    uint64_t payload_size;
} orc_frame_header_t;

typedef struct {
    orc_frame_header_t header;
    uint8_t* payload_data;
} orc_frame_t;

/* Growable byte buffer, same layout and growth rule as co_array_t
 * (inc/coldforce/core/co_array.h, src/core/co_array.c:83-112,183-194). */
typedef struct {
    size_t capacity;
    size_t count;
    size_t element_size;
    uint8_t* buffer;
} orc_bytes_t;

/* Batch descriptor: same 32-byte layout as cfws_frame_desc_t (include/cfws.h). */
typedef struct {
    uint64_t payload_off;
    uint64_t wire_off;
    uint64_t payload_size;
    uint32_t mask_key;     /* key byte j = (mask_key >> 8j) & 0xff, j = wire order */
    uint8_t fin;
    uint8_t opcode;
    uint8_t mask;
    uint8_t header_size;
} orc_desc_t;

orc_bytes_t* orc_bytes_create(void);
void orc_bytes_destroy(orc_bytes_t* b);

/* co_ws_frame_serialize (co_ws_frame.c:21-119): key from random(). */
bool orc_serialize(bool fin, uint8_t opcode, bool mask, const void* data,
                   size_t data_size, orc_bytes_t* buffer);

/* Same wire bytes with an explicit key; writes to out, returns frame bytes. */
size_t orc_serialize_keyed(bool fin, uint8_t opcode, bool mask, uint32_t key,
                           const uint8_t* data, size_t data_size, uint8_t* out);

/* Header size a serialize of this frame produces (co_ws_frame.c:41-91). */
uint32_t orc_header_size(uint64_t data_size, bool mask);

/* co_ws_frame_deserialize (co_ws_frame.c:121-247) with the max receive
 * payload (co_ws_config.c:29-35) passed explicitly. */
int orc_deserialize(orc_frame_t* frame, const uint8_t* data, size_t data_size,
                    size_t* index, size_t max_payload);
void orc_frame_init(orc_frame_t* frame);   /* co_ws_frame_create values */
void orc_frame_clear(orc_frame_t* frame);  /* frees payload_data */

/* srandom(seed), then 4 x (random() % 256) per masked frame in frame order,
 * exactly the draws sequential co_ws_frame_serialize calls make
 * (co_ws_frame.c:84 -> src/core/co_random.c:32-35). Unmasked frames get 0. */
void orc_keys(uint32_t seed, size_t n, const uint8_t* mask_flags, uint32_t* keys);

/* Batch serialize: frames back to back in desc order. Fills desc[i].wire_off
 * and header_size; returns total wire bytes. */
uint64_t orc_serialize_batch(const uint8_t* payload, orc_desc_t* desc, size_t n,
                             uint8_t* wire);

/* Batch deserialize: frame i parsed as co_ws_frame_deserialize(frame, wire,
 * wire_size, &starts[i]) preceded by the callers' 2-byte precheck
 * (co_ws_client.c:202-206). COMPLETE payloads are unmasked into `payload`
 * at offsets = exclusive scan of round_up(size, align); bytes between a
 * payload's end and the next offset are zero. With
 * ORC_DESERIALIZE_REASSEMBLE, data frames (opcode < 8) are packed with no
 * padding in stream order -- every fragmented message (TEXT/BINARY +
 * CONTINUATION..., co_ws_frame.h:28-30) comes out contiguous -- and control
 * frames (opcode 8-15) are packed after all data bytes. A COMPLETE frame
 * whose payload does not fit payload_capacity gets ORC_ERROR_OUT_OF_MEMORY
 * (the layout is unchanged). Returns min(total, capacity). */
#define ORC_DESERIALIZE_REASSEMBLE 1u
uint64_t orc_deserialize_batch(const uint8_t* wire, uint64_t wire_size,
                               const uint64_t* starts, size_t n,
                               uint64_t max_payload, uint32_t align, uint32_t flags,
                               orc_desc_t* desc, int32_t* status,
                               uint8_t* payload, uint64_t payload_capacity);

/* Split ops (cfws.h "split ops"): headers and payload loops of the codec as
 * separate passes over caller-laid-out frames. Bytes at or past the
 * destination capacity are not written.
 *   orc_encode_headers: co_ws_frame.c:34-91 at wire + desc[i].wire_off; sets
 *     header_size.
 *   orc_parse_headers:  co_ws_frame.c:131-213 (+ the callers' 2-byte
 *     precheck) at starts[i]: desc[i] (payload_off 0), status[i].
 *   orc_mask_batch:     co_ws_frame.c:93-97: wire[wire_off + header size of
 *     (payload_size, mask) + k] = payload[payload_off + k] ^ key[k % 4] (a copy
 *     when mask == 0).
 *   orc_unmask_batch:   co_ws_frame.c:232-242 for every frame whose status is
 *     COMPLETE (status NULL: every frame): payload[payload_off + k] =
 *     wire[wire_off + header_size + k] ^ key[k % 4] (a copy when mask == 0). */
void orc_encode_headers(orc_desc_t* desc, size_t n, uint8_t* wire, uint64_t wire_capacity);
void orc_parse_headers(const uint8_t* wire, uint64_t wire_size, const uint64_t* starts, size_t n,
                       uint64_t max_payload, orc_desc_t* desc, int32_t* status);
void orc_mask_batch(const uint8_t* payload, const orc_desc_t* desc, size_t n, uint8_t* wire,
                    uint64_t wire_capacity);
void orc_unmask_batch(const uint8_t* wire, const orc_desc_t* desc, const int32_t* status, size_t n,
                      uint8_t* payload, uint64_t payload_capacity);

/* WebSocket over HTTP/2 (src/ws_http2): see cfws_oracle.c. */
uint64_t orc_h2_send(const uint8_t* ws, uint64_t len, uint32_t max_frame, uint32_t sid,
                     uint8_t* out);
uint64_t orc_h2_serialize_batch(const uint8_t* payload, orc_desc_t* desc, size_t n,
                                uint32_t sid, uint32_t max_frame, uint8_t* tmp, uint8_t* out);
uint64_t orc_h2_deserialize_batch(const uint8_t* h2, uint64_t size, const uint64_t* index,
                                  size_t n, uint32_t max_frame, int32_t* h2_status,
                                  uint8_t* pool, uint64_t pool_cap, uint64_t max_payload,
                                  uint32_t align, orc_desc_t* msg_desc, int32_t* msg_status,
                                  uint8_t* payload, uint64_t payload_cap, uint64_t* n_msg);

/* Sequential frame-boundary walk of a packed wire stream, as the receive
 * loops do (co_ws_server.c:107-169): writes up to max_frames starts of
 * COMPLETE frames, returns the count; *consumed = bytes of whole frames. */
size_t orc_index_frames(const uint8_t* wire, uint64_t wire_size,
                        uint64_t max_payload, uint64_t* starts,
                        size_t max_frames, uint64_t* consumed);

/* One connection's receive loop over buf[begin, end) (co_ws_server.c:107-169):
 * returns the number of COMPLETE frames (starts beyond max_frames are not
 * written), *consumed = receive index after them, *stop = 0 when every byte
 * was consumed, else the code of the walk's last parse (1 = MORE_DATA, also
 * under 2 bytes left; -7001 / -7005 errors). */
size_t orc_index_stream(const uint8_t* buf, uint64_t begin, uint64_t end, uint64_t max_payload,
                        uint64_t* starts, size_t max_frames, uint64_t* consumed, int32_t* stop);

/* Synthetic payload bytes: byte at global offset o is byte (o % 8) of
 * splitmix64 output number (o / 8) for `seed` (little-endian). */
void orc_fill_splitmix(uint8_t* out, uint64_t n_bytes, uint64_t seed,
                       uint64_t byte_base);

/* CPU baseline: per-frame serialize(mask) + deserialize over n_frames frames
 * of frame_size bytes each, split over `threads` pthreads, repeated `iters`
 * times. Returns seconds for each phase; payload bytes / seconds = rate. */
int orc_cpu_bench(uint64_t n_frames, uint64_t frame_size, int threads,
                  int iters, double* mask_seconds, double* unmask_seconds);

/* Handshake accept key, co_ws_create_base64_accept_key
 * (co_ws_http_extension.c:26-57): out = base64(SHA-1(key || GUID)), 28
 * characters + NUL. */
void orc_sha1(const void* data, uint64_t n, uint8_t out[20]);
uint64_t orc_base64(const uint8_t* src, uint64_t n, char* out);
void orc_ws_accept_key(const char* key, uint64_t key_len, char out[29]);

#ifdef __cplusplus
}
#endif

#endif

