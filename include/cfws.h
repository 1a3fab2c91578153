/*
 * cfws.h -- MI355X batch WebSocket frame codec: C ABI over device arenas.
 *
 * This is the batch entry point that sits beside the drop-in per-frame API
 * (include/cfws_co_ws_frame.h). It covers the hot path of coldforce's
 * src/ws/co_ws_frame.c for many independent frames at once:
 *
 *   cfws_serialize_*   = co_ws_frame_serialize   (co_ws_frame.c:21-119)
 *                        for every frame of a batch: header encode + 4-byte
 *                        key XOR mask, frames packed back to back in a wire
 *                        arena exactly as sequential appends to one
 *                        co_byte_array_t would lay them out.
 *   cfws_deserialize_* = co_ws_frame_deserialize (co_ws_frame.c:121-247)
 *                        at each given frame start of a wire arena (as the
 *                        receive loops call it, co_ws_server.c:107-169):
 *                        header decode, MORE_DATA / INVALID_FRAME /
 *                        DATA_TOO_BIG decisions, copy + XOR unmask of every
 *                        COMPLETE payload into a payload arena.
 *
 * Every pointer argument named d_* is device memory (hipMalloc); `stream` is
 * a hipStream_t (NULL = default stream). Nothing here synchronises: results
 * are valid once the stream has reached the end of the call. All arenas
 * must be 16-byte aligned. The library needs a gfx950 device; with none it
 * returns CFWS_ERROR_NO_DEVICE (there is no CPU fallback).
 */
#ifndef CFWS_H
#define CFWS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Return codes of the batch API. */
#define CFWS_OK                       0
#define CFWS_ERROR_INVALID_ARGUMENT  (-1)
#define CFWS_ERROR_WORKSPACE         (-2)
#define CFWS_ERROR_HIP               (-3)
#define CFWS_ERROR_NO_DEVICE         (-4)

/* Per-frame status codes written by deserialize: the reference's own values
 * (inc/coldforce/ws/co_ws.h:25-39). */
#define CFWS_PARSE_COMPLETE           0
#define CFWS_PARSE_MORE_DATA          1
#define CFWS_ERROR_INVALID_FRAME     (-7001)
#define CFWS_ERROR_DATA_TOO_BIG      (-7005)
#define CFWS_ERROR_OUT_OF_MEMORY     (-7006)

/* Default max receive payload, co_ws_config.h:15. */
#define CFWS_DEFAULT_MAX_RECEIVE_PAYLOAD_SIZE ((uint64_t)32 * 1024 * 1024)

/*
 * One frame of a batch (32 bytes, device resident, array-of-structs).
 *   serialize:   in  payload_off, payload_size, mask_key, fin, opcode, mask
 *                out wire_off, header_size
 *   deserialize: in  wire_off (the frame start, from the caller's index)
 *                out everything else, as far as the header was parsed
 * mask_key holds the 4 key bytes in wire order: byte j = (mask_key >> 8j).
 * opcode is written to the wire verbatim, OR 0x80 when fin (co_ws_frame.c
 * :34-39); deserialize reports opcode = b0 & 0x7f (co_ws_frame.c:136-137).
 */
typedef struct cfws_frame_desc {
    uint64_t payload_off;
    uint64_t wire_off;
    uint64_t payload_size;
    uint32_t mask_key;
    uint8_t  fin;
    uint8_t  opcode;
    uint8_t  mask;
    uint8_t  header_size;
} cfws_frame_desc_t;

/* Library / device check: CFWS_OK when the calling thread's current HIP
 * device is a gfx950. Every visible device is probed once per process
 * (thread-safe); cfws_init_device checks one device by ordinal. */
int cfws_init(void);
int cfws_init_device(int device);
const char* cfws_last_error(void);
const char* cfws_version(void);

/* Bytes of device workspace a plan+execute over n_frames frames producing
 * at most out_capacity output bytes needs. */
size_t cfws_workspace_size(size_t n_frames, uint64_t out_capacity);

/* ---- serialize (client mask / server plain) ------------------------------
 * plan:    header sizes, wire offsets (prefix sum), tile map, and
 *          *d_wire_total = total wire bytes (not clamped to capacity).
 * execute: writes headers + (masked) payloads; bytes past wire_capacity are
 *          not written (check *d_wire_total <= wire_capacity).
 * The workspace carries the plan from plan to execute. */
int cfws_serialize_plan(cfws_frame_desc_t* d_desc, size_t n_frames,
                        uint64_t wire_capacity, uint64_t* d_wire_total,
                        void* d_workspace, size_t workspace_size, void* stream);
int cfws_serialize_execute(const void* d_payload, const cfws_frame_desc_t* d_desc,
                           size_t n_frames, void* d_wire, uint64_t wire_capacity,
                           const void* d_workspace, void* stream);
int cfws_serialize_batch(const void* d_payload, cfws_frame_desc_t* d_desc,
                         size_t n_frames, void* d_wire, uint64_t wire_capacity,
                         uint64_t* d_wire_total, void* d_workspace,
                         size_t workspace_size, void* stream);

/* ---- serialize a uniform batch (compact input) ----------------------------
 * Every frame has the same payload_size, fin, opcode and mask: n sequential
 * co_ws_frame_serialize calls (co_ws_frame.c:21-119) appending fixed-size
 * messages to one co_byte_array, with no descriptor table and no plan.
 * Frame i's payload is d_payload[i * payload_size, (i + 1) * payload_size)
 * and its key d_keys[i] (wire order, as cfws_frame_desc_t.mask_key; NULL
 * allowed when mask == 0); its frame is d_wire[i * W, (i + 1) * W), W =
 * header size (2..14, co_ws_frame.c:34-91) + payload_size. One launch, no
 * workspace; the bytes are those cfws_serialize_batch writes for the same
 * frames. Wire bytes at or past wire_capacity are not written;
 * *d_wire_total (may be NULL) = n * W. payload_size <= 2^31, n * W < 2^40. */
int cfws_serialize_uniform(const void* d_payload, const uint32_t* d_keys, size_t n_frames,
                           uint64_t payload_size, uint8_t fin, uint8_t opcode, uint8_t mask,
                           void* d_wire, uint64_t wire_capacity, uint64_t* d_wire_total,
                           void* stream);

/* ---- deserialize (server unmask / client plain) --------------------------
 * plan:    parses the header at each d_frame_index[i] against wire_size,
 *          writes d_desc[i] and d_status[i] (reference codes) and lays the
 *          COMPLETE payloads out:
 *            flags = 0: payload_off = exclusive prefix sum of
 *              round_up(payload_size, align) (align a power of two, 1..4096);
 *            flags = CFWS_DESERIALIZE_REASSEMBLE: data frames (opcode < 8)
 *              packed back to back in stream order, so the fragments of every
 *              message (TEXT/BINARY then CONTINUATION..., co_ws_frame.h:28-30)
 *              are contiguous; control frames (opcode 8-15) packed after all
 *              data bytes; align is ignored.
 *          A COMPLETE frame with a non-empty payload that does not fit
 *          payload_capacity gets CFWS_ERROR_OUT_OF_MEMORY (layout unchanged).
 *          *d_payload_total = min(sum, capacity).
 * execute: copies + unmasks every COMPLETE payload; bytes of the layout not
 *          covered by a payload (alignment padding, OOM frames) are zero.
 *          `flags` must be the plan's. */
#define CFWS_DESERIALIZE_REASSEMBLE 1u

int cfws_deserialize_plan(const void* d_wire, uint64_t wire_size,
                          const uint64_t* d_frame_index, size_t n_frames,
                          uint64_t max_payload, uint32_t align, uint32_t flags,
                          cfws_frame_desc_t* d_desc, int32_t* d_status,
                          uint64_t payload_capacity, uint64_t* d_payload_total,
                          void* d_workspace, size_t workspace_size, void* stream);
int cfws_deserialize_execute(const void* d_wire, const cfws_frame_desc_t* d_desc,
                             const int32_t* d_status, size_t n_frames, uint32_t flags,
                             void* d_payload, uint64_t payload_capacity,
                             const void* d_workspace, void* stream);
int cfws_deserialize_batch(const void* d_wire, uint64_t wire_size,
                           const uint64_t* d_frame_index, size_t n_frames,
                           uint64_t max_payload, uint32_t align, uint32_t flags,
                           cfws_frame_desc_t* d_desc, int32_t* d_status,
                           void* d_payload, uint64_t payload_capacity,
                           uint64_t* d_payload_total, void* d_workspace,
                           size_t workspace_size, void* stream);

/* ---- deserialize into fixed payload slots --------------------------------
 * The batch receive with frame i's payload at payload_off = i * slot_bytes
 * (slot_bytes a multiple of 16 in [16, 2^31]): the slab form of the
 * reference's one allocation per frame (co_ws_frame_deserialize,
 * src/ws/co_ws_frame.c:216-223). One launch, no workspace: no payload offset
 * depends on another frame, so each wire line is read once.
 *   d_desc[i], d_status[i]: as cfws_deserialize_plan (flags = 0), with the
 *     slot rule in place of the packing: a COMPLETE frame whose non-empty
 *     payload is longer than slot_bytes, or ends past payload_capacity, gets
 *     CFWS_ERROR_OUT_OF_MEMORY.
 *   slot i of a COMPLETE frame: the unmasked payload, then zeros up to the
 *     next 16-byte boundary (cut at the capacity); the rest of every slot,
 *     and the slots of all other frames, are not written.
 *   *d_payload_total (may be NULL) = min(n_frames * slot_bytes, capacity).
 * Frames of the same wire may be indexed in any order, overlapping or not. */
int cfws_deserialize_slots(const void* d_wire, uint64_t wire_size,
                           const uint64_t* d_frame_index, size_t n_frames,
                           uint64_t max_payload, uint64_t slot_bytes,
                           cfws_frame_desc_t* d_desc, int32_t* d_status,
                           void* d_payload, uint64_t payload_capacity,
                           uint64_t* d_payload_total, void* stream);

/* ---- compact per-frame output of the slot / scatter receives --------------
 * What the reference's frame object carries (co_ws_frame_header_t:
 * fin, opcode, payload_size, co_ws_frame.h:36-49) plus the status, in 8
 * bytes instead of the 36 of a descriptor + status (the payload offset is
 * the slot, or the caller's, and the key and header size are consumed by
 * the unmask). payload_size is the parsed length, UINT32_MAX when it does
 * not fit 32 bits (never for a COMPLETE frame: its payload fits its slot,
 * <= 2^31); status is the int32 code cast to 16 bits (every code fits). */
typedef struct cfws_frame_info {
    uint32_t payload_size;
    uint8_t  fin;
    uint8_t  opcode;
    int16_t  status;
} cfws_frame_info_t;

/* cfws_deserialize_slots / cfws_deserialize_scatter with d_info[i] (8-byte
 * aligned) in place of d_desc[i] and d_status[i]: the same decisions, the
 * same payload bytes; the fields equal the descriptor form's. */
int cfws_deserialize_slots_info(const void* d_wire, uint64_t wire_size,
                                const uint64_t* d_frame_index, size_t n_frames,
                                uint64_t max_payload, uint64_t slot_bytes,
                                cfws_frame_info_t* d_info, void* d_payload,
                                uint64_t payload_capacity, uint64_t* d_payload_total,
                                void* stream);
int cfws_deserialize_scatter_info(const void* d_wire, uint64_t wire_size,
                                  const uint64_t* d_frame_index, const uint64_t* d_payload_off,
                                  size_t n_frames, uint64_t max_payload, uint64_t max_slot,
                                  cfws_frame_info_t* d_info, void* d_payload,
                                  uint64_t payload_capacity, void* stream);

/* ---- slot receive of a uniform stream ------------------------------------
 * cfws_deserialize_slots_info with the index implicit: frame i is parsed at
 * i * frame_stride, as if d_frame_index[i] = i * frame_stride (the wire
 * cfws_serialize_uniform writes, frame_stride its header + payload bytes).
 * Same decisions, same d_info, payload and total as that indexed call; no
 * index is read. *d_mismatch (may be NULL; the call zeroes it first) = the
 * frames that are not COMPLETE frames of exactly frame_stride wire bytes.
 * Zero means each frame i parsed COMPLETE and ends where frame i + 1 starts:
 * the reference's receive loop (src/ws/co_ws_server.c:107-169 calling
 * co_ws_frame_deserialize, src/ws/co_ws_frame.c:129-247) would have taken
 * the same n frames from the start of the wire. Non-zero: the stream is not
 * uniform there; index it (cfws_index_frames_batch) and use the indexed
 * receive. frame_stride >= 2, n_frames * frame_stride < 2^63. */
int cfws_deserialize_slots_uniform(const void* d_wire, uint64_t wire_size, size_t n_frames,
                                   uint64_t frame_stride, uint64_t max_payload, uint64_t slot_bytes,
                                   cfws_frame_info_t* d_info, void* d_payload,
                                   uint64_t payload_capacity, uint64_t* d_payload_total,
                                   uint32_t* d_mismatch, void* stream);

/* ---- deserialize, each payload to the caller's offset ---------------------
 * cfws_deserialize_slots with payload_off = d_payload_off[i] (the caller's
 * own buffer for each frame, as the reference allocates one per frame,
 * co_ws_frame.c:216-223): one launch, each wire line read once. Every
 * offset must be a multiple of 16; max_slot (a multiple of 16 in [16, 2^31])
 * bounds the payloads. A COMPLETE frame with a non-empty payload gets
 * CFWS_ERROR_OUT_OF_MEMORY when that payload is longer than max_slot, ends
 * past payload_capacity, or has an offset that is not a multiple of 16; its
 * destination is not written. Otherwise as cfws_deserialize_slots: the
 * unmasked payload, then zeros to the next 16-byte boundary (cut at the
 * capacity); nothing else is written. Destinations that overlap are the
 * caller's to avoid. */
int cfws_deserialize_scatter(const void* d_wire, uint64_t wire_size,
                             const uint64_t* d_frame_index, const uint64_t* d_payload_off,
                             size_t n_frames, uint64_t max_payload, uint64_t max_slot,
                             cfws_frame_desc_t* d_desc, int32_t* d_status,
                             void* d_payload, uint64_t payload_capacity, void* stream);

/* ---- split ops: headers and payload XOR as separate passes ---------------
 * The two halves of the codec over frames the caller lays out itself (a send
 * path that gathers headers and payloads into iovecs, a receive path that
 * places payloads in its own buffers): every descriptor names its own source
 * and destination, nothing is packed and no workspace is needed.
 *   cfws_encode_headers: frame i's header (co_ws_frame.c:34-91: b0 = opcode
 *     | fin << 7, minimal 7/16/64-bit length, the 4 key bytes when mask) at
 *     d_wire + wire_off; sets header_size (2..14).
 *   cfws_parse_headers: co_ws_frame_deserialize's header decisions
 *     (co_ws_frame.c:131-213, with the callers' 2-byte precheck,
 *     co_ws_client.c:202-206) at d_frame_index[i] against wire_size: d_desc[i]
 *     (wire_off = the start, payload_off = 0) and d_status[i] -- the decode of
 *     cfws_deserialize_plan without its payload layout.
 *   cfws_mask_batch: the serialize payload loop (co_ws_frame.c:93-97):
 *     d_wire[wire_off + h + k] = d_payload[payload_off + k] ^ key[k % 4],
 *     k < payload_size, h = the header size of (payload_size, mask); a copy
 *     when mask == 0. Header bytes are not touched.
 *   cfws_unmask_batch: the deserialize payload loop (co_ws_frame.c:232-242):
 *     d_payload[payload_off + k] = d_wire[wire_off + header_size + k] ^
 *     key[k % 4] for every frame whose d_status is CFWS_PARSE_COMPLETE
 *     (d_status NULL: every frame); a copy when mask == 0.
 * Destination bytes at or past the capacity are not written. Destination
 * ranges of different frames must not overlap; sources may. max_payload_size
 * is an upper bound of payload_size over the batch: it sizes the grid (a
 * larger frame is still processed, by fewer workgroups). Arenas 16-byte
 * aligned. */
int cfws_encode_headers(cfws_frame_desc_t* d_desc, size_t n_frames, void* d_wire,
                        uint64_t wire_capacity, void* stream);
int cfws_parse_headers(const void* d_wire, uint64_t wire_size, const uint64_t* d_frame_index,
                       size_t n_frames, uint64_t max_payload, cfws_frame_desc_t* d_desc,
                       int32_t* d_status, void* stream);
int cfws_mask_batch(const void* d_payload, const cfws_frame_desc_t* d_desc, size_t n_frames,
                    uint64_t max_payload_size, void* d_wire, uint64_t wire_capacity,
                    void* stream);
/* cfws_mask_batch for frames the caller packed back to back (frame i's
 * header starts where frame i - 1's payload ends, as one co_byte_array of
 * sequential co_ws_frame_serialize calls lays them out) whose headers are
 * the bytes cfws_encode_headers writes. Same result bytes; the 16-byte
 * chunks a frame shares with its neighbour's payload and its own header are
 * then written whole, header bytes included (rewritten with the values
 * cfws_encode_headers wrote), instead of byte by byte after the stream
 * (DESIGN.md §3.8). Each adjacency is checked on the device: a boundary that
 * is not packed, or whose payloads are shorter than 16 bytes, is written as
 * by cfws_mask_batch. */
int cfws_mask_batch_packed(const void* d_payload, const cfws_frame_desc_t* d_desc, size_t n_frames,
                           uint64_t max_payload_size, void* d_wire, uint64_t wire_capacity,
                           void* stream);
int cfws_unmask_batch(const void* d_wire, const cfws_frame_desc_t* d_desc, const int32_t* d_status,
                      size_t n_frames, uint64_t max_payload_size, void* d_payload,
                      uint64_t payload_capacity, void* stream);

/* ---- receive-buffer frame indexing --------
 * The frame walk of the receive loops co_ws_server_on_tcp_receive_ready
 * (co_ws_server.c:107-169) / co_ws_client_on_tcp_receive_ready
 * (co_ws_client.c:200-270) over one connection's received bytes
 * buf[begin, end): from the receive index `begin`, while bytes remain, stop
 * when fewer than 2 are left or a frame does not parse COMPLETE against
 * data_size = end (co_ws_frame_deserialize's decisions, co_ws_frame.c
 * :131-213, with max_payload as co_ws_config_get_max_receive_payload_size).
 * Per connection it reports the starts of the COMPLETE frames, the receive
 * index after them (*consumed, where the reference leaves
 * receive_data.index) and why the walk stopped (*stop):
 *   CFWS_PARSE_COMPLETE      every byte consumed (the loop clears the buffer)
 *   CFWS_PARSE_MORE_DATA     under 2 bytes left, or a frame incomplete: wait
 *   CFWS_ERROR_INVALID_FRAME the frame at *consumed is not WS (HTTP fallback
 *                            / close 1002, co_ws_client.c:62-71)
 *   CFWS_ERROR_DATA_TOO_BIG  the frame at *consumed exceeds max_payload
 *                            (close 1009)
 *   CFWS_INDEX_FULL          host form only: `starts` is full and another
 *                            COMPLETE frame follows; resume at *consumed.
 * The starts feed cfws_deserialize_* (every frame they name is COMPLETE).
 *
 * Host form: one connection, on the calling thread (receive buffers in host
 * memory). Returns the number of starts written. */
#define CFWS_INDEX_FULL 2
size_t cfws_index_frames(const void* h_buf, uint64_t begin, uint64_t end, uint64_t max_payload,
                         uint64_t* starts, size_t max_starts, uint64_t* consumed, int32_t* stop);

/* Device form: n_conns connections of one device arena at once, connection
 * c = d_buf[d_begin[c], d_end[c]). d_first[c] = index of c's first start in
 * d_starts (exclusive prefix sum of the per-connection counts), *d_total =
 * all starts (unclamped); starts at positions >= starts_capacity are not
 * written. d_consumed / d_stop per connection as above. The workspace
 * (cfws_index_workspace_size) holds 64 starts per connection between the
 * walk and the scan that places them: 520 bytes per connection. */
size_t cfws_index_workspace_size(size_t n_conns);
int cfws_index_frames_batch(const void* d_buf, const uint64_t* d_begin, const uint64_t* d_end,
                            size_t n_conns, uint64_t max_payload, uint64_t* d_starts,
                            uint64_t starts_capacity, uint64_t* d_first, uint64_t* d_consumed,
                            int32_t* d_stop, uint64_t* d_total, void* d_workspace,
                            size_t workspace_size, void* stream);

/* ---- handshake accept keys ----------------
 * Sec-WebSocket-Accept for n connections at once, as
 * co_ws_create_base64_accept_key computes it for one
 * (co_ws_http_extension.c:26-57; used by the server's upgrade response :342
 * and the client's check :245): base64(SHA-1(key || "258EAFA5-E914-47DA-
 * 95CA-C5AB0DC85B11")) with '=' padding. Key c is the bytes
 * d_keys[d_key_off[c], d_key_off[c + 1]) (n + 1 offsets, any length); its
 * 28-character accept value + NUL goes to d_accept + CFWS_WS_ACCEPT_SLOT * c
 * (the slot's last 3 bytes are written as zeros when d_accept is 16-byte
 * aligned, and left alone otherwise). Offsets must not decrease: a key with
 * d_key_off[c + 1] < d_key_off[c] gets an all-zero slot (an empty string). */
#define CFWS_WS_ACCEPT_SLOT 32
int cfws_ws_accept_keys_batch(const void* d_keys, const uint64_t* d_key_off, size_t n,
                              char* d_accept, void* stream);

/* ---- WebSocket over HTTP/2 (src/ws_http2) ---------------------------------
 * Send: every WS frame of the batch is serialized (cfws_serialize_batch, into
 * d_wire) and carried in HTTP/2 DATA frames of at most max_frame_size payload
 * bytes (0 = the default 16384, co_http2.h:55), END_STREAM on the last DATA
 * frame of each WS frame -- co_http2_stream_send_ws_frame
 * (co_ws_http2_extension.c:166-199) -> co_http2_stream_send_data
 * (co_http2_stream.c:933-1013), DATA layout co_http2_frame.c:33-72 (9-byte
 * header: 24-bit BE length, type 0, flags, 31-bit BE stream id). The flow
 * control window is assumed to admit every frame. *d_h2_total is unclamped.
 * Receive: the DATA frames starting at d_h2_index[i] (one stream, in order)
 * are parsed (co_http2_frame.c:211-300; status per DATA frame below), their
 * payloads pooled into d_pool until END_STREAM (co_http2_stream.c:550-608),
 * and every pooled message goes through co_ws_frame_deserialize against its
 * own size (co_ws_http2_extension.c:134-164): d_msg_desc / d_msg_status get
 * one entry per message (room for n_h2 entries; entries n_messages..n_h2-1
 * are empty: status CFWS_PARSE_MORE_DATA, no payload, no header, payload_off
 * unspecified), payloads land in d_payload as cfws_deserialize_batch lays
 * them out (flags = 0). *n_messages is final on return: the host waits on an
 * event after the device plan, through 64 bytes of mapped pinned memory and
 * an event made once per device of `stream` (where the kernels run; not
 * necessarily the current device). A calling thread borrows them for its
 * lifetime and hands them back at exit, so threads that come and go reuse
 * them. The payload pass may still be running on the stream, as with the
 * other batch calls. When every DATA payload fits pool_capacity the pool is
 * virtual: WS headers are gathered and payload slices copied + unmasked
 * straight out of the DATA frames in one pass, and d_pool is not written;
 * otherwise the pool is materialised first (the capacity rule needs it) and
 * the one-pass form, already queued, stores nothing. */
#define CFWS_H2_DEFAULT_MAX_FRAME_SIZE 16384u
#define CFWS_H2_PARSE_COMPLETE    0     /* co_http.h:40-42 */
#define CFWS_H2_PARSE_MORE_DATA   1
#define CFWS_H2_PARSE_ERROR      (-1)
#define CFWS_H2_NOT_DATA          3     /* a complete non-DATA frame: no bytes */

size_t cfws_h2_serialize_workspace_size(size_t n_frames, uint64_t wire_capacity,
                                        uint64_t h2_capacity, uint32_t max_frame_size);
int cfws_h2_serialize_batch(const void* d_payload, cfws_frame_desc_t* d_desc, size_t n_frames,
                            uint32_t stream_id, uint32_t max_frame_size, void* d_wire,
                            uint64_t wire_capacity, void* d_h2, uint64_t h2_capacity,
                            uint64_t* d_h2_total, void* d_workspace, size_t workspace_size,
                            void* stream);
size_t cfws_h2_deserialize_workspace_size(size_t n_h2_frames, uint64_t pool_capacity,
                                          uint64_t payload_capacity);
int cfws_h2_deserialize_batch(const void* d_h2, uint64_t h2_size, const uint64_t* d_h2_index,
                              size_t n_h2_frames, uint32_t max_frame_size, int32_t* d_h2_status,
                              void* d_pool, uint64_t pool_capacity, uint64_t max_payload,
                              uint32_t align, cfws_frame_desc_t* d_msg_desc,
                              int32_t* d_msg_status, void* d_payload, uint64_t payload_capacity,
                              uint64_t* d_payload_total, size_t* n_messages,
                              void* d_workspace, size_t workspace_size, void* stream);

/* ---- host-memory pipeline ------------------------------------------------
 * The same codec over HOST buffers (socket send/receive side): the batch is
 * cut into chunks of frames; `depth` slots (1..4), each with a stream and
 * device staging of chunk_bytes per direction, overlap H2D, the device plan +
 * kernels and D2H of consecutive chunks. Host buffers should be pinned.
 * Synchronous: results are in host memory on return.
 * max_frames bounds the frames per chunk (descriptor staging). */
typedef struct cfws_pipeline cfws_pipeline_t;
int cfws_pipeline_create(uint64_t chunk_bytes, size_t max_frames, int depth,
                         cfws_pipeline_t** out);
void cfws_pipeline_destroy(cfws_pipeline_t* pipeline);
/* cfws_serialize_batch over host arenas; h_desc gets wire_off/header_size. */
int cfws_pipeline_serialize(cfws_pipeline_t* pipeline, const void* h_payload,
                            cfws_frame_desc_t* h_desc, size_t n_frames, void* h_wire,
                            uint64_t wire_capacity, uint64_t* wire_total);
/* cfws_deserialize_batch over host buffers, flags = 0 (the reassembly layout
 * needs the whole batch). Precondition: h_frame_index increasing, every
 * frame ending at or before the next start (what a receive loop's index
 * satisfies). */
int cfws_pipeline_deserialize(cfws_pipeline_t* pipeline, const void* h_wire,
                              uint64_t wire_size, const uint64_t* h_frame_index,
                              size_t n_frames, uint64_t max_payload, uint32_t align,
                              uint32_t flags, cfws_frame_desc_t* h_desc, int32_t* h_status,
                              void* h_payload, uint64_t payload_capacity,
                              uint64_t* payload_total);
/* The receive loop over one host buffer h_wire[begin, end): cfws_index_frames
 * (on the calling thread) then cfws_pipeline_deserialize of the COMPLETE
 * frames it found. *n_frames: in, the capacity of h_desc / h_status; out,
 * the frames deserialized. *consumed / *stop as cfws_index_frames reports
 * them (CFWS_INDEX_FULL: more frames follow; call again from *consumed). */
int cfws_pipeline_receive(cfws_pipeline_t* pipeline, const void* h_wire, uint64_t begin,
                          uint64_t end, uint64_t max_payload, uint32_t align,
                          cfws_frame_desc_t* h_desc, int32_t* h_status, size_t* n_frames,
                          uint64_t* consumed, int32_t* stop, void* h_payload,
                          uint64_t payload_capacity, uint64_t* payload_total);

/* WebSocket over HTTP/2 through host memory: cfws_h2_serialize_batch /
 * cfws_h2_deserialize_batch per chunk, with the copies overlapped as above.
 * Send: h_desc gets header_size / wire_off; *h2_total = DATA-stream bytes
 * (unclamped). Receive: h_h2_status[i] per DATA frame, one message entry per
 * pooled message (room for n entries), *n_messages, payloads laid out as the
 * batch call lays them out; chunks end where no message is open, so a
 * message larger than the chunk is an error. The index precondition of
 * cfws_pipeline_deserialize holds for DATA frames too. */
int cfws_pipeline_h2_serialize(cfws_pipeline_t* pipeline, const void* h_payload,
                               cfws_frame_desc_t* h_desc, size_t n, uint32_t stream_id,
                               uint32_t max_frame_size, void* h_h2, uint64_t h2_capacity,
                               uint64_t* h2_total);
int cfws_pipeline_h2_deserialize(cfws_pipeline_t* pipeline, const void* h_h2, uint64_t h2_size,
                                 const uint64_t* h_index, size_t n, uint32_t max_frame_size,
                                 uint64_t max_payload, uint32_t align, int32_t* h_h2_status,
                                 cfws_frame_desc_t* h_msg_desc, int32_t* h_msg_status,
                                 size_t* n_messages, void* h_payload, uint64_t payload_capacity,
                                 uint64_t* payload_total);

/* How the pipeline's D2H leg moves bytes into a MAPPED host output arena
 * (hipHostMalloc(..., hipHostMallocMapped)); unmapped arenas always take
 * SDMA. AUTO (the default): a kernel storing into the arena for serialize,
 * an SDMA copy for deserialize -- each direction's faster choice beside the
 * in-order H2D copies. DMA: SDMA both ways; KERNEL:
 * the kernel both ways. The environment variable CFWS_PIPELINE_D2H = auto |
 * dma | kernel sets the default of new pipelines. */
#define CFWS_PIPELINE_D2H_AUTO   0
#define CFWS_PIPELINE_D2H_DMA    1
#define CFWS_PIPELINE_D2H_KERNEL 2
int cfws_pipeline_set_d2h(cfws_pipeline_t* pipeline, int mode);

/* D2H by a kernel: copies d_src[0, n) to h_dst, a host buffer allocated (or
 * registered) MAPPED (hipHostMalloc(..., hipHostMallocMapped)), by 16-byte
 * stores over PCIe: the pipeline's D2H leg in CFWS_PIPELINE_D2H_KERNEL mode
 * (and serialize's in AUTO). CFWS_ERROR_INVALID_ARGUMENT when h_dst is
 * not mapped memory. cfws_mapped_device_pointer: h_ptr's device address when
 * it is mapped HIP host memory, else NULL. */
int cfws_copy_to_host(const void* d_src, void* h_dst, uint64_t n, void* stream);
void* cfws_mapped_device_pointer(const void* h_ptr);

/* ---- HIP graphs of a batch (cfws_graph.cpp) ------------------------------
 * A batch shape replayed over the same arenas: cfws_serialize_batch /
 * cfws_deserialize_batch with these exact arguments, captured once into a
 * hipGraph and launched with one call on any stream. Pointers, frame count
 * and capacities are fixed at capture; descriptor contents and payload /
 * wire bytes may change between launches (the plans run on the device at
 * every launch). For small batches, where launch latency rather than HBM
 * bounds a call. cfws_h2_deserialize_batch
 * synchronises and cannot be captured. */
typedef struct cfws_graph cfws_graph_t;
int cfws_graph_serialize(const void* d_payload, cfws_frame_desc_t* d_desc, size_t n, void* d_wire,
                         uint64_t wire_capacity, uint64_t* d_wire_total, void* d_workspace,
                         size_t workspace_size, cfws_graph_t** graph);
int cfws_graph_deserialize(const void* d_wire, uint64_t wire_size, const uint64_t* d_index, size_t n,
                           uint64_t max_payload, uint32_t align, uint32_t flags,
                           cfws_frame_desc_t* d_desc, int32_t* d_status, void* d_payload,
                           uint64_t payload_capacity, uint64_t* d_payload_total, void* d_workspace,
                           size_t workspace_size, cfws_graph_t** graph);
int cfws_graph_launch(cfws_graph_t* graph, void* stream);
void cfws_graph_destroy(cfws_graph_t* graph);

/* ---- single-buffer XOR (used by the per-frame drop-in path) --------------
 * d_dst[i] = d_src[i] ^ key byte (i + key_phase) % 4, i < n. */
int cfws_xor_mask(const void* d_src, void* d_dst, uint64_t n, uint32_t mask_key,
                  uint32_t key_phase, void* stream);

/* Mask keys for a batch, drawn exactly as sequential co_ws_frame_serialize
 * calls would draw them: 4 x (random() % 256) per frame whose mask flag is
 * set, in frame order, from the process's current random() state
 * (co_ws_frame.c:84 -> src/core/co_random.c:32-35). mask_flags == NULL
 * means every frame is masked; unmasked frames get key 0. Host memory. */
void cfws_draw_mask_keys(size_t n_frames, const uint8_t* mask_flags, uint32_t* keys);
/* The keys the same calls draw right after srandom(seed), taken from a
 * private copy of that generator (glibc random_r): other threads' rand() /
 * random() calls cannot interleave with the draws, and the process's
 * random() state is not touched. CFWS_OK, or CFWS_ERROR_INVALID_ARGUMENT. */
int cfws_draw_mask_keys_seeded(uint32_t seed, size_t n_frames, const uint8_t* mask_flags,
                               uint32_t* keys);

/* Frees the calling thread's drop-in staging buffers and stream
 * (cfws_frame.cpp) now; optional: a thread that exits without calling it
 * hands them back for reuse by later threads. */
void cfws_release_thread_resources(void);

/* Device policy of the drop-in co_ws_frame_* calls (cfws_frame.cpp). By
 * default (device -1) a thread's masked frames run on its current HIP device,
 * read on every frame. cfws_bind_thread_device(d) pins the calling thread to
 * device d whatever its current device is, so a server with one co_thread
 * per GPU (the reference hands accepted sockets to other threads,
 * co_net_worker.c:240) can spread its connections over the GPUs. A thread
 * whose device changes hands its stream and staging buffers back to a
 * per-device pool and borrows the new device's. CFWS_OK, or
 * CFWS_ERROR_INVALID_ARGUMENT / CFWS_ERROR_NO_DEVICE (d not a gfx950).
 * cfws_thread_device returns the device the next frame would use (-1 on
 * error). */
int cfws_bind_thread_device(int device);
int cfws_thread_device(void);

/* Size policy of the drop-in co_ws_frame_* calls (cfws_frame.cpp). A masked
 * payload of fewer than `bytes` bytes is XORed on the calling thread by the
 * library's own vector loop; payloads of `bytes` or more go to the device
 * (the frame service up to 32 KiB, a launch per frame above). Measured per
 * frame on the MI355X box, the calling thread is faster
 * at every size from 125 B to 4 MiB and spends less CPU time: a per-frame
 * device call copies the payload into and out of pinned staging on the
 * calling thread and waits on PCIe, and its wait spins (or, blocked on an
 * event, cost as much thread CPU time). So the default keeps every frame on
 * the calling thread and the device is opt-in: CFWS_DROPIN_GPU_MIN_DEFAULT
 * is SIZE_MAX; the CFWS_DROPIN_GPU_MIN environment variable (read at load)
 * or this call sets another threshold, 0 sends every masked frame to the
 * device. A frame below the threshold makes no HIP call and needs no
 * device; a frame at or above it fails without a gfx950 agent.
 * Process-wide. The batch ABI above has no host path at any size. */
#define CFWS_DROPIN_GPU_MIN_DEFAULT ((size_t)-1)
void cfws_set_dropin_gpu_min(size_t bytes);
size_t cfws_dropin_gpu_min(void);

/* ---- streaming device copy ------------------------------------------------
 * d_dst[i] = d_src[i], i < n: a bare HBM stream (the bench's copy ceiling,
 * the read + write shape of the codec without its frames). Pointers and n
 * multiples of 16. */
int cfws_device_copy(const void* d_src, void* d_dst, uint64_t n, void* stream);

/* ---- profiling ------------------------------------------------------------
 * `start` / `stop` (hipEvent_t) for the CALLING THREAD's next batch call
 * (any function above that takes a stream). That call takes the pair on
 * entry -- from then on no pair is pending -- and records `start` on its
 * stream right before its timed pass and `stop` right after it:
 *   cfws_serialize_batch / _execute, cfws_deserialize_batch / _execute:
 *     the streaming pass (xform_kernel with its edge workgroups; both
 *     passes of a reassembling execute are one timed span); for batches of
 *     small frames the one kernel the call launches instead (the small-batch
 *     kernel, or the fused plan + copy kernel of cfws_deserialize_batch);
 *   cfws_deserialize_slots / _scatter: their one kernel;
 *   cfws_h2_serialize_batch: its DATA-frame pass; cfws_h2_deserialize_batch:
 *     its fused payload pass, or, when the pooled bytes exceed pool_capacity
 *     (that pass then stores nothing), the pool + plan + payload passes of
 *     the general form that does the work.
 * Any other call, an error return, an empty batch, a graph capture / launch
 * or a pipeline call records nothing and drops the pair. NULL, NULL clears
 * a pending pair. Lets a caller time the one kernel of a multi-kernel call
 * that moves the bytes (bench.py's roofline figures). */
int cfws_time_next_pass(void* start, void* stop);

/* The kernel cfws_deserialize_batch's timed pass is for a call with these
 * sizes (its pointers valid): "deserialize_small_kernel" (one launch for a
 * small batch), "deserialize_plan_single_kernel<true>" (the fused plan +
 * copy of batches of small frames) or "xform_kernel<1>" (the execute after
 * the plan). The same rule the call applies, so a profile can name what it
 * timed. A static string. */
const char* cfws_deserialize_pass_kernel(size_t n_frames, uint64_t wire_size, uint32_t align,
                                         uint32_t flags, uint64_t payload_capacity);

/* The kernel the slot / scatter receives (cfws_deserialize_slots*,
 * cfws_deserialize_scatter*) launch for n_frames frames in wire_size bytes
 * and slots (max_slot) of slot_bytes: "deserialize_slots_piece_kernel" (one
 * wave per 2 KiB piece of a frame's slot: slots over 8,160 bytes whose frames
 * average over 1,040 bytes, and from 2 KiB slots that are multiples of 128
 * filling at least 85 % of their pieces, with frames averaging 85 % of the
 * slot), "deserialize_slots_kernel" (short frames in large slots: frames
 * averaging up to 1,040 bytes in slots over 8,160 bytes; frames of up to 1 KiB
 * filling under half their slot, or under 80 % of a slot of 1 KiB or more)
 * or "deserialize_slots_window_kernel" (the rest). The calls' own rule. A
 * static string. */
const char* cfws_deserialize_slots_pass_kernel(size_t n_frames, uint64_t wire_size, uint64_t slot_bytes);

/* The kernel cfws_serialize_uniform launches for frames of payload_size
 * bytes (masked or not): "serialize_uniform_small_kernel" (payloads of
 * 32-65,535 bytes, multiples of 16), "serialize_uniform_kernel" (other
 * frames of at least 32 wire bytes) or "serialize_uniform_bytes_kernel".
 * The call's own rule. A static string. */
const char* cfws_serialize_uniform_pass_kernel(uint64_t payload_size, uint8_t mask);

/* ---- synthetic input (bench / tests) -------------------------------------
 * d_dst[i] = byte ((byte_base + i) % 8) of splitmix64 output number
 * (byte_base + i) / 8 for `seed`; byte_base must be a multiple of 8. */
int cfws_fill_splitmix(void* d_dst, uint64_t n_bytes, uint64_t seed,
                       uint64_t byte_base, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* CFWS_H */
