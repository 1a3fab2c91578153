/*
 * cfws_co_ws_frame.h -- drop-in replacement ABI for coldforce's frame codec.
 *
 * libcfws.so exports these symbols with the exact prototypes and struct
 * layouts of the reference, so src/ws/co_ws_client.c, co_ws_server.c and
 * src/ws_http2/co_ws_http2_extension.c link against it unchanged (see
 * INTEGRATION.md). Each declaration cites the reference interface it
 * replaces. The payload XOR (mask on send, unmask on receive) runs on the
 * MI355X; header encode/decode and the byte-array bookkeeping stay on the
 * calling thread, as in the reference.
 *
 * Code built against coldforce's own headers does not include this file:
 * the guards below let it coexist with inc/coldforce/ws/co_ws_frame.h.
 */
#ifndef CFWS_CO_WS_FRAME_H
#define CFWS_CO_WS_FRAME_H

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#ifndef CO_ARRAY_H_INCLUDED
/* inc/coldforce/core/co_array.h:16-23 (co_byte_array_t = co_array_t,
 * inc/coldforce/core/co_byte_array.h:16). Serialize appends to it with the
 * reference growth rule (src/core/co_array.c:83-112). */
typedef struct {
    size_t capacity;
    size_t count;
    size_t element_size;
    uint8_t* buffer;
} co_array_t;
#endif
#ifndef CO_BYTE_ARRAY_H_INCLUDED
typedef co_array_t co_byte_array_t;
#endif

#ifndef CO_WS_FRAME_H_INCLUDED
/* inc/coldforce/ws/co_ws_frame.h:14-34 */
#define CO_WS_FRAME_HEADER_MIN_SIZE    2
#define CO_WS_FRAME_HEADER_MAX_SIZE    16
#define CO_WS_FRAME_MASK_SIZE          4
#define CO_WS_OPCODE_CONTINUATION   0x00
#define CO_WS_OPCODE_TEXT           0x01
#define CO_WS_OPCODE_BINARY         0x02
#define CO_WS_OPCODE_CLOSE          0x08
#define CO_WS_OPCODE_PING           0x09
#define CO_WS_OPCODE_PONG           0x0a

/* inc/coldforce/ws/co_ws_frame.h:36-49 -- callers read these fields
 * directly (co_ws_client.c:221-224, co_ws_http2_extension.c:157-160). */
typedef struct {
    bool fin;
    uint8_t opcode;
    uint64_t payload_size;
} co_ws_frame_header_t;

typedef struct {
    co_ws_frame_header_t header;
    uint8_t* payload_data;
} co_ws_frame_t;
#endif

#ifndef CO_WS_H_INCLUDED
/* inc/coldforce/ws/co_ws.h:25-39 */
#define CO_WS_ERROR_INVALID_FRAME   -7001
#define CO_WS_ERROR_DATA_TOO_BIG    -7005
#define CO_WS_ERROR_OUT_OF_MEMORY   -7006
#define CO_WS_PARSE_COMPLETE        0
#define CO_WS_PARSE_MORE_DATA       1
#endif

/* co_ws_frame.h:55-63 / co_ws_frame.c:21-119. Appends one frame to buffer;
 * with mask the 4 key bytes come from 4 x (random() % 256)
 * (co_random, src/core/co_random.c:32-35). */
bool co_ws_frame_serialize(bool fin, uint8_t opcode, bool mask, const void* data,
                           size_t data_size, co_byte_array_t* buffer);

/* co_ws_frame.h:65-71 / co_ws_frame.c:121-247. Parses one frame at
 * data[*index]; *index advances only on CO_WS_PARSE_COMPLETE. */
int co_ws_frame_deserialize(co_ws_frame_t* frame, const uint8_t* data,
                            const size_t data_size, size_t* index);

/* co_ws_frame.h:77-111 / co_ws_frame.c:253-320 */
co_ws_frame_t* co_ws_frame_create(void);
void co_ws_frame_destroy(co_ws_frame_t* frame);
bool co_ws_frame_get_fin(const co_ws_frame_t* frame);
uint8_t co_ws_frame_get_opcode(const co_ws_frame_t* frame);
uint64_t co_ws_frame_get_payload_size(const co_ws_frame_t* frame);
const uint8_t* co_ws_frame_get_payload_data(const co_ws_frame_t* frame);

/* inc/coldforce/ws/co_ws_config.h:29-39 / src/ws/co_ws_config.c:29-35 */
void co_ws_config_set_max_receive_payload_size(size_t max_receive_payload_size);
size_t co_ws_config_get_max_receive_payload_size(void);

#ifdef __cplusplus
}
#endif

#endif /* CFWS_CO_WS_FRAME_H */
