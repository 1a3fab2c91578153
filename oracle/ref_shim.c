/*
 * ref_shim.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Flat ctypes-friendly entry points around the REFERENCE codec, compiled by
 * oracle/Makefile together with four reference translation units taken in
 * place from /root/reference (src/ws/co_ws_frame.c, src/ws/co_ws_config.c,
 * src/core/co_array.c, src/core/co_random.c). Output goes only to
 * oracle/_ref/ (git-ignored). Used to pin the restatement (cfws_oracle.c)
 * and to generate tests/golden/ fixtures; optionally the "reference" CPU
 * baseline in bench.py.
 */
#include <stdlib.h>
#include <string.h>

#include <coldforce/core/co_byte_array.h>
#include <coldforce/ws/co_ws_config.h>
#include <coldforce/ws/co_ws_frame.h>

void ref_srandom(unsigned int seed) { srandom(seed); }

/* co_ws_frame_serialize into a fresh byte array (as co_ws_send does,
 * co_ws_client.c:443-449); copies the wire bytes out. Returns the frame
 * byte count, -1 if serialize failed, -2 if `cap` is too small. */
long long ref_serialize(int fin, unsigned char opcode, int mask, const void* data,
                        unsigned long long n, unsigned char* out,
                        unsigned long long cap)
{
    co_byte_array_t* b = co_byte_array_create();
    if (!co_ws_frame_serialize(fin != 0, opcode, mask != 0, data, (size_t)n, b)) {
        co_byte_array_destroy(b);
        return -1;
    }
    size_t cnt = co_byte_array_get_count(b);
    if (cnt > cap) {
        co_byte_array_destroy(b);
        return -2;
    }
    memcpy(out, co_byte_array_get_ptr(b, 0), cnt);
    co_byte_array_destroy(b);
    return (long long)cnt;
}

/* co_ws_frame_deserialize on a fresh frame; reports the frame fields and
 * copies the payload (plus its NUL terminator) when there is one. */
int ref_deserialize(const unsigned char* data, unsigned long long size,
                    unsigned long long* index, unsigned long long max_payload,
                    int* fin, int* opcode, unsigned long long* payload_size,
                    int* payload_is_null, unsigned char* payload_out,
                    unsigned long long cap)
{
    co_ws_config_set_max_receive_payload_size((size_t)max_payload);
    co_ws_frame_t* f = co_ws_frame_create();
    size_t idx = (size_t)*index;
    int r = co_ws_frame_deserialize(f, data, (size_t)size, &idx);
    *index = idx;
    *fin = f->header.fin;
    *opcode = f->header.opcode;
    *payload_size = f->header.payload_size;
    *payload_is_null = f->payload_data == NULL;
    if (r == 0 && f->payload_data != NULL && f->header.payload_size + 1 <= cap)
        memcpy(payload_out, f->payload_data, (size_t)f->header.payload_size + 1);
    co_ws_frame_destroy(f);
    co_ws_config_set_max_receive_payload_size(CO_WS_CONFIG_DEFAULT_MAX_RECEIVE_PAYLOAD_SIZE);
    return r;
}

/* n equal frames of fs payload bytes taken back to back from `arena`, each
 * through co_ws_frame_serialize into a fresh byte array (co_ws_send's call,
 * co_ws_client.c:443-449), the wire appended to `out`. Keys come from the
 * reference's own random() draws (co_ws_frame.c:93-97). Returns the wire
 * byte count, -1 if a serialize failed, -2 if `cap` is too small. */
long long ref_serialize_run(const unsigned char* arena, unsigned long long n,
                            unsigned long long fs, int fin, unsigned char opcode, int mask,
                            unsigned char* out, unsigned long long cap)
{
    unsigned long long total = 0;
    for (unsigned long long i = 0; i < n; ++i) {
        long long w = ref_serialize(fin, opcode, mask, arena + i * fs, fs, out + total, cap - total);
        if (w < 0) return w;
        total += (unsigned long long)w;
    }
    return (long long)total;
}

/* The receive loop's walk (co_ws_server.c:107-169) over data[0, size): each
 * frame through co_ws_frame_deserialize, its unmasked payload appended to
 * `out`. Returns the frame count, or -(1 + k) when frame k did not decode
 * COMPLETE, or -(1 << 40) if `cap` is too small. */
long long ref_deserialize_run(const unsigned char* data, unsigned long long size,
                              unsigned char* out, unsigned long long cap,
                              unsigned long long* out_len)
{
    size_t index = 0;
    unsigned long long used = 0;
    long long k = 0;
    while (index < size) {
        co_ws_frame_t* f = co_ws_frame_create();
        int r = co_ws_frame_deserialize(f, data, (size_t)size, &index);
        if (r != CO_WS_PARSE_COMPLETE) { co_ws_frame_destroy(f); return -(1 + k); }
        size_t n = (size_t)f->header.payload_size;
        if (used + n > cap) { co_ws_frame_destroy(f); return -(1LL << 40); }
        if (n) memcpy(out + used, f->payload_data, n);
        used += n;
        co_ws_frame_destroy(f);
        ++k;
    }
    *out_len = used;
    return k;
}

/* The receive loop of co_ws_server_on_tcp_receive_ready (co_ws_server.c
 * :107-169) around the reference's own co_ws_frame_deserialize, over
 * data[0, size) from receive index `begin`: the callbacks are replaced by
 * recording each COMPLETE frame's start. Returns the frame count. */
long long ref_index_stream(const unsigned char* data, unsigned long long size,
                           unsigned long long begin, unsigned long long max_payload,
                           unsigned long long* starts, unsigned long long max_frames,
                           unsigned long long* consumed, int* stop)
{
    co_ws_config_set_max_receive_payload_size((size_t)max_payload);
    size_t index = (size_t)begin;
    long long k = 0;
    int st = CO_WS_PARSE_COMPLETE;
    while (size > index) {
        if (size - index < CO_WS_FRAME_HEADER_MIN_SIZE) { st = CO_WS_PARSE_MORE_DATA; break; }
        co_ws_frame_t* f = co_ws_frame_create();
        size_t at = index;
        st = co_ws_frame_deserialize(f, data, (size_t)size, &index);
        co_ws_frame_destroy(f);
        if (st != CO_WS_PARSE_COMPLETE) break;
        if ((unsigned long long)k < max_frames) starts[k] = at;
        ++k;
    }
    *consumed = index;
    *stop = st;
    co_ws_config_set_max_receive_payload_size(CO_WS_CONFIG_DEFAULT_MAX_RECEIVE_PAYLOAD_SIZE);
    return k;
}

/* ---- HTTP/2 DATA framing through the reference's frame codec ------------
 * co_http2_frame.c (compiled in place) encodes / decodes each frame; the
 * split of one buffer into DATA frames restates co_http2_stream_send_data
 * (co_http2_stream.c:933-1013: first frame max_frame_size, then full frames,
 * END_STREAM on the last, one frame when it fits; window assumed open),
 * whose stream machinery needs a live connection. */
#include <coldforce/http2/co_http2_frame.h>

static void ref_h2_one(const uint8_t* data, uint32_t len, int end_stream, uint32_t sid,
                       co_byte_array_t* out)
{
    co_http2_frame_t* f = co_http2_create_data_frame(false, end_stream != 0, data, len, NULL, 0);
    f->header.stream_id = sid;
    co_http2_frame_serialize(f, out);
    co_http2_frame_destroy(f);
}

long long ref_h2_send(const unsigned char* ws, unsigned long long len, unsigned int max_frame,
                      unsigned int sid, unsigned char* out, unsigned long long cap)
{
    co_byte_array_t* b = co_byte_array_create();
    if (len <= max_frame) {
        ref_h2_one(ws, (uint32_t)len, 1, sid, b);
    } else {
        uint32_t index = max_frame;
        ref_h2_one(ws, max_frame, 0, sid, b);
        do {
            uint32_t sz = (len - index > max_frame) ? max_frame : (uint32_t)(len - index);
            ref_h2_one(ws + index, sz, len - index <= max_frame, sid, b);
            index += sz;
        } while (len > index);
    }
    size_t cnt = co_byte_array_get_count(b);
    long long r = (long long)cnt;
    if (cnt > cap) r = -2;
    else memcpy(out, co_byte_array_get_ptr(b, 0), cnt);
    co_byte_array_destroy(b);
    return r;
}

/* co_http2_frame_deserialize on buffer[index..]: result, header fields and
 * the DATA payload (padding stripped). */
int ref_h2_recv(const unsigned char* data, unsigned long long size, unsigned long long* index,
                unsigned int max_frame, unsigned int* length, unsigned int* type,
                unsigned int* flags, unsigned int* sid, unsigned char* payload,
                unsigned long long cap, unsigned long long* payload_len)
{
    co_byte_array_t* b = co_byte_array_create();
    co_byte_array_add(b, data, (size_t)size);
    co_http2_frame_t* f = co_http2_frame_create();
    size_t idx = (size_t)*index;
    int r = co_http2_frame_deserialize(b, &idx, max_frame, f);
    *index = idx;
    *length = f->header.length;
    *type = f->header.type;
    *flags = f->header.flags;
    *sid = f->header.stream_id;
    *payload_len = 0;
    if (r == 0 && f->header.type == 0 && f->payload.data.data_length <= cap) {
        *payload_len = f->payload.data.data_length;
        if (f->payload.data.data_length) memcpy(payload, f->payload.data.data, f->payload.data.data_length);
    }
    if (r == 0) co_http2_frame_destroy(f);
    else free(f);
    co_byte_array_destroy(b);
    return r;
}

/* ---- handshake accept key through the reference's co_sha1.c + co_base64.c
 * (compiled in place): the body of the static co_ws_create_base64_accept_key
 * (co_ws_http_extension.c:26-57), whose file needs the whole HTTP stack. */
#include <coldforce/http/co_base64.h>
#include <coldforce/http/co_sha1.h>

int ref_ws_accept_key(const char* key, unsigned long long key_len, char* out, unsigned long long cap)
{
    size_t key_data_size = (size_t)key_len + 36;
    char* key_data = malloc(key_data_size + 1);
    memcpy(key_data, key, (size_t)key_len);
    memcpy(key_data + key_len, "258EAFA5-E914-47DA-95CA-C5AB0DC85B11", 37);
    uint8_t sha1_hash[CO_SHA1_HASH_SIZE];
    co_sha1(key_data, (uint32_t)key_data_size, sha1_hash);
    free(key_data);
    char* b64;
    size_t b64_len;
    co_base64_encode(sha1_hash, sizeof(sha1_hash), &b64, &b64_len, true);
    int r = (int)b64_len;
    if (b64_len + 1 <= cap) memcpy(out, b64, b64_len + 1);
    else r = -1;
    free(b64);
    return r;
}
