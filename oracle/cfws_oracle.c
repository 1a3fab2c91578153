/*
 * cfws_oracle.c -- TEST INFRASTRUCTURE ONLY (see cfws_oracle.h).
 *
 * Clean-room CPU restatement of the coldforce RFC 6455 frame codec. Every
 * function cites the reference lines whose behaviour it restates; the
 * restatement is deliberately scalar (byte loop, key[i % 4]) so that it also
 * serves as the "port" CPU baseline.
 */
#include "cfws_oracle.h"

#include <stdlib.h>
#include <string.h>

/* ---- byte buffer: co_array_set_count / co_array_add growth rule ---------
 * src/core/co_array.c:83-112 (capacity doubles from 8 until > count),
 * :183-194 (append = grow + memcpy). */

orc_bytes_t* orc_bytes_create(void)
{
    orc_bytes_t* b = (orc_bytes_t*)malloc(sizeof(*b));
    if (!b) return NULL;
    b->capacity = 8;
    b->count = 0;
    b->element_size = 1;
    b->buffer = (uint8_t*)malloc(b->capacity);
    if (!b->buffer) { free(b); return NULL; }
    return b;
}

void orc_bytes_destroy(orc_bytes_t* b)
{
    if (b) { free(b->buffer); free(b); }
}

static bool orc_bytes_append(orc_bytes_t* b, const void* p, size_t n)
{
    size_t need = b->count + n;
    if (b->capacity <= need) {
        size_t cap = b->capacity * 2;
        while (cap <= need) cap *= 2;
        uint8_t* nb = (uint8_t*)realloc(b->buffer, cap);
        if (!nb) return false;
        b->buffer = nb;
        b->capacity = cap;
    }
    memcpy(b->buffer + b->count, p, n);
    b->count = need;
    return true;
}

/* ---- header encode: co_ws_frame.c:34-68 (b0, 7/16/64-bit length) and
 * :70-91 (mask bit + 4 key bytes after the length). The opcode byte is
 * OR-ed verbatim with 0x80 when fin is set (no 4-bit masking). */

uint32_t orc_header_size(uint64_t n, bool mask)
{
    uint32_t h = 2;
    if (n > 65535u) h += 8;
    else if (n > 125u) h += 2;
    if (mask) h += 4;
    return h;
}

static uint32_t orc_encode_header(bool fin, uint8_t opcode, bool mask,
                                  uint32_t key, uint64_t n, uint8_t* h)
{
    uint32_t pos = 2;
    h[0] = (uint8_t)(opcode | (fin ? 0x80u : 0u));
    if (n <= 125u) {
        h[1] = (uint8_t)n;
    } else if (n <= 65535u) {
        h[1] = 126;
        h[pos++] = (uint8_t)(n >> 8);
        h[pos++] = (uint8_t)n;
    } else {
        h[1] = 127;
        for (int s = 56; s >= 0; s -= 8) h[pos++] = (uint8_t)(n >> s);
    }
    if (mask) {
        h[1] |= 0x80u;
        for (int j = 0; j < 4; ++j) h[pos++] = (uint8_t)(key >> (8 * j));
    }
    return pos;
}

/* Key draw: co_random(mask_key, 4) (co_ws_frame.c:84), i.e. 4 sequential
 * (uint8_t)(random() % 256) (src/core/co_random.c:32-35). */
static uint32_t orc_draw_key(void)
{
    uint32_t k = 0;
    for (int j = 0; j < 4; ++j) k |= (uint32_t)(uint8_t)(random() % 256) << (8 * j);
    return k;
}

static void orc_xor_bytes(uint8_t* dst, const uint8_t* src, uint64_t n, uint32_t key)
{
    uint8_t kb[4] = {(uint8_t)key, (uint8_t)(key >> 8), (uint8_t)(key >> 16),
                     (uint8_t)(key >> 24)};
    for (uint64_t i = 0; i < n; ++i) dst[i] = src[i] ^ kb[i % 4];
}

/* co_ws_frame_serialize, co_ws_frame.c:21-119. With mask: malloc(n) first
 * (fails before anything is appended, :74-80), key, XOR (:93-97), append
 * header then payload (:99-104). */
bool orc_serialize(bool fin, uint8_t opcode, bool mask, const void* data,
                   size_t n, orc_bytes_t* buffer)
{
    uint8_t h[16];
    if (!mask) {
        uint32_t hs = orc_encode_header(fin, opcode, false, 0, n, h);
        orc_bytes_append(buffer, h, hs);
        if (n > 0) orc_bytes_append(buffer, data, n);
        return true;
    }
    uint8_t* tmp = (uint8_t*)malloc(n);
    if (tmp == NULL && n > 0) return false;
    uint32_t key = orc_draw_key();
    uint32_t hs = orc_encode_header(fin, opcode, true, key, n, h);
    orc_xor_bytes(tmp, (const uint8_t*)data, n, key);
    orc_bytes_append(buffer, h, hs);
    if (n > 0) orc_bytes_append(buffer, tmp, n);
    free(tmp);
    return true;
}

size_t orc_serialize_keyed(bool fin, uint8_t opcode, bool mask, uint32_t key,
                           const uint8_t* data, size_t n, uint8_t* out)
{
    uint32_t hs = orc_encode_header(fin, opcode, mask, key, n, out);
    if (mask) orc_xor_bytes(out + hs, data, n, key);
    else if (n) memcpy(out + hs, data, n);
    return hs + n;
}

/* ---- deserialize: co_ws_frame.c:121-247 ------------------------------- */

void orc_frame_init(orc_frame_t* f)
{   /* co_ws_frame_create, co_ws_frame.c:266-269 */
    f->header.fin = false;
    f->header.opcode = 0xff;
    f->header.payload_size = 0;
    f->payload_data = NULL;
}

void orc_frame_clear(orc_frame_t* f)
{
    free(f->payload_data);
    f->payload_data = NULL;
}

static uint64_t orc_be(const uint8_t* p, int nbytes)
{
    uint64_t v = 0;
    for (int i = 0; i < nbytes; ++i) v = (v << 8) | p[i];
    return v;
}

int orc_deserialize(orc_frame_t* f, const uint8_t* data, size_t data_size,
                    size_t* index, size_t max_payload)
{
    size_t p = *index;
    uint8_t b0 = data[p++];
    /* :136-142 -- RSV bits stay in the opcode, so any RSV bit => invalid. */
    f->header.fin = (b0 & 0x80u) != 0;
    f->header.opcode = (uint8_t)(b0 & 0x7fu);
    if (f->header.opcode > 0x0f) return ORC_ERROR_INVALID_FRAME;
    f->header.payload_size = 0;   /* :144-145 */
    f->payload_data = NULL;

    uint8_t b1 = data[p++];       /* :147-153 */
    bool mask = (b1 & 0x80u) != 0;
    uint8_t l7 = (uint8_t)(b1 & 0x7fu);
    if (l7 <= 125) {               /* :155-158 */
        f->header.payload_size = l7;
    } else {                       /* :159-188, no minimal-encoding check */
        int ext = (l7 == 126) ? 2 : 8;
        if (data_size - p < (size_t)ext) return ORC_PARSE_MORE_DATA;
        f->header.payload_size = orc_be(data + p, ext);
        p += (size_t)ext;
    }
    uint32_t key = 0;
    if (mask) {                    /* :190-201 */
        if (data_size - p < 4) return ORC_PARSE_MORE_DATA;
        key = (uint32_t)data[p] | (uint32_t)data[p + 1] << 8 |
              (uint32_t)data[p + 2] << 16 | (uint32_t)data[p + 3] << 24;
        p += 4;
    }
    uint64_t n = f->header.payload_size;
    /* :203-206 MORE_DATA is decided before the size limit (:208-213). */
    if ((uint64_t)(data_size - p) < n) return ORC_PARSE_MORE_DATA;
    if (n > (uint64_t)max_payload) return ORC_ERROR_DATA_TOO_BIG;
    if (n > 0) {                   /* :214-230 copy + NUL terminator */
        f->payload_data = (uint8_t*)malloc((size_t)n + 1);
        if (f->payload_data == NULL) return ORC_ERROR_OUT_OF_MEMORY;
        f->payload_data[n] = 0;
        if (mask) orc_xor_bytes(f->payload_data, data + p, n, key);  /* :232-242 */
        else memcpy(f->payload_data, data + p, (size_t)n);
        p += (size_t)n;
    }
    *index = p;                    /* :244, only on COMPLETE */
    return ORC_PARSE_COMPLETE;
}

/* ---- batch mirrors of the device ABI ---------------------------------- */

/* The keys n sequential co_ws_frame_serialize calls draw right after
 * srandom(seed) (co_net.c:46 seeds, co_random.c:32-35 draws): the same
 * generator (glibc's TYPE_3 additive generator on a 128-byte table, what
 * srandom seeds by default) run on a private copy through random_r, so no
 * other thread's rand()/random() -- the GPU runtime's libraries make such
 * calls on threads of their own -- can interleave with the draws. */
void orc_keys(uint32_t seed, size_t n, const uint8_t* mask_flags, uint32_t* keys)
{
    char table[128];
    struct random_data rd;
    memset(&rd, 0, sizeof rd);
    memset(table, 0, sizeof table);
    initstate_r(seed, table, sizeof table, &rd);
    for (size_t i = 0; i < n; ++i) {
        uint32_t k = 0;
        if (mask_flags == NULL || mask_flags[i]) {
            for (int j = 0; j < 4; ++j) {
                int32_t r = 0;
                random_r(&rd, &r);
                k |= (uint32_t)(uint8_t)(r % 256) << (8 * j);
            }
        }
        keys[i] = k;
    }
}

uint64_t orc_serialize_batch(const uint8_t* payload, orc_desc_t* d, size_t n,
                             uint8_t* wire)
{
    uint64_t off = 0;
    for (size_t i = 0; i < n; ++i) {
        d[i].wire_off = off;
        d[i].header_size = (uint8_t)orc_header_size(d[i].payload_size, d[i].mask != 0);
        off += orc_serialize_keyed(d[i].fin != 0, d[i].opcode, d[i].mask != 0,
                                   d[i].mask_key, payload + d[i].payload_off,
                                   (size_t)d[i].payload_size, wire + off);
    }
    return off;
}

/* Parse the header at `start` without copying the payload: the same
 * decisions as orc_deserialize (co_ws_frame.c:131-213). */
static int orc_parse_header(const uint8_t* w, uint64_t size, uint64_t start,
                            uint64_t max_payload, orc_desc_t* d)
{
    memset(d, 0, sizeof(*d));
    d->wire_off = start;
    if (start > size || size - start < 2) return ORC_PARSE_MORE_DATA;  /* caller precheck */
    uint8_t b0 = w[start], b1 = w[start + 1];
    d->fin = (uint8_t)(b0 >> 7);
    d->opcode = (uint8_t)(b0 & 0x7f);
    if (d->opcode > 0x0f) return ORC_ERROR_INVALID_FRAME;
    uint64_t p = start + 2;
    uint8_t l7 = b1 & 0x7f;
    d->mask = (uint8_t)(b1 >> 7);
    if (l7 <= 125) {
        d->payload_size = l7;
    } else {
        int ext = (l7 == 126) ? 2 : 8;
        if (size - p < (uint64_t)ext) return ORC_PARSE_MORE_DATA;
        d->payload_size = orc_be(w + p, ext);
        p += (uint64_t)ext;
    }
    if (d->mask) {
        if (size - p < 4) return ORC_PARSE_MORE_DATA;
        d->mask_key = (uint32_t)w[p] | (uint32_t)w[p + 1] << 8 |
                      (uint32_t)w[p + 2] << 16 | (uint32_t)w[p + 3] << 24;
        p += 4;
    }
    d->header_size = (uint8_t)(p - start);
    if (size - p < d->payload_size) return ORC_PARSE_MORE_DATA;
    if (d->payload_size > max_payload) return ORC_ERROR_DATA_TOO_BIG;
    return ORC_PARSE_COMPLETE;
}

static int orc_is_control(const orc_desc_t* d)
{   /* co_ws_frame.h:32-34: opcodes 0x8-0xF are control frames */
    return d->opcode <= 0x0f && (d->opcode & 0x08) != 0;
}

uint64_t orc_deserialize_batch(const uint8_t* wire, uint64_t wire_size,
                               const uint64_t* starts, size_t n,
                               uint64_t max_payload, uint32_t align, uint32_t flags,
                               orc_desc_t* d, int32_t* status,
                               uint8_t* payload, uint64_t cap)
{
    const int reasm = (flags & ORC_DESERIALIZE_REASSEMBLE) != 0;
    if (align == 0 || reasm) align = 1;
    /* layout first: it depends only on the parse results */
    uint64_t off = 0;
    for (size_t i = 0; i < n; ++i) {
        status[i] = orc_parse_header(wire, wire_size, starts[i], max_payload, &d[i]);
        int ok = status[i] == ORC_PARSE_COMPLETE && !(reasm && orc_is_control(&d[i]));
        uint64_t len = ok ? d[i].payload_size : 0;
        d[i].payload_off = off;
        off += (len + align - 1) / align * align;
    }
    uint64_t data_total = off, ctrl = 0;
    if (reasm) {
        for (size_t i = 0; i < n; ++i) {
            if (!orc_is_control(&d[i])) continue;
            d[i].payload_off = data_total + ctrl;
            if (status[i] == ORC_PARSE_COMPLETE) ctrl += d[i].payload_size;
        }
    }
    uint64_t total = data_total + ctrl;
    if (total > cap) total = cap;
    /* then the bytes: payloads, zero padding, capacity rule */
    for (size_t i = 0; i < n; ++i) {
        uint64_t o = d[i].payload_off;
        uint64_t len = status[i] == ORC_PARSE_COMPLETE ? d[i].payload_size : 0;
        uint64_t span = reasm ? len : (len + align - 1) / align * align;
        if (len && o + len > cap) {
            status[i] = ORC_ERROR_OUT_OF_MEMORY;
            len = 0;
        }
        if (len) {
            const uint8_t* src = wire + starts[i] + d[i].header_size;
            if (d[i].mask) orc_xor_bytes(payload + o, src, len, d[i].mask_key);
            else memcpy(payload + o, src, (size_t)len);
        }
        uint64_t end = o + span < cap ? o + span : cap;
        if (end > o + len) memset(payload + o + len, 0, (size_t)(end - o - len));
    }
    return total;
}

/* ---- split ops: the header and payload passes of co_ws_frame.c ------- */

/* Copies src[0, n) ^ key[k % 4] (mask) or src (no mask) to dst, keeping only
 * the destination bytes below `lim` (dst_off = dst's offset in its arena). */
static void orc_put_payload(uint8_t* arena, uint64_t dst_off, uint64_t lim, const uint8_t* src,
                            uint64_t n, bool mask, uint32_t key)
{
    if (dst_off >= lim) return;
    if (n > lim - dst_off) n = lim - dst_off;
    if (mask) orc_xor_bytes(arena + dst_off, src, n, key);
    else if (n) memcpy(arena + dst_off, src, (size_t)n);
}

void orc_encode_headers(orc_desc_t* d, size_t n, uint8_t* wire, uint64_t cap)
{   /* co_ws_frame.c:34-91 */
    for (size_t i = 0; i < n; ++i) {
        uint8_t h[16];
        uint32_t hs = orc_encode_header(d[i].fin != 0, d[i].opcode, d[i].mask != 0, d[i].mask_key,
                                        d[i].payload_size, h);
        d[i].header_size = (uint8_t)hs;
        for (uint32_t k = 0; k < hs; ++k)
            if (d[i].wire_off + k < cap) wire[d[i].wire_off + k] = h[k];
    }
}

void orc_parse_headers(const uint8_t* wire, uint64_t size, const uint64_t* starts, size_t n,
                       uint64_t max_payload, orc_desc_t* d, int32_t* status)
{   /* co_ws_frame.c:131-213 */
    for (size_t i = 0; i < n; ++i)
        status[i] = orc_parse_header(wire, size, starts[i], max_payload, &d[i]);
}

void orc_mask_batch(const uint8_t* payload, const orc_desc_t* d, size_t n, uint8_t* wire,
                    uint64_t cap)
{   /* co_ws_frame.c:93-97 */
    for (size_t i = 0; i < n; ++i)
        orc_put_payload(wire, d[i].wire_off + orc_header_size(d[i].payload_size, d[i].mask != 0),
                        cap, payload + d[i].payload_off, d[i].payload_size, d[i].mask != 0,
                        d[i].mask_key);
}

void orc_unmask_batch(const uint8_t* wire, const orc_desc_t* d, const int32_t* status, size_t n,
                      uint8_t* payload, uint64_t cap)
{   /* co_ws_frame.c:232-242 */
    for (size_t i = 0; i < n; ++i) {
        if (status && status[i] != ORC_PARSE_COMPLETE) continue;
        orc_put_payload(payload, d[i].payload_off, cap, wire + d[i].wire_off + d[i].header_size,
                        d[i].payload_size, d[i].mask != 0, d[i].mask_key);
    }
}

/* The receive loop of co_ws_server_on_tcp_receive_ready
 * (co_ws_server.c:107-169; co_ws_client.c:200-270 is the same walk) over one
 * connection's received bytes buf[begin, end): stop when under 2 bytes
 * remain (:109-113) or a frame is not COMPLETE (:144-166); the receive index
 * advances only over COMPLETE frames (co_ws_frame.c:244). */
size_t orc_index_stream(const uint8_t* buf, uint64_t begin, uint64_t end, uint64_t max_payload,
                        uint64_t* starts, size_t max_frames, uint64_t* consumed, int32_t* stop)
{
    size_t k = 0;
    uint64_t p = begin;
    int32_t st = ORC_PARSE_COMPLETE;
    orc_desc_t d;
    while (end > p) {
        if (end - p < 2) { st = ORC_PARSE_MORE_DATA; break; }
        /* the frame's data_size is the whole receive buffer: bytes before
         * `begin` are only ever skipped, so parse the tail from p. */
        st = orc_parse_header(buf, end, p, max_payload, &d);
        if (st != ORC_PARSE_COMPLETE) break;
        if (k < max_frames) starts[k] = p;
        ++k;
        p += d.header_size + d.payload_size;
    }
    if (consumed) *consumed = p;
    if (stop) *stop = st;
    return k;
}

size_t orc_index_frames(const uint8_t* wire, uint64_t size, uint64_t max_payload,
                        uint64_t* starts, size_t max_frames, uint64_t* consumed)
{
    size_t k = 0;
    uint64_t p = 0;
    orc_desc_t d;
    while (k < max_frames && p < size) {
        if (orc_parse_header(wire, size, p, max_payload, &d) != ORC_PARSE_COMPLETE) break;
        starts[k++] = p;
        p += d.header_size + d.payload_size;
    }
    if (consumed) *consumed = p;
    return k;
}

/* ---- synthetic data ---------------------------------------------------- */

static uint64_t orc_splitmix(uint64_t seed, uint64_t i)
{
    uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

void orc_fill_splitmix(uint8_t* out, uint64_t n, uint64_t seed, uint64_t base)
{
    for (uint64_t i = 0; i < n; ++i) {
        uint64_t o = base + i;
        out[i] = (uint8_t)(orc_splitmix(seed, o >> 3) >> (8 * (o & 7)));
    }
}

/* ---- flat entry points for ctypes (same shapes as ref_shim.c) ---------- */

void orc_srandom(unsigned int seed) { srandom(seed); }

long long orc_serialize_flat(int fin, unsigned char opcode, int mask, const void* data,
                             unsigned long long n, unsigned char* out,
                             unsigned long long cap)
{
    orc_bytes_t* b = orc_bytes_create();
    if (!b) return -1;
    if (!orc_serialize(fin != 0, opcode, mask != 0, data, (size_t)n, b)) {
        orc_bytes_destroy(b);
        return -1;
    }
    long long cnt = (long long)b->count;
    if ((unsigned long long)cnt > cap) cnt = -2;
    else memcpy(out, b->buffer, b->count);
    orc_bytes_destroy(b);
    return cnt;
}

int orc_deserialize_flat(const unsigned char* data, unsigned long long size,
                         unsigned long long* index, unsigned long long max_payload,
                         int* fin, int* opcode, unsigned long long* payload_size,
                         int* payload_is_null, unsigned char* payload_out,
                         unsigned long long cap)
{
    orc_frame_t f;
    orc_frame_init(&f);
    size_t idx = (size_t)*index;
    int r = orc_deserialize(&f, data, (size_t)size, &idx, (size_t)max_payload);
    *index = idx;
    *fin = f.header.fin;
    *opcode = f.header.opcode;
    *payload_size = f.header.payload_size;
    *payload_is_null = f.payload_data == NULL;
    if (r == 0 && f.payload_data != NULL && f.header.payload_size + 1 <= cap)
        memcpy(payload_out, f.payload_data, (size_t)f.header.payload_size + 1);
    orc_frame_clear(&f);
    return r;
}

/* ---- WebSocket over HTTP/2 --------------------------------------------- */

/* DATA frame encode, co_http2_frame.c:33-72 (no padding on send,
 * co_http2_create_data_frame(..., NULL, 0), co_http2_frame.c:628-700). */
static uint64_t orc_h2_data_frame(const uint8_t* data, uint32_t len, int end_stream,
                                  uint32_t sid, uint8_t* out)
{
    out[0] = (uint8_t)(len >> 16);
    out[1] = (uint8_t)(len >> 8);
    out[2] = (uint8_t)len;
    out[3] = 0;                                   /* DATA */
    out[4] = end_stream ? 0x1 : 0x0;              /* END_STREAM */
    sid &= 0x7fffffffu;
    out[5] = (uint8_t)(sid >> 24);
    out[6] = (uint8_t)(sid >> 16);
    out[7] = (uint8_t)(sid >> 8);
    out[8] = (uint8_t)sid;
    if (len) memcpy(out + 9, data, len);
    return 9 + (uint64_t)len;
}

/* co_http2_stream_send_data (co_http2_stream.c:933-1013) with end_stream and
 * a window that admits the frame: first frame max_frame_size, then full
 * frames, the last one END_STREAM; one frame when it fits. */
uint64_t orc_h2_send(const uint8_t* ws, uint64_t len, uint32_t S, uint32_t sid, uint8_t* out)
{
    if (len <= S) return orc_h2_data_frame(ws, (uint32_t)len, 1, sid, out);
    uint64_t at = orc_h2_data_frame(ws, S, 0, sid, out), idx = S;
    while (len > idx) {
        uint32_t sz = (len - idx > S) ? S : (uint32_t)(len - idx);
        at += orc_h2_data_frame(ws + idx, sz, len - idx <= S, sid, out + at);
        idx += sz;
    }
    return at;
}

uint64_t orc_h2_serialize_batch(const uint8_t* payload, orc_desc_t* d, size_t n, uint32_t sid,
                                uint32_t S, uint8_t* tmp, uint8_t* out)
{
    uint64_t at = 0;
    for (size_t i = 0; i < n; ++i) {
        d[i].header_size = (uint8_t)orc_header_size(d[i].payload_size, d[i].mask != 0);
        size_t w = orc_serialize_keyed(d[i].fin != 0, d[i].opcode, d[i].mask != 0, d[i].mask_key,
                                       payload + d[i].payload_off, (size_t)d[i].payload_size, tmp);
        at += orc_h2_send(tmp, w, S, sid, out + at);
    }
    return at;
}

/* co_http2_frame_deserialize's DATA path (co_http2_frame.c:211-300): status
 * 0 / 1 (MORE_DATA) / -1 (PARSE_ERROR: length > max frame size; also a pad
 * length that does not fit, where the reference underflows) / 3 (not DATA).
 * DATA payloads (padding stripped) are pooled until END_STREAM
 * (co_http2_stream.c:550-608); each pooled message is then parsed by
 * co_ws_frame_deserialize against its own size (co_ws_http2_extension.c:
 * 134-164). Layout of the WS payloads as orc_deserialize_batch (flags 0). */
uint64_t orc_h2_deserialize_batch(const uint8_t* h2, uint64_t size, const uint64_t* index,
                                  size_t n, uint32_t S, int32_t* h2_status, uint8_t* pool,
                                  uint64_t pool_cap, uint64_t max_payload, uint32_t align,
                                  orc_desc_t* msg_desc, int32_t* msg_status, uint8_t* payload,
                                  uint64_t payload_cap, uint64_t* n_msg_out)
{
    uint64_t pooled = 0, n_msg = 0, msg_start = 0;
    uint64_t* starts = (uint64_t*)malloc(sizeof(uint64_t) * (n + 1));
    uint64_t* ends = (uint64_t*)malloc(sizeof(uint64_t) * (n + 1));
    for (size_t i = 0; i < n; ++i) {
        uint64_t s = index[i];
        int st = 0;
        uint64_t dlen = 0, hs = 9;
        int es = 0;
        if (s > size || size - s < 9) st = 1;
        else {
            uint64_t len = (uint64_t)h2[s] << 16 | (uint64_t)h2[s + 1] << 8 | h2[s + 2];
            if (len > S) st = -1;
            else if (size - s - 9 < len) st = 1;
            else if (h2[s + 3] != 0) st = 3;
            else {
                uint64_t pad = 0;
                if (h2[s + 4] & 0x8) {
                    if (len < 1) st = -1;
                    else {
                        pad = h2[s + 9];
                        hs = 10;
                        if (pad + 1 > len) st = -1;
                    }
                }
                if (st == 0) {
                    dlen = len - (hs - 9) - pad;
                    es = h2[s + 4] & 0x1;
                }
            }
        }
        /* the pool layout is fixed by the parse; capacity only marks */
        uint64_t at = pooled;
        if (st == 0) pooled += dlen;
        if (st == 0 && dlen && at + dlen > pool_cap) st = ORC_ERROR_OUT_OF_MEMORY;
        h2_status[i] = st;
        if (st == 0) {
            memcpy(pool + at, h2 + s + hs, (size_t)dlen);
            if (es) {
                starts[n_msg] = msg_start;
                ends[n_msg] = at + dlen;
                ++n_msg;
                msg_start = at + dlen;
            }
        }
    }
    /* each message: co_ws_frame_deserialize(frame, msg, msg_size, &0) */
    uint64_t off = 0, total;
    if (align == 0) align = 1;
    for (uint64_t m = 0; m < n_msg; ++m) {
        uint64_t end = ends[m] < pool_cap ? ends[m] : pool_cap;   /* pool bytes only */
        uint64_t avail = end > starts[m] ? end - starts[m] : 0;
        int st = orc_parse_header(pool + starts[m], avail, 0, max_payload, &msg_desc[m]);
        msg_desc[m].wire_off = starts[m];
        uint64_t len = st == ORC_PARSE_COMPLETE ? msg_desc[m].payload_size : 0;
        uint64_t next = off + (len + align - 1) / align * align;
        if (len && off + len > payload_cap) {
            st = ORC_ERROR_OUT_OF_MEMORY;
            len = 0;
        }
        msg_status[m] = st;
        msg_desc[m].payload_off = off;
        if (len) {
            const uint8_t* src = pool + starts[m] + msg_desc[m].header_size;
            if (msg_desc[m].mask) orc_xor_bytes(payload + off, src, len, msg_desc[m].mask_key);
            else memcpy(payload + off, src, (size_t)len);
        }
        uint64_t pad_end = next < payload_cap ? next : payload_cap;
        if (pad_end > off + len) memset(payload + off + len, 0, (size_t)(pad_end - off - len));
        off = next;
    }
    total = off < payload_cap ? off : payload_cap;
    free(starts);
    free(ends);
    if (n_msg_out) *n_msg_out = n_msg;
    return total;
}

/* ---- handshake accept key ----------------------------
 * co_ws_create_base64_accept_key (co_ws_http_extension.c:26-57):
 * base64(SHA-1(key || GUID)) with '=' padding. SHA-1 as FIPS 180-4 (the
 * reference's co_sha1.c:55-283 is the classic public-domain transform);
 * base64 with the standard alphabet (co_base64.c:17-91). */
static uint32_t orc_rol(uint32_t v, int b) { return (v << b) | (v >> (32 - b)); }

static void orc_sha1_block(uint32_t st[5], const uint8_t* p)
{
    uint32_t w[80];
    for (int i = 0; i < 16; ++i)
        w[i] = (uint32_t)p[4 * i] << 24 | (uint32_t)p[4 * i + 1] << 16 | (uint32_t)p[4 * i + 2] << 8 | p[4 * i + 3];
    for (int i = 16; i < 80; ++i) w[i] = orc_rol(w[i - 3] ^ w[i - 8] ^ w[i - 14] ^ w[i - 16], 1);
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4];
    for (int i = 0; i < 80; ++i) {
        uint32_t f, k;
        if (i < 20) { f = (b & c) | (~b & d); k = 0x5a827999u; }
        else if (i < 40) { f = b ^ c ^ d; k = 0x6ed9eba1u; }
        else if (i < 60) { f = (b & c) | (b & d) | (c & d); k = 0x8f1bbcdcu; }
        else { f = b ^ c ^ d; k = 0xca62c1d6u; }
        const uint32_t t = orc_rol(a, 5) + f + e + k + w[i];
        e = d; d = c; c = orc_rol(b, 30); b = a; a = t;
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e;
}

void orc_sha1(const void* data, uint64_t n, uint8_t out[20])
{
    uint32_t st[5] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u, 0xc3d2e1f0u};
    const uint8_t* p = (const uint8_t*)data;
    uint64_t i = 0;
    for (; i + 64 <= n; i += 64) orc_sha1_block(st, p + i);
    uint8_t tail[128];
    memset(tail, 0, sizeof tail);
    const uint64_t r = n - i;
    if (r) memcpy(tail, p + i, (size_t)r);
    tail[r] = 0x80;
    const uint64_t tl = r + 9 <= 64 ? 64 : 128;
    const uint64_t bits = n * 8;
    for (int j = 0; j < 8; ++j) tail[tl - 1 - j] = (uint8_t)(bits >> (8 * j));
    orc_sha1_block(st, tail);
    if (tl == 128) orc_sha1_block(st, tail + 64);
    for (int j = 0; j < 20; ++j) out[j] = (uint8_t)(st[j >> 2] >> (8 * (3 - (j & 3))));
}

uint64_t orc_base64(const uint8_t* src, uint64_t n, char* out)
{
    static const char tab[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
    uint64_t o = 0;
    for (uint64_t i = 0; i < n; i += 3) {
        const uint32_t b0 = src[i], b1 = i + 1 < n ? src[i + 1] : 0, b2 = i + 2 < n ? src[i + 2] : 0;
        const uint32_t v = b0 << 16 | b1 << 8 | b2;
        out[o++] = tab[(v >> 18) & 63];
        out[o++] = tab[(v >> 12) & 63];
        out[o++] = i + 1 < n ? tab[(v >> 6) & 63] : '=';
        out[o++] = i + 2 < n ? tab[v & 63] : '=';
    }
    out[o] = 0;
    return o;
}

void orc_ws_accept_key(const char* key, uint64_t key_len, char out[29])
{
    static const char guid[] = "258EAFA5-E914-47DA-95CA-C5AB0DC85B11";
    uint8_t* buf = (uint8_t*)malloc((size_t)key_len + 36 + 1);
    memcpy(buf, key, (size_t)key_len);
    memcpy(buf + key_len, guid, 36);
    uint8_t h[20];
    orc_sha1(buf, key_len + 36, h);
    free(buf);
    orc_base64(h, 20, out);
}
