/*
 * cpu_bench.c -- TEST INFRASTRUCTURE ONLY: the CPU baseline bench.py reports
 * beside the GPU numbers (cpu_baseline leg).
 *
 * Per frame it does what a coldforce client/server pair does per 64 KiB
 * binary frame: the client's co_ws_send path (co_ws_client.c:427-460:
 * fresh byte array + co_ws_frame_serialize(mask = true)), then the
 * server's receive loop (co_ws_server.c:107-169: co_ws_frame_create +
 * co_ws_frame_deserialize + destroy). Frames are split into contiguous
 * ranges over `threads` pthreads; each phase is timed separately.
 *
 * Compiled twice by oracle/Makefile:
 *   - against the restatement (cfws_oracle.c)          -> kind "port"
 *   - with -DCFWS_BENCH_REF against the reference codec
 *     compiled from /root/reference/src                 -> kind "reference"
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#ifdef CFWS_BENCH_REF
int ref_ws_accept_key(const char* key, unsigned long long key_len, char* out, unsigned long long cap);
#define ACCEPT_BENCH_FN ref_accept_bench
#define ACCEPT(k, n, out) ref_ws_accept_key((k), (n), (out), 29)
#include <coldforce/core/co_byte_array.h>
#include <coldforce/ws/co_ws_config.h>
#include <coldforce/ws/co_ws_frame.h>
typedef co_byte_array_t bench_buf_t;
typedef co_ws_frame_t bench_frame_t;
#define BENCH_FN ref_cpu_bench
#define BUF_CREATE() co_byte_array_create()
#define BUF_DESTROY(b) co_byte_array_destroy(b)
#define BUF_PTR(b) co_byte_array_get_ptr((b), 0)
#define BUF_COUNT(b) co_byte_array_get_count(b)
#define SERIALIZE(data, n, b) co_ws_frame_serialize(true, 0x2, true, (data), (n), (b))
#define FRAME_NEW() co_ws_frame_create()
#define FRAME_FREE(f) co_ws_frame_destroy(f)
#define DESERIALIZE(f, p, n, idx) co_ws_frame_deserialize((f), (p), (n), (idx))
#else
#include "cfws_oracle.h"
#define ACCEPT_BENCH_FN orc_accept_bench
#define ACCEPT(k, n, out) orc_ws_accept_key((k), (n), (out))
typedef orc_bytes_t bench_buf_t;
typedef orc_frame_t bench_frame_t;
#define BENCH_FN orc_cpu_bench
#define BUF_CREATE() orc_bytes_create()
#define BUF_DESTROY(b) orc_bytes_destroy(b)
#define BUF_PTR(b) ((b)->buffer)
#define BUF_COUNT(b) ((b)->count)
#define SERIALIZE(data, n, b) orc_serialize(true, 0x2, true, (data), (n), (b))
static bench_frame_t* orc_frame_new(void)
{
    bench_frame_t* f = (bench_frame_t*)malloc(sizeof(*f));
    if (f) orc_frame_init(f);
    return f;
}
static void orc_frame_free(bench_frame_t* f)
{
    if (f) { orc_frame_clear(f); free(f); }
}
#define FRAME_NEW() orc_frame_new()
#define FRAME_FREE(f) orc_frame_free(f)
#define DESERIALIZE(f, p, n, idx) orc_deserialize((f), (p), (n), (idx), (size_t)32 << 20)
#endif

typedef struct {
    const uint8_t* payload;
    uint64_t first, count, frame_size;
    bench_buf_t** wire;
    volatile uint64_t sink;
    int fail;
} bench_job_t;

static void* bench_mask(void* arg)
{
    bench_job_t* j = (bench_job_t*)arg;
    for (uint64_t i = 0; i < j->count; ++i) {
        bench_buf_t* b = BUF_CREATE();
        if (!b || !SERIALIZE(j->payload + (j->first + i) * j->frame_size, j->frame_size, b))
            j->fail = 1;
        j->wire[i] = b;
    }
    return NULL;
}

static void* bench_unmask(void* arg)
{
    bench_job_t* j = (bench_job_t*)arg;
    uint64_t s = 0;
    for (uint64_t i = 0; i < j->count; ++i) {
        bench_frame_t* f = FRAME_NEW();
        size_t idx = 0;
        if (DESERIALIZE(f, BUF_PTR(j->wire[i]), BUF_COUNT(j->wire[i]), &idx) != 0) j->fail = 1;
        else s += f->payload_data[0];
        FRAME_FREE(f);
    }
    j->sink = s;
    return NULL;
}

static double bench_now(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

static double bench_phase(void* (*fn)(void*), bench_job_t* jobs, int threads)
{
    pthread_t tid[256];
    double t0 = bench_now();
    for (int t = 0; t < threads; ++t) pthread_create(&tid[t], NULL, fn, &jobs[t]);
    for (int t = 0; t < threads; ++t) pthread_join(tid[t], NULL);
    return bench_now() - t0;
}

int BENCH_FN(uint64_t n_frames, uint64_t frame_size, int threads, int iters,
             double* mask_seconds, double* unmask_seconds)
{
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    uint8_t* payload = (uint8_t*)malloc(n_frames * frame_size);
    bench_buf_t** wire = (bench_buf_t**)calloc(n_frames, sizeof(*wire));
    bench_job_t* jobs = (bench_job_t*)calloc((size_t)threads, sizeof(*jobs));
    if (!payload || !wire || !jobs) return -1;
    for (uint64_t i = 0; i < n_frames * frame_size; ++i)
        payload[i] = (uint8_t)(i * 2654435761u >> 13);
    uint64_t per = n_frames / (uint64_t)threads, rem = n_frames % (uint64_t)threads, at = 0;
    for (int t = 0; t < threads; ++t) {
        uint64_t c = per + ((uint64_t)t < rem ? 1 : 0);
        jobs[t].payload = payload;
        jobs[t].first = at;
        jobs[t].count = c;
        jobs[t].frame_size = frame_size;
        jobs[t].wire = wire + at;
        at += c;
    }
    double ms = 0, us = 0;
    int fail = 0;
    for (int it = 0; it < iters; ++it) {
        ms += bench_phase(bench_mask, jobs, threads);
        us += bench_phase(bench_unmask, jobs, threads);
        for (uint64_t i = 0; i < n_frames; ++i) { BUF_DESTROY(wire[i]); wire[i] = NULL; }
    }
    for (int t = 0; t < threads; ++t) fail |= jobs[t].fail;
    free(jobs);
    free(wire);
    free(payload);
    *mask_seconds = ms;
    *unmask_seconds = us;
    return fail ? -2 : 0;
}

/* ---- handshake accept keys ---------------------------
 * co_ws_create_base64_accept_key (co_ws_http_extension.c:26-57) once per
 * key, keys[off[i], off[i+1]), split into contiguous ranges over `threads`
 * pthreads, `iters` times: the connection storm a server's threads meet one
 * upgrade request at a time. */
typedef struct {
    const char* keys;
    const uint64_t* off;
    uint64_t first, count;
    int iters;
    volatile uint64_t sink;
} accept_job_t;

static void* accept_run(void* arg)
{
    accept_job_t* j = (accept_job_t*)arg;
    char out[32];
    uint64_t s = 0;
    for (int it = 0; it < j->iters; ++it)
        for (uint64_t i = j->first; i < j->first + j->count; ++i) {
            ACCEPT(j->keys + j->off[i], j->off[i + 1] - j->off[i], out);
            s += (uint8_t)out[0];
        }
    j->sink = s;
    return NULL;
}

int ACCEPT_BENCH_FN(const char* keys, const uint64_t* off, uint64_t n, int threads, int iters,
                    double* seconds)
{
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    accept_job_t* jobs = (accept_job_t*)calloc((size_t)threads, sizeof(*jobs));
    if (!jobs) return -1;
    uint64_t per = n / (uint64_t)threads, rem = n % (uint64_t)threads, at = 0;
    for (int t = 0; t < threads; ++t) {
        uint64_t c = per + ((uint64_t)t < rem ? 1 : 0);
        jobs[t].keys = keys;
        jobs[t].off = off;
        jobs[t].first = at;
        jobs[t].count = c;
        jobs[t].iters = iters;
        at += c;
    }
    pthread_t tid[256];
    double t0 = bench_now();
    for (int t = 0; t < threads; ++t) pthread_create(&tid[t], NULL, accept_run, &jobs[t]);
    for (int t = 0; t < threads; ++t) pthread_join(tid[t], NULL);
    *seconds = bench_now() - t0;
    free(jobs);
    return 0;
}

#ifdef CFWS_BENCH_REF
/* ---- WebSocket over HTTP/2 (config 5), reference only -------------------
 * Per WS frame, the send side of co_http2_stream_send_ws_frame
 * (co_ws_http2_extension.c:166-199): co_ws_frame_serialize(mask) into a
 * fresh byte array, then co_http2_stream_send_data's split
 * (co_http2_stream.c:933-1013: DATA frames of at most max_frame bytes,
 * END_STREAM on the last) with each DATA frame made by
 * co_http2_create_data_frame and serialized by co_http2_frame_serialize
 * (co_http2_frame.c:33-72) into the connection's send bytes (one byte
 * array per WS frame here; the stream's window assumed open). The receive
 * side: co_http2_frame_deserialize (co_http2_frame.c:211-300) of each DATA
 * frame, the stream's data pooling (co_http2_stream.c:550-608: the payload
 * taken as is when END_STREAM comes with an empty pool, else appended and
 * NUL-terminated), then co_http2_stream_receive_ws_frame's
 * co_ws_frame_deserialize (co_ws_http2_extension.c:134-164) and destroy.
 * All of it the reference's own code, compiled in place. */
#include <coldforce/http2/co_http2_frame.h>

typedef struct {
    const uint8_t* payload;
    uint64_t first, count, frame_size;
    uint32_t max_frame;
    co_byte_array_t** wire;
    volatile uint64_t sink;
    int fail;
} h2_job_t;

static void h2_data_frame(const uint8_t* data, uint32_t len, bool end_stream, co_byte_array_t* out)
{
    co_http2_frame_t* f = co_http2_create_data_frame(false, end_stream, data, len, NULL, 0);
    f->header.stream_id = 1;
    co_http2_frame_serialize(f, out);
    co_http2_frame_destroy(f);
}

static double h2_phase(void* (*fn)(void*), h2_job_t* jobs, int threads)
{
    pthread_t tid[256];
    double t0 = bench_now();
    for (int t = 0; t < threads; ++t) pthread_create(&tid[t], NULL, fn, &jobs[t]);
    for (int t = 0; t < threads; ++t) pthread_join(tid[t], NULL);
    return bench_now() - t0;
}

static void* h2_send_run(void* arg)
{
    h2_job_t* j = (h2_job_t*)arg;
    for (uint64_t i = 0; i < j->count; ++i) {
        co_byte_array_t* ws = co_byte_array_create();
        if (!co_ws_frame_serialize(true, 0x2, true, j->payload + (j->first + i) * j->frame_size,
                                   j->frame_size, ws))
            j->fail = 1;
        const uint8_t* p = co_byte_array_get_ptr(ws, 0);
        const uint32_t total = (uint32_t)co_byte_array_get_count(ws);
        co_byte_array_t* out = co_byte_array_create();
        if (total > j->max_frame) {
            uint32_t index = 0;
            do {
                const uint32_t sz = total - index > j->max_frame ? j->max_frame : total - index;
                h2_data_frame(p + index, sz, index + sz == total, out);
                index += sz;
            } while (index < total);
        } else {
            h2_data_frame(p, total, true, out);
        }
        co_byte_array_destroy(ws);
        j->wire[i] = out;
    }
    return NULL;
}

static void* h2_recv_run(void* arg)
{
    h2_job_t* j = (h2_job_t*)arg;
    uint64_t s = 0;
    for (uint64_t i = 0; i < j->count; ++i) {
        const co_byte_array_t* in = j->wire[i];
        const size_t n = co_byte_array_get_count(in);
        size_t idx = 0;
        co_byte_array_t* pool = NULL;
        while (idx < n) {
            co_http2_frame_t* f = co_http2_frame_create();
            if (co_http2_frame_deserialize(in, &idx, j->max_frame, f) != 0) {
                j->fail = 1;
                free(f);
                break;
            }
            if (f->header.flags & CO_HTTP2_FRAME_FLAG_END_STREAM) {
                uint8_t* ptr;
                size_t size;
                if (pool == NULL || co_byte_array_get_count(pool) == 0) {
                    ptr = f->payload.data.data;
                    size = f->payload.data.data_length;
                    f->payload.data.data = NULL;
                    f->payload.data.data_length = 0;
                } else {
                    if (f->payload.data.data_length > 0)
                        co_byte_array_add(pool, f->payload.data.data, f->payload.data.data_length);
                    co_byte_array_add(pool, "\0", 1);
                    size = co_byte_array_get_count(pool) - 1;
                    ptr = co_byte_array_detach(pool);
                }
                co_ws_frame_t* w = co_ws_frame_create();
                size_t unused = 0;
                if (co_ws_frame_deserialize(w, ptr, size, &unused) != 0) j->fail = 1;
                else s += w->payload_data[0];
                co_ws_frame_destroy(w);
                free(ptr);
            } else {
                if (pool == NULL) pool = co_byte_array_create();
                if (f->payload.data.data_length > 0)
                    co_byte_array_add(pool, f->payload.data.data, f->payload.data.data_length);
            }
            co_http2_frame_destroy(f);
        }
        if (pool) co_byte_array_destroy(pool);
    }
    j->sink = s;
    return NULL;
}

int ref_h2_cpu_bench(uint64_t n_frames, uint64_t frame_size, uint32_t max_frame, int threads, int iters,
                     double* send_seconds, double* recv_seconds)
{
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    uint8_t* payload = (uint8_t*)malloc(n_frames * frame_size);
    co_byte_array_t** wire = (co_byte_array_t**)calloc(n_frames, sizeof(*wire));
    h2_job_t* jobs = (h2_job_t*)calloc((size_t)threads, sizeof(*jobs));
    if (!payload || !wire || !jobs) return -1;
    for (uint64_t i = 0; i < n_frames * frame_size; ++i)
        payload[i] = (uint8_t)(i * 2654435761u >> 13);
    uint64_t per = n_frames / (uint64_t)threads, rem = n_frames % (uint64_t)threads, at = 0;
    for (int t = 0; t < threads; ++t) {
        uint64_t c = per + ((uint64_t)t < rem ? 1 : 0);
        jobs[t].payload = payload;
        jobs[t].first = at;
        jobs[t].count = c;
        jobs[t].frame_size = frame_size;
        jobs[t].max_frame = max_frame;
        jobs[t].wire = wire + at;
        at += c;
    }
    double ss = 0, rs = 0;
    int fail = 0;
    for (int it = 0; it < iters; ++it) {
        ss += h2_phase(h2_send_run, jobs, threads);
        rs += h2_phase(h2_recv_run, jobs, threads);
        for (uint64_t i = 0; i < n_frames; ++i) {
            if (wire[i]) co_byte_array_destroy(wire[i]);
            wire[i] = NULL;
        }
    }
    for (int t = 0; t < threads; ++t) fail |= jobs[t].fail;
    free(jobs);
    free(wire);
    free(payload);
    *send_seconds = ss;
    *recv_seconds = rs;
    return fail ? -2 : 0;
}
#endif

#ifndef CFWS_BENCH_REF
/* ---- receive-buffer indexing, port only --------------
 * The receive loop's walk over each connection's bytes [begin[c], end[c])
 * (orc_index_stream: co_ws_server.c:107-169's header decisions), connections
 * split over `threads` pthreads. Returns the frames found. */
typedef struct {
    const uint8_t* buf;
    const uint64_t* begin;
    const uint64_t* end;
    uint64_t first, count;
    uint64_t* scratch;
    uint64_t scratch_n;
    uint64_t frames;
} index_job_t;

static void* index_run(void* arg)
{
    index_job_t* j = (index_job_t*)arg;
    uint64_t f = 0;
    for (uint64_t c = j->first; c < j->first + j->count; ++c) {
        uint64_t consumed = 0;
        int32_t stop = 0;
        f += orc_index_stream(j->buf, j->begin[c], j->end[c], (uint64_t)32 << 20, j->scratch,
                              j->scratch_n, &consumed, &stop);
    }
    j->frames = f;
    return NULL;
}

int orc_index_bench(const uint8_t* buf, const uint64_t* begin, const uint64_t* end, uint64_t n_conn,
                    uint64_t max_frames_per_conn, int threads, double* seconds, uint64_t* frames)
{
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    index_job_t* jobs = (index_job_t*)calloc((size_t)threads, sizeof(*jobs));
    if (!jobs) return -1;
    uint64_t per = n_conn / (uint64_t)threads, rem = n_conn % (uint64_t)threads, at = 0;
    for (int t = 0; t < threads; ++t) {
        uint64_t c = per + ((uint64_t)t < rem ? 1 : 0);
        jobs[t].buf = buf;
        jobs[t].begin = begin;
        jobs[t].end = end;
        jobs[t].first = at;
        jobs[t].count = c;
        jobs[t].scratch_n = max_frames_per_conn;
        jobs[t].scratch = (uint64_t*)malloc(sizeof(uint64_t) * (max_frames_per_conn ? max_frames_per_conn : 1));
        at += c;
    }
    pthread_t tid[256];
    double t0 = bench_now();
    for (int t = 0; t < threads; ++t) pthread_create(&tid[t], NULL, index_run, &jobs[t]);
    for (int t = 0; t < threads; ++t) pthread_join(tid[t], NULL);
    *seconds = bench_now() - t0;
    uint64_t f = 0;
    for (int t = 0; t < threads; ++t) {
        f += jobs[t].frames;
        free(jobs[t].scratch);
    }
    *frames = f;
    free(jobs);
    return 0;
}
#endif
