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
