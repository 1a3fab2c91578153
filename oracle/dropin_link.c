/*
 * dropin_link.c -- TEST INFRASTRUCTURE ONLY: link-level drop-in check.
 *
 * A C program written against coldforce's OWN headers
 * (/root/reference/inc/coldforce/ws/co_ws_frame.h, co_ws_config.h,
 * core/co_byte_array.h) and linked against libcfws.so instead of
 * src/ws/co_ws_frame.c + co_ws_config.c. The byte array comes from the
 * reference's src/core/co_array.c, compiled in place, exactly as libco_core
 * supplies it to libco_ws. Built by oracle/Makefile (`make ref`) into
 * oracle/_ref/ only; tests/test_gpu_dropin.py runs it on the GPU box and
 * checks its output against the oracle.
 *
 * What it does, like co_ws_send + the receive loop would:
 *   srandom(seed); for each (size, mask): co_ws_frame_serialize(fin=1,
 *   opcode=2, mask, data, size, buf) appending to ONE byte array; prints the
 *   wire length and its FNV-1a 64; then walks the wire with
 *   co_ws_frame_deserialize, checking every payload (and its NUL
 *   terminator); then the error codes of a truncated frame, an RSV-bit
 *   frame and an over-limit frame.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <coldforce/core/co_byte_array.h>
#include <coldforce/ws/co_ws_config.h>
#include <coldforce/ws/co_ws_frame.h>

static uint64_t fnv1a(const uint8_t* p, size_t n)
{
    uint64_t h = 0xcbf29ce484222325ull;
    for (size_t i = 0; i < n; ++i) h = (h ^ p[i]) * 0x100000001b3ull;
    return h;
}

static void fill(uint8_t* d, size_t n)
{
    for (size_t i = 0; i < n; ++i) d[i] = (uint8_t)(i * 131u + n);
}

#include <time.h>

static double clk(clockid_t c)
{
    struct timespec t;
    clock_gettime(c, &t);
    return t.tv_sec + 1e-9 * t.tv_nsec;
}

static double now(void) { return clk(CLOCK_MONOTONIC); }

/* `dropin_link bench SIZE N`: per-frame latency of the drop-in, as a
 * receive/send loop sees it -- N x (co_ws_frame_serialize(mask) into a
 * cleared byte array + co_ws_frame_deserialize + co_ws_frame_destroy). */
static int bench(size_t size, long n)
{
    uint8_t* data = malloc(size + 1);
    fill(data, size);
    co_byte_array_t* b = co_byte_array_create();
    srandom(1);
    for (int warm = 0; warm < 2; ++warm) {
        co_byte_array_clear(b);
        if (!co_ws_frame_serialize(true, CO_WS_OPCODE_BINARY, true, data, size, b)) return 2;
    }
    double ts = 0, td = 0, cs = 0, cd = 0;
    const double p0 = clk(CLOCK_PROCESS_CPUTIME_ID), w0 = now();
    for (long i = 0; i < n; ++i) {
        co_byte_array_clear(b);
        const double c0 = clk(CLOCK_THREAD_CPUTIME_ID), t0 = now();
        if (!co_ws_frame_serialize(true, CO_WS_OPCODE_BINARY, true, data, size, b)) return 2;
        const double c1 = clk(CLOCK_THREAD_CPUTIME_ID), t1 = now();
        co_ws_frame_t* f = co_ws_frame_create();
        size_t index = 0;
        const int r = co_ws_frame_deserialize(f, co_byte_array_get_ptr(b, 0), co_byte_array_get_count(b),
                                              &index);
        const double c2 = clk(CLOCK_THREAD_CPUTIME_ID), t2 = now();
        cs += c1 - c0;
        cd += c2 - c1;
        if (r != CO_WS_PARSE_COMPLETE || memcmp(co_ws_frame_get_payload_data(f), data, size) != 0) return 3;
        co_ws_frame_destroy(f);
        ts += t1 - t0;
        td += t2 - t1;
    }
    /* wall time, the calling thread's CPU time, and the whole process's CPU
     * time per frame (the HIP runtime's own threads included) */
    const double pc = clk(CLOCK_PROCESS_CPUTIME_ID) - p0, wall = now() - w0;
    printf("{\"frame_bytes\": %zu, \"frames\": %ld, \"serialize_us\": %.2f, \"deserialize_us\": %.2f, "
           "\"serialize_cpu_us\": %.2f, \"deserialize_cpu_us\": %.2f, \"process_cpu_us_per_pair\": %.2f, "
           "\"wall_us_per_pair\": %.2f}\n",
           size, n, 1e6 * ts / n, 1e6 * td / n, 1e6 * cs / n, 1e6 * cd / n, 1e6 * pc / n, 1e6 * wall / n);
    co_byte_array_destroy(b);
    free(data);
    return 0;
}

int main(int argc, char** argv)
{
    if (argc > 3 && strcmp(argv[1], "bench") == 0)
        return bench((size_t)strtoull(argv[2], NULL, 10), strtol(argv[3], NULL, 10));
    const unsigned seed = argc > 1 ? (unsigned)strtoul(argv[1], NULL, 10) : 1u;
    static const size_t sizes[] = {0, 1, 125, 126, 1000, 65535, 65536, 70000};
    const size_t ns = sizeof sizes / sizeof sizes[0];
    uint8_t* data = malloc(70000 + 1);
    srandom(seed);
    co_byte_array_t* wire = co_byte_array_create();
    for (size_t s = 0; s < ns; ++s)
        for (int mask = 0; mask < 2; ++mask) {
            fill(data, sizes[s]);
            if (!co_ws_frame_serialize(true, CO_WS_OPCODE_BINARY, mask != 0, data, sizes[s], wire)) {
                printf("serialize failed size=%zu mask=%d\n", sizes[s], mask);
                return 2;
            }
        }
    const uint8_t* w = co_byte_array_get_ptr(wire, 0);
    const size_t count = co_byte_array_get_count(wire);
    printf("wire %zu %016llx\n", count, (unsigned long long)fnv1a(w, count));

    size_t index = 0, k = 0;
    while (index < count) {
        co_ws_frame_t* f = co_ws_frame_create();
        const int r = co_ws_frame_deserialize(f, w, count, &index);
        const size_t n = sizes[k / 2];
        fill(data, n);
        if (r != CO_WS_PARSE_COMPLETE || !co_ws_frame_get_fin(f) ||
            co_ws_frame_get_opcode(f) != CO_WS_OPCODE_BINARY || co_ws_frame_get_payload_size(f) != n ||
            (n == 0 && co_ws_frame_get_payload_data(f) != NULL) ||
            (n > 0 && (memcmp(co_ws_frame_get_payload_data(f), data, n) != 0 ||
                       co_ws_frame_get_payload_data(f)[n] != 0))) {
            printf("frame %zu mismatch (rc=%d)\n", k, r);
            return 3;
        }
        co_ws_frame_destroy(f);
        ++k;
    }
    printf("frames %zu ok\n", k);

    /* error paths, with the reference's codes */
    size_t at = 0;
    for (size_t j = 0; j < 8; ++j) {                                 /* skip to the 1000-B frame */
        co_ws_frame_t* g = co_ws_frame_create();
        co_ws_frame_deserialize(g, w, count, &at);
        co_ws_frame_destroy(g);
    }
    co_ws_frame_t* f = co_ws_frame_create();
    size_t i0 = 0;
    const int more = co_ws_frame_deserialize(f, w + at, 5, &i0);     /* payload truncated */
    const uint8_t rsv[2] = {0xc2, 0x00};
    i0 = 0;
    const int invalid = co_ws_frame_deserialize(f, rsv, 2, &i0);
    co_ws_config_set_max_receive_payload_size(100);
    i0 = at;
    const int too_big = co_ws_frame_deserialize(f, w, count, &i0);
    co_ws_config_set_max_receive_payload_size(CO_WS_CONFIG_DEFAULT_MAX_RECEIVE_PAYLOAD_SIZE);
    co_ws_frame_destroy(f);
    printf("codes %d %d %d index %zu\n", more, invalid, too_big, i0);
    co_byte_array_destroy(wire);
    free(data);
    return 0;
}
