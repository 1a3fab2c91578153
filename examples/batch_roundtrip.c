/*
 * batch_roundtrip.c -- the batch C ABI (include/cfws.h) from plain C, the way
 * a coldforce send/receive loop would drive it: no Python, no torch.
 *
 *   client side:  payloads (pinned host) -> H2D -> cfws_serialize_batch
 *                 (mask keys drawn like co_ws_frame_serialize draws them)
 *   server side:  cfws_index_frames_batch over the wire as one connection's
 *                 receive buffer -> cfws_deserialize_batch -> D2H payloads,
 *                 and the same frames through cfws_deserialize_slots (frame
 *                 i's payload at i * slot) and cfws_deserialize_scatter
 *                 (each payload to a buffer of its own size, last frame first)
 *   uniform batch: n frames of 256 B through cfws_serialize_uniform (payload
 *                 + one key per frame, no descriptors) and back through
 *                 cfws_deserialize_slots_uniform (frame i at i * its wire
 *                 bytes, no index; 8-byte records and a mismatch count)
 *
 * Checks that every payload comes back and that the wire equals what
 * sequential co_ws_frame_serialize calls (the drop-in, same library) append
 * to one co_byte_array_t for the same random() stream.
 *
 * build: make examples   ->  build/examples/batch_roundtrip
 * run:   build/examples/batch_roundtrip [n_frames] [max_payload]
 */
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "cfws.h"
#include "cfws_co_ws_frame.h"

#define CHECK(x)                                                                    \
    do {                                                                            \
        int rc_ = (x);                                                              \
        if (rc_ != 0) {                                                             \
            fprintf(stderr, "%s:%d: %s -> %d (%s)\n", __FILE__, __LINE__, #x, rc_,  \
                    cfws_last_error());                                             \
            return 1;                                                               \
        }                                                                           \
    } while (0)

int main(int argc, char** argv)
{
    const size_t n = argc > 1 ? strtoull(argv[1], NULL, 10) : 4096;
    const size_t max_len = argc > 2 ? strtoull(argv[2], NULL, 10) : 70000;
    CHECK(cfws_init());

    /* frames: sizes across every header form, payloads back to back */
    cfws_frame_desc_t* desc = calloc(n, sizeof *desc);
    uint8_t* mask = malloc(n);
    uint64_t arena = 0;
    srandom(12345);
    for (size_t i = 0; i < n; ++i) {
        const size_t pick[] = {0, 1, 125, 126, 1000, 65535, 65536, max_len};
        desc[i].payload_size = pick[random() % 8] % (max_len + 1);
        desc[i].payload_off = arena;
        desc[i].fin = 1;
        desc[i].opcode = (i % 5 == 0) ? 1 : 2;
        desc[i].mask = mask[i] = (i % 3) != 0;
        arena += desc[i].payload_size;
    }
    uint8_t* payload;
    CHECK(hipHostMalloc((void**)&payload, arena + 16, 0));
    for (uint64_t k = 0; k < arena; ++k) payload[k] = (uint8_t)(k * 2654435761u >> 13);

    /* keys exactly as n co_ws_frame_serialize calls would draw them */
    uint32_t* keys = malloc(n * sizeof *keys);
    srandom(777);
    cfws_draw_mask_keys(n, mask, keys);
    for (size_t i = 0; i < n; ++i) desc[i].mask_key = keys[i];

    /* the drop-in's wire for the same stream, for comparison */
    co_byte_array_t ref = {0};
    ref.element_size = 1;
    ref.capacity = 8;
    ref.buffer = malloc(8);
    srandom(777);
    for (size_t i = 0; i < n; ++i)
        if (!co_ws_frame_serialize(true, desc[i].opcode, desc[i].mask != 0,
                                   payload + desc[i].payload_off, desc[i].payload_size, &ref)) {
            fprintf(stderr, "drop-in serialize failed\n");
            return 1;
        }

    /* device arenas */
    const uint64_t wire_cap = arena + 14 * n + 64, back_cap = arena + 16 * n + 64;
    void *d_payload, *d_wire, *d_back, *d_ws_s, *d_ws_d, *d_ws_i;
    cfws_frame_desc_t *d_desc, *d_desc2;
    int32_t *d_status, *d_stop;
    uint64_t *d_total, *d_starts, *d_first, *d_consumed, *d_begin, *d_end, *d_ntot;
    const size_t ws_s = cfws_workspace_size(n, wire_cap), ws_d = cfws_workspace_size(n, back_cap);
    const size_t ws_i = cfws_index_workspace_size(1);
    CHECK(hipMalloc(&d_payload, arena + 16));
    CHECK(hipMalloc(&d_wire, wire_cap));
    CHECK(hipMalloc(&d_back, back_cap));
    CHECK(hipMalloc((void**)&d_desc, n * sizeof *d_desc));
    CHECK(hipMalloc((void**)&d_desc2, n * sizeof *d_desc2));
    CHECK(hipMalloc((void**)&d_status, n * sizeof *d_status));
    CHECK(hipMalloc((void**)&d_total, 8));
    CHECK(hipMalloc((void**)&d_starts, (n + 1) * 8));
    CHECK(hipMalloc((void**)&d_first, 8));
    CHECK(hipMalloc((void**)&d_consumed, 8));
    CHECK(hipMalloc((void**)&d_stop, 4));
    CHECK(hipMalloc((void**)&d_begin, 8));
    CHECK(hipMalloc((void**)&d_end, 8));
    CHECK(hipMalloc((void**)&d_ntot, 8));
    CHECK(hipMalloc(&d_ws_s, ws_s));
    CHECK(hipMalloc(&d_ws_d, ws_d));
    CHECK(hipMalloc(&d_ws_i, ws_i));
    hipStream_t st;
    CHECK(hipStreamCreate(&st));

    /* client: serialize */
    CHECK(hipMemcpyAsync(d_payload, payload, arena, hipMemcpyHostToDevice, st));
    CHECK(hipMemcpyAsync(d_desc, desc, n * sizeof *desc, hipMemcpyHostToDevice, st));
    CHECK(cfws_serialize_batch(d_payload, d_desc, n, d_wire, wire_cap, d_total, d_ws_s, ws_s, st));
    uint64_t wire_total = 0;
    CHECK(hipMemcpyAsync(&wire_total, d_total, 8, hipMemcpyDeviceToHost, st));
    CHECK(hipStreamSynchronize(st));
    uint8_t* wire = malloc(wire_total + 1);
    CHECK(hipMemcpy(wire, d_wire, wire_total, hipMemcpyDeviceToHost));
    const int same = wire_total == ref.count && memcmp(wire, ref.buffer, wire_total) == 0;

    /* server: the wire as one connection's receive buffer */
    const uint64_t begin = 0;
    CHECK(hipMemcpyAsync(d_begin, &begin, 8, hipMemcpyHostToDevice, st));
    CHECK(hipMemcpyAsync(d_end, &wire_total, 8, hipMemcpyHostToDevice, st));
    CHECK(cfws_index_frames_batch(d_wire, d_begin, d_end, 1, CFWS_DEFAULT_MAX_RECEIVE_PAYLOAD_SIZE,
                                  d_starts, n + 1, d_first, d_consumed, d_stop, d_ntot, d_ws_i, ws_i,
                                  st));
    uint64_t n_found = 0, consumed = 0;
    int32_t stop = -1;
    CHECK(hipMemcpyAsync(&n_found, d_ntot, 8, hipMemcpyDeviceToHost, st));
    CHECK(hipMemcpyAsync(&consumed, d_consumed, 8, hipMemcpyDeviceToHost, st));
    CHECK(hipMemcpyAsync(&stop, d_stop, 4, hipMemcpyDeviceToHost, st));
    CHECK(hipStreamSynchronize(st));
    CHECK(cfws_deserialize_batch(d_wire, wire_total, d_starts, n_found,
                                 CFWS_DEFAULT_MAX_RECEIVE_PAYLOAD_SIZE, 1, 0, d_desc2, d_status,
                                 d_back, back_cap, d_total, d_ws_d, ws_d, st));
    uint64_t back_total = 0;
    CHECK(hipMemcpyAsync(&back_total, d_total, 8, hipMemcpyDeviceToHost, st));
    CHECK(hipStreamSynchronize(st));
    uint8_t* back = malloc(back_total + 1);
    int32_t* status = malloc(n * sizeof *status);
    CHECK(hipMemcpy(back, d_back, back_total, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(status, d_status, n * sizeof *status, hipMemcpyDeviceToHost));
    int ok = same && n_found == n && consumed == wire_total && stop == CFWS_PARSE_COMPLETE &&
             back_total == arena && memcmp(back, payload, arena) == 0;
    for (size_t i = 0; ok && i < n; ++i) ok = status[i] == CFWS_PARSE_COMPLETE;

    /* the same frames into fixed slots of the largest payload, 16-aligned */
    const uint64_t slot = max_len < 16 ? 16 : (max_len + 15) / 16 * 16;
    void* d_slots;
    CHECK(hipMalloc(&d_slots, n * slot));
    CHECK(cfws_deserialize_slots(d_wire, wire_total, d_starts, n_found, CFWS_DEFAULT_MAX_RECEIVE_PAYLOAD_SIZE,
                                 slot, d_desc2, d_status, d_slots, n * slot, d_total, st));
    uint64_t slots_total = 0;
    CHECK(hipMemcpyAsync(&slots_total, d_total, 8, hipMemcpyDeviceToHost, st));
    CHECK(hipStreamSynchronize(st));
    uint8_t* slots = malloc(n * slot);
    CHECK(hipMemcpy(slots, d_slots, n * slot, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(status, d_status, n * sizeof *status, hipMemcpyDeviceToHost));
    int slots_ok = n_found == n && slots_total == n * slot;
    for (size_t i = 0; slots_ok && i < n; ++i)
        slots_ok = status[i] == CFWS_PARSE_COMPLETE &&
                   memcmp(slots + i * slot, payload + desc[i].payload_off, desc[i].payload_size) == 0;

    /* each payload to its own 16-aligned buffer, sized to it, in reverse
       frame order: the reference's one allocation per frame */
    uint64_t* off = malloc(n * sizeof *off);
    uint64_t sc_cap = 0;
    for (size_t k = n; k-- > 0;) {
        off[k] = sc_cap;
        sc_cap += (desc[k].payload_size + 15) / 16 * 16;
    }
    void *d_sc, *d_off;
    CHECK(hipMalloc(&d_sc, sc_cap + 16));
    CHECK(hipMalloc(&d_off, n * sizeof *off));
    CHECK(hipMemcpyAsync(d_off, off, n * sizeof *off, hipMemcpyHostToDevice, st));
    CHECK(cfws_deserialize_scatter(d_wire, wire_total, d_starts, (const uint64_t*)d_off, n_found,
                                   CFWS_DEFAULT_MAX_RECEIVE_PAYLOAD_SIZE, slot, d_desc2, d_status, d_sc,
                                   sc_cap + 16, st));
    CHECK(hipStreamSynchronize(st));
    uint8_t* sc = malloc(sc_cap + 16);
    CHECK(hipMemcpy(sc, d_sc, sc_cap + 16, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(status, d_status, n * sizeof *status, hipMemcpyDeviceToHost));
    int scatter_ok = n_found == n;
    for (size_t i = 0; scatter_ok && i < n; ++i)
        scatter_ok = status[i] == CFWS_PARSE_COMPLETE &&
                     memcmp(sc + off[i], payload + desc[i].payload_off, desc[i].payload_size) == 0;

    /* a uniform batch: n BINARY frames of 256 B, masked; the wire must equal
       the drop-in's appends for the same random() stream */
    const uint64_t U = 256, UW = U + 8;                        /* 2 + 2 (BE16 length) + 4 key */
    uint8_t* upay = malloc(n * U);
    for (uint64_t k = 0; k < n * U; ++k) upay[k] = (uint8_t)(k * 40503u >> 7);
    uint32_t* ukeys = malloc(n * sizeof *ukeys);
    srandom(4242);
    cfws_draw_mask_keys(n, NULL, ukeys);
    co_byte_array_t uref = {0};
    uref.element_size = 1;
    uref.capacity = 8;
    uref.buffer = malloc(8);
    srandom(4242);
    for (size_t i = 0; i < n; ++i)
        if (!co_ws_frame_serialize(true, CO_WS_OPCODE_BINARY, true, upay + i * U, U, &uref)) return 1;
    void *d_upay, *d_ukeys, *d_uwire, *d_uback, *d_uinfo, *d_umis;
    CHECK(hipMalloc(&d_upay, n * U));
    CHECK(hipMalloc(&d_ukeys, n * sizeof *ukeys));
    CHECK(hipMalloc(&d_uwire, n * UW + 16));
    CHECK(hipMalloc(&d_uback, n * U));
    CHECK(hipMalloc(&d_uinfo, n * sizeof(cfws_frame_info_t)));
    CHECK(hipMalloc(&d_umis, sizeof(uint32_t)));
    CHECK(hipMemcpyAsync(d_upay, upay, n * U, hipMemcpyHostToDevice, st));
    CHECK(hipMemcpyAsync(d_ukeys, ukeys, n * sizeof *ukeys, hipMemcpyHostToDevice, st));
    CHECK(cfws_serialize_uniform(d_upay, (const uint32_t*)d_ukeys, n, U, 1, CO_WS_OPCODE_BINARY, 1, d_uwire,
                                 n * UW + 16, d_total, st));
    CHECK(cfws_deserialize_slots_uniform(d_uwire, n * UW, n, UW, CFWS_DEFAULT_MAX_RECEIVE_PAYLOAD_SIZE, U,
                                         (cfws_frame_info_t*)d_uinfo, d_uback, n * U, NULL, (uint32_t*)d_umis,
                                         st));
    uint64_t utotal = 0;
    uint32_t umis = 1;
    CHECK(hipMemcpyAsync(&utotal, d_total, 8, hipMemcpyDeviceToHost, st));
    CHECK(hipMemcpyAsync(&umis, d_umis, 4, hipMemcpyDeviceToHost, st));
    CHECK(hipStreamSynchronize(st));
    uint8_t* uwire = malloc(n * UW);
    uint8_t* uback = malloc(n * U);
    cfws_frame_info_t* uinfo = malloc(n * sizeof *uinfo);
    CHECK(hipMemcpy(uwire, d_uwire, n * UW, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(uback, d_uback, n * U, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(uinfo, d_uinfo, n * sizeof *uinfo, hipMemcpyDeviceToHost));
    int uniform_ok = utotal == n * UW && umis == 0 && uref.count == n * UW &&
                     memcmp(uwire, uref.buffer, n * UW) == 0 && memcmp(uback, upay, n * U) == 0;
    for (size_t i = 0; uniform_ok && i < n; ++i)
        uniform_ok = uinfo[i].status == CFWS_PARSE_COMPLETE && uinfo[i].payload_size == U && uinfo[i].fin == 1 &&
                     uinfo[i].opcode == CO_WS_OPCODE_BINARY;

    printf("{\"frames\": %zu, \"payload_bytes\": %llu, \"wire_bytes\": %llu, "
           "\"wire_equals_dropin\": %s, \"indexed\": %llu, \"roundtrip\": %s, \"slots\": %s, "
           "\"scatter\": %s, \"uniform\": %s}\n",
           n, (unsigned long long)arena, (unsigned long long)wire_total, same ? "true" : "false",
           (unsigned long long)n_found, ok ? "true" : "false", slots_ok ? "true" : "false",
           scatter_ok ? "true" : "false", uniform_ok ? "true" : "false");
    return ok && slots_ok && scatter_ok && uniform_ok ? 0 : 2;
}
