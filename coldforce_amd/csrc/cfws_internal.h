// cfws_internal.h -- library-internal interfaces shared between the
// translation units of libcfws.so (not part of the C ABI).
#ifndef CFWS_INTERNAL_H
#define CFWS_INTERNAL_H

#include <stdint.h>

// Byte offset, inside a plan's workspace, of the u64 holding the UNCLAMPED
// layout total of pass 0 (the prefix sum before the capacity clamp).
uint64_t cfws_internal_grand_total_offset();

// Byte offset, in a cfws_h2_deserialize_batch workspace for these sizes, of
// the unclamped payload layout total of the messages.
uint64_t cfws_internal_h2_grand_total_offset(uint64_t n_h2, uint64_t pool_cap, uint64_t payload_cap);

// D2H by copy_out_kernel into device-mapped host memory at its DEVICE
// address dev_dst (cfws_mapped_device_pointer); no mapping check.
int cfws_internal_copy_out(const void* d_src, void* dev_dst, uint64_t n, void* stream);

// cfws_time_next_pass: an event pair (hipEvent_t) for the calling thread's
// NEXT public batch call. Every public call that launches work opens a
// CfwsPassScope on entry: the outermost scope moves the pending pair into
// the call (the pending slot is empty from then on) and drops whatever is
// left of it on exit, so a pair never outlives the call that took it (an
// error return, an empty batch, a path with no timed pass included). Inside
// the call, the launch site of its timed pass takes the pair once
// (cfws_internal_take_pass) and records start before / stop after its
// kernel; nested public calls (a batch call's plan and execute) share the
// outer call's pair.
struct CfwsPassEvents {
    void* start;
    void* stop;
};
CfwsPassEvents& cfws_internal_pass_events();     // the pending pair
CfwsPassEvents cfws_internal_take_pass();        // the current call's pair, once; then empty
struct CfwsPassScope {
    CfwsPassScope();
    ~CfwsPassScope();
    CfwsPassScope(const CfwsPassScope&) = delete;
    CfwsPassScope& operator=(const CfwsPassScope&) = delete;
};
// The timed pass's launch site: takes the call's pair (if it still holds
// one) and records start on `stream` now, stop when the timer goes out of
// scope (after the pass's kernels were queued).
struct CfwsPassTimer {
    explicit CfwsPassTimer(void* stream);
    ~CfwsPassTimer();
    CfwsPassTimer(const CfwsPassTimer&) = delete;
    CfwsPassTimer& operator=(const CfwsPassTimer&) = delete;
    CfwsPassEvents e;
    void* stream;
};

// The drop-in's frame service (cfws_ops.hip, used by cfws_frame.cpp): one
// resident workgroup per device that serves every calling thread of the
// process. Each thread owns a slot: a request word and a done word in the
// control page, and a kCfwsServiceMax-byte buffer; all in mapped host
// memory. The thread copies its frame into its buffer and posts the request
// word; the kernel XORs the buffer in place and writes the done word. No
// launch and no completion signal per frame. Control page words (u64):
//   [kCfwsServiceStopWord]   non-zero ends the kernel
//   [kCfwsServiceExitWord]   the generation of the last launch that ended
//   [kCfwsServiceReqWord + s]  slot s request: key (bits 0-31) | n - 1
//                            (bits 32-47) | seq (bits 48-63)
//   [kCfwsServiceDoneWord + s] slot s done: seq of its last finished
//                            request (bits 48-63)
// The kernel ends by itself after idle_ticks of the wall clock without a
// request or after life_ticks in all (every wave reaches that exit) and
// then writes `gen` to the exit word; requests it did not take stay posted
// for the next launch.
constexpr uint32_t kCfwsServiceMax = 65536;       // largest frame the service takes
constexpr uint32_t kCfwsServiceSlots = 64;        // calling threads per device
constexpr uint32_t kCfwsServiceStopWord = 0;
constexpr uint32_t kCfwsServiceExitWord = 1;
constexpr uint32_t kCfwsServiceReqWord = 16;      // 64 words: bytes 128-639
constexpr uint32_t kCfwsServiceDoneWord = 96;     // 64 words: bytes 768-1279
constexpr uint32_t kCfwsServiceCtlBytes = 4096;
extern "C" int cfws_internal_service_launch(uint64_t* dev_ctl, uint8_t* dev_bufs, uint64_t gen,
                                            uint64_t idle_ticks, uint64_t life_ticks, void* stream);

#endif
