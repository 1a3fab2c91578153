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

// The drop-in's frame service (cfws_ops.hip, used by cfws_frame.cpp): one
// resident workgroup that polls a mailbox in mapped host memory and XORs
// each posted frame in place in a mapped host buffer, so a masked frame
// costs no kernel launch and no completion signal. Mailbox words (u64):
//   [0] request: key (bits 0-31) | n - 1 (bits 32-47) | seq (bits 48-63)
//   [1] done:    seq of the last finished request (bits 48-63)
//   [2] stop:    non-zero ends the kernel
// The kernel also ends after idle_ticks of the wall clock without a request
// (every wave reaches that exit). last_seq: the seq done before this launch.
constexpr uint32_t kCfwsServiceMax = 65536;       // largest frame the service takes
extern "C" int cfws_internal_service_launch(uint64_t* dev_mbox, uint8_t* dev_buf, uint64_t idle_ticks,
                                            uint32_t last_seq, void* stream);

#endif
