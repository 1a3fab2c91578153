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

#endif
