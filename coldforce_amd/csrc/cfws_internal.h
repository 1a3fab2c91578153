// cfws_internal.h -- library-internal interfaces shared between the
// translation units of libcfws.so (not part of the C ABI).
#ifndef CFWS_INTERNAL_H
#define CFWS_INTERNAL_H

#include <stdint.h>

// Byte offset, inside a plan's workspace, of the u64 holding the UNCLAMPED
// layout total of pass 0 (the prefix sum before the capacity clamp).
uint64_t cfws_internal_grand_total_offset();

#endif
