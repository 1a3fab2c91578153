// cfws_graph.cpp -- HIP graphs of the batch codec (include/cfws.h, cfws_graph_*).
//
// A server loop that serializes or deserializes batches of the same shape
// over the same arenas (a send queue drained every tick, a receive buffer
// indexed every event) pays per batch the launch latency of the plan and
// execute kernels (two to four launches), which is the whole cost for small
// batches. Captured once into a hipGraph, a batch is one graph launch. The
// graph fixes the pointers, the frame count and the capacities; the
// descriptor contents, payload and wire bytes may change between launches,
// because the plans run on the device every time (keys, sizes and offsets
// are read at launch, not at capture).
//
// Capture runs on a private stream in thread-local capture mode, so other
// threads' HIP calls are not affected. Every cfws_serialize_batch /
// cfws_deserialize_batch step is asynchronous (no host synchronisation), so
// it captures as is; cfws_h2_deserialize_batch synchronises to return its
// message count and cannot be captured.
#include <hip/hip_runtime.h>

#include <stdio.h>

#include "cfws.h"
#include "cfws_internal.h"

struct cfws_graph {
    hipGraph_t graph = nullptr;
    hipGraphExec_t exec = nullptr;
};

namespace {

int graph_fail(const char* what, hipError_t e)
{
    fprintf(stderr, "cfws graph: %s: %s\n", what, hipGetErrorString(e));
    return CFWS_ERROR_HIP;
}

// Captures body(stream) into *out. body's own error code wins over the
// capture's.
template <typename Body>
int capture(Body body, cfws_graph_t** out)
{
    if (int rc = cfws_init()) return rc;
    if (!out) return CFWS_ERROR_INVALID_ARGUMENT;
    *out = nullptr;
    hipStream_t s = nullptr;
    hipError_t e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    if (e != hipSuccess) return graph_fail("stream", e);
    e = hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
    if (e != hipSuccess) {
        (void)hipStreamDestroy(s);
        return graph_fail("begin capture", e);
    }
    const int rc = body(s);
    hipGraph_t g = nullptr;
    e = hipStreamEndCapture(s, &g);
    (void)hipStreamDestroy(s);
    if (rc != CFWS_OK || e != hipSuccess) {
        if (g) (void)hipGraphDestroy(g);
        return rc != CFWS_OK ? rc : graph_fail("end capture", e);
    }
    auto* G = new cfws_graph;
    G->graph = g;
    e = hipGraphInstantiate(&G->exec, g, nullptr, nullptr, 0);
    if (e != hipSuccess) {
        cfws_graph_destroy(G);
        return graph_fail("instantiate", e);
    }
    *out = G;
    return CFWS_OK;
}

}  // namespace

extern "C" {

int cfws_graph_serialize(const void* d_payload, cfws_frame_desc_t* d_desc, size_t n, void* d_wire,
                         uint64_t wire_capacity, uint64_t* d_wire_total, void* d_workspace,
                         size_t workspace_size, cfws_graph_t** out)
{
    const CfwsPassScope pass_scope;
    (void)cfws_internal_take_pass();   // not timed (cfws_time_next_pass): the pair is dropped
    return capture([&](hipStream_t s) {
        return cfws_serialize_batch(d_payload, d_desc, n, d_wire, wire_capacity, d_wire_total,
                                    d_workspace, workspace_size, s);
    }, out);
}

int cfws_graph_deserialize(const void* d_wire, uint64_t wire_size, const uint64_t* d_index, size_t n,
                           uint64_t max_payload, uint32_t align, uint32_t flags,
                           cfws_frame_desc_t* d_desc, int32_t* d_status, void* d_payload,
                           uint64_t payload_capacity, uint64_t* d_payload_total, void* d_workspace,
                           size_t workspace_size, cfws_graph_t** out)
{
    const CfwsPassScope pass_scope;
    (void)cfws_internal_take_pass();   // not timed (cfws_time_next_pass): the pair is dropped
    return capture([&](hipStream_t s) {
        return cfws_deserialize_batch(d_wire, wire_size, d_index, n, max_payload, align, flags, d_desc,
                                      d_status, d_payload, payload_capacity, d_payload_total,
                                      d_workspace, workspace_size, s);
    }, out);
}

int cfws_graph_launch(cfws_graph_t* g, void* stream)
{
    const CfwsPassScope pass_scope;
    (void)cfws_internal_take_pass();   // not timed (cfws_time_next_pass): the pair is dropped
    if (!g || !g->exec) return CFWS_ERROR_INVALID_ARGUMENT;
    const hipError_t e = hipGraphLaunch(g->exec, static_cast<hipStream_t>(stream));
    return e == hipSuccess ? CFWS_OK : graph_fail("launch", e);
}

void cfws_graph_destroy(cfws_graph_t* g)
{
    if (!g) return;
    if (g->exec) (void)hipGraphExecDestroy(g->exec);
    if (g->graph) (void)hipGraphDestroy(g->graph);
    delete g;
}

}  // extern "C"
