// rse_dispatch.hpp -- the resident dispatcher of the synchronous small calls
// (rse_dispatch.hip), for the host codec (rse_codec.cpp).  Kept out of
// rse_kernels.hpp, whose text is part of every run-time module's source.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace rse {

// Whether one synchronous pass of rows (n_out x n_in GF(2^8) coefficients)
// over shards of len_bytes can run on the resident dispatcher (RSE_OPT_DISPATCH,
// RSE_OPT_DISPATCH_MAX_BYTES, 16-byte aligned shards and lengths).
bool dispatch_applies(int field, uint32_t n_in, uint32_t n_out, uint64_t len_bytes,
                      const uint8_t* const* in, uint8_t* const* out);
// out (check: compared with out, *mismatch) = rows x in on the current device's
// resident workgroup; returns when done.  dispatch_applies must hold.
hipError_t dispatch_run(const uint16_t* rows, uint32_t n_in, uint32_t n_out,
                        const uint8_t* const* in, uint8_t* const* out, uint64_t len_bytes,
                        bool check, bool* mismatch);
void dispatch_stop_all();
// A non-blocking stream at the highest (high) or lowest stream priority of the
// current device, or a plain one where the device has a single priority.  HIP
// maps streams onto at most GPU_MAX_HW_QUEUES hardware queues per priority,
// least-used first, and a queue starts its commands in order; torch's and
// most callers' streams are at the default priority, so a stream at another
// one does not share their queues.  The resident dispatcher runs on a
// low-priority stream (its kernel would hold up, until it idles out, every
// command queued behind it on a shared queue), the host pipeline's D2H copies
// on a high-priority one (rse_codec.cpp pipe_stream).
hipError_t side_priority_stream(bool high, hipStream_t* q);
int64_t dispatch_count();         // RSE_OPT_DISPATCHED
int64_t dispatch_launch_count();  // RSE_OPT_DISPATCH_LAUNCHES

}  // namespace rse
