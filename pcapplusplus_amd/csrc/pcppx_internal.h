// pcppx_internal.h — kernel launchers shared by the C-ABI layer (not part of the public ABI).
#pragma once

#include <hip/hip_runtime.h>

#include "pcppx.h"

namespace pcppx
{
int check_launch(const char* what, hipStream_t stream);
int launch_parse(const pcppx_batch* b, const pcppx_opts* o, pcppx_records* r, hipStream_t stream);
int launch_flow_count(const pcppx_summary* sum, const uint32_t* caplens, uint32_t n, uint32_t* keys,
                      uint64_t* packets, uint64_t* bytes, uint32_t capacity, uint64_t* stats, hipStream_t stream);
}  // namespace pcppx
