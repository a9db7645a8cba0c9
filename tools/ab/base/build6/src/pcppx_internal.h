// pcppx_internal.h — kernel launchers shared by the C-ABI layer (not part of the public ABI).
#pragma once

#include <hip/hip_runtime.h>

#include "pcppx.h"

namespace pcppx
{
int check_launch(const char* what, hipStream_t stream);
// wave_stats: null, or parse_waves(n) 16-B per-wave collectStats records, summed by launch_proto_stats_reduce
// win_stats: null, or the context's two 64-bit counters: a window sample (window_sample_kernel: ~64 tiles' live and
// deep-stack packets) runs ahead of the parse on the same stream and adds to them
int launch_parse(const pcppx_batch* b, const pcppx_opts* o, pcppx_records* r, hipStream_t stream,
                 void* wave_stats = nullptr, unsigned long long* win_stats = nullptr);
uint32_t parse_waves(uint32_t n);
int launch_proto_stats_reduce(const void* wave_stats, uint32_t n, uint64_t* out, hipStream_t stream);
int launch_filter(const pcppx_batch* b, const pcppx_records* r, uint32_t ml, const pcppx_match_spec* spec,
                  uint64_t seq_base, uint64_t* keys, uint64_t* first, uint32_t capacity, uint8_t* matched,
                  pcppx_packet_stats* stats, hipStream_t stream);
// the partitioned flow table (product): queues = P x rec_cap 16-B records, fill = P zeroed counters
uint32_t flow_partitions(uint32_t capacity);
uint32_t flow_queue_capacity(uint32_t n, uint32_t capacity);
int launch_flow_count_part(const pcppx_summary* sum, const uint32_t* dkeys, const uint32_t* caplens, uint32_t n,
                           uint32_t* keys, uint64_t* packets, uint64_t* bytes, uint32_t capacity, uint64_t* stats,
                           void* queues, uint32_t rec_cap, uint32_t* fill, hipStream_t stream);
int launch_parse_reasm(const pcppx_batch* b, const pcppx_opts* o, pcppx_records* r, pcppx_reasm_info* info,
                       hipStream_t stream, void* wave_stats = nullptr, unsigned long long* win_stats = nullptr);
int launch_reasm(const pcppx_batch* b, const pcppx_records* r, uint32_t ml, pcppx_reasm_info* info, hipStream_t stream);
// PCPPX_LAYOUT_DENSE on the host path: a chunk's FIXED rows (n x ml) -> its chains back to back (dense), the chain
// lengths read from n_layers[i * nl_stride] (a summary's or a brief's byte 14); *total = the entries written.
// block_sums: dense_blocks(n) words of scratch.
uint32_t dense_blocks(uint32_t n);
int launch_dense_compact(const pcppx_layer* fixed, const uint8_t* n_layers, uint32_t nl_stride, uint32_t n, uint32_t ml,
                         pcppx_layer* dense, uint32_t* block_sums, uint32_t* total, hipStream_t stream);
// the compacted chains to page-locked host memory through its device mapping (dst_mapped), positions chained across the
// chunks of a batch on the device: *cum_out = (*base_in or 0) + *count; at_base: entries at dst_mapped + base (else + 0)
int launch_dense_push(const pcppx_layer* dense, const uint32_t* count, const uint32_t* base_in, pcppx_layer* dst_mapped,
                      bool at_base, uint32_t* cum_out, hipStream_t stream);
}  // namespace pcppx
