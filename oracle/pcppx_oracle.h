/*
 * pcppx_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C CPU restatement of the reference Packet++ per-packet parse path, used as the parity checker
 * for the HIP engine and as the "port" CPU baseline. Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it. Its output format is the engine's (include/pcppx.h), with
 * the engine's contract for flagged packets (see pcppx_oracle.c header comment).
 *
 * Pinning: tests/test_oracle_vs_reference.py checks it against the real reference Packet++ built from
 * /root/reference by oracle/Makefile (oracle/_ref/libpcpp_ref.so) and against committed golden
 * records made by that reference (tests/golden/, generator tools/make_golden.py).
 */
#ifndef PCPPX_ORACLE_H
#define PCPPX_ORACLE_H

#include "pcppx.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Parse one packet. layers may be NULL (then opts->max_layers is only the depth cap). */
void pcppx_oracle_parse_packet(const uint8_t* pkt, uint32_t caplen, uint16_t linktype, const pcppx_opts* opts,
                               pcppx_summary* sum, pcppx_layer* layers);

/* Parse a host batch; threads > 1 interleaves packet indices over pthreads. */
int pcppx_oracle_parse_batch(const pcppx_batch* batch, const pcppx_opts* opts, pcppx_records* out, int threads);

/* Timed CPU baseline (parse + hashes + checksums per opts), returns seconds of the timed region. */
int pcppx_oracle_bench(const pcppx_batch* batch, const pcppx_opts* opts, int threads, double* seconds,
                       uint64_t* digest);

/* Reassembly front ends (include/pcppx.h pcppx_reasm_device) over a host batch and its engine-format
 * records (max_layers >= 1 per packet); info has n entries. */
int pcppx_oracle_reasm_batch(const pcppx_batch* batch, const pcppx_records* records, uint8_t max_layers,
                             pcppx_reasm_info* info);

/* Primitive restatements, exposed for the known-answer tests. */
uint16_t pcppx_oracle_checksum(const uint8_t* const* bufs, const uint32_t* lens, int nbufs); /* PacketUtils.cpp:12-64 */
uint32_t pcppx_oracle_fnv1(const uint8_t* buf, uint32_t len);                               /* PacketUtils.cpp:114-137 */

#ifdef __cplusplus
}
#endif

#endif
