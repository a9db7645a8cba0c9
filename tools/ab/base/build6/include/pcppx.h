/*
 * pcppx.h — C ABI of the MI355X packet-dissection engine (drop-in boundary).
 *
 * This is the boundary that replaces the per-packet Packet++ parse path
 *   RawPacket -> pcpp::Packet(RawPacket*, ...)          Packet++/src/Packet.cpp:202-209, :66-196
 *   pcpp::hash5Tuple / pcpp::hash2Tuple                  Packet++/src/PacketUtils.cpp:139-245
 *   IPv4 header checksum                                 Packet++/src/IPv4Layer.cpp:410-412
 *   TcpLayer/UdpLayer::calculateChecksum(false)          Packet++/src/TcpLayer.cpp:271, UdpLayer.cpp:47
 * with one batched call over many packets that sit in GPU memory (HBM).
 *
 * Conventions:
 *   - every function returns 0 or a negative PCPPX_E* code; nothing throws across the ABI;
 *   - the caller owns every buffer; records are arrays sized n (and n*max_layers);
 *   - a context belongs to one host thread and one GPU; contexts are never shared.
 *
 * Records mirror what a pcpp::Packet exposes after parsing:
 *   pcppx_layer   <-> Layer::getProtocol/getOsiModelLayer/getData()-raw/getHeaderLen/getDataLen
 *                      (Packet++/header/Layer.h, ProtocolType.h:35-284)
 *   pcppx_summary <-> Packet::isPacketOfType (proto_mask, Packet.cpp:614-640), hash5Tuple(false/true),
 *                      hash2Tuple, the IPv4/L4 checksums.
 * Layers the engine builds: Ethernet II / 802.3 / LLC, VLAN, MPLS, IPv4, IPv6 (+ extensions), GREv0/v1,
 * PPP_PPTP, ARP, ICMP (+ the IPv4 header an error message quotes), TCP, UDP, the VXLAN and GTPv1 tunnels
 * (+ the inner packet), Payload, Trailer, the first layers of link types Ethernet, raw IP (RAW, DLT_RAW1/2,
 * IPV4, IPV6), Linux SLL / SLL2 and Null/Loopback, and the first L7 layers it can name: HTTPRequest /
 * HTTPResponse (+ the Payload body), SSL records, DNS, SSH messages (port 22) and MySQL (port 3306, where no
 * dissector ahead of it in TcpLayer::parseNextLayer takes the other port).
 * Packets for which the reference would build a layer outside this scope (other L7 dissectors, IGMP, PPPoE,
 * NFLOG / Cisco HDLC first layers, ...) are flagged PCPPX_F_NEEDS_HOST_L7 / PCPPX_F_NEEDS_HOST_PROTO: their
 * layer prefix is exact, and the host owns the rest.
 */
#ifndef PCPPX_H
#define PCPPX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PCPPX_ABI_VERSION 7
/* the library is built with hidden visibility: exactly the functions declared here are exported */
#define PCPPX_API __attribute__((visibility("default")))
#define PCPPX_MAX_LAYERS 16     /* fixed depth cap; deeper chains set PCPPX_F_DEPTH_OVERFLOW */
#define PCPPX_MAX_CAPLEN 65535  /* larger packets are flagged PCPPX_F_OVERSIZE and not parsed */

/* error codes */
#define PCPPX_OK 0
#define PCPPX_E_INVAL -1    /* bad argument (null pointer, n too large, max_layers > 16 ...) */
#define PCPPX_E_NODEV -2    /* no HIP device / bad ordinal */
#define PCPPX_E_HIP -3      /* a HIP runtime call failed */
#define PCPPX_E_NOMEM -4    /* device or pinned allocation failed */
#define PCPPX_E_LINKTYPE -5 /* link type not handled by the device path */

/* pcppx_summary.flags */
#define PCPPX_F_NEEDS_HOST_L7 0x0001    /* an L4 payload would go to an L7 dissector the device does not
                                           build (TcpLayer.cpp:372-491, UdpLayer.cpp:103-178); chain stops at
                                           the L4 layer */
#define PCPPX_F_NEEDS_HOST_PROTO 0x0002 /* an out-of-scope L2/L3 layer would be built (PPPoE, IGMP, IPSec,
                                           VRRP, ICMPv6, STP, WoL); chain stops before it */
#define PCPPX_F_DEPTH_OVERFLOW 0x0004   /* more than max_layers layers; extra layers not written */
#define PCPPX_F_OVERSIZE 0x0008         /* caplen > PCPPX_MAX_CAPLEN: not parsed */
#define PCPPX_F_IP_CSUM 0x0010          /* ip_csum_* computed (an IPv4 layer exists and want_checksums) */
#define PCPPX_F_IP_CSUM_OK 0x0020       /* ip_csum_calc == ip_csum_stored */
#define PCPPX_F_L4_CSUM 0x0040          /* l4_csum_* computed (a TCP/UDP layer exists and want_checksums) */
#define PCPPX_F_L4_CSUM_OK 0x0080       /* l4_csum_calc == l4_csum_stored */
#define PCPPX_F_TRAILER 0x0100          /* last layer is a PacketTrailer (Packet.cpp:178-195) */
#define PCPPX_F_BAD_DESC 0x0200         /* offsets[i] + caplens[i] > batch data_len: not parsed */
/* The first L7 layer of a NEEDS_HOST_L7 packet, where the device can name it (the content checks of
 * TcpLayer.cpp:372-415 / UdpLayer.cpp:103-116 it restates): with PCPPX_F_L7_KNOWN set, the packet's chain holds
 * an HTTPRequest/HTTPResponse, SSL or DNS layer exactly when the matching bit is set, i.e.
 * Packet::isPacketOfType(HTTP / SSL / DNS) is decided. Not set for tunnels (VXLAN, GTPv1) whose inner packet only
 * the host parses (the VXLAN / GTPv1 tunnels the device builds itself are not NEEDS_HOST_L7). An HTTP / SSL /
 * DNS layer the device builds itself is in the records and proto_mask instead, with none of these bits: the
 * packet is not NEEDS_HOST_L7. */
#define PCPPX_F_L7_KNOWN 0x0400
#define PCPPX_F_L7_HTTP 0x0800
#define PCPPX_F_L7_SSL 0x1000
#define PCPPX_F_L7_DNS 0x2000
#define PCPPX_F_NEEDS_HOST \
	(PCPPX_F_NEEDS_HOST_L7 | PCPPX_F_NEEDS_HOST_PROTO | PCPPX_F_OVERSIZE | PCPPX_F_BAD_DESC)

/* One parsed layer, 8 bytes. */
typedef struct pcppx_layer {
	uint8_t proto;     /* pcpp::ProtocolType (ProtocolType.h:42-258) */
	uint8_t osi;       /* pcpp::OsiModelLayer (ProtocolType.h:266-284) */
	uint16_t offset;   /* Layer::getData() - RawPacket::getRawData() */
	uint16_t hdr_len;  /* Layer::getHeaderLen() */
	uint16_t data_len; /* Layer::getDataLen() */
} pcppx_layer;

/* Per-packet summary, 32 bytes. */
typedef struct pcppx_summary {
	uint32_t hash5;          /* pcpp::hash5Tuple(&packet, false) */
	uint32_t hash5_dir;      /* pcpp::hash5Tuple(&packet, true) */
	uint32_t hash2;          /* pcpp::hash2Tuple(&packet) */
	uint16_t flags;          /* PCPPX_F_* */
	uint8_t n_layers;        /* layers in the chain (capped at max_layers, see PCPPX_F_DEPTH_OVERFLOW) */
	uint8_t l4_layer;        /* index of the layer hash5Tuple takes its ports from (last TCP, else last
	                            UDP); 0xFF if none */
	uint64_t proto_mask;     /* bit p set iff some layer has protocol p: Packet::isPacketOfType(p) */
	uint16_t ip_csum_calc;   /* computeChecksum over the first IPv4 header, checksum field zeroed
	                            (IPv4Layer.cpp:410-412) — the value computeCalculateFields would store */
	uint16_t ip_csum_stored; /* be16 of the header's checksum field */
	uint16_t l4_csum_calc;   /* {Tcp,Udp}Layer::calculateChecksum(false) of layer l4_layer */
	uint16_t l4_csum_stored; /* be16 of that layer's checksum field */
} pcppx_summary;

/* The summary's first 16 bytes alone (ABI 7): what a caller that reads the layer records needs besides them. The
 * protocol mask is the OR of the recorded chain's protocols (pcppx_chain_proto_mask below: exact when the chain is
 * recorded whole -- no PCPPX_F_DEPTH_OVERFLOW and n_layers <= max_layers), and the checksum verdicts are the flags
 * (PCPPX_F_IP_CSUM[_OK], PCPPX_F_L4_CSUM[_OK]); only the computed / stored checksum values are not carried. */
typedef struct pcppx_brief {
	uint32_t hash5;     /* = pcppx_summary.hash5 */
	uint32_t hash5_dir; /* = pcppx_summary.hash5_dir */
	uint32_t hash2;     /* = pcppx_summary.hash2 */
	uint16_t flags;     /* = pcppx_summary.flags */
	uint8_t n_layers;   /* = pcppx_summary.n_layers */
	uint8_t l4_layer;   /* = pcppx_summary.l4_layer */
} pcppx_brief;

/* A batch of packets: bytes of packet i are data[offsets[i] .. offsets[i] + caplens[i]).
 * For the fast path packets should be stored back to back in ascending offset order (any order and
 * gaps are legal; they only cost bandwidth). */
typedef struct pcppx_batch {
	const uint8_t* data;
	const uint64_t* offsets;
	const uint32_t* caplens;
	uint64_t data_len; /* bytes addressable at data (bounds every packet) */
	uint32_t n;
	uint16_t linktype; /* pcpp::LinkLayerType (RawPacket.h:24-178) for every packet of the batch */
	uint16_t reserved;
} pcppx_batch;

/* pcpp::PacketParseOptions (Packet++/header/Packet.h:17-37) plus output selection. */
typedef struct pcppx_opts {
	uint32_t parse_until_family; /* pcpp::ProtocolTypeFamily; 0 = UnknownProtocol (parse everything) */
	uint8_t parse_until_osi;     /* pcpp::OsiModelLayer; 8 = OsiModelLayerUnknown */
	uint8_t want_checksums;      /* compute IPv4 / L4 checksums */
	uint8_t max_layers;          /* 0 = do not write layers; else layers stride per packet (1..16) */
	uint8_t window;              /* PCPPX_WINDOW_*: the header window the parse gathers per packet (a speed choice for
	                                the caller's traffic: the records are identical whichever window runs) */
	uint8_t layout;              /* PCPPX_LAYOUT_*: how pcppx_records.layers is laid out */
	uint8_t reserved[3];
} pcppx_opts;
#define PCPPX_WINDOW_DEFAULT 0 /* the engine's choice (ABI 7), from the traffic this context has parsed with it: ahead
                                  of those parses (each until the first decision, then one in 16) ~64 tiles of the batch
                                  count their deep stacks (a sampling kernel: after up to two VLAN tags an MPLS label,
                                  or an IP layer not followed by TCP / UDP); when more than 1 in 256 sampled packets
                                  had one, the next launches run as DEEP (checksum launches) / with the second round
                                  (parse-only), otherwise checksum launches gather one 96-B window (5 waves/SIMD) and
                                  parse-only ones run as SHORT. Until 2048 packets were sampled: one 96-B window for checksum launches,
                                  96 B + a second round up to 144 B for parse-only ones. pcppx_window_choice() */
#define PCPPX_WINDOW_DEEP 1    /* checksum launches too gather the two-round 144-B window: deep stacks stay on the
                                  fast path instead of the generic walk; 4 waves/SIMD. Parse-only: as DEFAULT */
#define PCPPX_WINDOW_SHORT 2   /* parse-only launches: one 96-B gather round and no second one (7 KiB of LDS per wave
                                  instead of 10: more waves per CU) -- faster on plain Eth / VLAN / IP / L4 traffic
                                  (IMIX 7%, 64-B packets 16%), about 2x slower on deep encapsulation, whose stacks past
                                  96 B take the generic walk. Checksum launches: as DEFAULT */

/* pcppx_records.layers layouts (pcppx_opts.layout). Both hold the same pcppx_layer entries, bit for bit:
 *   FIXED:  packet i's layer k is layers[i * max_layers + k], k < min(n_layers, max_layers); entries past
 *           n_layers are unspecified.
 *   PACKED: only the chain's entries are written, densely per 64-packet tile: the entries of tile t (packets
 *           64t .. 64t+63) start at layers[64 * t * max_layers], and packet i's entries follow those of the packets
 *           before it in its tile: layers[64 * t * max_layers + sum_{64t <= j < i} min(n_layers_j, max_layers) + k].
 *           The buffer is sized as for FIXED (n * max_layers entries); the summary or the brief is required (its
 *           n_layers decode the positions: pcppx_unpack_layers[_brief] below, pcppx::unpackLayers in include/pcppx.hpp). The write
 *           traffic is the chain, not max_layers rows per packet. max_layers <= PCPPX_PACKED_MAX_LAYERS. Device parse
 *           only; the consumers of a parse's records (pcppx_filter_device, pcppx_reasm_device) read FIXED records and
 *           refuse PACKED ones (pcppx_records.layout). */
#define PCPPX_LAYOUT_FIXED 0
#define PCPPX_LAYOUT_PACKED 1
#define PCPPX_PACKED_MAX_LAYERS 12
/*   DENSE (ABI 7, host path): the chains back to back over the whole batch, in packet order: packet i's entries are
 *           layers[sum_{j < i} min(n_layers_j, max_layers) + k]; pcppx_records.layers_written returns the total. The
 *           buffer must hold the total (n * max_layers entries always do; unwritten memory is never touched), and
 *           only the chains cross PCIe (config 3: 4.2 entries = 34 B per packet instead of 8 * max_layers).
 *           max_layers <= PCPPX_MAX_LAYERS. pcppx_parse_batch_host only. Entry positions are 32-bit: a batch with
 *           n * max_layers > UINT32_MAX is refused with PCPPX_E_INVAL (split it; 268M packets at max_layers 16). */
#define PCPPX_LAYOUT_DENSE 2

/* The 5-tuple extract (the compact record of the bandwidth runs), 48 bytes per packet: exactly the
 * fields pcpp::hash5Tuple reads (Packet++/src/PacketUtils.cpp:139-210), from the same layers as the summary's
 * hashes -- the first IPv4 layer, else the first IPv6 layer (getLayerOfType<IPv4Layer>() / <IPv6Layer>()), and
 * the last TCP layer, else the last UDP layer (getLayerOfType<TcpLayer>(true) / <UdpLayer>(true)). */
typedef struct pcppx_tuple {
	uint8_t src_ip[16]; /* IPv4: getSrcIPv4Address() bytes in packet order, then 12 zero bytes; IPv6: ipSrc; none: 0 */
	uint8_t dst_ip[16];
	uint16_t src_port;  /* the port layer's getSrcPort() (host order); 0 without a TCP/UDP layer */
	uint16_t dst_port;  /* getDstPort() */
	uint8_t ip_version; /* 4 or 6: which layer the addresses come from; 0 = no IP layer */
	uint8_t ip_proto;   /* that layer's protocol (IPv4) / nextHeader (IPv6) byte: hash5Tuple's last byte */
	uint8_t l4_proto;   /* pcpp::TCP (4) / pcpp::UDP (5): the port layer; 0 = none */
	uint8_t has_5tuple; /* 1 iff hash5Tuple hashes these fields: an IP layer, a TCP/UDP layer and no ICMP layer
	                       (PacketUtils.cpp:141-148); 0: hash5 == 0 */
	uint32_t hash5;     /* pcpp::hash5Tuple(&packet, false) (= pcppx_summary.hash5) */
	uint16_t flags;     /* pcppx_summary.flags (PCPPX_F_NEEDS_HOST*: the fields of a flagged packet are those of the
	                       chain prefix the device built) */
	uint8_t n_layers;   /* pcppx_summary.n_layers */
	uint8_t reserved;
} pcppx_tuple;

/* PacketStats::collectStats (Examples/DpdkExample-FilterTraffic/Common.h:83-104) over a parsed batch: word k of
 * pcppx_records.proto_stats (device memory, PCPPX_PROTO_STATS words, accumulated by += across calls) counts */
#define PCPPX_PS_PACKETS 0    /* packets of the batch */
#define PCPPX_PS_ETH 1        /* isPacketOfType(Ethernet) */
#define PCPPX_PS_ARP 2        /* isPacketOfType(ARP) */
#define PCPPX_PS_IPV4 3       /* isPacketOfType(IPv4) */
#define PCPPX_PS_IPV6 4       /* isPacketOfType(IPv6) */
#define PCPPX_PS_TCP 5        /* isPacketOfType(TCP) */
#define PCPPX_PS_UDP 6        /* isPacketOfType(UDP) */
#define PCPPX_PS_HTTP 7       /* isPacketOfType(HTTP), over the packets the device settles (below) */
#define PCPPX_PS_DNS 8        /* isPacketOfType(DNS), the same */
#define PCPPX_PS_SSL 9        /* isPacketOfType(SSL) (collectStats' tlsCount), the same */
#define PCPPX_PS_NEEDS_HOST 10 /* packets whose HTTP/DNS/SSL answer the host must complete: a chain stopped before an
                                 out-of-scope layer (NEEDS_HOST_PROTO), a bad record, or an L7 payload the device could
                                 not classify -- as pcppx_packet_stats.needs_host_count */
#define PCPPX_PROTO_STATS 16  /* words (11-15 are zero) */

/* Output arrays (same memory space as the batch for the _device call, host for the _host call). */
typedef struct pcppx_records {
	pcppx_summary* summary; /* n entries, or NULL when `brief` is set; may also be NULL on the device path when max_layers
	                           is 0 and one of tuples / flow_keys / proto_stats is set (e.g. a flow table's launch: dense
	                           keys + collectStats) */
	pcppx_layer* layers;    /* n * max_layers entries in pcppx_opts.layout, or NULL when max_layers == 0 */
	uint32_t* flow_keys;    /* optional (NULL): n entries, flow_keys[i] = summary[i].hash5 -- the dense column
	                           FilterTraffic's flow table is keyed by (pcppx_flow_count_keys_device reads 8 B per
	                           packet from it and caplens instead of 36 B through the summary) */
	pcppx_tuple* tuples;    /* optional (NULL): n 5-tuple extracts. Device path only */
	uint64_t* proto_stats;  /* optional (NULL): PCPPX_PROTO_STATS counters, accumulated (collectStats). Device path
	                           only; calls that set it on one context are ordered (they share its scratch) */
	uint8_t layout;         /* PCPPX_LAYOUT_* of `layers`: written by the parse calls (= opts->layout); read by
	                           pcppx_filter_device / pcppx_reasm_device, which refuse PCPPX_LAYOUT_PACKED records.
	                           Zero-initialised records are FIXED. */
	uint8_t reserved[7];
	pcppx_brief* brief;     /* optional (NULL), ABI 7: n 16-B briefs (the summary's first half), beside or instead of
	                           the summary -- the record a layer-reading caller needs (device and host paths) */
	uint64_t layers_written; /* out: layer entries written (PCPPX_LAYOUT_DENSE: the total of the chains) */
} pcppx_records;

/* Packet::isPacketOfType's mask (bit p for every protocol p of the chain) from a packet's recorded layers: equals
 * pcppx_summary.proto_mask when the chain is recorded whole (pcppx_brief) */
static inline uint64_t pcppx_chain_proto_mask(const pcppx_layer* chain, unsigned n_layers)
{
	uint64_t m = 0;
	for (unsigned k = 0; k < n_layers; ++k)
		m |= chain[k].proto < 64 ? 1ull << chain[k].proto : 0ull;
	return m;
}

/* The caller's own host parse of ONE packet — its Packet++ (`pcpp::Packet packet(&raw, parseUntil...)`) turned
 * into this engine's records: summary + up to opts->max_layers layers, as the engine would write them had it
 * finished the chain. The engine never calls it and libpcppx.so never links Packet++: the C++ facade
 * (pcppx.hpp, Engine::setHostParser) calls it for packets flagged PCPPX_F_NEEDS_HOST, so that a caller's
 * per-packet loop sees every packet completely. INTEGRATION.md §2 has an implementation over pcpp::Packet.
 * Returns 0 or a negative PCPPX_E_* code. */
typedef int (*pcppx_host_parse_fn)(const uint8_t* packet, uint32_t caplen, uint16_t linktype, const pcppx_opts* opts,
                                   pcppx_summary* summary, pcppx_layer* layers);

typedef struct pcppx_ctx pcppx_ctx;

/* library / device management */
PCPPX_API int pcppx_abi_version(void);
PCPPX_API const char* pcppx_strerror(int err);
PCPPX_API int pcppx_device_count(int* out);
PCPPX_API int pcppx_runtime_info(int device, char* buf, size_t len); /* HIP runtime/driver versions, device name */
PCPPX_API int pcppx_open(int device_ordinal, pcppx_ctx** out); /* one per host thread & GPU */
PCPPX_API void pcppx_close(pcppx_ctx* ctx);
PCPPX_API int pcppx_sync(pcppx_ctx* ctx);                      /* wait for everything queued on ctx's stream */
PCPPX_API void* pcppx_ctx_stream(pcppx_ctx* ctx);              /* the context's own hipStream_t */
/* the window a PCPPX_WINDOW_DEFAULT launch with / without checksums would run with now (waits for the last sample) */
PCPPX_API int pcppx_window_choice(pcppx_ctx* ctx, int want_checksums, int* window);
PCPPX_API void pcppx_default_opts(pcppx_opts* opts);           /* Packet(RawPacket*) defaults + checksums + 16 layers */

/* Device-resident parse. batch and records hold device pointers; the kernels are queued on
 * hip_stream (a hipStream_t; NULL = the null/default stream, as everywhere in HIP) and the call returns
 * without waiting. pcppx_ctx_stream() gives the context's own non-blocking stream. */
PCPPX_API int pcppx_parse_batch_device(pcppx_ctx* ctx, const pcppx_batch* batch, const pcppx_opts* opts,
                             pcppx_records* out, void* hip_stream);

/* Host-to-host parse: batch and records hold host pointers. The context stages the bytes through pinned
 * buffers in chunks, overlapping H2D copies, kernels and D2H copies; returns when out is filled. The FIXED or the DENSE
 * layout; a summary and / or a brief; records.tuples and records.proto_stats must be NULL (device-path outputs). */
PCPPX_API int pcppx_parse_batch_host(pcppx_ctx* ctx, const pcppx_batch* batch, const pcppx_opts* opts,
                           pcppx_records* out);

/* Per-flow counters keyed by hash5Tuple (Examples/DpdkExample-FilterTraffic/AppWorkerThread.h:99-125).
 * Device pointers: summary[n] from a previous parse, caplens[n]. The table is open-addressed with
 * `capacity` slots (power of two), split into min(512, max(1, capacity / 4096)) equal regions by the key's hash (a
 * flow lives in its region; every region has at least 4096 slots, or is the whole table); keys[i]==0 marks an
 * empty slot — flow key 0 (non-5-tuple packets, PacketUtils.cpp:141-148) is counted in stats[0] (packets) /
 * stats[1] (bytes) instead, and packets whose region had no free slot in stats[2]. Counts accumulate across
 * calls; calls on one context are ordered (they share its scratch). HBM scratch held by the context: record
 * queues of 16 B x min(n, 2^24) x ~1.25 (grown in stream order, freed by pcppx_close). */
/* The same over the dense key column a parse wrote (pcppx_records.flow_keys): keys_in[i] = hash5 of packet i. */
PCPPX_API int pcppx_flow_count_keys_device(pcppx_ctx* ctx, const uint32_t* keys_in, const uint32_t* caplens, uint32_t n,
                                           uint32_t* keys, uint64_t* packets, uint64_t* bytes, uint32_t capacity,
                                           uint64_t* stats, void* hip_stream);
PCPPX_API int pcppx_flow_count_device(pcppx_ctx* ctx, const pcppx_summary* summary, const uint32_t* caplens,
                            uint32_t n, uint32_t* keys, uint64_t* packets, uint64_t* bytes,
                            uint32_t capacity, uint64_t* stats, void* hip_stream);

/* ---- DpdkExample-FilterTraffic's worker on the device ----
 * PacketMatchingEngine::isMatched (Examples/DpdkExample-FilterTraffic/PacketMatchingEngine.h:43-107),
 * the matched-flow table keyed by hash5Tuple and PacketStats::collectStats (AppWorkerThread.h:85-139,
 * Common.h:83-104), over a parsed device batch (records from pcppx_parse_batch_device; max_layers >= 1).
 * Packet order is the worker's receive order: packet i of the batch has sequence number seq_base + i,
 * and a packet matches if it matches on its own or an earlier packet of the same 5-tuple flow matched.
 * The flow table (flow_keys / flow_first, `capacity` slots, power of two, zero-initialised) persists
 * across batches like the worker's m_FlowTable. */
typedef struct pcppx_match_spec {
	uint32_t src_ip;   /* IPv4Address::toInt() (network byte order in memory); 0 = any */
	uint32_t dst_ip;   /* 0 = any */
	uint16_t src_port; /* host order; 0 = any */
	uint16_t dst_port; /* 0 = any */
	uint8_t protocol;  /* pcpp::TCP (4) or pcpp::UDP (5); anything else = any */
	uint8_t reserved[3];
} pcppx_match_spec;

typedef struct pcppx_packet_stats { /* PacketStats, Examples/DpdkExample-FilterTraffic/Common.h:57-142 */
	uint64_t packet_count, eth_count, arp_count, ipv4_count, ipv6_count, tcp_count, udp_count;
	uint64_t http_count, dns_count, tls_count; /* isPacketOfType(HTTP / DNS / SSL) of the packets the device
	                                              settles: the first L7 layer of a NEEDS_HOST_L7 packet is
	                                              classified on the device (TcpLayer.cpp:372-415,
	                                              UdpLayer.cpp:103-116) */
	uint64_t matched_tcp_flows, matched_udp_flows, matched_packets;
	uint64_t needs_host_count;                  /* packets whose counters the host must complete: chains stopped
	                                              before an out-of-scope L2/L3 layer (NEEDS_HOST_PROTO), bad
	                                              records, or UDP tunnels (VXLAN, GTPv1) carrying inner packets */
	uint64_t flow_table_full;                   /* matched packets whose flow found no free slot in the device flow
	                                              table (capacity too small for the traffic's flows): the reference's
	                                              unordered_map never fills, so when this is non-zero the
	                                              matched_* counters and verdicts are no longer the reference's */
} pcppx_packet_stats;

PCPPX_API int pcppx_filter_device(pcppx_ctx* ctx, const pcppx_batch* batch, const pcppx_records* records, uint8_t max_layers,
                        const pcppx_match_spec* spec, uint64_t seq_base, uint64_t* flow_keys, uint64_t* flow_first,
                        uint32_t capacity, uint8_t* matched, pcppx_packet_stats* stats, void* hip_stream);

/* The same worker over host batches, with the flow table, packet sequence and statistics held by the
 * context (one context = one worker, AppWorkerThread.h:45-162): packets are staged to HBM, parsed and
 * filtered there; matched[i] = 1 for packets the worker would send on (AppWorkerThread.h:127-131).
 * *stats (may be NULL) receives the statistics accumulated since the last pcppx_filter_reset.
 * pcppx_filter_reset sizes (capacity: power of two, 0 = 4M slots) and clears the flow table; the first
 * pcppx_filter_batch_host call does it implicitly. */
PCPPX_API int pcppx_filter_reset(pcppx_ctx* ctx, uint32_t capacity);
PCPPX_API int pcppx_filter_batch_host(pcppx_ctx* ctx, const pcppx_batch* batch, const pcppx_match_spec* spec,
                            uint8_t* matched, pcppx_packet_stats* stats);

/* ---- reassembly front ends ----
 * The stateless per-packet half of the two reassemblers, over a parsed device batch:
 *   IPReassembly::processPacket up to its fragment-table lookup (Packet++/src/IPReassembly.cpp:281-322):
 *     non-IP / non-fragment / malformed classification, the fragment key hashPacket() (FNV-1 over src, dst,
 *     IP id: IPReassembly.cpp:103-115 for IPv4, :190-205 for IPv6), getFragmentId / getFragmentOffset and
 *     isFirstFragment / isLastFragment (IPv4Layer.cpp:415-438, IPv6Extensions.cpp:71-91);
 *   TcpReassembly::reassemblePacket up to its connection lookup (Packet++/src/TcpReassembly.cpp:81-141):
 *     non-IP / non-TCP / no-data classification, the TCP payload size and SYN/FIN/RST; the connection key
 *     is hash5Tuple = pcppx_summary.hash5 (TcpReassembly.cpp:141).
 * The stateful tables (fragment lists, connection map, callbacks) stay with the host caller.
 * A packet whose chain the engine did not finish (PCPPX_F_NEEDS_HOST_PROTO, OVERSIZE, BAD_DESC,
 * DEPTH_OVERFLOW, or NEEDS_HOST_L7 on a UDP payload) gets *_HOST unless its first IPv4 layer is recorded
 * (then ip_status is exact). NEEDS_HOST_L7 on a TCP payload is exact: the dissectors reached from TCP ports
 * (TcpLayer.cpp:372-491) build no further IP or TCP layer. */
#define PCPPX_IPR_NON_IP 0       /* IPReassembly::NON_IP_PACKET */
#define PCPPX_IPR_NON_FRAGMENT 1 /* IPReassembly::NON_FRAGMENT */
#define PCPPX_IPR_MALFORMED 2    /* IPReassembly::MALFORMED_FRAGMENT (payload size > data len, :315-320) */
#define PCPPX_IPR_FRAGMENT 3     /* a fragment: ip_key / frag_id / frag_offset set; the host table decides */
#define PCPPX_IPR_HOST 15        /* the packet's chain is not finished on the device: the host decides */
#define PCPPX_IPR_F_FIRST 0x10   /* isFirstFragment() */
#define PCPPX_IPR_F_LAST 0x20    /* isLastFragment() */
#define PCPPX_IPR_F_IPV6 0x40    /* the IPv6 wrapper was used (no IPv4 layer in the packet); a fragment header
                                    lies inside the IPv6 header, which a non-malformed fragment holds whole */

#define PCPPX_TCPR_NON_IP 0  /* TcpReassembly::NonIpPacket */
#define PCPPX_TCPR_NON_TCP 1 /* TcpReassembly::NonTcpPacket */
#define PCPPX_TCPR_NO_DATA 2 /* TcpReassembly::Ignore_PacketWithNoData */
#define PCPPX_TCPR_DATA 3    /* goes on to the connection table keyed by hash5 */
#define PCPPX_TCPR_HOST 15   /* the packet's chain is not finished on the device: the host decides */
#define PCPPX_TCPR_F_FIN 0x10
#define PCPPX_TCPR_F_SYN 0x20
#define PCPPX_TCPR_F_RST 0x40

typedef struct pcppx_reasm_info { /* 16 bytes per packet */
	uint32_t ip_key;      /* hashPacket() when ip_status is PCPPX_IPR_FRAGMENT, else 0 */
	uint32_t frag_id;     /* getFragmentId(): be16 IPv4 id / be32 IPv6 fragment id (0 unless a fragment) */
	uint16_t frag_offset; /* getFragmentOffset() in bytes (0 unless a fragment) */
	uint8_t ip_status;    /* PCPPX_IPR_* (low nibble) | PCPPX_IPR_F_* */
	uint8_t tcp_status;   /* PCPPX_TCPR_* (low nibble) | PCPPX_TCPR_F_* of the last TCP layer */
	uint32_t tcp_payload; /* the last TCP layer's getLayerPayloadSize() (0 without a TCP layer) */
} pcppx_reasm_info;

/* batch (device pointers) + its records from pcppx_parse_batch_device (max_layers >= 1, the same
 * max_layers here) -> info[n] (device). Queued on hip_stream; returns without waiting. */
PCPPX_API int pcppx_reasm_device(pcppx_ctx* ctx, const pcppx_batch* batch, const pcppx_records* records, uint8_t max_layers,
                       pcppx_reasm_info* info, void* hip_stream);

/* pcppx_parse_batch_device and pcppx_reasm_device in one pass: the parse kernel writes info[n] too, from the
 * header bytes it already holds (no second read of the packets or records). opts->max_layers >= 1. The
 * records and info equal those of the two calls made one after the other. */
PCPPX_API int pcppx_parse_batch_device_reasm(pcppx_ctx* ctx, const pcppx_batch* batch, const pcppx_opts* opts,
                                   pcppx_records* out, pcppx_reasm_info* info, void* hip_stream);

/* ---- host ingest: pcap / pcapng captures into packed batch buffers ---- */
typedef struct pcppx_pcap pcppx_pcap;
/* Open a capture; the format comes from its first 4 bytes as IFileReaderDevice::createReader
 * (Pcap++/src/PcapFileDevice.cpp:546-583): pcap as PcapFileReaderDevice::open (:707-768, incl. its version
 * and snapshot-length checks), pcapng as PcapNgFileReaderDevice::open (:1157-1176, LightPcapNg). */
PCPPX_API int pcppx_pcap_open(const char* path, pcppx_pcap** out);
/* RawPacket::getLinkLayerType of the packets of the last batch returned (before the first batch: of the
 * first packet). pcap: the file header's, LINKTYPE_INVALID (0xFFFF) outside LinkLayerType; pcapng: the
 * packet's interface's. */
PCPPX_API uint32_t pcppx_pcap_linktype(const pcppx_pcap* reader);
/* Append up to max_packets records back to back into data[0, data_cap) (pinned memory feeds
 * pcppx_parse_batch_host without a staging copy); *n_out = packets read (0 at end of file). Record checks
 * as PcapFileReaderDevice::readNextPacket (PcapFileDevice.cpp:799-886) / light_get_next_packet. A batch
 * holds one link type: it ends before a packet of another (pcapng interfaces). timestamps_ns may be NULL. */
PCPPX_API int pcppx_pcap_read_batch(pcppx_pcap* reader, uint8_t* data, uint64_t data_cap, uint64_t* offsets,
                          uint32_t* caplens, uint64_t* timestamps_ns, uint32_t max_packets, uint32_t* n_out,
                          uint64_t* bytes_out);
/* as pcppx_pcap_read_batch, plus each packet's original (wire) length, RawPacket::getFrameLength
 * (frame_lens may be NULL) */
PCPPX_API int pcppx_pcap_read_batch_ex(pcppx_pcap* reader, uint8_t* data, uint64_t data_cap, uint64_t* offsets,
                          uint32_t* caplens, uint32_t* frame_lens, uint64_t* timestamps_ns, uint32_t max_packets,
                          uint32_t* n_out, uint64_t* bytes_out);
/* Zero-copy: the next batch's packets stay where they are in the reader's memory-mapped file. *data = the map
 * base, *data_len = the file size, offsets[i] = the position of packet i's bytes in it (caplens / frame_lens /
 * timestamps_ns as pcppx_pcap_read_batch_ex; the same records and batch boundaries). The file's record headers lie
 * between the packets -- a gapped, ascending batch, which pcppx_parse_batch_host stages as near-contiguous ranges.
 * The bytes stay valid until pcppx_pcap_close. */
PCPPX_API int pcppx_pcap_map_batch(pcppx_pcap* reader, const uint8_t** data, uint64_t* data_len, uint64_t* offsets,
                                   uint32_t* caplens, uint32_t* frame_lens, uint64_t* timestamps_ns, uint32_t max_packets,
                                   uint32_t* n_out);
PCPPX_API void pcppx_pcap_close(pcppx_pcap* reader);

/* PCPPX_LAYOUT_PACKED layer entries (host memory, from a device parse) -> the FIXED layout: fixed[i * max_layers + k]
 * for k < min(summary[i].n_layers, max_layers), zero past each chain. max_layers <= PCPPX_PACKED_MAX_LAYERS. */
PCPPX_API int pcppx_unpack_layers(const pcppx_summary* summary, const pcppx_layer* packed, uint64_t n,
                                  uint32_t max_layers, pcppx_layer* fixed);
/* the same with the chain lengths from briefs (ABI 7) */
PCPPX_API int pcppx_unpack_layers_brief(const pcppx_brief* brief, const pcppx_layer* packed, uint64_t n,
                                        uint32_t max_layers, pcppx_layer* fixed);
PCPPX_API void* pcppx_host_alloc(size_t bytes); /* page-locked host memory (hipHostMalloc) */
PCPPX_API void pcppx_host_free(void* p);

#ifdef __cplusplus
}
#endif

#endif /* PCPPX_H */
