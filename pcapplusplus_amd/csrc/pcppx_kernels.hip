// pcppx_kernels.hip — gfx950 kernels of the packet-dissection engine.
//
// One lane owns one packet. A 256-lane workgroup stages the first 128 bytes of each of its packets
// from HBM into a private LDS slot (aligned 16-B loads), walks the packet's layer chain out of LDS
// (the per-layer rules of Packet++: Packet.cpp:66-196 and each Layer::parseNextLayer), then
//   - writes the layer records (8 B each) and a 32-B summary per packet,
//   - computes hash5Tuple / hash2Tuple (FNV-1, PacketUtils.cpp:114-245) from the staged header bytes,
//   - computes the IPv4 header and TCP/UDP pseudo-header checksums (PacketUtils.cpp:12-112) with the
//     ones'-complement sum taken mod 65535 over aligned 16-B chunks: a chunk's little-endian word sum
//     is byte-order independent up to a multiply by 256 (an odd start address), so each lane streams its
//     L4 bytes with aligned dwordx4 loads and never shifts bytes.
// Pure integer/byte work: no MFMA. The parse-side semantics are restated independently in
// oracle/pcppx_oracle.c, which is the parity checker for everything here.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "pcppx.h"
#include "pcppx_internal.h"

namespace pcppx
{
namespace
{

constexpr int kBlock = 256;

// ProtocolType ids (Packet++/header/ProtocolType.h:42-258)
enum : uint32_t
{
	P_ETH = 1, P_IPV4 = 2, P_IPV6 = 3, P_TCP = 4, P_UDP = 5, P_ARP = 8, P_VLAN = 9, P_ICMP = 10, P_MPLS = 14, P_GREV0 = 15,
	P_GREV1 = 16, P_PPTP = 17, P_SLL = 19, P_NULL = 21, P_PAYLOAD = 25, P_TRAILER = 30, P_DOT3 = 33, P_LLC = 44,
	P_SLL2 = 52, P_VXLAN = 26, P_GTPV1 = 32, P_NFLOG = 47, P_CISCO_HDLC = 58
};

// next-layer kinds of the chain walk
enum : uint32_t
{
	K_NONE = 0, K_ETH, K_DOT3, K_LLC, K_VLAN, K_MPLS, K_IPV4, K_IPV6, K_GRE0, K_GRE1, K_PPTP, K_TCP, K_UDP,
	K_PAYLOAD, K_OUT, K_ARP, K_SLL, K_SLL2, K_NULL,  // SLL / SLL2 / Null-Loopback: first layers only
	K_ICMP, K_VXLAN, K_GTP1,
	K_HDLC, K_NFLOG,  // Cisco HDLC / NFLOG: first layers only (round 6)
	// candidates: the layer a tryConstructNextLayerWithFallback would build if its isDataValid holds, else
	// Payload (Layer.h:474-483); resolved from the candidate's own first bytes when the walk reaches it
	C_IPV4, C_IPV6, C_TCP, C_IPVER, C_GRE, C_ETHG, C_LLC, C_ICMP, C_ETH, C_IPGTP
};

// explicit address spaces: keep packet reads as global_load / ds_read, never flat
typedef const __attribute__((address_space(1))) uint8_t* gptr8;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) u32x4* gptr16;
typedef const __attribute__((address_space(3))) uint8_t* lptr8;
typedef const __attribute__((address_space(3))) uint32_t* lptr32;
typedef __attribute__((address_space(3))) uint32_t* lptr32w;

struct Pkt
{
	gptr8 g;                   // packet start in global memory
	lptr8 s;                   // LDS slot base (byte 0 of the aligned window)
	uintptr_t a0;              // aligned window start address (g rounded down to 16)
	uint32_t mis;              // g - a0
	uint32_t lim;              // packet bytes available in LDS: [0, lim)
	uint32_t nch;              // staged 16-B chunks
};

__device__ __forceinline__ uint4 ld16(uintptr_t a)
{
	u32x4 v = *reinterpret_cast<gptr16>(a);
	return make_uint4(v.x, v.y, v.z, v.w);
}

__device__ __forceinline__ uint32_t rb(const Pkt& p, uint32_t j)
{
	if (j < p.lim)
		return p.s[p.mis + j];
	return p.g[j];
}
__device__ __forceinline__ uint32_t be16(const Pkt& p, uint32_t j)
{
	return (rb(p, j) << 8) | rb(p, j + 1);
}
__device__ __forceinline__ uint32_t le16(const Pkt& p, uint32_t j)
{
	return rb(p, j) | (rb(p, j + 1) << 8);
}
__device__ __forceinline__ uint32_t le32(const Pkt& p, uint32_t j)
{
	return rb(p, j) | (rb(p, j + 1) << 8) | (rb(p, j + 2) << 16) | (rb(p, j + 3) << 24);
}
// bytes j..j+3 of the packet, little-endian, from the LDS window: one aligned dword pair and a
// v_alignbyte. The slot's pad dword keeps both reads inside the slot; bytes at or past p.lim are
// garbage and only used by callers that checked j + 4 <= p.lim (or mask them off).
__device__ __forceinline__ uint32_t lds_u32(const Pkt& p, uint32_t j)
{
	const uint32_t pos = p.mis + j;
	lptr32 w = reinterpret_cast<lptr32>(p.s) + (pos >> 2);
	return __builtin_amdgcn_alignbyte(w[1], w[0], pos & 3);
}
__device__ __forceinline__ uint32_t swap16(uint32_t v)
{
	return ((v & 0xFF) << 8) | ((v >> 8) & 0xFF);
}
// little-endian 32/16-bit reads of packet bytes that exist (< caplen): LDS when staged, else bytes
__device__ __forceinline__ uint32_t rd32(const Pkt& p, uint32_t j)
{
	return j + 4 <= p.lim ? lds_u32(p, j) : le32(p, j);
}
__device__ __forceinline__ uint32_t rd16(const Pkt& p, uint32_t j)
{
	return j + 2 <= p.lim ? (lds_u32(p, j) & 0xFFFF) : le16(p, j);
}
// bytes j..j+3 of the packet from HBM as one unaligned dword load (gfx950 global loads take any byte alignment; the
// compiler merges four consecutive ones into one 16-B load). Only for bytes that exist (j + 4 <= caplen).
typedef uint32_t __attribute__((aligned(1))) u32_any;
typedef const __attribute__((address_space(1))) u32_any* gptr32_any;
__device__ __forceinline__ uint32_t ldu32(const Pkt& p, uint32_t j)
{
	return *reinterpret_cast<gptr32_any>(p.g + j);
}

// ---- validity predicates (isDataValid of each layer; cited in oracle/pcppx_oracle.c) ----
__device__ __forceinline__ bool ipv4_ok(const Pkt& p, uint32_t o, uint32_t n)
{
	if (n < 20)
		return false;
	uint32_t b = rb(p, o);
	return (b >> 4) == 4 && (b & 0xF) >= 5;
}
__device__ __forceinline__ bool ipv6_ok(const Pkt& p, uint32_t o, uint32_t n)
{
	return n >= 40 && (rb(p, o) >> 4) == 6;
}
__device__ __forceinline__ bool tcp_ok(const Pkt& p, uint32_t o, uint32_t n)
{
	if (n < 20)
		return false;
	uint32_t d = rb(p, o + 12) >> 4;
	return d >= 5 && n >= d * 4;
}
__device__ __forceinline__ bool eth_ok(const Pkt& p, uint32_t o, uint32_t n)
{
	return n >= 14 && be16(p, o + 12) >= 0x0600;
}
__device__ __forceinline__ bool dot3_ok(const Pkt& p, uint32_t o, uint32_t n)
{
	return n >= 14 && be16(p, o + 12) <= 0x05DC;
}
__device__ __forceinline__ bool llc_ok(const Pkt& p, uint32_t o, uint32_t n)
{
	return n >= 3 && !(rb(p, o) == 0xFF && rb(p, o + 1) == 0xFF);
}

// L7 trigger ports (engine contract = oracle tcp_l7_port / udp_l7_port), as 64K-bit tables in constant
// memory: one table read per port instead of a compare chain (whose per-lane masks are combined by scalar
// instructions, the walk's bottleneck)
constexpr uint16_t kTcpL7Ports[] = { 443, 261, 448, 465, 563, 614, 636, 989, 990, 992, 993, 994, 995, 80, 8080, 5060,
	                                 5061, 179, 22, 53, 5353, 5355, 23, 21, 20, 13400, 3496, 30490, 102, 25, 587, 389,
	                                 5432, 3306, 2123, 502 };
constexpr uint16_t kUdpL7Ports[] = { 53, 5353, 5355, 5060, 5061, 1812, 1813, 3799, 2152, 2123, 546, 547, 123, 13400,
	                                 3496, 30490, 51820 };
constexpr uint16_t kUdpL7DstPorts[] = { 4789, 0, 7, 9 };  // VXLAN, WakeOnLan (UdpLayer.cpp:103-165)
struct L7Tables
{
	uint32_t tcp[2048], udp[2048], udp_dst[2048];
	uint32_t tcp_other[2048];  // tcp minus the HTTP and SSL ports (whose dissectors the engine restates)
};
constexpr L7Tables make_l7_tables()
{
	L7Tables t{};
	for (uint16_t x : kTcpL7Ports)
		t.tcp[x >> 5] |= 1u << (x & 31);
	for (int k = 15; k < (int)(sizeof(kTcpL7Ports) / sizeof(kTcpL7Ports[0])); ++k)  // after 443..995, 80, 8080
		t.tcp_other[kTcpL7Ports[k] >> 5] |= 1u << (kTcpL7Ports[k] & 31);
	for (uint16_t x : kUdpL7Ports)
		t.udp[x >> 5] |= 1u << (x & 31);
	for (uint16_t x : kUdpL7DstPorts)
		t.udp_dst[x >> 5] |= 1u << (x & 31);
	return t;
}
__constant__ L7Tables kL7 = make_l7_tables();

__device__ __forceinline__ uint32_t port_bit(const uint32_t* t, uint32_t x)
{
	return (t[x >> 5] >> (x & 31)) & 1u;
}
__device__ __forceinline__ bool tcp_l7(uint32_t src, uint32_t dst)
{
	return (port_bit(kL7.tcp, src) | port_bit(kL7.tcp, dst)) != 0;
}
__device__ __forceinline__ bool udp_l7(uint32_t src, uint32_t dst)
{
	const uint32_t pr = (src << 16) | dst;  // DHCP 68->67, 67->68, 67->67
	const uint32_t dhcp = (uint32_t)(pr == ((68u << 16) | 67u)) | (uint32_t)(pr == ((67u << 16) | 68u)) |
	                      (uint32_t)(pr == ((67u << 16) | 67u));
	return (dhcp | port_bit(kL7.udp_dst, dst) | port_bit(kL7.udp, src) | port_bit(kL7.udp, dst)) != 0;
}
// SipLayer::detectSipMessageType keys, big-endian packed ("INVI" = 0x494E5649 ...): a perfect hash
// (k * 0x8a05a7) >> 27 over 32 slots, each slot's key checked
constexpr uint32_t kSipMul = 0x8a05a7u;
constexpr uint32_t kSipKeys[] = { 0x494E5649u, 0x41434B20u, 0x42594520u, 0x43414E43u, 0x52454749u,
	                              0x50524143u, 0x4F505449u, 0x53554253u, 0x4E4F5449u, 0x5055424Cu,
	                              0x494E464Fu, 0x52454645u, 0x4D455353u, 0x55504441u, 0x5349502Fu };
struct SipTable
{
	uint32_t key[32];
	uint32_t valid;
};
constexpr SipTable make_sip_table()
{
	SipTable t{};
	for (uint32_t k : kSipKeys)
	{
		const uint32_t h = (k * kSipMul) >> 27;
		t.key[h] = k;
		t.valid |= 1u << h;
	}
	return t;
}
__constant__ SipTable kSip = make_sip_table();
__device__ __forceinline__ bool sip_key(uint32_t k)
{
	const uint32_t h = (k * kSipMul) >> 27;
	return ((kSip.valid >> h) & 1u) && kSip.key[h] == k;
}

// Round 6: the same trigger sets as register tables for the fast path (ParseShape R6 bit 2). A perfect hash of the port
// (one 24-bit multiply and a bit-field extract; multipliers found by search, collision-freedom asserted below) picks a
// slot; the lane holding that slot of a table register hands its entry over by ds_bpermute -- an LDS-crossbar op, no
// memory round trip per packet. TCP: 64 slots, entry = port | 0x10000. UDP: slots 0-31 of the second register, entry =
// port | in kUdpL7Ports << 16 | in kUdpL7DstPorts << 17; lanes 32-63 of the same register hold the SIP key slots.
constexpr uint32_t kTcpSlotMul = 3871678u, kTcpSlotShift = 11, kUdpSlotMul = 12666738u, kUdpSlotShift = 8;
__host__ __device__ constexpr uint32_t tcp_slot(uint32_t x)
{
	return ((x * kTcpSlotMul) >> kTcpSlotShift) & 63u;
}
__host__ __device__ constexpr uint32_t udp_slot(uint32_t x)
{
	return ((x * kUdpSlotMul) >> kUdpSlotShift) & 31u;
}
struct L7Regs
{
	uint32_t tcp[64], udp_sip[64];
	bool perfect;  // every trigger port owns its slot alone
};
constexpr L7Regs make_l7_regs()
{
	L7Regs t{};
	t.perfect = true;
	for (uint16_t x : kTcpL7Ports)
	{
		t.perfect = t.perfect && t.tcp[tcp_slot(x)] == 0;
		t.tcp[tcp_slot(x)] = x | 0x10000u;
	}
	auto put = [&](uint16_t x, uint32_t bit) {
		uint32_t& e = t.udp_sip[udp_slot(x)];
		t.perfect = t.perfect && (e == 0 || (e & 0xFFFFu) == x);
		e = x | bit;
	};
	for (uint16_t x : kUdpL7Ports)
		put(x, t.udp_sip[udp_slot(x)] | 0x10000u);
	for (uint16_t x : kUdpL7DstPorts)
		put(x, t.udp_sip[udp_slot(x)] | 0x20000u);
	for (uint32_t k : kSipKeys)
		t.udp_sip[32 + ((k * kSipMul) >> 27)] = k;
	return t;
}
constexpr L7Regs kL7RegsHost = make_l7_regs();
static_assert(kL7RegsHost.perfect, "L7 port slot hashes must be collision-free");
__constant__ L7Regs kL7R = make_l7_regs();

// ---- the first L7 layer behind TCP/UDP (restated in oracle/pcppx_oracle.c: tcp_l7 / udp_l7) ----
// engine-internal class bits of l7_flags (never in a summary's flags: the layers are built): a MySqlLayer, SSH messages
constexpr uint32_t kL7MySql = 0x4000u, kL7Ssh = 0x8000u;
// TcpLayer::parseNextLayer (TcpLayer.cpp:372-491) tries HTTP request (dst 80/8080 + known method), HTTP response
// (src 80/8080 + known version + supported status code), SSL (SSL port + record header), then dissectors gated by
// their own ports, then Payload: a payload whose only trigger ports are HTTP / SSL ports and that fails those
// content checks is a plain Payload. UdpLayer::parseNextLayer (UdpLayer.cpp:103-183) is port-gated except for the
// SIP content heuristic. The flags name the first L7 layer (PCPPX_F_L7_*) where the device can.
struct HttpCodes
{
	uint32_t bits[16];  // status codes of intStatusCodeMap (HttpLayer.cpp:424-508), bit (code - 100)
};
constexpr HttpCodes make_http_codes()
{
	HttpCodes t{};
	const uint16_t codes[] = { 100, 101, 102, 103, 200, 201, 202, 203, 204, 205, 206, 207, 208, 226, 300, 301, 302,
		                       303, 304, 305, 306, 307, 308, 400, 401, 402, 403, 404, 405, 406, 407, 408, 409, 410,
		                       411, 412, 413, 414, 415, 416, 417, 418, 419, 420, 421, 422, 423, 424, 425, 426, 428,
		                       429, 431, 440, 444, 449, 450, 451, 494, 495, 496, 497, 498, 499, 500, 501, 502, 503,
		                       504, 505, 506, 507, 508, 509, 510, 511, 520, 521, 522, 523, 524, 598, 599 };
	for (uint16_t c : codes)
		t.bits[(c - 100) >> 5] |= 1u << ((c - 100) & 31);
	return t;
}
__constant__ HttpCodes kHttpCodes = make_http_codes();

constexpr uint64_t le_str(const char* m)
{
	uint64_t v = 0;
	for (int j = 0; m[j] != 0; ++j)
		v |= (uint64_t)(uint8_t)m[j] << (8 * j);
	return v;
}
__device__ __forceinline__ bool http_port(uint32_t x)
{
	return x == 80 || x == 8080;  // HttpMessage::isHttpPort, HttpLayer.h:74-77
}
__device__ __forceinline__ bool ssl_port(uint32_t x)
{
	return x == 443 || x == 261 || x == 448 || x == 465 || x == 563 || x == 614 || x == 636 || x == 989 || x == 990 ||
	       (x >= 992 && x <= 995);  // SSLLayer::isSSLPort, SSLLayer.h:488-510
}
__device__ __forceinline__ bool dns_port(uint32_t x)
{
	return x == 53 || x == 5353 || x == 5355;  // DnsLayer::isDnsPort, DnsLayer.h:468-479
}
// HttpRequestFirstLine::parseMethod != Unknown (HttpLayer.cpp:261-285; methods :145-155): the text before the first
// space is a known method; the longest is 7 bytes, so only the first 8 bytes matter
__device__ bool http_request(const Pkt& p, uint32_t o, uint32_t n)
{
	if (n < 4)
		return false;
	uint64_t w = 0;
	uint32_t sp = 8;
	for (uint32_t j = 0; j < 8; ++j)
	{
		const uint32_t c = j < n ? rb(p, o + j) : 0x100u;
		sp = (c == ' ' && sp == 8) ? j : sp;
		w |= (uint64_t)(c & 0xFF) << (8 * j);
	}
	if (sp == 8 || sp == 0 || sp >= n)
		return false;
	w &= (1ull << (8 * sp)) - 1;
	return (sp == 3 && (w == le_str("GET") || w == le_str("PUT"))) ||
	       (sp == 4 && (w == le_str("HEAD") || w == le_str("POST"))) ||
	       (sp == 5 && (w == le_str("TRACE") || w == le_str("PATCH"))) || (sp == 6 && w == le_str("DELETE")) ||
	       (sp == 7 && (w == le_str("OPTIONS") || w == le_str("CONNECT")));
}
// HttpResponseFirstLine::parseVersion != Unknown (HttpLayer.cpp:964-984) and a supported status code with a
// non-empty message (parseStatusCode :850-898, HttpResponseStatusCode(int, msg) :510-543, isUnsupportedCode
// HttpLayer.h:453-456)
__device__ bool http_response(const Pkt& p, uint32_t o, uint32_t n)
{
	if (n < 12)
		return false;
	uint32_t d[12];
#pragma unroll
	for (int j = 0; j < 12; ++j)
		d[j] = rb(p, o + j);
	if (d[0] != 'H' || d[1] != 'T' || d[2] != 'T' || d[3] != 'P' || d[4] != '/')
		return false;
	const bool ver = (d[5] == '0' && d[6] == '.' && d[7] == '9') || (d[5] == '1' && d[6] == '.' && (d[7] == '0' || d[7] == '1'));
	if (!ver || d[9] - '0' > 9u || d[10] - '0' > 9u || d[11] - '0' > 9u)
		return false;
	const uint32_t code = (d[9] - '0') * 100u + (d[10] - '0') * 10u + (d[11] - '0');
	if (code < 100 || code > 599 || !((kHttpCodes.bits[(code - 100) >> 5] >> ((code - 100) & 31)) & 1u))
		return false;
	uint32_t off = 13;
	while (off < n && rb(p, o + off) != '\n')
		++off;
	if (off >= n)
		return false;  // no end of the first line: HttpStatusCodeUnknown
	return off > 14 || (off == 14 && rb(p, o + 13) != '\r');  // a non-empty status message
}
// SSLLayer::IsSSLMessage past its port check (SSLLayer.cpp:14-40; SSLVersion::asEnum(true), SSLCommon.cpp:12-27)
__device__ bool ssl_record(const Pkt& p, uint32_t o, uint32_t n)
{
	if (n < 5)
		return false;
	const uint32_t t = rb(p, o), v = (rb(p, o + 1) << 8) | rb(p, o + 2), len = (rb(p, o + 3) << 8) | rb(p, o + 4);
	return len != 0 && t >= 20 && t <= 23 &&
	       ((v >= 0x0300 && v <= 0x0304) || (v >= 0x7f0e && v <= 0x7f1c) || v == 0xfb17 || v == 0xfb1a);
}
// The L7 decision for a TCP/UDP payload at [o, o+n) with ports sp/dp (host order): 0 = plain Payload, else
// PCPPX_F_NEEDS_HOST_L7 | PCPPX_F_L7_*. `trig` = the ports (or the SIP heuristic) trigger a dissector.
__device__ uint32_t l7_flags(const Pkt& p, bool tcp, uint32_t o, uint32_t n, uint32_t sp, uint32_t dp, bool sip, bool trig)
{
	if (!trig)
		return 0;
	const uint32_t known = PCPPX_F_NEEDS_HOST_L7 | PCPPX_F_L7_KNOWN;
	if (!tcp)
	{
		// DNS after DHCP and VXLAN (UdpLayer.cpp:103-115); then VXLAN (VxlanLayer.h:119-122) and GTPv1
		// (GtpLayer.h:386-389) bring an inner packet only the host parses
		const bool dhcp = (sp == 68 && dp == 67) || (sp == 67 && (dp == 68 || dp == 67));
		if (!dhcp && dp != 4789 && n >= 12 && (dns_port(sp) || dns_port(dp)))
			return known | PCPPX_F_L7_DNS;
		if (dp == 4789 || sp == 2152 || dp == 2152 || sp == 2123 || dp == 2123)
			return PCPPX_F_NEEDS_HOST_L7;
		return known;
	}
	if (http_port(dp) && http_request(p, o, n))
		return known | PCPPX_F_L7_HTTP;
	if (http_port(sp) && http_response(p, o, n))
		return known | PCPPX_F_L7_HTTP;
	if ((ssl_port(sp) || ssl_port(dp)) && ssl_record(p, o, n))
		return known | PCPPX_F_L7_SSL;
	// the rest of the chain is gated by ports other than HTTP's and SSL's
	if (!(port_bit(kL7.tcp_other, sp) | port_bit(kL7.tcp_other, dp)))
		return 0;
	// SSH (TcpLayer.cpp:407-410): port 22 on either side builds SSH messages (SSHLayer::createSSHMessage never fails)
	// unless the other port is SIP's or BGP's, whose branches come first and always take the payload
	if (sp == 22 || dp == 22)
	{
		const uint32_t o = sp == 22 ? dp : sp;
		if (o != 5060 && o != 5061 && o != 179)
			return known | kL7Ssh;
	}
	// MySQL (TcpLayer.cpp:469-478): MySqlLayer's factory never fails (MySqlLayer.cpp:462-470), so port 3306 on either
	// side builds it whenever the other port gates no dissector ahead of it (GTPv2 2123 and Modbus 502 come after it)
	if (sp == 3306 || dp == 3306)
	{
		const uint32_t o = sp == 3306 ? dp : sp;
		if (o == 3306 || o == 2123 || o == 502 || !port_bit(kL7.tcp_other, o))
			return known | kL7MySql;
	}
	// SIP / BGP / SSH (TcpLayer.cpp:387-410) come before DNS over TCP (14 bytes, DnsLayer.h:481-485) and take the
	// payload; nothing after DNS builds an HTTP, DNS or SSL layer
	const bool sbs = sp == 5060 || sp == 5061 || sp == 179 || sp == 22 || dp == 5060 || dp == 5061 || dp == 179 || dp == 22;
	return known | ((!sbs && n >= 14 && (dns_port(sp) || dns_port(dp))) ? PCPPX_F_L7_DNS : 0u);
}

// ---- the layers of a classified first L7 layer, built on the device (restated in oracle/pcppx_oracle.c:
// l7_layers): with no parse-until family, an HTTP / SSL / DNS class names the layer the reference builds, and its
// rules are short length walks. Each layer's data runs to the end of the L4 payload (no effect on the trailer). ----
constexpr uint32_t P_HTTP_REQ = 6, P_HTTP_RESP = 7, P_DNS = 13, P_SSL = 18, P_SSH = 35, P_MYSQL = 63;
constexpr uint32_t kL7Built = PCPPX_F_L7_HTTP | PCPPX_F_L7_SSL | PCPPX_F_L7_DNS | kL7MySql | kL7Ssh;

__device__ __forceinline__ uint32_t zero_bytes(uint32_t v)
{
	return (v - 0x01010101u) & ~v & 0x80808080u;  // the lowest flagged byte is the first zero byte
}
// payload bytes [j, j + 4G) at o as G dwords: from LDS where the window holds them, else as G dword loads issued
// together (one memory round trip per 4G bytes of an HTTP header walk instead of one per dword); bytes at or past n read
// as 0x01 (neither '\n', ' ' nor NUL). G: 2 in the checksum instance (its stream windows are live across the walk), 4 in
// the parse-only ones.
template <int G>
__device__ __forceinline__ void text_group(const Pkt& p, uint32_t o, uint32_t j, uint32_t n, uint32_t (&w)[G])
{
	if (o + j >= p.lim && j + 4 * G <= n)
	{
#pragma unroll
		for (int k = 0; k < G; ++k)
			w[k] = ldu32(p, o + j + 4 * k);
		return;
	}
#pragma unroll
	for (int k = 0; k < G; ++k)
	{
		const uint32_t jj = j + 4 * k;
		if (jj + 4 <= n)
			w[k] = o + jj + 4 <= p.lim ? lds_u32(p, o + jj) : ldu32(p, o + jj);
		else
		{
			uint32_t v = 0x01010101u;
			for (uint32_t b = 0; jj + b < n; ++b)
				v = (v & ~(0xFFu << (8 * b))) | (rb(p, o + jj + b) << (8 * b));
			w[k] = v;
		}
	}
}
// the first byte equal to c in payload bytes [a, n) of the payload at o (n if none)
template <int G>
__device__ __forceinline__ uint32_t find_byte(const Pkt& p, uint32_t o, uint32_t a, uint32_t n, uint32_t c)
{
	const uint32_t cc = c * 0x01010101u;
	for (uint32_t j = a; j < n; j += 4 * G)
	{
		uint32_t w[G];
		text_group<G>(p, o, j, n, w);
#pragma unroll
		for (int k = 0; k < G; ++k)
		{
			const uint32_t m = zero_bytes(w[k] ^ cc);
			if (m)
			{
				const uint32_t e = j + 4 * k + (__builtin_ctz(m) >> 3);
				return e < n ? e : n;
			}
		}
	}
	return n;
}
// the first '\n' in payload bytes [a, n) of the payload at o (n if none), 4G bytes per step; *nul: the first NUL before it;
// *first: the byte at a (a < n; from the first group read, so a caller needs no read of its own)
template <int G>
__device__ uint32_t scan_nl(const Pkt& p, uint32_t o, uint32_t a, uint32_t n, uint32_t* nul, uint32_t* first = nullptr)
{
	uint32_t z = n;
	for (uint32_t j = a; j < n; j += 4 * G)
	{
		uint32_t w[G];
		text_group<G>(p, o, j, n, w);
		if (first != nullptr && j == a)
			*first = w[0] & 0xFFu;
#pragma unroll
		for (int k = 0; k < G; ++k)
		{
			const uint32_t zl = zero_bytes(w[k] ^ 0x0A0A0A0Au), z0 = zero_bytes(w[k]);
			if (z == n && z0)
				z = j + 4 * k + (__builtin_ctz(z0) >> 3);
			if (zl)
			{
				const uint32_t e = j + 4 * k + (__builtin_ctz(zl) >> 3);
				*nul = z < e ? z : n;
				return e;
			}
		}
	}
	*nul = z;
	return n;
}
// HeaderField size (TextBasedProtocol.cpp:448-461): through the first '\n', else strnlen to the end
// (*first: the field's first byte, when the field is not empty)
template <int G>
__device__ __forceinline__ uint32_t tbp_field(const Pkt& p, uint32_t o, uint32_t a, uint32_t n, uint32_t* first)
{
	uint32_t nul;
	const uint32_t e = scan_nl<G>(p, o, a, n, &nul, first);
	return e < n ? e - a + 1 : nul - a;
}
// TextBasedProtocolMessage::parseFields + getHeaderLen (TextBasedProtocol.cpp:87-139,436-439)
template <int G>
__device__ uint32_t tbp_header_len(const Pkt& p, uint32_t o, uint32_t fl, uint32_t n)
{
	uint32_t c = 0;
	uint32_t off = fl, s = tbp_field<G>(p, o, off, n, &c);
	bool end = s == 0 || c == '\r' || c == '\n';
	while (!end && off + s < n)
	{
		const uint32_t s2 = tbp_field<G>(p, o, off + s, n, &c);
		if (s2 == 0)
			break;
		off += s;
		s = s2;
		end = c == '\r' || c == '\n';  // the new field's first byte
	}
	return off + s;
}
// HttpRequestFirstLine's end (HttpLayer.cpp:166-213, parseVersion :287-320): the first " HTTP/" after the method's
// space; with room for "x.y" the line ends after the next '\n', else (or with no version) at the end
template <int G>
__device__ uint32_t http_request_line(const Pkt& p, uint32_t o, uint32_t n)
{
	uint32_t sp = 0;
	while (rb(p, o + sp) != ' ')  // exists, < 8 (http_request)
		++sp;
	for (uint32_t v = sp + 1; v + 6 <= n; ++v)
	{
		v = find_byte<G>(p, o, v, n, ' ');  // the next space (4G bytes per step), then " HTTP/" at it
		if (v + 6 > n)
			break;
		if (rd32(p, o + v + 1) != 0x50545448u || rb(p, o + v + 5) != '/')  // "HTTP" as a little-endian dword
			continue;
		if (v + 9 > n)
			return n;
		uint32_t nul;
		const uint32_t e = scan_nl<G>(p, o, v + 6, n, &nul);
		return e < n ? e + 1 : n;
	}
	return n;
}
// a member of the parse-until family (ProtocolTypeFamily: up to four protocol bytes)
__device__ __forceinline__ bool family_has(uint32_t family, uint32_t proto)
{
	return family != 0 && (proto == (family & 0xFF) || (proto << 8) == (family & 0xFF00) ||
	                       (proto << 16) == (family & 0xFF0000) || (proto << 24) == (family & 0xFF000000u));
}
// The layers of a classified L7 payload at [o, o+n) (HTTP: HttpRequestLayer / HttpResponseLayer + a Payload body,
// HttpLayer.cpp:62-68,666-672,897-920; SSL: one SSLLayer per record, SSLLayer.cpp:88-106; DNS: DnsLayer, header =
// data, DnsLayer.h:353-372; MySQL: MySqlLayer, header = data, MySqlLayer.h:362-379; SSH: one message per layer,
// SSHLayer.cpp:18-40,46-56,135-170), appended at index `count`, each kept only if it passes the stop rules
// (Packet.cpp:134-155; the first that fails is rolled back and ends the chain); stops counting once past cap_layers
// (every further layer is another SSL record / SSH message: same mask, same DEPTH_OVERFLOW).
template <int G>
__device__ uint32_t l7_build(const Pkt& p, uint32_t lf, uint32_t o, uint32_t n, uint32_t dp, uint32_t count, uint32_t ml,
                             uint32_t cap_layers, uint32_t family, uint32_t until_osi, uint32_t& found,
                             uint32_t& stopped, uint64_t& mask, uint2* lay_out)
{
	auto emit = [&](uint32_t proto, uint32_t osi, uint32_t lo, uint32_t hdr, uint32_t dlen) -> bool {
		const bool member = family_has(family, proto);
		const bool osi_fail = osi > until_osi;
		found = (!osi_fail && member) ? 1u : found;
		if (osi_fail || (found && !member))
		{
			stopped = 1;
			return false;
		}
		if (lay_out && count < ml)
			lay_out[count] = make_uint2(proto | (osi << 8) | (lo << 16), (hdr & 0xFFFF) | (dlen << 16));
		mask |= 1ull << proto;
		++count;
		return true;
	};
	if (lf & PCPPX_F_L7_HTTP)
	{
		const bool req = http_port(dp) && http_request(p, o, n);  // l7_flags' order
		uint32_t fl;
		if (req)
			fl = http_request_line<G>(p, o, n);
		else
		{
			uint32_t nul;
			const uint32_t e = scan_nl<G>(p, o, 0, n, &nul);
			fl = e < n ? e + 1 : n;
		}
		const uint32_t h = tbp_header_len<G>(p, o, fl, n);
		if (emit(req ? P_HTTP_REQ : P_HTTP_RESP, 7, o, h, n) && n > h)
			emit(P_PAYLOAD, 7, o + h, n - h, n - h);
	}
	else if (lf & PCPPX_F_L7_SSL)
	{
		uint32_t ro = o, rem = n;
		for (;;)
		{
			uint32_t hl = 5 + ((rb(p, ro + 3) << 8) | rb(p, ro + 4));
			hl = hl < rem ? hl : rem;
			if (!emit(P_SSL, 6, ro, hl, rem) || rem <= hl || count > cap_layers || !ssl_record(p, ro + hl, rem - hl))
				break;
			ro += hl;
			rem -= hl;
		}
	}
	else if (lf & kL7MySql)
		emit(P_MYSQL, 7, o, n, n);
	else if (lf & kL7Ssh)
	{
		// createSSHMessage: an identification message ("SSH-" ... '\n': the rest), else a handshake message (packet
		// length + 4 within the data, padding <= packet length, a known message code: packet length + 4), else an
		// encrypted message (the rest); each message's next one follows it (SSHLayer::parseNextLayer)
		uint32_t ro = o, rem = n;
		for (;;)
		{
			uint32_t hl = rem;
			const bool ident = rem >= 5 && rb(p, ro) == 'S' && rb(p, ro + 1) == 'S' && rb(p, ro + 2) == 'H' &&
			                   rb(p, ro + 3) == '-' && rb(p, ro + rem - 1) == '\n';
			if (!ident && rem >= 6)
			{
				const uint32_t ml4 = (rb(p, ro) << 24) | (rb(p, ro + 1) << 16) | (rb(p, ro + 2) << 8) | rb(p, ro + 3);
				const uint32_t pad = rb(p, ro + 4), code = rb(p, ro + 5);
				if ((uint64_t)ml4 + 4 <= rem && pad <= ml4 && (code == 20 || code == 21 || (code >= 30 && code <= 49)))
					hl = ml4 + 4;
			}
			if (!emit(P_SSH, 7, ro, hl, rem) || rem <= hl || count > cap_layers)
				break;
			ro += hl;
			rem -= hl;
		}
	}
	else
		emit(P_DNS, 7, o, n, n);
	return count;
}

// Smallest OSI layer among the layers the host would build on an L4 payload the port / SIP triggers hand to
// a dissector (each Layer::getOsiModelLayer override; the table is in oracle/pcppx_oracle.c,
// tcp_l7_min_osi / udp_l7_min_osi): the parse-until stop rules roll that layer back when it lies above
// parseUntilLayer (Packet.cpp:134-140,168-175).
__device__ __forceinline__ uint32_t l7_min_osi(bool tcp, uint32_t sp, uint32_t dp, bool sip)
{
	const bool e102 = sp == 102 || dp == 102, e2123 = sp == 2123 || dp == 2123;
	const bool esip = sp == 5060 || sp == 5061 || dp == 5060 || dp == 5061;
	const uint32_t t = (e102 || e2123) ? 4u : (esip ? 5u : 7u);
	if (tcp)
	{
		// SSL ports (SSLLayer.h:488-510) give the presentation layer 6
		const bool ssl_s = sp == 443 || sp == 261 || sp == 448 || sp == 465 || sp == 563 || sp == 614 || sp == 636 ||
		                   sp == 989 || sp == 990 || (sp >= 992 && sp <= 995);
		const bool ssl_d = dp == 443 || dp == 261 || dp == 448 || dp == 465 || dp == 563 || dp == 614 || dp == 636 ||
		                   dp == 989 || dp == 990 || (dp >= 992 && dp <= 995);
		return t == 7u && (ssl_s || ssl_d) ? 6u : t;
	}
	uint32_t u = (esip || sip) ? 5u : 7u;
	u = (sp == 2152 || dp == 2152 || e2123) ? 4u : u;
	u = (sp == 51820 || dp == 51820) ? 3u : u;
	u = (dp == 4789 || dp == 0 || dp == 7 || dp == 9) ? 2u : u;
	return u;
}

__device__ __forceinline__ uint32_t fnv(uint32_t h, uint32_t b)
{
	return (h * 16777619u) ^ b;
}

// fold a u32 sum of 16-bit halves to its residue mod 65535 (0..65534)
__device__ __forceinline__ uint32_t mod65535(uint32_t x)
{
	x = (x & 0xFFFF) + (x >> 16);
	x = (x & 0xFFFF) + (x >> 16);
	return x == 0xFFFF ? 0 : x;
}

// v_sad_u16 against 0: |lo - 0| + |hi - 0| + acc, the sum of the two 16-bit halves in one instruction
__device__ __forceinline__ uint32_t halves(uint32_t v, uint32_t acc = 0)
{
	return __builtin_amdgcn_sad_u16(v, 0u, acc);
}

__device__ __forceinline__ uint32_t mask_dword(uint32_t v, uintptr_t b, uintptr_t lo, uintptr_t hi)
{
	// keep bytes of the dword at address b that fall in [lo, hi)
	int64_t s = (int64_t)lo - (int64_t)b, e = (int64_t)hi - (int64_t)b;
	s = s < 0 ? 0 : (s > 4 ? 4 : s);
	e = e < 0 ? 0 : (e > 4 ? 4 : e);
	if (e <= s)
		return 0;
	uint64_t m = ((1ull << (8 * e)) - 1) & ~((1ull << (8 * s)) - 1);
	return v & (uint32_t)m;
}

__device__ __forceinline__ uint32_t chunk_sum(uint4 v, uintptr_t c, uintptr_t lo, uintptr_t hi)
{
	if (c < lo || c + 16 > hi)
	{
		v.x = mask_dword(v.x, c, lo, hi);
		v.y = mask_dword(v.y, c + 4, lo, hi);
		v.z = mask_dword(v.z, c + 8, lo, hi);
		v.w = mask_dword(v.w, c + 12, lo, hi);
	}
	return halves(v.x) + halves(v.y) + halves(v.z) + halves(v.w);
}

// Residue mod 65535 of the little-endian 16-bit word sum of packet bytes [lo, hi) taken as a stream
// starting at lo (odd last byte zero-padded), i.e. computeChecksum's localSum before folding.
__device__ uint32_t range_residue(const Pkt& p, uint32_t lo, uint32_t hi)
{
	if (hi <= lo)
		return 0;
	const uintptr_t alo = (uintptr_t)p.g + lo, ahi = (uintptr_t)p.g + hi;
	uintptr_t c = alo & ~(uintptr_t)15;
	uint32_t acc = 0;
	// chunks still in the LDS window
	for (; c < ahi; c += 16)
	{
		uint32_t ci = (uint32_t)((c - p.a0) >> 4);
		if (ci >= p.nch || (p.a0 & 15) != 0)  // a re-gathered deep window starts at a dword: not memory chunks
			break;
		lptr32 w = reinterpret_cast<lptr32>(p.s) + ci * 4;
		uint4 v = make_uint4(w[0], w[1], w[2], w[3]);
		acc += chunk_sum(v, c, alo, ahi);
	}
	// the rest straight from HBM, 64 B per iteration
	for (; c + 64 <= ahi; c += 64)
	{
		uint4 v0 = ld16(c), v1 = ld16(c + 16), v2 = ld16(c + 32), v3 = ld16(c + 48);
		acc += chunk_sum(v0, c, alo, ahi) + chunk_sum(v1, c + 16, alo, ahi) + chunk_sum(v2, c + 32, alo, ahi) +
		       chunk_sum(v3, c + 48, alo, ahi);
	}
	for (; c < ahi; c += 16)
	{
		uint4 v = ld16(c);
		acc += chunk_sum(v, c, alo, ahi);
	}
	uint32_t r = mod65535(acc);
	if (alo & 1)
		r = (r * 256u) % 65535u;  // the stream's words are the memory words byte-swapped
	return r;
}

// computeChecksum's final step over a total whose true sum is known to be non-zero:
// fold -> [1, 0xFFFF] (0xFFFF iff residue 0), invert, htobe16
__device__ __forceinline__ uint32_t finish_checksum(uint32_t residue)
{
	uint32_t folded = residue == 0 ? 0xFFFFu : residue;
	uint32_t result = (~folded) & 0xFFFFu;
	return ((result >> 8) | (result << 8)) & 0xFFFFu;
}

// The first 16 bytes of a layer at [o, o+len), as four little-endian dwords: from the LDS window where
// staged, else byte by byte (HBM); bytes at or past caplen read as 0 and are never used (every field a
// layer reads lies inside its own length once the length checks below have passed).
struct Peek
{
	uint32_t q[4];
	__device__ __forceinline__ uint32_t b(uint32_t j) const { return (q[j >> 2] >> (8 * (j & 3))) & 0xFF; }
	__device__ __forceinline__ uint32_t be(uint32_t j) const { return (b(j) << 8) | b(j + 1); }
};

__device__ __forceinline__ Peek peek16(const Pkt& p, uint32_t o, uint32_t cap)
{
	Peek k;
	// the LDS window read runs for every lane (a lane past the window reads its slot's first bytes and
	// replaces them below): one divergent region, entered only when some lane is past the window
	const bool inwin = o + 16 <= p.lim;
	{
		const uint32_t pos = p.mis + (inwin ? o : 0u);
		lptr32 w = reinterpret_cast<lptr32>(p.s) + (pos >> 2);
		const uint32_t w0 = w[0], w1 = w[1], w2 = w[2], w3 = w[3], w4 = w[4];
		k.q[0] = __builtin_amdgcn_alignbyte(w1, w0, pos & 3);
		k.q[1] = __builtin_amdgcn_alignbyte(w2, w1, pos & 3);
		k.q[2] = __builtin_amdgcn_alignbyte(w3, w2, pos & 3);
		k.q[3] = __builtin_amdgcn_alignbyte(w4, w3, pos & 3);
	}
	if (!inwin)
	{
		// past the LDS window: the (at most two) aligned 16-B chunks holding [o, o+16) straight from HBM;
		// the second only if it starts inside the packet (bytes past caplen are never used)
		const uintptr_t a = (uintptr_t)p.g + o, base = a & ~(uintptr_t)15;
		const uint4 c0 = ld16(base);
		// the second chunk only matters if it starts inside the packet; otherwise re-read the first (the
		// address is selected, not the loaded value, so no branch)
		const uint4 c1 = ld16(base + 16 < (uintptr_t)p.g + cap ? base + 16 : base);
		const uint32_t d[8] = { c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w };
		const uint32_t sw = (uint32_t)(a >> 2) & 3, sb = (uint32_t)a & 3;
		// e[t] = d[sw + t] as and/or with constant masks: a select whose operand is a load is turned into
		// a branch by the compiler (to load conditionally), with its own exec-mask region
		const uint32_t m0 = sw == 0 ? ~0u : 0u, m1 = sw == 1 ? ~0u : 0u, m2 = sw == 2 ? ~0u : 0u,
		               m3 = sw == 3 ? ~0u : 0u;
		uint32_t e[5];
#pragma unroll
		for (int t = 0; t < 5; ++t)
			e[t] = (d[t] & m0) | (d[t + 1] & m1) | (d[t + 2] & m2) | (t + 3 < 8 ? (d[t + 3] & m3) : 0u);
#pragma unroll
		for (int t = 0; t < 4; ++t)
			k.q[t] = __builtin_amdgcn_alignbyte(e[t + 1], e[t], sb);
	}
	return k;
}

// Resolve a candidate kind from its own first bytes: the isDataValid of IPv4Layer (IPv4Layer.h:626-630),
// IPv6Layer (IPv6Layer.h:245-249), TcpLayer (TcpLayer.h:596-601), IPLayer::getIPVersion
// (IPLayer.cpp:5-25), GreLayer::getGREVersion (GreLayer.cpp:23-36, GreLayer.h:247-250,317-320),
// EthLayer / EthDot3Layer (EthLayer.cpp:100-117, EthDot3Layer.cpp:38-54) and LLCLayer (LLCLayer.cpp:49-52).
// Selects only: every lane of the wave evaluates every rule (no divergent branches).
__device__ __forceinline__ uint32_t resolve(uint32_t k, const Peek& q, uint32_t len)
{
	const uint32_t b0 = q.b(0), ver = b0 >> 4;
	k = k == C_IPVER ? (ver == 4 ? C_IPV4 : (ver == 6 ? C_IPV6 : K_PAYLOAD)) : k;
	// GtpV1Layer::parseNextLayer's sub-protocol byte (GtpLayer.cpp:585-599): 0x45-0x4e IPv4, 0x6_ IPv6
	k = k == C_IPGTP ? ((b0 >= 0x45 && b0 <= 0x4e) ? C_IPV4 : (ver == 6 ? C_IPV6 : K_PAYLOAD)) : k;
	const bool ok4 = len >= 20 && ver == 4 && (b0 & 0xF) >= 5;
	const bool ok6 = len >= 40 && ver == 6;
	const uint32_t d = q.b(12) >> 4;
	const bool okt = len >= 20 && d >= 5 && len >= 4 * d;
	const uint32_t gv = len < 4 ? 0xFF : (q.b(1) & 7);
	const uint32_t kg = gv == 0 ? K_GRE0 : ((gv == 1 && len >= 8) ? K_GRE1 : K_PAYLOAD);
	const uint32_t et = q.be(12);
	const uint32_t ke = len < 14 ? K_PAYLOAD : (et >= 0x0600 ? K_ETH : (et <= 0x05DC ? K_DOT3 : K_PAYLOAD));
	const bool okl = len >= 3 && !(b0 == 0xFF && q.b(1) == 0xFF);
	// IcmpLayer::isDataValid (IcmpLayer.h:619-660): the message type's struct fits; other types are no ICMP
	uint32_t need = 0xFFFFu;
	need = (b0 == 8 || b0 == 0 || b0 == 10 || b0 == 15 || b0 == 16) ? 4u : need;
	need = (b0 == 13 || b0 == 14) ? 20u : need;
	need = (b0 == 17 || b0 == 18) ? 12u : need;
	need = (b0 == 3 || b0 == 4 || b0 == 5 || b0 == 9 || b0 == 11 || b0 == 12) ? 8u : need;
	k = k == C_IPV4 ? (ok4 ? K_IPV4 : K_PAYLOAD) : k;
	k = k == C_IPV6 ? (ok6 ? K_IPV6 : K_PAYLOAD) : k;
	k = k == C_TCP ? (okt ? K_TCP : K_PAYLOAD) : k;
	k = k == C_GRE ? kg : k;
	k = k == C_ETHG ? ke : k;
	k = k == C_LLC ? (okl ? K_LLC : K_PAYLOAD) : k;
	k = k == C_ICMP ? (len >= need ? K_ICMP : K_PAYLOAD) : k;
	k = k == C_ETH ? ((len >= 14 && et >= 0x0600) ? K_ETH : K_PAYLOAD) : k;  // VXLAN: Ethernet, else Payload
	return k;
}

// The layer of (resolved) kind k at [o, o+len) and its successor, as Layer::parseNextLayer computes it:
//   EthLayer.cpp:28-69, EthDot3Layer.cpp:22-30, LLCLayer.cpp:24-41, VlanLayer.cpp:59-119,
//   MplsLayer.cpp:101-128, IPv4Layer.cpp:180-197,245-370, IPv6Layer.cpp:28-40,79-147,194-312,
//   GreLayer.cpp:195-252,547-566, TcpLayer.cpp:360-492, UdpLayer.cpp:92-184, ArpLayer.h:151-155,
//   PayloadLayer.h:61-81.
// Outputs: the layer (proto, osi, hdr, dlen) and the next kind nk at [po, po+pl) (possibly a candidate).
// Written as selects over the 16-byte peek: the wave's lanes sit on different layer kinds, and a switch
// would run every kind's branch with its own exec mask plus the scalar mask bookkeeping.
struct Step
{
	uint32_t proto, osi, hdr, dlen, nk, po, pl;
	bool l7done;  // a TCP/UDP payload whose next layer this step decided (a tunnel): no L7 decision after the walk
};

// GtpV1Layer::getHeaderLen (GtpLayer.cpp:602-632): 8 B; GTP-C adds its message length (at most the data); a
// G-PDU with any of the E / S / PN flags adds gtpv1_header_extra (4 B) and, with E, the extension chain
// (GtpExtension, :60-120,323-350: 4 * length byte, at most the rest; the next type is its last byte)
__device__ uint32_t gtp1_header_len(const Pkt& p, uint32_t o, uint32_t len, const Peek& q)
{
	const uint32_t fl = q.b(0);
	if (q.b(1) != 0xFF)
	{
		const uint32_t ml = q.be(2);
		return 8 + (ml > len - 8 ? len - 8 : ml);
	}
	if (len < 12 || !(fl & 7))
		return 8;
	uint32_t res = 12, nt = q.b(11);
	if (!(fl & 4) || nt == 0 || len <= 12)
		return res;
	uint32_t ed = 12, erem = len - 12;
	for (;;)
	{
		uint32_t tl = 4 * rb(p, o + ed);
		tl = tl <= erem ? tl : erem;
		res += tl;
		nt = tl >= 4 ? rb(p, o + ed + tl - 1) : 0u;
		if (nt == 0 || erem <= tl + 1)
			break;
		ed += tl;
		erem -= tl;
	}
	return res;
}

// NflogLayer (NflogLayer.cpp:41-96) at [o, o+len), len >= 4: the TLV records after the 4-byte nflog_header, {u16 length,
// u16 type} in host (little-endian) order, each align<4>(length) long, walked as TLVRecordReader walks them (TLVData.h:
// 238-312: a record needs >= 2 bytes left, a non-zero aligned length, and must fit). Returns getHeaderLen (the header +
// every record before the NFULA_PAYLOAD record + that record's 4-byte head); *pl: the payload record's aligned length
// - 4, or ~0u when there is no payload record.
__device__ uint32_t nflog_header_len(const Pkt& p, uint32_t o, uint32_t len, uint32_t* pl)
{
	const uint32_t tl = len - 4;
	uint32_t hdr = 4, pos = 0, total = tl >= 2 ? (rd16(p, o + 4) + 3u) & ~3u : 0u;
	bool have = total != 0 && total <= tl;
	*pl = ~0u;
	while (have)
	{
		if (rd16(p, o + 4 + pos + 2) == 9u)  // NFULA_PAYLOAD
		{
			*pl = total - 4;
			return hdr + 4;
		}
		hdr += total;
		pos += total;
		if (tl - pos < 2)
			break;
		total = (rd16(p, o + 4 + pos) + 3u) & ~3u;
		have = total != 0 && pos + total <= tl;
	}
	return hdr;
}

// The Cisco HDLC / NFLOG first layer of a packet of `cap` bytes (kind K_HDLC / K_NFLOG): CiscoHdlcLayer.cpp:43-67 (a
// 4-byte header, then IPv4 / IPv6 by its protocol field, else a Payload -- no length check, so a 4-byte packet gets an
// empty one) and NflogLayer.cpp:41-96 (nflog_header_len; a next layer iff the data runs past the 4-byte header and a
// payload record exists, of that record's length; IPv4 / IPv6 by the address family byte, 2 / 10, else a Payload).
// walk_chain builds these ahead of its loop, so their rules add nothing to the loop of the other link types.
__device__ Step first_layer_step(const Pkt& p, uint32_t k, uint32_t cap)
{
	const bool hd = k == K_HDLC;
	uint32_t pl = ~0u;
	const uint32_t hdr = hd ? 4u : nflog_header_len(p, 0, cap, &pl);
	const bool has_next = hd ? true : (cap > 4 && pl != ~0u);
	const uint32_t sel = hd ? rd16(p, 2) : rb(p, 0);
	const uint32_t v = hd ? swap16(sel) : sel;
	uint32_t nk = K_PAYLOAD;
	nk = (hd ? v == 0x0800 : v == 2) ? C_IPV4 : nk;
	nk = (hd ? v == 0x86DD : v == 10) ? C_IPV6 : nk;
	pl = hd ? cap - 4 : pl;
	return Step{ hd ? P_CISCO_HDLC : P_NFLOG, 2u, hdr, cap, has_next ? nk : (uint32_t)K_NONE, has_next ? hdr : 0u,
	             has_next ? pl : 0u, false };
}

// per-kind ProtocolType (6 bits) and OsiModelLayer (3 bits); kinds without a layer map to Payload / 7
constexpr uint32_t kind_proto(uint32_t k)
{
	return k == K_ETH ? P_ETH : k == K_DOT3 ? P_DOT3 : k == K_LLC ? P_LLC : k == K_VLAN ? P_VLAN : k == K_MPLS ? P_MPLS
	     : k == K_IPV4 ? P_IPV4 : k == K_IPV6 ? P_IPV6 : k == K_GRE0 ? P_GREV0 : k == K_GRE1 ? P_GREV1
	     : k == K_PPTP ? P_PPTP : k == K_TCP ? P_TCP : k == K_UDP ? P_UDP : k == K_ARP ? P_ARP : k == K_SLL ? P_SLL
	     : k == K_SLL2 ? P_SLL2 : k == K_NULL ? P_NULL : k == K_ICMP ? P_ICMP : P_PAYLOAD;
}
constexpr uint32_t kind_osi(uint32_t k)
{
	return (k == K_ETH || k == K_DOT3 || k == K_LLC || k == K_VLAN || k == K_SLL || k == K_SLL2 || k == K_NULL) ? 2
	     : (k == K_MPLS || k == K_IPV4 || k == K_IPV6 || k == K_GRE0 || k == K_GRE1 || k == K_ARP || k == K_ICMP) ? 3
	     : k == K_PPTP ? 5 : (k == K_TCP || k == K_UDP) ? 4 : 7;
}
constexpr uint64_t pack_proto(uint32_t first)
{
	uint64_t t = 0;
	for (uint32_t k = first; k < first + 10 && k <= K_ICMP; ++k)
		t |= (uint64_t)kind_proto(k) << (6 * (k - first));
	return t;
}
constexpr uint64_t pack_osi()
{
	uint64_t t = 0;
	for (uint32_t k = 0; k <= K_ICMP; ++k)
		t |= (uint64_t)kind_osi(k) << (3 * k);
	return t;
}
constexpr uint64_t kProtoLo = pack_proto(0), kProtoHi = pack_proto(10), kOsi = pack_osi();
static_assert(K_ICMP < 20 && 3 * K_ICMP + 3 <= 64 && P_SLL2 < 64, "kind tables");

__device__ __forceinline__ Step step_layer(const Pkt& p, uint32_t k, uint32_t o, uint32_t len, const Peek& q)
{
	const bool isE = k == K_ETH, isD = k == K_DOT3, isL = k == K_LLC, isV = k == K_VLAN, isM = k == K_MPLS;
	const bool is4 = k == K_IPV4, is6 = k == K_IPV6, isG = k == K_GRE0 || k == K_GRE1, isP = k == K_PPTP;
	const bool isT = k == K_TCP, isU = k == K_UDP, isA = k == K_ARP;
	const bool isS = k == K_SLL, isS2 = k == K_SLL2, isN = k == K_NULL, isI = k == K_ICMP;
	// IPv6 extension headers (IPv6Layer::parseExtensions, no bound check against dataLen): IPv6 lanes only
	uint32_t nh = q.b(6), ext = 0, last_ext = 0xFFFF;
	if (is6)
	{
		uint32_t eo = 40;
		while (eo <= len - 2)
		{
			// extension next-header values 0, 43, 44, 51 (AH), 60 as one 64-bit set (a compare chain becomes a
			// branch tree)
			constexpr uint64_t kExt = (1ull << 0) | (1ull << 43) | (1ull << 44) | (1ull << 51) | (1ull << 60);
			const bool ah = nh == 51;
			if (nh >= 64 || !((kExt >> nh) & 1ull))
				break;
			// the extension's next-header and length bytes: LDS window read for every lane, HBM only past it
			const uint32_t j = o + eo;
			const bool win = j + 2 <= p.lim;
			uint32_t two = lds_u32(p, win ? j : 0u) & 0xFFFFu;
			if (!win)
				two = le16(p, j);
			const uint32_t hl = two >> 8;
			const uint32_t el = ah ? 4u * (hl + 2) : 8u * (hl + 1);
			last_ext = nh;
			nh = two & 0xFFu;
			eo += el;
			ext += el;
		}
	}
	// protocol / OSI layer (ProtocolType.h) of kind k, read from per-kind tables packed into 64-bit
	// constants (two shifts instead of a select chain over every kind)
	const uint32_t kt = k < 20 ? k : 0u;  // the packed tables hold kinds 0-19; VXLAN / GTPv1 are set below
	const bool isVx = k == K_VXLAN, isG1 = k == K_GTP1;
	uint32_t proto = (uint32_t)((kt < 10 ? (kProtoLo >> (6 * kt)) : (kProtoHi >> (6 * (kt - 10)))) & 63u);
	uint32_t osi = (uint32_t)((kOsi >> (3 * kt)) & 7u);
	proto = isVx ? P_VXLAN : (isG1 ? P_GTPV1 : proto);
	osi = isVx ? 2u : (isG1 ? 4u : osi);  // VxlanLayer.h:141-144, GtpLayer.h:408-411
	// header length
	const uint32_t f0 = q.b(0), f1 = q.b(1);
	const uint32_t greh = 4 + ((f0 & 0xC0) ? 4 : 0) + ((f0 & 0x20) ? 4 : 0) + ((f0 & 0x10) ? 4 : 0) + ((f1 & 0x80) ? 4 : 0);
	uint32_t hdr = len;  // Payload: the whole remainder
	hdr = (isE || isD) ? 14 : hdr;
	hdr = isL ? 3 : hdr;
	hdr = (isV || isM || isP) ? 4 : hdr;
	hdr = is4 ? (f0 & 0xF) * 4 : hdr;
	hdr = is6 ? 40 + ext : hdr;
	hdr = isG ? greh : hdr;
	hdr = isT ? (q.b(12) >> 4) * 4 : hdr;
	hdr = isU ? 8 : hdr;
	hdr = isA ? 28 : hdr;
	hdr = isS ? 16 : hdr;   // sll_header (SllLayer.h:15-32), even when the packet is shorter
	hdr = isS2 ? 20 : hdr;  // sll2_header (Sll2Layer.h:15-35)
	hdr = isN ? 4 : hdr;    // the family dword (NullLoopbackLayer.h:66-69)
	// ICMP by message type (IcmpLayer::getHeaderLen, IcmpLayer.cpp:589-620): echo = the whole data; timestamp 20;
	// address mask 12; the error messages 8; router advertisement 8 + 8 per address, at most the data; else 4
	const uint32_t it = f0;
	const bool ierr = it == 3 || it == 4 || it == 5 || it == 11 || it == 12;
	uint32_t ih = (it == 0 || it == 8) ? len : 4u;
	ih = (it == 13 || it == 14) ? 20u : ih;
	ih = (it == 17 || it == 18) ? 12u : ih;
	ih = ierr ? 8u : ih;
	const uint32_t ra = 8 + 8 * q.b(4);
	ih = it == 9 ? (ra < len ? ra : len) : ih;
	hdr = isI ? ih : hdr;
	hdr = isVx ? 8 : hdr;  // vxlan_header (VxlanLayer.h:14-60)
	if (isG1)
		hdr = gtp1_header_len(p, o, len, q);
	// data length: IPv4 totalLength truncation (0 = TSO keeps it), IPv6 payloadLength + header, ARP 28
	uint32_t dlen = len;
	const uint32_t tl = q.be(2);
	const uint32_t hmin = hdr < len ? hdr : len;
	dlen = (is4 && tl < len && tl != 0) ? (tl > hmin ? tl : hmin) : dlen;
	const uint32_t total = q.be(4) + hdr;
	dlen = (is6 && total < len) ? total : dlen;
	dlen = isA ? 28 : dlen;
	// successor: exists iff the layer's data runs past its header (every kind's "no next layer" rule; Null/Loopback
	// always builds one, empty for a 4-byte packet: NullLoopbackLayer.cpp:50-99 has no length check)
	// (an ICMP error message always builds one, empty when the quote is: IcmpLayer.cpp:562-587)
	const bool has_next = (dlen > hdr || isN || (isI && ierr)) && !(isG1 && q.b(1) != 0xFF);  // GTP-C: last
	const uint32_t po = o + hdr, pl = has_next ? dlen - hdr : 0;
	// EtherType dispatch of Ethernet (EtherType at 12), VLAN and GRE (at 2), SLL (protocol_type at 14) and SLL2 (at
	// 0: SllLayer.cpp:49-102, Sll2Layer.cpp:63-121); PPP protocol of PPP_PPTP (at 2)
	const uint32_t et = isE ? q.be(12) : (isS ? q.be(14) : (isS2 ? q.be(0) : q.be(2)));
	uint32_t ne = K_PAYLOAD;
	ne = et == 0x0800 ? C_IPV4 : ne;
	ne = et == 0x86DD ? C_IPV6 : ne;
	ne = (et == 0x8100 || (et == 0x88A8 && !isG)) ? K_VLAN : ne;
	ne = et == 0x8847 ? K_MPLS : ne;
	ne = (et == 0x0806 && !isG) ? ((isE && pl < 28) ? K_PAYLOAD : K_ARP) : ne;
	ne = ((et == 0x8864 || et == 0x8863) && !isG) || (et == 0x0842 && isE) ? K_OUT : ne;
	ne = (et == 0x880B && isG) ? (pl >= 4 ? K_PPTP : K_PAYLOAD) : ne;
	ne = (et == 0x6558 && isG) ? C_ETHG : ne;
	ne = (et < 1500 && isV) ? C_LLC : ne;
	ne = (isE && pl < 4 && (ne == K_VLAN || ne == K_MPLS)) ? K_PAYLOAD : ne;
	ne = isP ? (et == 0x21 ? C_IPV4 : (et == 0x57 ? C_IPV6 : K_PAYLOAD)) : ne;
	ne = (isS2 && et == 0x0004) ? C_LLC : ne;  // Sll2ProtoTypeLLC (Sll2Layer.cpp:20,110-114)
	// Null/Loopback: NullLoopbackLayer::getFamily (NullLoopbackLayer.cpp:23-43: a byte-order guess; its BSWAP16 keeps
	// the shifted-out byte, :10) then an EtherType above 1500, else the BSD AF_INET / AF_INET6 values
	uint32_t fam = q.q[0];
	const uint32_t fsw = (fam >> 24) | ((fam & 0x00FF0000u) >> 8) | ((fam & 0x0000FF00u) << 8) | (fam << 24);
	const uint32_t f16 = fam & 0xFFFFu;
	fam = (fam & 0xFFFF0000u) ? (((fam & 0xFF000000u) == 0 && (fam & 0x00FF0000u) < 0x00060000u) ? fam >> 16 : fsw)
	                          : (((fam & 0xFFu) == 0 && (fam & 0xFF00u) < 0x0600u) ? ((f16 >> 8) | (f16 << 8)) : fam);
	const uint32_t fe = fam & 0xFFFFu;
	const bool nv4 = fam > 1500 ? fe == 0x0800 : fam == 2;
	const bool nv6 = fam > 1500 ? fe == 0x86DD : (fam == 24 || fam == 28 || fam == 30);
	const uint32_t nn = nv4 ? C_IPV4 : (nv6 ? C_IPV6 : K_PAYLOAD);
	// IP protocol / next-header dispatch (IPv4Layer.cpp:245-370, IPv6Layer.cpp:194-312)
	const uint32_t ipp = is4 ? q.b(9) : nh;
	uint32_t ni = K_PAYLOAD;
	ni = ipp == 17 ? (pl >= 8 ? K_UDP : K_PAYLOAD) : ni;
	ni = ipp == 6 ? C_TCP : ni;
	ni = ipp == 4 ? C_IPVER : ni;
	ni = ipp == 47 ? C_GRE : ni;
	ni = (ipp == 41 && is4) ? C_IPV6 : ni;
	ni = (ipp == 1 && is4) ? C_ICMP : ni;  // IPv4Layer.cpp:272-274
	ni = (ipp == 51 || ipp == 50 || ipp == 112 || (is4 && ipp == 2) || (!is4 && ipp == 58)) ? K_OUT : ni;
	const uint32_t b6 = q.b(6);
	const bool frag = (b6 & 0x20) || (((b6 & 0x1F) << 8) | q.b(7)) != 0;  // IPv4Layer.cpp:415-438
	ni = ((is4 && frag) || (is6 && last_ext == 44)) ? K_PAYLOAD : ni;
	uint32_t nk = K_PAYLOAD;
	nk = (isE || isV || isG || isP || isS || isS2) ? ne : nk;
	nk = isN ? nn : nk;
	nk = (is4 || is6) ? ni : nk;
	nk = isM ? ((q.b(2) & 1) ? C_IPVER : K_MPLS) : nk;  // bottom of stack: IPv4/IPv6 by version nibble
	nk = isD ? C_LLC : nk;
	nk = isL ? ((f0 == 0x42 && f1 == 0x42) ? K_OUT : K_PAYLOAD) : nk;
	nk = isI ? (ierr ? C_IPV4 : K_PAYLOAD) : nk;  // the quoted IPv4 header (tryConstruct), else a Payload
	// UDP tunnels, decided as UdpLayer::parseNextLayer does (:103-131): VXLAN by destination port (8 bytes,
	// VxlanLayer.h:97-100), GTPv1 by port and isGTPv1 (GtpLayer.cpp:199-207) where no earlier dissector takes the
	// payload: DHCP, DNS, SIP (port), RADIUS (port and RadiusLayer::isDataValid, RadiusLayer.cpp:238-247)
	const uint32_t usp = q.be(0), udp = q.be(2);
	const bool vx = isU && udp == 4789;
	const bool dhcp = (usp == 68 && udp == 67) || (usp == 67 && (udp == 68 || udp == 67));
	const bool dnsb = pl >= 12 && (dns_port(usp) || dns_port(udp));
	const bool sipp = usp == 5060 || usp == 5061 || udp == 5060 || udp == 5061;
	const bool radp = usp == 1812 || usp == 1813 || usp == 3799 || udp == 1812 || udp == 1813 || udp == 3799;
	const uint32_t rlen = q.be(10);  // the RADIUS length field (payload bytes 2-3)
	const bool rad = radp && pl >= 20 && rlen >= 20 && rlen <= pl;
	const bool gport = usp == 2152 || udp == 2152 || usp == 2123 || udp == 2123;
	const bool gtp = isU && gport && !vx && !dhcp && !dnsb && !sipp && !rad && pl >= 8 && (q.b(8) & 0xE0) == 0x20;
	nk = vx ? (pl >= 8 ? K_VXLAN : K_PAYLOAD) : nk;
	nk = gtp ? K_GTP1 : nk;
	nk = isVx ? C_ETH : nk;
	nk = isG1 ? C_IPGTP : nk;
	// TCP/UDP: a tentative Payload; walk_chain decides afterwards whether an L7 dissector takes it
	nk = has_next ? nk : K_NONE;
	return Step{ proto, osi, hdr, dlen, nk, has_next ? po : 0, pl, vx || gtp };
}

struct Params
{
	const uint8_t* data;
	const uint64_t* offsets;
	const uint32_t* caplens;
	uint64_t data_len;
	pcppx_summary* summary;
	pcppx_layer* layers;
	uint32_t* flow_keys;  // optional dense hash5 column
	uint32_t n;
	uint32_t family;
	uint32_t until_osi;
	uint32_t want_csum;
	uint32_t max_layers;
	uint32_t linktype;
	uint32_t fam_engine_only;  // family != 0 and every protocol of it is one the engine builds (host-computed)
	pcppx_reasm_info* reasm;  // fused reassembly front ends (pcppx_parse_batch_device_reasm), or null
	pcppx_tuple* tuples;      // optional 5-tuple extracts (pcppx_records.tuples)
	uint4* wave_stats;        // optional per-wave collectStats counters (16 x u8), reduced by proto_stats_reduce_kernel
	uint32_t packed;          // PCPPX_LAYOUT_PACKED: the chain's layer entries dense per 64-packet tile
	pcppx_brief* brief;       // optional 16-B brief (pcppx_records.brief): the summary's first half
};

// Everything the summary needs after the chain walk.
struct Walk
{
	uint32_t flags, n_layers;
	uint64_t mask;
	int32_t v4, v6;             // offsets of the first IPv4 / IPv6 layers (-1: none)
	uint32_t v4_dlen;
	int32_t l4i;                // hash5Tuple's port layer: last TCP, else last UDP (-1: none)
	uint32_t l4o, l4dlen, l4pp, l4ppo;  // its offset, dataLen, and the previous layer's proto/offset
	bool is_tcp;
};

// Packet::parsePacket (Packet.cpp:66-196): first layer by link type (createFirstLayer :827-923), the
// parseNextLayer chain with the parse-until stop rules (:123-175), and the trailer (:178-195).
// Layer records go straight to lay_out (uint2 per layer) when it is non-null.
template <int G = 2>
__device__ __forceinline__ Walk walk_chain(const Pkt& p, uint32_t cap, const Params& prm, uint2* lay_out)
{
	uint32_t flags = 0;
	uint32_t k;
	switch (prm.linktype)
	{
	case 1: k = C_ETHG; break;                    // Ethernet, else 802.3, else Payload
	case 101: case 12: case 14: k = C_IPVER; break;  // raw IP by version nibble
	case 228: k = C_IPV4; break;
	case 229: k = C_IPV6; break;
	case 113: k = K_SLL; break;                            // SllLayer: unchecked (Packet.cpp:849-852)
	case 276: k = cap >= 20 ? K_SLL2 : K_PAYLOAD; break;  // Sll2Layer::isDataValid (Sll2Layer.cpp:151-154)
	case 0: k = cap >= 4 ? K_NULL : K_PAYLOAD; break;     // NullLoopbackLayer::isDataValid (NullLoopbackLayer.h:86-89)
	case 239: k = cap >= 4 ? K_NFLOG : K_PAYLOAD; break;    // NflogLayer::isDataValid (NflogLayer.cpp:102-105)
	case 104: k = cap >= 4 ? K_HDLC : K_PAYLOAD; break;     // CiscoHdlcLayer::isDataValid (CiscoHdlcLayer.h:59-62)
	default: k = K_PAYLOAD; break;
	}

	const uint32_t ml = prm.max_layers;
	const uint32_t cap_layers = ml ? ml : PCPPX_MAX_LAYERS;
	uint32_t count = 0, found = 0, stopped = 0;
	uint64_t mask = 0;
	// loop-carried bookkeeping packed in 16-bit fields (offsets and lengths are < 2^16, counts < 2^8): fewer
	// live registers means fewer copies at the loop's joins
	uint32_t v4w = 0xFFFFu;    // first IPv4: offset | dataLen << 16 (offset 0xFFFF: none)
	uint32_t v6o = 0xFFFFu;    // first IPv6 offset (0xFFFF: none)
	uint32_t tcpA = 0, tcpB = 0, udpA = 0, udpB = 0;  // last TCP / UDP: index+1 | offset << 16,
	                                                 // dataLen | previous layer's offset << 16
	uint32_t pps = 0;          // previous layer's proto of the last TCP (bits 0-7) / UDP (8-15); bits 16-31: the
	                           // payload length of the last TCP/UDP layer (the L7 decision's input)
	uint32_t prev = 0;         // previous layer: proto | offset << 16
	uint32_t last_end = 0;
	uint32_t o = 0, len = cap;

	// Cisco HDLC / NFLOG (uniform on the link type): their first layer is built here, ahead of the loop. It is never
	// rolled back and is neither IP nor TCP/UDP, so of the loop's bookkeeping only the stop rules' state, the record,
	// the mask and the previous-layer fields apply.
	if (prm.linktype == 104 || prm.linktype == 239)
	{
		if (k == K_HDLC || k == K_NFLOG)
		{
			const Step s = first_layer_step(p, k, cap);
			const bool member = prm.family != 0 &&
			                    (s.proto == (prm.family & 0xFF) || (s.proto << 8) == (prm.family & 0xFF00) ||
			                     (s.proto << 16) == (prm.family & 0xFF0000) || (s.proto << 24) == (prm.family & 0xFF000000u));
			const bool osi_fail = s.osi > prm.until_osi;
			found = (!osi_fail && member) ? 1u : 0u;
			const bool fail = osi_fail || (found && !member);
			stopped = fail ? 1u : 0u;
			if (lay_out && ml)
				lay_out[0] = make_uint2(s.proto | (s.osi << 8), (s.hdr & 0xFFFF) | (s.dlen << 16));
			mask = 1ull << s.proto;
			prev = s.proto;
			last_end = s.dlen;
			count = 1;
			k = fail ? (uint32_t)K_NONE : s.nk; o = s.po; len = s.pl;
		}
	}

	// The loop body is written as selects around three divergent regions (the loop exits, the peek's HBM
	// fallback, the record store): the 64 lanes sit on different layer kinds, and every `if` becomes an
	// exec-mask region of scalar bookkeeping plus copies of each value live across it.
	while (k != K_NONE)
	{
		if (k == K_OUT)
		{
			// an out-of-scope layer: rolled back by the stop rules when every candidate fails one
			// (oracle/pcppx_oracle.c, family_engine_only): L2 candidates (PPPoE, WoL, STP) have OSI 2, the
			// IP-protocol ones (IGMP, AH, ESP, VRRP, ICMPv6) 3
			const uint32_t pp = prev & 0xFFu;
			const uint32_t kosi = (pp == P_IPV4 || pp == P_IPV6) ? 3u : 2u;
			if (!(count > 0 && (kosi > prm.until_osi || (found && prm.fam_engine_only))))
				flags |= PCPPX_F_NEEDS_HOST_PROTO;
			break;
		}
		const bool nob = k == K_PAYLOAD || k == K_ARP;  // reads no byte: peek at 0 (inside the packet), drop it
		Peek q = peek16(p, nob ? 0u : o, cap);
		const uint32_t keep = nob ? 0u : ~0u;  // a mask, not a select of the loaded value (see peek16)
#pragma unroll
		for (int t = 0; t < 4; ++t)
			q.q[t] &= keep;
		k = resolve(k, q, len);
		Step s = step_layer(p, k, o, len, q);
		uint32_t nk = s.nk;
		// stop rules (inclusive, then roll back one layer; the first layer is never rolled back)
		const uint32_t proto = s.proto;
		const bool member = prm.family != 0 &&
		                    (proto == (prm.family & 0xFF) || (proto << 8) == (prm.family & 0xFF00) ||
		                     (proto << 16) == (prm.family & 0xFF0000) || (proto << 24) == (prm.family & 0xFF000000u));
		const bool osi_fail = s.osi > prm.until_osi;
		found = (!osi_fail && member) ? 1u : found;
		const bool fail = osi_fail || (found && !member);
		stopped = fail ? 1u : stopped;
		if (fail && count > 0)
			break;
		nk = fail ? (uint32_t)K_NONE : nk;
		if (lay_out && count < ml)
			lay_out[count] = make_uint2(proto | (s.osi << 8) | (o << 16), (s.hdr & 0xFFFF) | (s.dlen << 16));
		mask |= 1ull << proto;
		v4w = (proto == P_IPV4 && v4w == 0xFFFFu) ? (o | (s.dlen << 16)) : v4w;
		v6o = (proto == P_IPV6 && v6o == 0xFFFFu) ? o : v6o;
		// the last TCP / UDP layer, as and/or with lane masks (a run of selects on one condition is
		// otherwise folded into a branch)
		const uint32_t mT = proto == P_TCP ? ~0u : 0u, mU = proto == P_UDP ? ~0u : 0u;
		const uint32_t a_new = (count + 1) | (o << 16);
		const uint32_t b_new = (s.dlen & 0xFFFFu) | (prev & 0xFFFF0000u);
		tcpA = (tcpA & ~mT) | (a_new & mT);
		tcpB = (tcpB & ~mT) | (b_new & mT);
		udpA = (udpA & ~mU) | (a_new & mU);
		udpB = (udpB & ~mU) | (b_new & mU);
		const uint32_t mP = (mT & 0xFFu) | (mU & 0xFF00u) | ((mT | mU) & 0xFFFF0000u);
		const uint32_t p_new = (prev & 0xFFu) * 0x101u | ((s.l7done ? 0u : s.pl) << 16);
		pps = (pps & ~mP) | (p_new & mP);
		prev = proto | (o << 16);
		last_end = o + s.dlen;
		++count;
		k = nk; o = s.po; len = s.pl;
	}

	// L7 dispatch of the last TCP/UDP layer's payload (TcpLayer.cpp:372-491, UdpLayer.cpp:103-178): the port
	// tables and the SIP heuristic, read once per packet after the walk so their latency is not on the
	// walk's critical path. A payload the reference would hand to an L7 dissector ends the chain after the
	// L4 layer (the tentative Payload layer is dropped) and flags the packet for the host.
	// the last TCP/UDP layer: whichever of the two came later
	const bool l7_tcp = (tcpA & 0xFFFFu) > (udpA & 0xFFFFu);
	const uint32_t l7A = l7_tcp ? tcpA : udpA, l7B = l7_tcp ? tcpB : udpB;
	const uint32_t l7_o = l7A >> 16, l7_next = l7A & 0xFFFFu, l7_end = l7_o + (l7B & 0xFFFFu), l7_pl = pps >> 16;
	if (l7_pl > 0 && !(flags & PCPPX_F_NEEDS_HOST_PROTO))
	{
		const uint32_t pw = rd32(p, l7_o);
		const uint32_t sp = swap16(pw), dp = swap16(pw >> 16);
		const bool sip = !l7_tcp && l7_pl >= 4 && sip_key(__builtin_bswap32(rd32(p, l7_o + 8)));
		const bool trig = l7_tcp ? tcp_l7(sp, dp) : (udp_l7(sp, dp) || sip);
		uint32_t lf = trig ? l7_flags(p, l7_tcp, l7_end - l7_pl, l7_pl, sp, dp, sip, true) : 0u;
		// parse-until options and a layer left to the host: it is rolled back (Packet.cpp:134-155,168-175)
		// when every candidate lies above parseUntilLayer, or the family was found and holds only engine-built
		// protocols (a classified layer is built below, under the stop rules themselves)
		if (lf && !(lf & kL7Built) && (prm.family != 0 || prm.until_osi < 8))  // uniform
		{
			if (l7_min_osi(l7_tcp, sp, dp, sip) > prm.until_osi || (found && prm.fam_engine_only))
				lf = 0;
		}
		if (lf)
		{
			if (count > l7_next)  // the tentative Payload was recorded
			{
				count = l7_next;
				mask &= ~(1ull << P_PAYLOAD);
				last_end = l7_end;
			}
			// a classified HTTP / SSL / DNS layer: built here with the layers behind it; anything else is the host's
			if (lf & kL7Built)
				count = l7_build<G>(p, lf, l7_end - l7_pl, l7_pl, dp, count, ml, cap_layers, prm.family, prm.until_osi,
				                 found, stopped, mask, lay_out);
			else
				flags |= lf;
		}
	}

	if (count > 0 && prm.family == 0 && prm.until_osi == 8 && !stopped &&
	    !(flags & (PCPPX_F_NEEDS_HOST_L7 | PCPPX_F_NEEDS_HOST_PROTO)) && last_end < cap)
	{
		uint32_t tl = cap - last_end;
		if (lay_out && count < ml)
			lay_out[count] = make_uint2(P_TRAILER | (2u << 8) | (last_end << 16), (tl & 0xFFFF) | (tl << 16));
		mask |= 1ull << P_TRAILER;
		++count;
		flags |= PCPPX_F_TRAILER;
	}
	if (count > cap_layers) flags |= PCPPX_F_DEPTH_OVERFLOW;

	Walk w;
	w.flags = flags;
	w.n_layers = count > cap_layers ? cap_layers : count;
	w.mask = mask;
	w.v4 = (v4w & 0xFFFFu) == 0xFFFFu ? -1 : (int32_t)(v4w & 0xFFFFu);
	w.v6 = v6o == 0xFFFFu ? -1 : (int32_t)v6o;
	w.v4_dlen = v4w >> 16;
	w.is_tcp = tcpA != 0;
	const uint32_t A = w.is_tcp ? tcpA : udpA, B = w.is_tcp ? tcpB : udpB;
	w.l4i = (int32_t)(A & 0xFFFFu) - 1;  // -1: no TCP/UDP layer (A == 0)
	w.l4o = A >> 16;
	w.l4dlen = B & 0xFFFFu;
	w.l4pp = w.is_tcp ? (pps & 0xFFu) : ((pps >> 8) & 0xFFu);
	w.l4ppo = B >> 16;
	return w;
}

__device__ __forceinline__ uint32_t fnv4(uint32_t h, uint32_t v)
{
	h = fnv(h, v & 0xFF);
	h = fnv(h, (v >> 8) & 0xFF);
	h = fnv(h, (v >> 16) & 0xFF);
	return fnv(h, v >> 24);
}

// hash5Tuple (both directions) and hash2Tuple (PacketUtils.cpp:139-245) from the addresses of the IP
// header at ipo (s/d: na little-endian dwords each) and the raw port word pw of the L4 layer (has_l4).
// Byte sequences: [port_a port_b ip_a ip_b proto] and [ip_a ip_b], the pair ordered as the reference
// orders it (raw-order port compare, then LE u32 (IPv4) / memcmp (IPv6) address compare).
// The address dwords past the first (IPv6) are hashed under a select, not a branch: a wave mixing IPv4 and IPv6 lanes
// runs them either way, and the selects spare the exec-mask bookkeeping of 24 branches (kBranchy: the branches, a
// tools-only diagnostic).
// kV4Skip (R6 bit 3): the address dwords past the first are hashed only when some active lane hashes an IPv6 pair (a
// wave-uniform branch on a ballot): a wave of IPv4 packets runs 3 x 2-3 dword steps instead of 3 x 8-9.
template <bool kBranchy = false, bool kV4Skip = false>
__device__ __forceinline__ void tuple_hashes(const uint32_t (&s)[4], const uint32_t (&d)[4], uint32_t na, bool has_l4,
                                             uint32_t pw, uint32_t proto, uint32_t& h5, uint32_t& h5d, uint32_t& h2)
{
	const bool any6 = !kV4Skip || __ballot(na != 1) != 0;  // uniform over the active lanes
	auto add4 = [&](uint32_t h, uint32_t k, uint32_t v) -> uint32_t {
		if (k > 0 && !any6)
			return h;
		if (kBranchy)
			return k < na ? fnv4(h, v) : h;
		const uint32_t y = fnv4(h, v);
		return k < na ? y : h;
	};
	int cmp = 0;  // sign of memcmp(dst, src) (IPv6) / (dst <=> src) as LE u32 (IPv4)
	if (na == 1)
		cmp = d[0] < s[0] ? -1 : (d[0] > s[0] ? 1 : 0);
	else
	{
#pragma unroll
		for (int k = 3; k >= 0; --k)
		{
			const uint32_t a = __builtin_bswap32(d[k]), b = __builtin_bswap32(s[k]);
			cmp = a < b ? -1 : (a > b ? 1 : cmp);
		}
	}
	const bool sw2 = cmp < 0;
	uint32_t x = 2166136261u;
#pragma unroll
	for (int k = 0; k < 4; ++k)
		x = add4(x, (uint32_t)k, sw2 ? d[k] : s[k]);
#pragma unroll
	for (int k = 0; k < 4; ++k)
		x = add4(x, (uint32_t)k, sw2 ? s[k] : d[k]);
	h2 = x;
	h5 = h5d = 0;
	if (!has_l4)
		return;
	const uint32_t sp = pw & 0xFFFF, dp = pw >> 16;  // raw network-order values, LE-loaded
	for (int dir = 0; dir < 2; ++dir)
	{
		const bool swap = !dir && (dp < sp || (dp == sp && cmp < 0));
		uint32_t y = 2166136261u;
		const uint32_t fp = swap ? dp : sp, sp2 = swap ? sp : dp;
		y = fnv(fnv(y, fp & 0xFF), fp >> 8);
		y = fnv(fnv(y, sp2 & 0xFF), sp2 >> 8);
#pragma unroll
		for (int k = 0; k < 4; ++k)
			y = add4(y, (uint32_t)k, swap ? d[k] : s[k]);
#pragma unroll
		for (int k = 0; k < 4; ++k)
			y = add4(y, (uint32_t)k, swap ? s[k] : d[k]);
		y = fnv(y, proto);
		if (dir) h5d = y; else h5 = y;
	}
}

// hash5Tuple / hash2Tuple of a generic-walk packet: addresses of the first IPv4 (else first IPv6) layer,
// ports of the last TCP (else last UDP) layer, the IP layer's protocol / next-header byte. Dword reads
// from the LDS window where the bytes are staged (rd32), else from HBM.
template <bool kV4Skip = false>
__device__ __forceinline__ void hashes(const Pkt& p, const Walk& w, uint32_t& h5, uint32_t& h5d, uint32_t& h2)
{
	h5 = h5d = h2 = 0;
	if (w.v4 < 0 && w.v6 < 0)
		return;
	const bool v4 = w.v4 >= 0;
	const uint32_t ipo = v4 ? (uint32_t)w.v4 : (uint32_t)w.v6;
	const uint32_t na = v4 ? 1 : 4;
	const uint32_t so = ipo + (v4 ? 12 : 8), dofs = ipo + (v4 ? 16 : 24);
	uint32_t s[4], d[4];
#pragma unroll
	for (int k = 0; k < 4; ++k)
	{
		s[k] = (uint32_t)k < na ? rd32(p, so + 4 * k) : 0;
		d[k] = (uint32_t)k < na ? rd32(p, dofs + 4 * k) : 0;
	}
	const bool has_l4 = w.l4i >= 0 && !(w.mask & (1ull << P_ICMP));  // ICMP: no 5-tuple (PacketUtils.cpp:144-145)
	const uint32_t pw = has_l4 ? rd32(p, w.l4o) : 0;
	tuple_hashes<false, kV4Skip>(s, d, na, has_l4, pw, rb(p, ipo + (v4 ? 9 : 6)), h5, h5d, h2);
}

// ---- the three hashes of a whole wave (round 6, ParseShape R6 bit 1) ----
// A packet's hash inputs, gathered by whichever walk parsed it: the first IPv4 (else first IPv6) layer's addresses (na
// dwords each, zero past na: also the 5-tuple extract's address fields), the port layer's raw port dword (pw, whenever a
// TCP / UDP layer exists), and meta = IP protocol / next-header byte | IPv4 << 8 | IPv6 << 9 | hashed ports << 10 (a port
// layer, an IP layer and no ICMP, PacketUtils.cpp:141-148) | a port layer << 11.
struct HashIn
{
	uint32_t s[4], d[4], pw, meta;
};
__device__ __forceinline__ HashIn hash_in_none()
{
	HashIn h;
#pragma unroll
	for (int k = 0; k < 4; ++k)
		h.s[k] = h.d[k] = 0;
	h.pw = h.meta = 0;
	return h;
}
// the inputs hashes() reads, from the LDS window where staged, else HBM (a generic-walk packet)
__device__ __forceinline__ HashIn hash_in_walk(const Pkt& p, const Walk& w)
{
	HashIn h = hash_in_none();
	const bool v4 = w.v4 >= 0, ip = v4 || w.v6 >= 0;
	const uint32_t ipo = v4 ? (uint32_t)w.v4 : (uint32_t)w.v6;
	const uint32_t na = ip ? (v4 ? 1u : 4u) : 0u;
	const uint32_t so = ipo + (v4 ? 12 : 8), dofs = ipo + (v4 ? 16 : 24);
#pragma unroll
	for (int k = 0; k < 4; ++k)
	{
		h.s[k] = (uint32_t)k < na ? rd32(p, so + 4 * k) : 0u;
		h.d[k] = (uint32_t)k < na ? rd32(p, dofs + 4 * k) : 0u;
	}
	const bool l4 = w.l4i >= 0;
	const bool has5 = l4 && !(w.mask & (1ull << P_ICMP));
	h.pw = l4 ? rd32(p, w.l4o) : 0u;
	h.meta = (ip ? (rb(p, ipo + (v4 ? 9 : 6)) | (v4 ? 0x100u : 0x200u) | (has5 ? 0x400u : 0u)) : 0u) | (l4 ? 0x800u : 0u);
	return h;
}
// hash5Tuple (both directions) and hash2Tuple (PacketUtils.cpp:114-245) of every lane's packet, all 64 lanes together
// (call with the wave converged). The byte sequences are tuple_hashes': [ports addr_a addr_b proto] and [addr_a addr_b].
// IPv4 packets hash their 3 x 13 / 8 bytes in their own lanes. An IPv6 packet's chains are 37 / 37 / 32 bytes: run in its
// own lane they would hold every lane of a mixed wave for them, so each IPv6 chain goes to a lane of its own instead --
// chain k of the r-th IPv6 packet to slot k * n6 + r (k: 0 hash2Tuple, 1 hash5Tuple direction-unique, 2 hash5Tuple with
// the pair swapped, needed only when the reference swaps it), 64 slots per round, the inputs and results moved by
// ds_bpermute. `own`: 64 words of LDS scratch (the rank -> lane map).
__device__ __forceinline__ void wave_tuple_hashes(const HashIn& x, uint32_t* own, uint32_t& h5, uint32_t& h5d, uint32_t& h2)
{
	const uint32_t lane = threadIdx.x & 63u;
	const bool v4 = x.meta & 0x100u, v6 = x.meta & 0x200u, l4 = x.meta & 0x400u;
	const uint32_t proto = x.meta & 0xFFu;
	// the address order: dst <=> src as LE u32 (IPv4) / memcmp(dst, src) (IPv6)
	int cmp = x.d[0] < x.s[0] ? -1 : (x.d[0] > x.s[0] ? 1 : 0);
	if (!v4)
	{
		cmp = 0;
#pragma unroll
		for (int k = 3; k >= 0; --k)
		{
			const uint32_t a = __builtin_bswap32(x.d[k]), b = __builtin_bswap32(x.s[k]);
			cmp = a < b ? -1 : (a > b ? 1 : cmp);
		}
	}
	const bool sw2 = cmp < 0;
	const uint32_t sp = x.pw & 0xFFFF, dp = x.pw >> 16;  // raw network-order values, LE-loaded
	const bool swap = dp < sp || (dp == sp && cmp < 0);
	constexpr uint32_t iv = 2166136261u;
	h2 = h5 = h5d = 0;
	if (__ballot(v4))  // uniform
	{
		const uint32_t a = sw2 ? x.d[0] : x.s[0], b = sw2 ? x.s[0] : x.d[0];
		const uint32_t y2 = fnv4(fnv4(iv, a), b);
		const uint32_t yd = fnv(fnv4(fnv4(fnv4(iv, x.pw), x.s[0]), x.d[0]), proto);
		uint32_t ys = yd;
		if (__ballot(v4 && l4 && swap))  // uniform
		{
			const uint32_t t = fnv(fnv4(fnv4(fnv4(iv, (x.pw >> 16) | (x.pw << 16)), x.d[0]), x.s[0]), proto);
			ys = swap ? t : yd;
		}
		h2 = v4 ? y2 : 0u;
		h5d = v4 && l4 ? yd : 0u;
		h5 = v4 && l4 ? ys : 0u;
	}
	const uint64_t m6 = __ballot(v6);
	if (m6)  // uniform
	{
		const uint32_t n6 = (uint32_t)__popcll(m6);
		const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m6 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m6, 0u));
		if (v6)
			own[rank] = lane;
		__syncthreads();  // one wave per block: orders the map's writes before its reads
		const uint32_t fl = proto | (sw2 ? 0x100u : 0u);
		uint32_t r0 = 0, r1 = 0, r2 = 0;
		for (uint32_t base = 0; base < 3 * n6; base += 64)  // uniform
		{
			const uint32_t t = base + lane;
			const uint32_t k = t >= 2 * n6 ? 2u : (t >= n6 ? 1u : 0u);
			const uint32_t o = own[(t - k * n6) & 63u];
			uint32_t S[4], D[4];
#pragma unroll
			for (int j = 0; j < 4; ++j)
			{
				S[j] = __shfl(x.s[j], (int)o, 64);
				D[j] = __shfl(x.d[j], (int)o, 64);
			}
			const uint32_t pw = __shfl(x.pw, (int)o, 64), of = __shfl(fl, (int)o, 64);
			const bool dfirst = k == 2 || (k == 0 && (of & 0x100u));
			const uint32_t yp = fnv4(iv, k == 2 ? (pw >> 16) | (pw << 16) : pw);
			uint32_t y = k ? yp : iv;
#pragma unroll
			for (int j = 0; j < 4; ++j)
				y = fnv4(y, dfirst ? D[j] : S[j]);
#pragma unroll
			for (int j = 0; j < 4; ++j)
				y = fnv4(y, dfirst ? S[j] : D[j]);
			const uint32_t yq = fnv(y, of & 0xFFu);
			y = k ? yq : y;
			// each owner takes its chains' results from the slots of this round
			const uint32_t q0 = rank, q1 = n6 + rank, q2 = 2 * n6 + rank;
			const uint32_t g0 = __shfl(y, (int)(q0 & 63u), 64), g1 = __shfl(y, (int)(q1 & 63u), 64),
			               g2 = __shfl(y, (int)(q2 & 63u), 64);
			r0 = (q0 >= base && q0 < base + 64) ? g0 : r0;
			r1 = (q1 >= base && q1 < base + 64) ? g1 : r1;
			r2 = (q2 >= base && q2 < base + 64) ? g2 : r2;
		}
		if (v6)
		{
			h2 = r0;
			h5d = l4 ? r1 : 0u;
			h5 = l4 ? (swap ? r2 : r1) : 0u;
		}
	}
}

// write_tuple from the inputs the hashes used (the same bytes: the fields hash5Tuple reads)
__device__ __forceinline__ void write_tuple_in(const HashIn& x, const Walk& w, uint32_t h5, pcppx_tuple* out)
{
	const bool ip = (x.meta & 0x300u) != 0, l4 = (x.meta & 0x800u) != 0;
	const uint32_t ports = swap16(x.pw) | (swap16(x.pw >> 16) << 16);  // getSrcPort / getDstPort (host order)
	const bool has5 = (x.meta & 0x400u) != 0;
	const uint32_t meta = (ip ? ((x.meta & 0x100u) ? 4u : 6u) : 0u) | ((x.meta & 0xFFu) << 8) |
	                      ((l4 ? (w.is_tcp ? P_TCP : P_UDP) : 0u) << 16) | ((has5 ? 1u : 0u) << 24);
	uint4* o = reinterpret_cast<uint4*>(out);
	o[0] = make_uint4(x.s[0], x.s[1], x.s[2], x.s[3]);
	o[1] = make_uint4(x.d[0], x.d[1], x.d[2], x.d[3]);
	o[2] = make_uint4(ports, meta, h5, (w.flags & 0xFFFFu) | ((w.n_layers & 0xFFu) << 16));
}

// IPv4 header checksum (IPv4Layer.cpp:410-412): computeChecksum over min(IHL*4, dataLen) header bytes
// with the checksum field zeroed. Returns calc; *stored gets the field.
__device__ __forceinline__ uint32_t ipv4_checksum(const Pkt& p, const Walk& w, uint32_t* stored)
{
	const uint32_t o = (uint32_t)w.v4;
	uint32_t hl = (rb(p, o) & 0xF) * 4;
	if (hl > w.v4_dlen) hl = w.v4_dlen;
	uint32_t r = range_residue(p, o, o + hl);
	*stored = be16(p, o + 10);
	r = (r + 65535u - mod65535(le16(p, o + 10))) % 65535u;  // field is stream word 5 (even offset)
	return finish_checksum(r);
}

// {Tcp,Udp}Layer::calculateChecksum(false) (TcpLayer.cpp:271-311, UdpLayer.cpp:47-90) given the
// residue of the L4 bytes as a stream: subtract the checksum field, add the pseudo header
// (computePseudoHdrChecksum, PacketUtils.cpp:66-112), fold; UDP maps 0 to 0xFFFF.
// the header-byte inputs of l4_checksum (read while the LDS window holds them): the checksum field as a
// little-endian stream word, and the pseudo header's halves-sum (computePseudoHdrChecksum, PacketUtils.cpp:66-112)
__device__ __forceinline__ void l4_inputs(const Pkt& p, const Walk& w, uint32_t* fw, uint32_t* ph)
{
	*fw = rd16(p, w.l4o + (w.is_tcp ? 16 : 6));
	uint32_t h = 0;
	if (w.l4pp == P_IPV4 || w.l4pp == P_IPV6)
	{
		const uint32_t as = w.l4pp == P_IPV4 ? w.l4ppo + 12 : w.l4ppo + 8;
		const uint32_t nd = w.l4pp == P_IPV4 ? 2 : 8;  // dwords of src+dst
		for (uint32_t j = 0; j < nd; ++j) h += halves(rd32(p, as + 4 * j));
		h += ((w.l4dlen & 0xFF) << 8) | ((w.l4dlen >> 8) & 0xFF);  // htobe16(dataLen)
		h += (w.is_tcp ? 6u : 17u) << 8;                              // htobe16(protocol)
	}
	*ph = h;
}

__device__ __forceinline__ uint32_t l4_checksum_from(const Walk& w, uint32_t l4_residue, uint32_t fw, uint32_t ph,
                                                     uint32_t* stored)
{
	*stored = swap16(fw);
	uint32_t res = 0;
	if (w.l4pp == P_IPV4 || w.l4pp == P_IPV6)
	{
		uint32_t r = (l4_residue + 65535u - mod65535(fw)) % 65535u;
		r = (r + mod65535(ph)) % 65535u;
		res = finish_checksum(r);
	}
	if (!w.is_tcp && res == 0)
		res = 0xFFFF;
	return res;
}

__device__ __forceinline__ uint32_t l4_checksum(const Pkt& p, const Walk& w, uint32_t l4_residue, uint32_t* stored)
{
	uint32_t fw, ph;
	l4_inputs(p, w, &fw, &ph);
	return l4_checksum_from(w, l4_residue, fw, ph, stored);
}

__device__ __forceinline__ void write_summary(pcppx_summary* out, uint32_t h5, uint32_t h5d, uint32_t h2,
                                              uint32_t flags, uint32_t n_layers, int32_t l4i, uint64_t mask,
                                              uint32_t ipc, uint32_t ips, uint32_t l4c, uint32_t l4s)
{
	uint4 s0 = make_uint4(h5, h5d, h2, flags | (n_layers << 16) | ((l4i >= 0 ? (uint32_t)l4i : 0xFFu) << 24));
	uint4 s1 = make_uint4((uint32_t)mask, (uint32_t)(mask >> 32), ipc | (ips << 16), l4c | (l4s << 16));
	reinterpret_cast<uint4*>(out)[0] = s0;
	reinterpret_cast<uint4*>(out)[1] = s1;
}

// the 5-tuple extract (pcppx_tuple): the fields hash5Tuple reads (PacketUtils.cpp:139-210) -- the first IPv4, else first
// IPv6 layer's addresses and protocol / next-header byte, the port layer's (last TCP, else last UDP) ports -- read the
// way hashes() reads them (the LDS window where staged, else HBM); three 16-B stores
__device__ __forceinline__ void write_tuple(const Pkt& p, const Walk& w, uint32_t h5, pcppx_tuple* out)
{
	const bool v4 = w.v4 >= 0, ip = v4 || w.v6 >= 0;
	const uint32_t ipo = v4 ? (uint32_t)w.v4 : (uint32_t)w.v6;
	const uint32_t na = ip ? (v4 ? 1u : 4u) : 0u;
	const uint32_t so = ipo + (v4 ? 12 : 8), dofs = ipo + (v4 ? 16 : 24);
	uint32_t s[4], d[4];
#pragma unroll
	for (int k = 0; k < 4; ++k)
	{
		s[k] = (uint32_t)k < na ? rd32(p, so + 4 * k) : 0u;
		d[k] = (uint32_t)k < na ? rd32(p, dofs + 4 * k) : 0u;
	}
	const bool l4 = w.l4i >= 0;
	const uint32_t pw = l4 ? rd32(p, w.l4o) : 0u;  // raw network-order ports, LE-loaded
	const uint32_t ports = swap16(pw) | (swap16(pw >> 16) << 16);  // getSrcPort / getDstPort (host order)
	const uint32_t ipp = ip ? rb(p, ipo + (v4 ? 9 : 6)) : 0u;
	const bool has5 = ip && l4 && !(w.mask & (1ull << P_ICMP));  // PacketUtils.cpp:141-148
	const uint32_t meta = (ip ? (v4 ? 4u : 6u) : 0u) | (ipp << 8) | ((l4 ? (w.is_tcp ? P_TCP : P_UDP) : 0u) << 16) |
	                      ((has5 ? 1u : 0u) << 24);
	uint4* o = reinterpret_cast<uint4*>(out);
	o[0] = make_uint4(s[0], s[1], s[2], s[3]);
	o[1] = make_uint4(d[0], d[1], d[2], d[3]);
	o[2] = make_uint4(ports, meta, h5, (w.flags & 0xFFFFu) | ((w.n_layers & 0xFFu) << 16));
}

// PacketStats::collectStats (Examples/DpdkExample-FilterTraffic/Common.h:83-104) of one wave of packets: 11 ballot counts
// (<= 64 each) packed as bytes into one 16-B record per wave (PCPPX_PS_* order), written by lane 0. Same rules as
// filter_apply_kernel: HTTP / DNS / SSL only for the packets the device settles.
__device__ __forceinline__ void wave_proto_stats(bool in, uint64_t mask, uint32_t flags, uint4* out)
{
	const bool settled = (flags & (PCPPX_F_NEEDS_HOST_PROTO | PCPPX_F_OVERSIZE | PCPPX_F_BAD_DESC)) == 0 &&
	                     (!(flags & PCPPX_F_NEEDS_HOST_L7) || (flags & PCPPX_F_L7_KNOWN));
	const bool http = (flags & PCPPX_F_L7_HTTP) || (mask & ((1ull << P_HTTP_REQ) | (1ull << P_HTTP_RESP)));
	const bool dns = (flags & PCPPX_F_L7_DNS) || (mask & (1ull << P_DNS));
	const bool ssl = (flags & PCPPX_F_L7_SSL) || (mask & (1ull << P_SSL));
	auto cnt = [&](bool pr) { return (uint32_t)__popcll(__ballot(in && pr)); };
	const uint32_t x = cnt(true) | (cnt((mask >> P_ETH) & 1) << 8) | (cnt((mask >> P_ARP) & 1) << 16) |
	                   (cnt((mask >> P_IPV4) & 1) << 24);
	const uint32_t y = cnt((mask >> P_IPV6) & 1) | (cnt((mask >> P_TCP) & 1) << 8) | (cnt((mask >> P_UDP) & 1) << 16) |
	                   (cnt(settled && http) << 24);
	const uint32_t z = cnt(settled && dns) | (cnt(settled && ssl) << 8) | (cnt(!settled) << 16);
	if ((threadIdx.x & 63) == 0)
		*out = make_uint4(x, y, z, 0u);
}

// descriptor checks shared by both kernels: returns 0 if the packet is parseable, else its flags
__device__ __forceinline__ uint32_t desc_flags(uint64_t off, uint32_t cap, uint64_t data_len, bool* empty)
{
	*empty = false;
	if (off + cap > data_len || off + cap < off)
		return PCPPX_F_BAD_DESC;
	if (cap > PCPPX_MAX_CAPLEN)
		return PCPPX_F_OVERSIZE;
	if (cap == 0)
		*empty = true;
	return 0;
}

// ---------------- fast path: straight-line stages over the LDS window ----------------
//
// Ethernet, up to two 802.1Q/802.1ad tags, up to three MPLS labels, an IPv4 or IPv6 layer (IPv6 with up to three
// extension headers; an IPv4 fragment or a last Fragment extension makes the rest a Payload), optionally a GREv0
// layer and an inner IPv4 / IPv6 layer, then TCP or UDP, Payload (or an L7 flag) and a trailer; no parse-until
// options. Each optional stage (MPLS, IPv6 extensions, GRE) runs only when some lane of the wave needs it (a scalar
// branch on a ballot), so plain Eth/[VLAN]/IP/L4 waves pay for the plain stages only. Every byte read must sit in
// the LDS window; anything else (or any rule this path does not cover) makes the packet "not applicable" and the
// generic walk_chain() runs for it. Same rules and records as walk_chain() (bit-exact in tests/).

// A fast-path packet, packed into five registers (it stays live across the checksum stream): offsets and header
// lengths inside the LDS window fit 8 bits, data lengths 16 bits.
struct Fast
{
	uint32_t a;  // o1 | h1 << 8 | o2 << 16 | h2 << 24: the first / inner IP layer's offset and header length
	uint32_t b;  // d1 | d2 << 16: their data lengths
	uint32_t c;  // l4o | l4hdr << 8 | gh << 16 | nv << 24 | nm << 26 | gre << 28 | v6a << 29 | v6b << 30 | l4 << 31
	uint32_t d;  // l4dlen | trailer << 16 (until fast_l7: the last IP layer's end)
	uint32_t e;  // tcp | payload << 1 | simple << 2 | l7 flags << 16 (PCPPX_F_NEEDS_HOST_L7 | PCPPX_F_L7_*)
	__device__ __forceinline__ uint32_t o1() const { return a & 0xFF; }
	__device__ __forceinline__ uint32_t h1() const { return (a >> 8) & 0xFF; }
	__device__ __forceinline__ uint32_t o2() const { return (a >> 16) & 0xFF; }
	__device__ __forceinline__ uint32_t h2() const { return a >> 24; }
	__device__ __forceinline__ uint32_t d1() const { return b & 0xFFFF; }
	__device__ __forceinline__ uint32_t d2() const { return b >> 16; }
	__device__ __forceinline__ uint32_t l4o() const { return c & 0xFF; }
	__device__ __forceinline__ uint32_t l4hdr() const { return (c >> 8) & 0xFF; }
	__device__ __forceinline__ uint32_t gh() const { return (c >> 16) & 0xFF; }
	__device__ __forceinline__ uint32_t nv() const { return (c >> 24) & 3; }
	__device__ __forceinline__ uint32_t nm() const { return (c >> 26) & 3; }
	__device__ __forceinline__ uint32_t gre() const { return (c >> 28) & 1; }
	__device__ __forceinline__ uint32_t v6a() const { return (c >> 29) & 1; }
	__device__ __forceinline__ uint32_t v6b() const { return (c >> 30) & 1; }
	__device__ __forceinline__ uint32_t l4() const { return c >> 31; }
	__device__ __forceinline__ uint32_t l4dlen() const { return d & 0xFFFF; }
	__device__ __forceinline__ uint32_t trailer() const { return d >> 16; }
	__device__ __forceinline__ uint32_t tcp() const { return e & 1; }
	__device__ __forceinline__ uint32_t payload() const { return (e >> 1) & 1; }
	__device__ __forceinline__ uint32_t simple() const { return (e >> 2) & 1; }
	__device__ __forceinline__ uint32_t l7() const { return e >> 16; }
};

// an IP layer at [o, o+len): IPv4Layer::isDataValid (IPv4Layer.h:626-630), initLayerInPacket (IPv4Layer.cpp:180-197),
// isFragment (:415-418); IPv6Layer::isDataValid (IPv6Layer.h:245-249) and its fixed header (the extension headers
// are walked by the caller). Selects over the same three dwords for both versions.
struct IpDec
{
	uint32_t ok, hdr, dlen, nh, frag, plen;  // plen: IPv6 payload length
};
__device__ __forceinline__ IpDec ip_decode(const Pkt& p, uint32_t o, uint32_t len, bool v6)
{
	const uint32_t w0 = lds_u32(p, o);      // ver/ihl, tos, total length (v4) | ver/tc/flow (v6)
	const uint32_t w1 = lds_u32(p, o + 4);  // id, frag (v4) | payload length, next header, hop limit (v6)
	const uint32_t w2 = lds_u32(p, o + 8);  // ttl, protocol, checksum (v4)
	const uint32_t b0 = w0 & 0xFF;
	IpDec d;
	const uint32_t h4 = (b0 & 0xF) * 4, tl = swap16(w0 >> 16), hmin = h4 < len ? h4 : len;
	const uint32_t dl4 = (tl < len && tl != 0) ? (tl > hmin ? tl : hmin) : len;
	const uint32_t b6 = (w1 >> 16) & 0xFF, b7 = w1 >> 24;
	d.plen = swap16(w1);
	const uint32_t tot6 = d.plen + 40;
	d.ok = v6 ? (len >= 40 && (b0 >> 4) == 6) : (len >= 20 && (b0 >> 4) == 4 && (b0 & 0xF) >= 5);
	d.hdr = v6 ? 40u : h4;
	d.dlen = v6 ? (tot6 < len ? tot6 : len) : dl4;
	d.nh = v6 ? b6 : ((w2 >> 8) & 0xFF);
	d.frag = !v6 && ((b6 & 0x20) || (((b6 & 0x1F) << 8) | b7) != 0);
	return d;
}

__device__ __forceinline__ bool fast_walk(const Pkt& p, uint32_t cap, const Params& prm, Fast& f)
{
	bool ok = prm.linktype == 1 && prm.family == 0 && prm.until_osi == 8 && p.lim >= 20 && cap > 14;
	// Ethernet (EthLayer.cpp:28-69, isDataValid :100-117)
	uint32_t et = swap16(lds_u32(p, 12));
	ok = ok && et >= 0x0600;
	uint32_t o = 14, len = cap - 14, nv = 0, nm = 0;
	// up to two VLAN tags (VlanLayer.cpp:59-119): each needs len > 4 so that a next layer follows
#pragma unroll
	for (int t = 0; t < 2; ++t)
	{
		const bool vl = (et == 0x8100 || et == 0x88A8) && len > 4 && o + 8 <= p.lim;
		const uint32_t e2 = swap16(lds_u32(p, vl ? o : 0) >> 16);
		et = vl ? e2 : et;
		o = vl ? o + 4 : o;
		len = vl ? len - 4 : len;
		nv += vl ? 1 : 0;
	}
	// up to three MPLS labels (MplsLayer.cpp:101-128): a label has a next layer only with >= 5 bytes (which also
	// covers Ethernet's >= 4 bytes, EthLayer.cpp:28-69); not bottom of stack: another label (unchecked); bottom of
	// stack: IPv4 / IPv6 by the next nibble
	if (__ballot(ok && et == 0x8847))  // wave-uniform
	{
#pragma unroll
		for (int t = 0; t < 3; ++t)
		{
			const bool ml = et == 0x8847 && len >= 5 && o + 5 <= p.lim;
			const uint32_t w = lds_u32(p, ml ? o : 0), nb = (lds_u32(p, ml ? o + 4 : 0) & 0xFF) >> 4;
			const uint32_t nxt = ((w >> 16) & 1) ? (nb == 4 ? 0x0800u : (nb == 6 ? 0x86DDu : 0xFFFFu)) : 0x8847u;
			et = ml ? nxt : et;
			o = ml ? o + 4 : o;
			len = ml ? len - 4 : len;
			nm += ml ? 1 : 0;
		}
	}
	// the first IP layer: its fixed header, then IPv6's extension headers (IPv6Layer::parseExtensions,
	// IPv6Layer.cpp:79-147: next headers 0/43/44/60 take 8*(len+1) bytes, AH 51 4*(len+2); no bound check)
	const bool v6a = et == 0x86DD;
	ok = ok && (et == 0x0800 || v6a) && o + (v6a ? 40 : 20) <= p.lim;  // the fixed header (addresses included)
	IpDec d1 = ip_decode(p, o, len, v6a);
	ok = ok && d1.ok;
	constexpr uint64_t kExt = (1ull << 0) | (1ull << 43) | (1ull << 44) | (1ull << 51) | (1ull << 60);
	uint32_t ext = 0, last_ext = 0xFFu;
	if (__ballot(ok && v6a && d1.nh < 64 && ((kExt >> d1.nh) & 1ull)))  // wave-uniform
	{
		uint32_t eo = 40;
#pragma unroll
		for (int t = 0; t < 3; ++t)
		{
			const bool e = v6a && d1.nh < 64 && ((kExt >> d1.nh) & 1ull) && eo + 2 <= len && o + eo + 2 <= p.lim;
			const uint32_t two = lds_u32(p, e ? o + eo : 0) & 0xFFFFu;
			const uint32_t el = d1.nh == 51 ? 4u * ((two >> 8) + 2) : 8u * ((two >> 8) + 1);
			last_ext = e ? d1.nh : last_ext;
			d1.nh = e ? (two & 0xFFu) : d1.nh;
			ext += e ? el : 0u;
			eo += e ? el : 0u;
		}
		// a chain longer than the stage walks (or one leaving the window) goes to the generic walk
		ok = ok && !(v6a && d1.nh < 64 && ((kExt >> d1.nh) & 1ull) && eo + 2 <= len);
		// IPv6Layer: header = 40 + extensions; dataLen = payloadLength + header when shorter (IPv6Layer.cpp:28-40)
		if (v6a)
		{
			d1.hdr = 40 + ext;
			const uint32_t tot = d1.plen + d1.hdr;
			d1.dlen = tot < len ? tot : len;
		}
	}
	// IP dispatch (IPv4Layer.cpp:245-370, IPv6Layer.cpp:194-312): a fragment (IPv4) or a last Fragment extension
	// (IPv6) -> Payload; 47 -> GRE; 6 / 17 -> TCP / UDP; anything else -> the generic walk
	const bool frag1 = d1.frag || (v6a && last_ext == 44);
	ok = ok && d1.dlen > d1.hdr && (frag1 || d1.nh == 6 || d1.nh == 17 || d1.nh == 47);
	uint32_t lo = o + d1.hdr, lp = ok ? d1.dlen - d1.hdr : 0, lnh = d1.nh;  // the last IP layer's payload
	// GREv0 (GreLayer.cpp:23-36,195-252): flags C/R, K, S, A add 4 bytes each; EtherType IPv4 / IPv6 (tryConstruct)
	uint32_t gre = 0, gh = 0, o2 = 0;
	IpDec d2{};
	bool v6b = false;
	if (__ballot(ok && !frag1 && d1.nh == 47))  // wave-uniform
	{
		const bool g = ok && !frag1 && d1.nh == 47;
		ok = ok && (!g || lo + 4 <= p.lim);
		const uint32_t gw = lds_u32(p, g ? lo : 0);
		const uint32_t f0 = gw & 0xFF, f1 = (gw >> 8) & 0xFF, get = swap16(gw >> 16);
		gh = 4 + ((f0 & 0xC0) ? 4 : 0) + ((f0 & 0x20) ? 4 : 0) + ((f0 & 0x10) ? 4 : 0) + ((f1 & 0x80) ? 4 : 0);
		ok = ok && (!g || (lp >= 4 && (f1 & 7) == 0 && lp > gh && (get == 0x0800 || get == 0x86DD)));
		v6b = get == 0x86DD;
		o2 = lo + gh;
		const uint32_t len2 = g ? lp - gh : 0;
		ok = ok && (!g || o2 + (v6b ? 40 : 20) <= p.lim);
		d2 = ip_decode(p, g && ok ? o2 : 0, len2, v6b);
		// the inner layer: valid, not a fragment, no extension headers, TCP / UDP behind it
		ok = ok && (!g || (d2.ok && !d2.frag && d2.dlen > d2.hdr && (d2.nh == 6 || d2.nh == 17)));
		gre = g ? 1u : 0u;
		lo = g ? o2 + d2.hdr : lo;
		lp = g ? (ok ? d2.dlen - d2.hdr : 0) : lp;
		lnh = g ? d2.nh : lnh;
	}
	// TCP / UDP (TcpLayer::isDataValid TcpLayer.h:596-601; UDP needs 8 bytes), unless a fragment made a Payload
	const bool l4 = !frag1;
	const bool tcp = l4 && lnh == 6;
	ok = ok && (!l4 || lo + (tcp ? 20 : 8) <= p.lim);
	const uint32_t doff = (lds_u32(p, (ok && tcp) ? lo + 12 : 0) & 0xFF) >> 4;
	ok = ok && (!l4 || (tcp ? (lp >= 20 && doff >= 5 && lp >= doff * 4) : lp >= 8));
	const uint32_t l4hdr = !l4 ? 0u : (tcp ? doff * 4 : 8u);
	const bool payload = lp > l4hdr;
	// the SIP heuristic (UDP payloads of >= 4 B) reads 4 payload bytes from LDS too
	ok = ok && (!l4 || tcp || !payload || lp - 8 < 4 || lo + 12 <= p.lim);
	// the IPv4 header checksum reads the whole first IPv4 header from LDS too
	ok = ok && (v6a || o + d1.hdr <= p.lim) && (!gre || !v6a || v6b || o2 + d2.hdr <= p.lim);
	// until fast_l7: trailer = the last IP layer's end, no L7 flags (the L7 decision is taken after the hashes)
	const uint32_t end = gre ? o2 + d2.dlen : o + d1.dlen;
	f.a = (o & 0xFF) | ((d1.hdr & 0xFF) << 8) | ((o2 & 0xFF) << 16) | ((d2.hdr & 0xFF) << 24);
	f.b = (d1.dlen & 0xFFFF) | (d2.dlen << 16);
	f.c = (lo & 0xFF) | ((l4hdr & 0xFF) << 8) | ((gh & 0xFF) << 16) | (nv << 24) | (nm << 26) | (gre << 28) |
	      ((v6a ? 1u : 0u) << 29) | ((v6b ? 1u : 0u) << 30) | ((l4 ? 1u : 0u) << 31);
	f.d = (lp & 0xFFFF) | (end << 16);
	f.e = (tcp ? 1u : 0u) | ((payload ? 1u : 0u) << 1) | ((nm == 0 && ext == 0 && !frag1 && !gre) ? 4u : 0u);
	// everything above sits inside the window (< 256 B), lengths below 64 KiB (caplen cap)
	ok = ok && o + d1.hdr < 256 && o2 + d2.hdr < 256 && lo < 256;
	return ok;
}

// The table words the L7 trigger of a fast-path packet needs (tcp_l7 / udp_l7 / sip_key: port bitmap words and the
// SIP key slot), loaded ahead of the hashes so that their latency hides behind them (fast_l7 consumes them).
struct L7Pre
{
	uint32_t ws, wd, wu, sk;  // src / dst port words of the TCP or UDP bitmap, dst word of udp_dst, SIP slot key
};
__device__ __forceinline__ L7Pre fast_l7_pre(const Pkt& p, const Fast& f)
{
	L7Pre r{ 0u, 0u, 0u, 0u };
	if (f.payload() && f.l4())
	{
		const uint32_t pw = lds_u32(p, f.l4o());
		const uint32_t sport = swap16(pw), dport = swap16(pw >> 16);
		const uint32_t* t = f.tcp() ? kL7.tcp : kL7.udp;
		r.ws = t[sport >> 5];
		r.wd = t[dport >> 5];
		if (!f.tcp())
		{
			r.wu = kL7.udp_dst[dport >> 5];
			if (f.l4dlen() - 8 >= 4)  // the SIP heuristic's 4 payload bytes (in the window: fast_walk)
				r.sk = kSip.key[(__builtin_bswap32(lds_u32(p, f.l4o() + 8)) * kSipMul) >> 27];
		}
	}
	return r;
}

// fast_l7_pre's words from the register tables (kL7R, R6 bit 2): called by every lane of the wave (ds_bpermute reads the
// table registers of all 64 lanes), `on` for the fast-path packets with a payload behind their TCP / UDP layer. Each
// word holds only the bit fast_l7 tests (a port's bit of its 32-port group), the SIP slot's key as kSip.key holds it.
__device__ __forceinline__ L7Pre l7_pre_regs(const Pkt& p, const Fast& f, bool on, uint32_t rt, uint32_t rus)
{
	const uint32_t l4o = on ? f.l4o() : 0u;
	const uint32_t pw = lds_u32(p, l4o);
	const uint32_t sport = swap16(pw), dport = swap16(pw >> 16);
	// the SIP heuristic's 4 payload bytes (read only when they lie in the window: fast_walk)
	const bool sipw = on && !f.tcp() && f.l4dlen() - 8 >= 4;
	const uint32_t key = __builtin_bswap32(lds_u32(p, sipw ? l4o + 8 : 0u));
	auto bperm = [](uint32_t reg, uint32_t slot) {
		return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(slot << 2), (int)reg);
	};
	const uint32_t ts = bperm(rt, tcp_slot(sport)), td = bperm(rt, tcp_slot(dport));
	const uint32_t us = bperm(rus, udp_slot(sport)), ud = bperm(rus, udp_slot(dport));
	const uint32_t sk = bperm(rus, 32u + ((key * kSipMul) >> 27));
	const bool tcp = f.tcp() != 0;
	const bool hs = tcp ? ts == (sport | 0x10000u) : (us & 0x1FFFFu) == (sport | 0x10000u);
	const bool hd = tcp ? td == (dport | 0x10000u) : (ud & 0x1FFFFu) == (dport | 0x10000u);
	const bool hu = !tcp && (ud & 0x2FFFFu) == (dport | 0x20000u);
	L7Pre r;
	r.ws = on && hs ? 1u << (sport & 31) : 0u;
	r.wd = on && hd ? 1u << (dport & 31) : 0u;
	r.wu = on && hu ? 1u << (dport & 31) : 0u;
	r.sk = sipw ? sk : 0u;
	return r;
}

// L7 dispatch of a fast-path packet (same rules as walk_chain's): an L7 payload ends the chain after the
// L4 layer, with no Payload and no trailer. `pre`: fast_l7_pre's words (the same tests as tcp_l7 / udp_l7 / sip_key)
__device__ __forceinline__ void fast_l7(const Pkt& p, Fast& f, uint32_t cap, const L7Pre& pre)
{
	const bool payload = f.payload() != 0, tcp = f.tcp() != 0;
	const uint32_t l4o = f.l4o(), l4dlen = f.l4dlen();
	uint32_t lf = 0;
	if (payload && f.l4())
	{
		const uint32_t pw = lds_u32(p, l4o);
		const uint32_t sport = swap16(pw), dport = swap16(pw >> 16);
		const uint32_t pb = ((pre.ws >> (sport & 31)) | (pre.wd >> (dport & 31))) & 1u;
		bool sip = false;
		if (!tcp && l4dlen - 8 >= 4)
		{
			const uint32_t k = __builtin_bswap32(lds_u32(p, l4o + 8)), h = (k * kSipMul) >> 27;
			sip = ((kSip.valid >> h) & 1u) && pre.sk == k;
		}
		const uint32_t pr = (sport << 16) | dport;  // DHCP 68->67, 67->68, 67->67
		const bool dhcp = pr == ((68u << 16) | 67u) || pr == ((67u << 16) | 68u) || pr == ((67u << 16) | 67u);
		const bool trig = tcp ? pb != 0 : (pb != 0 || dhcp || ((pre.wu >> (dport & 31)) & 1u) || sip);
		if (trig)
			lf = l7_flags(p, tcp, l4o + f.l4hdr(), l4dlen - f.l4hdr(), sport, dport, sip, true);
	}
	const bool l7 = lf != 0;
	const uint32_t end = f.trailer();
	const uint32_t tl = (!l7 && end < cap) ? cap - end : 0;
	f.d = (f.d & 0xFFFF) | (tl << 16);
	f.e = (f.e & ~2u) | ((payload && !l7) ? 2u : 0u) | (lf << 16);
}

// layer indexes of a fast-path packet: IP1 at k1; GRE and IP2 after it; the L4 layer at kl
__device__ __forceinline__ uint32_t fast_k1(const Fast& f)
{
	return 1 + f.nv() + f.nm();
}

// The deep-stack pre-scan of a packet's first LDS window: Ethernet, up to two VLAN tags, then an MPLS label or an IP
// layer not followed directly by TCP / UDP (GRE, IPv6 extension headers, ...) -- the stacks the two-round window is for.
// *et / *o: the ethertype and offset after the VLAN tags.
__device__ __forceinline__ bool deep_stack(const Pkt& p, uint32_t* et_out, uint32_t* o_out)
{
	uint32_t et = swap16(lds_u32(p, 12)), o = 14;
#pragma unroll
	for (int t = 0; t < 2; ++t)
	{
		const bool vl = (et == 0x8100 || et == 0x88A8) && o + 8 <= p.lim;
		const uint32_t e2 = swap16(lds_u32(p, vl ? o : 0) >> 16);
		et = vl ? e2 : et;
		o = vl ? o + 4 : o;
	}
	// the IPv6 next header (byte 6) under o + 8 <= lim, the IPv4 protocol (byte 9) under o + 10 <= lim: never a byte past
	// the staged window (window_sample_kernel leaves the chunks past a short frame unwritten)
	const uint32_t ipw = lds_u32(p, o + 8 <= p.lim ? o + 4 : 0), ipv = lds_u32(p, o + 10 <= p.lim ? o + 8 : 0);
	const uint32_t nh = et == 0x86DD ? (ipw >> 16) & 0xFF : (ipv >> 8) & 0xFF;
	*et_out = et;
	*o_out = o;
	return et == 0x8847 || ((et == 0x0800 || et == 0x86DD) && nh != 6 && nh != 17);
}

// the Walk summary of a fast-path packet
__device__ __forceinline__ Walk fast_to_walk(const Fast& f, uint32_t ml)
{
	const uint32_t cap_layers = ml ? ml : PCPPX_MAX_LAYERS;
	const uint32_t gre = f.gre(), v6a = f.v6a(), v6b = f.v6b(), l4 = f.l4(), tcp = f.tcp(), payload = f.payload();
	const uint32_t trailer = f.trailer();
	const uint32_t k1 = fast_k1(f), kl = k1 + 1 + 2 * gre;
	const uint32_t count = kl + l4 + payload + (trailer ? 1 : 0);
	Walk w;
	w.flags = f.l7() | (trailer ? PCPPX_F_TRAILER : 0) | (count > cap_layers ? PCPPX_F_DEPTH_OVERFLOW : 0);
	w.n_layers = count > cap_layers ? cap_layers : count;
	w.mask = (1ull << P_ETH) | (f.nv() ? (1ull << P_VLAN) : 0) | (f.nm() ? (1ull << P_MPLS) : 0) |
	         (1ull << (v6a ? P_IPV6 : P_IPV4)) | (gre ? (1ull << P_GREV0) | (1ull << (v6b ? P_IPV6 : P_IPV4)) : 0) |
	         (l4 ? (1ull << (tcp ? P_TCP : P_UDP)) : 0) | (payload ? (1ull << P_PAYLOAD) : 0) |
	         (trailer ? (1ull << P_TRAILER) : 0);
	// the first IPv4 / IPv6 layers (hash5Tuple's addresses, the IPv4 checksum)
	const bool v4b = gre && !v6b;
	w.v4 = !v6a ? (int32_t)f.o1() : (v4b ? (int32_t)f.o2() : -1);
	w.v6 = v6a ? (int32_t)f.o1() : ((gre && v6b) ? (int32_t)f.o2() : -1);
	w.v4_dlen = !v6a ? f.d1() : f.d2();
	w.l4i = l4 ? (int32_t)kl : -1;
	w.l4o = f.l4o();
	w.l4dlen = f.l4dlen();
	const bool lv6 = gre ? v6b : v6a;
	w.l4pp = lv6 ? P_IPV6 : P_IPV4;
	w.l4ppo = gre ? f.o2() : f.o1();
	w.is_tcp = tcp;
	return w;
}

// the layer records of a fast-path packet in chain order, at most ml of them: sink(k, record) for k = 0, 1, ... (one
// predicated store per possible layer instead of a select chain per record slot)
template <class Sink>
__device__ __forceinline__ void fast_emit(const Fast& f, uint32_t cap, uint32_t ml, Sink sink)
{
	const uint32_t nv = f.nv(), nm = f.nm(), gre = f.gre(), l4 = f.l4(), payload = f.payload(), tl = f.trailer();
	const uint32_t o1 = f.o1(), h1 = f.h1(), d1 = f.d1(), o2 = f.o2(), h2 = f.h2(), d2 = f.d2();
	const uint32_t lasto = gre ? o2 : o1, lasth = gre ? h2 : h1, lastd = gre ? d2 : d1;
	uint32_t k = 0;
	auto emit = [&](bool on, uint32_t proto, uint32_t osi, uint32_t o, uint32_t hdr, uint32_t dlen) {
		if (on && k < ml)
			sink(k, make_uint2(proto | (osi << 8) | (o << 16), (hdr & 0xFFFF) | (dlen << 16)));
		k += on ? 1u : 0u;
	};
	emit(true, P_ETH, 2, 0, 14, cap);
	emit(nv > 0, P_VLAN, 2, 14, 4, cap - 14);
	emit(nv > 1, P_VLAN, 2, 18, 4, cap - 18);
	const uint32_t mo = 14 + 4 * nv;  // MPLS labels follow the tags
	emit(nm > 0, P_MPLS, 3, mo, 4, cap - mo);
	emit(nm > 1, P_MPLS, 3, mo + 4, 4, cap - mo - 4);
	emit(nm > 2, P_MPLS, 3, mo + 8, 4, cap - mo - 8);
	emit(true, f.v6a() ? P_IPV6 : P_IPV4, 3, o1, h1, d1);
	emit(gre != 0, P_GREV0, 3, o1 + h1, f.gh(), d1 - h1);
	emit(gre != 0, f.v6b() ? P_IPV6 : P_IPV4, 3, o2, h2, d2);
	emit(l4 != 0, f.tcp() ? P_TCP : P_UDP, 4, f.l4o(), f.l4hdr(), f.l4dlen());
	const uint32_t po = l4 ? f.l4o() + f.l4hdr() : lasto + lasth, pl = l4 ? f.l4dlen() - f.l4hdr() : lastd - lasth;
	emit(payload != 0, P_PAYLOAD, 7, po, pl, pl);
	emit(tl != 0, P_TRAILER, 2, lasto + lastd, tl, tl);
}

// the same inputs of a fast-path packet: every byte in the LDS window
__device__ __forceinline__ HashIn hash_in_fast(const Pkt& p, const Fast& f, const Walk& w)
{
	HashIn h;
	const bool v4 = w.v4 >= 0;
	const uint32_t ipo = v4 ? (uint32_t)w.v4 : (uint32_t)w.v6;
	const uint32_t na = v4 ? 1 : 4;
	const uint32_t so = ipo + (v4 ? 12 : 8), dofs = ipo + (v4 ? 16 : 24);
#pragma unroll
	for (int k = 0; k < 4; ++k)
	{
		h.s[k] = (uint32_t)k < na ? lds_u32(p, so + 4 * k) : 0u;
		h.d[k] = (uint32_t)k < na ? lds_u32(p, dofs + 4 * k) : 0u;
	}
	const uint32_t proto = (lds_u32(p, ipo + (v4 ? 8 : 4)) >> (v4 ? 8 : 16)) & 0xFF;
	const bool l4 = f.l4() != 0;  // TCP / UDP only: no ICMP on the fast path
	h.pw = l4 ? lds_u32(p, f.l4o()) : 0u;
	h.meta = proto | (v4 ? 0x100u : 0x200u) | (l4 ? 0xC00u : 0u);
	return h;
}

// hash5Tuple x2 + hash2Tuple of a fast-path packet (every byte in the LDS window): the first IPv4 (else the first
// IPv6) layer's addresses and protocol / next-header byte, the L4 layer's ports
template <bool kBranchy = false, bool kV4Skip = false>
__device__ __forceinline__ void fast_hashes(const Pkt& p, const Fast& f, const Walk& w, uint32_t& h5, uint32_t& h5d,
                                            uint32_t& h2)
{
	uint32_t s[4], d[4];
	const bool v4 = w.v4 >= 0;
	const uint32_t ipo = v4 ? (uint32_t)w.v4 : (uint32_t)w.v6;
	const uint32_t na = v4 ? 1 : 4;
	const uint32_t so = ipo + (v4 ? 12 : 8), dofs = ipo + (v4 ? 16 : 24);
#pragma unroll
	for (int k = 0; k < 4; ++k)
	{
		s[k] = (uint32_t)k < na ? lds_u32(p, so + 4 * k) : 0;
		d[k] = (uint32_t)k < na ? lds_u32(p, dofs + 4 * k) : 0;
	}
	const uint32_t proto = (lds_u32(p, ipo + (v4 ? 8 : 4)) >> (v4 ? 8 : 16)) & 0xFF;
	tuple_hashes<kBranchy, kV4Skip>(s, d, na, f.l4() != 0, lds_u32(p, f.l4o()), proto, h5, h5d, h2);
}

// IPv4 header checksum of the first IPv4 layer, from dword reads of the (fully staged) header
__device__ __forceinline__ uint32_t fast_ipv4_checksum(const Pkt& p, const Walk& w, uint32_t* stored)
{
	const uint32_t o = (uint32_t)w.v4;
	const uint32_t hl = (lds_u32(p, o) & 0xF) * 4;  // <= dataLen: the fast path only takes IP layers with a successor
	uint32_t acc = 0;
	for (uint32_t t = 0; t < hl; t += 4)
		acc += halves(lds_u32(p, o + t));
	const uint32_t w5 = lds_u32(p, o + 8) >> 16;  // bytes 10-11 as a LE word
	*stored = swap16(w5);
	uint32_t r = (mod65535(acc) + 65535u - mod65535(w5)) % 65535u;
	return finish_checksum(r);
}

// ---- reassembly front ends (include/pcppx.h pcppx_reasm_device) ----
// Lane per packet over the parse records: the stateless half of IPReassembly::processPacket
// (IPReassembly.cpp:284-322) and TcpReassembly::reassemblePacket (TcpReassembly.cpp:96-136). Restated
// identically in oracle/pcppx_oracle.c (reasm_packet), which pins it against the reference.
struct ReasmParams
{
	const uint8_t* data;
	const uint64_t* offsets;
	const pcppx_summary* summary;
	const pcppx_layer* layers;
	uint32_t n, ml;
	pcppx_reasm_info* info;
};

__device__ __forceinline__ uint32_t fnv_bytes(uint32_t h, const uint8_t* p, uint32_t n)
{
	for (uint32_t j = 0; j < n; ++j)
		h = fnv(h, p[j]);
	return h;
}

// One packet's reassembly record from its summary flags, n_layers and layer records (lay: max_layers
// entries) and its bytes (pkt): shared by reasm_kernel and the tile kernel's fused output.
__device__ uint4 reasm_one(uint32_t sflags, uint32_t n_layers, const pcppx_layer* lay, uint32_t ml, const uint8_t* pkt)
{
	const uint32_t nl = n_layers < ml ? n_layers : ml;
	int v4 = -1, v6 = -1, tcp = -1;
	uint32_t last = 0;
	for (uint32_t k = 0; k < nl; ++k)
	{
		const uint32_t pr = lay[k].proto;
		v4 = (pr == P_IPV4 && v4 < 0) ? (int)k : v4;
		v6 = (pr == P_IPV6 && v6 < 0) ? (int)k : v6;
		tcp = pr == P_TCP ? (int)k : tcp;
		last = pr;
	}
	// the chain is unfinished unless every layer the reassemblers look at is on the device (pcppx.h)
	bool unfinished = (sflags & (PCPPX_F_NEEDS_HOST_PROTO | PCPPX_F_OVERSIZE | PCPPX_F_BAD_DESC |
	                               PCPPX_F_DEPTH_OVERFLOW)) != 0;
	unfinished = unfinished || ((sflags & PCPPX_F_NEEDS_HOST_L7) && !(nl > 0 && last == P_TCP));
	uint32_t key = 0, fid = 0, foff = 0, ips, ts, pay = 0;
	if (v4 >= 0)
	{
		// IPv4 wrapper (IPReassembly.cpp:68-140): isFragment / getFragmentOffset (IPv4Layer.cpp:415-438)
		const pcppx_layer L = lay[v4];
		const uint8_t* ip = pkt + L.offset;
		const uint32_t b6 = ip[6], fo = ((b6 & 0x1F) << 8) | ip[7];
		const bool more = (b6 & 0x20) != 0;
		if (!more && fo == 0)
			ips = PCPPX_IPR_NON_FRAGMENT;
		else if (L.hdr_len > L.data_len)  // getLayerPayloadSize() > getDataLen() (:315-320)
			ips = PCPPX_IPR_MALFORMED;
		else
		{
			ips = PCPPX_IPR_FRAGMENT | (fo == 0 ? PCPPX_IPR_F_FIRST : 0) | (!more ? PCPPX_IPR_F_LAST : 0);
			fid = ((uint32_t)ip[4] << 8) | ip[5];
			foff = (fo * 8) & 0xFFFF;
			key = fnv_bytes(fnv_bytes(fnv_bytes(2166136261u, ip + 12, 4), ip + 16, 4), ip + 4, 2);  // :103-115
		}
	}
	else if (unfinished)
		ips = PCPPX_IPR_HOST;
	else if (v6 >= 0)
	{
		// IPv6 wrapper (IPReassembly.cpp:142-231): the first fragmentation extension of the list
		// parseExtensions built (IPv6Layer.cpp:79-147), replayed up to the recorded header length
		const pcppx_layer L = lay[v6];
		const uint8_t* ip = pkt + L.offset;
		uint32_t nh = ip[6], eo = 40, fe = 0;
		bool have = false;
		while (eo < L.hdr_len)
		{
			if (nh == 44 && !have)
			{
				have = true;
				fe = eo;
			}
			const uint32_t el = nh == 51 ? 4u * ((uint32_t)ip[eo + 1] + 2) : 8u * ((uint32_t)ip[eo + 1] + 1);
			nh = ip[eo];
			eo += el;
		}
		if (!have)
			ips = PCPPX_IPR_F_IPV6 | PCPPX_IPR_NON_FRAGMENT;
		else if (L.hdr_len > L.data_len)
			ips = PCPPX_IPR_F_IPV6 | PCPPX_IPR_MALFORMED;
		else
		{
			const uint8_t* f = ip + fe;  // ip6_frag: next header, reserved, offset+flags, id (IPv6Extensions.h)
			const uint32_t off = ((uint32_t)f[2] << 8) | (f[3] & 0xF8u);  // IPv6Extensions.cpp:87-91
			ips = PCPPX_IPR_F_IPV6 | PCPPX_IPR_FRAGMENT | (off == 0 ? PCPPX_IPR_F_FIRST : 0) |
			      ((f[3] & 1) ? 0 : PCPPX_IPR_F_LAST);
			fid = ((uint32_t)f[4] << 24) | ((uint32_t)f[5] << 16) | ((uint32_t)f[6] << 8) | f[7];
			foff = off;
			key = fnv_bytes(fnv_bytes(fnv_bytes(2166136261u, ip + 8, 16), ip + 24, 16), f + 4, 4);  // :190-205
		}
	}
	else
		ips = PCPPX_IPR_NON_IP;
	if (unfinished)
		ts = PCPPX_TCPR_HOST;
	else if (v4 < 0 && v6 < 0)
		ts = PCPPX_TCPR_NON_IP;
	else if (tcp < 0)
		ts = PCPPX_TCPR_NON_TCP;
	else
	{
		const pcppx_layer L = lay[tcp];
		const uint32_t fl = pkt[L.offset + 13];  // FIN bit 0, SYN bit 1, RST bit 2 (TcpLayer.h:30-52)
		pay = (uint32_t)L.data_len - L.hdr_len;
		ts = ((pay == 0 && (fl & 7) == 0) ? PCPPX_TCPR_NO_DATA : PCPPX_TCPR_DATA) | ((fl & 1) ? PCPPX_TCPR_F_FIN : 0) |
		     ((fl & 2) ? PCPPX_TCPR_F_SYN : 0) | ((fl & 4) ? PCPPX_TCPR_F_RST : 0);
	}
	return make_uint4(key, fid, foff | (ips << 16) | (ts << 24), pay);
}

__global__ __launch_bounds__(kBlock) void reasm_kernel(ReasmParams rp)
{
	const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
	if (i >= rp.n)
		return;
	const pcppx_summary sm = rp.summary[i];
	// read only below a recorded layer: the descriptor was checked by the parse
	reinterpret_cast<uint4*>(rp.info)[i] = reasm_one(sm.flags, sm.n_layers, rp.layers + (size_t)i * rp.ml, rp.ml,
	                                                 rp.data + rp.offsets[i]);
}

// ================= tile kernel: one wave = one tile of 64 consecutive packets =================
//
// (1) descriptors, coalesced; (2) each packet's first 112 B gathered into LDS with 8 lanes per packet
// (one 16-B piece each: 8 packets per wave-instruction instead of 64 scattered lines); (3) lane-per-
// packet chain walk, hashes and IPv4 checksum out of LDS; (4) the L4 checksums: the wave streams the
// tile's byte span once with coalesced 16-B-per-lane loads, turns each 16-B chunk into its sum of
// 16-bit halves and a wave-wide inclusive prefix (DPP scan) into an LDS window; every packet lane
// then takes the sum of its whole-chunk L4 range as a difference of two prefixes and adds its two
// partial edge chunks. The ones'-complement sum only needs the byte-order fix-up for an odd L4
// start at the very end (a multiply by 256 mod 65535).
constexpr int kTile = 64;

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x)
{
	// Hillis-Steele inside 16-lane rows, then row broadcasts (wave64 on a GFX9-family target)
	x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false);  // row_shr:1
	x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false);  // row_shr:2
	x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false);  // row_shr:4
	x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false);  // row_shr:8
	x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);  // row_bcast:15
	x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);  // row_bcast:31
	return x;
}

// min / max / sum of one value per lane by DPP (row_shr 1/2/4/8 inside 16-lane rows, then the row broadcasts): lane 63
// ends with the whole wave's, read into an SGPR -- no LDS round trips (the ds_bpermute butterflies of wave_min_u64 & co.
// wait on LDS at every one of their six steps)
template <class Op>
__device__ __forceinline__ uint32_t wave_reduce_dpp(uint32_t x, uint32_t ident, Op op)
{
	x = op(x, (uint32_t)__builtin_amdgcn_update_dpp((int)ident, (int)x, 0x111, 0xF, 0xF, false));  // row_shr:1
	x = op(x, (uint32_t)__builtin_amdgcn_update_dpp((int)ident, (int)x, 0x112, 0xF, 0xF, false));  // row_shr:2
	x = op(x, (uint32_t)__builtin_amdgcn_update_dpp((int)ident, (int)x, 0x114, 0xF, 0xF, false));  // row_shr:4
	x = op(x, (uint32_t)__builtin_amdgcn_update_dpp((int)ident, (int)x, 0x118, 0xF, 0xF, false));  // row_shr:8
	x = op(x, (uint32_t)__builtin_amdgcn_update_dpp((int)ident, (int)x, 0x142, 0xA, 0xF, false));  // row_bcast:15
	x = op(x, (uint32_t)__builtin_amdgcn_update_dpp((int)ident, (int)x, 0x143, 0xC, 0xF, false));  // row_bcast:31
	return (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
}

__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v)
{
	for (int m = 32; m >= 1; m >>= 1)
	{
		uint64_t o = __shfl_xor(v, m, 64);
		v = o < v ? o : v;
	}
	return v;
}
__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v)
{
	for (int m = 32; m >= 1; m >>= 1)
	{
		uint64_t o = __shfl_xor(v, m, 64);
		v = o > v ? o : v;
	}
	return v;
}
__device__ __forceinline__ uint64_t uniform_u64(uint64_t v)
{
	const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
	const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
	return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v)
{
	for (int m = 32; m >= 1; m >>= 1)
		v += __shfl_xor(v, m, 64);
	return v;
}

// masked halves-sum of the bytes [lo, hi) of one 16-B chunk (LDS copy if staged, else HBM)
__device__ __forceinline__ uint32_t edge_sum(const Pkt& p, uintptr_t lo, uintptr_t hi)
{
	if (hi <= lo)
		return 0;
	const uintptr_t c = lo & ~(uintptr_t)15;
	const uint32_t ci = (uint32_t)((c - p.a0) >> 4);
	uint4 v;
	if (ci < p.nch && (p.a0 & 15) == 0)  // a re-gathered deep window starts at a dword: its chunks are not memory's
	{
		lptr32 w = reinterpret_cast<lptr32>(p.s) + ci * 4;
		v = make_uint4(w[0], w[1], w[2], w[3]);
	}
	else
		v = ld16(c);
	return chunk_sum(v, c, lo, hi);
}

// halves-sum of whole chunks [c0, c1) straight from HBM (fallback for tiles whose span is not packed)
__device__ uint32_t full_chunks_sum(uintptr_t c0, uintptr_t c1)
{
	uint32_t acc = 0;
	uintptr_t c = c0;
	for (; c + 64 <= c1; c += 64)
	{
		uint4 v0 = ld16(c), v1 = ld16(c + 16), v2 = ld16(c + 32), v3 = ld16(c + 48);
		acc += halves(v0.x) + halves(v0.y) + halves(v0.z) + halves(v0.w) + halves(v1.x) + halves(v1.y) +
		       halves(v1.z) + halves(v1.w) + halves(v2.x) + halves(v2.y) + halves(v2.z) + halves(v2.w) +
		       halves(v3.x) + halves(v3.y) + halves(v3.z) + halves(v3.w);
	}
	for (; c < c1; c += 16)
	{
		uint4 v = ld16(c);
		acc += halves(v.x) + halves(v.y) + halves(v.z) + halves(v.w);
	}
	return acc;
}

// The header extent of a deep stack, from the first gather window: where fast_walk stops reading (the L4 layer's
// first 20 bytes: TCP's fixed header, UDP's header + the SIP heuristic's 4 payload bytes) for up to three MPLS
// labels, IPv6 extension headers and GREv0 + an inner IP layer -- the same steps as fast_walk, without its validity
// checks (a too-short window only sends a packet to the generic walk, which reads on from HBM). Any stack it cannot
// follow inside the window, or one that does not end in TCP / UDP / a fragment, asks for the whole window (0xFFFF).
// et / o: the EtherType and offset after the VLAN tags.
__device__ __forceinline__ uint32_t deep_extent(const Pkt& p, uint32_t et, uint32_t o)
{
#pragma unroll
	for (int t = 0; t < 3; ++t)
	{
		const bool ml = et == 0x8847 && o + 5 <= p.lim;
		const uint32_t w = lds_u32(p, ml ? o : 0), nb = (lds_u32(p, ml ? o + 4 : 0) & 0xFF) >> 4;
		const uint32_t nxt = ((w >> 16) & 1) ? (nb == 4 ? 0x0800u : (nb == 6 ? 0x86DDu : 0xFFFFu)) : 0x8847u;
		et = ml ? nxt : et;
		o = ml ? o + 4 : o;
	}
	const bool v6 = et == 0x86DD;
	bool ok = (et == 0x0800 || v6) && o + (v6 ? 40 : 20) <= p.lim;
	const uint32_t w0 = lds_u32(p, ok ? o : 0), w1 = lds_u32(p, ok ? o + 4 : 0), w2 = lds_u32(p, ok ? o + 8 : 0);
	uint32_t hdr = v6 ? 40u : (w0 & 0xF) * 4;
	uint32_t nh = v6 ? (w1 >> 16) & 0xFF : (w2 >> 8) & 0xFF;
	bool frag = !v6 && ((w1 & 0xFF3F0000u) != 0);  // IPv4 MF / fragment offset (bytes 6-7)
	constexpr uint64_t kExt = (1ull << 0) | (1ull << 43) | (1ull << 44) | (1ull << 51) | (1ull << 60);
#pragma unroll
	for (int t = 0; t < 3; ++t)
	{
		const bool e = ok && v6 && nh < 64 && ((kExt >> nh) & 1ull) && o + hdr + 2 <= p.lim;
		const uint32_t two = lds_u32(p, e ? o + hdr : 0) & 0xFFFFu;
		const uint32_t el = nh == 51 ? 4u * ((two >> 8) + 2) : 8u * ((two >> 8) + 1);
		frag = frag || (e && nh == 44);
		frag = frag && !(e && nh != 44);  // only a LAST Fragment extension makes the rest a Payload
		nh = e ? (two & 0xFFu) : nh;
		hdr += e ? el : 0u;
	}
	ok = ok && !(v6 && nh < 64 && ((kExt >> nh) & 1ull));
	uint32_t l4 = o + hdr;
	const bool g = ok && !frag && nh == 47;
	ok = ok && (!g || l4 + 4 <= p.lim);
	const uint32_t gw = lds_u32(p, g && ok ? l4 : 0);
	const uint32_t f0 = gw & 0xFF, f1 = (gw >> 8) & 0xFF, get = swap16(gw >> 16);
	const uint32_t gh = 4 + ((f0 & 0xC0) ? 4 : 0) + ((f0 & 0x20) ? 4 : 0) + ((f0 & 0x10) ? 4 : 0) + ((f1 & 0x80) ? 4 : 0);
	const uint32_t o2 = l4 + gh;
	const bool v6b = get == 0x86DD;
	ok = ok && (!g || ((get == 0x0800 || v6b) && o2 + 10 <= p.lim));
	const uint32_t i0 = lds_u32(p, g && ok ? o2 : 0), i1 = lds_u32(p, g && ok ? o2 + 4 : 0), i2 = lds_u32(p, g && ok ? o2 + 8 : 0);
	l4 = g ? o2 + (v6b ? 40u : (i0 & 0xF) * 4) : l4;
	nh = g ? (v6b ? (i1 >> 16) & 0xFF : (i2 >> 8) & 0xFF) : nh;
	ok = ok && (frag || nh == 6 || nh == 17);
	return ok ? l4 + 20 : 0xFFFFu;
}

constexpr uint32_t kRowMaxMl = 12;  // layer rows staged in LDS up to this max_layers; beyond, direct stores

// The shape switches of one parse_tile_kernel instance. The product instances use ParseShape<> (below: only the
// checksum instance of PCPPX_WINDOW_DEEP differs, in EarlyB); the diagnostics exist for tools/ab/libpcppx_ab.so only.
//   NT: non-temporal record stores (write-once data; profiles/r01_ab_nontemporal.txt); the span-stream loads use the
//     default policy since round 4 (their lines are the ones the header gather reads too: config 3 -1.7%,
//     profiles/r04k_ab_cfg3.txt)
//   FillTails: the staged FIXED layer rows are zero-filled past n_layers and stored whole: full-line stores, 3.5% faster
//     on config 3 than storing only the chain's records (profiles/r02_ab_tails.txt)
//   TightR2: the second gather round reads only up to the deep stack's header extent (deep_extent) instead of the whole
//     window (profiles/r02_ab_tight_r2.txt)
//   Realign: a deep stack that ends past the window is re-gathered from a dword-aligned start (mis <= 3 instead of <= 15)
//     so that it fits (profiles/r02_ab_realign.txt)
//   EarlyB: the second span-stream window is issued with the first, before the header gather (0.8-0.9% on config 3,
//     profiles/r03_ab_earlyB_*.txt)
//   diagnostics (wrong or marked records; static_assert'ed out of libpcppx.so): StreamOnly (no header gather / parse;
//     L4 range = [14, caplen)), MarkFast (flags bit 0x8000 on the packets the fast path took), GatherOnly (descriptors,
//     both gather rounds for every packet and the record stores, no parse: the memory time of the access pattern),
//     SkipGeneric (packets off the fast path are not walked: the time the generic walk costs), Skip (a fast-path stage
//     left out, for its cost: bit 0 the hashes, bit 1 the L7 decision, bit 2 the layer rows; bit 3: the L7 table reads
//     after the hashes instead of before; bit 4: non-temporal span-stream loads (rounds 1-3) instead of default-policy
//     ones; bit 5:
//     the IPv6 address dwords hashed under branches instead of selects; records unchanged by bits 3-5; bit 6: only the
//     first half of a PACKED run stored)
//   R6 (round 6, records unchanged by every bit): bit 0 the tile span from 32-bit DPP reductions (wave_reduce_dpp)
//     instead of 64-bit ds_bpermute butterflies; bit 1 the three hashes taken by the whole wave after both walks
//     (wave_tuple_hashes: IPv4 packets in their own lanes, IPv6 packets' chains spread over the wave's lanes); bit 2 the
//     L7 trigger ports looked up in register tables by ds_bpermute (l7_pre_regs) instead of constant-memory bitmaps;
//     bit 3 (with bit 1 off) the per-lane hashes skip the IPv6 address dwords in waves of IPv4 packets (tuple_hashes);
//     bit 4 the span stream issues no window loads past the tile's last window
template <bool kNT = true, bool kFillTails = true, bool kTightR2 = true, bool kRealign = true, bool kEarlyB = true,
          bool kStreamOnly = false, bool kMarkFast = false, bool kGatherOnly = false, bool kSkipGeneric = false,
          int kSkip = 0, int kR6 = 28>
struct ParseShape
{
	static constexpr bool NT = kNT, FillTails = kFillTails, TightR2 = kTightR2, Realign = kRealign, EarlyB = kEarlyB;
	static constexpr bool StreamOnly = kStreamOnly, MarkFast = kMarkFast, GatherOnly = kGatherOnly,
	                      SkipGeneric = kSkipGeneric;
	static constexpr int Skip = kSkip, R6 = kR6;
};

// One wave = one 64-packet tile. MinWaves: __launch_bounds__ minimum waves per SIMD (1 = the compiler's choice).
// SWin: span-stream window in 16-B chunks (SWin/64 wave-loads in flight per buffer, two buffers). Chunks: 16-B header
// chunks a packet's LDS window holds (the stage: 64 slots of 4 * Chunks + 1 dwords). Csum: the instance computes
// checksums when the launch asks (false: a parse-only instance, no span stream). Chunks1 < Chunks: a two-round
// gather: first min(packet, Chunks1) chunks for every packet, then up to Chunks for the packets the fast path could not
// take from the first window (deep stacks).
template <int MinWaves, int SWin, int Chunks, bool Csum, int Chunks1, class S = ParseShape<>>
__global__ __launch_bounds__(kTile, MinWaves) void parse_tile_kernel(Params prm)
{
	constexpr int kTSlotDw = 4 * Chunks + 1;  // + 1 pad dword against bank conflicts
	// stage doubles as the layer-record staging area at the end (64 rows x (ml+1) padded records x 8 B)
	__shared__ uint32_t stage[kTile * kTSlotDw];
	__shared__ uint64_t m_a0[kTile];
	__shared__ uint32_t m_nch[kTile];  // gather range of each packet: chunks [bits 8-15, bits 0-7)
	// layer rows staged in LDS up to this max_layers (a row = ml + 1 padded 8-B records); beyond, direct stores
	constexpr uint32_t kRowMl = (uint32_t)kTSlotDw / 2 - 1 < kRowMaxMl ? (uint32_t)kTSlotDw / 2 - 1 : kRowMaxMl;
	static_assert(kTile * (kRowMl + 1) * 2 <= kTile * kTSlotDw, "stage too small for layer rows");
	static_assert(Chunks1 <= Chunks && Chunks < 256, "gather rounds");
	// PCPPX_LAYOUT_PACKED stages a tile's chains (kTile * PCPPX_PACKED_MAX_LAYERS entries) in the stage
	constexpr bool kPackedOk = kTSlotDw >= 2 * PCPPX_PACKED_MAX_LAYERS;
#ifndef PCPPX_TOOLS_AB
	// the diagnostic switches write wrong or marked records: only tools/ab/libpcppx_ab.so (built with PCPPX_TOOLS_AB)
	// may instantiate them, never libpcppx.so; and every product instance can stage a PACKED run
	static_assert(!S::MarkFast && !S::GatherOnly && !S::SkipGeneric && !S::StreamOnly && S::Skip == 0,
	              "tools-only parse_tile_kernel switch");
	static_assert(kPackedOk, "a product instance must stage PCPPX_LAYOUT_PACKED rows");
#endif
	constexpr bool NT = S::NT, StreamOnly = S::StreamOnly, MarkFast = S::MarkFast, FillTails = S::FillTails,
	               GatherOnly = S::GatherOnly, SkipGeneric = S::SkipGeneric, TightR2 = S::TightR2, Realign = S::Realign;
	const bool want_csum = Csum && prm.want_csum;  // uniform

	const uint32_t lane = threadIdx.x;
	const uint32_t i = blockIdx.x * kTile + lane;
	const bool in = i < prm.n;
	const uint64_t off = in ? prm.offsets[i] : 0;
	const uint32_t cap = in ? prm.caplens[i] : 0;
	bool empty = true;
	const uint32_t bad = in ? desc_flags(off, cap, prm.data_len, &empty) : 0;
	const bool live = in && !bad && !empty;
	// R6 bit 2: this lane's slots of the L7 register tables (one coalesced 256-B read each, issued with the descriptors)
	uint32_t l7_rt = 0, l7_rus = 0;
	if ((S::R6 & 4) && !S::StreamOnly && !S::GatherOnly)
	{
		l7_rt = kL7R.tcp[lane];
		l7_rus = kL7R.udp_sip[lane];
	}

	// ---- tile span for the L4 checksum stream: whole packets, known before the parse, so the first
	// stream window is issued now and lands while the headers are gathered and parsed ----
	const uint64_t pkt_addr = (uint64_t)(uintptr_t)prm.data + off;
	// wave reductions are uniform: moved to SGPRs so the window loop is a scalar loop
	uint64_t smin, emax, wire;
	if (S::R6 & 1)
	{
		// round 6: 32-bit DPP reductions of each packet's span against one live packet's address (wave-uniform), and
		// of the caplens (<= 65535 each: the tile's sum fits 32 bits). A span that is not within +-2 GiB of that base
		// cannot stream anyway (emax - smin <= 2 * wire + 64 KiB), so such a tile only skips the reductions.
		const uint64_t lm = __ballot(live);
		smin = ~0ull;
		emax = wire = 0;
		if (want_csum && lm)  // uniform
		{
			const int first = __builtin_ctzll(lm);
			const uint64_t base = (((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(pkt_addr >> 32), first) << 32) |
			                       (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)pkt_addr, first)) & ~15ull;
			const int64_t d0 = (int64_t)((pkt_addr & ~15ull) - base), d1 = (int64_t)(((pkt_addr + cap + 15) & ~15ull) - base);
			const bool far = live && (d0 < INT32_MIN || d0 > INT32_MAX || d1 < INT32_MIN || d1 > INT32_MAX);
			if (!__ballot(far))  // uniform
			{
				const int32_t lo = (int32_t)wave_reduce_dpp(live ? (uint32_t)(int32_t)d0 : (uint32_t)INT32_MAX, (uint32_t)INT32_MAX,
				                                            [](uint32_t a, uint32_t b) { return (int32_t)a < (int32_t)b ? a : b; });
				const int32_t hi = (int32_t)wave_reduce_dpp(live ? (uint32_t)(int32_t)d1 : (uint32_t)INT32_MIN, (uint32_t)INT32_MIN,
				                                            [](uint32_t a, uint32_t b) { return (int32_t)a > (int32_t)b ? a : b; });
				smin = base + (uint64_t)(int64_t)lo;
				emax = base + (uint64_t)(int64_t)hi;
				wire = wave_reduce_dpp(live ? cap : 0u, 0u, [](uint32_t a, uint32_t b) { return a + b; });
			}
		}
	}
	else
	{
		smin = uniform_u64(wave_min_u64(live ? (pkt_addr & ~15ull) : ~0ull));
		emax = uniform_u64(wave_max_u64(live ? ((pkt_addr + cap + 15) & ~15ull) : 0ull));
		wire = uniform_u64(wave_sum_u64(live ? cap : 0));
	}
	const bool stream = want_csum && emax > smin && emax - smin <= 2 * wire + 65536;  // uniform
	const uint32_t nchunks = stream ? (uint32_t)((emax - smin) >> 4) : 0;
	uint4 va[SWin / 64], vb[SWin / 64];
	auto load = [&](uint4 (&v)[SWin / 64], uint32_t win) {
#pragma unroll
		for (int k = 0; k < SWin / 64; ++k)
		{
			// clamped, not masked: lanes past the span re-read its last chunk (same line, no extra
			// traffic); their values lie after every prefix target, so they are inert
			const uint32_t c = win * SWin + 64 * k + lane;
			const uintptr_t a = smin + 16ull * (c < nchunks ? c : nchunks - 1);
			if (NT && (S::Skip & 16))  // diagnostic: the round 1-3 non-temporal stream loads
			{
				const u32x4 t = __builtin_nontemporal_load(reinterpret_cast<gptr16>(a));
				v[k] = make_uint4(t.x, t.y, t.z, t.w);
			}
			else
				v[k] = ld16(a);
		}
	};
	if (stream)
		load(va, 0);
	if (S::EarlyB && stream)  // both stream windows in flight during the gather and the parse
		load(vb, 1);

	// ---- (2) header gather into LDS: 8 lanes per packet, one 16-B chunk each (8 packets per wave-instruction) ----
	Pkt p;
	p.g = (gptr8)(prm.data + (live ? off : 0));
	p.a0 = (uintptr_t)p.g & ~(uintptr_t)15;
	p.mis = (uint32_t)((uintptr_t)p.g - p.a0);
	const uint32_t need = (p.mis + cap + 15) >> 4;  // chunks holding the whole packet
	p.nch = (live && !StreamOnly) ? (need < (uint32_t)Chunks1 ? need : (uint32_t)Chunks1) : 0;
	m_a0[lane] = p.a0;
	m_nch[lane] = p.nch;
	auto gather = [&]() {  // chunks [lo, hi) of every packet of the tile (m_nch)
#pragma unroll
		for (int r = 0; r < (Chunks + 7) / 8; ++r)
		{
			const uint32_t sub = (lane & 7) + 8 * r, grp = lane >> 3;
			uint4 v[8];
#pragma unroll
			for (int j = 0; j < 8; ++j)
			{
				const uint32_t q = 8 * j + grp, rg = m_nch[q];
				if (sub >= (rg >> 8) && sub < (rg & 0xFF))
					v[j] = ld16(m_a0[q] + 16 * sub);
			}
#pragma unroll
			for (int j = 0; j < 8; ++j)
			{
				const uint32_t q = 8 * j + grp, rg = m_nch[q];
				if (sub >= (rg >> 8) && sub < (rg & 0xFF))
				{
					lptr32w slot = (lptr32w)(stage) + q * kTSlotDw + 4 * sub;
					slot[0] = v[j].x;
					slot[1] = v[j].y;
					slot[2] = v[j].z;
					slot[3] = v[j].w;
				}
			}
		}
	};
	__syncthreads();
	gather();
	__syncthreads();
	p.s = reinterpret_cast<lptr8>((lptr32w)(stage) + lane * kTSlotDw);
	auto set_lim = [&]() {
		const uint32_t staged = 16 * p.nch - p.mis;
		p.lim = (live && p.nch) ? (staged < cap ? staged : cap) : 0;
	};
	set_lim();
	if (Chunks1 < Chunks)
	{
		// second round before any walk: the rest of the window for the stacks the first round cannot hold (an MPLS
		// label, or an IP layer not followed directly by TCP / UDP: GRE, IPv6 extension headers, ...), from a
		// pre-scan of the Ethernet / VLAN / IP fields of the first window
		uint32_t et, o;
		const bool deep = deep_stack(p, &et, &o);
		uint32_t full = need < (uint32_t)Chunks ? need : (uint32_t)Chunks;
		bool more = live && !StreamOnly && (deep || GatherOnly) && full > p.nch;
		uint32_t from = p.nch;  // the second round gathers chunks [from, full)
		if (TightR2 && !GatherOnly && __ballot(more))  // wave-uniform: waves without a deep stack skip the extent
		{
			// only as far as the fast path reads: the deep stack's header extent, when the first window names it
			const uint32_t ext = deep_extent(p, et, o);
			uint32_t xc = (p.mis + ext + 15) >> 4;
			// a stack ending past the 16-B-aligned window (up to 15 B of it lie before the packet), or one whose end the
			// first window does not show: this lane re-gathers its whole window from a dword-aligned start instead, so
			// that the fast path still takes it
			const bool past = ext != 0xFFFFu ? xc > (uint32_t)Chunks : (need > (uint32_t)Chunks && p.mis > 3);
			// the re-gathered window holds only 16-B pieces that lie wholly inside the packet: a piece starting at a
			// dword could otherwise run past the end of the batch buffer (the packet's tail stays readable from HBM)
			const uint32_t mis4 = (uint32_t)((uintptr_t)p.g & 3), whole4 = (mis4 + cap) >> 4;
			const bool realign = Realign && more && past && whole4 >= (uint32_t)Chunks;
			if (realign)
			{
				p.a0 = (uintptr_t)p.g - mis4;
				p.mis = mis4;
				m_a0[lane] = p.a0;
				full = (uint32_t)Chunks;
				xc = (p.mis + ext + 15) >> 4;
				from = 0;
			}
			full = xc < full ? xc : full;
			more = more && full > from;
		}
		if (__ballot(more))  // wave-uniform
		{
			m_nch[lane] = more ? (full | (from << 8)) : 0u;
			__syncthreads();
			gather();
			__syncthreads();
			p.nch = more ? full : p.nch;
			set_lim();
		}
	}
	Fast f{};
	bool fast = live && !StreamOnly && !GatherOnly && fast_walk(p, cap, prm, f);
	constexpr bool kL7Regs = (S::R6 & 4) && !StreamOnly && !GatherOnly && !(S::Skip & 8);
	constexpr bool kWaveHash = (S::R6 & 2) && !StreamOnly && !GatherOnly && !(S::Skip & 1);
	// R6 bit 2: the fast path's L7 trigger words from the register tables, by the whole wave (converged here)
	L7Pre pre_r{ 0u, 0u, 0u, 0u };
	if (kL7Regs && __ballot(fast))  // uniform
		pre_r = l7_pre_regs(p, f, fast && f.payload() && f.l4(), l7_rt, l7_rus);

	// ---- (3) chain walk, hashes, IPv4 checksum: fast path, else the generic walk ----
	const uint32_t ml = prm.max_layers;
	const bool stage_layers = prm.layers != nullptr && ml != 0;
	Walk w;
	w.flags = bad;
	w.n_layers = 0;
	w.mask = 0;
	w.v4 = w.v6 = -1;
	w.l4i = -1;
	w.l4o = w.l4dlen = 0;
	w.is_tcp = false;
	uint32_t h5 = 0, h5d = 0, h2 = 0, ipc = 0, ips = 0, l4c = 0, l4s = 0;
	if (live && StreamOnly)
	{
		w.l4i = 0;
		w.l4o = 14;
		w.l4dlen = cap > 14 ? cap - 14 : 0;
		w.is_tcp = true;
		w.l4pp = 0;
	}
	else if (live && !GatherOnly)
	{
		if (fast)
		{
			// the L7 table reads first: their latency hides behind the hashes
			L7Pre pre = kL7Regs ? pre_r : ((S::Skip & 8) ? L7Pre{ 0u, 0u, 0u, 0u } : fast_l7_pre(p, f));
			if (!(S::Skip & 1) && !kWaveHash)
				fast_hashes<(S::Skip & 32) != 0, (S::R6 & 8) != 0>(p, f, fast_to_walk(f, ml), h5, h5d, h2);
			if (S::Skip & 8)  // diagnostic: the round-3 order (table reads after the hashes)
				pre = fast_l7_pre(p, f);
			if (!(S::Skip & 2))
				fast_l7(p, f, cap, pre);
			// a classified HTTP / SSL / DNS payload or a UDP tunnel (VXLAN, GTPv1: an unclassified L7 flag): the
			// generic walk builds their layers
			const uint32_t l7 = f.l7();
			fast = !(l7 & kL7Built) && !((l7 & PCPPX_F_NEEDS_HOST_L7) && !(l7 & PCPPX_F_L7_KNOWN));
		}
		if (fast)
		{
			w = fast_to_walk(f, ml);
			if (want_csum && w.v4 >= 0)
			{
				ipc = fast_ipv4_checksum(p, w, &ips);
				w.flags |= PCPPX_F_IP_CSUM | (ipc == ips ? PCPPX_F_IP_CSUM_OK : 0);
			}
		}
		else if (!SkipGeneric)
		{
			uint2* lay_out = stage_layers ? reinterpret_cast<uint2*>(prm.layers) + (size_t)i * ml : nullptr;
			w = walk_chain<Csum ? 2 : 4>(p, cap, prm, lay_out);
			if (!kWaveHash)
				hashes<(S::R6 & 8) != 0>(p, w, h5, h5d, h2);
			if (want_csum && w.v4 >= 0)
			{
				ipc = ipv4_checksum(p, w, &ips);
				w.flags |= PCPPX_F_IP_CSUM | (ipc == ips ? PCPPX_F_IP_CSUM_OK : 0);
			}
		}
	}

	// the TCP flags byte for the fused reassembly output (the LDS stage is reused by the layer rows below)
	const uint32_t tcp_fl = (prm.reasm != nullptr && fast && f.simple() && f.tcp()) ? (uint32_t)p.s[p.mis + f.l4o() + 13] : 0u;

	// ---- (4) L4 checksums over the tile span ----
	if (want_csum)  // uniform
	{
		const bool need = live && w.l4i >= 0;
		const uintptr_t as = (uintptr_t)p.g + w.l4o, ae = as + w.l4dlen;
		const uintptr_t f0 = (as + 15) & ~(uintptr_t)15, f1 = ae & ~(uintptr_t)15;
		const bool full = need && f0 < f1;
		const bool tail = need && f0 <= f1 && f1 < ae;  // partial last chunk [f1, ae)
		uint32_t fsum = 0, tsum = 0;
		bool tail_done = false;
		if (stream)
		{
			// Stream the tile span once, 4 x 1 KiB wave-loads per window, two register windows in
			// flight. Per 64-chunk group: halves-sums -> DPP inclusive scan -> running prefix P; each
			// lane picks P(c1-1) and P(c0-1) of its own whole-chunk L4 range and its partial tail chunk
			// straight out of the owning lanes' registers (ds_bpermute), only in groups where some lane
			// needs them.
			const int32_t t0 = full ? (int32_t)((f0 - smin) >> 4) - 1 : -2;  // P(c0-1); -1 -> 0
			const int32_t t1 = full ? (int32_t)((f1 - smin) >> 4) - 1 : -2;  // P(c1-1)
			const int32_t te = tail ? (int32_t)((f1 - smin) >> 4) : -2;      // tail chunk
			uint32_t p0 = 0, p1 = 0, carry = 0;
			const uint32_t nwin = (nchunks + SWin - 1) / SWin;
			auto process = [&](uint4 (&v)[SWin / 64], uint32_t win) {
#pragma unroll
				for (int k = 0; k < SWin / 64; ++k)
				{
					const int32_t g = (int32_t)(win * SWin + 64 * k);
					const uint32_t h = halves(v[k].x) + halves(v[k].y) + halves(v[k].z) + halves(v[k].w);
					const uint32_t x = wave_incl_scan(h);
					const uint32_t pre = carry + x;
					const bool in0 = t0 >= g && t0 < g + 64, in1 = t1 >= g && t1 < g + 64;
					if (__ballot(in0 || in1))
					{
						const uint32_t q0 = __shfl(pre, (t0 - g) & 63, 64);
						const uint32_t q1 = __shfl(pre, (t1 - g) & 63, 64);
						p0 = in0 ? q0 : p0;
						p1 = in1 ? q1 : p1;
					}
					const bool ine = te >= g && te < g + 64;
					if (__ballot(ine))
					{
						const int src = (te - g) & 63;
						const uint4 d = make_uint4(__shfl(v[k].x, src, 64), __shfl(v[k].y, src, 64),
						                           __shfl(v[k].z, src, 64), __shfl(v[k].w, src, 64));
						if (ine)
						{
							tsum = chunk_sum(d, f1, f1, ae);
							tail_done = true;
						}
					}
					carry += (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
				}
			};
			// straight-line body (windows padded to an even count; loads past the span are clamped) so
			// the compiler's vmcnt accounting sees one fixed issue order: one window always in flight
			if (!S::EarlyB)
				load(vb, 1);
			for (uint32_t wi = 0; wi < nwin; wi += 2)
			{
				process(va, wi);
				// R6 bit 4: no loads past the span's last window (a tile of small packets streams 2-3 windows: the padded
				// loads of windows nwin, nwin + 1 were never consumed, yet held the wave until they returned)
				if (!(S::R6 & 16) || wi + 2 < nwin)
					load(va, wi + 2);
				process(vb, wi + 1);
				if (!(S::R6 & 16) || wi + 3 < nwin)
					load(vb, wi + 3);
			}
			if (full)
				fsum = p1 - p0;
		}
		else if (full)
			fsum = full_chunks_sum(f0, f1);
		if (need)
		{
			uint32_t acc = mod65535(fsum);
			if (f0 <= f1)
				acc += edge_sum(p, as, f0) + (tail_done ? tsum : edge_sum(p, f1, ae));
			else
				acc += edge_sum(p, as, ae);
			uint32_t r = mod65535(acc);
			if (as & 1)
				r = (r * 256u) % 65535u;
			l4c = l4_checksum(p, w, r, &l4s);
			w.flags |= PCPPX_F_L4_CSUM | (l4c == l4s ? PCPPX_F_L4_CSUM_OK : 0);
		}
	}

	// R6 bit 1: the hashes of the whole wave, after the span stream (its two register windows are dead here), from inputs
	// read out of the LDS window (intact until the layer rows below) or, past it, from HBM
	HashIn hin = hash_in_none();
	if (kWaveHash)
	{
		if (live && fast)
			hin = hash_in_fast(p, f, w);
		else if (live && !SkipGeneric)
			hin = hash_in_walk(p, w);
		wave_tuple_hashes(hin, m_nch, h5, h5d, h2);
	}

	if (in && NT && prm.summary != nullptr)
	{
		const uint32_t l4b = w.l4i >= 0 ? (uint32_t)w.l4i : 0xFFu;
		u32x4 s0, s1;
		s0.x = h5; s0.y = h5d; s0.z = h2; s0.w = w.flags | (MarkFast && fast ? 0x8000u : 0u) | (w.n_layers << 16) | (l4b << 24);
		s1.x = (uint32_t)w.mask; s1.y = (uint32_t)(w.mask >> 32); s1.z = ipc | (ips << 16); s1.w = l4c | (l4s << 16);
		u32x4* so = reinterpret_cast<u32x4*>(prm.summary + i);
		__builtin_nontemporal_store(s0, so);
		__builtin_nontemporal_store(s1, so + 1);
	}
	else if (in && prm.summary != nullptr)
		write_summary(prm.summary + i, h5, h5d, h2, w.flags, w.n_layers, w.l4i, w.mask, ipc, ips, l4c, l4s);
	// the 16-B brief: the summary's first half (hashes, flags, chain length, port layer) -- one coalesced 16-B store per
	// lane; a caller that reads the layer rows derives isPacketOfType from them and the checksum verdicts are the flags
	if (in && prm.brief != nullptr)
	{
		const uint32_t l4b = w.l4i >= 0 ? (uint32_t)w.l4i : 0xFFu;
		u32x4 s0;
		s0.x = h5; s0.y = h5d; s0.z = h2; s0.w = w.flags | (MarkFast && fast ? 0x8000u : 0u) | (w.n_layers << 16) | (l4b << 24);
		__builtin_nontemporal_store(s0, reinterpret_cast<u32x4*>(prm.brief + i));
	}
	if (in && prm.flow_keys != nullptr)
		__builtin_nontemporal_store(h5, prm.flow_keys + i);
	if (in && prm.tuples != nullptr)  // the LDS window is still intact here (the rows below reuse it)
	{
		if (kWaveHash)
			write_tuple_in(hin, w, h5, prm.tuples + i);
		else
			write_tuple(p, w, h5, prm.tuples + i);
	}
	if (prm.wave_stats != nullptr)  // uniform
		wave_proto_stats(in, w.mask, w.flags, prm.wave_stats + blockIdx.x);
	// ---- (5) layer records of fast-path packets: rows built in LDS, written with coalesced stores (whole rows,
	// zero past the chain, with FillTails; the generic walk writes only the chain's records) ----
	typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
	typedef __attribute__((address_space(3))) u32x2* lptr64w;
	// PCPPX_LAYOUT_PACKED: the tile's chains dense in LDS (entry excl + k of the lane's exclusive prefix), stored as one
	// contiguous run of entries from the tile's base (an instance that cannot stage it is refused by the launch)
	if (kPackedOk && stage_layers && prm.packed)  // uniform
	{
		const uint32_t cnt = in ? (w.n_layers < ml ? w.n_layers : ml) : 0u;
		const uint32_t incl = wave_incl_scan(cnt);
		const uint32_t excl = incl - cnt;
		const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
		u32x2* dst = reinterpret_cast<u32x2*>(prm.layers) + (size_t)blockIdx.x * kTile * ml;
		__syncthreads();  // every lane is done with the header stage
		lptr64w rows = (lptr64w)(stage);
		if (fast && !(S::Skip & 4))
			fast_emit(f, cap, ml, [&](uint32_t k, uint2 r) {
				u32x2 e;
				e.x = r.x;
				e.y = r.y;
				rows[excl + k] = e;
			});
		else
			for (uint32_t k = 0; k < cnt; ++k)  // the generic walk wrote this lane's chain at its fixed-layout slot
				rows[excl + k] = dst[lane * ml + k];
		__syncthreads();
		// (diagnostic Skip bit 6: only the first half of the run is stored -- the time's sensitivity to the row bytes)
		const uint32_t stored = (S::Skip & 64) ? total / 2 : total;
		for (uint32_t r = lane; r < stored; r += kTile)
			__builtin_nontemporal_store(rows[r], &dst[r]);
	}
	else if (stage_layers && ml > kRowMl)  // uniform: deep records, each fast lane stores its own row
	{
		if (fast)
		{
			uint2* dst = reinterpret_cast<uint2*>(prm.layers) + (size_t)i * ml;
			fast_emit(f, cap, ml, [&](uint32_t k, uint2 r) { dst[k] = r; });
		}
	}
	else if (stage_layers)  // uniform
	{
		__syncthreads();  // every lane is done with the header stage
		m_nch[lane] = (fast || GatherOnly) ? (FillTails ? ml : w.n_layers) : 0u;  // records of the row to store
		lptr64w rows = (lptr64w)(stage);
		const uint32_t rs = ml + 1;  // padded row stride (records): breaks the power-of-two bank pattern
		if (FillTails && (fast || GatherOnly))
			for (uint32_t k = 0; k < ml; ++k)
				rows[lane * rs + k] = u32x2{ 0u, 0u };
		if (fast)
			fast_emit(f, cap, ml, [&](uint32_t k, uint2 r) {
				u32x2 e;
				e.x = r.x;
				e.y = r.y;
				rows[lane * rs + k] = e;
			});
		__syncthreads();
		const uint32_t first = blockIdx.x * kTile;
		const uint32_t nrows = prm.n - first < (uint32_t)kTile ? prm.n - first : (uint32_t)kTile;
		u32x2* dst = reinterpret_cast<u32x2*>(prm.layers) + (size_t)first * ml;
		// kTile / ml rows per pass, lane -> (row, record): consecutive lanes write consecutive records
		const uint32_t per = kTile / ml, rr = lane / ml, kk = lane - rr * ml;
		for (uint32_t r0 = 0; r0 < nrows; r0 += per)
		{
			const uint32_t r = r0 + rr;
			if (rr < per && r < nrows && kk < m_nch[r])
			{
				if (NT)
					__builtin_nontemporal_store(rows[r * rs + kk], &dst[r * ml + kk]);
				else
					dst[r * ml + kk] = rows[r * rs + kk];
			}
		}
	}

	// ---- (6) fused reassembly front ends (same records as reasm_kernel): plain fast-path packets straight from
	// their parse (IPv4 not a fragment, IPv6 without extensions, the TCP flags byte read before the LDS reuse), every
	// other packet from its layer records ----
	if (prm.reasm != nullptr)  // uniform pointer
	{
		__syncthreads();  // the fast-path rows of (5) were stored by other lanes
		__threadfence_block();
	}
	if (prm.reasm != nullptr && in)
	{
		uint4 r;
		if (fast && f.simple())
		{
			const uint32_t nl = w.n_layers, ipk = 1 + f.nv(), l4k = 2 + f.nv();
			const bool unfinished = (w.flags & PCPPX_F_DEPTH_OVERFLOW) || ((w.flags & PCPPX_F_NEEDS_HOST_L7) && !f.tcp());
			const bool v4r = !f.v6a() && ipk < nl, v6r = f.v6a() && ipk < nl, tcpr = f.tcp() && l4k < nl;
			const uint32_t ipst = v4r ? PCPPX_IPR_NON_FRAGMENT
			                          : (unfinished ? PCPPX_IPR_HOST
			                                        : (v6r ? (PCPPX_IPR_F_IPV6 | PCPPX_IPR_NON_FRAGMENT) : PCPPX_IPR_NON_IP));
			uint32_t ts, pay = 0;
			if (unfinished)
				ts = PCPPX_TCPR_HOST;
			else if (!v4r && !v6r)
				ts = PCPPX_TCPR_NON_IP;
			else if (!tcpr)
				ts = PCPPX_TCPR_NON_TCP;
			else
			{
				const uint32_t fl = tcp_fl;
				pay = f.l4dlen() - f.l4hdr();
				ts = ((pay == 0 && (fl & 7) == 0) ? PCPPX_TCPR_NO_DATA : PCPPX_TCPR_DATA) |
				     ((fl & 1) ? PCPPX_TCPR_F_FIN : 0) | ((fl & 2) ? PCPPX_TCPR_F_SYN : 0) | ((fl & 4) ? PCPPX_TCPR_F_RST : 0);
			}
			r = make_uint4(0, 0, (ipst << 16) | (ts << 24), pay);
		}
		else
			r = reasm_one(w.flags, w.n_layers, prm.layers + (size_t)i * ml, ml, prm.data + off);
		reinterpret_cast<uint4*>(prm.reasm)[i] = r;
	}
}

// ---- the engine's header-window choice (pcppx_ctx, PCPPX_WINDOW_DEFAULT): a sample of the batch's stacks ----
// About 64 tiles of a batch, evenly spread (every `stride`-th tile), count their live packets and the deep stacks among
// them (deep_stack over each packet's first 48 B staged in LDS, as the parse's first window holds them: Ethernet links
// only); one wave per sampled tile, two atomics per wave into the context's counters `win`. A kernel of its own, which
// the context launches before some of its parses, so that the parse kernel carries no sampling code.
__global__ __launch_bounds__(kTile) void window_sample_kernel(Params prm, uint32_t stride, unsigned long long* win)
{
	constexpr uint32_t kCh = 3, kSlotDw = 4 * kCh + 1;  // + 1 pad dword: lds_u32's second read stays in the slot
	__shared__ uint32_t stage[kTile * kSlotDw];
	const uint32_t lane = threadIdx.x;
	const uint32_t i = blockIdx.x * stride * kTile + lane;
	const bool in = i < prm.n;
	const uint64_t off = in ? prm.offsets[i] : 0;
	const uint32_t cap = in ? prm.caplens[i] : 0;
	bool empty = true;
	const uint32_t bad = in ? desc_flags(off, cap, prm.data_len, &empty) : 0;
	const bool live = in && !bad && !empty;
	Pkt p;
	p.g = (gptr8)(prm.data + (live ? off : 0));
	p.a0 = (uintptr_t)p.g & ~(uintptr_t)15;
	p.mis = (uint32_t)((uintptr_t)p.g - p.a0);
	const uint32_t need = (p.mis + cap + 15) >> 4;  // chunks holding the whole packet (none past the batch)
	p.nch = live ? (need < kCh ? need : kCh) : 0u;
	lptr32w slot = (lptr32w)(stage) + lane * kSlotDw;
	for (uint32_t c = 0; c < kCh; ++c)
		if (c < p.nch)
		{
			const uint4 v = ld16(p.a0 + 16 * c);
			slot[4 * c] = v.x;
			slot[4 * c + 1] = v.y;
			slot[4 * c + 2] = v.z;
			slot[4 * c + 3] = v.w;
		}
	p.s = reinterpret_cast<lptr8>(slot);
	const uint32_t staged = 16 * p.nch - p.mis;
	p.lim = (live && p.nch) ? (staged < cap ? staged : cap) : 0u;
	uint32_t et, o;
	const bool dp = live && p.lim >= 14 && deep_stack(p, &et, &o);  // reads < 34 B: 48 B - 15 staged at least
	const uint32_t nl = (uint32_t)__popcll(__ballot(live)), nd = (uint32_t)__popcll(__ballot(dp));
	if (lane == 0 && nl != 0)
	{
		atomicAdd(win, (unsigned long long)nl);
		atomicAdd(win + 1, (unsigned long long)nd);
	}
}

// ---- collectStats totals: the per-wave counters of a parse (wave_proto_stats) summed into the caller's
// PCPPX_PROTO_STATS words (one 64-bit atomic per counter and block) ----
__global__ __launch_bounds__(kBlock) void proto_stats_reduce_kernel(const uint4* __restrict__ part, uint32_t nw,
                                                                  unsigned long long* out)
{
	constexpr int kC = 11;  // PCPPX_PS_PACKETS .. PCPPX_PS_NEEDS_HOST
	uint32_t a[kC];
#pragma unroll
	for (int k = 0; k < kC; ++k)
		a[k] = 0;
	// 8 independent record loads in flight per thread (128 blocks cover 262k waves = 16.7M packets in one round trip)
	constexpr uint32_t kU = 8;
	for (uint32_t b0 = blockIdx.x * kBlock * kU; b0 < nw; b0 += gridDim.x * kBlock * kU)
	{
		uint4 v[kU];
#pragma unroll
		for (uint32_t u = 0; u < kU; ++u)
		{
			const uint32_t j = b0 + u * kBlock + threadIdx.x;
			v[u] = j < nw ? part[j] : make_uint4(0, 0, 0, 0);
		}
#pragma unroll
		for (uint32_t u = 0; u < kU; ++u)
		{
			const uint32_t w[3] = { v[u].x, v[u].y, v[u].z };
#pragma unroll
			for (int k = 0; k < kC; ++k)
				a[k] += (w[k >> 2] >> (8 * (k & 3))) & 0xFFu;
		}
	}
	__shared__ unsigned long long s_part[kBlock / 64][kC];
	const uint32_t wv = threadIdx.x >> 6;
#pragma unroll
	for (int k = 0; k < kC; ++k)
	{
		const unsigned long long t = wave_sum_u64(a[k]);
		if ((threadIdx.x & 63) == 0)
			s_part[wv][k] = t;
	}
	__syncthreads();
	if (threadIdx.x < (uint32_t)kC)
	{
		unsigned long long t = 0;
		for (uint32_t q = 0; q < kBlock / 64; ++q)
			t += s_part[q][threadIdx.x];
		if (t)
			atomicAdd(&out[threadIdx.x], t);
	}
}

// ---- per-flow counters keyed by hash5Tuple (FilterTraffic's flow table, AppWorkerThread.h:99-125) ----
// A block aggregates 1024 packets at a time in an LDS hash table (LDS atomics), then adds one
// {packets, bytes} pair per distinct flow to the HBM table: Zipf-skewed traffic puts a hot flow in most
// packets of a batch, and per-packet global atomics on its slot would serialise.
// Shape variants (block threads, LDS slots, packets per batch) are A/B'd in profiles/r01_ab_flow_shape.txt;
// every shape keeps fewer packets per batch than LDS slots (hot flows kept only while kept + batch fit).
constexpr uint32_t kFlowHot = 2;                    // flows with more packets stay in LDS between flushes
constexpr uint32_t log2u(uint32_t v) { return v <= 1 ? 0 : 1 + log2u(v >> 1); }

// With `packed` (a zeroed u64 per slot, launches of < 2^24 packets) a flush adds {packets, bytes} as one
// 64-bit atomic (packets << 40 | bytes: < 2^24 packets x < 2^16 B fit 40 bits) and flow_unpack_kernel
// moves the sums into the table's own counters afterwards: one global atomic per distinct flow and flush.
// Partitioned flush (kPart): the table is split into P = 2^log2p regions by the key's top hash bits, and instead of
// global atomics on the table a block appends each distinct key of a batch, {key, packed count}, to its partition's
// record queue (one global atomic per partition per batch reserves the space); flow_merge_kernel then gives every
// partition to one block, which folds its queue in LDS and updates its own table region with plain loads and stores.
// A full queue falls back to atomics on the region.
constexpr uint32_t kFlowMaxParts = 1024;  // flow-table partitions (merge blocks) at most
struct FlowPart
{
	uint4* recs;       // P queues of rec_cap records {key, 0, packed lo, packed hi}
	uint32_t rec_cap;
	uint32_t* fill;    // P queue lengths (zero before the launch)
	uint32_t log2p;    // partitions
	uint32_t log2r;    // slots per region
};

__device__ __forceinline__ uint32_t flow_part(uint32_t key, uint32_t log2p)
{
	return log2p ? (key * 0x9E3779B1u) >> (32 - log2p) : 0u;
}
__device__ __forceinline__ uint32_t flow_region_slot(uint32_t key, uint32_t log2r)
{
	return (key * 0x85EBCA6Bu) & ((1u << log2r) - 1u);
}
// insert / find `key` in its region and add the counts with device atomics (the queue-overflow path); false: full
__device__ bool flow_region_add_atomic(uint32_t* keys, unsigned long long* packets, unsigned long long* bytes,
                                       const FlowPart& fp, uint32_t key, unsigned long long pk, unsigned long long by)
{
	const uint32_t rbase = flow_part(key, fp.log2p) << fp.log2r, rm = (1u << fp.log2r) - 1u;
	uint32_t r = flow_region_slot(key, fp.log2r);
	for (uint32_t probe = 0; probe <= rm; ++probe)
	{
		const uint32_t prev = atomicCAS(&keys[rbase + r], 0u, key);
		if (prev == 0u || prev == key)
		{
			atomicAdd(&packets[rbase + r], pk);
			atomicAdd(&bytes[rbase + r], by);
			return true;
		}
		r = (r + 1) & rm;
	}
	return false;
}

// kDense: keys come from the dense column `dkeys` (pcppx_records.flow_keys) instead of the summaries' hash5.
// kOnePass (partitioned flush): the hot-flow decision is taken in the partition pass (a hot slot is kept while the kept
// count stays within the bound, first come first kept) instead of in a pass and a barrier of its own.
template <uint32_t kFB, uint32_t kFlowLds, uint32_t kFlowBatch, uint32_t kHot = kFlowHot, bool kPrefetch = false,
          bool kPart = false, bool kDense = false, bool kOnePass = false>
__global__ __launch_bounds__(kFB) void flow_count_kernel(const pcppx_summary* __restrict__ sum,
                                                            const uint32_t* __restrict__ caplens, uint32_t n,
                                                            uint32_t* keys, unsigned long long* packets,
                                                            unsigned long long* bytes, uint32_t capacity,
                                                            unsigned long long* stats, unsigned long long* packed,
                                                            FlowPart fpart = FlowPart{}, const uint32_t* dkeys = nullptr)
{
	__shared__ uint32_t s_bin[kPart ? kFlowMaxParts : 1], s_base[kPart ? kFlowMaxParts : 1];  // per-partition counts / offsets
	__shared__ uint32_t s_key[kFlowLds];
	__shared__ unsigned long long s_cnt[kFlowLds];  // packets << 40 | bytes (launches hold < 2^24 packets)
	__shared__ uint32_t s_kept;
	const uint32_t t = threadIdx.x;
	const uint32_t m = capacity - 1;
	unsigned long long z_pk = 0, z_by = 0, lost = 0;  // flow key 0 (PacketUtils.cpp:141-148); table full
	for (uint32_t j = t; j < kFlowLds; j += kFB)
	{
		s_key[j] = 0;
		s_cnt[j] = 0;
	}
	if (kPart)
		for (uint32_t j = t; j < kFlowMaxParts; j += kFB)
			s_bin[j] = 0;
	__syncthreads();
	// kPrefetch: the next batch's keys and lengths are loaded into registers before this batch's flush,
	// so their latency overlaps the flush's HBM reads and atomics
	constexpr uint32_t kR = kFlowBatch / kFB;
	uint32_t pkey[kR], plen[kR], pvalid = 0;
	auto fetch = [&](uint64_t b) {
		pvalid = 0;
#pragma unroll
		for (uint32_t r = 0; r < kR; ++r)
		{
			const uint64_t i = b + r * kFB + t;
			pkey[r] = i < n ? (kDense ? dkeys[i] : sum[i].hash5) : 0u;
			plen[r] = i < n ? caplens[i] : 0u;
			pvalid |= (i < n ? 1u : 0u) << r;
		}
	};
	if (kPrefetch)
		fetch((uint64_t)blockIdx.x * kFlowBatch);
	for (uint64_t base = (uint64_t)blockIdx.x * kFlowBatch; base < n; base += (uint64_t)gridDim.x * kFlowBatch)
	{
#pragma unroll
		for (uint32_t r = 0; r < kR; ++r)
		{
			const uint64_t i = base + r * kFB + t;
			const bool valid = kPrefetch ? ((pvalid >> r) & 1u) != 0 : i < n;
			const uint32_t key = !valid ? 0u : (kPrefetch ? pkey[r] : (kDense ? dkeys[i] : sum[i].hash5));
			const uint32_t len = !valid ? 0u : (kPrefetch ? plen[r] : caplens[i]);
			if (valid && key == 0)  // flow key 0 (PacketUtils.cpp:141-148): counted, not tabled
			{
				z_pk += 1;
				z_by += len;
			}
			if (!valid || key == 0)
				continue;
			const unsigned long long add = (1ull << 40) | len;
			static_assert(kFlowBatch < kFlowLds && kFlowBatch % kFB == 0 && (kFlowLds & (kFlowLds - 1)) == 0, "flow shape");
			uint32_t slot = (key * 0x9E3779B1u) >> (32 - log2u(kFlowLds));  // top bits
			while (true)  // at most kFlowBatch keys in kFlowLds slots: always terminates
			{
				const uint32_t prev = atomicCAS(&s_key[slot], 0u, key);
				if (prev == 0u || prev == key)
				{
					atomicAdd(&s_cnt[slot], add);
					break;
				}
				slot = (slot + 1) & (kFlowLds - 1);
			}
		}
		if (kPrefetch)
			fetch(base + (uint64_t)gridDim.x * kFlowBatch);
		if (t == 0)
			s_kept = 0;
		__syncthreads();
		// flush: read the HBM slot of every distinct key first (all loads in flight together); present
		// keys -- every flow after its first batch -- take no-return atomics, new ones a CAS insert.
		// Hot flows (more than kFlowHot packets so far) stay in LDS until the block's last batch: every
		// block meets the top Zipf flows in every batch, and same-address atomics serialise. They are
		// kept only while they fill at most half of the table, so the next batch always fits.
		const bool last = base + (uint64_t)gridDim.x * kFlowBatch >= n;  // uniform
		constexpr uint32_t kPer = kFlowLds / kFB;
		if constexpr (kPart && kOnePass)
		{
			uint32_t fk[kPer], fs[kPer], fseen[kPer];
#pragma unroll
			for (uint32_t u = 0; u < kPer; ++u)
			{
				const uint32_t j = u * kFB + t;
				const uint32_t key = s_key[j];
				// kept only while at most half the table minus half a batch is kept, so the next batch always fits
				const bool keep = key != 0 && !last && (s_cnt[j] >> 40) > kHot &&
				                  atomicAdd(&s_kept, 1u) < kFlowLds / 2 - kFlowBatch / 2;
				fk[u] = keep ? 0u : key;
				fs[u] = flow_part(fk[u], fpart.log2p);
				fseen[u] = fk[u] ? atomicAdd(&s_bin[fs[u]], 1u) : 0u;
			}
			__syncthreads();
			for (uint32_t b = t; b < (1u << fpart.log2p); b += kFB)
			{
				const uint32_t c = s_bin[b];
				s_base[b] = c ? atomicAdd(&fpart.fill[b], c) : 0u;
				s_bin[b] = 0;
			}
			__syncthreads();
#pragma unroll
			for (uint32_t u = 0; u < kPer; ++u)
			{
				const uint32_t j = u * kFB + t;
				const uint32_t key = fk[u];
				if (key == 0)
					continue;
				const uint32_t pos = s_base[fs[u]] + fseen[u];
				const unsigned long long c = s_cnt[j];
				if (pos < fpart.rec_cap)
					fpart.recs[(size_t)fs[u] * fpart.rec_cap + pos] = make_uint4(key, 0u, (uint32_t)c, (uint32_t)(c >> 32));
				else if (!flow_region_add_atomic(keys, packets, bytes, fpart, key, c >> 40, c & ((1ull << 40) - 1)))
					lost += c >> 40;
				s_key[j] = 0;
				s_cnt[j] = 0;
			}
			__syncthreads();
			continue;
		}
		uint32_t hot = 0;
#pragma unroll
		for (uint32_t u = 0; u < kPer; ++u)
			hot |= ((s_cnt[u * kFB + t] >> 40) > kHot ? 1u : 0u) << u;
		if (!last && hot)
			atomicAdd(&s_kept, (uint32_t)__popc(hot));
		__syncthreads();
		const bool keep_hot = !last && s_kept <= kFlowLds / 2 - kFlowBatch / 2;  // uniform
		uint32_t fk[kPer], fs[kPer], fseen[kPer];
		if constexpr (kPart)
		{
			// queue every distinct key: rank within its partition (LDS), one reservation per partition (global)
#pragma unroll
			for (uint32_t u = 0; u < kPer; ++u)
			{
				const uint32_t j = u * kFB + t;
				fk[u] = (keep_hot && ((hot >> u) & 1u)) ? 0u : s_key[j];
				fs[u] = flow_part(fk[u], fpart.log2p);
				fseen[u] = fk[u] ? atomicAdd(&s_bin[fs[u]], 1u) : 0u;
			}
			__syncthreads();
			for (uint32_t b = t; b < (1u << fpart.log2p); b += kFB)
			{
				const uint32_t c = s_bin[b];
				s_base[b] = c ? atomicAdd(&fpart.fill[b], c) : 0u;
				s_bin[b] = 0;
			}
			__syncthreads();
#pragma unroll
			for (uint32_t u = 0; u < kPer; ++u)
			{
				const uint32_t j = u * kFB + t;
				const uint32_t key = fk[u];
				if (key == 0)
					continue;
				const uint32_t pos = s_base[fs[u]] + fseen[u];
				const unsigned long long c = s_cnt[j];
				if (pos < fpart.rec_cap)
					fpart.recs[(size_t)fs[u] * fpart.rec_cap + pos] = make_uint4(key, 0u, (uint32_t)c, (uint32_t)(c >> 32));
				else if (!flow_region_add_atomic(keys, packets, bytes, fpart, key, c >> 40, c & ((1ull << 40) - 1)))
					lost += c >> 40;
				s_key[j] = 0;
				s_cnt[j] = 0;
			}
			__syncthreads();
			continue;
		}
#pragma unroll
		for (uint32_t u = 0; u < kPer; ++u)
		{
			const uint32_t j = u * kFB + t;
			fk[u] = (keep_hot && ((hot >> u) & 1u)) ? 0u : s_key[j];
			fs[u] = (fk[u] * 0x9E3779B1u) & m;
			fseen[u] = fk[u] ? keys[fs[u]] : 0u;
		}
#pragma unroll
		for (uint32_t u = 0; u < kPer; ++u)
		{
			const uint32_t j = u * kFB + t;
			const uint32_t key = fk[u];
			if (key == 0)
				continue;
			uint32_t slot = fs[u];
			bool done = fseen[u] == key;  // a slot's key never changes once set: a plain read is enough
			for (uint32_t probe = 0; !done && probe < capacity; ++probe)
			{
				const uint32_t prev = atomicCAS(&keys[slot], 0u, key);
				if (prev == 0u || prev == key)
					done = true;
				else
					slot = (slot + 1) & m;
			}
			if (done && packed)
				atomicAdd(&packed[slot], s_cnt[j]);
			else if (done)
			{
				atomicAdd(&packets[slot], s_cnt[j] >> 40);
				atomicAdd(&bytes[slot], s_cnt[j] & ((1ull << 40) - 1));
			}
			else
				lost += s_cnt[j] >> 40;
			s_key[j] = 0;
			s_cnt[j] = 0;
		}
		__syncthreads();
	}
	z_pk = wave_sum_u64(z_pk);
	z_by = wave_sum_u64(z_by);
	lost = wave_sum_u64(lost);
	if ((t & 63) == 0)
	{
		if (z_pk)
		{
			atomicAdd(&stats[0], z_pk);
			atomicAdd(&stats[1], z_by);
		}
		if (lost)
			atomicAdd(&stats[2], lost);
	}
}

__global__ __launch_bounds__(kBlock) void flow_unpack_kernel(unsigned long long* packets, unsigned long long* bytes,
                                                             unsigned long long* packed, uint32_t capacity)
{
	for (uint32_t j = blockIdx.x * kBlock + threadIdx.x; j < capacity; j += gridDim.x * kBlock)
	{
		const unsigned long long v = packed[j];
		if (v)
		{
			packets[j] += v >> 40;
			bytes[j] += v & ((1ull << 40) - 1);
			packed[j] = 0;
		}
	}
}

// The merge step of the partitioned flush: block p folds partition p's queue in an LDS hash table (kPerT records per
// thread per round; flushed whenever more than half full), then adds each distinct key's counts into its own table
// region -- which no other block touches, so the counts take plain loads and stores (a CAS only claims a new key's
// slot against the block's other threads). Resets the queue length for the next launch.
// kAhead: rounds of queue records in flight ahead of the round being inserted.
template <uint32_t kMB, uint32_t kMLds, uint32_t kPerT, uint32_t kAhead = 1>
__global__ __launch_bounds__(kMB) void flow_merge_kernel(FlowPart fp, uint32_t* keys, unsigned long long* packets,
                                                         unsigned long long* bytes, unsigned long long* stats)
{
	__shared__ uint32_t s_key[kMLds];
	__shared__ unsigned long long s_cnt[kMLds];
	__shared__ uint32_t s_used;
	static_assert(kMB * kPerT <= kMLds / 4 && (kMLds & (kMLds - 1)) == 0, "merge table");
	const uint32_t t = threadIdx.x, p = blockIdx.x;
	const uint32_t cnt = fp.fill[p] < fp.rec_cap ? fp.fill[p] : fp.rec_cap;
	const uint4* q = fp.recs + (size_t)p * fp.rec_cap;
	const uint32_t rbase = p << fp.log2r, rm = (1u << fp.log2r) - 1u;
	for (uint32_t j = t; j < kMLds; j += kMB)
	{
		s_key[j] = 0;
		s_cnt[j] = 0;
	}
	if (t == 0)
		s_used = 0;
	__syncthreads();
	unsigned long long lost = 0;
	// the next kAhead rounds' records are loaded before this round's inserts (their latency hides behind them)
	static_assert(kAhead >= 1, "merge lookahead");
	uint4 nxt[kAhead][kPerT];
	auto fetch = [&](uint4 (&v)[kPerT], uint32_t base) {
#pragma unroll
		for (uint32_t k = 0; k < kPerT; ++k)
		{
			const uint32_t idx = base + k * kMB + t;
			v[k] = idx < cnt ? q[idx] : make_uint4(0, 0, 0, 0);
		}
	};
#pragma unroll
	for (uint32_t a = 0; a < kAhead; ++a)
		fetch(nxt[a], a * kMB * kPerT);
	for (uint32_t base = 0; base < cnt; base += kMB * kPerT)
	{
		uint4 rec[kPerT];
#pragma unroll
		for (uint32_t k = 0; k < kPerT; ++k)
			rec[k] = nxt[0][k];
#pragma unroll
		for (uint32_t a = 0; a + 1 < kAhead; ++a)
#pragma unroll
			for (uint32_t k = 0; k < kPerT; ++k)
				nxt[a][k] = nxt[a + 1][k];
		fetch(nxt[kAhead - 1], base + kAhead * kMB * kPerT);
#pragma unroll
		for (uint32_t k = 0; k < kPerT; ++k)
		{
			const uint32_t key = rec[k].x;
			if (key == 0)
				continue;
			// a hash independent of the partition's (a partition's keys share the top bits of key * 0x9E3779B1)
			uint32_t slot = (key * 0xC2B2AE35u) >> (32 - log2u(kMLds));
			while (true)  // the table is at most 3/4 full: terminates
			{
				const uint32_t prev = atomicCAS(&s_key[slot], 0u, key);
				if (prev == 0u || prev == key)
				{
					if (prev == 0u)
						atomicAdd(&s_used, 1u);
					atomicAdd(&s_cnt[slot], ((unsigned long long)rec[k].w << 32) | rec[k].z);
					break;
				}
				slot = (slot + 1) & (kMLds - 1);
			}
		}
		__syncthreads();
		const bool flush = base + kMB * kPerT >= cnt || s_used > kMLds / 2;  // uniform
		if (flush)
		{
			// the home slot of every distinct key is read first (all loads in flight together), then claimed / added
			constexpr uint32_t kPerF = kMLds / kMB;
			uint32_t fkey[kPerF], fr[kPerF], fprev[kPerF];
#pragma unroll
			for (uint32_t u = 0; u < kPerF; ++u)
			{
				fkey[u] = s_key[u * kMB + t];
				fr[u] = flow_region_slot(fkey[u], fp.log2r);
				fprev[u] = fkey[u] ? keys[rbase + fr[u]] : 0u;
			}
#pragma unroll
			for (uint32_t u = 0; u < kPerF; ++u)
			{
				const uint32_t j = u * kMB + t, key = fkey[u];
				if (key == 0)
					continue;
				const unsigned long long c = s_cnt[j];
				uint32_t r = fr[u], prev = fprev[u];
				bool done = false;
				for (uint32_t probe = 0; probe <= rm; ++probe)
				{
					if (probe > 0)
						prev = keys[rbase + r];
					if (prev == 0u)
						prev = atomicCAS(&keys[rbase + r], 0u, key);
					if (prev == 0u || prev == key)
					{
						packets[rbase + r] += c >> 40;
						bytes[rbase + r] += c & ((1ull << 40) - 1);
						done = true;
						break;
					}
					r = (r + 1) & rm;
				}
				if (!done)
					lost += c >> 40;
				s_key[j] = 0;
				s_cnt[j] = 0;
			}
			__syncthreads();
			if (t == 0)
				s_used = 0;
		}
		__syncthreads();
	}
	lost = wave_sum_u64(lost);
	if ((t & 63) == 0 && lost)
		atomicAdd(&stats[2], lost);
	if (t == 0)
		fp.fill[p] = 0;
}

// ---- DpdkExample-FilterTraffic's worker on the device (AppWorkerThread.h:85-139) ----
struct FilterParams
{
	const uint8_t* data;
	const uint64_t* offsets;
	const pcppx_summary* summary;
	const pcppx_layer* layers;
	uint32_t n, ml;
	uint32_t src_ip, dst_ip, src_port, dst_port, protocol;
	uint64_t seq_base;
	unsigned long long* keys;
	unsigned long long* first;
	uint32_t capacity;
	uint8_t* matched;
	unsigned long long* stats;  // pcppx_packet_stats as 14 u64
};

// PacketMatchingEngine::isMatched (PacketMatchingEngine.h:43-107) over the engine's records: the first
// IPv4 layer's addresses, the first TCP (else first UDP) layer's ports, isPacketOfType(TCP/UDP).
__device__ bool filter_is_matched(const FilterParams& fp, uint32_t i, uint64_t mask, uint32_t nl)
{
	const bool m_sip = fp.src_ip != 0, m_dip = fp.dst_ip != 0, m_sp = fp.src_port != 0, m_dp = fp.dst_port != 0;
	const bool m_proto = fp.protocol == P_TCP || fp.protocol == P_UDP;
	if (!(m_sip || m_dip || m_sp || m_dp || m_proto))
		return true;
	const uint8_t* pkt = fp.data + fp.offsets[i];
	int v4 = -1, tcp = -1, udp = -1;
	const pcppx_layer* lay = fp.layers + (size_t)i * fp.ml;
	for (uint32_t k = 0; k < nl; ++k)
	{
		const uint32_t pr = lay[k].proto;
		const int o = (int)lay[k].offset;
		if (pr == P_IPV4 && v4 < 0) v4 = o;
		if (pr == P_TCP && tcp < 0) tcp = o;
		if (pr == P_UDP && udp < 0) udp = o;
	}
	if (m_sip || m_dip)
	{
		if (!(mask & (1ull << P_IPV4)) || v4 < 0)
			return false;
		const uint32_t sip = pkt[v4 + 12] | (pkt[v4 + 13] << 8) | (pkt[v4 + 14] << 16) | ((uint32_t)pkt[v4 + 15] << 24);
		const uint32_t dip = pkt[v4 + 16] | (pkt[v4 + 17] << 8) | (pkt[v4 + 18] << 16) | ((uint32_t)pkt[v4 + 19] << 24);
		if (m_sip && sip != fp.src_ip)
			return false;
		if (m_dip && dip != fp.dst_ip)
			return false;
	}
	if (m_sp || m_dp)
	{
		int l4 = -1;
		if ((mask & (1ull << P_TCP)) && tcp >= 0) l4 = tcp;
		else if ((mask & (1ull << P_UDP)) && udp >= 0) l4 = udp;
		if (l4 < 0)
			return false;
		const uint32_t sp = (pkt[l4] << 8) | pkt[l4 + 1], dp = (pkt[l4 + 2] << 8) | pkt[l4 + 3];
		if (m_sp && sp != fp.src_port)
			return false;
		if (m_dp && dp != fp.dst_port)
			return false;
	}
	if (m_proto)
	{
		if (fp.protocol == P_TCP && !(mask & (1ull << P_TCP)))
			return false;
		if (fp.protocol == P_UDP && !(mask & (1ull << P_UDP)))
			return false;
	}
	return true;
}

__device__ __forceinline__ uint32_t flow_mix(uint32_t key)
{
	return key * 0x9E3779B1u;
}

constexpr uint32_t kStatFlowTableFull = 14;  // pcppx_packet_stats::flow_table_full (u64 index)
__global__ __launch_bounds__(kBlock) void filter_mark_kernel(FilterParams fp)
{
	const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
	if (i >= fp.n)
		return;
	const pcppx_summary& sm = fp.summary[i];
	const uint32_t nl = sm.n_layers < fp.ml ? sm.n_layers : fp.ml;
	if (!filter_is_matched(fp, i, sm.proto_mask, nl))
		return;
	const unsigned long long key = (1ull << 32) | sm.hash5;
	const uint32_t m = fp.capacity - 1;
	uint32_t slot = flow_mix(sm.hash5) & m;
	const unsigned long long mine = ~(unsigned long long)(fp.seq_base + i);
	for (uint32_t probe = 0; probe < fp.capacity; ++probe)
	{
		// plain reads first: a set key never changes, and first[] only grows, so a hot flow's packets
		// after its first skip both atomics
		unsigned long long prev = fp.keys[slot];
		if (prev != key)
			prev = atomicCAS(&fp.keys[slot], 0ull, key);
		if (prev == 0ull || prev == key)
		{
			// stored as ~seq with atomicMax, so a zero-initialised table means "no match yet"
			if (fp.first[slot] < mine)
				atomicMax(&fp.first[slot], mine);
			return;
		}
		slot = (slot + 1) & m;
	}
	atomicAdd(&fp.stats[kStatFlowTableFull], 1ull);  // no free slot: results no longer the reference's (pcppx.h)
}

__device__ __forceinline__ void wave_count(unsigned long long* ctr, bool pred)
{
	const unsigned long long b = __ballot(pred);
	if ((threadIdx.x & 63) == 0 && b)
		atomicAdd(ctr, (unsigned long long)__popcll(b));
}

__global__ __launch_bounds__(kBlock) void filter_apply_kernel(FilterParams fp)
{
	const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
	const bool in = i < fp.n;
	uint64_t mask = 0;
	uint32_t flags = 0;
	bool matched = false, new_tcp = false, new_udp = false, settled = false;
	uint32_t l7 = 0;
	if (in)
	{
		const pcppx_summary& sm = fp.summary[i];
		mask = sm.proto_mask;
		flags = sm.flags;
		const uint32_t nl = sm.n_layers < fp.ml ? sm.n_layers : fp.ml;
		// the packet's counters are the device's unless its chain stopped before a layer it does not see: an
		// out-of-scope L2/L3 layer, a bad record, or an L7 layer the parse could not classify (PCPPX_F_L7_KNOWN)
		settled = (flags & (PCPPX_F_NEEDS_HOST_PROTO | PCPPX_F_OVERSIZE | PCPPX_F_BAD_DESC)) == 0 &&
		          (!(flags & PCPPX_F_NEEDS_HOST_L7) || (flags & PCPPX_F_L7_KNOWN));
		// isPacketOfType(HTTP / DNS / SSL): the built layers (proto_mask), else the class of a host-owned first L7 layer
		l7 = ((flags & PCPPX_F_L7_HTTP) || (mask & ((1ull << P_HTTP_REQ) | (1ull << P_HTTP_RESP))) ? 1u : 0u) |
		     ((flags & PCPPX_F_L7_DNS) || (mask & (1ull << P_DNS)) ? 2u : 0u) |
		     ((flags & PCPPX_F_L7_SSL) || (mask & (1ull << P_SSL)) ? 4u : 0u);
		const bool own = filter_is_matched(fp, i, mask, nl);
		const unsigned long long key = (1ull << 32) | sm.hash5;
		const uint64_t seq = fp.seq_base + i;
		const uint32_t m = fp.capacity - 1;
		uint32_t slot = flow_mix(sm.hash5) & m;
		uint64_t first = ~0ull;
		for (uint32_t probe = 0; probe < fp.capacity; ++probe)
		{
			const unsigned long long kk = fp.keys[slot];
			if (kk == key)
			{
				first = ~(uint64_t)fp.first[slot];
				break;
			}
			if (kk == 0ull)
				break;
			slot = (slot + 1) & m;
		}
		matched = own || first < seq;
		if (own && first == seq)  // the flow's first matching packet: a new matched flow
		{
			new_tcp = (mask & (1ull << P_TCP)) != 0;
			new_udp = !new_tcp && (mask & (1ull << P_UDP)) != 0;
		}
		fp.matched[i] = matched ? 1 : 0;
	}
	unsigned long long* st = fp.stats;
	wave_count(st + 0, in);
	wave_count(st + 1, (mask >> P_ETH) & 1);
	wave_count(st + 2, (mask >> P_ARP) & 1);
	wave_count(st + 3, (mask >> P_IPV4) & 1);
	wave_count(st + 4, (mask >> P_IPV6) & 1);
	wave_count(st + 5, (mask >> P_TCP) & 1);
	wave_count(st + 6, (mask >> P_UDP) & 1);
	wave_count(st + 10, new_tcp);
	wave_count(st + 11, new_udp);
	wave_count(st + 12, matched);
	wave_count(st + 7, settled && (l7 & 1));
	wave_count(st + 8, settled && (l7 & 2));
	wave_count(st + 9, settled && (l7 & 4));
	wave_count(st + 13, in && !settled);
}

// the protocols the engine builds itself (ProtocolType.h:42-258), GenericPayload excluded: a parse-until
// family made only of these never holds a layer the host would build (oracle/pcppx_oracle.c,
// family_engine_only)
bool family_engine_only(uint32_t fam)
{
	if (fam == 0)
		return false;
	for (int k = 0; k < 4; ++k)
	{
		const uint32_t b = (fam >> (8 * k)) & 0xFFu;
		const bool own = b == P_ETH || b == P_IPV4 || b == P_IPV6 || b == P_TCP || b == P_UDP || b == P_ARP ||
		                 b == P_VLAN || b == P_MPLS || b == P_GREV0 || b == P_GREV1 || b == P_PPTP ||
		                 b == P_TRAILER || b == P_DOT3 || b == P_LLC || b == P_ICMP || b == P_NFLOG || b == P_CISCO_HDLC ||
		                 // a classified first L7 layer is built, an unclassified one is none of these
		                 b == P_HTTP_REQ || b == P_HTTP_RESP || b == P_DNS || b == P_SSL || b == P_MYSQL || b == P_SSH;
		if (b != 0 && !own)
			return false;
	}
	return true;
}

Params make_params(const pcppx_batch* b, const pcppx_opts* o, pcppx_records* r, pcppx_reasm_info* info)
{
	Params prm;
	prm.data = b->data;
	prm.offsets = b->offsets;
	prm.caplens = b->caplens;
	prm.data_len = b->data_len;
	prm.summary = r->summary;
	prm.flow_keys = r->flow_keys;
	prm.layers = o->max_layers ? r->layers : nullptr;
	prm.n = b->n;
	prm.family = o->parse_until_family;
	prm.until_osi = o->parse_until_osi;
	prm.want_csum = o->want_checksums;
	prm.max_layers = o->max_layers;
	prm.linktype = b->linktype;
	prm.fam_engine_only = family_engine_only(o->parse_until_family) ? 1u : 0u;
	prm.reasm = info;
	prm.tuples = r->tuples;
	prm.wave_stats = nullptr;
	prm.packed = o->layout == PCPPX_LAYOUT_PACKED ? 1u : 0u;
	prm.brief = r->brief;
	return prm;
}

// the parse kernel's shape: 5 waves/SIMD (87 VGPRs, 7 KiB LDS), 2 x 2 KiB span-stream windows, non-temporal span
// loads and record stores -- the fastest of the measured shapes
// (profiles/r01_ab_occupancy.txt, r01_ab_windows.txt, r01_ab_window160.txt, r01_ab_nontemporal.txt; the
// other shapes are built only into tools/ab/libpcppx_ab.so)
constexpr int kParseWaves = 5, kParseSWin = 128;
// 96-B header windows since round 2: every Eth / VLAN / IPv4|IPv6 / TCP|UDP stack fits (deeper stacks take the generic
// walk's HBM peeks past the window); 1.5% faster than 112 B on config 3 in two interleaved A/Bs, and a two-round
// 96 + 16 B gather is slower (profiles/r02_ab_windows96.txt)
constexpr int kParseChunks = 6;
// round 3: both stream windows are issued before the header gather (EarlyB; same 96 VGPRs): 0.8-0.9% on config 3 in
// interleaved A/Bs, fixed and packed layouts (profiles/r03_ab_earlyB_*.txt)
#define PCPPX_PARSE_KERNEL parse_tile_kernel<kParseWaves, kParseSWin, kParseChunks, true, kParseChunks>
// parse-only launches (no checksums): no span stream; a 144-B window reached in two gather rounds (96 B for every
// packet, the rest only for the deep stacks the first window cannot hold): 99.7% of config 5's deep stacks take the
// fast path; 16 waves/CU of LDS (144 B: 0.88 ms on config 5, 160 B: 1.00 ms at 14 waves/CU, 112 B: 1.17 ms with
// 22% of the packets on the generic walk; gpurun_out r02l_ab_cfg5 -> profiles/r02_ab_parse_only.txt)
// Round 6: the first round holds 128 B (8 chunks) instead of 96: most deep stacks end inside it, so fewer waves take the
// dependent second round (config 5 -2.9% in an interleaved A/B, records identical: tools/ab variant 240 against 219,
// profiles/r06c_ab6_cfg5.txt); plain stacks take the SHORT instance, not this one
constexpr int kParseOnlyChunks = 9, kParseOnlyChunks1 = 8;
constexpr int kParseDeepChunks1 = 6;  // the DEEP checksum instance keeps its measured 96-B first round
#define PCPPX_PARSE_ONLY_KERNEL parse_tile_kernel<1, 64, kParseOnlyChunks, false, kParseOnlyChunks1>
// checksum launches with opts.window = PCPPX_WINDOW_DEEP: the parse-only instance's two-round 144-B window (tight second
// round, dword-aligned re-gather) with the span stream; LDS 10 KiB, 4 waves/SIMD; the second stream window is issued
// after the parse (EarlyB off: this instance's register budget)
#define PCPPX_PARSE_DEEP_KERNEL                                                                                        \
	parse_tile_kernel<4, kParseSWin, kParseOnlyChunks, true, kParseDeepChunks1, ParseShape<true, true, true, true, false>>
// parse-only launches with opts.window = PCPPX_WINDOW_SHORT: one 96-B round, LDS 7 KiB (22 waves/CU, 5 waves/SIMD of
// registers): config 4 0.464 -> 0.432 ms, config 2 43.2 -> 36.3 us, config 5 0.75 -> 1.61 ms (tools/ab variant 60,
// profiles/r03_ab_windows_persist.txt)
#define PCPPX_PARSE_SHORT_KERNEL parse_tile_kernel<1, 64, kParseChunks, false, kParseChunks>

// the flow-table shape: 1024-thread blocks, 8192 LDS slots, 4096-packet batches with the next batch prefetched,
// 256 persistent blocks (profiles/r01_ab_flow_shape.txt, r01_ab_flow_grid.txt)
#define PCPPX_FLOW_KERNEL flow_count_kernel<1024, 8192, 4096, kFlowHot, true>
// the partitioned flush (product): the same aggregation over 6144-packet batches (fewer flushes: count + merge
// 0.178 -> 0.168 ms on config 4, profiles/r04g_ab_flow_list.txt shape 12) with the one-pass flush (-4.6%,
// profiles/r04r_ab_flow_onepass.txt), then per-partition queues and one merge block per partition
#define PCPPX_FLOW_PART_KERNEL flow_count_kernel<1024, 8192, kFlowBatchPk, kFlowHot, true, true, false, true>
#define PCPPX_FLOW_PART_DENSE_KERNEL flow_count_kernel<1024, 8192, kFlowBatchPk, kFlowHot, true, true, true, true>
// merge: 512-thread blocks with a 4096-slot LDS table (48 KiB: 3 blocks per CU) over 512 partitions -- count + merge
// 0.194 -> 0.181 ms on config 4 against 1024 threads / 8192 slots / 256 partitions (profiles/r03_ab_flow_merge.txt);
// three rounds of queue records in flight (-1 to -2%, profiles/r04f_ab_flow_merge_batch.txt shape 9)
#define PCPPX_FLOW_MERGE_KERNEL flow_merge_kernel<kFlowMergeThreads, 4096, 2, 3>
constexpr uint32_t kFlowThreads = 1024, kFlowBatchPk = 6144, kFlowBlocks = 256;
constexpr uint32_t kPackedMax = (1u << 24) - 1;  // packets per launch the packed LDS/HBM counters hold
constexpr uint32_t kFlowPartLog2 = 9;            // flow-table partitions (merge blocks); at most kFlowMaxParts
constexpr uint32_t kFlowMinRegionLog2 = 12;      // slots per partition at least (capacity 2^21+ -> 512 partitions)
constexpr uint32_t kFlowMergeThreads = 512;

// ---- PCPPX_LAYOUT_DENSE (host path): FIXED rows -> the chains back to back ----
// Two small kernels per host-path chunk (<= 256k packets): dense_count_kernel sums each 1024-packet block's chain
// lengths; dense_copy_kernel takes its block's base as the sum of the blocks before it (at most 256 words), scans its
// threads' counts (4 consecutive packets per thread) and copies each chain's entries to its dense position. On-device
// traffic is the FIXED rows once (8 * ml B per packet, ~6 us per chunk at HBM rates); what crosses PCIe is the chains.
constexpr uint32_t kDenseThreads = 256, kDensePer = 4, kDenseBlockPk = kDenseThreads * kDensePer;

__device__ __forceinline__ uint32_t block_sum_256(uint32_t v, uint32_t* lds)
{
	for (int o = 32; o > 0; o >>= 1)
		v += __shfl_xor(v, o);
	const uint32_t wv = threadIdx.x >> 6;
	if ((threadIdx.x & 63) == 0)
		lds[wv] = v;
	__syncthreads();
	const uint32_t t = lds[0] + lds[1] + lds[2] + lds[3];
	__syncthreads();
	return t;
}

__global__ __launch_bounds__(kDenseThreads) void dense_count_kernel(const uint8_t* __restrict__ nl, uint32_t stride,
                                                                    uint32_t n, uint32_t ml, uint32_t* __restrict__ bsum)
{
	__shared__ uint32_t lds[4];
	uint32_t s = 0;
	for (uint32_t k = 0; k < kDensePer; ++k)
	{
		const uint32_t i = blockIdx.x * kDenseBlockPk + k * kDenseThreads + threadIdx.x;
		if (i < n)
			s += min((uint32_t)nl[(size_t)i * stride], ml);
	}
	s = block_sum_256(s, lds);
	if (threadIdx.x == 0)
		bsum[blockIdx.x] = s;
}

__global__ __launch_bounds__(kDenseThreads) void dense_copy_kernel(const uint2* __restrict__ fixed,
                                                                   const uint8_t* __restrict__ nl, uint32_t stride,
                                                                   uint32_t n, uint32_t ml,
                                                                   const uint32_t* __restrict__ bsum, uint2* __restrict__ dense,
                                                                   uint32_t* __restrict__ total)
{
	__shared__ uint32_t lds[4];
	__shared__ uint32_t wsum[4];
	// the block's base: the chain lengths of every block before it
	uint32_t b = 0;
	for (uint32_t j = threadIdx.x; j < blockIdx.x; j += kDenseThreads)
		b += bsum[j];
	const uint32_t base = block_sum_256(b, lds);
	// this thread's 4 consecutive packets, their counts and the thread's exclusive offset in the block
	const uint32_t i0 = blockIdx.x * kDenseBlockPk + threadIdx.x * kDensePer;
	uint32_t c[kDensePer], mine = 0;
	for (uint32_t k = 0; k < kDensePer; ++k)
	{
		c[k] = i0 + k < n ? min((uint32_t)nl[(size_t)(i0 + k) * stride], ml) : 0u;
		mine += c[k];
	}
	uint32_t incl = mine;  // inclusive wave scan, then the waves' totals
	const uint32_t lane = threadIdx.x & 63;
	for (uint32_t o = 1; o < 64; o <<= 1)
	{
		const uint32_t t = __shfl_up(incl, o);
		incl += lane >= o ? t : 0u;
	}
	if (lane == 63)
		wsum[threadIdx.x >> 6] = incl;
	__syncthreads();
	uint32_t wbase = 0;
	for (uint32_t w = 0; w < (threadIdx.x >> 6); ++w)
		wbase += wsum[w];
	uint32_t pos = base + wbase + incl - mine;
	for (uint32_t k = 0; k < kDensePer; ++k)
	{
		const uint2* src = fixed + (size_t)(i0 + k) * ml;
		for (uint32_t e = 0; e < c[k]; ++e)
			dense[pos + e] = src[e];
		pos += c[k];
	}
	if (blockIdx.x == gridDim.x - 1 && threadIdx.x == kDenseThreads - 1)
		*total = pos;  // the last thread of the last block ends the batch's chains
}

// The chunk's chains (dense[0, *count)) to the caller's page-locked records through their device mapping, coalesced
// (64 lanes store 512 contiguous bytes): no host round trip to learn the count before a copy can be sized. The chunks
// of a host batch chain their positions on the device: *base_in (the chunks before this one, null for the first) +
// this chunk's count -> *cum_out; `at_base` places the entries at base (the caller's array) or at 0 (a staging buffer).
__global__ __launch_bounds__(kDenseThreads) void dense_push_kernel(const uint2* __restrict__ dense,
                                                                   const uint32_t* __restrict__ count,
                                                                   const uint32_t* __restrict__ base_in, uint2* dst,
                                                                   uint32_t at_base, uint32_t* __restrict__ cum_out)
{
	const uint32_t cnt = *count, base = base_in != nullptr ? *base_in : 0u;
	uint2* out = dst + (at_base ? base : 0u);
	const uint32_t step = gridDim.x * kDenseThreads;
	for (uint32_t j = blockIdx.x * kDenseThreads + threadIdx.x; j < cnt; j += 4 * step)
	{
		uint2 v[4];  // four loads in flight per lane
#pragma unroll
		for (uint32_t u = 0; u < 4; ++u)
			if (j + u * step < cnt)
				v[u] = dense[j + u * step];
#pragma unroll
		for (uint32_t u = 0; u < 4; ++u)
			if (j + u * step < cnt)
				out[j + u * step] = v[u];
	}
	__threadfence_system();  // host memory: visible to the host at the event behind this kernel, whatever its caching
	if (blockIdx.x == 0 && threadIdx.x == 0)
		*cum_out = base + cnt;
}

}  // namespace

uint32_t dense_blocks(uint32_t n)
{
	return (n + kDenseBlockPk - 1) / kDenseBlockPk;
}

int launch_dense_compact(const pcppx_layer* fixed, const uint8_t* n_layers, uint32_t nl_stride, uint32_t n, uint32_t ml,
                         pcppx_layer* dense, uint32_t* block_sums, uint32_t* total, hipStream_t stream)
{
	if (n == 0 || ml == 0)
		return hipMemsetAsync(total, 0, sizeof(uint32_t), stream) == hipSuccess ? PCPPX_OK : PCPPX_E_HIP;
	const uint32_t g = dense_blocks(n);
	hipLaunchKernelGGL(dense_count_kernel, dim3(g), dim3(kDenseThreads), 0, stream, n_layers, nl_stride, n, ml,
	                   block_sums);
	hipLaunchKernelGGL(dense_copy_kernel, dim3(g), dim3(kDenseThreads), 0, stream,
	                   reinterpret_cast<const uint2*>(fixed), n_layers, nl_stride, n, ml, block_sums,
	                   reinterpret_cast<uint2*>(dense), total);
	return check_launch("dense_compact", stream);
}

int launch_dense_push(const pcppx_layer* dense, const uint32_t* count, const uint32_t* base_in, pcppx_layer* dst_mapped,
                      bool at_base, uint32_t* cum_out, hipStream_t stream)
{
	hipLaunchKernelGGL(dense_push_kernel, dim3(128), dim3(kDenseThreads), 0, stream, reinterpret_cast<const uint2*>(dense),
	                   count, base_in, reinterpret_cast<uint2*>(dst_mapped), at_base ? 1u : 0u, cum_out);
	return check_launch("dense_push", stream);
}

namespace
{
}  // namespace

int check_launch(const char* what, hipStream_t /*stream*/)
{
	const hipError_t e = hipGetLastError();
	if (e != hipSuccess)
	{
		fprintf(stderr, "pcppx: %s failed: %s\n", what, hipGetErrorString(e));
		return PCPPX_E_HIP;
	}
	return PCPPX_OK;
}

namespace
{
// the instance for the (already resolved) window: checksum launches DEFAULT one round / DEEP two rounds; parse-only
// launches two rounds / SHORT one round
int launch_instance(const pcppx_opts* o, const Params& prm, uint32_t n, hipStream_t stream, const char* what)
{
	const dim3 grid((n + kTile - 1) / kTile);
	if (o->want_checksums && o->window == PCPPX_WINDOW_DEEP)
		hipLaunchKernelGGL(PCPPX_PARSE_DEEP_KERNEL, grid, dim3(kTile), 0, stream, prm);
	else if (o->want_checksums)
		hipLaunchKernelGGL(PCPPX_PARSE_KERNEL, grid, dim3(kTile), 0, stream, prm);
	else if (o->window == PCPPX_WINDOW_SHORT)
		hipLaunchKernelGGL(PCPPX_PARSE_SHORT_KERNEL, grid, dim3(kTile), 0, stream, prm);
	else
		hipLaunchKernelGGL(PCPPX_PARSE_ONLY_KERNEL, grid, dim3(kTile), 0, stream, prm);
	return check_launch(what, stream);
}

// the window sample (Ethernet batches): about 64 evenly spread tiles of the batch, ahead of its parse on the same stream
int launch_window_sample(const Params& prm, unsigned long long* win, hipStream_t stream)
{
	if (win == nullptr || prm.linktype != 1)
		return PCPPX_OK;
	const uint32_t tiles = (prm.n + kTile - 1) / kTile, stride = tiles >> 6 ? tiles >> 6 : 1u;
	hipLaunchKernelGGL(window_sample_kernel, dim3((tiles + stride - 1) / stride), dim3(kTile), 0, stream, prm, stride, win);
	return check_launch("window_sample_kernel", stream);
}
}  // namespace

int launch_parse(const pcppx_batch* b, const pcppx_opts* o, pcppx_records* r, hipStream_t stream, void* wave_stats,
                 unsigned long long* win_stats)
{
	if (b->n == 0)
		return PCPPX_OK;
	Params prm = make_params(b, o, r, nullptr);
	prm.wave_stats = static_cast<uint4*>(wave_stats);
	const int rc = launch_window_sample(prm, win_stats, stream);
	return rc != PCPPX_OK ? rc : launch_instance(o, prm, b->n, stream, "parse_tile_kernel");
}

int launch_parse_reasm(const pcppx_batch* b, const pcppx_opts* o, pcppx_records* r, pcppx_reasm_info* info,
                       hipStream_t stream, void* wave_stats, unsigned long long* win_stats)
{
	if (b->n == 0)
		return PCPPX_OK;
	Params prm = make_params(b, o, r, info);
	prm.wave_stats = static_cast<uint4*>(wave_stats);
	const int rc = launch_window_sample(prm, win_stats, stream);
	return rc != PCPPX_OK ? rc : launch_instance(o, prm, b->n, stream, "parse_tile_kernel(reasm)");
}

uint32_t parse_waves(uint32_t n)
{
	return (n + kTile - 1) / kTile;
}

int launch_proto_stats_reduce(const void* wave_stats, uint32_t n, uint64_t* out, hipStream_t stream)
{
	if (n == 0)
		return PCPPX_OK;
	const uint32_t nw = parse_waves(n);
	const uint32_t blocks = (nw + 8 * kBlock - 1) / (8 * kBlock);
	hipLaunchKernelGGL(proto_stats_reduce_kernel, dim3(blocks < 128 ? blocks : 128), dim3(kBlock), 0, stream,
	                   static_cast<const uint4*>(wave_stats), nw, reinterpret_cast<unsigned long long*>(out));
	return check_launch("proto_stats_reduce_kernel", stream);
}

int launch_filter(const pcppx_batch* b, const pcppx_records* r, uint32_t ml, const pcppx_match_spec* spec,
                  uint64_t seq_base, uint64_t* keys, uint64_t* first, uint32_t capacity, uint8_t* matched,
                  pcppx_packet_stats* stats, hipStream_t stream)
{
	if (b->n == 0)
		return PCPPX_OK;
	FilterParams fp;
	fp.data = b->data;
	fp.offsets = b->offsets;
	fp.summary = r->summary;
	fp.layers = r->layers;
	fp.n = b->n;
	fp.ml = ml;
	fp.src_ip = spec->src_ip;
	fp.dst_ip = spec->dst_ip;
	fp.src_port = spec->src_port;
	fp.dst_port = spec->dst_port;
	fp.protocol = spec->protocol;
	fp.seq_base = seq_base;
	fp.keys = reinterpret_cast<unsigned long long*>(keys);
	fp.first = reinterpret_cast<unsigned long long*>(first);
	fp.capacity = capacity;
	fp.matched = matched;
	fp.stats = reinterpret_cast<unsigned long long*>(stats);
	const dim3 grid((b->n + kBlock - 1) / kBlock);
	hipLaunchKernelGGL(filter_mark_kernel, grid, dim3(kBlock), 0, stream, fp);
	int rc = check_launch("filter_mark_kernel", stream);
	if (rc != PCPPX_OK)
		return rc;
	hipLaunchKernelGGL(filter_apply_kernel, grid, dim3(kBlock), 0, stream, fp);
	return check_launch("filter_apply_kernel", stream);
}

// log2 of the partitions: every region keeps at least 2^kFlowMinRegionLog2 slots, so a flow is only lost when its
// region is full, not while a small table still has free slots elsewhere (a single region = the plain
// open-addressed table)
uint32_t flow_partitions_log2(uint32_t capacity)
{
	const uint32_t l = log2u(capacity);
	const uint32_t lp = l > kFlowMinRegionLog2 ? l - kFlowMinRegionLog2 : 0u;
	return lp < kFlowPartLog2 ? lp : kFlowPartLog2;
}

uint32_t flow_partitions(uint32_t capacity)
{
	return 1u << flow_partitions_log2(capacity);
}

// Records per partition queue. A launch queues at most one record per packet in total (a record carries at least
// one packet no earlier record carried), so one partition needs `per` and P partitions need per/P each for keys
// spread evenly by the hash, plus a quarter and a constant for the spread; a full queue falls back to atomics on
// the region (correct, slower).
uint32_t flow_queue_capacity(uint32_t n, uint32_t capacity)
{
	const uint32_t per = kPackedMax < n ? kPackedMax : n;
	const uint32_t parts = flow_partitions(capacity);
	if (parts == 1)
		return per;
	const uint32_t even = (per + parts - 1) / parts;
	return even + even / 4 + 4096;
}

int launch_flow_count_part(const pcppx_summary* sum, const uint32_t* dkeys, const uint32_t* caplens, uint32_t n,
                           uint32_t* keys, uint64_t* packets, uint64_t* bytes, uint32_t capacity, uint64_t* stats,
                           void* queues, uint32_t rec_cap, uint32_t* fill, hipStream_t stream)
{
	auto* pk = reinterpret_cast<unsigned long long*>(packets);
	auto* by = reinterpret_cast<unsigned long long*>(bytes);
	auto* st = reinterpret_cast<unsigned long long*>(stats);
	const uint32_t l = log2u(capacity), lp = flow_partitions_log2(capacity);
	const FlowPart fp{ static_cast<uint4*>(queues), rec_cap, fill, lp, l - lp };
	for (uint32_t done = 0; done < n;)
	{
		const uint32_t cnt = n - done < kPackedMax ? n - done : kPackedMax;
		const uint32_t batches = (cnt + kFlowBatchPk - 1) / kFlowBatchPk;
		const dim3 grid(batches < kFlowBlocks ? batches : kFlowBlocks);
		if (dkeys != nullptr)
			hipLaunchKernelGGL(PCPPX_FLOW_PART_DENSE_KERNEL, grid, dim3(kFlowThreads), 0, stream, nullptr, caplens + done, cnt,
			                   keys, pk, by, capacity, st, nullptr, fp, dkeys + done);
		else
			hipLaunchKernelGGL(PCPPX_FLOW_PART_KERNEL, grid, dim3(kFlowThreads), 0, stream, sum + done, caplens + done, cnt,
			                   keys, pk, by, capacity, st, nullptr, fp, nullptr);
		int rc = check_launch("flow_count_kernel(partitioned)", stream);
		if (rc != PCPPX_OK)
			return rc;
		hipLaunchKernelGGL(PCPPX_FLOW_MERGE_KERNEL, dim3(1u << lp), dim3(kFlowMergeThreads), 0, stream, fp, keys, pk, by, st);
		rc = check_launch("flow_merge_kernel", stream);
		if (rc != PCPPX_OK)
			return rc;
		done += cnt;
	}
	return PCPPX_OK;
}

int launch_reasm(const pcppx_batch* b, const pcppx_records* r, uint32_t ml, pcppx_reasm_info* info, hipStream_t stream)
{
	if (b->n == 0)
		return PCPPX_OK;
	ReasmParams rp{ b->data, b->offsets, r->summary, r->layers, b->n, ml, info };
	hipLaunchKernelGGL(reasm_kernel, dim3((b->n + kBlock - 1) / kBlock), dim3(kBlock), 0, stream, rp);
	return check_launch("reasm_kernel", stream);
}

}  // namespace pcppx
