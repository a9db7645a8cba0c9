/*
 * pcppx_oracle.c — TEST INFRASTRUCTURE ONLY: the parity checker, never the product path.
 *
 * A scalar, allocation-free C restatement of the reference Packet++ per-packet parse path
 * (SURVEY.md §8a rows a1-a17). Every rule cites the reference file:line it restates (paths relative
 * to the reference root). The output is the engine's record format (include/pcppx.h).
 *
 * Engine contract for layers this path does not dissect (restated identically by the HIP kernels):
 *   - where the reference would hand an L4 payload to an L7 dissector (port/content triggers of
 *     TcpLayer.cpp:372-491 and UdpLayer.cpp:103-178, incl. the SIP content heuristic
 *     SipLayer.cpp:127-160) the chain stops after the TCP/UDP layer and PCPPX_F_NEEDS_HOST_L7 is set;
 *   - except that a classified HTTP / SSL / DNS first L7 layer is built, with the layers behind it, and so
 *     are the VXLAN and GTPv1 tunnels over UDP with the packet they carry;
 *   - where it would build an out-of-scope L2/L3 layer (PPPoE, WoL, IGMP, AH, ESP, VRRP, ICMPv6, STP,
 *     ...) the chain stops before it and PCPPX_F_NEEDS_HOST_PROTO is set (NFLOG and Cisco HDLC first layers are
 *     built since round 6);
 *   - no trailer is appended to a flagged chain; hashes and checksums are computed over the emitted chain.
 * For unflagged packets every field equals the reference; for flagged packets the emitted layers are an
 * exact prefix of the reference chain.
 *
 * Pinned against the real reference (oracle/_ref/libpcpp_ref.so) and committed golden records: see
 * tests/test_oracle_vs_reference.py.
 */
#define _POSIX_C_SOURCE 200809L
#include "pcppx_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* ---- ProtocolType ids (Packet++/header/ProtocolType.h:42-258) and OSI (:266-284) ---- */
enum {
	P_ETH = 1, P_IPV4 = 2, P_IPV6 = 3, P_TCP = 4, P_UDP = 5, P_ARP = 8, P_VLAN = 9, P_ICMP = 10, P_MPLS = 14,
	P_GREV0 = 15, P_GREV1 = 16, P_PPTP = 17, P_SLL = 19, P_NULL = 21, P_PAYLOAD = 25, P_TRAILER = 30, P_DOT3 = 33,
	P_LLC = 44, P_SLL2 = 52, P_VXLAN = 26, P_GTPV1 = 32, P_NFLOG = 47, P_CISCO_HDLC = 58
};

enum kind { K_NONE = 0, K_ETH, K_DOT3, K_LLC, K_VLAN, K_MPLS, K_IPV4, K_IPV6, K_GRE0, K_GRE1, K_PPTP,
	        K_TCP, K_UDP, K_PAYLOAD, K_OUT, K_L7, K_ARP, K_SLL, K_SLL2, K_NULL, K_ICMP, K_VXLAN, K_GTP1,
	        K_NFLOG, K_HDLC };

static uint16_t be16(const uint8_t* p) { return (uint16_t)((p[0] << 8) | p[1]); }
static uint16_t le16(const uint8_t* p) { return (uint16_t)(p[0] | (p[1] << 8)); }
static uint32_t le32(const uint8_t* p)
{
	return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
static uint16_t bswap16(uint16_t v) { return (uint16_t)((v >> 8) | (v << 8)); }

/* ---- isDataValid restatements ---- */
/* EthLayer::isDataValid, Packet++/src/EthLayer.cpp:100-117 */
static int eth_valid(const uint8_t* p, uint32_t n) { return n >= 14 && be16(p + 12) >= 0x0600; }
/* EthDot3Layer::isDataValid, Packet++/src/EthDot3Layer.cpp:38-54 */
static int dot3_valid(const uint8_t* p, uint32_t n) { return n >= 14 && be16(p + 12) <= 0x05DC; }
/* LLCLayer::isDataValid, Packet++/src/LLCLayer.cpp:49-52 */
static int llc_valid(const uint8_t* p, uint32_t n) { return n >= 3 && !(p[0] == 0xFF && p[1] == 0xFF); }
/* IPv4Layer::isDataValid, Packet++/header/IPv4Layer.h:626-630 (iphdr bitfields: IHL low nibble) */
static int ipv4_valid(const uint8_t* p, uint32_t n) { return n >= 20 && (p[0] >> 4) == 4 && (p[0] & 0xF) >= 5; }
/* IPv6Layer::isDataValid, Packet++/header/IPv6Layer.h:245-249 */
static int ipv6_valid(const uint8_t* p, uint32_t n) { return n >= 40 && (p[0] >> 4) == 6; }
/* IcmpLayer::isDataValid, Packet++/header/IcmpLayer.h:619-660: the type's message struct fits (icmphdr 4 B; timestamp
 * 20; address mask 12; unreachable / redirect / time exceeded / source quench / param problem / router
 * advertisement 8); other types are not ICMP */
static int icmp_valid(const uint8_t* p, uint32_t n)
{
	if (n < 4) return 0;
	switch (p[0]) {
	case 8: case 0: case 10: case 15: case 16: return 1;
	case 13: case 14: return n >= 20;
	case 17: case 18: return n >= 12;
	case 3: case 5: case 4: case 11: case 12: case 9: return n >= 8;
	default: return 0;
	}
}
/* TcpLayer::isDataValid, Packet++/header/TcpLayer.h:596-601 */
static int tcp_valid(const uint8_t* p, uint32_t n) { return n >= 20 && (p[12] >> 4) >= 5 && n >= (uint32_t)(p[12] >> 4) * 4; }

/* ---- L7 trigger sets (engine contract; reference dispatch chains cited) ---- */
/* SSLLayer::isSSLPort, Packet++/header/SSLLayer.h:488-510 */
static int ssl_port(uint16_t x)
{
	switch (x) {
	case 443: case 261: case 448: case 465: case 563: case 614: case 636:
	case 989: case 990: case 992: case 993: case 994: case 995: return 1;
	default: return 0;
	}
}
/* Ports gating TcpLayer::parseNextLayer's dispatch, Packet++/src/TcpLayer.cpp:372-491 */
static int tcp_l7_port(uint16_t x)
{
	if (ssl_port(x)) return 1;
	switch (x) {
	case 80: case 8080:              /* HTTP, HttpLayer.h:74-77 */
	case 5060: case 5061:            /* SIP, SipLayer.h:112-115 */
	case 179:                        /* BGP, BgpLayer.h:65-68 */
	case 22:                         /* SSH, SSHLayer.h:92-95 */
	case 53: case 5353: case 5355:   /* DNS, DnsLayer.h:468-479 */
	case 23:                         /* Telnet, TelnetLayer.h:276-279 */
	case 21: case 20:                /* FTP / FTP-data, FtpLayer.h:24-34 */
	case 13400: case 3496:           /* DoIP, DoIpLayer.h:666-670 */
	case 30490:                      /* SOME/IP(-SD), SomeIpSdLayer.h:569-572 */
	case 102:                        /* TPKT, TpktLayer.h:82-85 */
	case 25: case 587:               /* SMTP, SmtpLayer.h:27-30 */
	case 389:                        /* LDAP, LdapLayer.h:346-349 */
	case 5432:                       /* Postgres, PostgresLayer.h:508-511 */
	case 3306:                       /* MySQL, MySqlLayer.h:306-309 */
	case 2123:                       /* GTPv2, GtpLayer.h:996-999 */
	case 502:                        /* Modbus, ModbusLayer.h:99-102 */
		return 1;
	default: return 0;
	}
}
/* Ports gating UdpLayer::parseNextLayer's dispatch, Packet++/src/UdpLayer.cpp:103-165 */
static int udp_l7_port(uint16_t src, uint16_t dst)
{
	/* DhcpLayer::isDhcpPorts, DhcpLayer.h:784-788 */
	if ((src == 68 && dst == 67) || (src == 67 && dst == 68) || (src == 67 && dst == 67)) return 1;
	if (dst == 4789) return 1;                                  /* VXLAN (dst), VxlanLayer.h:119-122 */
	if (dst == 0 || dst == 7 || dst == 9) return 1;             /* WoL (dst), WakeOnLanLayer.h:105-108 */
	for (int k = 0; k < 2; ++k) {
		uint16_t x = k ? dst : src;
		switch (x) {
		case 53: case 5353: case 5355:       /* DNS */
		case 5060: case 5061:                /* SIP */
		case 1812: case 1813: case 3799:     /* RADIUS, RadiusLayer.h:273-284 */
		case 2152: case 2123:                /* GTPv1/v2, GtpLayer.h:386-389,996-999 */
		case 546: case 547:                  /* DHCPv6, DhcpV6Layer.h:388-391 */
		case 123:                            /* NTP, NtpLayer.h:531-534 */
		case 13400: case 3496:               /* DoIP */
		case 30490:                          /* SOME/IP */
		case 51820:                          /* WireGuard, WireGuardLayer.h:67-70 */
			return 1;
		default: break;
		}
	}
	return 0;
}
/* SipLayer::detectSipMessageType, Packet++/src/SipLayer.cpp:127-160 (pack4 at :19-25: bytes are
 * sign-extended chars, so a byte >= 0x80 in positions 1..3 can never match an ASCII key) */
static int sip_heuristic(const uint8_t* p, uint32_t n)
{
	static const char* keys[] = { "INVI", "ACK ", "BYE ", "CANC", "REGI", "PRAC", "OPTI", "SUBS",
		                          "NOTI", "PUBL", "INFO", "REFE", "MESS", "UPDA", "SIP/" };
	if (n < 4) return 0; /* with n == 3 the packed key's low byte is 0: no key matches */
	for (unsigned k = 0; k < sizeof(keys) / sizeof(keys[0]); ++k)
		if (memcmp(p, keys[k], 4) == 0) return 1;
	return 0;
}

/* ---- the first L7 layer behind TCP/UDP: the dispatch chains' content checks the engine restates ----
 * TcpLayer::parseNextLayer (TcpLayer.cpp:372-491) tries, in order, HTTP request (dst port 80/8080 and a known
 * method), HTTP response (src port 80/8080, known version and supported status code), SSL (SSL port and a
 * record header), then dissectors that are all gated by their own ports, then Payload. So a payload whose
 * only trigger ports are HTTP / SSL ports and whose content passes neither check is a plain Payload: exact,
 * no flag. Every other trigger leaves the packet to the host (NEEDS_HOST_L7) with the class of its first L7
 * layer where the engine can name it (PCPPX_F_L7_*), for PacketStats::collectStats (Common.h:83-104). */
static const uint16_t kHttpCodes[] = { /* intStatusCodeMap, HttpLayer.cpp:424-508 */
	100, 101, 102, 103, 200, 201, 202, 203, 204, 205, 206, 207, 208, 226, 300, 301, 302, 303, 304, 305, 306,
	307, 308, 400, 401, 402, 403, 404, 405, 406, 407, 408, 409, 410, 411, 412, 413, 414, 415, 416, 417, 418,
	419, 420, 421, 422, 423, 424, 425, 426, 428, 429, 431, 440, 444, 449, 450, 451, 494, 495, 496, 497, 498,
	499, 500, 501, 502, 503, 504, 505, 506, 507, 508, 509, 510, 511, 520, 521, 522, 523, 524, 598, 599 };
/* HttpMessage::isHttpPort, HttpLayer.h:74-77 */
static int http_port(uint16_t x) { return x == 80 || x == 8080; }
/* HttpRequestFirstLine::parseMethod != HttpMethodUnknown, HttpLayer.cpp:261-285 (HttpMethodStringToEnum :145-155) */
static int http_request(const uint8_t* d, uint32_t n)
{
	static const char* methods[] = { "GET", "HEAD", "POST", "PUT", "DELETE", "TRACE", "OPTIONS", "CONNECT", "PATCH" };
	if (n < 4) return 0;
	uint32_t sp = 0;
	while (sp < n && d[sp] != ' ') ++sp;
	if (sp == 0 || sp == n) return 0;
	for (unsigned k = 0; k < sizeof(methods) / sizeof(methods[0]); ++k)
		if (strlen(methods[k]) == sp && memcmp(d, methods[k], sp) == 0) return 1;
	return 0;
}
/* HttpResponseFirstLine::parseVersion != Unknown (HttpLayer.cpp:964-984, HttpVersionStringToEnum :160-164) and
 * !parseStatusCode(..).isUnsupportedCode() (:850-898; HttpResponseStatusCode(int, msg) :510-543 maps codes outside
 * intStatusCodeMap to values > 599, isUnsupportedCode HttpLayer.h:453-456) */
static int http_response(const uint8_t* d, uint32_t n)
{
	if (n < 8 || memcmp(d, "HTTP/", 5) != 0) return 0;
	if (memcmp(d + 5, "0.9", 3) != 0 && memcmp(d + 5, "1.0", 3) != 0 && memcmp(d + 5, "1.1", 3) != 0) return 0;
	if (n < 12) return 0;
	for (int j = 9; j < 12; ++j)
		if (d[j] < '0' || d[j] > '9') return 0;
	uint32_t off = 13;
	while (off < n && d[off] != '\n') ++off;
	if (off >= n) return 0;                                  /* no end of line: HttpStatusCodeUnknown */
	uint32_t mlen = off - 13;
	if (mlen > 0 && d[off - 1] == '\r') --mlen;             /* messageString.pop_back() */
	if (mlen == 0) return 0;
	int code = (d[9] - '0') * 100 + (d[10] - '0') * 10 + (d[11] - '0');
	for (unsigned k = 0; k < sizeof(kHttpCodes) / sizeof(kHttpCodes[0]); ++k)
		if (kHttpCodes[k] == code) return 1;
	return 0;
}
/* SSLLayer::IsSSLMessage, SSLLayer.cpp:14-40 (ports checked by the caller; SSLVersion::asEnum(true),
 * SSLCommon.cpp:12-27) */
static int ssl_record(const uint8_t* d, uint32_t n)
{
	if (n < 5) return 0;                        /* sizeof(ssl_tls_record_layer) */
	if (d[3] == 0 && d[4] == 0) return 0;       /* length 0 */
	if (d[0] < 20 || d[0] > 23) return 0;       /* record type */
	uint32_t v = ((uint32_t)d[1] << 8) | d[2];
	return (v >= 0x0300 && v <= 0x0304) || (v >= 0x7f0e && v <= 0x7f1c) || v == 0xfb17 || v == 0xfb1a;
}
static int dns_port(uint16_t x) { return x == 53 || x == 5353 || x == 5355; } /* DnsLayer::isDnsPort, DnsLayer.h:468-479 */

/* engine-internal class bits (never in a summary's flags): the payload is a MySqlLayer / SSH messages the engine builds */
#define L7_MYSQL 0x4000
#define L7_SSH 0x8000
/* TCP payload (sp/dp host order): 0 = plain Payload, else PCPPX_F_NEEDS_HOST_L7 | class bits */
static uint16_t tcp_l7(const uint8_t* d, uint32_t n, uint16_t sp, uint16_t dp)
{
	if (http_port(dp) && http_request(d, n)) return PCPPX_F_NEEDS_HOST_L7 | PCPPX_F_L7_KNOWN | PCPPX_F_L7_HTTP;
	if (http_port(sp) && http_response(d, n)) return PCPPX_F_NEEDS_HOST_L7 | PCPPX_F_L7_KNOWN | PCPPX_F_L7_HTTP;
	if ((ssl_port(sp) || ssl_port(dp)) && ssl_record(d, n))
		return PCPPX_F_NEEDS_HOST_L7 | PCPPX_F_L7_KNOWN | PCPPX_F_L7_SSL;
	/* the rest of the chain is gated by ports other than HTTP's and SSL's */
	int other = 0;
	for (int k = 0; k < 2; ++k) {
		uint16_t x = k ? dp : sp;
		if (tcp_l7_port(x) && !http_port(x) && !ssl_port(x)) other = 1;
	}
	if (!other) return 0;
	/* SSH (TcpLayer.cpp:407-410): port 22 on either side builds SSH messages (SSHLayer::createSSHMessage never fails,
	 * SSHLayer.cpp:18-30) unless the other port is SIP's or BGP's, whose branches (:387-406) come first and take the
	 * payload */
	if (sp == 22 || dp == 22) {
		const uint16_t o = sp == 22 ? dp : sp;
		if (o != 5060 && o != 5061 && o != 179) return PCPPX_F_NEEDS_HOST_L7 | PCPPX_F_L7_KNOWN | L7_SSH;
	}
	/* MySQL (TcpLayer.cpp:469-478): MySqlLayer's factory never fails (MySqlLayer.cpp:462-470), so port 3306 on either
	 * side builds it whenever the other port gates no dissector ahead of it in the chain (GTPv2 2123 and Modbus 502
	 * come after it); the engine builds that layer (L7_MYSQL). With another trigger port the earlier dissector's own
	 * validity decides, and the packet stays the host's. */
	if (sp == 3306 || dp == 3306) {
		const uint16_t o = sp == 3306 ? dp : sp;
		if (o == 3306 || o == 2123 || o == 502 || !tcp_l7_port(o) || http_port(o) || ssl_port(o))
			return PCPPX_F_NEEDS_HOST_L7 | PCPPX_F_L7_KNOWN | L7_MYSQL;
	}
	/* SIP (TcpLayer.cpp:387-402), BGP (:403-406) and SSH (:407-410) come before DNS and always take the payload;
	 * DnsOverTcpLayer needs 14 bytes (DnsLayer::isDataValid(.., true), DnsLayer.h:481-485); nothing after DNS
	 * builds an HTTP, DNS or SSL layer */
	uint16_t cls = PCPPX_F_L7_KNOWN;
	int sip_bgp_ssh = 0;
	for (int k = 0; k < 2; ++k) {
		uint16_t x = k ? dp : sp;
		if (x == 5060 || x == 5061 || x == 179 || x == 22) sip_bgp_ssh = 1;
	}
	if (!sip_bgp_ssh && n >= 14 && (dns_port(sp) || dns_port(dp))) cls |= PCPPX_F_L7_DNS;
	return PCPPX_F_NEEDS_HOST_L7 | cls;
}
/* UDP payload: 0 = plain Payload, else PCPPX_F_NEEDS_HOST_L7 | class bits (UdpLayer.cpp:103-183) */
static uint16_t udp_l7(uint32_t n, uint16_t sp, uint16_t dp, int sip)
{
	if (!udp_l7_port(sp, dp) && !sip) return 0;
	int dhcp = (sp == 68 && dp == 67) || (sp == 67 && dp == 68) || (sp == 67 && dp == 67);
	/* DnsLayer after DHCP and VXLAN (UdpLayer.cpp:103-115): 12 bytes (DnsLayer.h:481-485) and a DNS port */
	if (!dhcp && dp != 4789 && n >= 12 && (dns_port(sp) || dns_port(dp)))
		return PCPPX_F_NEEDS_HOST_L7 | PCPPX_F_L7_KNOWN | PCPPX_F_L7_DNS;
	/* VXLAN (dst 4789, VxlanLayer.h:119-122) and GTPv1 (2152/2123, GtpLayer.h:386-389) carry a whole inner
	 * packet whose layers only the host sees */
	if (dp == 4789 || sp == 2152 || dp == 2152 || sp == 2123 || dp == 2123) return PCPPX_F_NEEDS_HOST_L7;
	return PCPPX_F_NEEDS_HOST_L7 | PCPPX_F_L7_KNOWN;
}

/* ---- the classified first L7 layers the engine builds itself (HTTP, SSL, DNS) ----
 * With no parse-until family, a payload classified HTTP / SSL / DNS above (the layer the reference builds is then
 * certain) gets the reference's layers instead of NEEDS_HOST_L7. Each layer's data runs to the end of the L4
 * payload, so the trailer rule is the plain Payload's. */
enum { P_HTTP_REQ = 6, P_HTTP_RESP = 7, P_DNS = 13, P_SSL = 18, P_SSH = 35, P_MYSQL = 63 };
typedef struct {
	uint8_t proto, osi;
	uint32_t off, hdr, dlen;
} lay;
/* HeaderField::HeaderField size, TextBasedProtocol.cpp:448-461: through the first '\n', else strnlen to the end */
static uint32_t tbp_field(const uint8_t* d, uint32_t a, uint32_t n)
{
	const uint8_t* e = (const uint8_t*)memchr(d + a, '\n', n - a);
	if (e) return (uint32_t)(e - (d + a)) + 1;
	return (uint32_t)strnlen((const char*)d + a, n - a);
}
/* TextBasedProtocolMessage::parseFields + getHeaderLen (TextBasedProtocol.cpp:87-139,436-439): fields from the
 * end of the first line until an end-of-header field (size 0, or starting '\r' / '\n'), the end of the data, or
 * an empty field; the header ends with the last field kept */
static uint32_t tbp_header_len(const uint8_t* d, uint32_t fl, uint32_t n)
{
	uint32_t off = fl, s = tbp_field(d, off, n);
	int end = s == 0 || d[off] == '\r' || d[off] == '\n';
	while (!end && off + s < n) {
		uint32_t s2 = tbp_field(d, off + s, n);
		if (s2 == 0) break;
		off += s;
		s = s2;
		end = d[off] == '\r' || d[off] == '\n';
	}
	return off + s;
}
/* HttpRequestFirstLine (HttpLayer.cpp:166-213, parseVersion :287-320, cross_platform_memmem GeneralUtils.cpp:86-113):
 * the first " HTTP/" after the method's space; with room for "x.y" the line ends at the next '\n', else (or with
 * no version) at the end of the data */
static uint32_t http_request_line(const uint8_t* d, uint32_t n)
{
	uint32_t sp = 0;
	while (d[sp] != ' ') ++sp; /* exists: http_request() */
	for (uint32_t v = sp + 1; v + 6 <= n; ++v) {
		if (memcmp(d + v, " HTTP/", 6) != 0) continue;
		if (v + 9 > n) return n;
		const uint8_t* e = (const uint8_t*)memchr(d + v + 6, '\n', n - v - 6);
		return e ? (uint32_t)(e - d) + 1 : n;
	}
	return n;
}
/* HttpResponseFirstLine (HttpLayer.cpp:897-920): through the first '\n' */
static uint32_t http_response_line(const uint8_t* d, uint32_t n)
{
	const uint8_t* e = (const uint8_t*)memchr(d, '\n', n);
	return e ? (uint32_t)(e - d) + 1 : n;
}
/* The layers of a classified L7 payload at [off, off+n) behind the L4 layer l4, appended at index count:
 *   HTTP: HttpRequestLayer / HttpResponseLayer (HttpLayer.cpp:62-68,666-672), a Payload for the body
 *         (TextBasedProtocolMessage::parseNextLayer, TextBasedProtocol.cpp:427-434);
 *   SSL:  one SSLLayer per record (SSLLayer::getHeaderLen / parseNextLayer, SSLLayer.cpp:88-106; every record type
 *         has protocol SSL, OSI presentation, SSLLayer.h:246-249) while the rest is another record header;
 *   DNS:  DnsLayer / DnsOverTcpLayer, header = the whole data, no next layer (DnsLayer.h:353-372);
 *   MySQL: MySqlLayer, header = the whole data, application layer, no next layer (MySqlLayer.h:362-379);
 *   SSH:  one layer per message (SSHLayer::createSSHMessage / parseNextLayer, SSHLayer.cpp:18-40): an identification
 *         message ("SSH-" ... '\n', SSHLayer.cpp:46-56) or an encrypted one takes the rest, a handshake message
 *         (:135-170) its packet length + 4; application layer (SSHLayer.h:107-110).
 * Each layer passes the stop rules of Packet::parsePacket (Packet.cpp:134-155) before it is kept; the first one
 * that fails is rolled back (:168-175) and ends the chain (*stopped). Returns the new count; *last is the last
 * layer kept. */
static int family_member(uint32_t fam, uint8_t p);
static int l7_layers(const uint8_t* pkt, uint32_t off, uint32_t n, uint16_t cls, const lay* l4, const pcppx_opts* opts,
                     int* found, int* stopped, pcppx_layer* layers, int cap, int count, uint64_t* mask, lay* last)
{
	const uint8_t* d = pkt + off;
	lay L = { 0, 7, off, 0, n };
#define EMIT() do { \
		int member_ = family_member(opts->parse_until_family, L.proto); \
		int fail_ = L.osi > opts->parse_until_osi; \
		if (!fail_) { \
			if (opts->parse_until_family != 0 && member_) *found = 1; \
			if (*found && !member_) fail_ = 1; \
		} \
		if (fail_) { *stopped = 1; goto done; } \
		if (layers && count < cap) { \
			pcppx_layer* o = &layers[count]; \
			o->proto = L.proto; o->osi = L.osi; \
			o->offset = (uint16_t)L.off; o->hdr_len = (uint16_t)L.hdr; o->data_len = (uint16_t)L.dlen; \
		} \
		*mask |= (uint64_t)1 << L.proto; *last = L; ++count; } while (0)
	if (cls & PCPPX_F_L7_HTTP) {
		const int req = http_port(be16(pkt + l4->off + 2)) && http_request(d, n); /* tcp_l7's order */
		L.proto = req ? P_HTTP_REQ : P_HTTP_RESP;
		L.hdr = tbp_header_len(d, req ? http_request_line(d, n) : http_response_line(d, n), n);
		EMIT();
		if (n > L.hdr) {
			L.proto = P_PAYLOAD; L.off = off + L.hdr; L.dlen = n - L.hdr; L.hdr = L.dlen;
			EMIT();
		}
	} else if (cls & PCPPX_F_L7_SSL) {
		uint32_t ro = off, rem = n;
		for (;;) {
			uint32_t hl = 5u + be16(pkt + ro + 3);
			if (hl > rem) hl = rem;
			L.proto = P_SSL; L.osi = 6; L.off = ro; L.hdr = hl; L.dlen = rem;
			EMIT();
			if (rem <= hl || !ssl_record(pkt + ro + hl, rem - hl)) break;
			ro += hl;
			rem -= hl;
		}
	} else if (cls & L7_MYSQL) {
		L.proto = P_MYSQL; L.hdr = n;
		EMIT();
	} else if (cls & L7_SSH) {
		uint32_t ro = off, rem = n;
		for (;;) {
			const uint8_t* m = pkt + ro;
			uint32_t hl = rem;
			const int ident = rem >= 5 && memcmp(m, "SSH-", 4) == 0 && m[rem - 1] == '\n';
			if (!ident && rem >= 6) {
				const uint32_t ml4 = ((uint32_t)m[0] << 24) | ((uint32_t)m[1] << 16) | ((uint32_t)m[2] << 8) | m[3];
				if ((uint64_t)ml4 + 4 <= rem && m[4] <= ml4 && (m[5] == 20 || m[5] == 21 || (m[5] >= 30 && m[5] <= 49)))
					hl = ml4 + 4;
			}
			L.proto = P_SSH; L.osi = 7; L.off = ro; L.hdr = hl; L.dlen = rem;
			EMIT();
			if (rem <= hl) break;
			ro += hl;
			rem -= hl;
		}
	} else {
		L.proto = P_DNS; L.hdr = n;
		EMIT();
	}
#undef EMIT
done:
	return count;
}

/* ---- parse-until roll-back of a layer this path does not build (Packet.cpp:134-155, 168-175) ----
 * Where the chain reaches a layer the engine leaves to the host (an L7 dissector, or an out-of-scope
 * L2/L3 layer), Packet::parsePacket still builds it and then applies the stop rules to it: it is rolled
 * back (and with it everything the host would parse behind it) when its OSI layer is above
 * parseUntilLayer, or when the parse-until family was already found and the layer is not a member. The
 * engine does not know WHICH layer the host builds, only the candidates; the roll-back is certain when it
 * holds for every candidate:
 *   - every candidate's OSI layer exceeds parse_until_osi (min_osi below: the smallest candidate OSI), or
 *   - the family was found and holds only protocols the engine itself builds, which no candidate is
 *     (GenericPayload excluded: a port-triggered dissector may fall back to Payload).
 * The chain is then exact and ends before that layer: no NEEDS_HOST flag.
 *
 * Candidate OSI layers (each Layer::getOsiModelLayer override in Packet++/header):
 *   TCP payload (TcpLayer.cpp:372-491): TPKT 102 (TpktLayer.h:98-101) and GTPv2 2123 (GtpLayer.h:1112-1115)
 *     transport 4; SIP 5060/5061 session 5 (SipLayer.h:96-99); SSL presentation 6 (SSLLayer.h:246-249);
 *     every other dissector and Payload application 7.
 *   UDP payload (UdpLayer.cpp:103-183): VXLAN dst 4789 (VxlanLayer.h:141-144) and WakeOnLan dst 0/7/9
 *     (WakeOnLanLayer.h:133-135) data link 2; WireGuard 51820 network 3 (WireGuardLayer.h:114-117); GTPv1
 *     2152/2123 (GtpLayer.h:386-389,408-411) and GTPv2 2123 transport 4; SIP by port or by the content
 *     heuristic session 5; the rest 7.
 *   Out-of-scope L2 layers (PPPoE PPPoELayer.h:92, WakeOnLan, STP StpLayer.h:204-207) 2; out-of-scope
 *   IP-protocol layers (ICMP, IGMP, AH, VRRP, ICMPv6: network 3; ESP transport 4) 3. */
static uint8_t tcp_l7_min_osi(uint16_t sp, uint16_t dp)
{
	if (sp == 102 || dp == 102 || sp == 2123 || dp == 2123) return 4;
	if (sp == 5060 || sp == 5061 || dp == 5060 || dp == 5061) return 5;
	if (ssl_port(sp) || ssl_port(dp)) return 6;
	return 7;
}
static uint8_t udp_l7_min_osi(uint16_t sp, uint16_t dp, int sip_content)
{
	if (dp == 4789 || dp == 0 || dp == 7 || dp == 9) return 2;
	if (sp == 51820 || dp == 51820) return 3;
	if (sp == 2152 || dp == 2152 || sp == 2123 || dp == 2123) return 4;
	if (sp == 5060 || sp == 5061 || dp == 5060 || dp == 5061 || sip_content) return 5;
	return 7;
}
/* a classified first L7 layer has its own OSI layer (HttpLayer.h:87-90 application, SSLLayer.h:246-249
 * presentation, DnsLayer.h:369-372 application); otherwise the smallest over the port candidates */
static uint8_t l7_osi(uint16_t cls, uint8_t min_osi)
{
	if (cls & PCPPX_F_L7_SSL) return 6;
	if (cls & (PCPPX_F_L7_HTTP | PCPPX_F_L7_DNS | L7_MYSQL | L7_SSH)) return 7;
	return min_osi;
}
/* the protocols the engine builds itself (ProtocolType.h:42-258), GenericPayload excluded */
static int engine_proto(uint32_t p)
{
	switch (p) {
	case P_ETH: case P_IPV4: case P_IPV6: case P_TCP: case P_UDP: case P_ARP: case P_VLAN: case P_MPLS:
	case P_GREV0: case P_GREV1: case P_PPTP: case P_TRAILER: case P_DOT3: case P_LLC: case P_ICMP: return 1;
	case P_VXLAN: case P_GTPV1: return 1; /* decided exactly at the UDP layer, never a host candidate */
	case P_NFLOG: case P_CISCO_HDLC: return 1; /* first layers the engine builds (round 6) */
	/* a classified first L7 layer is built, an unclassified one is none of these */
	case P_HTTP_REQ: case P_HTTP_RESP: case P_DNS: case P_SSL: case P_MYSQL: case P_SSH: return 1;
	default: return 0;
	}
}
static int family_engine_only(uint32_t fam)
{
	if (fam == 0) return 0;
	for (int k = 0; k < 4; ++k) {
		uint32_t b = (fam >> (8 * k)) & 0xFF;
		if (b != 0 && !engine_proto(b)) return 0;
	}
	return 1;
}

/* ---- computeChecksum, Packet++/src/PacketUtils.cpp:12-64 ---- */
uint16_t pcppx_oracle_checksum(const uint8_t* const* bufs, const uint32_t* lens, int nbufs)
{
	uint32_t sum = 0;
	for (int i = 0; i < nbufs; ++i) {
		uint32_t local = 0;
		for (uint32_t j = 0; j < lens[i] / 2; ++j) local += le16(bufs[i] + 2 * j);
		if (lens[i] % 2) local += bufs[i][lens[i] - 1]; /* be16toh(lastByte << 8) on LE == lastByte */
		while (local >> 16) local = (local & 0xFFFF) + (local >> 16);
		sum += local;
	}
	while (sum >> 16) sum = (sum & 0xFFFF) + (sum >> 16);
	uint16_t result = (uint16_t)~sum;
	return bswap16(result); /* htobe16 */
}

/* ---- fnvHash (FNV-1 32), Packet++/src/PacketUtils.cpp:114-137 ---- */
static uint32_t fnv_update(uint32_t h, const uint8_t* p, uint32_t n)
{
	for (uint32_t j = 0; j < n; ++j) { h *= 16777619u; h ^= p[j]; }
	return h;
}
uint32_t pcppx_oracle_fnv1(const uint8_t* buf, uint32_t len) { return fnv_update(2166136261u, buf, len); }

/* ProtocolTypeFamily membership, ProtocolType.h:293-298 + Layer.cpp:47-50 */
static int family_member(uint32_t fam, uint8_t p)
{
	uint32_t q = p;
	return p != 0 && (q == (fam & 0xff) || (q << 8) == (fam & 0xff00) || (q << 16) == (fam & 0xff0000) ||
	                  (q << 24) == (fam & 0xff000000u));
}

/* Build layer `k` at [off, off+len) and report its next layer through nk, noff, nlen.
 * Returns the layer descriptor. */
static lay make_layer(const uint8_t* pkt, int k, uint32_t off, uint32_t len, int* nk, uint32_t* noff, uint32_t* nlen,
                      uint8_t* nosi, uint16_t* ncls)
{
	const uint8_t* p = pkt + off;
	lay L = { 0, 0, off, 0, len };
	*nk = K_NONE;
	*nosi = 7; /* smallest OSI layer of the host-built candidates when *nk is K_OUT / K_L7 */
	*ncls = 0; /* K_L7: PCPPX_F_NEEDS_HOST_L7 | PCPPX_F_L7_* */
	uint32_t po, pl; /* payload of this layer */
#define NEXT(K, O, N) do { *nk = (K); *noff = (O); *nlen = (N); } while (0)
	switch (k) {
	case K_ETH: /* EthLayer::parseNextLayer, Packet++/src/EthLayer.cpp:28-69 */
		L.proto = P_ETH; L.osi = 2; L.hdr = 14;
		if (len <= 14) break;
		po = off + 14; pl = len - 14;
		switch (be16(p + 12)) {
		case 0x0800: NEXT(ipv4_valid(pkt + po, pl) ? K_IPV4 : K_PAYLOAD, po, pl); break;
		case 0x86DD: NEXT(ipv6_valid(pkt + po, pl) ? K_IPV6 : K_PAYLOAD, po, pl); break;
		case 0x8100: case 0x88A8: NEXT(pl >= 4 ? K_VLAN : K_PAYLOAD, po, pl); break;
		case 0x8847: NEXT(pl >= 4 ? K_MPLS : K_PAYLOAD, po, pl); break;
		case 0x0806: NEXT(pl >= 28 ? K_ARP : K_PAYLOAD, po, pl); break; /* ArpLayer::isDataValid, ArpLayer.h:279-282 */
		case 0x8864: case 0x8863: case 0x0842: NEXT(K_OUT, po, pl); *nosi = 2; break; /* PPPoE, WoL */
		default: NEXT(K_PAYLOAD, po, pl); break;
		}
		break;
	case K_SLL:  /* SllLayer::parseNextLayer, Packet++/src/SllLayer.cpp:49-102 (protocol_type at 14, SllLayer.h:15-32) */
	case K_SLL2: /* Sll2Layer::parseNextLayer, Packet++/src/Sll2Layer.cpp:63-121 (protocol_type at 0, Sll2Layer.h:15-35) */
		L.proto = k == K_SLL ? P_SLL : P_SLL2; L.osi = 2; L.hdr = k == K_SLL ? 16 : 20;
		if (len <= L.hdr) break;
		po = off + L.hdr; pl = len - L.hdr;
		switch (be16(p + (k == K_SLL ? 14 : 0))) {
		case 0x0800: NEXT(ipv4_valid(pkt + po, pl) ? K_IPV4 : K_PAYLOAD, po, pl); break;
		case 0x86DD: NEXT(ipv6_valid(pkt + po, pl) ? K_IPV6 : K_PAYLOAD, po, pl); break;
		case 0x0806: NEXT(K_ARP, po, pl); break;                  /* unchecked */
		case 0x8100: case 0x88A8: NEXT(K_VLAN, po, pl); break;    /* unchecked */
		case 0x8864: case 0x8863: NEXT(K_OUT, po, pl); *nosi = 2; break; /* PPPoE */
		case 0x8847: NEXT(K_MPLS, po, pl); break;                 /* unchecked */
		case 0x0004: /* Sll2ProtoTypeLLC, Sll2Layer.cpp:20,110-114 */
			if (k == K_SLL2) { NEXT(llc_valid(pkt + po, pl) ? K_LLC : K_PAYLOAD, po, pl); break; }
			NEXT(K_PAYLOAD, po, pl); break;
		default: NEXT(K_PAYLOAD, po, pl); break;
		}
		break;
	case K_HDLC: /* CiscoHdlcLayer::parseNextLayer, Packet++/src/CiscoHdlcLayer.cpp:43-67: a 4-byte header (address,
	              * control, protocol), no length check -- a 4-byte packet gets an empty Payload */
		L.proto = P_CISCO_HDLC; L.osi = 2; L.hdr = 4;
		po = off + 4; pl = len - 4;
		switch (be16(p + 2)) {
		case 0x0800: NEXT(ipv4_valid(pkt + po, pl) ? K_IPV4 : K_PAYLOAD, po, pl); break;
		case 0x86DD: NEXT(ipv6_valid(pkt + po, pl) ? K_IPV6 : K_PAYLOAD, po, pl); break;
		default: NEXT(K_PAYLOAD, po, pl); break;
		}
		break;
	case K_NFLOG: { /* NflogLayer, Packet++/src/NflogLayer.cpp:41-96: a 4-byte nflog_header (family, version, resource
	                 * id), then TLVs {u16 length, u16 type, value} (host byte order), each taking align<4>(length) bytes
	                 * (NflogLayer.h NflogTlv::getTotalSize), walked as TLVRecordReader does (TLVData.h:238-312) */
		L.proto = P_NFLOG; L.osi = 2; L.hdr = 4;
		const uint32_t tl = len - 4; /* the TLV stream */
		uint32_t pos = 0;            /* current record, relative to the stream */
		int found_payload = 0, have = 0;
		uint32_t total = 0;
		if (tl >= 2) { /* getFirstTLVRecord: canAssign, then the record must fit and be non-empty */
			total = (le16(p + 4) + 3u) & ~3u;
			have = total != 0 && total <= tl;
		}
		while (have) {
			if (le16(p + 4 + pos + 2) == 9) { found_payload = 1; break; } /* NFULA_PAYLOAD */
			L.hdr += total;                                             /* getHeaderLen: every record before it */
			pos += total;
			/* getNextTLVRecord: canAssign (>= 2 bytes left), a non-empty record that fits */
			if (tl - pos < 2) { have = 0; break; }
			total = (le16(p + 4 + pos) + 3u) & ~3u;
			have = total != 0 && pos + total <= tl;
		}
		if (!found_payload) break;
		L.hdr += 4; /* the payload record's length and type */
		if (len <= 4) break; /* parseNextLayer: m_DataLen <= sizeof(nflog_header) */
		po = off + 4 + pos + 4; pl = total - 4;
		switch (p[0]) { /* the address family: NflogFamilyIpv4 = 2, NflogFamilyIpv6 = 10 */
		case 2: NEXT(ipv4_valid(pkt + po, pl) ? K_IPV4 : K_PAYLOAD, po, pl); break;
		case 10: NEXT(ipv6_valid(pkt + po, pl) ? K_IPV6 : K_PAYLOAD, po, pl); break;
		default: NEXT(K_PAYLOAD, po, pl); break;
		}
		break;
	}
	case K_NULL: { /* NullLoopbackLayer::getFamily :23-43, parseNextLayer :50-99 (no length check: a 4-byte packet
	                * gets an empty next layer) */
		L.proto = P_NULL; L.osi = 2; L.hdr = 4;
		po = off + 4; pl = len - 4;
		uint32_t fam = le32(p);
		if (fam & 0xFFFF0000u) {
			if ((fam & 0xFF000000u) == 0 && (fam & 0x00FF0000u) < 0x00060000u) fam >>= 16;
			else fam = (fam >> 24) | ((fam >> 8) & 0xFF00u) | ((fam << 8) & 0xFF0000u) | (fam << 24);
		} else if ((fam & 0xFFu) == 0 && (fam & 0xFF00u) < 0x0600u) {
			/* BSWAP16 (:10) does not truncate to 16 bits: x >> 8 | x << 8 of a 32-bit value */
			fam = ((fam & 0xFFFFu) >> 8) | ((fam & 0xFFFFu) << 8);
		}
		int v4 = 0, v6 = 0;
		if (fam > 1500) { /* Ieee8023MaxLength: an EtherType */
			v4 = (uint16_t)fam == 0x0800; v6 = (uint16_t)fam == 0x86DD;
		} else {
			v4 = fam == 2; v6 = fam == 24 || fam == 28 || fam == 30; /* BSD AF_INET / AF_INET6 variants */
		}
		if (v4) NEXT(ipv4_valid(pkt + po, pl) ? K_IPV4 : K_PAYLOAD, po, pl);
		else if (v6) NEXT(ipv6_valid(pkt + po, pl) ? K_IPV6 : K_PAYLOAD, po, pl);
		else NEXT(K_PAYLOAD, po, pl);
		break;
	}
	case K_DOT3: /* EthDot3Layer::parseNextLayer, Packet++/src/EthDot3Layer.cpp:22-30 */
		L.proto = P_DOT3; L.osi = 2; L.hdr = 14;
		if (len <= 14) break;
		po = off + 14; pl = len - 14;
		NEXT(llc_valid(pkt + po, pl) ? K_LLC : K_PAYLOAD, po, pl);
		break;
	case K_LLC: /* LLCLayer::parseNextLayer, Packet++/src/LLCLayer.cpp:24-41 */
		L.proto = P_LLC; L.osi = 2; L.hdr = 3;
		if (len <= 3) break;
		po = off + 3; pl = len - 3;
		if (p[0] == 0x42 && p[1] == 0x42) { NEXT(K_OUT, po, pl); *nosi = 2; } /* STP (or Payload): host */
		else NEXT(K_PAYLOAD, po, pl);
		break;
	case K_VLAN: /* VlanLayer::parseNextLayer, Packet++/src/VlanLayer.cpp:59-119 */
		L.proto = P_VLAN; L.osi = 2; L.hdr = 4;
		if (len <= 4) break;
		po = off + 4; pl = len - 4;
		switch (be16(p + 2)) {
		case 0x0800: NEXT(ipv4_valid(pkt + po, pl) ? K_IPV4 : K_PAYLOAD, po, pl); break;
		case 0x86DD: NEXT(ipv6_valid(pkt + po, pl) ? K_IPV6 : K_PAYLOAD, po, pl); break;
		case 0x8100: case 0x88A8: NEXT(K_VLAN, po, pl); break; /* unchecked */
		case 0x8847: NEXT(K_MPLS, po, pl); break;              /* unchecked */
		case 0x0806: NEXT(K_ARP, po, pl); break; /* unchecked */
		case 0x8864: case 0x8863: NEXT(K_OUT, po, pl); *nosi = 2; break;
		default:
			if (be16(p + 2) < 1500) NEXT(llc_valid(pkt + po, pl) ? K_LLC : K_PAYLOAD, po, pl);
			else NEXT(K_PAYLOAD, po, pl);
			break;
		}
		break;
	case K_MPLS: /* MplsLayer::parseNextLayer, Packet++/src/MplsLayer.cpp:101-128 */
		L.proto = P_MPLS; L.osi = 3; L.hdr = 4;
		if (len < 5) break;
		po = off + 4; pl = len - 4;
		if (!(p[2] & 1)) { NEXT(K_MPLS, po, pl); break; } /* not bottom-of-stack: unchecked */
		switch (p[4] >> 4) {
		case 4: NEXT(ipv4_valid(pkt + po, pl) ? K_IPV4 : K_PAYLOAD, po, pl); break;
		case 6: NEXT(ipv6_valid(pkt + po, pl) ? K_IPV6 : K_PAYLOAD, po, pl); break;
		default: NEXT(K_PAYLOAD, po, pl); break;
		}
		break;
	case K_IPV4: { /* IPv4Layer: initLayerInPacket Packet++/src/IPv4Layer.cpp:180-197; parseNextLayer :245-370 */
		L.proto = P_IPV4; L.osi = 3; L.hdr = (uint32_t)(p[0] & 0xF) * 4;
		uint32_t tl = be16(p + 2);
		if (tl < len && tl != 0) {
			uint32_t hmin = L.hdr < len ? L.hdr : len;
			L.dlen = tl > hmin ? tl : hmin;
		}
		if (L.dlen <= L.hdr || L.hdr == 0) break;
		po = off + L.hdr; pl = L.dlen - L.hdr;
		/* isFragment :415-418, getFragmentFlags/Offset :430-438 */
		if ((p[6] & 0x20) || (((p[6] & 0x1F) << 8) | p[7]) != 0) { NEXT(K_PAYLOAD, po, pl); break; }
		switch (p[9]) {
		case 17: NEXT(pl >= 8 ? K_UDP : K_PAYLOAD, po, pl); break;
		case 6: NEXT(tcp_valid(pkt + po, pl) ? K_TCP : K_PAYLOAD, po, pl); break;
		case 4: /* IPLayer::getIPVersion, Packet++/src/IPLayer.cpp:5-25 */
			switch (pkt[po] >> 4) {
			case 4: NEXT(ipv4_valid(pkt + po, pl) ? K_IPV4 : K_PAYLOAD, po, pl); break;
			case 6: NEXT(ipv6_valid(pkt + po, pl) ? K_IPV6 : K_PAYLOAD, po, pl); break;
			default: NEXT(K_PAYLOAD, po, pl); break;
			}
			break;
		case 47: /* GreLayer::getGREVersion, Packet++/src/GreLayer.cpp:23-36 */
			if (pl < 4) NEXT(K_PAYLOAD, po, pl);
			else if ((pkt[po + 1] & 7) == 0) NEXT(K_GRE0, po, pl);
			else if ((pkt[po + 1] & 7) == 1) NEXT(pl >= 8 ? K_GRE1 : K_PAYLOAD, po, pl);
			else NEXT(K_PAYLOAD, po, pl);
			break;
		case 41: NEXT(ipv6_valid(pkt + po, pl) ? K_IPV6 : K_PAYLOAD, po, pl); break;
		case 1: NEXT(icmp_valid(pkt + po, pl) ? K_ICMP : K_PAYLOAD, po, pl); break; /* tryConstruct, :272-274 */
		case 2: case 51: case 50: case 112: NEXT(K_OUT, po, pl); *nosi = 3; break; /* IGMP AH ESP VRRP */
		default: NEXT(K_PAYLOAD, po, pl); break;
		}
		break;
	}
	case K_IPV6: { /* IPv6Layer ctor Packet++/src/IPv6Layer.cpp:28-40; parseExtensions :79-147 */
		L.proto = P_IPV6; L.osi = 3;
		uint8_t nh = p[6];
		uint32_t eo = 40, ext = 0;
		int last_ext = -1;
		while (eo <= len - 2) {
			uint32_t el;
			if (nh == 44 || nh == 0 || nh == 60 || nh == 43) el = 8u * ((uint32_t)p[eo + 1] + 1); /* IPv6Extensions.h:40-43 */
			else if (nh == 51) el = 4u * ((uint32_t)p[eo + 1] + 2);                            /* IPv6Extensions.h:480-483 */
			else break;
			last_ext = nh;
			nh = p[eo];
			eo += el;
			ext += el;
		}
		L.hdr = 40 + ext;
		uint32_t total = (uint32_t)be16(p + 4) + L.hdr; /* payloadLength + getHeaderLen() */
		if (total < len) L.dlen = total;
		/* parseNextLayer :194-312 */
		if (L.dlen <= L.hdr) break;
		po = off + L.hdr; pl = L.dlen - L.hdr;
		if (last_ext == 44) { NEXT(K_PAYLOAD, po, pl); break; }
		switch (nh) {
		case 17: NEXT(pl >= 8 ? K_UDP : K_PAYLOAD, po, pl); break;
		case 6: NEXT(tcp_valid(pkt + po, pl) ? K_TCP : K_PAYLOAD, po, pl); break;
		case 4:
			switch (pkt[po] >> 4) {
			case 4: NEXT(ipv4_valid(pkt + po, pl) ? K_IPV4 : K_PAYLOAD, po, pl); break;
			case 6: NEXT(ipv6_valid(pkt + po, pl) ? K_IPV6 : K_PAYLOAD, po, pl); break;
			default: NEXT(K_PAYLOAD, po, pl); break;
			}
			break;
		case 47:
			if (pl < 4) NEXT(K_PAYLOAD, po, pl);
			else if ((pkt[po + 1] & 7) == 0) NEXT(K_GRE0, po, pl);
			else if ((pkt[po + 1] & 7) == 1) NEXT(pl >= 8 ? K_GRE1 : K_PAYLOAD, po, pl);
			else NEXT(K_PAYLOAD, po, pl);
			break;
		case 51: case 50: case 58: case 112: NEXT(K_OUT, po, pl); *nosi = 3; break; /* AH ESP ICMPv6 VRRP */
		default: NEXT(K_PAYLOAD, po, pl); break;
		}
		break;
	}
	case K_GRE0:
	case K_GRE1: { /* GreLayer::getHeaderLen :237-252, parseNextLayer :195-235; bitfields GreLayer.h:14-57 */
		L.proto = k == K_GRE0 ? P_GREV0 : P_GREV1; L.osi = 3;
		L.hdr = 4;
		if ((p[0] & 0x80) || (p[0] & 0x40)) L.hdr += 4; /* checksum | routing */
		if (p[0] & 0x20) L.hdr += 4;                    /* key */
		if (p[0] & 0x10) L.hdr += 4;                    /* sequence */
		if (p[1] & 0x80) L.hdr += 4;                    /* ack */
		if (len <= L.hdr) break;
		po = off + L.hdr; pl = len - L.hdr;
		switch (be16(p + 2)) {
		case 0x0800: NEXT(ipv4_valid(pkt + po, pl) ? K_IPV4 : K_PAYLOAD, po, pl); break;
		case 0x86DD: NEXT(ipv6_valid(pkt + po, pl) ? K_IPV6 : K_PAYLOAD, po, pl); break;
		case 0x8100: NEXT(K_VLAN, po, pl); break; /* unchecked */
		case 0x8847: NEXT(K_MPLS, po, pl); break; /* unchecked */
		case 0x880B: NEXT(pl >= 4 ? K_PPTP : K_PAYLOAD, po, pl); break;
		case 0x6558:
			if (eth_valid(pkt + po, pl)) NEXT(K_ETH, po, pl);
			else NEXT(dot3_valid(pkt + po, pl) ? K_DOT3 : K_PAYLOAD, po, pl);
			break;
		default: NEXT(K_PAYLOAD, po, pl); break;
		}
		break;
	}
	case K_PPTP: /* PPP_PPTPLayer::parseNextLayer, Packet++/src/GreLayer.cpp:547-566 */
		L.proto = P_PPTP; L.osi = 5; L.hdr = 4;
		if (len <= 4) break;
		po = off + 4; pl = len - 4;
		switch (be16(p + 2)) {
		case 0x21: NEXT(ipv4_valid(pkt + po, pl) ? K_IPV4 : K_PAYLOAD, po, pl); break;
		case 0x57: NEXT(ipv6_valid(pkt + po, pl) ? K_IPV6 : K_PAYLOAD, po, pl); break;
		default: NEXT(K_PAYLOAD, po, pl); break;
		}
		break;
	case K_TCP: /* TcpLayer::getHeaderLen TcpLayer.h:565-568; parseNextLayer TcpLayer.cpp:360-492 */
		L.proto = P_TCP; L.osi = 4; L.hdr = (uint32_t)(p[12] >> 4) * 4;
		if (len <= L.hdr) break;
		po = off + L.hdr; pl = len - L.hdr;
		*ncls = tcp_l7(pkt + po, pl, be16(p), be16(p + 2));
		NEXT(*ncls ? K_L7 : K_PAYLOAD, po, pl);
		*nosi = l7_osi(*ncls, tcp_l7_min_osi(be16(p), be16(p + 2)));
		break;
	case K_UDP: /* UdpLayer::parseNextLayer, Packet++/src/UdpLayer.cpp:92-184 */
		L.proto = P_UDP; L.osi = 4; L.hdr = 8;
		if (len <= 8) break;
		po = off + 8; pl = len - 8;
		{
			/* the tunnels, decided here as UdpLayer::parseNextLayer does (:103-131): VXLAN by destination port
			 * (tryConstruct, VxlanLayer.h:97-100: 8 bytes), GTPv1 by port and GtpV1Layer::isGTPv1 (GtpLayer.cpp:
			 * 199-207) where no earlier dissector takes the payload: DHCP, DNS, SIP (by port), RADIUS (by port and
			 * RadiusLayer::isDataValid, RadiusLayer.cpp:238-247: 20 <= length field <= data) */
			const uint16_t sp = be16(p), dp = be16(p + 2);
			if (dp == 4789) { NEXT(pl >= 8 ? K_VXLAN : K_PAYLOAD, po, pl); break; }
			int dhcp = (sp == 68 && dp == 67) || (sp == 67 && dp == 68) || (sp == 67 && dp == 67);
			int dnsb = pl >= 12 && (dns_port(sp) || dns_port(dp));
			int sipp = 0, radp = 0;
			for (int k = 0; k < 2; ++k) {
				uint16_t x = k ? dp : sp;
				if (x == 5060 || x == 5061) sipp = 1;
				if (x == 1812 || x == 1813 || x == 3799) radp = 1;
			}
			int rad = radp && pl >= 20 && be16(pkt + po + 2) >= 20 && be16(pkt + po + 2) <= pl;
			int gport = sp == 2152 || dp == 2152 || sp == 2123 || dp == 2123;
			if (gport && !dhcp && !dnsb && !sipp && !rad && pl >= 8 && (pkt[po] & 0xE0) == 0x20) {
				NEXT(K_GTP1, po, pl);
				break;
			}
			int sip = sip_heuristic(pkt + po, pl);
			*ncls = udp_l7(pl, sp, dp, sip);
			NEXT(*ncls ? K_L7 : K_PAYLOAD, po, pl);
			*nosi = l7_osi(*ncls, udp_l7_min_osi(be16(p), be16(p + 2), sip));
		}
		break;
	case K_VXLAN: /* VxlanLayer (OSI data link, VxlanLayer.h:130-144): 8-byte header; parseNextLayer VxlanLayer.cpp:50-58:
	               * Ethernet (tryConstruct), else a Payload */
		L.proto = P_VXLAN; L.osi = 2; L.hdr = 8;
		if (len <= 8) break;
		po = off + 8; pl = len - 8;
		NEXT(eth_valid(pkt + po, pl) ? K_ETH : K_PAYLOAD, po, pl);
		break;
	case K_GTP1: { /* GtpV1Layer (OSI transport, GtpLayer.h:408-411): getHeaderLen GtpLayer.cpp:602-632, the extension
	                * chain GtpExtension :60-120 and :323-350; parseNextLayer :560-600 (G-PDU only) */
		L.proto = P_GTPV1; L.osi = 4; L.hdr = 8;
		const uint8_t fl = p[0], mt = p[1];
		if (mt != 0xFF) {
			uint32_t ml = be16(p + 2);
			L.hdr += ml > len - 8 ? len - 8 : ml;
			break; /* GTP-C: the last layer */
		}
		if (len >= 12 && (fl & 7)) {
			L.hdr += 4; /* gtpv1_header_extra */
			uint32_t nt = p[11];
			if ((fl & 4) && nt != 0 && len > 12) {
				uint32_t ed = 12, erem = len - 12;
				for (;;) {
					uint32_t tl = 4u * p[ed];
					if (tl > erem) tl = erem;
					L.hdr += tl;
					nt = tl >= 4 ? p[ed + tl - 1] : 0;
					if (nt == 0 || erem <= tl + 1) break;
					ed += tl;
					erem -= tl;
				}
			}
		}
		if (len <= L.hdr) break;
		po = off + L.hdr; pl = len - L.hdr;
		{
			uint8_t sub = pkt[po];
			if (sub >= 0x45 && sub <= 0x4e) NEXT(ipv4_valid(pkt + po, pl) ? K_IPV4 : K_PAYLOAD, po, pl);
			else if ((sub & 0xf0) == 0x60) NEXT(ipv6_valid(pkt + po, pl) ? K_IPV6 : K_PAYLOAD, po, pl);
			else NEXT(K_PAYLOAD, po, pl);
		}
		break;
	}
	case K_ICMP: { /* IcmpLayer (OSI network, IcmpLayer.h:611-614): getHeaderLen by message type, IcmpLayer.cpp:589-620
	                * (getMessageType :36-43); parseNextLayer :562-587: the error messages carry the offending IPv4
	                * header (tryConstruct IPv4, else a Payload, even an empty one), the rest a Payload past the header */
		L.proto = P_ICMP; L.osi = 3;
		int err = 0;
		switch (p[0]) {
		case 0: case 8: L.hdr = len; break;
		case 13: case 14: L.hdr = 20; break;
		case 17: case 18: L.hdr = 12; break;
		case 3: case 4: case 5: case 11: case 12: L.hdr = 8; err = 1; break;
		case 9: { uint32_t ra = 8u + 8u * p[4]; L.hdr = ra > len ? len : ra; break; }
		default: L.hdr = 4; break; /* 10, 15, 16 */
		}
		po = off + L.hdr; pl = len - L.hdr;
		if (err) NEXT(ipv4_valid(pkt + po, pl) ? K_IPV4 : K_PAYLOAD, po, pl);
		else if (len > L.hdr) NEXT(K_PAYLOAD, po, pl);
		break;
	}
	case K_ARP: /* ArpLayer: dataLen := sizeof(arphdr) = 28 whatever remains, no next (ArpLayer.h:151-155,242-273) */
		L.proto = P_ARP; L.osi = 3; L.hdr = 28; L.dlen = 28;
		break;
	case K_PAYLOAD: /* PayloadLayer: header = whole data, no next (PayloadLayer.h:61-81) */
		L.proto = P_PAYLOAD; L.osi = 7; L.hdr = len;
		break;
	default: break;
	}
#undef NEXT
	return L;
}

/* the 5-tuple extract (include/pcppx.h pcppx_tuple): the fields hash5Tuple reads, PacketUtils.cpp:139-210 -- the first
 * IPv4 layer (getLayerOfType<IPv4Layer>()), else the first IPv6 layer: ipSrc / ipDst and protocol / nextHeader
 * (:177-201); the last TCP layer, else the last UDP layer (getLayerOfType<TcpLayer>(true) / <UdpLayer>(true),
 * :157-169): getSrcPort / getDstPort (TcpLayer.cpp:54-62, UdpLayer.cpp:37-45: be16toh of the header fields); 5-tuple
 * iff an IP layer, a port layer and no ICMP layer (:141-148) */
static void fill_tuple(const uint8_t* pkt, const pcppx_summary* sum, int have_ipv4, const lay* ip4, int have_ipv6,
                       const lay* ip6, int l4_idx, int l4_is_tcp, const lay* l4, pcppx_tuple* t)
{
	memset(t, 0, sizeof(*t));
	if (have_ipv4) {
		const uint8_t* ip = pkt + ip4->off;
		memcpy(t->src_ip, ip + 12, 4);
		memcpy(t->dst_ip, ip + 16, 4);
		t->ip_version = 4;
		t->ip_proto = ip[9];
	} else if (have_ipv6) {
		const uint8_t* ip = pkt + ip6->off;
		memcpy(t->src_ip, ip + 8, 16);
		memcpy(t->dst_ip, ip + 24, 16);
		t->ip_version = 6;
		t->ip_proto = ip[6];
	}
	if (l4_idx >= 0) {
		const uint8_t* lp = pkt + l4->off;
		t->src_port = be16(lp);
		t->dst_port = be16(lp + 2);
		t->l4_proto = l4_is_tcp ? P_TCP : P_UDP;
	}
	t->has_5tuple = (have_ipv4 || have_ipv6) && l4_idx >= 0 && !(sum->proto_mask & ((uint64_t)1 << P_ICMP));
	t->hash5 = sum->hash5;
	t->flags = sum->flags;
	t->n_layers = sum->n_layers;
}

static void parse_packet(const uint8_t* pkt, uint32_t caplen, uint16_t linktype, const pcppx_opts* opts,
                         pcppx_summary* sum, pcppx_layer* layers, pcppx_tuple* tup);

void pcppx_oracle_parse_packet(const uint8_t* pkt, uint32_t caplen, uint16_t linktype, const pcppx_opts* opts,
                               pcppx_summary* sum, pcppx_layer* layers)
{
	parse_packet(pkt, caplen, linktype, opts, sum, layers, NULL);
}

static void parse_packet(const uint8_t* pkt, uint32_t caplen, uint16_t linktype, const pcppx_opts* opts,
                         pcppx_summary* sum, pcppx_layer* layers, pcppx_tuple* tup)
{
	if (tup) memset(tup, 0, sizeof(*tup));
	memset(sum, 0, sizeof(*sum));
	sum->l4_layer = 0xFF;
	int cap = opts->max_layers ? opts->max_layers : PCPPX_MAX_LAYERS;
	uint16_t flags = 0;
	if (caplen > PCPPX_MAX_CAPLEN) { sum->flags = PCPPX_F_OVERSIZE; if (tup) tup->flags = PCPPX_F_OVERSIZE; return; }
	if (caplen == 0) return; /* createFirstLayer returns nullptr, Packet.cpp:829-831 */

	/* first layer: Packet::createFirstLayer, Packet++/src/Packet.cpp:827-923 */
	int k;
	switch (linktype) {
	case 1: /* LINKTYPE_ETHERNET */
		k = eth_valid(pkt, caplen) ? K_ETH : dot3_valid(pkt, caplen) ? K_DOT3 : K_PAYLOAD;
		break;
	case 101: case 12: case 14: /* LINKTYPE_RAW, DLT_RAW1, DLT_RAW2 */
		k = ((pkt[0] & 0xF0) == 0x40 && ipv4_valid(pkt, caplen)) ? K_IPV4
		    : ((pkt[0] & 0xF0) == 0x60 && ipv6_valid(pkt, caplen)) ? K_IPV6 : K_PAYLOAD;
		break;
	case 228: k = ipv4_valid(pkt, caplen) ? K_IPV4 : K_PAYLOAD; break; /* LINKTYPE_IPV4 */
	case 229: k = ipv6_valid(pkt, caplen) ? K_IPV6 : K_PAYLOAD; break; /* LINKTYPE_IPV6 */
	case 113: k = K_SLL; break;                                   /* LINKTYPE_LINUX_SLL: unchecked */
	case 276: k = caplen >= 20 ? K_SLL2 : K_PAYLOAD; break;        /* Sll2Layer::isDataValid, Sll2Layer.cpp:151-154 */
	case 0: k = caplen >= 4 ? K_NULL : K_PAYLOAD; break;           /* NullLoopbackLayer::isDataValid, NullLoopbackLayer.h:86-89 */
	case 239: k = caplen >= 4 ? K_NFLOG : K_PAYLOAD; break; /* NflogLayer::isDataValid, NflogLayer.cpp:102-105 */
	case 104: k = caplen >= 4 ? K_HDLC : K_PAYLOAD; break;  /* CiscoHdlcLayer::isDataValid, CiscoHdlcLayer.h:59-62 */
	default: k = K_PAYLOAD; break;
	}

	/* chain walk with the stop rules of Packet::parsePacket, Packet++/src/Packet.cpp:123-175 */
	lay chain_first_ipv4 = { 0 }, chain_first_ipv6 = { 0 };
	int have_ipv4 = 0, have_ipv6 = 0, l4_idx = -1, l4_is_tcp = 0, last_udp = -1, last_tcp = -1;
	lay last_tcp_l = { 0 }, last_udp_l = { 0 }, prev_of_tcp = { 0 }, prev_of_udp = { 0 };
	lay prev = { 0 }, last = { 0 };
	int count = 0, found = 0, stopped_by_rule = 0;
	uint64_t mask = 0;
	uint32_t off = 0, len = caplen;
	uint8_t kosi = 7; /* smallest candidate OSI layer of k when k is K_OUT / K_L7 */
	uint16_t kcls = 0; /* k == K_L7: the flags it brings */
	const int fam_engine_only = family_engine_only(opts->parse_until_family);
	while (k != K_NONE) {
		if (k == K_OUT || k == K_L7) {
			/* a classified HTTP / SSL / DNS layer: the engine builds it and the layers behind it, each under the
			 * stop rules */
			if (k == K_L7 && (kcls & (PCPPX_F_L7_HTTP | PCPPX_F_L7_SSL | PCPPX_F_L7_DNS | L7_MYSQL | L7_SSH))) {
				const lay l4l = last;
				count = l7_layers(pkt, off, len, kcls, &l4l, opts, &found, &stopped_by_rule, layers, cap, count,
				                  &mask, &last);
				break;
			}
			/* the host would build this layer, then the stop rules would roll it back (see above) */
			if (count > 0 && (kosi > opts->parse_until_osi || (found && fam_engine_only))) {
				stopped_by_rule = 1;
				break;
			}
			flags |= k == K_OUT ? PCPPX_F_NEEDS_HOST_PROTO : kcls;
			break;
		}
		int nk; uint32_t noff = 0, nlen = 0;
		uint8_t nosi = 7;
		uint16_t ncls = 0;
		lay L = make_layer(pkt, k, off, len, &nk, &noff, &nlen, &nosi, &ncls);
		int member = family_member(opts->parse_until_family, L.proto);
		int fail = L.osi > opts->parse_until_osi;
		if (!fail) {
			if (opts->parse_until_family != 0 && member) found = 1;
			if (found && !member) fail = 1;
		}
		if (fail) {
			stopped_by_rule = 1;
			if (count > 0) break; /* roll back the layer (Packet.cpp:170-175) */
			nk = K_NONE;          /* the first layer is kept, but not parsed further */
		}
		/* record */
		if (layers && count < cap) {
			pcppx_layer* o = &layers[count];
			o->proto = L.proto; o->osi = L.osi;
			o->offset = (uint16_t)L.off; o->hdr_len = (uint16_t)L.hdr; o->data_len = (uint16_t)L.dlen;
		}
		mask |= (uint64_t)1 << L.proto;
		if (L.proto == P_IPV4 && !have_ipv4) { have_ipv4 = 1; chain_first_ipv4 = L; }
		if (L.proto == P_IPV6 && !have_ipv6) { have_ipv6 = 1; chain_first_ipv6 = L; }
		if (L.proto == P_TCP) { last_tcp = count; last_tcp_l = L; prev_of_tcp = prev; }
		if (L.proto == P_UDP) { last_udp = count; last_udp_l = L; prev_of_udp = prev; }
		prev = L;
		last = L;
		++count;
		k = nk; off = noff; len = nlen; kosi = nosi; kcls = ncls;
	}
	/* trailer: Packet.cpp:178-195 (only with no parse-until options, and not for flagged chains) */
	if (count > 0 && opts->parse_until_family == 0 && opts->parse_until_osi == 8 && !stopped_by_rule &&
	    !(flags & (PCPPX_F_NEEDS_HOST_L7 | PCPPX_F_NEEDS_HOST_PROTO))) {
		int64_t tl = (int64_t)caplen - ((int64_t)last.off + last.dlen);
		if (tl > 0) {
			if (layers && count < cap) {
				pcppx_layer* o = &layers[count];
				o->proto = P_TRAILER; o->osi = 2;
				o->offset = (uint16_t)(last.off + last.dlen); o->hdr_len = (uint16_t)tl; o->data_len = (uint16_t)tl;
			}
			mask |= (uint64_t)1 << P_TRAILER;
			++count;
			flags |= PCPPX_F_TRAILER;
		}
	}
	if (count > cap) flags |= PCPPX_F_DEPTH_OVERFLOW;
	sum->n_layers = (uint8_t)(count > cap ? cap : count);
	sum->proto_mask = mask;

	/* l4 layer: getLayerOfType<TcpLayer>(true) else <UdpLayer>(true), PacketUtils.cpp:157-169 */
	lay l4 = { 0 }, l4prev = { 0 };
	if (last_tcp >= 0) { l4_idx = last_tcp; l4_is_tcp = 1; l4 = last_tcp_l; l4prev = prev_of_tcp; }
	else if (last_udp >= 0) { l4_idx = last_udp; l4 = last_udp_l; l4prev = prev_of_udp; }
	if (l4_idx >= 0 && l4_idx < 255) sum->l4_layer = (uint8_t)l4_idx;

	/* hash5Tuple, PacketUtils.cpp:139-210 (ICMP never appears in an emitted chain: it is OUT) */
	int has_ip = have_ipv4 || have_ipv6;
	for (int dir = 0; dir < 2; ++dir) {
		uint32_t h = 0;
		if (has_ip && l4_idx >= 0 && !(mask & ((uint64_t)1 << P_ICMP))) { /* ICMP: 0, PacketUtils.cpp:144-145 */
			const uint8_t* lp = pkt + l4.off;
			uint16_t sp = le16(lp), dp = le16(lp + 2); /* raw network-order values */
			int s = 0;
			if (!dir && dp < sp) s = 1;
			const uint8_t* ports[2];
			ports[0 + s] = lp; ports[1 - s] = lp + 2;
			h = 2166136261u;
			h = fnv_update(h, ports[0], 2);
			h = fnv_update(h, ports[1], 2);
			if (have_ipv4) {
				const uint8_t* ip = pkt + chain_first_ipv4.off;
				if (!dir && sp == dp && le32(ip + 16) < le32(ip + 12)) s = 1;
				const uint8_t* a[2];
				a[0 + s] = ip + 12; a[1 - s] = ip + 16;
				h = fnv_update(h, a[0], 4);
				h = fnv_update(h, a[1], 4);
				h = fnv_update(h, ip + 9, 1);
			} else {
				const uint8_t* ip = pkt + chain_first_ipv6.off;
				if (!dir && sp == dp && memcmp(ip + 24, ip + 8, 16) < 0) s = 1;
				const uint8_t* a[2];
				a[0 + s] = ip + 8; a[1 - s] = ip + 24;
				h = fnv_update(h, a[0], 16);
				h = fnv_update(h, a[1], 16);
				h = fnv_update(h, ip + 6, 1);
			}
		}
		if (dir) sum->hash5_dir = h; else sum->hash5 = h;
	}
	/* hash2Tuple, PacketUtils.cpp:212-245 */
	if (have_ipv4) {
		const uint8_t* ip = pkt + chain_first_ipv4.off;
		int s = le32(ip + 16) < le32(ip + 12);
		const uint8_t* a[2];
		a[0 + s] = ip + 12; a[1 - s] = ip + 16;
		uint32_t h = fnv_update(2166136261u, a[0], 4);
		sum->hash2 = fnv_update(h, a[1], 4);
	} else if (have_ipv6) {
		const uint8_t* ip = pkt + chain_first_ipv6.off;
		int s = memcmp(ip + 24, ip + 8, 16) < 0;
		const uint8_t* a[2];
		a[0 + s] = ip + 8; a[1 - s] = ip + 24;
		uint32_t h = fnv_update(2166136261u, a[0], 16);
		sum->hash2 = fnv_update(h, a[1], 16);
	}

	if (opts->want_checksums) {
		if (have_ipv4) { /* IPv4Layer::computeCalculateFields, IPv4Layer.cpp:410-412 */
			const uint8_t* ip = pkt + chain_first_ipv4.off;
			uint32_t hl = (uint32_t)(ip[0] & 0xF) * 4;
			if (hl > chain_first_ipv4.dlen) hl = chain_first_ipv4.dlen;
			uint8_t hdr[60];
			memcpy(hdr, ip, hl);
			hdr[10] = hdr[11] = 0;
			const uint8_t* b[1] = { hdr };
			uint32_t n[1] = { hl };
			sum->ip_csum_calc = pcppx_oracle_checksum(b, n, 1);
			sum->ip_csum_stored = be16(ip + 10);
			flags |= PCPPX_F_IP_CSUM;
			if (sum->ip_csum_calc == sum->ip_csum_stored) flags |= PCPPX_F_IP_CSUM_OK;
		}
		if (l4_idx >= 0) {
			/* {Tcp,Udp}Layer::calculateChecksum(false): TcpLayer.cpp:271-311, UdpLayer.cpp:47-90;
			 * computePseudoHdrChecksum PacketUtils.cpp:66-112 */
			const uint8_t* lp = pkt + l4.off;
			uint32_t field = l4_is_tcp ? 16 : 6;
			uint16_t res = 0;
			if (l4prev.proto == P_IPV4 || l4prev.proto == P_IPV6) {
				uint8_t* tmp = (uint8_t*)malloc(l4.dlen ? l4.dlen : 1);
				memcpy(tmp, lp, l4.dlen);
				tmp[field] = tmp[field + 1] = 0;
				uint8_t proto = l4_is_tcp ? 6 : 17;
				uint16_t ph[18];
				uint32_t phlen;
				const uint8_t* ip = pkt + l4prev.off;
				if (l4prev.proto == P_IPV4) {
					uint32_t src = le32(ip + 12), dst = le32(ip + 16);
					ph[0] = (uint16_t)(src >> 16); ph[1] = (uint16_t)(src & 0xFFFF);
					ph[2] = (uint16_t)(dst >> 16); ph[3] = (uint16_t)(dst & 0xFFFF);
					ph[4] = bswap16((uint16_t)l4.dlen);
					ph[5] = bswap16(proto);
					phlen = 12;
				} else {
					memcpy(ph, ip + 8, 16);
					memcpy(ph + 8, ip + 24, 16);
					ph[16] = bswap16((uint16_t)l4.dlen);
					ph[17] = bswap16(proto);
					phlen = 36;
				}
				const uint8_t* b[2] = { tmp, (const uint8_t*)ph };
				uint32_t n[2] = { l4.dlen, phlen };
				res = pcppx_oracle_checksum(b, n, 2);
				free(tmp);
			}
			if (!l4_is_tcp && res == 0) res = 0xFFFF;
			sum->l4_csum_calc = res;
			sum->l4_csum_stored = be16(lp + field);
			flags |= PCPPX_F_L4_CSUM;
			if (sum->l4_csum_calc == sum->l4_csum_stored) flags |= PCPPX_F_L4_CSUM_OK;
		}
	}
	sum->flags = flags;
	if (tup)
		fill_tuple(pkt, sum, have_ipv4, &chain_first_ipv4, have_ipv6, &chain_first_ipv6, l4_idx, l4_is_tcp, &l4, tup);
}

/* ---- reassembly front ends, from a packet's engine-format records ---- */
static void reasm_packet(const uint8_t* pkt, const pcppx_summary* s, const pcppx_layer* lay, int ml,
                         pcppx_reasm_info* out)
{
	memset(out, 0, sizeof(*out));
	int nl = s->n_layers < ml ? s->n_layers : ml;
	int v4 = -1, v6 = -1, tcp = -1;
	for (int k = 0; k < nl; ++k) {
		if (lay[k].proto == P_IPV4 && v4 < 0) v4 = k;
		if (lay[k].proto == P_IPV6 && v6 < 0) v6 = k;
		if (lay[k].proto == P_TCP) tcp = k;
	}
	/* chain not finished on the device (include/pcppx.h): an L7 dissector behind a TCP port adds no IP/TCP
	 * layer (TcpLayer.cpp:372-491), every other unfinished case may */
	int unfinished = (s->flags & (PCPPX_F_NEEDS_HOST_PROTO | PCPPX_F_OVERSIZE | PCPPX_F_BAD_DESC |
	                              PCPPX_F_DEPTH_OVERFLOW)) != 0;
	if ((s->flags & PCPPX_F_NEEDS_HOST_L7) && !(nl > 0 && lay[nl - 1].proto == P_TCP)) unfinished = 1;

	/* IPReassembly::processPacket, Packet++/src/IPReassembly.cpp:284-322: the IPv4 wrapper when the packet
	 * has an IPv4 layer (getLayerOfType<IPv4Layer>() = the first), else the IPv6 wrapper (first IPv6) */
	uint8_t ips;
	if (v4 >= 0) {
		const pcppx_layer* L = &lay[v4];
		const uint8_t* ip = pkt + L->offset;
		uint32_t fo = ((uint32_t)(ip[6] & 0x1F) << 8) | ip[7];
		int more = (ip[6] & 0x20) != 0;
		if (!more && fo == 0) ips = PCPPX_IPR_NON_FRAGMENT;   /* IPv4Layer::isFragment, IPv4Layer.cpp:415-418 */
		else if (L->hdr_len > L->data_len) ips = PCPPX_IPR_MALFORMED; /* size_t getLayerPayloadSize wraps */
		else {
			ips = PCPPX_IPR_FRAGMENT;
			out->frag_id = be16(ip + 4);                      /* IPReassembly.cpp:98-101 */
			out->frag_offset = (uint16_t)(fo * 8);            /* IPv4Layer::getFragmentOffset :435-438 */
			if (fo == 0) ips |= PCPPX_IPR_F_FIRST;            /* isFirstFragment :420-423 */
			if (!more) ips |= PCPPX_IPR_F_LAST;               /* isLastFragment :425-428 */
			uint32_t h = fnv_update(2166136261u, ip + 12, 4); /* hashPacket :103-115: src, dst, raw ipId */
			h = fnv_update(h, ip + 16, 4);
			out->ip_key = fnv_update(h, ip + 4, 2);
		}
	} else if (unfinished) {
		ips = PCPPX_IPR_HOST;
	} else if (v6 >= 0) {
		const pcppx_layer* L = &lay[v6];
		const uint8_t* ip = pkt + L->offset;
		/* getExtensionOfType<IPv6FragmentationHeader>() (IPv6Layer.h:203-210) over the extension list
		 * parseExtensions built (IPv6Layer.cpp:79-147): replay that walk up to the recorded header length */
		uint32_t nh = ip[6], eo = 40, fe = 0;
		int have_frag = 0;
		while (eo < L->hdr_len) {
			if (nh == 44 && !have_frag) { have_frag = 1; fe = eo; }
			uint32_t el = nh == 51 ? 4u * ((uint32_t)ip[eo + 1] + 2) : 8u * ((uint32_t)ip[eo + 1] + 1);
			nh = ip[eo];
			eo += el;
		}
		ips = PCPPX_IPR_F_IPV6;
		if (!have_frag) ips |= PCPPX_IPR_NON_FRAGMENT;         /* IPReassembly.cpp:156-159 */
		else if (L->hdr_len > L->data_len) ips |= PCPPX_IPR_MALFORMED;
		else {
			/* ip6_frag fields (IPv6Extensions.h): nextHeader, reserved, fragOffsetAndFlags, id; inside the
			 * header [0, hdr_len), which hdr_len <= data_len keeps inside the packet */
			const uint8_t* f = ip + fe;
			uint32_t off = ((uint32_t)f[2] << 8) | (f[3] & 0xF8); /* getFragmentOffset IPv6Extensions.cpp:87-91 */
			ips |= PCPPX_IPR_FRAGMENT;
			out->frag_id = ((uint32_t)f[4] << 24) | ((uint32_t)f[5] << 16) | ((uint32_t)f[6] << 8) | f[7];
			out->frag_offset = (uint16_t)off;
			if (off == 0) ips |= PCPPX_IPR_F_FIRST;              /* isFirstFragment :71-74 */
			if (!(f[3] & 1)) ips |= PCPPX_IPR_F_LAST;            /* isLastFragment / isMoreFragments :76-85 */
			uint32_t h = fnv_update(2166136261u, ip + 8, 16);    /* hashPacket IPReassembly.cpp:190-205 */
			h = fnv_update(h, ip + 24, 16);
			out->ip_key = fnv_update(h, f + 4, 4);
		}
	} else {
		ips = PCPPX_IPR_NON_IP;
	}
	out->ip_status = ips;

	/* TcpReassembly::reassemblePacket, Packet++/src/TcpReassembly.cpp:96-136 */
	uint8_t ts;
	if (unfinished) ts = PCPPX_TCPR_HOST;
	else if (v4 < 0 && v6 < 0) ts = PCPPX_TCPR_NON_IP;   /* isPacketOfType(IP) :96-103 */
	else if (tcp < 0) ts = PCPPX_TCPR_NON_TCP;           /* getLayerOfType<TcpLayer>(true) :106-110 (ICMP never
	                                                        sits in a finished chain: it is out of scope) */
	else {
		const pcppx_layer* L = &lay[tcp];
		uint8_t fl = pkt[L->offset + 13];                /* tcphdr bitfields, TcpLayer.h:30-52 */
		uint32_t pay = (uint32_t)L->data_len - L->hdr_len;
		int fin = fl & 1, syn = (fl >> 1) & 1, rst = (fl >> 2) & 1;
		ts = (pay == 0 && !syn && !fin && !rst) ? PCPPX_TCPR_NO_DATA : PCPPX_TCPR_DATA; /* :124-136 */
		ts |= (fin ? PCPPX_TCPR_F_FIN : 0) | (syn ? PCPPX_TCPR_F_SYN : 0) | (rst ? PCPPX_TCPR_F_RST : 0);
		out->tcp_payload = pay;
	}
	out->tcp_status = ts;
}

int pcppx_oracle_reasm_batch(const pcppx_batch* b, const pcppx_records* r, uint8_t max_layers, pcppx_reasm_info* info)
{
	if (!b || !r || !r->summary || !r->layers || !info || max_layers == 0 || max_layers > PCPPX_MAX_LAYERS)
		return PCPPX_E_INVAL;
	for (uint32_t i = 0; i < b->n; ++i) {
		const pcppx_summary* s = &r->summary[i];
		const uint8_t* pkt = (s->flags & PCPPX_F_BAD_DESC) ? b->data : b->data + b->offsets[i];
		reasm_packet(pkt, s, r->layers + (size_t)i * max_layers, max_layers, &info[i]);
	}
	return PCPPX_OK;
}

/* ---- batch drivers ---- */
typedef struct {
	const pcppx_batch* b;
	const pcppx_opts* o;
	pcppx_records* r;
	int t, nt;
	uint64_t acc;
} job;

static void* run_job(void* arg)
{
	job* j = (job*)arg;
	uint64_t acc = 0;
	int ml = j->o->max_layers;
	for (uint32_t i = (uint32_t)j->t; i < j->b->n; i += (uint32_t)j->nt) {
		pcppx_summary s;
		pcppx_summary* sp = j->r ? &j->r->summary[i] : &s;
		pcppx_layer scratch[PCPPX_MAX_LAYERS];
		pcppx_layer* lp = (j->r && j->r->layers && ml) ? j->r->layers + (size_t)i * ml : (ml ? scratch : NULL);
		pcppx_tuple* tp = (j->r && j->r->tuples) ? &j->r->tuples[i] : NULL;
		if (j->b->offsets[i] + j->b->caplens[i] > j->b->data_len) {
			memset(sp, 0, sizeof(*sp));
			sp->l4_layer = 0xFF;
			sp->flags = PCPPX_F_BAD_DESC;
			if (tp) { memset(tp, 0, sizeof(*tp)); tp->flags = PCPPX_F_BAD_DESC; }
			continue;
		}
		parse_packet(j->b->data + j->b->offsets[i], j->b->caplens[i], j->b->linktype, j->o, sp, lp, tp);
		acc += sp->hash5 + sp->hash5_dir + sp->hash2 + sp->l4_csum_calc + sp->ip_csum_calc + sp->n_layers;
	}
	j->acc = acc;
	return NULL;
}

static int run_all(const pcppx_batch* b, const pcppx_opts* o, pcppx_records* r, int threads, uint64_t* digest)
{
	if (threads < 1) threads = 1;
	if (threads > 256) threads = 256;
	job jobs[256];
	pthread_t th[256];
	for (int t = 0; t < threads; ++t) {
		jobs[t].b = b; jobs[t].o = o; jobs[t].r = r; jobs[t].t = t; jobs[t].nt = threads; jobs[t].acc = 0;
	}
	if (threads == 1) run_job(&jobs[0]);
	else {
		for (int t = 0; t < threads; ++t) pthread_create(&th[t], NULL, run_job, &jobs[t]);
		for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
	}
	if (digest) {
		uint64_t d = 0;
		for (int t = 0; t < threads; ++t) d += jobs[t].acc;
		*digest = d;
	}
	return PCPPX_OK;
}

int pcppx_oracle_parse_batch(const pcppx_batch* b, const pcppx_opts* o, pcppx_records* r, int threads)
{
	if (!b || !o || !r || !r->summary || o->max_layers > PCPPX_MAX_LAYERS) return PCPPX_E_INVAL;
	return run_all(b, o, r, threads, NULL);
}

int pcppx_oracle_bench(const pcppx_batch* b, const pcppx_opts* o, int threads, double* seconds, uint64_t* digest)
{
	if (!b || !o || !seconds || o->max_layers > PCPPX_MAX_LAYERS) return PCPPX_E_INVAL;
	struct timespec t0, t1;
	clock_gettime(CLOCK_MONOTONIC, &t0);
	run_all(b, o, NULL, threads, digest);
	clock_gettime(CLOCK_MONOTONIC, &t1);
	*seconds = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
	return PCPPX_OK;
}
