/* pcppx.hpp — the Packet++-shaped C++ facade over the engine's C ABI (pcppx.h). Header-only, no HIP types, no
 * Packet++ dependency.
 *
 * A reference caller writes, per packet (Examples/PcapPlusPlus-benchmark/benchmark.cpp:89-95,
 * Examples/DpdkExample-FilterTraffic/AppWorkerThread.h:85-139):
 *
 *   pcpp::RawPacket rawPacket;
 *   while (reader.getNextPacket(rawPacket)) {
 *       pcpp::Packet packet(&rawPacket, pcpp::TCP);              // Packet++/src/Packet.cpp:202-209
 *       if (packet.isPacketOfType(pcpp::TCP)) flows[pcpp::hash5Tuple(&packet)]++;
 *   }
 *
 * With the engine the only change is a batch prepass: the reader fills a RawPacketVector, one call parses the
 * whole batch on the GPU, and the per-packet loop runs unchanged over pcppx::Packet views with the same names
 * (isPacketOfType, getLayerOfType<IPv4Layer/TcpLayer/UdpLayer>, getFirstLayer, hash5Tuple(&packet), ...):
 *
 *   pcppx::Engine engine(0);
 *   engine.setHostParser(myPacketPlusPlusParse);                  // optional, see below
 *   pcppx::RawPacketVector batch;
 *   while (reader.getNextPackets(batch, 1 << 20) > 0) {
 *       pcppx::ParsedBatch parsed = engine.parse(batch, pcppx::PacketParseOptions(pcppx::TCP));
 *       for (pcppx::Packet packet : parsed)
 *           if (packet.isPacketOfType(pcppx::TCP)) flows[pcppx::hash5Tuple(&packet)]++;
 *   }
 *
 * Packets the engine leaves to the host (PCPPX_F_NEEDS_HOST: an L7 dissector, an out-of-scope L2/L3 layer) carry
 * an exact layer prefix. A caller that registers a host parser (pcppx_host_parse_fn: its own Packet++ parse of one
 * packet) gets them completed inside Engine::parse, so every Packet view answers as
 * pcpp::Packet would; without one, needsHost() reports them. libpcppx.so never links Packet++.
 *
 * Errors are reported as pcppx::Error (a std::runtime_error carrying the PCPPX_E_* code).
 */
#ifndef PCPPX_HPP
#define PCPPX_HPP

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <utility>
#include <vector>

#include "pcppx.h"

namespace pcppx
{
/* ProtocolType / ProtocolTypeFamily / OsiModelLayer values of Packet++/header/ProtocolType.h:42-284 */
using ProtocolType = uint8_t;
using ProtocolTypeFamily = uint32_t;
constexpr ProtocolType UnknownProtocol = 0, Ethernet = 1, IPv4 = 2, IPv6 = 3, TCP = 4, UDP = 5, HTTPRequest = 6,
                       HTTPResponse = 7, ARP = 8, VLAN = 9, ICMP = 10, DNS = 13, MPLS = 14, GREv0 = 15, GREv1 = 16,
                       PPP_PPTP = 17, SSL = 18, GenericPayload = 25, PacketTrailer = 30, EthernetDot3 = 33, LLC = 44;
constexpr ProtocolTypeFamily IP = 0x203, GRE = 0xf10, HTTP = 0x607;
enum OsiModelLayer : uint8_t
{
	OsiModelPhysicalLayer = 1,
	OsiModelDataLinkLayer = 2,
	OsiModelNetworkLayer = 3,
	OsiModelTransportLayer = 4,
	OsiModelSesionLayer = 5,
	OsiModelPresentationLayer = 6,
	OsiModelApplicationLayer = 7,
	OsiModelLayerUnknown = 8
};

/* facade-level summary flag: the records were filled by the caller's host parser (Engine::setHostParser) */
constexpr uint16_t F_HOST_PARSED = 0x4000;

class Error : public std::runtime_error
{
public:
	Error(int code, const std::string& what) : std::runtime_error(what + ": " + pcppx_strerror(code)), m_Code(code) {}
	int code() const { return m_Code; }

private:
	int m_Code;
};

inline void check(int rc, const char* what)
{
	if (rc != PCPPX_OK)
		throw Error(rc, what);
}

/* pcpp::IPv4Address (Common++/header/IpAddress.h:37-40): the four bytes in memory order */
class IPv4Address
{
public:
	IPv4Address() = default;
	explicit IPv4Address(uint32_t addrAsInt) : m_Int(addrAsInt) {}
	explicit IPv4Address(const std::string& dotted)
	{
		unsigned v[4];
		char tail;
		if (std::sscanf(dotted.c_str(), "%u.%u.%u.%u%c", &v[0], &v[1], &v[2], &v[3], &tail) != 4 || v[0] > 255 ||
		    v[1] > 255 || v[2] > 255 || v[3] > 255)
			throw Error(PCPPX_E_INVAL, "bad IPv4 address '" + dotted + "'");
		const uint8_t b[4] = { (uint8_t)v[0], (uint8_t)v[1], (uint8_t)v[2], (uint8_t)v[3] };
		std::memcpy(&m_Int, b, 4);
	}
	uint32_t toInt() const { return m_Int; }
	std::string toString() const
	{
		uint8_t b[4];
		std::memcpy(b, &m_Int, 4);
		char s[16];
		std::snprintf(s, sizeof(s), "%u.%u.%u.%u", b[0], b[1], b[2], b[3]);
		return s;
	}
	bool operator==(const IPv4Address& o) const { return m_Int == o.m_Int; }
	bool operator!=(const IPv4Address& o) const { return m_Int != o.m_Int; }
	static const IPv4Address Zero;

private:
	uint32_t m_Int = 0;
};
inline const IPv4Address IPv4Address::Zero{};

/* An allocator whose resize() leaves new elements uninitialised: batch buffers are sized for the largest batch and
 * then filled by the reader / the engine, so zero-filling them first (256 MiB of packet buffer per read) would cost
 * more than the read itself. */
template <class T>
struct DefaultInitAllocator : std::allocator<T>
{
	template <class U>
	struct rebind
	{
		using other = DefaultInitAllocator<U>;
	};
	DefaultInitAllocator() = default;
	template <class U>
	DefaultInitAllocator(const DefaultInitAllocator<U>&) noexcept
	{}
	template <class U>
	void construct(U* p) noexcept(std::is_nothrow_default_constructible<U>::value)
	{
		::new (static_cast<void*>(p)) U;
	}
	template <class U, class... A>
	void construct(U* p, A&&... a)
	{
		::new (static_cast<void*>(p)) U(std::forward<A>(a)...);
	}
};
template <class T>
using buffer = std::vector<T, DefaultInitAllocator<T>>;

/* PacketParseOptions (Packet++/header/Packet.h:17-37) plus the engine's record options */
struct PacketParseOptions
{
	ProtocolTypeFamily parseUntilProtocol = UnknownProtocol;
	OsiModelLayer parseUntilLayer = OsiModelLayerUnknown;
	bool computeChecksums = true; /* IPv4 header + TCP/UDP checksum verification */
	uint8_t maxLayers = PCPPX_MAX_LAYERS;
	bool deepWindow = false;  /* PCPPX_WINDOW_DEEP: two-round 144-B header window for checksum launches over deep stacks */
	bool shortWindow = false; /* PCPPX_WINDOW_SHORT: one 96-B round for parse-only launches over plain stacks (ignored
	                             when deepWindow is set) */

	PacketParseOptions() = default;
	PacketParseOptions(ProtocolTypeFamily until, OsiModelLayer layer = OsiModelLayerUnknown)
	    : parseUntilProtocol(until), parseUntilLayer(layer)
	{}

	pcppx_opts toC() const
	{
		pcppx_opts o;
		pcppx_default_opts(&o);
		o.parse_until_family = parseUntilProtocol;
		o.parse_until_osi = parseUntilLayer;
		o.want_checksums = computeChecksums ? 1 : 0;
		o.max_layers = maxLayers;
		o.window = deepWindow ? PCPPX_WINDOW_DEEP : (shortWindow ? PCPPX_WINDOW_SHORT : PCPPX_WINDOW_DEFAULT);
		return o;
	}
};

/* A batch of raw packets back to back in one buffer: packet i = data[offsets[i], offsets[i] + caplens[i]).
 * Plays the role of pcpp::RawPacketVector (Packet++/header/RawPacket.h) for the batch prepass. */
struct RawPacketVector
{
	buffer<uint8_t> data;
	buffer<uint64_t> offsets;
	buffer<uint32_t> caplens;
	buffer<uint64_t> timestampsNs;
	buffer<uint32_t> frameLens; /* RawPacket::getFrameLength (original wire length) */
	uint16_t linkType = 1; /* LINKTYPE_ETHERNET */

	size_t size() const { return caplens.size(); }
	void clear()
	{
		data.clear();
		offsets.clear();
		caplens.clear();
		timestampsNs.clear();
		frameLens.clear();
	}
	/* RawPacket::setRawData-style append (Packet++/header/RawPacket.h) */
	void add(const uint8_t* bytes, uint32_t len, uint64_t tsNs = 0)
	{
		offsets.push_back(data.size());
		caplens.push_back(len);
		timestampsNs.push_back(tsNs);
		frameLens.push_back(len);
		data.insert(data.end(), bytes, bytes + len);
	}
	const uint8_t* packetData(size_t i) const { return data.data() + offsets[i]; }
	pcppx_batch toC() const
	{
		return pcppx_batch{ data.data(), offsets.data(), caplens.data(), data.size(), (uint32_t)caplens.size(),
			                linkType, 0 };
	}
};
using RawBatch = RawPacketVector;

/* PcapFileReaderDevice / PcapNgFileReaderDevice (Pcap++/header/PcapFileDevice.h): open / getNextPackets / close.
 * The format (pcap or pcapng) comes from the file's first bytes; a batch holds one link type (pcapng
 * interfaces may differ), given by getLinkLayerType() after the batch is read. */
class PcapFileReaderDevice
{
public:
	explicit PcapFileReaderDevice(std::string fileName) : m_FileName(std::move(fileName)) {}
	~PcapFileReaderDevice() { close(); }
	PcapFileReaderDevice(const PcapFileReaderDevice&) = delete;
	PcapFileReaderDevice& operator=(const PcapFileReaderDevice&) = delete;

	bool open() { return m_Reader != nullptr || pcppx_pcap_open(m_FileName.c_str(), &m_Reader) == PCPPX_OK; }
	bool isOpened() const { return m_Reader != nullptr; }
	void close()
	{
		pcppx_pcap_close(m_Reader);
		m_Reader = nullptr;
	}
	uint32_t getLinkLayerType() const { return pcppx_pcap_linktype(m_Reader); }

	/* IFileReaderDevice::getNextPackets(RawPacketVector&, int numOfPacketsToRead) (PcapFileDevice.cpp:604-624):
	 * replaces `batch` with the next packets (at most numOfPacketsToRead, -1 = as many as maxBytes holds); returns
	 * the count, 0 at end of file. */
	int getNextPackets(RawPacketVector& batch, int numOfPacketsToRead = -1, uint64_t maxBytes = 256ull << 20)
	{
		if (!open())
			throw Error(PCPPX_E_INVAL, "PcapFileReaderDevice::open(" + m_FileName + ")");
		const uint32_t maxPackets = numOfPacketsToRead > 0 ? (uint32_t)numOfPacketsToRead : (uint32_t)(maxBytes / 16);
		batch.data.resize(maxBytes);
		batch.offsets.resize(maxPackets);
		batch.caplens.resize(maxPackets);
		batch.timestampsNs.resize(maxPackets);
		batch.frameLens.resize(maxPackets);
		uint32_t n = 0;
		uint64_t used = 0;
		check(pcppx_pcap_read_batch_ex(m_Reader, batch.data.data(), maxBytes, batch.offsets.data(), batch.caplens.data(),
		                               batch.frameLens.data(), batch.timestampsNs.data(), maxPackets, &n, &used),
		      "pcppx_pcap_read_batch_ex");
		batch.data.resize(used);
		batch.offsets.resize(n);
		batch.caplens.resize(n);
		batch.timestampsNs.resize(n);
		batch.frameLens.resize(n);
		batch.linkType = (uint16_t)getLinkLayerType();
		return (int)n;
	}

private:
	std::string m_FileName;
	pcppx_pcap* m_Reader = nullptr;
};
using PcapNgFileReaderDevice = PcapFileReaderDevice;
using IFileReaderDevice = PcapFileReaderDevice;

/* One layer of a parsed packet: Layer::getProtocol / getOsiModelLayer / getData / getHeaderLen / getDataLen /
 * getLayerPayloadSize / isMemberOfProtocolFamily (Packet++/header/Layer.h) */
class Layer
{
public:
	Layer() = default;
	Layer(const pcppx_layer* rec, const uint8_t* raw) : m_Rec(rec), m_Raw(raw) {}
	ProtocolType getProtocol() const { return m_Rec->proto; }
	OsiModelLayer getOsiModelLayer() const { return (OsiModelLayer)m_Rec->osi; }
	const uint8_t* getData() const { return m_Raw + m_Rec->offset; }
	size_t getHeaderLen() const { return m_Rec->hdr_len; }
	size_t getDataLen() const { return m_Rec->data_len; }
	size_t getLayerPayloadSize() const { return m_Rec->data_len - m_Rec->hdr_len; }
	const uint8_t* getLayerPayload() const { return getData() + getHeaderLen(); }
	bool isMemberOfProtocolFamily(ProtocolTypeFamily family) const
	{
		const uint32_t p = m_Rec->proto;
		return p != 0 && (p == (family & 0xFF) || (p << 8) == (family & 0xFF00) || (p << 16) == (family & 0xFF0000) ||
		                  (p << 24) == (family & 0xFF000000u));
	}
	uint16_t getOffset() const { return m_Rec->offset; }
	bool valid() const { return m_Rec != nullptr; }

protected:
	uint16_t be16(size_t j) const { return (uint16_t)((getData()[j] << 8) | getData()[j + 1]); }
	const pcppx_layer* m_Rec = nullptr;
	const uint8_t* m_Raw = nullptr;
};

/* typed views: the accessors the two reference callers use */
class IPv4Layer : public Layer /* Packet++/header/IPv4Layer.h */
{
public:
	static constexpr ProtocolType kProtocol = IPv4;
	using Layer::Layer;
	IPv4Address getSrcIPv4Address() const { return IPv4Address(rd32(12)); }
	IPv4Address getDstIPv4Address() const { return IPv4Address(rd32(16)); }
	uint8_t getProtocolField() const { return getData()[9]; }
	bool isFragment() const { return (getData()[6] & 0x20) || (((getData()[6] & 0x1F) << 8) | getData()[7]) != 0; }

private:
	uint32_t rd32(size_t j) const
	{
		uint32_t v;
		std::memcpy(&v, getData() + j, 4);
		return v;
	}
};
class IPv6Layer : public Layer /* Packet++/header/IPv6Layer.h */
{
public:
	static constexpr ProtocolType kProtocol = IPv6;
	using Layer::Layer;
	const uint8_t* getSrcIPv6AddressBytes() const { return getData() + 8; }
	const uint8_t* getDstIPv6AddressBytes() const { return getData() + 24; }
};
class TcpLayer : public Layer /* Packet++/header/TcpLayer.h: ports in host order */
{
public:
	static constexpr ProtocolType kProtocol = TCP;
	using Layer::Layer;
	uint16_t getSrcPort() const { return be16(0); }
	uint16_t getDstPort() const { return be16(2); }
	uint8_t getFlags() const { return getData()[13]; }
};
class UdpLayer : public Layer /* Packet++/header/UdpLayer.h */
{
public:
	static constexpr ProtocolType kProtocol = UDP;
	using Layer::Layer;
	uint16_t getSrcPort() const { return be16(0); }
	uint16_t getDstPort() const { return be16(2); }
};

/* what getLayerOfType<T>() returns: a layer view that tests like the reference's T* (null when absent) */
template <class T>
class LayerPtr
{
public:
	LayerPtr() = default;
	explicit LayerPtr(const T& v) : m_V(v), m_Ok(true) {}
	const T* operator->() const { return &m_V; }
	const T& operator*() const { return m_V; }
	explicit operator bool() const { return m_Ok; }
	bool operator==(std::nullptr_t) const { return !m_Ok; }
	bool operator!=(std::nullptr_t) const { return m_Ok; }

private:
	T m_V{};
	bool m_Ok = false;
};

/* A parsed packet: the pcpp::Packet (Packet++/header/Packet.h) queries of the two callers */
class Packet
{
public:
	Packet(const pcppx_summary* s, const pcppx_layer* layers, uint8_t maxLayers, const uint8_t* raw, uint32_t caplen)
	    : m_Sum(s), m_Layers(layers), m_MaxLayers(maxLayers), m_Raw(raw), m_Caplen(caplen)
	{}

	/* Packet::isPacketOfType (Packet.cpp:614-640), for a protocol or a family. On a packet the engine left to the
	 * host and no host parser completed, the answer covers its exact layer prefix plus the HTTP / SSL / DNS class
	 * of its first L7 layer when the device named it (PCPPX_F_L7_KNOWN) */
	bool isPacketOfType(ProtocolTypeFamily family) const
	{
		uint64_t mask = m_Sum->proto_mask;
		if (m_Sum->flags & PCPPX_F_L7_KNOWN)
			mask |= ((m_Sum->flags & PCPPX_F_L7_HTTP) ? (1ull << HTTPRequest) | (1ull << HTTPResponse) : 0) |
			        ((m_Sum->flags & PCPPX_F_L7_SSL) ? 1ull << SSL : 0) | ((m_Sum->flags & PCPPX_F_L7_DNS) ? 1ull << DNS : 0);
		for (int k = 0; k < 4; ++k)
		{
			const uint32_t p = (family >> (8 * k)) & 0xFF;
			if (p != 0 && p < 64 && (mask >> p) & 1)
				return true;
		}
		return false;
	}
	size_t getLayerCount() const { return m_Sum->n_layers; }
	/* records held for the first min(getLayerCount(), maxLayers) layers */
	size_t getRecordedLayerCount() const { return m_Sum->n_layers < m_MaxLayers ? m_Sum->n_layers : m_MaxLayers; }
	Layer getLayer(size_t k) const { return Layer(m_Layers + k, m_Raw); }
	Layer getFirstLayer() const { return getRecordedLayerCount() ? getLayer(0) : Layer(); }
	Layer getLastLayer() const { return getRecordedLayerCount() ? getLayer(getRecordedLayerCount() - 1) : Layer(); }
	/* getLayerOfType<T>(reverse) (Packet.h:388-431): the first (or, reverse, the last) recorded layer of T */
	template <class T>
	LayerPtr<T> getLayerOfType(bool reverseOrder = false) const
	{
		const size_t n = getRecordedLayerCount();
		for (size_t j = 0; j < n; ++j)
		{
			const size_t k = reverseOrder ? n - 1 - j : j;
			if (m_Layers[k].proto == T::kProtocol)
				return LayerPtr<T>(T(m_Layers + k, m_Raw));
		}
		return LayerPtr<T>();
	}

	/* the raw packet (RawPacket::getRawData / getRawDataLen) */
	const uint8_t* getRawData() const { return m_Raw; }
	uint32_t getRawDataLen() const { return m_Caplen; }

	/* engine flags: the host must finish the packet (an L7 or an out-of-scope L2/L3 layer) and no host parser did */
	bool needsHost() const { return (m_Sum->flags & PCPPX_F_NEEDS_HOST) != 0; }
	/* the records come from the caller's host parser (Engine::setHostParser) */
	bool wasHostParsed() const { return (m_Sum->flags & F_HOST_PARSED) != 0; }
	bool hasTrailer() const { return (m_Sum->flags & PCPPX_F_TRAILER) != 0; }
	/* IPv4Layer::computeCalculateFields checksum vs the stored one (IPv4Layer.cpp:410-412) */
	bool hasIPv4Checksum() const { return (m_Sum->flags & PCPPX_F_IP_CSUM) != 0; }
	bool isIPv4ChecksumValid() const { return (m_Sum->flags & PCPPX_F_IP_CSUM_OK) != 0; }
	/* TcpLayer/UdpLayer::calculateChecksum(false) vs the stored checksum (TcpLayer.cpp:271, UdpLayer.cpp:47) */
	bool hasL4Checksum() const { return (m_Sum->flags & PCPPX_F_L4_CSUM) != 0; }
	bool isL4ChecksumValid() const { return (m_Sum->flags & PCPPX_F_L4_CSUM_OK) != 0; }
	uint16_t calculatedL4Checksum() const { return m_Sum->l4_csum_calc; }
	uint16_t calculatedIPv4Checksum() const { return m_Sum->ip_csum_calc; }
	const pcppx_summary& summary() const { return *m_Sum; }

private:
	const pcppx_summary* m_Sum;
	const pcppx_layer* m_Layers;
	uint8_t m_MaxLayers;
	const uint8_t* m_Raw;
	uint32_t m_Caplen;
};
using ParsedPacket = Packet;
using ParsedLayer = Layer;

/* pcpp::hash5Tuple / hash2Tuple (Packet++/header/PacketUtils.h:58-91) */
inline uint32_t hash5Tuple(const Packet* packet, bool const& directionUnique = false)
{
	return directionUnique ? packet->summary().hash5_dir : packet->summary().hash5;
}
inline uint32_t hash2Tuple(const Packet* packet)
{
	return packet->summary().hash2;
}

/* Records of one parsed batch (owns them); indexes into the RawPacketVector it was parsed from. */
class ParsedBatch
{
public:
	ParsedBatch(const RawPacketVector& raw, uint8_t maxLayers)
	    : m_Raw(&raw), m_MaxLayers(maxLayers), summaries(raw.size()), layers(raw.size() * (size_t)maxLayers)
	{}
	size_t size() const { return summaries.size(); }
	Packet operator[](size_t i) const
	{
		return Packet(&summaries[i], layers.data() + i * m_MaxLayers, m_MaxLayers, m_Raw->packetData(i),
		              m_Raw->caplens[i]);
	}
	class iterator
	{
	public:
		iterator(const ParsedBatch* b, size_t i) : m_B(b), m_I(i) {}
		Packet operator*() const { return (*m_B)[m_I]; }
		iterator& operator++()
		{
			++m_I;
			return *this;
		}
		bool operator!=(const iterator& o) const { return m_I != o.m_I; }

	private:
		const ParsedBatch* m_B;
		size_t m_I;
	};
	iterator begin() const { return iterator(this, 0); }
	iterator end() const { return iterator(this, size()); }
	uint8_t maxLayers() const { return m_MaxLayers; }
	/* packets whose records the host parser filled */
	size_t hostParsed = 0;

private:
	const RawPacketVector* m_Raw;
	uint8_t m_MaxLayers;

public:
	buffer<pcppx_summary> summaries; /* filled by the engine (or the host parser) for every packet */
	buffer<pcppx_layer> layers;       /* entries past a packet's chain are unspecified, as in pcppx.h */
};

/* PCPPX_LAYOUT_PACKED entries (include/pcppx.h) -> the FIXED layout: packet i's chain starts at its tile's base
 * 64 * t * maxLayers plus the chains of the packets before it in the tile (summary n_layers, capped at maxLayers).
 * fixed: n * maxLayers entries; entries past a chain are zeroed. */
inline void unpackLayers(const pcppx_summary* summary, const pcppx_layer* packed, size_t n, uint32_t maxLayers,
                         pcppx_layer* fixed)
{
	size_t pos = 0;
	for (size_t i = 0; i < n; ++i)
	{
		if (i % 64 == 0)
			pos = i * maxLayers;
		const uint32_t cnt = summary[i].n_layers < maxLayers ? summary[i].n_layers : maxLayers;
		for (uint32_t k = 0; k < maxLayers; ++k)
			fixed[i * maxLayers + k] = k < cnt ? packed[pos + k] : pcppx_layer{};
		pos += cnt;
	}
}

/* PacketMatchingEngine's criteria (Examples/DpdkExample-FilterTraffic/PacketMatchingEngine.h:28-41) */
struct MatchSpec
{
	pcppx_match_spec spec{};
	MatchSpec() = default;
	/* addresses as dotted quads ("" = any); ports host order (0 = any); protocol TCP / UDP (else any) */
	MatchSpec(const std::string& srcIp, const std::string& dstIp, uint16_t srcPort, uint16_t dstPort,
	          ProtocolType protocol)
	{
		spec.src_ip = srcIp.empty() ? 0 : IPv4Address(srcIp).toInt();
		spec.dst_ip = dstIp.empty() ? 0 : IPv4Address(dstIp).toInt();
		spec.src_port = srcPort;
		spec.dst_port = dstPort;
		spec.protocol = protocol;
	}
};

/* One GPU worker: a pcppx context. */
class Engine
{
public:
	explicit Engine(int device = 0) { check(pcppx_open(device, &m_Ctx), "pcppx_open"); }
	~Engine() { pcppx_close(m_Ctx); }
	Engine(const Engine&) = delete;
	Engine& operator=(const Engine&) = delete;

	/* the caller's own Packet++ parse of one packet, used to complete packets the engine flags NEEDS_HOST */
	void setHostParser(pcppx_host_parse_fn fn) { m_HostParser = fn; }

	/* Packet(&rawPacket, options) for every packet of the batch, host to host through HBM; flagged packets are
	 * completed by the host parser when one is set */
	ParsedBatch parse(const RawPacketVector& batch, const PacketParseOptions& options = PacketParseOptions()) const
	{
		ParsedBatch out(batch, options.maxLayers);
		parseInto(batch, options, out);
		return out;
	}
	void parseInto(const RawPacketVector& batch, const PacketParseOptions& options, ParsedBatch& out) const
	{
		const pcppx_batch b = batch.toC();
		const pcppx_opts o = options.toC();
		pcppx_records r{ out.summaries.data(), options.maxLayers ? out.layers.data() : nullptr, nullptr, nullptr, nullptr };
		check(pcppx_parse_batch_host(m_Ctx, &b, &o, &r), "pcppx_parse_batch_host");
		out.hostParsed = 0;
		if (m_HostParser == nullptr || options.maxLayers == 0)
			return;
		for (size_t i = 0; i < batch.size(); ++i)
		{
			pcppx_summary& s = out.summaries[i];
			if (!(s.flags & PCPPX_F_NEEDS_HOST) || (s.flags & PCPPX_F_BAD_DESC))
				continue;
			pcppx_layer* lay = out.layers.data() + i * (size_t)options.maxLayers;
			check(m_HostParser(batch.packetData(i), batch.caplens[i], batch.linkType, &o, &s, lay), "host parser");
			s.flags = (uint16_t)(s.flags | F_HOST_PARSED);
			++out.hostParsed;
		}
	}

	/* FilterTraffic's whole worker on the device (AppWorkerThread.h:85-139): matched[i] = 1 for packets to send on;
	 * the flow table persists across calls until resetFilter() */
	pcppx_packet_stats filter(const RawPacketVector& batch, const MatchSpec& spec, std::vector<uint8_t>& matched)
	{
		matched.assign(batch.size(), 0);
		const pcppx_batch b = batch.toC();
		pcppx_packet_stats st;
		check(pcppx_filter_batch_host(m_Ctx, &b, &spec.spec, matched.data(), &st), "pcppx_filter_batch_host");
		return st;
	}
	void resetFilter(uint32_t flowTableSlots = 0) { check(pcppx_filter_reset(m_Ctx, flowTableSlots), "pcppx_filter_reset"); }

	pcppx_ctx* handle() const { return m_Ctx; }

private:
	pcppx_ctx* m_Ctx = nullptr;
	pcppx_host_parse_fn m_HostParser = nullptr;
};

}  // namespace pcppx

#endif /* PCPPX_HPP */
