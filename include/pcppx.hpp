/* pcppx.hpp — a Packet++-shaped C++ view over the engine's C ABI (pcppx.h). Header-only, no HIP types.
 *
 * Callers of the reference write `pcpp::Packet packet(&rawPacket, parseUntil); packet.isPacketOfType(TCP);
 * pcpp::hash5Tuple(&packet)` per packet (Packet++/header/Packet.h:17-37, :107-116, :271-282;
 * Packet++/header/PacketUtils.h:80-91). Here a whole batch is parsed by one call and each packet is a
 * ParsedPacket view with the same names over the batch's records:
 *
 *   pcppx::PcapFileReaderDevice reader("in.pcap");           // Pcap++/header/PcapFileDevice.h
 *   pcppx::RawBatch batch;
 *   pcppx::Engine engine(0);                                 // one GPU = one worker
 *   while (reader.getNextPackets(batch, 1 << 20) > 0) {
 *       pcppx::ParsedBatch parsed = engine.parse(batch, pcppx::PacketParseOptions{pcppx::TCP});
 *       for (size_t i = 0; i < parsed.size(); ++i) {
 *           pcppx::ParsedPacket p = parsed[i];
 *           if (p.isPacketOfType(pcppx::TCP)) flows[p.hash5Tuple()]++;
 *       }
 *   }
 *
 * Errors are reported as pcppx::Error (a std::runtime_error carrying the PCPPX_E_* code).
 */
#ifndef PCPPX_HPP
#define PCPPX_HPP

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "pcppx.h"

namespace pcppx
{
/* ProtocolType / ProtocolTypeFamily / OsiModelLayer values of Packet++/header/ProtocolType.h */
using ProtocolType = uint8_t;
using ProtocolTypeFamily = uint32_t;
constexpr ProtocolType UnknownProtocol = 0, Ethernet = 1, IPv4 = 2, IPv6 = 3, TCP = 4, UDP = 5, ARP = 8, VLAN = 9,
                       MPLS = 14, GREv0 = 15, GREv1 = 16, PPP_PPTP = 17, GenericPayload = 25, PacketTrailer = 30,
                       EthernetDot3 = 33, LLC = 44;
constexpr ProtocolTypeFamily IP = 0x203, GRE = 0xf10;
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

/* PacketParseOptions (Packet++/header/Packet.h:17-37) plus the engine's record options */
struct PacketParseOptions
{
	ProtocolTypeFamily parseUntilProtocol = UnknownProtocol;
	OsiModelLayer parseUntilLayer = OsiModelLayerUnknown;
	bool computeChecksums = true; /* IPv4 header + TCP/UDP checksum verification */
	uint8_t maxLayers = PCPPX_MAX_LAYERS;

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
		return o;
	}
};

/* Packets back to back in one buffer: packet i = data[offsets[i], offsets[i] + caplens[i]). */
struct RawBatch
{
	std::vector<uint8_t> data;
	std::vector<uint64_t> offsets;
	std::vector<uint32_t> caplens;
	std::vector<uint64_t> timestampsNs;
	uint16_t linkType = 1; /* LINKTYPE_ETHERNET */

	size_t size() const { return caplens.size(); }
	void clear()
	{
		data.clear();
		offsets.clear();
		caplens.clear();
		timestampsNs.clear();
	}
	/* RawPacket-style append (RawPacket::setRawData, Packet++/header/RawPacket.h) */
	void add(const uint8_t* bytes, uint32_t len, uint64_t tsNs = 0)
	{
		offsets.push_back(data.size());
		caplens.push_back(len);
		timestampsNs.push_back(tsNs);
		data.insert(data.end(), bytes, bytes + len);
	}
	const uint8_t* packetData(size_t i) const { return data.data() + offsets[i]; }
	pcppx_batch toC() const
	{
		return pcppx_batch{ data.data(), offsets.data(), caplens.data(), data.size(), (uint32_t)caplens.size(),
			                linkType, 0 };
	}
};

/* PcapFileReaderDevice (Pcap++/header/PcapFileDevice.h): open / getNextPackets / close */
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

	/* Replace `batch` with the next packets (at most maxPackets / maxBytes); returns the count, 0 at EOF. */
	size_t getNextPackets(RawBatch& batch, uint32_t maxPackets = 1u << 20, uint64_t maxBytes = 256ull << 20)
	{
		if (!open())
			throw Error(PCPPX_E_INVAL, "PcapFileReaderDevice::open(" + m_FileName + ")");
		batch.data.resize(maxBytes);
		batch.offsets.resize(maxPackets);
		batch.caplens.resize(maxPackets);
		batch.timestampsNs.resize(maxPackets);
		uint32_t n = 0;
		uint64_t used = 0;
		check(pcppx_pcap_read_batch(m_Reader, batch.data.data(), maxBytes, batch.offsets.data(), batch.caplens.data(),
		                            batch.timestampsNs.data(), maxPackets, &n, &used),
		      "pcppx_pcap_read_batch");
		batch.data.resize(used);
		batch.offsets.resize(n);
		batch.caplens.resize(n);
		batch.timestampsNs.resize(n);
		batch.linkType = (uint16_t)getLinkLayerType();
		return n;
	}

private:
	std::string m_FileName;
	pcppx_pcap* m_Reader = nullptr;
};

/* One layer of a parsed packet: Layer's getProtocol / getOsiModelLayer / getData / getHeaderLen / getDataLen
 * (Packet++/header/Layer.h) */
class ParsedLayer
{
public:
	ParsedLayer(const pcppx_layer* rec, const uint8_t* raw) : m_Rec(rec), m_Raw(raw) {}
	ProtocolType getProtocol() const { return m_Rec->proto; }
	OsiModelLayer getOsiModelLayer() const { return (OsiModelLayer)m_Rec->osi; }
	const uint8_t* getData() const { return m_Raw + m_Rec->offset; }
	size_t getHeaderLen() const { return m_Rec->hdr_len; }
	size_t getDataLen() const { return m_Rec->data_len; }
	size_t getLayerPayloadSize() const { return m_Rec->data_len - m_Rec->hdr_len; }
	uint16_t getOffset() const { return m_Rec->offset; }

private:
	const pcppx_layer* m_Rec;
	const uint8_t* m_Raw;
};

/* A parsed packet: the Packet (Packet++/header/Packet.h) queries this path answers */
class ParsedPacket
{
public:
	ParsedPacket(const pcppx_summary* s, const pcppx_layer* layers, uint8_t maxLayers, const uint8_t* raw)
	    : m_Sum(s), m_Layers(layers), m_MaxLayers(maxLayers), m_Raw(raw)
	{}

	/* Packet::isPacketOfType (Packet.cpp:614-640), for a protocol or a family */
	bool isPacketOfType(ProtocolTypeFamily family) const
	{
		for (int k = 0; k < 4; ++k)
		{
			const uint32_t p = (family >> (8 * k)) & 0xFF;
			if (p != 0 && p < 64 && (m_Sum->proto_mask >> p) & 1)
				return true;
		}
		return false;
	}
	size_t getLayerCount() const { return m_Sum->n_layers; }
	/* records held for the first min(getLayerCount(), maxLayers) layers */
	size_t getRecordedLayerCount() const { return m_Sum->n_layers < m_MaxLayers ? m_Sum->n_layers : m_MaxLayers; }
	ParsedLayer getLayer(size_t k) const { return ParsedLayer(m_Layers + k, m_Raw); }
	ParsedLayer getFirstLayer() const { return getLayer(0); }
	ParsedLayer getLastLayer() const { return getLayer(getRecordedLayerCount() - 1); }
	/* getLayerOfType<T>(): first recorded layer of `proto`, or false */
	bool getLayerOfType(ProtocolType proto, ParsedLayer* out) const
	{
		for (size_t k = 0; k < getRecordedLayerCount(); ++k)
			if (m_Layers[k].proto == proto)
			{
				*out = getLayer(k);
				return true;
			}
		return false;
	}
	/* PacketUtils.h:80-91 */
	uint32_t hash5Tuple(bool const& directionUnique = false) const
	{
		return directionUnique ? m_Sum->hash5_dir : m_Sum->hash5;
	}
	uint32_t hash2Tuple() const { return m_Sum->hash2; }

	/* engine flags: the host must finish the packet (L7, or an L2-L4 protocol outside the device path) */
	bool needsHost() const { return (m_Sum->flags & PCPPX_F_NEEDS_HOST) != 0; }
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
};

/* Records of one parsed batch (owns them); indexes into the RawBatch it was parsed from. */
class ParsedBatch
{
public:
	ParsedBatch(const RawBatch& raw, uint8_t maxLayers)
	    : m_Raw(&raw), m_MaxLayers(maxLayers), summaries(raw.size()), layers(raw.size() * (size_t)maxLayers)
	{}
	size_t size() const { return summaries.size(); }
	ParsedPacket operator[](size_t i) const
	{
		return ParsedPacket(&summaries[i], layers.data() + i * m_MaxLayers, m_MaxLayers, m_Raw->packetData(i));
	}

private:
	const RawBatch* m_Raw;
	uint8_t m_MaxLayers;

public:
	std::vector<pcppx_summary> summaries;
	std::vector<pcppx_layer> layers;
};

/* PacketMatchingEngine's criteria (Examples/DpdkExample-FilterTraffic/PacketMatchingEngine.h:28-41) */
struct MatchSpec
{
	pcppx_match_spec spec{};
	MatchSpec() = default;
	/* addresses as dotted quads ("" = any); ports host order (0 = any); protocol TCP / UDP (else any) */
	MatchSpec(const std::string& srcIp, const std::string& dstIp, uint16_t srcPort, uint16_t dstPort,
	          ProtocolType protocol)
	{
		spec.src_ip = parseIPv4(srcIp);
		spec.dst_ip = parseIPv4(dstIp);
		spec.src_port = srcPort;
		spec.dst_port = dstPort;
		spec.protocol = protocol;
	}
	/* IPv4Address::toInt(): the four address bytes in memory order */
	static uint32_t parseIPv4(const std::string& dotted)
	{
		if (dotted.empty())
			return 0;
		uint8_t b[4] = { 0, 0, 0, 0 };
		unsigned v[4];
		char tail;
		if (std::sscanf(dotted.c_str(), "%u.%u.%u.%u%c", &v[0], &v[1], &v[2], &v[3], &tail) != 4 || v[0] > 255 ||
		    v[1] > 255 || v[2] > 255 || v[3] > 255)
			throw Error(PCPPX_E_INVAL, "bad IPv4 address '" + dotted + "'");
		for (int k = 0; k < 4; ++k)
			b[k] = (uint8_t)v[k];
		uint32_t out;
		std::memcpy(&out, b, 4);
		return out;
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

	/* Packet(&rawPacket, options) for every packet of the batch, host to host through HBM */
	ParsedBatch parse(const RawBatch& batch, const PacketParseOptions& options = PacketParseOptions()) const
	{
		ParsedBatch out(batch, options.maxLayers);
		parseInto(batch, options, out);
		return out;
	}
	void parseInto(const RawBatch& batch, const PacketParseOptions& options, ParsedBatch& out) const
	{
		const pcppx_batch b = batch.toC();
		const pcppx_opts o = options.toC();
		pcppx_records r{ out.summaries.data(), options.maxLayers ? out.layers.data() : nullptr };
		check(pcppx_parse_batch_host(m_Ctx, &b, &o, &r), "pcppx_parse_batch_host");
	}

	/* FilterTraffic's worker (AppWorkerThread.h:85-139): matched[i] = 1 for packets to send on; the flow
	 * table persists across calls until resetFilter() */
	pcppx_packet_stats filter(const RawBatch& batch, const MatchSpec& spec, std::vector<uint8_t>& matched)
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
};

}  // namespace pcppx

#endif /* PCPPX_HPP */
