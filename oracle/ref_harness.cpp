// ref_harness.cpp — TEST INFRASTRUCTURE ONLY (part of oracle/).
//
// Our own harness around the *real* reference Packet++ (compiled from /root/reference sources by
// oracle/Makefile into oracle/_ref/). It turns a pcppx_batch into pcppx records by driving the
// reference API exactly as its own callers do:
//   Packet(RawPacket*, false, parseUntil, parseUntilLayer)      Packet++/src/Packet.cpp:202-209
//   layer walk: getProtocol/getOsiModelLayer/getData/getHeaderLen/getDataLen   Packet++/header/Layer.h
//   hash5Tuple(&p, false|true), hash2Tuple(&p)                  Packet++/src/PacketUtils.cpp:139-245
//   IPv4 header checksum as IPv4Layer::computeCalculateFields   Packet++/src/IPv4Layer.cpp:410-412
//   TcpLayer/UdpLayer::calculateChecksum(false)                 TcpLayer.cpp:271-311, UdpLayer.cpp:47-90
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library.
// It never ships in the product path.

#include "pcppx.h"

#include "Packet.h"
#include "RawPacket.h"
#include "IPv4Layer.h"
#include "IPv6Layer.h"
#include "TcpLayer.h"
#include "UdpLayer.h"
#include "PacketUtils.h"
#include "IPv6Extensions.h"
#include "IPReassembly.h"
#include "TcpReassembly.h"
#include "EndianPortable.h"
#include "Logger.h"
#include "PacketMatchingEngine.h"  // Examples/DpdkExample-FilterTraffic/PacketMatchingEngine.h (header-only)

#include <chrono>
#include <cstring>
#include <thread>
#include <unordered_map>
#include <vector>

namespace
{
	uint16_t be16at(const uint8_t* p)
	{
		return static_cast<uint16_t>((p[0] << 8) | p[1]);
	}

	void fillRecord(pcpp::Packet& packet, const uint8_t* raw, const pcppx_opts* opts, pcppx_summary* sum,
	                pcppx_layer* layers)
	{
		std::memset(sum, 0, sizeof(*sum));
		sum->l4_layer = 0xFF;
		int cap = opts->max_layers;
		int idx = 0;
		uint64_t mask = 0;
		pcpp::Layer* last = nullptr;
		for (pcpp::Layer* l = packet.getFirstLayer(); l != nullptr; l = l->getNextLayer(), ++idx)
		{
			mask |= (uint64_t)1 << (l->getProtocol() & 63);
			if (layers != nullptr && idx < cap)
			{
				pcppx_layer& o = layers[idx];
				o.proto = l->getProtocol();
				o.osi = static_cast<uint8_t>(l->getOsiModelLayer());
				o.offset = static_cast<uint16_t>(l->getData() - raw);
				o.hdr_len = static_cast<uint16_t>(l->getHeaderLen());
				o.data_len = static_cast<uint16_t>(l->getDataLen());
			}
			last = l;
		}
		uint16_t flags = 0;
		int limit = cap > 0 ? cap : PCPPX_MAX_LAYERS;
		if (idx > limit)
			flags |= PCPPX_F_DEPTH_OVERFLOW;
		sum->n_layers = static_cast<uint8_t>(idx > limit ? limit : idx);
		sum->proto_mask = mask;
		if (last != nullptr && last->getProtocol() == pcpp::PacketTrailer)
			flags |= PCPPX_F_TRAILER;

		sum->hash5 = pcpp::hash5Tuple(&packet, false);
		sum->hash5_dir = pcpp::hash5Tuple(&packet, true);
		sum->hash2 = pcpp::hash2Tuple(&packet);

		// index of the layer hash5Tuple reads its ports from (PacketUtils.cpp:157-169)
		pcpp::Layer* l4 = packet.getLayerOfType<pcpp::TcpLayer>(true);
		if (l4 == nullptr)
			l4 = packet.getLayerOfType<pcpp::UdpLayer>(true);
		if (l4 != nullptr)
		{
			int i = 0;
			for (pcpp::Layer* l = packet.getFirstLayer(); l != l4; l = l->getNextLayer())
				++i;
			sum->l4_layer = static_cast<uint8_t>(i);
		}

		if (opts->want_checksums)
		{
			pcpp::IPv4Layer* ip = packet.getLayerOfType<pcpp::IPv4Layer>();
			if (ip != nullptr)
			{
				size_t hl = (std::min)(static_cast<size_t>(ip->getIPv4Header()->internetHeaderLength * 4),
				                       ip->getDataLen());
				std::vector<uint8_t> hdr(ip->getData(), ip->getData() + hl);
				if (hl >= 12)
				{
					hdr[10] = 0;
					hdr[11] = 0;
				}
				pcpp::ScalarBuffer<uint16_t> sb = { reinterpret_cast<uint16_t*>(hdr.data()), hl };
				sum->ip_csum_calc = pcpp::computeChecksum(&sb, 1);
				sum->ip_csum_stored = be16at(ip->getData() + 10);
				flags |= PCPPX_F_IP_CSUM;
				if (sum->ip_csum_calc == sum->ip_csum_stored)
					flags |= PCPPX_F_IP_CSUM_OK;
			}
			if (l4 != nullptr)
			{
				if (l4->getProtocol() == pcpp::TCP)
				{
					sum->l4_csum_calc = static_cast<pcpp::TcpLayer*>(l4)->calculateChecksum(false);
					sum->l4_csum_stored = be16at(l4->getData() + 16);
				}
				else
				{
					sum->l4_csum_calc = static_cast<pcpp::UdpLayer*>(l4)->calculateChecksum(false);
					sum->l4_csum_stored = be16at(l4->getData() + 6);
				}
				flags |= PCPPX_F_L4_CSUM;
				if (sum->l4_csum_calc == sum->l4_csum_stored)
					flags |= PCPPX_F_L4_CSUM_OK;
			}
		}
		sum->flags = flags;
	}

	struct Prepared
	{
		std::vector<uint8_t> bytes;  // private mutable copy: calculateChecksum zeroes+restores a field
		std::vector<pcpp::RawPacket> raws;
	};

	void prepare(const pcppx_batch* b, Prepared& p)
	{
		uint64_t total = 0;
		for (uint32_t i = 0; i < b->n; ++i)
			total += b->caplens[i];
		p.bytes.resize(total + 1);
		p.raws.clear();
		p.raws.reserve(b->n);
		uint64_t pos = 0;
		timeval ts{ 0, 0 };
		for (uint32_t i = 0; i < b->n; ++i)
		{
			std::memcpy(p.bytes.data() + pos, b->data + b->offsets[i], b->caplens[i]);
			p.raws.emplace_back(p.bytes.data() + pos, static_cast<int>(b->caplens[i]), ts, false,
			                    static_cast<pcpp::LinkLayerType>(b->linktype));
			pos += b->caplens[i];
		}
	}
}  // namespace

extern "C"
{
	// DpdkExample-FilterTraffic's per-packet worker loop (AppWorkerThread.h:85-139) over a host batch, with
	// the real PacketMatchingEngine and hash5Tuple; PacketStats::collectStats is restated from
	// Common.h:83-104 (Common.h itself includes DPDK headers). matched[i] = whether packet i was matched.
	int pcppx_ref_filter(const pcppx_batch* b, const pcppx_match_spec* spec, uint8_t* matched,
	                     pcppx_packet_stats* st)
	{
		if (b == nullptr || spec == nullptr || matched == nullptr || st == nullptr)
			return PCPPX_E_INVAL;
		pcpp::Logger::getInstance().suppressLogs();
		Prepared p;
		prepare(b, p);
		PacketMatchingEngine engine(pcpp::IPv4Address(spec->src_ip), pcpp::IPv4Address(spec->dst_ip), spec->src_port,
		                            spec->dst_port, static_cast<pcpp::ProtocolType>(spec->protocol));
		std::unordered_map<uint32_t, bool> flowTable;
		std::memset(st, 0, sizeof(*st));
		for (uint32_t i = 0; i < b->n; ++i)
		{
			pcpp::Packet parsedPacket(&p.raws[i]);
			st->packet_count++;
			st->eth_count += parsedPacket.isPacketOfType(pcpp::Ethernet);
			st->arp_count += parsedPacket.isPacketOfType(pcpp::ARP);
			st->ipv4_count += parsedPacket.isPacketOfType(pcpp::IPv4);
			st->ipv6_count += parsedPacket.isPacketOfType(pcpp::IPv6);
			st->tcp_count += parsedPacket.isPacketOfType(pcpp::TCP);
			st->udp_count += parsedPacket.isPacketOfType(pcpp::UDP);
			st->http_count += parsedPacket.isPacketOfType(pcpp::HTTP);
			st->dns_count += parsedPacket.isPacketOfType(pcpp::DNS);
			st->tls_count += parsedPacket.isPacketOfType(pcpp::SSL);
			bool packetMatched;
			uint32_t hash = pcpp::hash5Tuple(&parsedPacket);
			auto it = flowTable.find(hash);
			if (it != flowTable.end() && it->second)
				packetMatched = true;
			else
			{
				packetMatched = engine.isMatched(parsedPacket);
				if (packetMatched)
				{
					flowTable[hash] = true;
					if (parsedPacket.isPacketOfType(pcpp::TCP))
						st->matched_tcp_flows++;
					else if (parsedPacket.isPacketOfType(pcpp::UDP))
						st->matched_udp_flows++;
				}
			}
			if (packetMatched)
				st->matched_packets++;
			matched[i] = packetMatched ? 1 : 0;
		}
		return PCPPX_OK;
	}

	// Reassembly front ends of the real reference per packet, as a first sighting: a fresh IPReassembly
	// (processPacket status, Packet++/src/IPReassembly.cpp:281-) and a fresh TcpReassembly (reassemblePacket
	// status, Packet++/src/TcpReassembly.cpp:81-) per packet, the fragment key through the public
	// PacketKey::getHashValue (IPReassembly.cpp:233-269: the same bytes as hashPacket) and the fragment / TCP
	// fields through the layers' own accessors.
	int pcppx_ref_reasm(const pcppx_batch* b, pcppx_reasm_info* out)
	{
		if (b == nullptr || out == nullptr)
			return PCPPX_E_INVAL;
		pcpp::Logger::getInstance().suppressLogs();
		Prepared p;
		prepare(b, p);
		for (uint32_t i = 0; i < b->n; ++i)
		{
			pcppx_reasm_info& o = out[i];
			std::memset(&o, 0, sizeof(o));
			pcpp::Packet packet(&p.raws[i]);
			{
				pcpp::IPReassembly ipr;
				pcpp::IPReassembly::ReassemblyStatus st = pcpp::IPReassembly::NON_IP_PACKET;
				pcpp::Packet* r = ipr.processPacket(&packet, st);
				if (r != nullptr && r != &packet)
					delete r;
				uint8_t s = PCPPX_IPR_FRAGMENT;
				if (st == pcpp::IPReassembly::NON_IP_PACKET)
					s = PCPPX_IPR_NON_IP;
				else if (st == pcpp::IPReassembly::NON_FRAGMENT)
					s = PCPPX_IPR_NON_FRAGMENT;
				else if (st == pcpp::IPReassembly::MALFORMED_FRAGMENT)
					s = PCPPX_IPR_MALFORMED;
				const bool v4 = packet.isPacketOfType(pcpp::IPv4);
				if (!v4 && s != PCPPX_IPR_NON_IP)
					s |= PCPPX_IPR_F_IPV6;
				if ((s & 0xF) == PCPPX_IPR_FRAGMENT && v4)
				{
					auto* ip = packet.getLayerOfType<pcpp::IPv4Layer>();
					const uint16_t id = be16toh(ip->getIPv4Header()->ipId);
					o.frag_id = id;
					o.frag_offset = ip->getFragmentOffset();
					s |= (ip->isFirstFragment() ? PCPPX_IPR_F_FIRST : 0) | (ip->isLastFragment() ? PCPPX_IPR_F_LAST : 0);
					o.ip_key =
					    pcpp::IPReassembly::IPv4PacketKey(id, ip->getSrcIPv4Address(), ip->getDstIPv4Address()).getHashValue();
				}
				else if ((s & 0xF) == PCPPX_IPR_FRAGMENT)
				{
					auto* ip = packet.getLayerOfType<pcpp::IPv6Layer>();
					auto* fh = ip->getExtensionOfType<pcpp::IPv6FragmentationHeader>();
					const uint32_t id = be32toh(fh->getFragHeader()->id);
					o.frag_id = id;
					o.frag_offset = fh->getFragmentOffset();
					s |= (fh->isFirstFragment() ? PCPPX_IPR_F_FIRST : 0) | (fh->isLastFragment() ? PCPPX_IPR_F_LAST : 0);
					o.ip_key =
					    pcpp::IPReassembly::IPv6PacketKey(id, ip->getSrcIPv6Address(), ip->getDstIPv6Address()).getHashValue();
				}
				o.ip_status = s;
			}
			{
				pcpp::TcpReassembly tcr([](int8_t, const pcpp::TcpStreamData&, void*) {});
				const auto st = tcr.reassemblePacket(packet);
				uint8_t s = PCPPX_TCPR_DATA;
				if (st == pcpp::TcpReassembly::NonIpPacket)
					s = PCPPX_TCPR_NON_IP;
				else if (st == pcpp::TcpReassembly::NonTcpPacket)
					s = PCPPX_TCPR_NON_TCP;
				else if (st == pcpp::TcpReassembly::Ignore_PacketWithNoData)
					s = PCPPX_TCPR_NO_DATA;
				auto* tcp = packet.getLayerOfType<pcpp::TcpLayer>(true);
				if (tcp != nullptr && s != PCPPX_TCPR_NON_IP && s != PCPPX_TCPR_NON_TCP)
				{
					const pcpp::tcphdr* h = tcp->getTcpHeader();
					s |= (h->finFlag ? PCPPX_TCPR_F_FIN : 0) | (h->synFlag ? PCPPX_TCPR_F_SYN : 0) |
					     (h->rstFlag ? PCPPX_TCPR_F_RST : 0);
					o.tcp_payload = static_cast<uint32_t>(tcp->getLayerPayloadSize());
				}
				o.tcp_status = s;
			}
		}
		return PCPPX_OK;
	}

	// pcppx_host_parse_fn (include/pcppx.h) over the real reference: the completion step for packets the engine
	// flags NEEDS_HOST, as a caller's own Packet++ performs it. Test infrastructure: the
	// example programs load it only when a test passes this library to them.
	int pcppx_host_parse(const uint8_t* pkt, uint32_t caplen, uint16_t linktype, const pcppx_opts* opts,
	                     pcppx_summary* summary, pcppx_layer* layers)
	{
		if (pkt == nullptr || opts == nullptr || summary == nullptr)
			return PCPPX_E_INVAL;
		pcpp::Logger::getInstance().suppressLogs();
		std::vector<uint8_t> bytes(pkt, pkt + caplen);  // calculateChecksum zeroes and restores a field
		bytes.push_back(0);
		timeval ts{ 0, 0 };
		pcpp::RawPacket raw(bytes.data(), static_cast<int>(caplen), ts, false, static_cast<pcpp::LinkLayerType>(linktype));
		pcpp::Packet packet(&raw, false, opts->parse_until_family, static_cast<pcpp::OsiModelLayer>(opts->parse_until_osi));
		fillRecord(packet, raw.getRawData(), opts, summary, opts->max_layers > 0 ? layers : nullptr);
		return PCPPX_OK;
	}

	// The 5-tuple extract (include/pcppx.h pcppx_tuple) through the reference's own accessors, for every packet of a
	// host batch parsed as Packet(&raw): the first IPv4 layer (getLayerOfType<IPv4Layer>()) else the first IPv6
	// layer, their getSrc/DstIPv4Address / getSrc/DstIPv6Address and protocol / nextHeader; the port layer
	// hash5Tuple takes (getLayerOfType<TcpLayer>(true), else <UdpLayer>(true), PacketUtils.cpp:157-169) and its
	// getSrcPort / getDstPort; has_5tuple = isPacketOfType(IPv4|IPv6) && !ICMP && (TCP|UDP) (PacketUtils.cpp:141-148);
	// hash5 = hash5Tuple(&packet). flags is left 0 (the engine's own), n_layers = the chain length.
	int pcppx_ref_tuples(const pcppx_batch* b, pcppx_tuple* out)
	{
		if (b == nullptr || out == nullptr)
			return PCPPX_E_INVAL;
		pcpp::Logger::getInstance().suppressLogs();
		Prepared p;
		prepare(b, p);
		for (uint32_t i = 0; i < b->n; ++i)
		{
			pcppx_tuple& t = out[i];
			std::memset(&t, 0, sizeof(t));
			pcpp::Packet packet(&p.raws[i]);
			if (auto* v4 = packet.getLayerOfType<pcpp::IPv4Layer>())
			{
				const uint32_t s4 = v4->getSrcIPv4Address().toInt(), d4 = v4->getDstIPv4Address().toInt();
				std::memcpy(t.src_ip, &s4, 4);
				std::memcpy(t.dst_ip, &d4, 4);
				t.ip_version = 4;
				t.ip_proto = v4->getIPv4Header()->protocol;
			}
			else if (auto* v6 = packet.getLayerOfType<pcpp::IPv6Layer>())
			{
				std::memcpy(t.src_ip, v6->getSrcIPv6Address().toBytes(), 16);
				std::memcpy(t.dst_ip, v6->getDstIPv6Address().toBytes(), 16);
				t.ip_version = 6;
				t.ip_proto = v6->getIPv6Header()->nextHeader;
			}
			if (auto* tcp = packet.getLayerOfType<pcpp::TcpLayer>(true))
			{
				t.src_port = tcp->getSrcPort();
				t.dst_port = tcp->getDstPort();
				t.l4_proto = pcpp::TCP;
			}
			else if (auto* udp = packet.getLayerOfType<pcpp::UdpLayer>(true))
			{
				t.src_port = udp->getSrcPort();
				t.dst_port = udp->getDstPort();
				t.l4_proto = pcpp::UDP;
			}
			t.has_5tuple = (packet.isPacketOfType(pcpp::IPv4) || packet.isPacketOfType(pcpp::IPv6)) &&
			               !packet.isPacketOfType(pcpp::ICMP) &&
			               (packet.isPacketOfType(pcpp::TCP) || packet.isPacketOfType(pcpp::UDP));
			t.hash5 = pcpp::hash5Tuple(&packet);
			int nl = 0;
			for (pcpp::Layer* l = packet.getFirstLayer(); l != nullptr; l = l->getNextLayer())
				++nl;
			t.n_layers = static_cast<uint8_t>(nl > 255 ? 255 : nl);
		}
		return PCPPX_OK;
	}

	// Parse a host batch with the reference Packet++ and fill host records.
	int pcppx_ref_parse_batch(const pcppx_batch* b, const pcppx_opts* opts, pcppx_records* out)
	{
		if (b == nullptr || opts == nullptr || out == nullptr || out->summary == nullptr)
			return PCPPX_E_INVAL;
		pcpp::Logger::getInstance().suppressLogs();
		Prepared p;
		prepare(b, p);
		for (uint32_t i = 0; i < b->n; ++i)
		{
			pcpp::Packet packet(&p.raws[i], false, opts->parse_until_family,
			                    static_cast<pcpp::OsiModelLayer>(opts->parse_until_osi));
			pcppx_layer* layers = (out->layers != nullptr && opts->max_layers > 0)
			                          ? out->layers + static_cast<size_t>(i) * opts->max_layers
			                          : nullptr;
			fillRecord(packet, p.raws[i].getRawData(), opts, &out->summary[i], layers);
		}
		return PCPPX_OK;
	}

	// Timed CPU baseline: the reference parse (+hash5Tuple both directions, hash2Tuple, and the
	// checksums when opts->want_checksums) over the batch, packets preloaded as RawPackets in the style
	// of BM_PacketPureParsing (Examples/PcapPlusPlus-benchmark/benchmark-google.cpp:209-264), packet
	// indices interleaved over `threads` threads. Returns seconds of the timed region.
	int pcppx_ref_bench(const pcppx_batch* b, const pcppx_opts* opts, int threads, double* seconds,
	                    uint64_t* digest)
	{
		if (b == nullptr || opts == nullptr || seconds == nullptr || threads < 1)
			return PCPPX_E_INVAL;
		pcpp::Logger::getInstance().suppressLogs();
		Prepared p;
		prepare(b, p);
		std::vector<uint64_t> part(threads, 0);
		auto work = [&](int t) {
			uint64_t acc = 0;
			for (uint32_t i = t; i < b->n; i += threads)
			{
				pcpp::Packet packet(&p.raws[i], false, opts->parse_until_family,
				                    static_cast<pcpp::OsiModelLayer>(opts->parse_until_osi));
				acc += pcpp::hash5Tuple(&packet, false);
				acc += pcpp::hash5Tuple(&packet, true);
				acc += pcpp::hash2Tuple(&packet);
				if (opts->want_checksums)
				{
					pcpp::IPv4Layer* ip = packet.getLayerOfType<pcpp::IPv4Layer>();
					if (ip != nullptr)
					{
						size_t hl = (std::min)(static_cast<size_t>(ip->getIPv4Header()->internetHeaderLength * 4),
						                       ip->getDataLen());
						uint8_t hdr[64];
						std::memcpy(hdr, ip->getData(), hl);
						hdr[10] = hdr[11] = 0;
						pcpp::ScalarBuffer<uint16_t> sb = { reinterpret_cast<uint16_t*>(hdr), hl };
						acc += pcpp::computeChecksum(&sb, 1);
					}
					pcpp::TcpLayer* tcp = packet.getLayerOfType<pcpp::TcpLayer>(true);
					if (tcp != nullptr)
						acc += tcp->calculateChecksum(false);
					else
					{
						pcpp::UdpLayer* udp = packet.getLayerOfType<pcpp::UdpLayer>(true);
						if (udp != nullptr)
							acc += udp->calculateChecksum(false);
					}
				}
			}
			part[t] = acc;
		};
		auto t0 = std::chrono::steady_clock::now();
		if (threads == 1)
			work(0);
		else
		{
			std::vector<std::thread> pool;
			for (int t = 0; t < threads; ++t)
				pool.emplace_back(work, t);
			for (auto& th : pool)
				th.join();
		}
		auto t1 = std::chrono::steady_clock::now();
		*seconds = std::chrono::duration<double>(t1 - t0).count();
		if (digest != nullptr)
		{
			uint64_t d = 0;
			for (auto v : part)
				d += v;
			*digest = d;
		}
		return PCPPX_OK;
	}
}
