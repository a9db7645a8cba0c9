/**
 * DpdkExample-FilterTraffic's worker on the GPU parse engine
 * ==========================================================
 * The reference worker (Examples/DpdkExample-FilterTraffic/AppWorkerThread.h:45-162, PacketStats Common.h:57-142,
 * PacketMatchingEngine.h:43-107, the stats table main.cpp:244-264) over the engine's facade (`namespace pcpp =
 * pcppx`), with a capture file in place of the DPDK RX queues: receivePackets fills each burst of RawPackets from
 * pages the reader has already parsed on the GPU (the batch prepass runs inside the library), and the burst loop --
 * `pcpp::Packet parsedPacket(packetArr[i])`, collectStats, hash5Tuple, the flow table, isMatched, the pcap writer --
 * is the reference's. Packets the engine leaves to the host are completed by the caller's own Packet++ parse
 * (--host-parser <lib.so> exporting pcppx_host_parse), so every counter, HTTP/DNS/TLS included, is the reference's.
 *
 * --device-worker runs the whole worker on the GPU instead (pcppx_filter_batch_host: flow table, matching and
 * statistics in HBM); its HTTP/DNS/TLS counters cover the packets the device settles ("left to host" counts the
 * rest).
 *
 *   filter_traffic -f in.pcap [-o out.pcap] [-s SRC_IP] [-d DST_IP] [-S SRC_PORT] [-D DST_PORT] [-P TCP|UDP]
 *                  [-b BURST] [--host-parser <lib.so>] [--device-worker]
 * BURST: packets per receivePackets call (MAX_RECEIVE_BURST, 64) or, with --device-worker, per device batch (1M).
 */
#include <dlfcn.h>

#include <cstdio>
#include <cstdlib>
#include <iomanip>
#include <iostream>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#include "pcppx.hpp"

namespace pcpp = pcppx;

namespace
{
/* PacketStats (Common.h:57-142) */
struct PacketStats
{
	uint64_t packetCount = 0, ethCount = 0, arpCount = 0, ipv4Count = 0, ipv6Count = 0, tcpCount = 0, udpCount = 0,
	         httpCount = 0, dnsCount = 0, tlsCount = 0;
	uint64_t matchedTcpFlows = 0, matchedUdpFlows = 0, matchedPackets = 0;
	uint64_t leftToHost = 0; /* packets a counter of which the device could not settle (device worker only) */

	void collectStats(const pcppx::Packet& packet)
	{
		packetCount++;
		if (packet.isPacketOfType(pcppx::Ethernet))
			ethCount++;
		if (packet.isPacketOfType(pcppx::ARP))
			arpCount++;
		if (packet.isPacketOfType(pcppx::IPv4))
			ipv4Count++;
		if (packet.isPacketOfType(pcppx::IPv6))
			ipv6Count++;
		if (packet.isPacketOfType(pcppx::TCP))
			tcpCount++;
		if (packet.isPacketOfType(pcppx::UDP))
			udpCount++;
		if (packet.isPacketOfType(pcppx::HTTP))
			httpCount++;
		if (packet.isPacketOfType(pcppx::DNS))
			dnsCount++;
		if (packet.isPacketOfType(pcppx::SSL))
			tlsCount++;
		if (packet.needsHost())
			leftToHost++;
	}
};

/* PacketMatchingEngine (PacketMatchingEngine.h:15-107): source / destination IPv4, ports, TCP|UDP */
class PacketMatchingEngine
{
public:
	PacketMatchingEngine(const pcppx::IPv4Address& srcIp, const pcppx::IPv4Address& dstIp, uint16_t srcPort,
	                     uint16_t dstPort, pcppx::ProtocolType protocol)
	    : m_SrcIp(srcIp), m_DstIp(dstIp), m_SrcPort(srcPort), m_DstPort(dstPort), m_Protocol(protocol),
	      m_MatchSrcIp(srcIp != pcppx::IPv4Address::Zero), m_MatchDstIp(dstIp != pcppx::IPv4Address::Zero),
	      m_MatchSrcPort(srcPort != 0), m_MatchDstPort(dstPort != 0),
	      m_MatchProtocol(protocol == pcppx::TCP || protocol == pcppx::UDP)
	{}

	bool isMatched(const pcppx::Packet& packet) const
	{
		if (m_MatchSrcIp || m_MatchDstIp)
		{
			if (!packet.isPacketOfType(pcppx::IPv4))
				return false;
			auto ip4Layer = packet.getLayerOfType<pcppx::IPv4Layer>();
			if (m_MatchSrcIp && ip4Layer->getSrcIPv4Address() != m_SrcIp)
				return false;
			if (m_MatchDstIp && ip4Layer->getDstIPv4Address() != m_DstIp)
				return false;
		}
		if (m_MatchSrcPort || m_MatchDstPort)
		{
			uint16_t srcPort, dstPort;
			if (packet.isPacketOfType(pcppx::TCP))
			{
				srcPort = packet.getLayerOfType<pcppx::TcpLayer>()->getSrcPort();
				dstPort = packet.getLayerOfType<pcppx::TcpLayer>()->getDstPort();
			}
			else if (packet.isPacketOfType(pcppx::UDP))
			{
				srcPort = packet.getLayerOfType<pcppx::UdpLayer>()->getSrcPort();
				dstPort = packet.getLayerOfType<pcppx::UdpLayer>()->getDstPort();
			}
			else
				return false;
			if (m_MatchSrcPort && srcPort != m_SrcPort)
				return false;
			if (m_MatchDstPort && dstPort != m_DstPort)
				return false;
		}
		if (m_MatchProtocol)
		{
			if (m_Protocol == pcppx::TCP && !packet.isPacketOfType(pcppx::TCP))
				return false;
			if (m_Protocol == pcppx::UDP && !packet.isPacketOfType(pcppx::UDP))
				return false;
		}
		return true;
	}

	pcppx::MatchSpec spec() const
	{
		pcppx::MatchSpec s;
		s.spec.src_ip = m_SrcIp.toInt();
		s.spec.dst_ip = m_DstIp.toInt();
		s.spec.src_port = m_SrcPort;
		s.spec.dst_port = m_DstPort;
		s.spec.protocol = m_Protocol;
		return s;
	}

private:
	pcppx::IPv4Address m_SrcIp, m_DstIp;
	uint16_t m_SrcPort, m_DstPort;
	pcppx::ProtocolType m_Protocol;
	bool m_MatchSrcIp, m_MatchDstIp, m_MatchSrcPort, m_MatchDstPort, m_MatchProtocol;
};

/* the worker (AppWorkerThread.h:45-162): the input file replaces the DPDK RX queues */
class AppWorkerThread
{
public:
	AppWorkerThread(pcppx::Engine& engine, const PacketMatchingEngine& matchingEngine, size_t burst)
	    : m_Engine(engine), m_PacketMatchingEngine(matchingEngine), m_Burst(burst)
	{}
	PacketStats& getStats() { return m_Stats; }

	/* AppWorkerThread::run (AppWorkerThread.h:45-162): the capture is the RX queue (receivePackets fills a burst
	 * of RawPackets from pages the reader has already parsed on the GPU), and the burst loop is the reference's */
	bool run(pcppx::PcapFileReaderDevice* dev, pcpp::PcapFileWriterDevice* pcapWriter)
	{
		std::vector<pcpp::RawPacket*> packetArr(m_Burst, nullptr);

		// main loop, runs until the capture ends
		while (!m_Stop)
		{
			// receive packets from the capture (was dev->receivePackets(packetArr, MAX_RECEIVE_BURST, rxQueue))
			uint16_t packetsReceived = dev->receivePackets(packetArr.data(), (uint16_t)m_Burst, 0);
			if (packetsReceived == 0)
				break;

			for (int i = 0; i < packetsReceived; i++)
			{
				// parse packet
				pcpp::Packet parsedPacket(packetArr[i]);

				// collect packet statistics
				m_Stats.collectStats(parsedPacket);

				bool packetMatched;

				// hash the packet by 5-tuple and look in the flow table to see whether this packet belongs to an
				// existing or new flow
				uint32_t hash = pcpp::hash5Tuple(&parsedPacket);
				auto iter3 = m_FlowTable.find(hash);

				// if packet belongs to an already existing flow
				if (iter3 != m_FlowTable.end() && iter3->second)
				{
					packetMatched = true;
				}
				else  // packet belongs to a new flow
				{
					packetMatched = m_PacketMatchingEngine.isMatched(parsedPacket);
					if (packetMatched)
					{
						// put new flow in flow table
						m_FlowTable[hash] = true;

						// collect stats
						if (parsedPacket.isPacketOfType(pcpp::TCP))
						{
							m_Stats.matchedTcpFlows++;
						}
						else if (parsedPacket.isPacketOfType(pcpp::UDP))
						{
							m_Stats.matchedUdpFlows++;
						}
					}
				}

				if (packetMatched)
				{
					// save packet to file if needed
					if (pcapWriter != nullptr)
					{
						pcapWriter->writePacket(*packetArr[i]);
					}

					m_Stats.matchedPackets++;
				}
			}
		}

		// free packet array
		for (size_t i = 0; i < packetArr.size(); i++)
		{
			if (packetArr[i] != nullptr)
				delete packetArr[i];
		}
		return true;
	}

	/* the whole worker on the GPU: flow table, matching and statistics in HBM (pcppx_filter_batch_host) */
	bool runOnDevice(pcppx::PcapFileReaderDevice& reader, pcpp::PcapFileWriterDevice* pcapWriter)
	{
		pcppx::RawBatch packetArr;
		std::vector<uint8_t> matched;
		pcppx_packet_stats s{};
		m_Engine.resetFilter();
		const pcppx::MatchSpec spec = m_PacketMatchingEngine.spec();
		while (reader.getNextBatch(packetArr, (int)m_Burst) > 0)
		{
			s = m_Engine.filter(packetArr, spec, matched);
			if (pcapWriter != nullptr)
				for (size_t i = 0; i < packetArr.size(); ++i)
					if (matched[i])
					{
						const uint64_t ts = packetArr.timestampsNs[i];
						pcpp::RawPacket raw(packetArr.packetData(i), (int)packetArr.caplens[i],
						                    timespec{ (time_t)(ts / 1000000000ull), (long)(ts % 1000000000ull) }, false,
						                    packetArr.linkType);
						(void)raw.setRawData(packetArr.packetData(i), (int)packetArr.caplens[i], false,
						                     raw.getPacketTimeStamp(), packetArr.linkType, (int)packetArr.frameLens[i]);
						pcapWriter->writePacket(raw);
					}
		}
		m_Stats.packetCount = s.packet_count;
		m_Stats.ethCount = s.eth_count;
		m_Stats.arpCount = s.arp_count;
		m_Stats.ipv4Count = s.ipv4_count;
		m_Stats.ipv6Count = s.ipv6_count;
		m_Stats.tcpCount = s.tcp_count;
		m_Stats.udpCount = s.udp_count;
		m_Stats.httpCount = s.http_count;
		m_Stats.dnsCount = s.dns_count;
		m_Stats.tlsCount = s.tls_count;
		m_Stats.matchedTcpFlows = s.matched_tcp_flows;
		m_Stats.matchedUdpFlows = s.matched_udp_flows;
		m_Stats.matchedPackets = s.matched_packets;
		m_Stats.leftToHost = s.needs_host_count;
		return true;
	}

private:
	pcppx::Engine& m_Engine;
	const PacketMatchingEngine& m_PacketMatchingEngine;
	size_t m_Burst;
	bool m_Stop = false;
	PacketStats m_Stats;
	std::unordered_map<uint32_t, bool> m_FlowTable;
};

void printRow(const std::string& name, uint64_t v)
{
	std::cout << "| " << std::left << std::setw(21) << name << "| " << std::right << std::setw(10) << v << " |\n";
}
void printSeparator()
{
	std::cout << "+----------------------+-----------+\n";
}
/* printStats (main.cpp:244-264) */
void printStats(const PacketStats& threadStats, const std::string& columnName)
{
	printSeparator();
	std::cout << "| " << std::left << std::setw(21) << columnName << "| " << std::right << std::setw(10) << "Count"
	          << " |\n";
	printSeparator();
	printRow("Eth count", threadStats.ethCount);
	printRow("ARP count", threadStats.arpCount);
	printRow("IPv4 count", threadStats.ipv4Count);
	printRow("IPv6 count", threadStats.ipv6Count);
	printRow("TCP count", threadStats.tcpCount);
	printRow("UDP count", threadStats.udpCount);
	printRow("HTTP count", threadStats.httpCount);
	printRow("DNS count", threadStats.dnsCount);
	printRow("TLS count", threadStats.tlsCount);
	printSeparator();
	printRow("Matched TCP flows", threadStats.matchedTcpFlows);
	printRow("Matched UDP flows", threadStats.matchedUdpFlows);
	printSeparator();
	printRow("Matched packet count", threadStats.matchedPackets);
	printRow("Total packet count", threadStats.packetCount);
	printRow("Left to host", threadStats.leftToHost);
	printSeparator();
}

void usage(const char* argv0)
{
	std::cout << "Usage: " << argv0
	          << " -f <in.pcap> [-o <out.pcap>] [-s <src ip>] [-d <dst ip>] [-S <src port>] [-D <dst port>]"
	             " [-P <TCP|UDP>] [-b <burst>] [--host-parser <lib.so>] [--device-worker]\n";
}

pcppx_host_parse_fn loadHostParser(const std::string& path)
{
	void* lib = dlopen(path.c_str(), RTLD_NOW | RTLD_LOCAL);
	if (lib == nullptr)
		throw pcppx::Error(PCPPX_E_INVAL, std::string("dlopen: ") + dlerror());
	auto fn = reinterpret_cast<pcppx_host_parse_fn>(dlsym(lib, "pcppx_host_parse"));
	if (fn == nullptr)
		throw pcppx::Error(PCPPX_E_INVAL, path + " does not export pcppx_host_parse");
	return fn;
}
}  // namespace

int main(int argc, char* argv[])
{
	std::string in, out, sip, dip, hostParser;
	uint16_t sport = 0, dport = 0;
	size_t burst = 0;  // 0: 64 per receivePackets call, 1M per device-worker batch
	bool deviceWorker = false;
	pcppx::ProtocolType proto = pcppx::UnknownProtocol;
	for (int k = 1; k < argc; ++k)
	{
		const std::string a = argv[k];
		if (a == "--device-worker")
		{
			deviceWorker = true;
			continue;
		}
		if (k + 1 >= argc)
		{
			usage(argv[0]);
			return 1;
		}
		const std::string v = argv[++k];
		if (a == "-f") in = v;
		else if (a == "-o") out = v;
		else if (a == "-s") sip = v;
		else if (a == "-d") dip = v;
		else if (a == "-S") sport = (uint16_t)std::atoi(v.c_str());
		else if (a == "-D") dport = (uint16_t)std::atoi(v.c_str());
		else if (a == "-b") burst = (size_t)std::atol(v.c_str());
		else if (a == "--host-parser") hostParser = v;
		else if (a == "-P")
		{
			if (v == "TCP") proto = pcppx::TCP;
			else if (v == "UDP") proto = pcppx::UDP;
			else
			{
				std::cerr << "protocol must be TCP or UDP\n";  // main.cpp's -P check
				return 1;
			}
		}
		else
		{
			usage(argv[0]);
			return 1;
		}
	}
	if (in.empty() || burst > (deviceWorker ? (size_t)UINT32_MAX : (size_t)UINT16_MAX))
	{
		usage(argv[0]);
		return 1;
	}
	try
	{
		const PacketMatchingEngine matchingEngine(sip.empty() ? pcppx::IPv4Address::Zero : pcppx::IPv4Address(sip),
		                                          dip.empty() ? pcppx::IPv4Address::Zero : pcppx::IPv4Address(dip),
		                                          sport, dport, proto);
		pcppx::Engine engine(0);
		if (!hostParser.empty())
		{
			const pcppx_host_parse_fn fn = loadHostParser(hostParser);
			pcppx::setHostParser(fn);  // the per-packet worker's Packets
			engine.setHostParser(fn);
		}
		pcppx::PcapFileReaderDevice reader(in);
		if (!reader.open())
		{
			std::cerr << "cannot open " << in << "\n";
			return 1;
		}
		std::unique_ptr<pcpp::PcapFileWriterDevice> pcapWriter;
		if (!out.empty())
		{
			pcapWriter = std::make_unique<pcpp::PcapFileWriterDevice>(out, reader.getLinkLayerType());
			if (!pcapWriter->open())
			{
				std::cerr << "Couldn't open pcap writer device\n";
				return 1;
			}
		}
		AppWorkerThread worker(engine, matchingEngine, burst ? burst : (deviceWorker ? 1u << 20 : 64));
		if (deviceWorker)
			worker.runOnDevice(reader, pcapWriter.get());
		else
			worker.run(&reader, pcapWriter.get());
		if (pcapWriter && pcapWriter->packetsNotWritten())
			std::cerr << pcapWriter->packetsNotWritten() << " matched packets not written: link type differs from the "
			          << "output file's\n";
		pcapWriter.reset();
		printStats(worker.getStats(), deviceWorker ? "GPU worker" : "Worker");
	}
	catch (const pcppx::Error& e)
	{
		std::cerr << e.what() << "\n";
		return 2;
	}
	return 0;
}
