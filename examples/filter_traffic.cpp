// filter_traffic.cpp — DpdkExample-FilterTraffic's worker (AppWorkerThread.h:85-139) over a pcap file, on
// the GPU. Packets are matched with PacketMatchingEngine's criteria (PacketMatchingEngine.h:43-107); once
// a packet of a 5-tuple flow matches, every later packet of that flow matches too (the worker's flow table
// keyed by hash5Tuple). Matched packets are written to an output pcap (the worker's
// writeMatchedPacketsToFile, AppWorkerThread.h:68-75,127-131); the statistics are printed as
// main.cpp:244-264 prints them. The input file replaces the DPDK RX queues.
//
//   filter_traffic -f in.pcap [-o out.pcap] [-s SRC_IP] [-d DST_IP] [-S SRC_PORT] [-D DST_PORT] [-P TCP|UDP]
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iomanip>
#include <iostream>
#include <string>
#include <vector>

#include "pcppx.hpp"

namespace
{
void usage(const char* argv0)
{
	std::cout << "Usage: " << argv0
	          << " -f <in.pcap> [-o <out.pcap>] [-s <src ip>] [-d <dst ip>] [-S <src port>] [-D <dst port>]"
	             " [-P <TCP|UDP>]\n";
}

void row(const std::string& name, uint64_t v)
{
	std::cout << "| " << std::left << std::setw(22) << name << "| " << std::right << std::setw(12) << v << " |\n";
}

// PacketStats table (main.cpp:244-264). HTTP/DNS/TLS are L7 and counted by the host for packets flagged
// PCPPX_F_NEEDS_HOST_L7; this tool reports the flagged count instead.
void printStats(const pcppx_packet_stats& s)
{
	std::cout << "+------------------------------------------+\n";
	row("Eth count", s.eth_count);
	row("ARP count", s.arp_count);
	row("IPv4 count", s.ipv4_count);
	row("IPv6 count", s.ipv6_count);
	row("TCP count", s.tcp_count);
	row("UDP count", s.udp_count);
	row("left to host", s.needs_host_count);
	row("Matched TCP flows", s.matched_tcp_flows);
	row("Matched UDP flows", s.matched_udp_flows);
	row("Total packet count", s.packet_count);
	row("Matched packet count", s.matched_packets);
	std::cout << "+------------------------------------------+\n";
}

struct PcapWriter
{
	FILE* f = nullptr;
	bool open(const std::string& path, uint32_t linktype)
	{
		f = std::fopen(path.c_str(), "wb");
		if (f == nullptr)
			return false;
		const uint32_t magic = 0xa1b2c3d4, snap = 262144;
		const uint16_t vmaj = 2, vmin = 4;
		const int32_t zone = 0;
		const uint32_t sig = 0;
		std::fwrite(&magic, 4, 1, f);
		std::fwrite(&vmaj, 2, 1, f);
		std::fwrite(&vmin, 2, 1, f);
		std::fwrite(&zone, 4, 1, f);
		std::fwrite(&sig, 4, 1, f);
		std::fwrite(&snap, 4, 1, f);
		std::fwrite(&linktype, 4, 1, f);
		return true;
	}
	void write(const pcppx::RawBatch& b, size_t i)
	{
		const uint64_t ts = b.timestampsNs[i];
		const uint32_t h[4] = { (uint32_t)(ts / 1000000000ull), (uint32_t)(ts % 1000000000ull / 1000ull), b.caplens[i],
			                    b.caplens[i] };
		std::fwrite(h, 4, 4, f);
		std::fwrite(b.packetData(i), 1, b.caplens[i], f);
	}
	~PcapWriter()
	{
		if (f)
			std::fclose(f);
	}
};
}  // namespace

int main(int argc, char* argv[])
{
	std::string in, out, sip, dip;
	uint16_t sport = 0, dport = 0;
	pcppx::ProtocolType proto = pcppx::UnknownProtocol;
	for (int k = 1; k < argc; ++k)
	{
		const std::string a = argv[k];
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
	if (in.empty())
	{
		usage(argv[0]);
		return 1;
	}
	try
	{
		const pcppx::MatchSpec spec(sip, dip, sport, dport, proto);
		pcppx::Engine engine(0);
		engine.resetFilter();
		pcppx::PcapFileReaderDevice reader(in);
		if (!reader.open())
		{
			std::cerr << "cannot open " << in << "\n";
			return 1;
		}
		PcapWriter writer;
		if (!out.empty() && !writer.open(out, reader.getLinkLayerType()))
		{
			std::cerr << "cannot create " << out << "\n";
			return 1;
		}
		pcppx::RawBatch batch;
		std::vector<uint8_t> matched;
		pcppx_packet_stats stats{};
		while (reader.getNextPackets(batch, 1u << 20) > 0)
		{
			stats = engine.filter(batch, spec, matched);
			if (writer.f)
				for (size_t i = 0; i < batch.size(); ++i)
					if (matched[i])
						writer.write(batch, i);
		}
		printStats(stats);
	}
	catch (const pcppx::Error& e)
	{
		std::cerr << e.what() << "\n";
		return 2;
	}
	return 0;
}
