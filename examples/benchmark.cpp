/**
 * PcapPlusPlus benchmark application on the GPU parse engine
 * ==========================================================
 * The reference application (Examples/PcapPlusPlus-benchmark/benchmark.cpp:60-109) over the engine's facade
 * (include/pcppx.hpp) instead of Packet++ / Pcap++: `namespace pcpp = pcppx`, and the packet loop is the reference's
 * token for token -- reader.getNextPacket(rawPacket) hands out packets of pages the reader has already parsed on the
 * GPU (the batch prepass runs inside the library, ahead of the loop), and Packet(&rawPacket, pcpp::TCP) binds to
 * that packet's records.
 *
 *   benchmark <input-file> <dns|packet> <repetitions> [--host-parser <lib.so>] [--dump]
 *
 * Output: "<packets per run> <average ms per run>", as the reference. Two engine-side options, taken off the command
 * line before the reference's argument check: --host-parser names a library exporting `pcppx_host_parse`
 * (include/pcppx.h, pcppx_host_parse_fn): the caller's own Packet++ parse, which completes the packets the engine
 * leaves to the host (an L7 layer it does not dissect); --dump prints every packet's layer list and hash5Tuple in the
 * first run (the tests compare them with the reference). The dns mode iterates DnsLayer's queries and answers, an L7
 * dissector the engine does not build: it is refused.
 */
#include <dlfcn.h>

#include <cinttypes>
#include <cstdio>
#include <iostream>
#include <chrono>
#include <string>
#include <vector>
#include <numeric>

#include "pcppx.hpp"

namespace pcpp = pcppx;
using namespace pcpp;

size_t count = 0;

namespace
{
bool dumpPackets = false;

// --dump: "<index> <n_layers> <proto>:<offset>:<hdr_len>:<data_len> ... h5=<hash5Tuple> h5d=<dir> h2=<hash2Tuple>"
void dump(size_t index, const Packet& packet)
{
	std::printf("%zu %zu", index, packet.getLayerCount());
	for (size_t k = 0; k < packet.getRecordedLayerCount(); ++k)
	{
		const Layer l = packet.getLayer(k);
		std::printf(" %u:%u:%zu:%zu", l.getProtocol(), l.getOffset(), l.getHeaderLen(), l.getDataLen());
	}
	std::printf(" h5=%" PRIu32 " h5d=%" PRIu32 " h2=%" PRIu32 " host=%d\n", hash5Tuple(&packet),
	            hash5Tuple(&packet, true), hash2Tuple(&packet), packet.wasHostParsed() ? 1 : 0);
}

pcppx_host_parse_fn loadHostParser(const std::string& path)
{
	void* lib = dlopen(path.c_str(), RTLD_NOW | RTLD_LOCAL);
	if (lib == nullptr)
		throw Error(PCPPX_E_INVAL, std::string("dlopen: ") + dlerror());
	auto fn = reinterpret_cast<pcppx_host_parse_fn>(dlsym(lib, "pcppx_host_parse"));
	if (fn == nullptr)
		throw Error(PCPPX_E_INVAL, path + " does not export pcppx_host_parse");
	return fn;
}

// take the engine-side options off argv; false on a malformed one
bool engineOptions(int& argc, char* argv[])
{
	int out = 1;
	for (int k = 1; k < argc; ++k)
	{
		const std::string a = argv[k];
		if (a == "--dump")
			dumpPackets = true;
		else if (a == "--host-parser")
		{
			if (k + 1 >= argc)
				return false;
			setHostParser(loadHostParser(argv[++k]));
		}
		else
			argv[out++] = argv[k];
	}
	argc = out;
	return true;
}
}  // namespace

bool handle_packet(Packet& packet)
{
	if (dumpPackets)
		dump(count, packet);
	count++;
	return true;
}

int main(int argc, char* argv[])
{
	try
	{
		if (!engineOptions(argc, argv))
		{
			std::cout << "Usage: " << *argv << " <input-file> <dns|packet> <repetitions> [--host-parser <lib.so>] [--dump]\n";
			return 1;
		}
		if (argc != 4)
		{
			std::cout << "Usage: " << *argv << " <input-file> <dns|packet> <repetitions>\n";
			return 1;
		}
		std::string input_type(argv[2]);
		if (input_type == "dns")
		{
			// dns mode walks DnsLayer's queries and answers (benchmark.cpp:30-52): an L7 dissector, left to Packet++
			std::cerr << "only packet mode runs on the engine: dns mode iterates DnsLayer resources (L7)\n";
			return 1;
		}
		int total_runs = std::stoi(argv[3]);
		size_t total_packets = 0;
		std::vector<std::chrono::high_resolution_clock::duration> durations;
		for (int i = 0; i < total_runs; ++i)
		{
			count = 0;
			PcapFileReaderDevice reader(argv[1]);
			reader.open();
			std::chrono::high_resolution_clock::time_point start;
			{
				start = std::chrono::high_resolution_clock::now();
				RawPacket rawPacket;
				while (reader.getNextPacket(rawPacket))
				{
					Packet packet(&rawPacket, pcpp::TCP);
					handle_packet(packet);
				}
			}
			auto end = std::chrono::high_resolution_clock::now();
			durations.push_back(end - start);
			total_packets += count;
			reader.close();
			dumpPackets = false;
		}
		auto total_time =
		    std::accumulate(durations.begin(), durations.end(), std::chrono::high_resolution_clock::duration(0));

		using std::chrono::duration_cast;
		using std::chrono::milliseconds;
		auto total_time_in_ms = duration_cast<milliseconds>(total_time).count();
		std::cout << (total_packets / total_runs) << " " << (total_time_in_ms / durations.size()) << std::endl;
	}
	catch (const Error& e)
	{
		std::cerr << e.what() << "\n";
		return 2;
	}
	return 0;
}
