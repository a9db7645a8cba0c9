/**
 * PcapPlusPlus benchmark application on the GPU parse engine
 * ==========================================================
 * The reference application (Examples/PcapPlusPlus-benchmark/benchmark.cpp:60-109), with one change: instead of
 * reading one RawPacket and building one Packet at a time, the reader fills a batch (getNextPackets, the reference's
 * IFileReaderDevice batch read) and the engine parses the whole batch on the GPU (the batch prepass); the next
 * batch is read by a reader thread meanwhile. The per-packet handler then runs over Packet views with
 * pcpp::Packet's names, as before.
 *
 *   benchmark <input-file> packet <repetitions> [--host-parser <lib.so>] [--dump]
 *
 * Output: "<packets per run> <average ms per run>", as the reference. The reference's dns mode iterates DnsLayer's
 * queries and answers, an L7 dissector outside the engine: it is refused. Packets the engine leaves to the host
 * (an L7 layer it does not dissect) are completed by the caller's own Packet++ parse when --host-parser names a
 * library exporting `pcppx_host_parse` (include/pcppx.h, pcppx_host_parse_fn). --dump also prints every
 * packet's layer list and hash5Tuple (used by the tests to compare with the reference).
 */
#include <dlfcn.h>

#include <chrono>
#include <cinttypes>
#include <cstdio>
#include <future>
#include <iostream>
#include <numeric>
#include <string>
#include <vector>

#include "pcppx.hpp"

using namespace pcppx;

size_t count = 0;

bool handle_packet(Packet& packet)
{
	(void)packet;
	count++;
	return true;
}

namespace
{
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
}  // namespace

int main(int argc, char* argv[])
{
	if (argc < 4)
	{
		std::cout << "Usage: " << *argv << " <input-file> packet <repetitions> [--host-parser <lib.so>] [--dump]\n";
		return 1;
	}
	std::string input_type(argv[2]);
	if (input_type != "packet")
	{
		// dns mode walks DnsLayer's queries and answers (benchmark.cpp:30-52): an L7 dissector, left to Packet++
		std::cerr << "only packet mode runs on the engine: dns mode iterates DnsLayer resources (L7)\n";
		return 1;
	}
	int total_runs = std::stoi(argv[3]);
	std::string hostParser;
	bool dumpPackets = false;
	for (int k = 4; k < argc; ++k)
	{
		const std::string a = argv[k];
		if (a == "--host-parser" && k + 1 < argc)
			hostParser = argv[++k];
		else if (a == "--dump")
			dumpPackets = true;
		else
		{
			std::cout << "Usage: " << *argv << " <input-file> packet <repetitions> [--host-parser <lib.so>] [--dump]\n";
			return 1;
		}
	}
	size_t total_packets = 0;
	std::vector<std::chrono::high_resolution_clock::duration> durations;
	try
	{
		Engine engine(0);
		if (!hostParser.empty())
			engine.setHostParser(loadHostParser(hostParser));
		RawPacketVector bufs[2];  // batch k is parsed while batch k+1 is read (a reader thread; distinct buffers)
		for (int i = 0; i < total_runs; ++i)
		{
			count = 0;
			size_t index = 0;
			PcapFileReaderDevice reader(argv[1]);
			reader.open();
			std::chrono::high_resolution_clock::time_point start;
			{
				start = std::chrono::high_resolution_clock::now();
				PacketParseOptions options(TCP);  // Packet(&rawPacket, pcpp::TCP)
				options.computeChecksums = false;
				int cur = 0;
				auto next = std::async(std::launch::async, [&] { return reader.getNextPackets(bufs[0], 1 << 20); });
				while (next.get() > 0)
				{
					next = std::async(std::launch::async,
					                  [&, k = cur ^ 1] { return reader.getNextPackets(bufs[k], 1 << 20); });
					ParsedBatch parsed = engine.parse(bufs[cur], options);  // the batch prepass
					for (Packet packet : parsed)
					{
						handle_packet(packet);
						if (dumpPackets && i == 0)
							dump(index, packet);
						++index;
					}
					cur ^= 1;
				}
			}
			auto end = std::chrono::high_resolution_clock::now();
			durations.push_back(end - start);
			total_packets += count;
			reader.close();
		}
	}
	catch (const Error& e)
	{
		std::cerr << e.what() << "\n";
		return 2;
	}
	auto total_time =
	    std::accumulate(durations.begin(), durations.end(), std::chrono::high_resolution_clock::duration(0));

	using std::chrono::duration_cast;
	using std::chrono::milliseconds;
	auto total_time_in_ms = duration_cast<milliseconds>(total_time).count();
	std::cout << (total_packets / total_runs) << " " << (total_time_in_ms / durations.size()) << std::endl;
	return 0;
}
