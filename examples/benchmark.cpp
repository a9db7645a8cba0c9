// benchmark.cpp — the PcapPlusPlus benchmark application's packet mode
// (Examples/PcapPlusPlus-benchmark/benchmark.cpp:60-115) on the engine.
//
//   benchmark <input-file> packet <repetitions>
//
// Each repetition reads the whole capture and parses every packet until TCP (Packet(&raw, pcpp::TCP),
// benchmark.cpp:91) and counts it (handle_packet, :54-58); the output line is the reference's:
// "<packets per run> <average ms per run>". The parse runs on the GPU in batches of up to 1M packets.
// The reference's dns mode needs DnsLayer (L7, out of this path's scope) and is not offered.
#include <chrono>
#include <cstdlib>
#include <iostream>
#include <numeric>
#include <string>
#include <vector>

#include "pcppx.hpp"

int main(int argc, char* argv[])
{
	if (argc != 4)
	{
		std::cout << "Usage: " << *argv << " <input-file> <packet> <repetitions>\n";
		return 1;
	}
	const std::string input_type(argv[2]);
	if (input_type != "packet")
	{
		std::cerr << "only packet mode is supported (dns mode parses L7)\n";
		return 1;
	}
	const int total_runs = std::stoi(argv[3]);
	size_t total_packets = 0;
	std::vector<std::chrono::high_resolution_clock::duration> durations;
	try
	{
		pcppx::Engine engine(0);
		pcppx::PacketParseOptions options(pcppx::TCP);
		options.computeChecksums = false;  // Packet(&raw, TCP) parses layers only
		options.maxLayers = 8;
		pcppx::RawBatch batch;
		for (int i = 0; i < total_runs; ++i)
		{
			size_t count = 0;
			pcppx::PcapFileReaderDevice reader(argv[1]);
			if (!reader.open())
			{
				std::cerr << "cannot open " << argv[1] << "\n";
				return 1;
			}
			const auto start = std::chrono::high_resolution_clock::now();
			while (reader.getNextPackets(batch, 1u << 20) > 0)
			{
				pcppx::ParsedBatch parsed = engine.parse(batch, options);
				count += parsed.size();  // handle_packet: count++
			}
			const auto end = std::chrono::high_resolution_clock::now();
			durations.push_back(end - start);
			total_packets += count;
			reader.close();
		}
	}
	catch (const pcppx::Error& e)
	{
		std::cerr << e.what() << "\n";
		return 2;
	}
	const auto total_time =
	    std::accumulate(durations.begin(), durations.end(), std::chrono::high_resolution_clock::duration(0));
	using std::chrono::duration_cast;
	using std::chrono::milliseconds;
	const auto total_time_in_ms = duration_cast<milliseconds>(total_time).count();
	std::cout << (total_packets / total_runs) << " " << (total_time_in_ms / durations.size()) << std::endl;
	return 0;
}
