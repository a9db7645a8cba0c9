/* benchmark_google — the reference's Google-benchmark parse benchmarks (Examples/PcapPlusPlus-benchmark/
 * benchmark-google.cpp: BM_FileRead, BM_PacketParsing, BM_PacketPureParsing) over the engine's Packet++-shaped facade.
 * The loops are the reference's token for token (benchmark_google_loops.inc; tests/test_facade.py checks them against
 * the reference); the namespace alias is the only change. oracle/ref_benchmark_google.cpp compiles the same loops
 * against the reference Packet++ built from source.
 *
 *   benchmark_google --pcap-file <file> [--pcap-file ...] [--min-time S] [--iterations N] [--repetitions R]
 *                    [--benchmark BM_PacketPureParsing]
 */
#include "pcppx.hpp"

namespace pcpp = pcppx;

#include "benchmark_google_loops.inc"

int main(int argc, char** argv)
{
	try
	{
		const int rc = runBenchmarks(argc, argv, "engine");
		const uint64_t pk = pcppx::detail::Service::packetsParsed(), by = pcppx::detail::Service::recordBytes();
		std::printf("{\"impl\": \"engine\", \"gpu_parses\": %llu, \"packets_parsed\": %llu, \"record_bytes\": %llu, "
		            "\"record_bytes_per_packet\": %.2f}\n",
		            (unsigned long long)pcppx::detail::Service::parsesSoFar(), (unsigned long long)pk, (unsigned long long)by,
		            pk ? (double)by / (double)pk : 0.0);
		return rc;
	}
	catch (const pcppx::Error& e)
	{
		std::fprintf(stderr, "%s\n", e.what());
		return 6;
	}
}
