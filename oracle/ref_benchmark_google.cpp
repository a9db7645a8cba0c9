/* ref_benchmark_google — TEST INFRASTRUCTURE (the CPU figure beside examples/benchmark_google): the same loops
 * (examples/benchmark_google_loops.inc: the reference's BM_FileRead / BM_PacketParsing / BM_PacketPureParsing bodies,
 * Examples/PcapPlusPlus-benchmark/benchmark-google.cpp:15-64,149-264) compiled against the reference Packet++ and Pcap++
 * file devices built from source under /root/reference (oracle/Makefile). One core. */
#include <Packet.h>
#include <PcapFileDevice.h>

#include "../examples/benchmark_google_loops.inc"

int main(int argc, char** argv)
{
	return runBenchmarks(argc, argv, "reference");
}
