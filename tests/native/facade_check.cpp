/* facade_check — test driver for the per-packet entry points of include/pcppx.hpp (tests/test_facade.py).
 *
 *   facade_check read <packet|burst:N|batch:N> <outdir> <capture>...
 *       reads every capture through PcapFileReaderDevice::getNextPacket, receivePackets (bursts of N) or
 *       getNextPackets (batches of N) and writes <outdir>/<k>.bin: per packet u32 caplen, u32 frame length,
 *       u64 timestamp (ns), u32 link type, then the bytes; a file holding "NOOPEN" when open() fails.  (CPU only.)
 *   facade_check parse <capture> <outfile> <plan>
 *       reads the capture with getNextPacket and builds, per packet, the Packets the plan names (a comma-separated
 *       list of variants, applied to packet i in turn: full | tcp | ip | osi2 | osi3 | osi4 | own | copy | free);
 *       writes per packet and variant the pcppx_summary (32 B) and the PCPPX_MAX_LAYERS layer records the Packet
 *       holds (zero past its chain).  (GPU.)
 *   facade_check parsevec <capture> <outfile> <plan> <reader|own|copy>
 *       the RawPacketVector forms (Examples/PcapPlusPlus-benchmark/benchmark-google.cpp:231-260): reader =
 *       IFileReaderDevice::tryCreateReader + getNextPackets(vector) and Packet(vector.at(i), ...) per packet; own = the
 *       caller's own RawPackets (heap copies of the bytes, takeOwnership) pushed into a RawPacketVector, then the
 *       Packets; copy = a copy of the reader's vector (PointerVector's deep copy: every RawPacket copied, records
 *       with it). Writes the records as `parse` does; prints {"gpu_parses": N} (pcppx_parse_batch_host calls the
 *       per-packet entry points made).  (GPU.)
 *   facade_check retain <capture> <every>
 *       getNextPacket + Packet(&raw) over the capture, keeping a copy of every <every>-th RawPacket (and building a
 *       Packet on each copy after the reader is closed); prints {"kept", "pinned_while_reading", "pinned_after"}: the
 *       page-locked record bytes held by live pages -- copies own their bytes and records, so none after.  (GPU.)
 *   facade_check create <file>
 *       IFileReaderDevice::tryCreateReader: prints "null", "noopen" or "packets N" (getNextPacket to the end).  (CPU.)
 *   facade_check time <capture> <reps>
 *       the phases of the reference benchmark's packet loop (open, first getNextPacket, first Packet(&raw, TCP), the
 *       rest of the loop, close), averaged over reps after one untimed run; one JSON line, microseconds.  (GPU.)
 *   env PCPPX_CHECK_HOST_PARSER=<lib.so>: register that library's pcppx_host_parse with setHostParser.
 *   env PCPPX_CHECK_PAGE_CHECKSUMS=1: setPageChecksums(true) (the records then carry the checksum verdicts and values).
 */
#include <dlfcn.h>

#include <chrono>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "pcppx.hpp"

namespace
{
void put(std::FILE* f, const void* p, size_t n)
{
	if (n && std::fwrite(p, 1, n, f) != n)
	{
		std::perror("fwrite");
		std::exit(3);
	}
}

void putRaw(std::FILE* f, const pcppx::RawPacket& r)
{
	const uint32_t cap = (uint32_t)r.getRawDataLen(), flen = (uint32_t)r.getFrameLength(), lt = r.getLinkLayerType();
	const timespec ts = r.getPacketTimeStamp();
	const uint64_t tns = (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
	put(f, &cap, 4);
	put(f, &flen, 4);
	put(f, &tns, 8);
	put(f, &lt, 4);
	put(f, r.getRawData(), cap);
}

int readMode(const std::string& mode, const std::string& outdir, int nfiles, char** files)
{
	for (int k = 0; k < nfiles; ++k)
	{
		const std::string out = outdir + "/" + std::to_string(k) + ".bin";
		std::FILE* f = std::fopen(out.c_str(), "wb");
		if (f == nullptr)
			return 2;
		pcppx::PcapFileReaderDevice reader(files[k]);
		if (!reader.open())
		{
			put(f, "NOOPEN", 6);
			std::fclose(f);
			continue;
		}
		if (mode == "packet")
		{
			pcppx::RawPacket raw;
			while (reader.getNextPacket(raw))
				putRaw(f, raw);
		}
		else if (mode.rfind("burst:", 0) == 0)
		{
			const int n = std::atoi(mode.c_str() + 6);
			std::vector<pcppx::RawPacket*> arr((size_t)n, nullptr);
			for (;;)
			{
				const uint16_t got = reader.receivePackets(arr.data(), (uint16_t)n, 0);
				if (got == 0)
					break;
				for (uint16_t i = 0; i < got; ++i)
					putRaw(f, *arr[i]);
			}
			for (auto* p : arr)
				delete p;
		}
		else if (mode == "vector" || mode.rfind("vector:", 0) == 0)
		{
			// getNextPackets(RawPacketVector&) appends page-bound RawPackets: all at once, or N per call
			const int n = mode == "vector" ? -1 : std::atoi(mode.c_str() + 7);
			pcppx::RawPacketVector v;
			while (reader.getNextPackets(v, n) > 0 && n > 0)
			{
			}
			for (pcppx::RawPacket* p : v)
				putRaw(f, *p);
		}
		else if (mode.rfind("batch:", 0) == 0)
		{
			const int n = std::atoi(mode.c_str() + 6);
			pcppx::RawBatch b;
			while (reader.getNextBatch(b, n) > 0)
				for (size_t i = 0; i < b.size(); ++i)
				{
					const uint64_t t = b.timestampsNs[i];
					pcppx::RawPacket raw;
					raw.setRawData(b.packetData(i), (int)b.caplens[i], false,
					               timespec{ (time_t)(t / 1000000000ull), (long)(t % 1000000000ull) }, b.linkType,
					               (int)b.frameLens[i]);
					putRaw(f, raw);
				}
		}
		else
			return 1;
		reader.close();
		std::fclose(f);
	}
	return 0;
}

void putPacket(std::FILE* f, const pcppx::Packet& p)
{
	put(f, &p.summary(), sizeof(pcppx_summary));
	pcppx_layer lay[PCPPX_MAX_LAYERS];
	std::memset(lay, 0, sizeof(lay));
	for (size_t k = 0; k < p.getRecordedLayerCount() && k < PCPPX_MAX_LAYERS; ++k)
	{
		const pcppx::Layer l = p.getLayer(k);
		lay[k] = pcppx_layer{ l.getProtocol(), (uint8_t)l.getOsiModelLayer(), l.getOffset(), (uint16_t)l.getHeaderLen(),
			                  (uint16_t)l.getDataLen() };
	}
	put(f, lay, sizeof(lay));
}

int parseMode(const char* capture, const char* outfile, const std::string& plan)
{
	std::vector<std::string> variants;
	for (size_t a = 0; a <= plan.size();)
	{
		size_t b = plan.find(',', a);
		if (b == std::string::npos)
			b = plan.size();
		variants.push_back(plan.substr(a, b - a));
		a = b + 1;
	}
	std::FILE* f = std::fopen(outfile, "wb");
	if (f == nullptr)
		return 2;
	pcppx::PcapFileReaderDevice reader(capture);
	if (!reader.open())
		return 4;
	pcppx::RawPacket raw;
	size_t i = 0;
	while (reader.getNextPacket(raw))
	{
		const std::string& v = variants[i % variants.size()];
		if (v == "full")
			putPacket(f, pcppx::Packet(&raw));
		else if (v == "tcp")
			putPacket(f, pcppx::Packet(&raw, pcppx::TCP));
		else if (v == "ip")
			putPacket(f, pcppx::Packet(&raw, pcppx::IP));
		else if (v == "osi3")
			putPacket(f, pcppx::Packet(&raw, pcppx::OsiModelNetworkLayer));
		else if (v == "osi2")
			putPacket(f, pcppx::Packet(&raw, pcppx::OsiModelDataLinkLayer));
		else if (v == "osi4")
			putPacket(f, pcppx::Packet(&raw, false, pcppx::UnknownProtocol, pcppx::OsiModelTransportLayer));
		else if (v == "own")  // the caller's own bytes: a one-packet batch
		{
			pcppx::RawPacket mine(raw.getRawData(), raw.getRawDataLen(), timespec{ 0, 0 }, false, raw.getLinkLayerType());
			putPacket(f, pcppx::Packet(&mine));
		}
		else if (v == "copy")  // a copy shares the page
		{
			pcppx::RawPacket c(raw);
			putPacket(f, pcppx::Packet(&c, pcppx::TCP));
		}
		else if (v == "free")  // freeRawPacket: the Packet deletes a heap copy of the caller's bytes
		{
			uint8_t* bytes = new uint8_t[raw.getRawDataLen() > 0 ? raw.getRawDataLen() : 1];
			std::memcpy(bytes, raw.getRawData(), (size_t)raw.getRawDataLen());
			auto* heap = new pcppx::RawPacket(bytes, raw.getRawDataLen(), timespec{ 0, 0 }, true, raw.getLinkLayerType());
			putPacket(f, pcppx::Packet(heap, true));
		}
		else
			return 1;
		++i;
	}
	std::fclose(f);
	return 0;
}
void putVariant(std::FILE* f, pcppx::RawPacket* raw, const std::string& v)
{
	if (v == "full")
		putPacket(f, pcppx::Packet(raw));
	else if (v == "tcp")
		putPacket(f, pcppx::Packet(raw, pcppx::TCP));
	else if (v == "ip")
		putPacket(f, pcppx::Packet(raw, pcppx::IP));
	else if (v == "osi3")
		putPacket(f, pcppx::Packet(raw, pcppx::OsiModelNetworkLayer));
	else if (v == "osi2")
		putPacket(f, pcppx::Packet(raw, pcppx::OsiModelDataLinkLayer));
	else if (v == "osi4")
		putPacket(f, pcppx::Packet(raw, false, pcppx::UnknownProtocol, pcppx::OsiModelTransportLayer));
	else
		throw std::runtime_error("variant " + v);
}

int parseVecMode(const char* capture, const char* outfile, const std::string& plan, const std::string& how)
{
	std::vector<std::string> variants;
	for (size_t a = 0; a <= plan.size();)
	{
		size_t b = plan.find(',', a);
		if (b == std::string::npos)
			b = plan.size();
		variants.push_back(plan.substr(a, b - a));
		a = b + 1;
	}
	auto reader = pcppx::IFileReaderDevice::tryCreateReader(capture);
	if (reader == nullptr || !reader->open())
		return 4;
	pcppx::RawPacketVector rawPackets;
	reader->getNextPackets(rawPackets);
	pcppx::RawPacketVector other;
	pcppx::RawPacketVector* use = &rawPackets;
	if (how == "own")
	{
		for (pcppx::RawPacket* p : rawPackets)
		{
			const int len = p->getRawDataLen();
			uint8_t* bytes = new uint8_t[len > 0 ? len : 1];
			std::memcpy(bytes, p->getRawData(), (size_t)(len > 0 ? len : 0));
			other.pushBack(new pcppx::RawPacket(bytes, len, p->getPacketTimeStamp(), true, p->getLinkLayerType()));
		}
		rawPackets.clear();  // the reader's pages go: only the caller's own bytes remain
		use = &other;
	}
	else if (how == "copy")
	{
		// build the first Packet on the reader's vector (its first page parsed), then copy the whole vector
		{
			pcppx::Packet first(rawPackets.at(0));
			(void)first;
		}
		other = rawPackets;
		rawPackets.clear();
		use = &other;
	}
	else if (how != "reader")
		return 1;
	std::FILE* f = std::fopen(outfile, "wb");
	if (f == nullptr)
		return 2;
	for (size_t i = 0; i < use->size(); ++i)
		putVariant(f, use->at((int)i), variants[i % variants.size()]);
	std::fclose(f);
	std::printf("{\"packets\": %zu, \"gpu_parses\": %llu}\n", use->size(),
	            (unsigned long long)pcppx::detail::Service::instance().parses());
	return 0;
}

int timeMode(const char* capture, int reps)
{
	using clk = std::chrono::steady_clock;
	double acc[6] = { 0, 0, 0, 0, 0, 0 };
	size_t packets = 0;
	for (int r = 0; r <= reps; ++r)
	{
		clk::time_point t0, t1, t2, t3, t4, t5;
		size_t n = 0, tcp = 0;
		{
			t0 = clk::now();
			pcppx::PcapFileReaderDevice reader(capture);
			if (!reader.open())
				return 4;
			t1 = clk::now();
			pcppx::RawPacket raw;
			t2 = t3 = t1;
			if (reader.getNextPacket(raw))
			{
				t2 = clk::now();
				{
					pcppx::Packet p(&raw, pcppx::TCP);
					tcp += p.isPacketOfType(pcppx::TCP) ? 1 : 0;
				}
				t3 = clk::now();
				++n;
				while (reader.getNextPacket(raw))
				{
					pcppx::Packet p(&raw, pcppx::TCP);
					tcp += p.isPacketOfType(pcppx::TCP) ? 1 : 0;
					++n;
				}
			}
			t4 = clk::now();
			reader.close();
			t5 = clk::now();
		}  // the RawPacket and the reader go out of scope
		const auto t6 = clk::now();
		if (r == 0)
			continue;  // untimed: HIP initialisation, pinned pools
		packets = n;
		const double d[6] = { std::chrono::duration<double, std::micro>(t1 - t0).count(),
			                  std::chrono::duration<double, std::micro>(t2 - t1).count(),
			                  std::chrono::duration<double, std::micro>(t3 - t2).count(),
			                  std::chrono::duration<double, std::micro>(t4 - t3).count(),
			                  std::chrono::duration<double, std::micro>(t5 - t4).count(),
			                  std::chrono::duration<double, std::micro>(t6 - t5).count() };
		for (int k = 0; k < 6; ++k)
			acc[k] += d[k];
	}
	std::printf("{\"packets\": %zu, \"reps\": %d, \"open_us\": %.1f, \"first_packet_us\": %.1f, \"first_parse_us\": %.1f, "
	            "\"loop_us\": %.1f, \"close_us\": %.1f, \"destroy_us\": %.1f}\n",
	            packets, reps, acc[0] / reps, acc[1] / reps, acc[2] / reps, acc[3] / reps, acc[4] / reps, acc[5] / reps);
	return 0;
}
}  // namespace

int main(int argc, char** argv)
{
	try
	{
		if (std::getenv("PCPPX_CHECK_PAGE_CHECKSUMS") != nullptr)
			pcppx::setPageChecksums(true);
		if (const char* lib = std::getenv("PCPPX_CHECK_HOST_PARSER"))
		{
			void* h = dlopen(lib, RTLD_NOW | RTLD_LOCAL);
			auto fn = h ? reinterpret_cast<pcppx_host_parse_fn>(dlsym(h, "pcppx_host_parse")) : nullptr;
			if (fn == nullptr)
				return 5;
			pcppx::setHostParser(fn);
		}
		if (argc >= 4 && std::string(argv[1]) == "read")
			return readMode(argv[2], argv[3], argc - 4, argv + 4);
		if (argc == 4 && std::string(argv[1]) == "time")
			return timeMode(argv[2], std::atoi(argv[3]));
		if (argc == 4 && std::string(argv[1]) == "retain")
		{
			std::vector<pcppx::RawPacket> kept;
			size_t peak = 0, i = 0;
			{
				pcppx::PcapFileReaderDevice reader(argv[2]);
				if (!reader.open())
					return 4;
				const size_t every = (size_t)std::atoll(argv[3]);
				pcppx::RawPacket raw;
				while (reader.getNextPacket(raw))
				{
					pcppx::Packet p(&raw);
					(void)p;
					if (i++ % every == 0)
						kept.push_back(raw);
					const size_t out = pcppx::detail::PinnedPool::instance().outstanding();
					peak = out > peak ? out : peak;
				}
				raw.clear();
				reader.close();
			}
			uint64_t h = 0;
			for (pcppx::RawPacket& k : kept)
			{
				pcppx::Packet p(&k);
				h += pcppx::hash5Tuple(&p);
			}
			std::printf("{\"kept\": %zu, \"pinned_while_reading\": %zu, \"pinned_after\": %zu, \"h\": %llu}\n",
			            kept.size(), peak, pcppx::detail::PinnedPool::instance().outstanding(), (unsigned long long)h);
			return 0;
		}
		if (argc == 3 && std::string(argv[1]) == "create")
		{
			auto reader = pcppx::IFileReaderDevice::tryCreateReader(argv[2]);
			if (reader == nullptr)
			{
				std::printf("null\n");
				return 0;
			}
			if (!reader->open())
			{
				std::printf("noopen\n");
				return 0;
			}
			pcppx::RawPacket raw;
			size_t n = 0;
			while (reader->getNextPacket(raw))
				++n;
			std::printf("packets %zu\n", n);
			return 0;
		}
		if (argc == 6 && std::string(argv[1]) == "parsevec")
			return parseVecMode(argv[2], argv[3], argv[4], argv[5]);
		if (argc == 5 && std::string(argv[1]) == "parse")
			return parseMode(argv[2], argv[3], argv[4]);
	}
	catch (const pcppx::Error& e)
	{
		std::fprintf(stderr, "%s\n", e.what());
		return 6;
	}
	catch (const std::exception& e)
	{
		std::fprintf(stderr, "%s\n", e.what());
		return 7;
	}
	std::fprintf(stderr, "usage: facade_check read <mode> <outdir> <capture>... | parse <capture> <out> <plan>\n");
	return 1;
}
