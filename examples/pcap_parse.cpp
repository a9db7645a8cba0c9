/**
 * pcap_parse — a capture file to parse records, end to end
 * ============================================================================
 * The file side of the reference's readers (IFileReaderDevice::getNextPackets, Pcap++/src/PcapFileDevice.cpp:770-792)
 * feeding Packet(&raw) for every packet, on the engine: the reader maps the capture and hands out batches that point
 * into the map (pcppx_pcap_map_batch: no per-packet copy); pcppx_parse_batch_host stages each batch to HBM in chunks
 * (the record headers between packets ride along), parses it on the GPU and returns the records into page-locked
 * arrays. A reader thread walks the next batch's record headers while the current batch is parsed.
 *
 *   pcap_parse <file> [--batch N] [--layers L] [--checksums 0|1] [--reps R] [--copy]
 *
 * --copy reads with pcppx_pcap_read_batch into page-locked buffers instead (one copy on the host, then DMA straight
 * from them). Prints one JSON line: packets, file and wire bytes, seconds (best of R), Mpackets/s, GB/s of file and
 * wire bytes, the reader's share, and a digest of the hash5 records (so the records are consumed).
 */
#include <chrono>
#include <cinttypes>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <future>
#include <string>
#include <sys/stat.h>
#include <vector>

#include "pcppx.hpp"

namespace
{
struct Pinned
{
	void* p = nullptr;
	explicit Pinned(size_t bytes) : p(pcppx_host_alloc(bytes))
	{
		if (p == nullptr)
			throw pcppx::Error(PCPPX_E_NOMEM, "pcppx_host_alloc");
	}
	~Pinned() { pcppx_host_free(p); }
	template <class T> T* as() const { return static_cast<T*>(p); }
};

struct Batch
{
	std::vector<uint64_t> offsets;
	std::vector<uint32_t> caplens;
	pcppx_batch b{};
	double read_s = 0;
	uint64_t wire = 0;
};

struct CopyBatch
{
	Pinned data, offsets, caplens;
	pcppx_batch b{};
	double read_s = 0;
	CopyBatch(size_t cap, uint32_t n) : data(cap), offsets(n * 8ull), caplens(n * 4ull) {}
};

double now()
{
	return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
}  // namespace

int main(int argc, char* argv[])
{
	if (argc < 2)
	{
		std::fprintf(stderr, "usage: %s <file> [--batch N] [--layers L] [--checksums 0|1] [--reps R] [--copy]\n", argv[0]);
		return 1;
	}
	const std::string path = argv[1];
	uint32_t batchN = 1u << 20;
	uint8_t layers = 8;
	bool csum = true, copyMode = false;
	int reps = 3;
	for (int k = 2; k < argc; ++k)
	{
		const std::string a = argv[k];
		if (a == "--copy")
			copyMode = true;
		else if (k + 1 < argc && a == "--batch")
			batchN = (uint32_t)std::atol(argv[++k]);
		else if (k + 1 < argc && a == "--layers")
			layers = (uint8_t)std::atoi(argv[++k]);
		else if (k + 1 < argc && a == "--checksums")
			csum = std::atoi(argv[++k]) != 0;
		else if (k + 1 < argc && a == "--reps")
			reps = std::atoi(argv[++k]);
		else
		{
			std::fprintf(stderr, "bad argument %s\n", a.c_str());
			return 1;
		}
	}
	struct stat st;
	if (stat(path.c_str(), &st) != 0)
	{
		std::fprintf(stderr, "cannot stat %s\n", path.c_str());
		return 1;
	}
	try
	{
		pcppx::Engine engine(0);
		pcppx_opts o;
		pcppx_default_opts(&o);
		o.want_checksums = csum ? 1 : 0;
		o.max_layers = layers;
		Pinned sum(batchN * sizeof(pcppx_summary)), lay((size_t)batchN * (layers ? layers : 1) * sizeof(pcppx_layer));
		pcppx_records rec{};
		rec.summary = sum.as<pcppx_summary>();
		rec.layers = layers ? lay.as<pcppx_layer>() : nullptr;
		double best = 1e30, best_read = 0;
		uint64_t packets = 0, wire = 0, digest = 0;
		for (int r = 0; r < reps; ++r)
		{
			const double t0 = now();
			pcppx_pcap* reader = nullptr;
			pcppx::check(pcppx_pcap_open(path.c_str(), &reader), "pcppx_pcap_open");
			uint64_t np = 0, nw = 0, dg = 0;
			double read_s = 0;
			if (!copyMode)
			{
				auto next = [&](Batch& bt) {
					const double r0 = now();
					bt.offsets.resize(batchN);
					bt.caplens.resize(batchN);
					const uint8_t* base = nullptr;
					uint64_t size = 0;
					uint32_t n = 0;
					pcppx::check(pcppx_pcap_map_batch(reader, &base, &size, bt.offsets.data(), bt.caplens.data(), nullptr,
					                                  nullptr, batchN, &n),
					             "pcppx_pcap_map_batch");
					bt.b = pcppx_batch{ base, bt.offsets.data(), bt.caplens.data(), size, n,
						                (uint16_t)pcppx_pcap_linktype(reader), 0 };
					bt.wire = 0;
					for (uint32_t i = 0; i < n; ++i)
						bt.wire += bt.caplens[i];
					bt.read_s = now() - r0;
				};
				Batch bufs[2];
				next(bufs[0]);
				for (int k = 0;; ++k)
				{
					Batch& cur = bufs[k & 1];
					if (cur.b.n == 0)
						break;
					auto fut = std::async(std::launch::async, next, std::ref(bufs[(k + 1) & 1]));
					pcppx::check(pcppx_parse_batch_host(engine.handle(), &cur.b, &o, &rec), "pcppx_parse_batch_host");
					for (uint32_t i = 0; i < cur.b.n; ++i)
						dg += rec.summary[i].hash5;
					np += cur.b.n;
					nw += cur.wire;
					read_s += cur.read_s;
					fut.get();
				}
			}
			else
			{
				const size_t cap = 512ull << 20;
				CopyBatch* bufs[2] = { new CopyBatch(cap, batchN), new CopyBatch(cap, batchN) };
				auto next = [&](CopyBatch& bt) {
					const double r0 = now();
					uint32_t n = 0;
					uint64_t used = 0;
					pcppx::check(pcppx_pcap_read_batch(reader, bt.data.as<uint8_t>(), cap, bt.offsets.as<uint64_t>(),
					                                   bt.caplens.as<uint32_t>(), nullptr, batchN, &n, &used),
					             "pcppx_pcap_read_batch");
					bt.b = pcppx_batch{ bt.data.as<uint8_t>(), bt.offsets.as<uint64_t>(), bt.caplens.as<uint32_t>(), used, n,
						                (uint16_t)pcppx_pcap_linktype(reader), 0 };
					bt.read_s = now() - r0;
				};
				next(*bufs[0]);
				for (int k = 0;; ++k)
				{
					CopyBatch& cur = *bufs[k & 1];
					if (cur.b.n == 0)
						break;
					auto fut = std::async(std::launch::async, next, std::ref(*bufs[(k + 1) & 1]));
					pcppx::check(pcppx_parse_batch_host(engine.handle(), &cur.b, &o, &rec), "pcppx_parse_batch_host");
					for (uint32_t i = 0; i < cur.b.n; ++i)
						dg += rec.summary[i].hash5;
					np += cur.b.n;
					nw += cur.b.data_len;
					read_s += cur.read_s;
					fut.get();
				}
				delete bufs[0];
				delete bufs[1];
			}
			pcppx_pcap_close(reader);
			const double t = now() - t0;
			if (t < best)
			{
				best = t;
				best_read = read_s;
			}
			packets = np;
			wire = nw;
			digest = dg;
		}
		std::printf("{\"file\": \"%s\", \"mode\": \"%s\", \"packets\": %" PRIu64 ", \"file_bytes\": %lld, \"wire_bytes\": %" PRIu64
		            ", \"max_layers\": %u, \"checksums\": %s, \"batch\": %u, \"seconds\": %.6f, \"Mpackets_per_s\": %.2f, "
		            "\"file_GBps\": %.2f, \"wire_GBps\": %.2f, \"reader_seconds\": %.6f, \"hash5_digest\": %" PRIu64 "}\n",
		            path.c_str(), copyMode ? "copy" : "map", packets, (long long)st.st_size, wire, layers,
		            csum ? "true" : "false", batchN, best, packets / best / 1e6, st.st_size / best / 1e9, wire / best / 1e9,
		            best_read, digest);
	}
	catch (const pcppx::Error& e)
	{
		std::fprintf(stderr, "%s\n", e.what());
		return 1;
	}
	return 0;
}
