// ingest_fuzz.cpp — host-only sanitizer / fuzz driver for the capture reader (csrc/pcppx_pcap.cpp).
//
// Built by tests/test_ingest.py with -fsanitize=address,undefined (no HIP: the reader is plain C++):
//   g++ -std=c++17 -g -O1 -fsanitize=address,undefined -fno-sanitize-recover=all -Iinclude \
//       pcapplusplus_amd/csrc/pcppx_pcap.cpp tools/ingest_fuzz.cpp -o ingest_fuzz
//   ingest_fuzz <iterations per file> <file>...
// Each file is read whole with small batch limits (so batches split on packet count, buffer size and
// pcapng link-type changes), then <iterations> seeded mutations of it (word overwrites, byte flips,
// truncations, slice duplications/deletions — the classes of tests/ingest_cases.py) are written to a
// scratch file and read the same way. Any out-of-bounds access or UB aborts under the sanitizers.
// Prints "files=<n> cases=<n> packets=<n>" on success.
#include "pcppx.h"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <random>
#include <string>
#include <vector>

namespace
{
uint64_t read_all(const std::string& path, uint32_t max_packets, uint64_t cap)
{
	pcppx_pcap* r = nullptr;
	if (pcppx_pcap_open(path.c_str(), &r) != PCPPX_OK)
		return 0;
	std::vector<uint8_t> data(cap);
	std::vector<uint64_t> offs(max_packets), ts(max_packets);
	std::vector<uint32_t> caps(max_packets), frames(max_packets);
	uint64_t total = 0;
	for (;;)
	{
		uint32_t n = 0;
		uint64_t used = 0;
		int rc = pcppx_pcap_read_batch_ex(r, data.data(), cap, offs.data(), caps.data(), frames.data(), ts.data(),
		                                  max_packets, &n, &used);
		if (rc == PCPPX_E_NOMEM)
		{
			cap *= 4;  // one record larger than the buffer: grow and retry
			data.resize(cap);
			continue;
		}
		if (rc != PCPPX_OK || n == 0)
			break;
		uint64_t sum = 0;
		for (uint32_t i = 0; i < n; ++i)
		{
			if (offs[i] + caps[i] > used)
				std::abort();
			sum += caps[i];
		}
		if (sum != used)
			std::abort();
		(void)pcppx_pcap_linktype(r);
		total += n;
	}
	pcppx_pcap_close(r);
	return total;
}

void mutate(std::vector<uint8_t>& b, std::mt19937_64& rng)
{
	if (b.empty())
		return;
	auto pick = [&](size_t n) { return n ? (size_t)(rng() % n) : 0; };
	static const uint32_t kWords[] = {0, 1, 4, 8, 11, 12, 13, 16, 20, 28, 31, 32, 33, 0xFFFF, 0x10000, 0x40000,
	                                  0x40001, 0x7FFFFFFF, 0xFFFFFFFF};
	switch (rng() % 6)
	{
	case 0:
	{
		size_t pos = pick(b.size() > 4 ? std::min<size_t>(b.size() - 4, 4096) : 1) & ~size_t(3);
		uint32_t v = (rng() & 1) ? kWords[pick(sizeof(kWords) / 4)] : (uint32_t)rng();
		if (pos + 4 <= b.size())
			std::memcpy(&b[pos], &v, 4);
		break;
	}
	case 1:
		for (int k = 0, m = 1 + (int)pick(5); k < m; ++k)
			b[pick(std::min<size_t>(b.size(), 512))] ^= (uint8_t)(1u << pick(8));
		break;
	case 2:
		b.resize(pick(b.size()));
		break;
	case 3:
	{
		size_t i = pick(b.size()), j = std::min(b.size(), i + 1 + pick(200));
		std::vector<uint8_t> s(b.begin() + i, b.begin() + j);
		b.insert(b.begin() + i, s.begin(), s.end());
		break;
	}
	case 4:
	{
		size_t i = pick(b.size()), j = std::min(b.size(), i + 1 + pick(64));
		b.erase(b.begin() + i, b.begin() + j);
		break;
	}
	default:
		for (size_t i = pick(b.size()), e = std::min(b.size(), i + 1 + pick(32)); i < e; ++i)
			b[i] = (uint8_t)rng();
	}
}
}  // namespace

int main(int argc, char** argv)
{
	if (argc < 3)
	{
		std::fprintf(stderr, "usage: %s <iterations> <file>...\n", argv[0]);
		return 2;
	}
	const int iters = std::atoi(argv[1]);
	const char* tmpdir = std::getenv("TMPDIR");
	const std::string scratch = std::string(tmpdir ? tmpdir : "/tmp") + "/ingest_fuzz_case";
	std::mt19937_64 rng(12345);
	uint64_t cases = 0, packets = 0;
	for (int a = 2; a < argc; ++a)
	{
		std::ifstream f(argv[a], std::ios::binary);
		std::vector<uint8_t> orig((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
		packets += read_all(argv[a], 7, 3000);
		++cases;
		for (int k = 0; k < iters; ++k)
		{
			std::vector<uint8_t> m = orig;
			for (int t = 0, nm = 1 + (int)(rng() % 3); t < nm; ++t)
				mutate(m, rng);
			{
				std::ofstream o(scratch, std::ios::binary | std::ios::trunc);
				o.write(reinterpret_cast<const char*>(m.data()), (std::streamsize)m.size());
			}
			packets += read_all(scratch, 1 + (uint32_t)(rng() % 64), 1 + rng() % 70000);
			++cases;
		}
	}
	std::remove(scratch.c_str());
	std::printf("files=%d cases=%llu packets=%llu\n", argc - 2, (unsigned long long)cases, (unsigned long long)packets);
	return 0;
}
