// pcppx_pcap.cpp — host ingest: pcap files straight into packed (optionally pinned) batch buffers.
//
// Follows the reference reader's rules (Pcap++/src/PcapFileDevice.cpp): magic detection incl. the
// swapped, nanosecond and Kuznetzov variants (:53-60, :667-705), the 24-B file header and 16-B record
// header (:66-87), and readNextPacket's checks (:799-880): caplen > len, caplen > 256 KiB or an
// out-of-range sub-second field end the stream; caplen beyond the snapshot length is truncated.
// Unlike PcapFileReaderDevice::getNextPacket (:770-792: one heap allocation + copy per packet), records
// are copied once from a memory-mapped file into the caller's batch buffers, back to back.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <hip/hip_runtime.h>

#include <cstring>
#include <new>

#include "pcppx.h"

namespace
{
constexpr uint32_t kMagic = 0xa1b2c3d4, kMagicSwapped = 0xd4c3b2a1;
constexpr uint32_t kKuz = 0xa1b2cd34, kKuzSwapped = 0x34cdb2a1;
constexpr uint32_t kNsec = 0xa1b23c4d, kNsecSwapped = 0x4d3cb2a1;
constexpr uint32_t kMaxRecord = 256 * 1024;

uint32_t sw32(uint32_t v)
{
	return __builtin_bswap32(v);
}
}  // namespace

struct pcppx_pcap
{
	const uint8_t* map = nullptr;
	size_t size = 0;
	size_t pos = 0;
	bool swap = false, nsec = false;
	uint32_t rec_hdr = 16;
	uint32_t snaplen = 0;
	uint32_t linktype = 0;
	bool done = false;
};

extern "C"
{
	int pcppx_pcap_open(const char* path, pcppx_pcap** out)
	{
		if (path == nullptr || out == nullptr)
			return PCPPX_E_INVAL;
		*out = nullptr;
		int fd = open(path, O_RDONLY);
		if (fd < 0)
			return PCPPX_E_INVAL;
		struct stat st;
		if (fstat(fd, &st) != 0 || st.st_size < 24)
		{
			close(fd);
			return PCPPX_E_INVAL;
		}
		void* m = mmap(nullptr, (size_t)st.st_size, PROT_READ, MAP_PRIVATE, fd, 0);
		close(fd);
		if (m == MAP_FAILED)
			return PCPPX_E_NOMEM;
		madvise(m, (size_t)st.st_size, MADV_SEQUENTIAL);
		pcppx_pcap* r = new (std::nothrow) pcppx_pcap();
		if (r == nullptr)
		{
			munmap(m, (size_t)st.st_size);
			return PCPPX_E_NOMEM;
		}
		r->map = static_cast<const uint8_t*>(m);
		r->size = (size_t)st.st_size;
		uint32_t magic;
		std::memcpy(&magic, r->map, 4);
		switch (magic)
		{
		case kMagic: break;
		case kMagicSwapped: r->swap = true; break;
		case kNsec: r->nsec = true; break;
		case kNsecSwapped: r->nsec = r->swap = true; break;
		case kKuz: r->rec_hdr = 24; break;
		case kKuzSwapped: r->rec_hdr = 24; r->swap = true; break;
		default:
			munmap(m, r->size);
			delete r;
			return PCPPX_E_INVAL;
		}
		uint32_t snap, lt;
		std::memcpy(&snap, r->map + 16, 4);
		std::memcpy(&lt, r->map + 20, 4);
		r->snaplen = r->swap ? sw32(snap) : snap;
		r->linktype = (r->swap ? sw32(lt) : lt) & 0x0FFFFFFF;
		r->pos = 24;
		*out = r;
		return PCPPX_OK;
	}

	uint32_t pcppx_pcap_linktype(const pcppx_pcap* r)
	{
		return r ? r->linktype : 0;
	}

	int pcppx_pcap_read_batch(pcppx_pcap* r, uint8_t* data, uint64_t data_cap, uint64_t* offsets, uint32_t* caplens,
	                          uint64_t* timestamps_ns, uint32_t max_packets, uint32_t* n_out, uint64_t* bytes_out)
	{
		if (r == nullptr || data == nullptr || offsets == nullptr || caplens == nullptr || n_out == nullptr)
			return PCPPX_E_INVAL;
		uint32_t n = 0;
		uint64_t used = 0;
		while (!r->done && n < max_packets && r->pos + r->rec_hdr <= r->size)
		{
			uint32_t h[4];
			std::memcpy(h, r->map + r->pos, 16);
			if (r->swap)
				for (uint32_t& x : h)
					x = sw32(x);
			const uint32_t sec = h[0], sub = h[1], cap = h[2], len = h[3];
			if (cap > len || cap > kMaxRecord || sub >= (r->nsec ? 1000000000u : 1000000u) ||
			    r->pos + r->rec_hdr + cap > r->size)
			{
				r->done = true;  // readNextPacket returns false: the stream ends here
				break;
			}
			const uint32_t keep = (r->snaplen != 0 && cap > r->snaplen) ? r->snaplen : cap;
			if (used + keep > data_cap)
			{
				if (n == 0)
					return PCPPX_E_NOMEM;  // a single record does not fit the caller's buffer
				break;
			}
			std::memcpy(data + used, r->map + r->pos + r->rec_hdr, keep);
			offsets[n] = used;
			caplens[n] = keep;
			if (timestamps_ns)
				timestamps_ns[n] = (uint64_t)sec * 1000000000ull + (r->nsec ? sub : (uint64_t)sub * 1000ull);
			used += keep;
			r->pos += r->rec_hdr + cap;
			++n;
		}
		*n_out = n;
		if (bytes_out)
			*bytes_out = used;
		return PCPPX_OK;
	}

	void pcppx_pcap_close(pcppx_pcap* r)
	{
		if (r == nullptr)
			return;
		munmap(const_cast<uint8_t*>(r->map), r->size);
		delete r;
	}

	void* pcppx_host_alloc(size_t bytes)
	{
		void* p = nullptr;
		if (hipHostMalloc(&p, bytes ? bytes : 1) != hipSuccess)
			return nullptr;
		return p;
	}

	void pcppx_host_free(void* p)
	{
		if (p)
			(void)hipHostFree(p);
	}
}
