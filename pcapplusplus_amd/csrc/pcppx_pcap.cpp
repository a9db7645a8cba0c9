// pcppx_pcap.cpp — host ingest: pcap and pcapng captures straight into packed (optionally pinned) batches.
//
// Plain C++ (no HIP): the same file builds into libpcppx.so and into the host-only sanitizer/fuzz
// driver (tools/ingest_fuzz.cpp, -fsanitize=address,undefined).
//
// The format is detected from the first four bytes, as IFileReaderDevice::createReader does
// (Pcap++/src/PcapFileDevice.cpp:283-325,404-458), and read as the device for that format would:
//
// pcap — PcapFileReaderDevice (PcapFileDevice.cpp):
//   open (:707-768): 24-B file header; the six pcap magics (:53-60, :283-325; the Kuznetzov "modified"
//   magics are accepted but, like the reference, read with the plain 16-B record header of :79-86);
//   version_major 2 or 543 (:747); 0 < snaplen <= 1 MiB (:754-759); linktype through toLinkLayerType
//   (:89-209: a value outside the LinkLayerType list becomes LINKTYPE_INVALID 0xFFFF).
//   readNextPacket (:799-886): a short record header, caplen > len, caplen > 256 KiB, a sub-second
//   field out of range, or packet bytes cut by the end of the file end the stream; caplen beyond the
//   snapshot length keeps the first snaplen bytes and skips the rest (a skip that runs past the end of
//   the file still delivers the packet: istream::ignore only sets eofbit).
//
// pcapng — PcapNgFileReaderDevice (:1157-1243) over LightPcapNg
//   (3rdParty/LightPcapNg/LightPcapNg/src/light_pcapng.c, light_pcapng_ext.c):
//   light_read_record (light_pcapng.c:341-423): type + total length + body + trailing length; a short
//   read or a trailing length that differs ends the stream. The first block must be a section header
//   (light_pcapng_ext.c:43-55), else the capture holds no packets.
//   light_get_next_packet (light_pcapng_ext.c:380-479): blocks other than EPB/SPB are skipped; every
//   interface description block met on the way is appended to one file-wide list (at most 32,
//   MAX_SUPPORTED_INTERFACE_BLOCKS; sections do not reset it), with its link type (u16) and
//   timestamp resolution from if_tsresol (:140-167: 10^v or 2^(v-128) ticks/s into a uint32, default
//   10^6; options parsed as __parse_options, light_pcapng.c:36-93).
//   EPB (light_pcapng.c:150-194): caplen clamped to block_total_length - 32 (GH #2180 patch); an
//   interface id outside the list gives linktype 0xFFFF and timestamp 0; a timestamp whose seconds are
//   0 or exceed UINT64_MAX / 1e9 is 0 (light_pcapng_ext.c:419-445).
//   SPB (light_pcapng.c:196-211, light_pcapng_ext.c:451-466): caplen = original length, linktype of
//   interface 0, timestamp 0.
//   Where the reference's behaviour is undefined (it reads past its heap buffer), this reader ends the
//   stream instead: a block total length below 12 (SPB: 16), an EPB/IDB body shorter than its fixed
//   fields (a short section header only gives it a garbage version: it still opens the section), an SPB whose original length exceeds its body (we keep the body), or an SPB before any
//   interface (the reference reads an uninitialised link type; we return 0xFFFF).
//
// Unlike getNextPacket (one heap allocation + copy per packet, :770-792), records are copied once from
// a memory-mapped file into the caller's batch buffers, back to back. A batch holds packets of one link
// type only (pcapng interfaces may differ): it ends before a packet of another link type.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstring>
#include <new>
#include <thread>
#include <vector>

#include "pcppx.h"

namespace
{
constexpr uint32_t kMagic = 0xa1b2c3d4, kMagicSwapped = 0xd4c3b2a1;
constexpr uint32_t kKuz = 0xa1b2cd34, kKuzSwapped = 0x34cdb2a1;
constexpr uint32_t kNsec = 0xa1b23c4d, kNsecSwapped = 0x4d3cb2a1;
constexpr uint32_t kPcapNgMagic = 0x0A0D0D0A;  // section header block type (PcapFileDevice.cpp:331-335)
constexpr uint32_t kMaxRecord = 256 * 1024;     // readNextPacket MAX_PACKET_SIZE (:832)
constexpr uint32_t kMaxSnaplen = 1024 * 1024;   // open MAX_SNAPLEN (:754)
constexpr uint32_t kLinkInvalid = 0xFFFF;       // LINKTYPE_INVALID (Packet++/header/RawPacket.h:250)

// pcapng block types and options (light_pcapng.h)
constexpr uint32_t kShb = 0x0A0D0D0A, kIdb = 0x00000001, kSpb = 0x00000003, kEpb = 0x00000006;
constexpr uint16_t kOptTsresol = 9;
constexpr uint32_t kMaxInterfaces = 32;  // MAX_SUPPORTED_INTERFACE_BLOCKS (light_pcapng_ext.h:46)

uint32_t sw32(uint32_t v)
{
	return __builtin_bswap32(v);
}

uint32_t ld32(const uint8_t* p)
{
	uint32_t v;
	std::memcpy(&v, p, 4);
	return v;
}

uint16_t ld16(const uint8_t* p)
{
	uint16_t v;
	std::memcpy(&v, p, 2);
	return v;
}

// toLinkLayerType (PcapFileDevice.cpp:89-209): the LinkLayerType values of RawPacket.h:24-248
bool known_linktype(uint32_t v)
{
	static const uint16_t kKnown[] = {
		0,   1,   3,   6,   7,   8,   9,   10,  12,  14,  50,  51,  100, 101, 104, 105, 107, 108, 113, 114, 117,
		119, 122, 123, 127, 129, 138, 139, 140, 141, 142, 143, 144, 147, 148, 149, 150, 151, 152, 153, 154, 155,
		156, 157, 158, 159, 160, 161, 162, 163, 165, 166, 169, 170, 171, 177, 187, 189, 192, 195, 196, 197, 201,
		202, 203, 204, 205, 206, 209, 215, 220, 224, 225, 226, 227, 228, 229, 230, 231, 235, 236, 237, 239, 240,
		241, 242, 243, 244, 245, 247, 248, 249, 250, 251, 253, 254, 255, 256, 257, 258, 259, 260, 261, 262, 263,
		264, 276,
	};
	for (uint16_t k : kKnown)
		if (v == k)
			return true;
	return false;
}

uint64_t int_pow(uint64_t x, uint32_t y)
{
	uint64_t r = 1;
	for (uint32_t i = 0; i < y; ++i)
		r *= x;
	return r;
}

// Parallel record walk of large pcap regions (pcppx_pcap_map_batch). The chain of record starts is sequential by
// nature -- each header's caplen gives the next position, one dependent memory access per packet (~0.1 us on a
// capture the caches do not hold) -- so a region is cut into kParThreads segments, each thread walks its segment
// from a re-synchronised start (the first position from which kSyncChain records in a row pass readNextPacket's
// checks), and the merge accepts a segment's chain only from a record start the chain before it actually lands on;
// a segment whose chain it does not land on is walked again from that start. The walk is deterministic, so the
// result is exactly the sequential walk's (a false start only costs the re-walk).
constexpr size_t kParRegion = 256ull << 20;  // bytes per parallel round
constexpr size_t kParMin = 16ull << 20;      // fewer bytes left: walk sequentially (starting 2-16 threads per call costs
                                             // more than walking a smaller region on one: a 10k-packet, 8-MB capture
                                             // mapped 0.3 ms slower in parallel, profiles/r05zd_facade_probe.txt)
constexpr unsigned kParThreads = 16;         // at most; one per MiB of the region at least
constexpr unsigned kParChains = 4;           // interleaved chains (segments) per thread
// fn(t) for t in [0, T): on new threads where they can be started, the rest on the calling thread (a thread that
// cannot be created never fails the read). An out-of-memory in any fn(t) -- a worker's or the caller's -- is caught
// where it happens, every thread is joined, and then std::bad_alloc is rethrown on the calling thread, where the
// reader falls back to the sequential walk (an exception leaving a std::thread, or a joinable thread destroyed during
// unwinding, would call std::terminate).
template <class F>
void run_parallel(unsigned T, const F& fn)
{
	std::atomic<bool> oom{ false };
	auto guarded = [&](unsigned t) {
		try
		{
			fn(t);
		}
		catch (const std::bad_alloc&)
		{
			oom.store(true);
		}
	};
	std::vector<std::thread> th;
	unsigned started = 1;
	try
	{
		th.reserve(T);
		for (; started < T; ++started)
			th.emplace_back(guarded, started);
	}
	catch (...)
	{
	}
	guarded(0u);
	for (unsigned t = started; t < T; ++t)
		guarded(t);
	for (auto& x : th)
		x.join();
	if (oom.load())
		throw std::bad_alloc();
}

unsigned par_threads(size_t bytes)
{
	if (bytes < kParMin)
		return 1;  // the calling thread alone
	const size_t t = bytes >> 20;
	return t > kParThreads ? kParThreads : (unsigned)t;
}
constexpr size_t kSyncScan = 1u << 16;  // bytes a segment searches for a plausible record start
constexpr int kSyncChain = 4;

struct Chain
{
	std::vector<size_t> starts;  // record starts below the segment's end
	size_t end = 0;              // the first record start at or past it, or where the stream ends
	bool stop = false;           // the stream ends at `end` (an invalid record)
};

struct Packet
{
	const uint8_t* bytes;
	uint32_t keep, frame_len, linktype;
	uint64_t ts_ns;
	size_t next_pos;  // where the stream continues after this packet
};
}  // namespace

struct pcppx_pcap
{
	const uint8_t* map = nullptr;
	size_t size = 0;
	size_t pos = 0;
	bool ng = false;
	bool swap = false, nsec = false;
	uint32_t snaplen = 0;
	uint32_t linktype = 0;  // pcap: the file's; pcapng: of the last batch returned (before it: of the first packet)
	bool done = false;
	// the record starts of the last parallel walk not yet handed out (a batch that ends inside a walked region leaves
	// the rest here for the next batch instead of walking it again)
	std::vector<size_t> pend;
	size_t pend_i = 0, pend_end = 0;
	bool pend_stop = false, pend_ok = false;
	// an allocation of the parallel walk failed: the reader goes on with the sequential walk (same records)
	bool par_off = false;
	// pcapng: the file-wide interface list of light_pcapng_file_info
	uint32_t n_if = 0;
	uint16_t if_link[kMaxInterfaces];
	uint32_t if_ticks[kMaxInterfaces];

	// pcap record at pos (readNextPacket). false = the stream ends here.
	bool next_pcap(Packet& pk) const
	{
		return pcap_at(pos, pk);
	}
	bool pcap_at(size_t pos, Packet& pk) const
	{
		if (size - pos < 16)
			return false;
		uint32_t h[4];
		std::memcpy(h, map + pos, 16);
		if (swap)
			for (uint32_t& x : h)
				x = sw32(x);
		const uint32_t sec = h[0], sub = h[1], cap = h[2], len = h[3];
		if (cap > len || cap > kMaxRecord || sub >= (nsec ? 1000000000u : 1000000u))
			return false;
		const uint32_t keep = cap > snaplen ? snaplen : cap;
		const size_t body = pos + 16;
		if (size - body < keep)
			return false;  // "Failed to read packet data"
		pk.bytes = map + body;
		pk.keep = keep;
		pk.frame_len = len;
		pk.linktype = linktype;
		pk.ts_ns = (uint64_t)sec * 1000000000ull + (nsec ? sub : (uint64_t)sub * 1000ull);
		pk.next_pos = (size - body < cap) ? size : body + cap;  // the skipped tail may run past the end
		return true;
	}

	// light_read_record at p: block type, total length and body bounds; false = the stream ends.
	bool ng_block(size_t p, uint32_t& type, uint32_t& total) const
	{
		if (size - p < 8)
			return false;
		type = ld32(map + p);
		total = ld32(map + p + 4);
		if (total < 12 || size - p < (size_t)total)
			return false;
		return ld32(map + p + total - 4) == total;
	}

	// __append_interface_block_to_file_info for the IDB at p (light_pcapng_ext.c:140-167)
	bool ng_interface(size_t p, uint32_t total)
	{
		if (total < 20)
			return false;  // link type + reserved + snaplen do not fit
		const uint8_t* body = map + p + 8;
		if (n_if >= kMaxInterfaces)
			return true;
		uint32_t ticks = 1000000;
		// __parse_options (light_pcapng.c:36-93): max_len = total - 20 bytes of options; stop at the end
		// option, a length that does not fit, or a zero-length option.
		int32_t max_len = (int32_t)(total - 20);
		const uint8_t* o = body + 8;
		while (max_len > 4)
		{
			const uint16_t code = ld16(o), len = ld16(o + 2);
			if ((int32_t)len > max_len - 4)
				break;
			const uint16_t actual = (len % 4) == 0 ? len : (uint16_t)((len / 4 + 1) * 4);
			if (actual == 0 || (int32_t)actual > max_len - 4)
				break;
			if (code == kOptTsresol)
			{
				const uint8_t v = o[4];
				ticks = (uint32_t)(v < 128 ? int_pow(10, v) : int_pow(2, v - 128u));
				break;  // light_get_option returns the first match
			}
			if (code == 0)
				break;
			o += 4 + actual;
			max_len = (uint16_t)(max_len - actual - 4);  // remaining_size is a uint16_t
		}
		if_link[n_if] = ld16(body);
		if_ticks[n_if] = ticks;
		++n_if;
		return true;
	}

	// light_get_next_packet from pos: interface blocks on the way are appended (and pos moves past
	// them, so a packet left for the next batch does not append them twice).
	bool next_pcapng(Packet& pk)
	{
		for (;;)
		{
			uint32_t type, total;
			if (!ng_block(pos, type, total))
				return false;
			if (type == kIdb)
			{
				if (!ng_interface(pos, total))
					return false;
				pos += total;
				continue;
			}
			if (type == kEpb)
			{
				if (total < 32)
					return false;  // the five fixed fields do not fit
				const uint8_t* body = map + pos + 8;
				const uint32_t ifid = ld32(body), hi = ld32(body + 4), lo = ld32(body + 8);
				uint32_t cap = ld32(body + 12);
				const uint32_t orig = ld32(body + 16);
				const uint32_t max_cap = total > 32 ? total - 32 : 0;
				if (cap > max_cap)
					cap = max_cap;
				pk.bytes = body + 20;
				pk.keep = cap;
				pk.frame_len = orig;
				pk.ts_ns = 0;
				pk.linktype = kLinkInvalid;
				if (ifid < n_if)
				{
					const uint64_t t = ((uint64_t)hi << 32) + lo;
					const uint64_t tps = if_ticks[ifid];
					const uint64_t secs = tps != 0 ? t / tps : 0;
					if (secs <= UINT64_MAX / 1000000000ull && secs != 0)
						pk.ts_ns = secs * 1000000000ull + (1000000000ull * (t % tps)) / tps;
					pk.linktype = if_link[ifid];
				}
				pk.next_pos = pos + total;
				return true;
			}
			if (type == kSpb)
			{
				if (total < 16)
					return false;
				const uint8_t* body = map + pos + 8;
				const uint32_t orig = ld32(body), avail = total - 16;
				pk.bytes = body + 4;
				pk.keep = orig < avail ? orig : avail;
				pk.frame_len = orig;
				pk.ts_ns = 0;
				pk.linktype = n_if > 0 ? if_link[0] : kLinkInvalid;
				pk.next_pos = pos + total;
				return true;
			}
			pos += total;  // section header, statistics, name resolution, custom, unknown: skipped
		}
	}

	bool next(Packet& pk)
	{
		return ng ? next_pcapng(pk) : next_pcap(pk);
	}

	// a parallel walk of the next region when no walked starts are pending
	bool parallel_ready() const
	{
		return !ng && !done && !par_off && (pend_ok || size - pos >= kParMin);
	}
	void fill_pending()
	{
		if (pend_ok)
			return;
		const size_t region_end = pos + std::min(size - pos, kParRegion);
		parallel_starts(region_end, pend, &pend_end, &pend_stop);
		pend_i = 0;
		pend_ok = true;
	}
	// k pending starts handed out; true when starts are left (the batch is full: it ends before the next one)
	bool consume(size_t k)
	{
		pend_i += k;
		if (pend_i < pend.size())
		{
			pos = pend[pend_i];
			return true;
		}
		pos = pend_end;
		pend_ok = false;
		if (pend_stop)
			done = true;
		return false;
	}

	// the sequential chain from p (a record start or a guess) up to hi
	void walk(size_t p, size_t hi, Chain& c) const
	{
		Packet pk;
		while (p < hi)
		{
			if (!pcap_at(p, pk))
			{
				c.end = p;
				c.stop = true;
				return;
			}
			c.starts.push_back(p);
			p = pk.next_pos;
		}
		c.end = p;
	}

	bool plausible(size_t p) const
	{
		Packet pk;
		for (int k = 0; k < kSyncChain; ++k)
		{
			if (!pcap_at(p, pk))
				return false;
			p = pk.next_pos;
			if (p >= size)
				return true;
		}
		return true;
	}

	// every record start in [pos, region_end) (and *end, *stop as Chain's), as the sequential walk finds them.
	// The region is cut into kParChains segments per thread, and each thread advances its segments' chains in lockstep:
	// a chain is one dependent header read per record (the next position comes from this header's caplen), so the
	// interleaved chains keep kParChains of those reads in flight per core instead of one.
	void parallel_starts(size_t region_end, std::vector<size_t>& out, size_t* end, bool* stop) const
	{
		const unsigned T = par_threads(region_end - pos), S = T * kParChains;
		std::vector<size_t> lo(S + 1);
		for (unsigned t = 0; t <= S; ++t)
			lo[t] = pos + (region_end - pos) / S * t;
		lo[S] = region_end;
		std::vector<Chain> seg(S);
		run_parallel(T, [&](unsigned t) {
				struct Cur
				{
					size_t p, hi;
					bool on;
				};
				Cur w[kParChains];
				for (unsigned k = 0; k < kParChains; ++k)
				{
					const unsigned g = t * kParChains + k;
					size_t s0 = lo[g];
					w[k] = Cur{ s0, lo[g + 1], true };
					if (g > 0)
					{
						const size_t lim = std::min(lo[g + 1], lo[g] + kSyncScan);
						while (s0 < lim && !plausible(s0))
							++s0;
						if (s0 >= lim)
						{
							seg[g].end = lo[g];  // no start found: the merge walks this segment
							w[k].on = false;
							continue;
						}
						w[k].p = s0;
					}
					if (w[k].p >= w[k].hi)
					{
						seg[g].end = w[k].p;
						w[k].on = false;
					}
				}
				for (unsigned live = kParChains; live;)
				{
					live = 0;
					for (unsigned k = 0; k < kParChains; ++k)
					{
						if (!w[k].on)
							continue;
						Chain& c = seg[t * kParChains + k];
						Packet pk{};
						if (!pcap_at(w[k].p, pk))
						{
							c.end = w[k].p;  // walk()'s rules: the stream ends here
							c.stop = true;
							w[k].on = false;
							continue;
						}
						c.starts.push_back(w[k].p);
						w[k].p = pk.next_pos;
						if (w[k].p >= w[k].hi)
						{
							c.end = w[k].p;
							w[k].on = false;
							continue;
						}
						++live;
					}
				}
			});
		// the accepted part of every segment, in order (a segment whose chain the true chain does not land on is walked
		// again from the true position), then one parallel copy into `out`
		std::vector<std::pair<const std::vector<size_t>*, size_t>> take;
		take.reserve(S);
		std::vector<Chain> redo(S);
		take.emplace_back(&seg[0].starts, 0);
		*end = seg[0].end;
		*stop = seg[0].stop;
		for (unsigned t = 1; t < S && !*stop; ++t)
		{
			const std::vector<size_t>& c = seg[t].starts;
			auto it = std::lower_bound(c.begin(), c.end(), *end);
			if (it != c.end() && *it == *end)
			{
				take.emplace_back(&c, (size_t)(it - c.begin()));  // the true chain lands on this segment's chain
				*end = seg[t].end;
				*stop = seg[t].stop;
			}
			else
			{
				walk(*end, lo[t + 1], redo[t]);
				take.emplace_back(&redo[t].starts, 0);
				*end = redo[t].end;
				*stop = redo[t].stop;
			}
		}
		std::vector<size_t> at(take.size() + 1, 0);
		for (size_t j = 0; j < take.size(); ++j)
			at[j + 1] = at[j] + (take[j].first->size() - take[j].second);
		out.resize(at.back());
		run_parallel(T, [&](unsigned t) {
				for (size_t j = t; j < take.size(); j += T)
					std::copy(take[j].first->begin() + (ptrdiff_t)take[j].second, take[j].first->end(),
					          out.begin() + (ptrdiff_t)at[j]);
			});
	}
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
		if (fstat(fd, &st) != 0 || st.st_size < 4)
		{
			close(fd);
			return PCPPX_E_INVAL;
		}
		// a small capture is mapped populated (one kernel call instead of a page fault per 4 KiB on the first walk)
		constexpr off_t kPopulateMax = 64 << 20;
		void* m = mmap(nullptr, (size_t)st.st_size, PROT_READ, MAP_PRIVATE | (st.st_size <= kPopulateMax ? MAP_POPULATE : 0),
		               fd, 0);
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
		auto fail = [&](int rc) {
			munmap(m, r->size);
			delete r;
			return rc;
		};
		const uint32_t magic = ld32(r->map);
		if (magic == kPcapNgMagic)
		{
			// light_pcapng_open_read: the first record must be a well-formed section header, else the
			// device opens with no packets (light_pcapng_ext.c:183-224, 43-55)
			r->ng = true;
			uint32_t type, total;
			if (r->ng_block(0, type, total) && type == kShb)
			{
				r->pos = total;
				Packet pk;
				if (r->next_pcapng(pk))  // leaves pos at the first packet block (past the interfaces before it)
					r->linktype = pk.linktype;  // the link type of the first batch
			}
			else
				r->done = true;
			*out = r;
			return PCPPX_OK;
		}
		switch (magic)
		{
		case kMagic: case kKuz: break;
		case kMagicSwapped: case kKuzSwapped: r->swap = true; break;
		case kNsec: r->nsec = true; break;
		case kNsecSwapped: r->nsec = r->swap = true; break;
		default: return fail(PCPPX_E_INVAL);  // not pcap / pcapng (snoop and zstd archives: not supported)
		}
		if (r->size < 24)
			return fail(PCPPX_E_INVAL);  // "Cannot read pcap file header"
		uint16_t vmaj = ld16(r->map + 4);
		uint32_t snap = ld32(r->map + 16), lt = ld32(r->map + 20);
		if (r->swap)
		{
			vmaj = (uint16_t)((vmaj >> 8) | (vmaj << 8));
			snap = sw32(snap);
			lt = sw32(lt);
		}
		if (vmaj != 2 && vmaj != 543)
			return fail(PCPPX_E_INVAL);
		if (snap == 0 || snap > kMaxSnaplen)
			return fail(PCPPX_E_INVAL);
		r->snaplen = snap;
		r->linktype = known_linktype(lt) ? lt : kLinkInvalid;
		r->pos = 24;
		*out = r;
		return PCPPX_OK;
	}

	uint32_t pcppx_pcap_linktype(const pcppx_pcap* r)
	{
		return r ? r->linktype : 0;
	}

	int pcppx_pcap_read_batch_ex(pcppx_pcap* r, uint8_t* data, uint64_t data_cap, uint64_t* offsets, uint32_t* caplens,
	                             uint32_t* frame_lens, uint64_t* timestamps_ns, uint32_t max_packets, uint32_t* n_out,
	                             uint64_t* bytes_out)
	{
		if (r == nullptr || data == nullptr || offsets == nullptr || caplens == nullptr || n_out == nullptr)
			return PCPPX_E_INVAL;
		uint32_t n = 0;
		uint64_t used = 0;
		// large pcap regions: the parallel walk (identical records), then the fields and the copies in parallel. Its
		// scratch (record starts, segment chains) can be tens of MB: when an allocation fails the reader state is as
		// before the failed step (pos at the next record, n the packets already placed) and the sequential walk goes on.
		while (n < max_packets && r->parallel_ready())
		try
		{
			r->fill_pending();
			const size_t* starts = r->pend.data() + r->pend_i;
			const size_t avail = r->pend.size() - r->pend_i;
			// the records that fit: at most max_packets, and their bytes within data_cap (as the sequential loop below)
			size_t k = 0;
			std::vector<uint64_t> dst;
			dst.reserve(std::min(avail, (size_t)(max_packets - n)));
			while (k < avail && n + k < max_packets)
			{
				Packet pk{};
				(void)r->pcap_at(starts[k], pk);
				if (used + pk.keep > data_cap)
					break;
				dst.push_back(used);
				used += pk.keep;
				++k;
			}
			if (k == 0 && n == 0 && avail)
				return PCPPX_E_NOMEM;  // a single record does not fit the caller's buffer
			const unsigned T = par_threads(k * 512);
			run_parallel(T, [&](unsigned t) {
					for (size_t i = k * t / T; i < k * (t + 1) / T; ++i)
					{
						Packet pk{};
						(void)r->pcap_at(starts[i], pk);
						if (pk.keep)
							std::memcpy(data + dst[i], pk.bytes, pk.keep);
						offsets[n + i] = dst[i];
						caplens[n + i] = pk.keep;
						if (frame_lens)
							frame_lens[n + i] = pk.frame_len == 0xFFFFFFFFu ? pk.keep : pk.frame_len;
						if (timestamps_ns)
							timestamps_ns[n + i] = pk.ts_ns;
					}
				});
			n += (uint32_t)k;
			if (r->consume(k))
				break;
		}
		catch (const std::bad_alloc&)
		{
			r->par_off = true;
		}
		while (!r->done && n < max_packets)
		{
			Packet pk;
			if (!r->next(pk))
			{
				r->done = true;  // readNextPacket / light_get_next_packet return false: the stream ends here
				break;
			}
			if (n > 0 && pk.linktype != r->linktype)
				break;  // one link type per batch: the packet opens the next batch
			if (used + pk.keep > data_cap)
			{
				if (n == 0)
					return PCPPX_E_NOMEM;  // a single record does not fit the caller's buffer
				break;
			}
			r->linktype = pk.linktype;
			if (pk.keep)
				std::memcpy(data + used, pk.bytes, pk.keep);
			offsets[n] = used;
			caplens[n] = pk.keep;
			if (frame_lens)  // RawPacket::setRawData takes an int frameLength; -1 means "the captured length" (RawPacket.cpp:107)
				frame_lens[n] = pk.frame_len == 0xFFFFFFFFu ? pk.keep : pk.frame_len;
			if (timestamps_ns)
				timestamps_ns[n] = pk.ts_ns;
			used += pk.keep;
			r->pos = pk.next_pos;
			++n;
		}
		*n_out = n;
		if (bytes_out)
			*bytes_out = used;
		return PCPPX_OK;
	}

	// The same records without the copy: the batch points into the reader's map (offsets relative to *data = the map
	// base; the file's record headers / block framing lie between the packets).
	int pcppx_pcap_map_batch(pcppx_pcap* r, const uint8_t** data, uint64_t* data_len, uint64_t* offsets,
	                         uint32_t* caplens, uint32_t* frame_lens, uint64_t* timestamps_ns, uint32_t max_packets,
	                         uint32_t* n_out)
	{
		if (r == nullptr || data == nullptr || data_len == nullptr || offsets == nullptr || caplens == nullptr ||
		    n_out == nullptr)
			return PCPPX_E_INVAL;
		*data = r->map;
		*data_len = r->size;
		uint32_t n = 0;
		// large pcap regions: the parallel walk (identical records), then the fields of each record in parallel (an
		// allocation failure falls back to the sequential walk, as in pcppx_pcap_read_batch_ex)
		while (n < max_packets && r->parallel_ready())
		try
		{
			r->fill_pending();
			const size_t* starts = r->pend.data() + r->pend_i;
			const size_t k = std::min(r->pend.size() - r->pend_i, (size_t)(max_packets - n));
			const unsigned T = par_threads(k * 512);
			run_parallel(T, [&](unsigned t) {
					for (size_t i = k * t / T; i < k * (t + 1) / T; ++i)
					{
						Packet pk{};
						(void)r->pcap_at(starts[i], pk);  // a record of the chain: valid
						offsets[n + i] = (uint64_t)(pk.bytes - r->map);
						caplens[n + i] = pk.keep;
						if (frame_lens)
							frame_lens[n + i] = pk.frame_len == 0xFFFFFFFFu ? pk.keep : pk.frame_len;
						if (timestamps_ns)
							timestamps_ns[n + i] = pk.ts_ns;
					}
				});
			n += (uint32_t)k;
			if (r->consume(k))
				break;  // the batch is full: the next one starts at the first pending record
		}
		catch (const std::bad_alloc&)
		{
			r->par_off = true;
		}
		while (!r->done && n < max_packets)
		{
			Packet pk;
			if (!r->next(pk))
			{
				r->done = true;
				break;
			}
			if (n > 0 && pk.linktype != r->linktype)
				break;  // one link type per batch
			r->linktype = pk.linktype;
			offsets[n] = (uint64_t)(pk.bytes - r->map);
			caplens[n] = pk.keep;
			if (frame_lens)
				frame_lens[n] = pk.frame_len == 0xFFFFFFFFu ? pk.keep : pk.frame_len;
			if (timestamps_ns)
				timestamps_ns[n] = pk.ts_ns;
			r->pos = pk.next_pos;
			++n;
		}
		*n_out = n;
		return PCPPX_OK;
	}

	int pcppx_pcap_read_batch(pcppx_pcap* r, uint8_t* data, uint64_t data_cap, uint64_t* offsets, uint32_t* caplens,
	                          uint64_t* timestamps_ns, uint32_t max_packets, uint32_t* n_out, uint64_t* bytes_out)
	{
		return pcppx_pcap_read_batch_ex(r, data, data_cap, offsets, caplens, nullptr, timestamps_ns, max_packets, n_out,
		                                bytes_out);
	}

	void pcppx_pcap_close(pcppx_pcap* r)
	{
		if (r == nullptr)
			return;
		munmap(const_cast<uint8_t*>(r->map), r->size);
		delete r;
	}
}
