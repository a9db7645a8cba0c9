/* pcppx.hpp — the Packet++-shaped C++ facade over the engine's C ABI (pcppx.h). Header-only, no HIP types, no
 * Packet++ dependency.
 *
 * A reference caller's per-packet loop compiles against it unchanged (namespace aside:
 * Examples/PcapPlusPlus-benchmark/benchmark.cpp:89-95, Examples/DpdkExample-FilterTraffic/AppWorkerThread.h:85-139):
 *
 *   pcppx::PcapFileReaderDevice reader(path);          // Pcap++/header/PcapFileDevice.h
 *   reader.open();
 *   pcppx::RawPacket rawPacket;
 *   while (reader.getNextPacket(rawPacket)) {           // Pcap++/src/PcapFileDevice.cpp:770-792
 *       pcppx::Packet packet(&rawPacket, pcppx::TCP);   // Packet++/src/Packet.cpp:198-232
 *       if (packet.isPacketOfType(pcppx::TCP)) flows[pcppx::hash5Tuple(&packet)]++;
 *   }
 *
 * How the per-packet entry points reach the GPU (the batch prepass moved inside the library):
 *  - the reader memory-maps the capture; a mapper thread indexes the records of the next pages (up to 1M packets
 *    each, pcppx_pcap_map_batch: no per-packet copy) ahead of the caller;
 *  - a parser thread parses each page on the GPU (pcppx_parse_batch_host: staged to HBM, parsed, records DMA'd into
 *    page-locked memory) while the caller walks the page before it;
 *  - getNextPacket(rawPacket) points rawPacket at the packet's bytes in the map and at its page (no copy; the
 *    RawPacket keeps the page, and with it the map, alive);
 *  - Packet(&rawPacket, parseUntil...) binds to that packet's records. The reader learns the parse-until options
 *    from the first Packet built on a page and parses the next pages with them; a Packet with other options than
 *    its page was parsed with re-parses that page on the GPU for those options (kept beside the first), so every
 *    chain is exactly the one Packet::parsePacket builds for the options given (Packet.cpp:66-196);
 *  - a RawPacket that did not come from a reader (the caller's own bytes) is parsed as a one-packet batch.
 * Packets the engine leaves to the host (PCPPX_F_NEEDS_HOST: an L7 dissector, an out-of-scope L2/L3 layer) carry an
 * exact layer prefix; with a host parser registered (pcppx::setHostParser: the caller's own Packet++ parse of one
 * packet) they are completed before the caller sees them. libpcppx.so never links Packet++.
 *
 * The batch API remains for callers that want it: RawBatch + Engine::parse -> ParsedBatch of Packet views.
 *
 * Errors are reported as pcppx::Error (a std::runtime_error carrying the PCPPX_E_* code).
 */
#ifndef PCPPX_HPP
#define PCPPX_HPP

#include <sys/time.h>

#include <algorithm>
#include <atomic>
#include <iterator>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <ctime>
#include <deque>
#include <fstream>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <type_traits>
#include <utility>
#include <vector>

#include "pcppx.h"

namespace pcppx
{
/* ProtocolType / ProtocolTypeFamily / OsiModelLayer values of Packet++/header/ProtocolType.h:33-284 */
using ProtocolType = uint8_t;
using ProtocolTypeFamily = uint32_t;
constexpr ProtocolType UnknownProtocol = 0, Ethernet = 1, IPv4 = 2, IPv6 = 3, TCP = 4, UDP = 5, HTTPRequest = 6,
                       HTTPResponse = 7, ARP = 8, VLAN = 9, ICMP = 10, DNS = 13, MPLS = 14, GREv0 = 15, GREv1 = 16,
                       PPP_PPTP = 17, SSL = 18, GenericPayload = 25, PacketTrailer = 30, EthernetDot3 = 33, LLC = 44;
constexpr ProtocolTypeFamily IP = 0x203, GRE = 0xf10, HTTP = 0x607;
enum OsiModelLayer : uint8_t
{
	OsiModelPhysicalLayer = 1,
	OsiModelDataLinkLayer = 2,
	OsiModelNetworkLayer = 3,
	OsiModelTransportLayer = 4,
	OsiModelSesionLayer = 5,
	OsiModelPresentationLayer = 6,
	OsiModelApplicationLayer = 7,
	OsiModelLayerUnknown = 8
};

/* pcpp::LinkLayerType values the engine parses (Packet++/header/RawPacket.h:24-178) */
using LinkLayerType = uint16_t;
constexpr LinkLayerType LINKTYPE_NULL = 0, LINKTYPE_ETHERNET = 1, LINKTYPE_DLT_RAW1 = 12, LINKTYPE_DLT_RAW2 = 14,
                        LINKTYPE_RAW = 101, LINKTYPE_LINUX_SLL = 113, LINKTYPE_IPV4 = 228, LINKTYPE_IPV6 = 229,
                        LINKTYPE_LINUX_SLL2 = 276, LINKTYPE_INVALID = 0xFFFF;

/* facade-level summary flag: the records were filled by the caller's host parser (setHostParser) */
constexpr uint16_t F_HOST_PARSED = 0x4000;

class Error : public std::runtime_error
{
public:
	Error(int code, const std::string& what) : std::runtime_error(what + ": " + pcppx_strerror(code)), m_Code(code) {}
	int code() const { return m_Code; }

private:
	int m_Code;
};

inline void check(int rc, const char* what)
{
	if (rc != PCPPX_OK)
		throw Error(rc, what);
}

/* pcpp::IPv4Address (Common++/header/IpAddress.h:37-40): the four bytes in memory order */
class IPv4Address
{
public:
	IPv4Address() = default;
	explicit IPv4Address(uint32_t addrAsInt) : m_Int(addrAsInt) {}
	explicit IPv4Address(const std::string& dotted)
	{
		unsigned v[4];
		char tail;
		if (std::sscanf(dotted.c_str(), "%u.%u.%u.%u%c", &v[0], &v[1], &v[2], &v[3], &tail) != 4 || v[0] > 255 ||
		    v[1] > 255 || v[2] > 255 || v[3] > 255)
			throw Error(PCPPX_E_INVAL, "bad IPv4 address '" + dotted + "'");
		const uint8_t b[4] = { (uint8_t)v[0], (uint8_t)v[1], (uint8_t)v[2], (uint8_t)v[3] };
		std::memcpy(&m_Int, b, 4);
	}
	uint32_t toInt() const { return m_Int; }
	std::string toString() const
	{
		uint8_t b[4];
		std::memcpy(b, &m_Int, 4);
		char s[16];
		std::snprintf(s, sizeof(s), "%u.%u.%u.%u", b[0], b[1], b[2], b[3]);
		return s;
	}
	bool operator==(const IPv4Address& o) const { return m_Int == o.m_Int; }
	bool operator!=(const IPv4Address& o) const { return m_Int != o.m_Int; }
	static const IPv4Address Zero;

private:
	uint32_t m_Int = 0;
};
inline const IPv4Address IPv4Address::Zero{};

/* An allocator whose resize() leaves new elements uninitialised: batch buffers are sized for the largest batch and
 * then filled by the reader / the engine, so zero-filling them first (256 MiB of packet buffer per read) would cost
 * more than the read itself. */
template <class T>
struct DefaultInitAllocator : std::allocator<T>
{
	template <class U>
	struct rebind
	{
		using other = DefaultInitAllocator<U>;
	};
	DefaultInitAllocator() = default;
	template <class U>
	DefaultInitAllocator(const DefaultInitAllocator<U>&) noexcept
	{}
	template <class U>
	void construct(U* p) noexcept(std::is_nothrow_default_constructible<U>::value)
	{
		::new (static_cast<void*>(p)) U;
	}
	template <class U, class... A>
	void construct(U* p, A&&... a)
	{
		::new (static_cast<void*>(p)) U(std::forward<A>(a)...);
	}
};
template <class T>
using buffer = std::vector<T, DefaultInitAllocator<T>>;

/* PacketParseOptions (Packet++/header/Packet.h:17-37) plus the engine's record options */
struct PacketParseOptions
{
	ProtocolTypeFamily parseUntilProtocol = UnknownProtocol;
	OsiModelLayer parseUntilLayer = OsiModelLayerUnknown;
	bool computeChecksums = true; /* IPv4 header + TCP/UDP checksum verification */
	uint8_t maxLayers = PCPPX_MAX_LAYERS;
	bool deepWindow = false;  /* PCPPX_WINDOW_DEEP: two-round 144-B header window for checksum launches over deep stacks */
	bool shortWindow = false; /* PCPPX_WINDOW_SHORT: one 96-B round for parse-only launches over plain stacks (ignored
	                             when deepWindow is set) */

	PacketParseOptions() = default;
	PacketParseOptions(ProtocolTypeFamily until, OsiModelLayer layer = OsiModelLayerUnknown)
	    : parseUntilProtocol(until), parseUntilLayer(layer)
	{}

	pcppx_opts toC() const
	{
		pcppx_opts o;
		pcppx_default_opts(&o);
		o.parse_until_family = parseUntilProtocol;
		o.parse_until_osi = parseUntilLayer;
		o.want_checksums = computeChecksums ? 1 : 0;
		o.max_layers = maxLayers;
		o.window = deepWindow ? PCPPX_WINDOW_DEEP : (shortWindow ? PCPPX_WINDOW_SHORT : PCPPX_WINDOW_DEFAULT);
		return o;
	}
};

/* ---- process-wide settings of the per-packet entry points ---- */
namespace detail
{
inline int& defaultDevice()
{
	static int d = 0;
	return d;
}
inline std::atomic<pcppx_host_parse_fn>& hostParser()
{
	static std::atomic<pcppx_host_parse_fn> f{ nullptr };
	return f;
}
inline std::atomic<bool>& pageChecksums()
{
	static std::atomic<bool> c{ false };
	return c;
}
}  // namespace detail

/* The GPU the per-packet entry points (readers, Packet(RawPacket*)) use; set before the first one runs. */
inline void setDefaultDevice(int device)
{
	detail::defaultDevice() = device;
}
/* The caller's own Packet++ parse of one packet (pcppx_host_parse_fn): completes the packets the
 * engine flags PCPPX_F_NEEDS_HOST before a Packet is built on them. nullptr = leave them flagged. */
inline void setHostParser(pcppx_host_parse_fn fn)
{
	detail::hostParser().store(fn);
}
/* Packet(RawPacket*, ...) computes no checksum in Packet++ (Packet.cpp:66-196), so the per-packet entry points parse
 * without them; with this set they also verify the IPv4 / TCP / UDP checksums (Packet::isIPv4ChecksumValid ... carry
 * the computed values). Set before the Packets it should apply to. */
inline void setPageChecksums(bool on)
{
	detail::pageChecksums().store(on);
}

class RawPacket;

namespace detail
{
/* Page-locked blocks for record pages, reused across pages and readers (pinning memory is slow). Blocks go back to
 * the pool when a page is released; at most kKeep bytes stay cached. The pool is never destroyed: the process may
 * outlive the HIP runtime's teardown at exit. */
class PinnedPool
{
public:
	static PinnedPool& instance()
	{
		static PinnedPool* p = new PinnedPool();
		return *p;
	}
	void* take(size_t bytes, size_t* got)
	{
		bytes = (bytes + kGrain - 1) & ~(kGrain - 1);
		{
			std::lock_guard<std::mutex> g(m_Mu);
			auto it = m_Free.lower_bound(bytes);
			if (it != m_Free.end() && it->first <= 2 * bytes)
			{
				void* p = it->second;
				*got = it->first;
				m_Cached -= it->first;
				m_Out += it->first;
				m_Free.erase(it);
				return p;
			}
		}
		void* p = pcppx_host_alloc(bytes);
		if (p == nullptr)
			throw Error(PCPPX_E_NOMEM, "pcppx_host_alloc");
		*got = bytes;
		m_Out += bytes;
		return p;
	}
	void give(void* p, size_t bytes)
	{
		if (p == nullptr)
			return;
		m_Out -= bytes;
		{
			std::lock_guard<std::mutex> g(m_Mu);
			if (m_Cached + bytes <= kKeep)
			{
				m_Free.emplace(bytes, p);
				m_Cached += bytes;
				return;
			}
		}
		pcppx_host_free(p);
	}

	/* page-locked bytes held by live record pages (taken and not given back) */
	size_t outstanding() const { return m_Out.load(); }

private:
	static constexpr size_t kGrain = 1u << 20;
	std::atomic<size_t> m_Out{ 0 };
	static constexpr size_t kKeep = 2ull << 30;
	std::mutex m_Mu;
	std::multimap<size_t, void*> m_Free;
	size_t m_Cached = 0;
};

/* The context the per-packet entry points parse on: one per process (device defaultDevice()), its calls serialised
 * (a pcppx context is used by one thread at a time; every entry point selects its device itself). Never destroyed,
 * like the pool. */
class Service
{
public:
	static Service& instance()
	{
		static Service* s = new Service(defaultDevice());
		return *s;
	}
	void parse(const pcppx_batch& b, const pcppx_opts& o, pcppx_records& r)
	{
		std::lock_guard<std::mutex> g(m_Mu);
		check(pcppx_parse_batch_host(m_Ctx, &b, &o, &r), "pcppx_parse_batch_host");
		++counter();
	}
	/* GPU parses the per-packet entry points have made (one per page, group or re-parse) */
	uint64_t parses() const { return counter().load(); }
	static uint64_t parsesSoFar() { return counter().load(); }  // without opening the device
	/* packets parsed and record bytes the parses brought back over PCIe (briefs / summaries + layer entries) */
	static void noteRecords(uint64_t packets, uint64_t bytes)
	{
		recordStats()[0] += packets;
		recordStats()[1] += bytes;
	}
	static uint64_t packetsParsed() { return recordStats()[0].load(); }
	static uint64_t recordBytes() { return recordStats()[1].load(); }

private:
	explicit Service(int device) { check(pcppx_open(device, &m_Ctx), "pcppx_open"); }
	static std::atomic<uint64_t>& counter()
	{
		static std::atomic<uint64_t> c{ 0 };
		return c;
	}
	static std::atomic<uint64_t>* recordStats()
	{
		static std::atomic<uint64_t> st[2] = { { 0 }, { 0 } };
		return st;
	}
	std::mutex m_Mu;
	pcppx_ctx* m_Ctx = nullptr;
};

/* Complete the packets the engine left to the host with fn (records at stride maxLayers); returns how many. */
inline size_t completeOnHost(pcppx_host_parse_fn fn, const uint8_t* data, const uint64_t* offsets,
                             const uint32_t* caplens, uint32_t n, uint16_t linkType, const pcppx_opts& o,
                             pcppx_summary* sum, pcppx_layer* lay)
{
	if (fn == nullptr || o.max_layers == 0)
		return 0;
	size_t done = 0;
	for (uint32_t i = 0; i < n; ++i)
	{
		pcppx_summary& s = sum[i];
		if (!(s.flags & PCPPX_F_NEEDS_HOST) || (s.flags & PCPPX_F_BAD_DESC))
			continue;
		check(fn(data + offsets[i], caplens[i], linkType, &o, &s, lay + (size_t)i * o.max_layers), "host parser");
		s.flags = (uint16_t)(s.flags | F_HOST_PARSED);
		++done;
	}
	return done;
}

/* Packet::parsePacket's options (Packet.cpp:66-196): what a page's records were parsed for (+ whether the checksums
 * were verified, setPageChecksums) */
struct ParseKey
{
	ProtocolTypeFamily family = UnknownProtocol;
	uint8_t osi = OsiModelLayerUnknown;
	bool csum = false;
	bool operator==(const ParseKey& o) const { return family == o.family && osi == o.osi && csum == o.csum; }
	/* the per-packet parse: every layer of the chain (PCPPX_MAX_LAYERS) in the DENSE layout, with the 16-B brief -- or
	 * the 32-B summary when checksums are verified (the computed values ride in it) */
	pcppx_opts opts() const
	{
		pcppx_opts o;
		pcppx_default_opts(&o);
		o.parse_until_family = family;
		o.parse_until_osi = osi;
		o.want_checksums = csum ? 1 : 0;
		o.layout = PCPPX_LAYOUT_DENSE;
		return o;
	}
};

/* one packet's complete records: a summary (proto_mask included) and its first PCPPX_MAX_LAYERS layers -- a packet the
 * host parser completed, one whose chain is deeper than the records hold, or a copied RawPacket's (the copy owns its
 * bytes and keeps no page alive, as a copied pcpp::RawPacket owns a copy of the bytes: RawPacket.cpp copyDataFrom) */
struct CopiedRecords
{
	ParseKey key;
	pcppx_summary sum{};
	pcppx_layer lay[PCPPX_MAX_LAYERS]{};
};

/* One page's records for one ParseKey (ABI 7): per packet the 16-B brief (or, checksums verified, the 32-B summary,
 * whose first half is the brief) and the chain's layer entries back to back (PCPPX_LAYOUT_DENSE: only the chains cross
 * PCIe, 50 B per config-3 packet), both DMA'd into page-locked memory; first[i] = packet i's first entry. Packets whose
 * records the chain alone cannot give -- completed by the host parser (F_HOST_PARSED) or deeper than PCPPX_MAX_LAYERS
 * (PCPPX_F_DEPTH_OVERFLOW: the protocol mask then covers layers the entries do not hold) -- carry complete records in
 * `side`, looked up by index. */
struct Records
{
	ParseKey key;
	uint32_t n = 0;
	pcppx_brief* brief = nullptr;   // n (the summaries' first halves when sum is set)
	pcppx_summary* sum = nullptr;   // n when key.csum
	pcppx_layer* lay = nullptr;     // the chains (up to n * PCPPX_MAX_LAYERS entries)
	std::unique_ptr<uint32_t[]> first;
	uint64_t entries = 0;           // layers_written
	std::vector<uint32_t> sideIdx;  // ascending
	std::vector<CopiedRecords> side;

	Records(ParseKey k, uint32_t count) : key(k), n(count), first(new uint32_t[count ? count : 1])
	{
		const size_t head = (size_t)n * (k.csum ? sizeof(pcppx_summary) : sizeof(pcppx_brief));
		m_Block = PinnedPool::instance().take(head + (size_t)n * PCPPX_MAX_LAYERS * sizeof(pcppx_layer), &m_Bytes);
		if (k.csum)
			sum = static_cast<pcppx_summary*>(m_Block);
		brief = static_cast<pcppx_brief*>(m_Block);  // stride: briefOf()
		lay = reinterpret_cast<pcppx_layer*>(static_cast<uint8_t*>(m_Block) + head);
	}
	~Records() { PinnedPool::instance().give(m_Block, m_Bytes); }
	Records(const Records&) = delete;
	Records& operator=(const Records&) = delete;

	const pcppx_brief* briefOf(uint32_t i) const
	{
		return sum ? reinterpret_cast<const pcppx_brief*>(sum + i) : brief + i;
	}
	pcppx_brief* briefOf(uint32_t i) { return sum ? reinterpret_cast<pcppx_brief*>(sum + i) : brief + i; }
	const CopiedRecords* sideFor(uint32_t i) const
	{
		auto it = std::lower_bound(sideIdx.begin(), sideIdx.end(), i);
		return it != sideIdx.end() && *it == i ? &side[(size_t)(it - sideIdx.begin())] : nullptr;
	}
	/* packet i's complete records (a copy's): the side entry, or the summary / the brief + the chain's mask */
	void complete(uint32_t i, CopiedRecords* c) const
	{
		if (const CopiedRecords* s = sideFor(i))
		{
			*c = *s;
			return;
		}
		c->key = key;
		const pcppx_brief* b = briefOf(i);
		const uint32_t cnt = b->n_layers < PCPPX_MAX_LAYERS ? b->n_layers : PCPPX_MAX_LAYERS;
		std::memset(c->lay, 0, sizeof(c->lay));
		std::memcpy(c->lay, lay + first[i], cnt * sizeof(pcppx_layer));
		if (sum != nullptr)
			c->sum = sum[i];
		else
		{
			c->sum = pcppx_summary{};
			std::memcpy(&c->sum, b, sizeof(pcppx_brief));
			c->sum.proto_mask = pcppx_chain_proto_mask(c->lay, cnt);
		}
	}

private:
	void* m_Block = nullptr;
	size_t m_Bytes = 0;
};

/* the capture map: closed when the reader and every page of it are gone */
struct MapHandle
{
	pcppx_pcap* reader = nullptr;
	~MapHandle() { pcppx_pcap_close(reader); }
};

class ReaderCore;

/* A run of consecutive packets of one capture and one link type, pointing into the map, with its GPU records -- or
 * (a group, `group` set) the caller's own RawPackets of one link type that were parsed together: base is the lowest
 * of their byte addresses and offsets[i] the distance of packet i's bytes from it (a gapped batch, legal in
 * pcppx_batch). A group member that is released or given other bytes leaves the group: its caplen becomes 0 under
 * groupMu, so a later parse of the group (other options) never reads bytes the caller has freed. */
struct Page
{
	std::shared_ptr<MapHandle> map;  // keeps the bytes valid (reader pages)
	std::weak_ptr<ReaderCore> core;  // the reader, to learn the parse options from the caller's Packets
	bool group = false;
	mutable std::mutex groupMu;      // a group's parse vs. its members leaving
	const uint8_t* base = nullptr;
	uint64_t dataLen = 0;
	uint16_t linkType = LINKTYPE_ETHERNET;
	uint32_t n = 0;
	buffer<uint64_t> offsets, tsNs;
	buffer<uint32_t> caplens, frameLens;

	/* records for the reader's options, published once (acquire / release); 0 mapped, 1 parsing, 2 parsed */
	std::atomic<const Records*> primary{ nullptr };
	std::atomic<int> state{ 0 };
	int error = PCPPX_OK;
	std::mutex mu;
	std::condition_variable cv;
	std::unique_ptr<Records> primaryOwned;
	std::vector<std::unique_ptr<Records>> extra;  // records for other options (a Packet that asked for them)

	std::unique_ptr<Records> parseRecords(ParseKey k) const
	{
		auto r = std::make_unique<Records>(k, n);
		const pcppx_opts o = k.opts();
		const pcppx_batch b{ base, offsets.data(), caplens.data(), dataLen, n, linkType, 0 };
		pcppx_records rec{};
		if (k.csum)
			rec.summary = r->sum;
		else
			rec.brief = r->brief;
		rec.layers = r->lay;
		Service::instance().parse(b, o, rec);
		r->entries = rec.layers_written;
		Service::noteRecords(n, (uint64_t)n * (k.csum ? sizeof(pcppx_summary) : sizeof(pcppx_brief)) +
		                            rec.layers_written * sizeof(pcppx_layer));
		// each chain's first entry; the packets that need complete records beside the chain
		std::vector<uint32_t> deep, host;
		const pcppx_host_parse_fn fn = hostParser().load();
		uint32_t pos = 0;
		for (uint32_t i = 0; i < n; ++i)
		{
			r->first[i] = pos;
			const pcppx_brief* bi = r->briefOf(i);
			pos += bi->n_layers < PCPPX_MAX_LAYERS ? bi->n_layers : PCPPX_MAX_LAYERS;
			if (fn != nullptr && (bi->flags & PCPPX_F_NEEDS_HOST) && !(bi->flags & PCPPX_F_BAD_DESC))
				host.push_back(i);
			else if (!k.csum && (bi->flags & PCPPX_F_DEPTH_OVERFLOW))
				deep.push_back(i);
		}
		if (pos != r->entries)
			throw Error(PCPPX_E_HIP, "page records: chain entries do not add up");
		completeSide(*r, k, deep, host, fn);
		return r;
	}
	/* complete records of the few packets the chain alone does not describe: chains deeper than the records (their
	 * summaries from one small FIXED parse of just those packets), and packets the host parser completes */
	void completeSide(Records& r, ParseKey k, const std::vector<uint32_t>& deep, const std::vector<uint32_t>& host,
	                  pcppx_host_parse_fn fn) const
	{
		std::vector<uint32_t> all;
		std::merge(deep.begin(), deep.end(), host.begin(), host.end(), std::back_inserter(all));
		if (all.empty())
			return;
		r.sideIdx = all;
		r.side.resize(all.size());
		pcppx_opts o = k.opts();
		o.layout = PCPPX_LAYOUT_FIXED;
		if (!deep.empty())
		{
			buffer<uint64_t> off(deep.size());
			buffer<uint32_t> cap(deep.size());
			for (size_t j = 0; j < deep.size(); ++j)
			{
				off[j] = offsets[deep[j]];
				cap[j] = caplens[deep[j]];
			}
			std::vector<pcppx_summary> ds(deep.size());
			std::vector<pcppx_layer> dl(deep.size() * PCPPX_MAX_LAYERS);
			const pcppx_batch b{ base, off.data(), cap.data(), dataLen, (uint32_t)deep.size(), linkType, 0 };
			pcppx_records rec{};
			rec.summary = ds.data();
			rec.layers = dl.data();
			Service::instance().parse(b, o, rec);
			Service::noteRecords(0, deep.size() * (sizeof(pcppx_summary) + PCPPX_MAX_LAYERS * sizeof(pcppx_layer)));
			for (size_t j = 0; j < deep.size(); ++j)
			{
				CopiedRecords& c = r.side[(size_t)(std::lower_bound(all.begin(), all.end(), deep[j]) - all.begin())];
				c.key = k;
				c.sum = ds[j];
				std::memcpy(c.lay, dl.data() + j * PCPPX_MAX_LAYERS, sizeof(c.lay));
			}
		}
		for (uint32_t i : host)
		{
			CopiedRecords& c = r.side[(size_t)(std::lower_bound(all.begin(), all.end(), i) - all.begin())];
			c.key = k;
			std::memset(&c.sum, 0, sizeof(c.sum));
			check(fn(base + offsets[i], caplens[i], linkType, &o, &c.sum, c.lay), "host parser");
			c.sum.flags = (uint16_t)(c.sum.flags | F_HOST_PARSED);
			pcppx_brief* bi = r.briefOf(i);
			bi->flags = (uint16_t)(bi->flags | F_HOST_PARSED);  // Packet: look the packet up in `side`
		}
	}
	/* parse for k unless another thread has started: false if it has */
	bool tryParse(ParseKey k)
	{
		int idle = 0;
		if (!state.compare_exchange_strong(idle, 1))
			return false;
		std::unique_ptr<Records> r;
		int err = PCPPX_OK;
		try
		{
			r = parseRecords(k);
		}
		catch (const Error& e)
		{
			err = e.code();
		}
		catch (const std::bad_alloc&)
		{
			err = PCPPX_E_NOMEM;
		}
		{
			std::lock_guard<std::mutex> g(mu);
			primaryOwned = std::move(r);
			error = err;
			primary.store(primaryOwned.get(), std::memory_order_release);
			state.store(2);
		}
		cv.notify_all();
		return true;
	}
	/* the records for k (Packet's slow path: the page not parsed yet, or parsed for other options) */
	const Records* recordsFor(ParseKey k);
};

/* The reader's pipeline: a mapper thread indexes pages ahead of the caller, a parser thread parses them on the GPU
 * once the caller's parse options are known. */
class ReaderCore : public std::enable_shared_from_this<ReaderCore>
{
public:
	static constexpr size_t kAhead = 2;  // pages mapped ahead of the caller's
	// packets in the first page, then x4 per page up to kMaxPage. A capture of kLargeCapture bytes or more starts with
	// 1k packets, so the caller starts on a small parse while the next pages are parsed (first pass over a 1M-packet
	// IMIX pcap 70 vs 87 ms, r06y_dropin_*.json); a smaller one with 16k, so that it takes one GPU round trip, not
	// three (the drop-in benchmark.cpp on config 1's 10k-packet pcap 1.19 vs 1.98 ms, on example.pcap 0.86 vs 1.20 ms)
	static constexpr uint32_t kFirstPageSmall = 1u << 14, kFirstPageLarge = 1u << 10;
	static constexpr uint64_t kLargeCapture = 32ull << 20;
	static constexpr uint32_t kMaxPage = 1u << 20;

	ReaderCore(pcppx_pcap* r, uint64_t fileBytes)
	    : m_Map(std::make_shared<MapHandle>()), m_FirstPage(fileBytes >= kLargeCapture ? kFirstPageLarge : kFirstPageSmall)
	{
		m_Map->reader = r;
	}
	~ReaderCore() { stop(); }
	ReaderCore(const ReaderCore&) = delete;
	ReaderCore& operator=(const ReaderCore&) = delete;

	void start()
	{
		m_Mapper = std::thread([this] { mapLoop(); });
		m_Parser = std::thread([this] { parseLoop(); });
	}
	void stop()
	{
		{
			std::lock_guard<std::mutex> g(m_Mu);
			m_Stop = true;
		}
		m_Cv.notify_all();
		if (m_Mapper.joinable())
			m_Mapper.join();
		if (m_Parser.joinable())
			m_Parser.join();
		std::lock_guard<std::mutex> g(m_Mu);
		m_Pages.clear();
		m_ToParse.clear();
	}
	/* the next page in capture order; nullptr at the end of the capture (or after a read error: error()) */
	std::shared_ptr<Page> nextPage()
	{
		std::unique_lock<std::mutex> g(m_Mu);
		m_Cv.wait(g, [&] { return !m_Pages.empty() || m_Eof || m_Stop; });
		if (m_Pages.empty())
			return nullptr;
		std::shared_ptr<Page> p = std::move(m_Pages.front());
		m_Pages.pop_front();
		g.unlock();
		m_Cv.notify_all();
		return p;
	}
	/* the caller built a Packet with these options: parse the following pages for them */
	void learn(ParseKey k)
	{
		{
			std::lock_guard<std::mutex> g(m_Mu);
			if (m_KeyKnown && m_Key == k)
				return;
			m_Key = k;
			m_KeyKnown = true;
		}
		m_Cv.notify_all();
	}
	int error() const
	{
		std::lock_guard<std::mutex> g(m_Mu);
		return m_Error;
	}

private:
	void mapLoop()
	{
		uint32_t size = m_FirstPage;
		for (;;)
		{
			{
				std::unique_lock<std::mutex> g(m_Mu);
				m_Cv.wait(g, [&] { return m_Stop || m_Pages.size() < kAhead; });
				if (m_Stop)
					return;
			}
			auto pg = std::make_shared<Page>();
			int rc = PCPPX_OK;
			uint32_t n = 0;
			try
			{
				pg->map = m_Map;
				pg->core = weak_from_this();
				pg->offsets.resize(size);
				pg->tsNs.resize(size);
				pg->caplens.resize(size);
				pg->frameLens.resize(size);
				rc = pcppx_pcap_map_batch(m_Map->reader, &pg->base, &pg->dataLen, pg->offsets.data(), pg->caplens.data(),
				                          pg->frameLens.data(), pg->tsNs.data(), size, &n);
			}
			catch (const std::bad_alloc&)
			{
				rc = PCPPX_E_NOMEM;
			}
			std::lock_guard<std::mutex> g(m_Mu);
			if (rc != PCPPX_OK || n == 0)
			{
				m_Error = rc;
				m_Eof = true;
				m_Cv.notify_all();
				return;
			}
			pg->n = n;
			pg->linkType = (uint16_t)pcppx_pcap_linktype(m_Map->reader);
			m_Pages.push_back(pg);
			m_ToParse.push_back(pg);
			m_Cv.notify_all();
			size = size < kMaxPage / 4 ? size * 4 : kMaxPage;
		}
	}
	void parseLoop()
	{
		for (;;)
		{
			std::shared_ptr<Page> pg;
			ParseKey k;
			{
				std::unique_lock<std::mutex> g(m_Mu);
				m_Cv.wait(g, [&] { return m_Stop || (m_KeyKnown && !m_ToParse.empty()); });
				if (m_Stop)
					return;
				pg = m_ToParse.front().lock();  // expired: the caller is done with the page
				m_ToParse.pop_front();
				k = m_Key;
			}
			if (pg)
				(void)pg->tryParse(k);
		}
	}

	std::shared_ptr<MapHandle> m_Map;
	const uint32_t m_FirstPage;
	mutable std::mutex m_Mu;
	std::condition_variable m_Cv;
	std::deque<std::shared_ptr<Page>> m_Pages;   // mapped, not yet handed to the caller
	std::deque<std::weak_ptr<Page>> m_ToParse;   // mapped, not yet parsed (in capture order)
	bool m_Eof = false, m_Stop = false, m_KeyKnown = false;
	ParseKey m_Key;
	int m_Error = PCPPX_OK;
	std::thread m_Mapper, m_Parser;
};

inline const Records* Page::recordsFor(ParseKey k)
{
	const Records* r = primary.load(std::memory_order_acquire);
	if (r != nullptr && r->key == k)
		return r;
	if (auto c = core.lock())
		c->learn(k);  // the next pages are parsed for k
	if (state.load() != 2 && !tryParse(k))
	{
		std::unique_lock<std::mutex> g(mu);
		cv.wait(g, [&] { return state.load() == 2; });
	}
	std::lock_guard<std::mutex> g(mu);
	if (error != PCPPX_OK)
		throw Error(error, "parse of a capture page");
	r = primary.load(std::memory_order_acquire);
	if (r != nullptr && r->key == k)
		return r;
	// parsed for other options: parse the page again for these, kept beside the first records
	for (const auto& e : extra)
		if (e->key == k)
			return e.get();
	std::unique_lock<std::mutex> gl(groupMu, std::defer_lock);
	if (group)
		gl.lock();  // the members still alive: a released member's caplen is 0
	extra.push_back(parseRecords(k));
	return extra.back().get();
}

/* The caller's own RawPackets (not from a reader) that no Packet has been built on yet. The first Packet built on
 * one of them parses every pending RawPacket in one GPU batch per link type (a group, above), so that a caller
 * that fills a RawPacketVector itself and then builds Packets on it -- BM_PacketPureParsing's pattern,
 * Examples/PcapPlusPlus-benchmark/benchmark-google.cpp:231-260 -- pays one GPU round trip for the whole vector, not
 * one per packet. The mutex guards the pending list and the group membership fields of registered RawPackets. */
class OwnedRegistry
{
public:
	static OwnedRegistry& instance()
	{
		static OwnedRegistry* r = new OwnedRegistry();  // never destroyed, like the Service
		return *r;
	}
	inline void add(RawPacket* r);
	inline void remove(RawPacket* r);
	/* the group and index of r's records for k (r is registered; parses the pending RawPackets if r is one) */
	inline const Records* recordsFor(RawPacket* r, ParseKey k, uint32_t* index);

private:
	static constexpr size_t npos = ~(size_t)0;
	std::mutex m_Mu;
	std::vector<RawPacket*> m_Pending;  // nullptr: removed since
	size_t m_Removed = 0;
	inline void compact();
};
}  // namespace detail

/* pcpp::RawPacket (Packet++/header/RawPacket.h:288-566): a packet's bytes, lengths, timestamp and link type.
 * A RawPacket filled by a reader (getNextPacket / getNextPackets) refers to the packet's bytes in the reader's memory
 * map and to the page of GPU records they were parsed into; it keeps both alive (no copy is made). One made from the
 * caller's bytes (the constructors / setRawData) owns them when takeOwnership is set, as in the reference, and is
 * parsed on the GPU together with the caller's other pending RawPackets when the first Packet is built on one of them
 * (detail::OwnedRegistry). A copy owns a copy of the bytes and of the packet's records, never the page (RawPacket.cpp
 * copyDataFrom). The bytes are read-only (packet crafting is outside the engine). */
class RawPacket
{
public:
	RawPacket() = default;
	RawPacket(const uint8_t* pRawData, int rawDataLen, timeval timestamp, bool takeOwnership,
	          LinkLayerType layerType = LINKTYPE_ETHERNET)
	{
		setRawData(pRawData, rawDataLen, takeOwnership, timestamp, layerType);
	}
	RawPacket(const uint8_t* pRawData, int rawDataLen, timespec timestamp, bool takeOwnership,
	          LinkLayerType layerType = LINKTYPE_ETHERNET)
	{
		setRawData(pRawData, rawDataLen, takeOwnership, timestamp, layerType);
	}
	virtual ~RawPacket() { release(); }
	RawPacket(const RawPacket& other) { copyFrom(other); }
	RawPacket& operator=(const RawPacket& other)
	{
		if (this != &other)
		{
			release();
			copyFrom(other);
		}
		return *this;
	}
	virtual RawPacket* clone() const { return new RawPacket(*this); }

	bool setRawData(const uint8_t* pRawData, int rawDataLen, bool takeOwnership, timeval timestamp,
	                LinkLayerType layerType = LINKTYPE_ETHERNET, int frameLength = -1)
	{
		return setRawData(pRawData, rawDataLen, takeOwnership,
		                  timespec{ timestamp.tv_sec, (long)timestamp.tv_usec * 1000 }, layerType, frameLength);
	}
	bool setRawData(const uint8_t* pRawData, int rawDataLen, bool takeOwnership, timespec timestamp,
	                LinkLayerType layerType = LINKTYPE_ETHERNET, int frameLength = -1)
	{
		release();
		m_RawData = pRawData;
		m_RawDataLen = rawDataLen;
		m_FrameLength = frameLength == -1 ? rawDataLen : frameLength;
		m_TsNs = (uint64_t)timestamp.tv_sec * 1000000000ull + (uint64_t)timestamp.tv_nsec;
		m_OwnsRawData = takeOwnership;
		m_LinkLayerType = layerType;
		m_RawPacketSet = true;
		if (m_RawData != nullptr)
			detail::OwnedRegistry::instance().add(this);
		return true;
	}

	const uint8_t* getRawData() const { return m_RawData; }
	int getRawDataLen() const { return m_RawDataLen; }
	int getFrameLength() const { return m_FrameLength; }
	LinkLayerType getLinkLayerType() const { return m_LinkLayerType; }
	timespec getPacketTimeStamp() const
	{
		return timespec{ (time_t)(m_TsNs / 1000000000ull), (long)(m_TsNs % 1000000000ull) };
	}
	bool isPacketSet() const { return m_RawPacketSet; }
	virtual void clear() { release(); }

private:
	friend class PcapFileReaderDevice;
	friend class Packet;
	friend class detail::OwnedRegistry;

	void release()
	{
		if (m_Registered)
			detail::OwnedRegistry::instance().remove(this);
		if (m_OwnsRawData)
			delete[] m_RawData;
		m_RawData = nullptr;
		m_RawDataLen = m_FrameLength = 0;
		m_TsNs = 0;
		m_OwnsRawData = m_RawPacketSet = false;
		m_Page.reset();
		m_Index = 0;
		m_Copied.reset();
	}
	/* the records of this packet for its page's parse options, if that page has been parsed */
	std::shared_ptr<const detail::CopiedRecords> copyRecords() const
	{
		if (m_Copied != nullptr)
			return m_Copied;
		if (m_Registered || m_Page == nullptr)
			return nullptr;  // the caller's own bytes: a group's fields are written under the registry's lock
		const detail::Records* r = m_Page->primary.load(std::memory_order_acquire);
		if (r == nullptr)
			return nullptr;
		auto c = std::make_shared<detail::CopiedRecords>();
		r->complete(m_Index, c.get());
		return c;
	}
	void copyFrom(const RawPacket& o)
	{
		m_RawDataLen = o.m_RawDataLen;
		m_FrameLength = o.m_FrameLength;
		m_TsNs = o.m_TsNs;
		m_LinkLayerType = o.m_LinkLayerType;
		m_RawPacketSet = o.m_RawPacketSet;
		if (o.m_RawData == nullptr)
			return;
		uint8_t* copy = new uint8_t[o.m_RawDataLen > 0 ? o.m_RawDataLen : 1];
		std::memcpy(copy, o.m_RawData, o.m_RawDataLen > 0 ? (size_t)o.m_RawDataLen : 0);
		m_RawData = copy;
		m_OwnsRawData = true;
		m_Copied = o.copyRecords();
		detail::OwnedRegistry::instance().add(this);
	}
	/* getNextPacket's per-packet step: point at packet i of a page (the page pointer changes once per page) */
	void setFromPage(const std::shared_ptr<detail::Page>& pg, uint32_t i)
	{
		if (m_Registered || m_Copied != nullptr || (m_Page != nullptr && m_Page->group))
		{
			release();
		}
		else if (m_OwnsRawData)
		{
			delete[] m_RawData;
			m_OwnsRawData = false;
		}
		if (m_Page.get() != pg.get())
			m_Page = pg;
		const detail::Page& p = *pg;
		m_Index = i;
		m_RawData = p.base + p.offsets[i];
		m_RawDataLen = (int)p.caplens[i];
		m_FrameLength = (int)p.frameLens[i];
		m_TsNs = p.tsNs[i];
		m_LinkLayerType = p.linkType;
		m_RawPacketSet = true;
	}

	const uint8_t* m_RawData = nullptr;
	int m_RawDataLen = 0;
	int m_FrameLength = 0;
	uint64_t m_TsNs = 0;
	bool m_OwnsRawData = false;
	bool m_RawPacketSet = false;
	bool m_Registered = false;  // the caller's own bytes: in detail::OwnedRegistry (pending or in a group)
	LinkLayerType m_LinkLayerType = LINKTYPE_ETHERNET;
	std::shared_ptr<detail::Page> m_Page;  // a reader's page, or (registered) the group this packet was parsed in
	uint32_t m_Index = 0;
	size_t m_PendingSlot = ~(size_t)0;                   // registered, not yet parsed: the pending-list slot
	std::shared_ptr<const detail::CopiedRecords> m_Copied;  // records copied with the bytes (copy constructor)
};

namespace detail
{
inline void OwnedRegistry::add(RawPacket* r)
{
	std::lock_guard<std::mutex> g(m_Mu);
	r->m_Registered = true;
	r->m_PendingSlot = m_Pending.size();
	m_Pending.push_back(r);
}

inline void OwnedRegistry::compact()
{
	size_t w = 0;
	for (RawPacket* p : m_Pending)
		if (p != nullptr)
		{
			p->m_PendingSlot = w;
			m_Pending[w++] = p;
		}
	m_Pending.resize(w);
	m_Removed = 0;
}

inline void OwnedRegistry::remove(RawPacket* r)
{
	std::shared_ptr<Page> grp;
	uint32_t idx = 0;
	{
		std::lock_guard<std::mutex> g(m_Mu);
		if (r->m_PendingSlot != npos)
		{
			m_Pending[r->m_PendingSlot] = nullptr;
			if (++m_Removed > 4096 && m_Removed * 2 > m_Pending.size())
				compact();
		}
		r->m_PendingSlot = npos;
		r->m_Registered = false;
		if (r->m_Page != nullptr && r->m_Page->group)
		{
			grp = std::move(r->m_Page);
			idx = r->m_Index;
		}
	}
	if (grp != nullptr)
	{
		std::lock_guard<std::mutex> gl(grp->groupMu);  // waits for a parse of the group in flight
		grp->caplens[idx] = 0;
	}
}

inline const Records* OwnedRegistry::recordsFor(RawPacket* r, ParseKey k, uint32_t* index)
{
	std::shared_ptr<Page> grp;
	std::vector<std::shared_ptr<Page>> fresh;  // groups made here, parsed below (their groupMu held)
	{
		std::lock_guard<std::mutex> g(m_Mu);
		if (r->m_PendingSlot != npos)
		{
			// every pending RawPacket -> one group per link type, in the order they were registered
			std::map<LinkLayerType, std::vector<RawPacket*>> byType;
			for (RawPacket* p : m_Pending)
				if (p != nullptr)
					byType[p->m_LinkLayerType].push_back(p);
			m_Pending.clear();
			m_Removed = 0;
			for (auto& kv : byType)
			{
				auto pg = std::make_shared<Page>();
				pg->group = true;
				pg->linkType = kv.first;
				const std::vector<RawPacket*>& mem = kv.second;
				uintptr_t lo = ~(uintptr_t)0, hi = 0;
				for (RawPacket* p : mem)
				{
					const uintptr_t a = reinterpret_cast<uintptr_t>(p->m_RawData);
					const uint32_t len = p->m_RawDataLen > 0 ? (uint32_t)p->m_RawDataLen : 0;
					lo = a < lo ? a : lo;
					hi = a + len > hi ? a + len : hi;
				}
				pg->n = (uint32_t)mem.size();
				pg->base = reinterpret_cast<const uint8_t*>(lo);
				pg->dataLen = hi - lo;
				pg->offsets.resize(mem.size());
				pg->caplens.resize(mem.size());
				for (uint32_t i = 0; i < pg->n; ++i)
				{
					RawPacket* p = mem[i];
					pg->offsets[i] = reinterpret_cast<uintptr_t>(p->m_RawData) - lo;
					pg->caplens[i] = p->m_RawDataLen > 0 ? (uint32_t)p->m_RawDataLen : 0;
					p->m_Page = pg;
					p->m_Index = i;
					p->m_PendingSlot = npos;
				}
				pg->state.store(1);  // parsed below; a Packet on another member waits for it
				pg->groupMu.lock();
				fresh.push_back(std::move(pg));
			}
		}
		grp = r->m_Page;
		*index = r->m_Index;
	}
	for (auto& pg : fresh)
	{
		std::unique_ptr<Records> rec;
		int err = PCPPX_OK;
		try
		{
			rec = pg->parseRecords(k);
		}
		catch (const Error& e)
		{
			err = e.code();
		}
		catch (const std::bad_alloc&)
		{
			err = PCPPX_E_NOMEM;
		}
		pg->groupMu.unlock();
		{
			std::lock_guard<std::mutex> g(pg->mu);
			pg->primaryOwned = std::move(rec);
			pg->error = err;
			pg->primary.store(pg->primaryOwned.get(), std::memory_order_release);
			pg->state.store(2);
		}
		pg->cv.notify_all();
	}
	const Records* rec = grp->primary.load(std::memory_order_acquire);
	if (rec != nullptr && rec->key == k)
		return rec;
	return grp->recordsFor(k);
}
}  // namespace detail

/* pcpp::PointerVector (Common++/header/PointerVector.h:44-350): a vector of owned pointers; the elements are freed
 * when removed or when the vector is destroyed, and a copy of the vector copies the elements (clone() for polymorphic
 * ones). */
template <typename T, typename Deleter = std::default_delete<T>>
class PointerVector
{
public:
	using VectorIterator = typename std::vector<T*>::iterator;
	using ConstVectorIterator = typename std::vector<T*>::const_iterator;

	PointerVector() = default;
	PointerVector(const PointerVector& other) : m_Vector(deepCopy(other.m_Vector)) {}
	PointerVector(PointerVector&& other) noexcept : m_Vector(std::move(other.m_Vector)) { other.m_Vector.clear(); }
	~PointerVector() { freeAll(); }
	PointerVector& operator=(const PointerVector& other)
	{
		if (this != &other)
		{
			std::vector<T*> copy = deepCopy(other.m_Vector);
			freeAll();
			m_Vector = std::move(copy);
		}
		return *this;
	}
	PointerVector& operator=(PointerVector&& other) noexcept
	{
		if (this != &other)
		{
			freeAll();
			m_Vector = std::move(other.m_Vector);
			other.m_Vector.clear();
		}
		return *this;
	}

	void clear()
	{
		freeAll();
		m_Vector.clear();
	}
	void pushBack(std::nullptr_t, bool = true) = delete;
	/* takes ownership of element (freed here if the push fails and freeElementOnError is set) */
	void pushBack(T* element, bool freeElementOnError = true)
	{
		if (element == nullptr)
			throw std::invalid_argument("Element is nullptr");
		try
		{
			m_Vector.push_back(element);
		}
		catch (const std::exception&)
		{
			if (freeElementOnError)
				Deleter()(element);
			throw;
		}
	}
	void pushBack(std::unique_ptr<T> element)
	{
		if (!element)
			throw std::invalid_argument("Element is nullptr");
		m_Vector.push_back(element.get());
		element.release();
	}
	VectorIterator begin() { return m_Vector.begin(); }
	ConstVectorIterator begin() const { return m_Vector.begin(); }
	VectorIterator end() { return m_Vector.end(); }
	ConstVectorIterator end() const { return m_Vector.end(); }
	size_t size() const { return m_Vector.size(); }
	size_t capacity() const { return m_Vector.capacity(); }
	void reserve(size_t newSize) { m_Vector.reserve(newSize); }
	T* front() const { return m_Vector.front(); }
	T* back() const { return m_Vector.back(); }
	/* frees the element at position; returns the iterator after it */
	VectorIterator erase(VectorIterator position)
	{
		Deleter()(*position);
		return m_Vector.erase(position);
	}
	VectorIterator erase(ConstVectorIterator first, ConstVectorIterator last)
	{
		for (auto it = first; it != last; ++it)
			Deleter()(*it);
		return m_Vector.erase(first, last);
	}
	/* removes the element at position without freeing it (the caller owns it); position moves to the next one */
	T* getAndRemoveFromVector(VectorIterator& position)
	{
		T* result = *position;
		position = m_Vector.erase(position);
		return result;
	}
	std::unique_ptr<T> getAndDetach(size_t index)
	{
		auto it = m_Vector.begin() + (std::ptrdiff_t)index;
		return getAndDetach(it);
	}
	std::unique_ptr<T> getAndDetach(VectorIterator& position)
	{
		std::unique_ptr<T> result(*position);
		position = m_Vector.erase(position);
		return result;
	}
	std::unique_ptr<T> getAndDetach(const VectorIterator& position)
	{
		std::unique_ptr<T> result(*position);
		m_Vector.erase(position);
		return result;
	}
	T* at(int index) const { return m_Vector.at((size_t)index); }
	T** data() { return m_Vector.data(); }

private:
	template <class U>
	static auto copyOne(const U& obj, int) -> decltype(obj.clone(), (U*)nullptr)
	{
		return obj.clone();
	}
	template <class U>
	static U* copyOne(const U& obj, long)
	{
		return new U(obj);
	}
	static std::vector<T*> deepCopy(const std::vector<T*>& src)
	{
		std::vector<T*> out;
		out.reserve(src.size());
		try
		{
			for (T* p : src)
				out.push_back(copyOne<T>(*p, 0));
		}
		catch (...)
		{
			for (T* p : out)
				Deleter()(p);
			throw;
		}
		return out;
	}
	void freeAll()
	{
		for (T* p : m_Vector)
			Deleter()(p);
	}
	std::vector<T*> m_Vector;
};

/* pcpp::RawPacketVector (Pcap++/header/Device.h:14): what IFileReaderDevice::getNextPackets fills */
using RawPacketVector = PointerVector<RawPacket>;

/* A batch of raw packets back to back in one buffer: packet i = data[offsets[i], offsets[i] + caplens[i]). The batch
 * API's container (Engine::parse / Engine::filter, PcapFileReaderDevice::getNextBatch): one copy of the bytes in
 * one buffer, the shape pcppx_batch takes. */
struct RawBatch
{
	buffer<uint8_t> data;
	buffer<uint64_t> offsets;
	buffer<uint32_t> caplens;
	buffer<uint64_t> timestampsNs;
	buffer<uint32_t> frameLens; /* RawPacket::getFrameLength (original wire length) */
	uint16_t linkType = LINKTYPE_ETHERNET;

	size_t size() const { return caplens.size(); }
	void clear()
	{
		data.clear();
		offsets.clear();
		caplens.clear();
		timestampsNs.clear();
		frameLens.clear();
	}
	/* RawPacket::setRawData-style append (Packet++/header/RawPacket.h) */
	void add(const uint8_t* bytes, uint32_t len, uint64_t tsNs = 0, uint32_t frameLen = 0)
	{
		offsets.push_back(data.size());
		caplens.push_back(len);
		timestampsNs.push_back(tsNs);
		frameLens.push_back(frameLen ? frameLen : len);
		data.insert(data.end(), bytes, bytes + len);
	}
	const uint8_t* packetData(size_t i) const { return data.data() + offsets[i]; }
	pcppx_batch toC() const
	{
		return pcppx_batch{ data.data(), offsets.data(), caplens.data(), data.size(), (uint32_t)caplens.size(),
			                linkType, 0 };
	}
};

/* PcapFileReaderDevice / PcapNgFileReaderDevice (Pcap++/header/PcapFileDevice.h): the format (pcap or pcapng) comes
 * from the file's first bytes (IFileReaderDevice::createReader, PcapFileDevice.cpp:546-583). open() starts the
 * page pipeline (see the top of this file); close() stops it (RawPackets already read stay valid). */
class PcapFileReaderDevice
{
public:
	explicit PcapFileReaderDevice(std::string fileName) : m_FileName(std::move(fileName)) {}
	~PcapFileReaderDevice() { close(); }
	PcapFileReaderDevice(const PcapFileReaderDevice&) = delete;
	PcapFileReaderDevice& operator=(const PcapFileReaderDevice&) = delete;

	/* PcapFileReaderDevice::open (PcapFileDevice.cpp:707-768): false when already open or the file is not a
	 * readable pcap / pcapng capture */
	bool open()
	{
		if (m_Core != nullptr)
			return false;  // "File already opened"
		pcppx_pcap* r = nullptr;
		if (pcppx_pcap_open(m_FileName.c_str(), &r) != PCPPX_OK)
			return false;
		m_OpenLinkType = (LinkLayerType)pcppx_pcap_linktype(r);
		std::ifstream f(m_FileName, std::ifstream::ate | std::ifstream::binary);
		const std::streamoff bytes = f ? (std::streamoff)f.tellg() : 0;
		m_Core = std::make_shared<detail::ReaderCore>(r, bytes > 0 ? (uint64_t)bytes : 0u);
		m_Core->start();
		return true;
	}
	bool isOpened() const { return m_Core != nullptr; }
	void close()
	{
		if (m_Core != nullptr)
			m_Core->stop();
		m_Core.reset();
		m_Cur.reset();
		m_Pos = 0;
	}
	/* the link type of the packets being read (before the first packet: of the first packet) */
	LinkLayerType getLinkLayerType() const { return m_Cur ? m_Cur->linkType : m_OpenLinkType; }
	const std::string& getFileName() const { return m_FileName; }

	/* IFileReaderDevice::getNextPacket (PcapFileDevice.cpp:770-792): false at the end of the capture, on a read
	 * error, or when the reader is not open */
	bool getNextPacket(RawPacket& rawPacket)
	{
		if (m_Cur == nullptr || m_Pos >= m_Cur->n)
		{
			if (!advance())
				return false;
		}
		rawPacket.setFromPage(m_Cur, m_Pos++);
		return true;
	}

	/* DpdkDevice::receivePackets(MBufRawPacket**, ...) (Pcap++/src/DpdkDevice.cpp:922-990) with the capture as the
	 * RX queue: fills rawPacketsArr[0..k) (allocating a RawPacket where an entry is null) and returns k, 0 at the end */
	uint16_t receivePackets(RawPacket** rawPacketsArr, uint16_t rawPacketArrLength, uint16_t rxQueueId = 0)
	{
		(void)rxQueueId;
		if (rawPacketsArr == nullptr)
			return 0;
		uint16_t k = 0;
		for (; k < rawPacketArrLength; ++k)
		{
			if (rawPacketsArr[k] == nullptr)
				rawPacketsArr[k] = new RawPacket();
			if (!getNextPacket(*rawPacketsArr[k]))
				break;
		}
		return k;
	}

	/* IFileReaderDevice::getNextPackets(RawPacketVector&, int numOfPacketsToRead = -1) (PcapFileDevice.cpp:604-624):
	 * appends the next packets (all that remain when numOfPacketsToRead < 0) to packetVec as new RawPackets and returns
	 * how many. Each refers to its bytes in the map and to its page of GPU records (no copy), like getNextPacket's. */
	int getNextPackets(RawPacketVector& packetVec, int numOfPacketsToRead = -1)
	{
		int numOfPacketsRead = 0;
		for (; numOfPacketsToRead < 0 || numOfPacketsRead < numOfPacketsToRead; numOfPacketsRead++)
		{
			if (m_Cur == nullptr || m_Pos >= m_Cur->n)
			{
				if (!advance())
					break;
			}
			std::unique_ptr<RawPacket> p(new RawPacket());
			p->setFromPage(m_Cur, m_Pos++);
			packetVec.pushBack(std::move(p));
		}
		return numOfPacketsRead;
	}

	/* The batch API's read (one copy of the bytes into one buffer, the shape pcppx_batch takes): replaces `batch` with
	 * the next packets (at most numOfPacketsToRead, -1 = as many as maxBytes holds; one link type per batch); returns
	 * the count, 0 at the end of the capture. */
	int getNextBatch(RawBatch& batch, int numOfPacketsToRead = -1, uint64_t maxBytes = 256ull << 20)
	{
		batch.clear();
		int n = 0;
		while (numOfPacketsToRead < 0 || n < numOfPacketsToRead)
		{
			if (m_Cur == nullptr || m_Pos >= m_Cur->n)
			{
				if (!advance())
					break;
				if (n > 0 && m_Cur->linkType != batch.linkType)
					break;  // the next batch starts with this page
			}
			const uint32_t cap = m_Cur->caplens[m_Pos];
			if (n > 0 && batch.data.size() + cap > maxBytes)
				break;
			if (n == 0)
			{
				batch.linkType = m_Cur->linkType;
				if (numOfPacketsToRead > 0)
				{
					batch.offsets.reserve((size_t)numOfPacketsToRead);
					batch.caplens.reserve((size_t)numOfPacketsToRead);
					batch.timestampsNs.reserve((size_t)numOfPacketsToRead);
					batch.frameLens.reserve((size_t)numOfPacketsToRead);
				}
			}
			batch.add(m_Cur->base + m_Cur->offsets[m_Pos], cap, m_Cur->tsNs[m_Pos], m_Cur->frameLens[m_Pos]);
			++m_Pos;
			++n;
		}
		return n;
	}

	/* IFileDevice::getFileSize (PcapFileDevice.cpp:598-602) */
	uint64_t getFileSize() const
	{
		std::ifstream f(m_FileName, std::ifstream::ate | std::ifstream::binary);
		return f ? (uint64_t)f.tellg() : 0;
	}

	/* IFileReaderDevice::createReader (PcapFileDevice.cpp:546-583): the reader for the file's format, from its first
	 * bytes (detectFileFormat, :403-458) -- pcap (micro- or nanosecond magic, either byte order) and pcapng. Throws
	 * std::runtime_error when the file cannot be opened or its format is not one of those: Kuznetzov's modified pcap
	 * (the reference's switch has no case for it either), zstd-compressed pcapng (as a reference build without zstd
	 * support) and snoop (outside this engine). The device is not opened. */
	static std::unique_ptr<PcapFileReaderDevice> createReader(const std::string& fileName)
	{
		std::ifstream f(fileName, std::ios_base::binary);
		if (f.fail())
			throw std::runtime_error("Could not open file: " + fileName);
		uint8_t b[8] = { 0 };
		f.read(reinterpret_cast<char*>(b), sizeof(b));
		const std::streamsize got = f.gcount();
		uint32_t magic = 0;
		std::memcpy(&magic, b, 4);
		if (got >= 4)
		{
			if (magic == 0xa1b2c3d4u || magic == 0xd4c3b2a1u || magic == 0xa1b23c4du || magic == 0x4d3cb2a1u ||
			    magic == 0x0A0D0D0Au)
				return std::unique_ptr<PcapFileReaderDevice>(new PcapFileReaderDevice(fileName));
			if (magic == 0x28B52FFDu || magic == 0xFD2FB528u)
				throw std::runtime_error("PcapNG Zstd compressed files are not supported in this build of PcapPlusPlus");
		}
		throw std::runtime_error("File format of " + fileName + " is not supported");
	}
	/* IFileReaderDevice::tryCreateReader (PcapFileDevice.cpp:585-596): createReader, or nullptr where it throws */
	static std::unique_ptr<PcapFileReaderDevice> tryCreateReader(const std::string& fileName)
	{
		try
		{
			return createReader(fileName);
		}
		catch (const std::runtime_error& e)
		{
			std::fprintf(stderr, "%s\n", e.what());  // PCPP_LOG_ERROR
			return nullptr;
		}
	}

private:
	bool advance()
	{
		if (m_Core == nullptr)
			return false;
		m_Cur.reset();
		m_Pos = 0;
		m_Cur = m_Core->nextPage();
		return m_Cur != nullptr;
	}

	std::string m_FileName;
	std::shared_ptr<detail::ReaderCore> m_Core;
	std::shared_ptr<detail::Page> m_Cur;
	uint32_t m_Pos = 0;
	LinkLayerType m_OpenLinkType = LINKTYPE_ETHERNET;
};
using PcapNgFileReaderDevice = PcapFileReaderDevice;
using IFileReaderDevice = PcapFileReaderDevice;

/* PcapFileWriterDevice (Pcap++/src/PcapFileDevice.cpp:892-1119): classic pcap, micro- or nanosecond timestamps; a
 * packet of another link type than the file's is refused and counted (writePacket :1026-1039). */
class PcapFileWriterDevice
{
public:
	explicit PcapFileWriterDevice(const std::string& fileName, LinkLayerType linkLayerType = LINKTYPE_ETHERNET,
	                              bool nanosecondsPrecision = false)
	    : m_FileName(fileName),
	      m_LinkType(linkLayerType == LINKTYPE_DLT_RAW1 || linkLayerType == LINKTYPE_DLT_RAW2 ? LINKTYPE_RAW
	                                                                                          : linkLayerType),
	      m_Nano(nanosecondsPrecision)
	{}
	~PcapFileWriterDevice() { close(); }
	PcapFileWriterDevice(const PcapFileWriterDevice&) = delete;
	PcapFileWriterDevice& operator=(const PcapFileWriterDevice&) = delete;

	bool open()
	{
		if (m_File.is_open())
			return false;
		m_File.open(m_FileName, std::ios::binary | std::ios::out);
		if (!m_File.is_open())
			return false;
		const uint32_t hdr[6] = { m_Nano ? 0xa1b23c4du : 0xa1b2c3d4u, 2u | (4u << 16), 0, 0, 262144, m_LinkType };
		return (bool)m_File.write(reinterpret_cast<const char*>(hdr), sizeof(hdr));
	}
	bool writePacket(const RawPacket& packet)
	{
		if (!m_File.is_open())
			return false;
		if (packet.getLinkLayerType() != m_LinkType)
		{
			++m_NotWritten;  // "Cannot write a packet with a different link type"
			return false;
		}
		const timespec ts = packet.getPacketTimeStamp();
		const uint32_t h[4] = { (uint32_t)ts.tv_sec, (uint32_t)(m_Nano ? ts.tv_nsec : ts.tv_nsec / 1000),
			                    (uint32_t)packet.getRawDataLen(), (uint32_t)packet.getFrameLength() };
		if (!m_File.write(reinterpret_cast<const char*>(h), sizeof(h)) ||
		    !m_File.write(reinterpret_cast<const char*>(packet.getRawData()), packet.getRawDataLen()))
		{
			++m_NotWritten;
			return false;
		}
		++m_Written;
		return true;
	}
	void flush()
	{
		if (m_File.is_open())
			m_File.flush();
	}
	void close()
	{
		if (m_File.is_open())
			m_File.close();
	}
	uint64_t packetsWritten() const { return m_Written; }
	uint64_t packetsNotWritten() const { return m_NotWritten; }

private:
	std::string m_FileName;
	uint32_t m_LinkType;
	bool m_Nano;
	std::ofstream m_File;
	uint64_t m_Written = 0, m_NotWritten = 0;
};

/* One layer of a parsed packet: Layer::getProtocol / getOsiModelLayer / getData / getHeaderLen / getDataLen /
 * getLayerPayloadSize / isMemberOfProtocolFamily (Packet++/header/Layer.h) */
class Layer
{
public:
	Layer() = default;
	Layer(const pcppx_layer* rec, const uint8_t* raw) : m_Rec(rec), m_Raw(raw) {}
	ProtocolType getProtocol() const { return m_Rec->proto; }
	OsiModelLayer getOsiModelLayer() const { return (OsiModelLayer)m_Rec->osi; }
	const uint8_t* getData() const { return m_Raw + m_Rec->offset; }
	size_t getHeaderLen() const { return m_Rec->hdr_len; }
	size_t getDataLen() const { return m_Rec->data_len; }
	size_t getLayerPayloadSize() const { return m_Rec->data_len - m_Rec->hdr_len; }
	const uint8_t* getLayerPayload() const { return getData() + getHeaderLen(); }
	bool isMemberOfProtocolFamily(ProtocolTypeFamily family) const
	{
		const uint32_t p = m_Rec->proto;
		return p != 0 && (p == (family & 0xFF) || (p << 8) == (family & 0xFF00) || (p << 16) == (family & 0xFF0000) ||
		                  (p << 24) == (family & 0xFF000000u));
	}
	uint16_t getOffset() const { return m_Rec->offset; }
	bool valid() const { return m_Rec != nullptr; }

protected:
	uint16_t be16(size_t j) const { return (uint16_t)((getData()[j] << 8) | getData()[j + 1]); }
	const pcppx_layer* m_Rec = nullptr;
	const uint8_t* m_Raw = nullptr;
};

/* typed views: the accessors the two reference callers use */
class IPv4Layer : public Layer /* Packet++/header/IPv4Layer.h */
{
public:
	static constexpr ProtocolType kProtocol = IPv4;
	using Layer::Layer;
	IPv4Address getSrcIPv4Address() const { return IPv4Address(rd32(12)); }
	IPv4Address getDstIPv4Address() const { return IPv4Address(rd32(16)); }
	uint8_t getProtocolField() const { return getData()[9]; }
	bool isFragment() const { return (getData()[6] & 0x20) || (((getData()[6] & 0x1F) << 8) | getData()[7]) != 0; }

private:
	uint32_t rd32(size_t j) const
	{
		uint32_t v;
		std::memcpy(&v, getData() + j, 4);
		return v;
	}
};
class IPv6Layer : public Layer /* Packet++/header/IPv6Layer.h */
{
public:
	static constexpr ProtocolType kProtocol = IPv6;
	using Layer::Layer;
	const uint8_t* getSrcIPv6AddressBytes() const { return getData() + 8; }
	const uint8_t* getDstIPv6AddressBytes() const { return getData() + 24; }
};
class TcpLayer : public Layer /* Packet++/header/TcpLayer.h: ports in host order */
{
public:
	static constexpr ProtocolType kProtocol = TCP;
	using Layer::Layer;
	uint16_t getSrcPort() const { return be16(0); }
	uint16_t getDstPort() const { return be16(2); }
	uint8_t getFlags() const { return getData()[13]; }
};
class UdpLayer : public Layer /* Packet++/header/UdpLayer.h */
{
public:
	static constexpr ProtocolType kProtocol = UDP;
	using Layer::Layer;
	uint16_t getSrcPort() const { return be16(0); }
	uint16_t getDstPort() const { return be16(2); }
};

/* what getLayerOfType<T>() returns: a layer view that tests like the reference's T* (null when absent) */
template <class T>
class LayerPtr
{
public:
	LayerPtr() = default;
	explicit LayerPtr(const T& v) : m_V(v), m_Ok(true) {}
	const T* operator->() const { return &m_V; }
	const T& operator*() const { return m_V; }
	explicit operator bool() const { return m_Ok; }
	bool operator==(std::nullptr_t) const { return !m_Ok; }
	bool operator!=(std::nullptr_t) const { return m_Ok; }

private:
	T m_V{};
	bool m_Ok = false;
};

/* A parsed packet: the pcpp::Packet (Packet++/header/Packet.h) queries of the two callers. Built from a RawPacket
 * (the reference's constructors) or as a view into a ParsedBatch. Like the reference's Packet it reads the
 * RawPacket's bytes and must not outlive the RawPacket's current contents. */
class Packet
{
public:
	/* Packet::Packet(RawPacket*, bool freeRawPacket, ProtocolType / ProtocolTypeFamily parseUntil, OsiModelLayer)
	 * and the short forms (Packet.h:94-134, Packet.cpp:198-234) */
	explicit Packet(RawPacket* rawPacket, bool freeRawPacket = false, ProtocolType parseUntil = UnknownProtocol,
	                OsiModelLayer parseUntilLayer = OsiModelLayerUnknown)
	{
		bind(rawPacket, freeRawPacket, parseUntil, parseUntilLayer);
	}
	explicit Packet(RawPacket* rawPacket, bool freeRawPacket, ProtocolTypeFamily parseUntil,
	                OsiModelLayer parseUntilLayer = OsiModelLayerUnknown)
	{
		bind(rawPacket, freeRawPacket, parseUntil, parseUntilLayer);
	}
	explicit Packet(RawPacket* rawPacket, ProtocolType parseUntil)
	{
		bind(rawPacket, false, parseUntil, OsiModelLayerUnknown);
	}
	explicit Packet(RawPacket* rawPacket, ProtocolTypeFamily parseUntilFamily)
	{
		bind(rawPacket, false, parseUntilFamily, OsiModelLayerUnknown);
	}
	explicit Packet(RawPacket* rawPacket, OsiModelLayer parseUntilLayer)
	{
		bind(rawPacket, false, UnknownProtocol, parseUntilLayer);
	}
	/* a view into records the caller holds (ParsedBatch) */
	Packet(const pcppx_summary* s, const pcppx_layer* layers, uint8_t maxLayers, const uint8_t* raw, uint32_t caplen)
	    : m_Brief(reinterpret_cast<const pcppx_brief*>(s)), m_Sum(s), m_Layers(layers), m_MaxLayers(maxLayers), m_Raw(raw),
	      m_Caplen(caplen)
	{}

	/* Packet::isPacketOfType (Packet.cpp:614-640), for a protocol or a family. On a packet the engine left to the
	 * host and no host parser completed, the answer covers its exact layer prefix plus the HTTP / SSL / DNS class
	 * of its first L7 layer when the device named it (PCPPX_F_L7_KNOWN) */
	bool isPacketOfType(ProtocolTypeFamily family) const
	{
		uint64_t mask = protoMask();
		const uint16_t fl = m_Brief->flags;
		if (fl & PCPPX_F_L7_KNOWN)
			mask |= ((fl & PCPPX_F_L7_HTTP) ? (1ull << HTTPRequest) | (1ull << HTTPResponse) : 0) |
			        ((fl & PCPPX_F_L7_SSL) ? 1ull << SSL : 0) | ((fl & PCPPX_F_L7_DNS) ? 1ull << DNS : 0);
		for (int k = 0; k < 4; ++k)
		{
			const uint32_t p = (family >> (8 * k)) & 0xFF;
			if (p != 0 && p < 64 && (mask >> p) & 1)
				return true;
		}
		return false;
	}
	size_t getLayerCount() const { return m_Brief->n_layers; }
	/* records held for the first min(getLayerCount(), maxLayers) layers */
	size_t getRecordedLayerCount() const { return m_Brief->n_layers < m_MaxLayers ? m_Brief->n_layers : m_MaxLayers; }
	Layer getLayer(size_t k) const { return Layer(m_Layers + k, m_Raw); }
	Layer getFirstLayer() const { return getRecordedLayerCount() ? getLayer(0) : Layer(); }
	Layer getLastLayer() const { return getRecordedLayerCount() ? getLayer(getRecordedLayerCount() - 1) : Layer(); }
	/* getLayerOfType<T>(reverse) (Packet.h:388-431): the first (or, reverse, the last) recorded layer of T */
	template <class T>
	LayerPtr<T> getLayerOfType(bool reverseOrder = false) const
	{
		const size_t n = getRecordedLayerCount();
		for (size_t j = 0; j < n; ++j)
		{
			const size_t k = reverseOrder ? n - 1 - j : j;
			if (m_Layers[k].proto == T::kProtocol)
				return LayerPtr<T>(T(m_Layers + k, m_Raw));
		}
		return LayerPtr<T>();
	}

	/* the raw packet (RawPacket::getRawData / getRawDataLen) */
	const uint8_t* getRawData() const { return m_Raw; }
	uint32_t getRawDataLen() const { return m_Caplen; }

	/* engine flags: the host must finish the packet (an L7 or an out-of-scope L2/L3 layer) and no host parser did */
	bool needsHost() const { return (m_Brief->flags & PCPPX_F_NEEDS_HOST) != 0; }
	/* the records come from the caller's host parser (setHostParser / Engine::setHostParser) */
	bool wasHostParsed() const { return (m_Brief->flags & F_HOST_PARSED) != 0; }
	bool hasTrailer() const { return (m_Brief->flags & PCPPX_F_TRAILER) != 0; }
	/* IPv4Layer::computeCalculateFields checksum vs the stored one (IPv4Layer.cpp:410-412): verified where the parse
	 * computed checksums (setPageChecksums, PacketParseOptions::computeChecksums) */
	bool hasIPv4Checksum() const { return (m_Brief->flags & PCPPX_F_IP_CSUM) != 0; }
	bool isIPv4ChecksumValid() const { return (m_Brief->flags & PCPPX_F_IP_CSUM_OK) != 0; }
	/* TcpLayer/UdpLayer::calculateChecksum(false) vs the stored checksum (TcpLayer.cpp:271, UdpLayer.cpp:47) */
	bool hasL4Checksum() const { return (m_Brief->flags & PCPPX_F_L4_CSUM) != 0; }
	bool isL4ChecksumValid() const { return (m_Brief->flags & PCPPX_F_L4_CSUM_OK) != 0; }
	uint16_t calculatedL4Checksum() const { return m_Sum ? m_Sum->l4_csum_calc : 0; }
	uint16_t calculatedIPv4Checksum() const { return m_Sum ? m_Sum->ip_csum_calc : 0; }
	/* hashes, flags, chain length, port layer (pcppx_brief) */
	const pcppx_brief& brief() const { return *m_Brief; }
	/* the whole summary: the records' own, or built from the brief with the chain's protocol mask (checksum values 0:
	 * the parse computed none) */
	const pcppx_summary& summary() const
	{
		if (m_Sum != nullptr)
			return *m_Sum;
		m_Full = pcppx_summary{};
		std::memcpy(&m_Full, m_Brief, sizeof(pcppx_brief));
		m_Full.proto_mask = protoMask();
		return m_Full;
	}

private:
	static const pcppx_summary* emptySummary()
	{
		static const pcppx_summary s{ 0, 0, 0, 0, 0, 0xFF, 0, 0, 0, 0, 0 };
		return &s;
	}
	uint64_t protoMask() const
	{
		return m_Sum ? m_Sum->proto_mask : pcppx_chain_proto_mask(m_Layers, (unsigned)getRecordedLayerCount());
	}
	/* packet i of a page's / group's records */
	void bindRecords(const detail::Records* r, uint32_t i)
	{
		const pcppx_brief* b = r->briefOf(i);
		if (b->flags & (F_HOST_PARSED | PCPPX_F_DEPTH_OVERFLOW))
			if (const detail::CopiedRecords* c = r->sideFor(i))
			{
				m_Sum = &c->sum;  // complete records beside the chain
				m_Brief = reinterpret_cast<const pcppx_brief*>(m_Sum);
				m_Layers = c->lay;
				return;
			}
		m_Brief = b;
		m_Sum = r->sum ? r->sum + i : nullptr;
		m_Layers = r->lay + r->first[i];
	}
	void bind(RawPacket* raw, bool freeRawPacket, ProtocolTypeFamily parseUntil, OsiModelLayer parseUntilLayer)
	{
		m_Sum = emptySummary();
		m_Brief = reinterpret_cast<const pcppx_brief*>(m_Sum);
		m_MaxLayers = PCPPX_MAX_LAYERS;
		if (raw == nullptr)
			return;  // Packet::setRawPacket: no RawPacket, no layers (Packet.cpp:60-61)
		if (freeRawPacket)
			m_OwnedRaw.reset(raw);
		m_Raw = raw->m_RawData;
		m_Caplen = raw->m_RawDataLen > 0 ? (uint32_t)raw->m_RawDataLen : 0;
		const detail::ParseKey k{ parseUntil, parseUntilLayer, detail::pageChecksums().load(std::memory_order_relaxed) };
		if (raw->m_Copied != nullptr && raw->m_Copied->key == k)
		{
			m_Sum = &raw->m_Copied->sum;  // records copied with the bytes
			m_Brief = reinterpret_cast<const pcppx_brief*>(m_Sum);
			m_Layers = raw->m_Copied->lay;
			return;
		}
		if (raw->m_Registered)
		{
			// the caller's own bytes: parsed with every other pending RawPacket in one batch, or already in a group
			uint32_t idx = 0;
			const detail::Records* r = detail::OwnedRegistry::instance().recordsFor(raw, k, &idx);  // sets idx
			bindRecords(r, idx);
			return;
		}
		if (detail::Page* p = raw->m_Page.get())
		{
			const detail::Records* r = p->primary.load(std::memory_order_acquire);
			if (r == nullptr || !(r->key == k))
				r = p->recordsFor(k);
			bindRecords(r, raw->m_Index);
		}
		// else no data: createFirstLayer builds nothing (Packet.cpp:88-94)
	}

	const pcppx_brief* m_Brief = nullptr;  // always set (a summary's first half where m_Sum is)
	const pcppx_summary* m_Sum = nullptr;  // complete records, where the parse or the side table has them
	const pcppx_layer* m_Layers = nullptr;
	uint8_t m_MaxLayers = 0;
	const uint8_t* m_Raw = nullptr;
	uint32_t m_Caplen = 0;
	mutable pcppx_summary m_Full;         // summary() of brief-backed records (assigned whole before any read)
	std::shared_ptr<RawPacket> m_OwnedRaw;  // freeRawPacket
};
using ParsedPacket = Packet;
using ParsedLayer = Layer;

/* pcpp::hash5Tuple / hash2Tuple (Packet++/header/PacketUtils.h:58-91) */
inline uint32_t hash5Tuple(const Packet* packet, bool const& directionUnique = false)
{
	return directionUnique ? packet->brief().hash5_dir : packet->brief().hash5;
}
inline uint32_t hash2Tuple(const Packet* packet)
{
	return packet->brief().hash2;
}

/* Records of one parsed batch (owns them); indexes into the RawBatch it was parsed from. */
class ParsedBatch
{
public:
	ParsedBatch(const RawBatch& raw, uint8_t maxLayers)
	    : m_Raw(&raw), m_MaxLayers(maxLayers), summaries(raw.size()), layers(raw.size() * (size_t)maxLayers)
	{}
	size_t size() const { return summaries.size(); }
	Packet operator[](size_t i) const
	{
		return Packet(&summaries[i], layers.data() + i * m_MaxLayers, m_MaxLayers, m_Raw->packetData(i),
		              m_Raw->caplens[i]);
	}
	class iterator
	{
	public:
		iterator(const ParsedBatch* b, size_t i) : m_B(b), m_I(i) {}
		Packet operator*() const { return (*m_B)[m_I]; }
		iterator& operator++()
		{
			++m_I;
			return *this;
		}
		bool operator!=(const iterator& o) const { return m_I != o.m_I; }

	private:
		const ParsedBatch* m_B;
		size_t m_I;
	};
	iterator begin() const { return iterator(this, 0); }
	iterator end() const { return iterator(this, size()); }
	uint8_t maxLayers() const { return m_MaxLayers; }
	/* packets whose records the host parser filled */
	size_t hostParsed = 0;

private:
	const RawBatch* m_Raw;
	uint8_t m_MaxLayers;

public:
	buffer<pcppx_summary> summaries; /* filled by the engine (or the host parser) for every packet */
	buffer<pcppx_layer> layers;       /* entries past a packet's chain are unspecified, as in pcppx.h */
};

/* PCPPX_LAYOUT_PACKED entries (include/pcppx.h) -> the FIXED layout: packet i's chain starts at its tile's base
 * 64 * t * maxLayers plus the chains of the packets before it in the tile (summary n_layers, capped at maxLayers).
 * fixed: n * maxLayers entries; entries past a chain are zeroed. */
inline void unpackLayers(const pcppx_summary* summary, const pcppx_layer* packed, size_t n, uint32_t maxLayers,
                         pcppx_layer* fixed)
{
	size_t pos = 0;
	for (size_t i = 0; i < n; ++i)
	{
		if (i % 64 == 0)
			pos = i * maxLayers;
		const uint32_t cnt = summary[i].n_layers < maxLayers ? summary[i].n_layers : maxLayers;
		for (uint32_t k = 0; k < maxLayers; ++k)
			fixed[i * maxLayers + k] = k < cnt ? packed[pos + k] : pcppx_layer{};
		pos += cnt;
	}
}

/* PacketMatchingEngine's criteria (Examples/DpdkExample-FilterTraffic/PacketMatchingEngine.h:28-41) */
struct MatchSpec
{
	pcppx_match_spec spec{};
	MatchSpec() = default;
	/* addresses as dotted quads ("" = any); ports host order (0 = any); protocol TCP / UDP (else any) */
	MatchSpec(const std::string& srcIp, const std::string& dstIp, uint16_t srcPort, uint16_t dstPort,
	          ProtocolType protocol)
	{
		spec.src_ip = srcIp.empty() ? 0 : IPv4Address(srcIp).toInt();
		spec.dst_ip = dstIp.empty() ? 0 : IPv4Address(dstIp).toInt();
		spec.src_port = srcPort;
		spec.dst_port = dstPort;
		spec.protocol = protocol;
	}
};

/* One GPU worker for the batch API: a pcppx context. */
class Engine
{
public:
	explicit Engine(int device = 0) { check(pcppx_open(device, &m_Ctx), "pcppx_open"); }
	~Engine() { pcppx_close(m_Ctx); }
	Engine(const Engine&) = delete;
	Engine& operator=(const Engine&) = delete;

	/* the caller's own Packet++ parse of one packet, used to complete packets the engine flags NEEDS_HOST */
	void setHostParser(pcppx_host_parse_fn fn) { m_HostParser = fn; }

	/* Packet(&rawPacket, options) for every packet of the batch, host to host through HBM; flagged packets are
	 * completed by the host parser when one is set */
	ParsedBatch parse(const RawBatch& batch, const PacketParseOptions& options = PacketParseOptions()) const
	{
		ParsedBatch out(batch, options.maxLayers);
		parseInto(batch, options, out);
		return out;
	}
	void parseInto(const RawBatch& batch, const PacketParseOptions& options, ParsedBatch& out) const
	{
		const pcppx_batch b = batch.toC();
		const pcppx_opts o = options.toC();
		pcppx_records r{};
		r.summary = out.summaries.data();
		r.layers = options.maxLayers ? out.layers.data() : nullptr;
		check(pcppx_parse_batch_host(m_Ctx, &b, &o, &r), "pcppx_parse_batch_host");
		out.hostParsed = detail::completeOnHost(m_HostParser, batch.data.data(), batch.offsets.data(),
		                                        batch.caplens.data(), (uint32_t)batch.size(), batch.linkType, o,
		                                        out.summaries.data(), out.layers.data());
	}

	/* FilterTraffic's whole worker on the device (AppWorkerThread.h:85-139): matched[i] = 1 for packets to send on;
	 * the flow table persists across calls until resetFilter() */
	pcppx_packet_stats filter(const RawBatch& batch, const MatchSpec& spec, std::vector<uint8_t>& matched)
	{
		matched.assign(batch.size(), 0);
		const pcppx_batch b = batch.toC();
		pcppx_packet_stats st;
		check(pcppx_filter_batch_host(m_Ctx, &b, &spec.spec, matched.data(), &st), "pcppx_filter_batch_host");
		return st;
	}
	void resetFilter(uint32_t flowTableSlots = 0) { check(pcppx_filter_reset(m_Ctx, flowTableSlots), "pcppx_filter_reset"); }

	pcppx_ctx* handle() const { return m_Ctx; }

private:
	pcppx_ctx* m_Ctx = nullptr;
	pcppx_host_parse_fn m_HostParser = nullptr;
};

}  // namespace pcppx

#endif /* PCPPX_HPP */
