// pcppx_capi.cpp — the C ABI of include/pcppx.h: contexts, argument checks, kernel launches and the
// pinned, double-buffered host-to-host pipeline.
//
// One context = one GPU + one host thread (the DpdkExample-FilterTraffic model of one private worker
// per core, AppWorkerThread.h:45-162, mapped to one worker per GPU). Nothing here touches packet bytes
// on the CPU except the copy into pinned staging on the host path.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "pcppx.h"
#include "pcppx_internal.h"

namespace
{
constexpr size_t kChunkBytes = 64u << 20;    // packet bytes per host-path chunk
constexpr uint32_t kChunkPackets = 1u << 18;  // packets per host-path chunk

struct Slot
{
	hipStream_t st = nullptr;
	hipEvent_t done = nullptr;
	uint8_t* h_data = nullptr;
	uint64_t* h_off = nullptr;
	uint32_t* h_cap = nullptr;
	pcppx_summary* h_sum = nullptr;
	pcppx_layer* h_lay = nullptr;  // FIXED rows, or (DENSE) the chunk's chains
	pcppx_brief* h_brief = nullptr;
	uint32_t* h_total = nullptr;   // DENSE: the chunk's chain entries, and the batch's up to the chunk's end
	uint8_t* d_data = nullptr;
	uint64_t* d_off = nullptr;
	uint32_t* d_cap = nullptr;
	pcppx_summary* d_sum = nullptr;
	pcppx_layer* d_lay = nullptr;
	pcppx_brief* d_brief = nullptr;
	pcppx_layer* d_dense = nullptr;  // DENSE: the chunk's chains back to back
	uint32_t* d_dsum = nullptr;      // DENSE: per-block chain totals, the chunk's total, the batch's up to the chunk's end
	hipEvent_t parsed = nullptr;     // DENSE: the chunk's chains pushed (the next chunk's positions follow them)
	uint8_t* h_match = nullptr;  // host filter path: per-packet verdicts
	uint8_t* d_match = nullptr;
	bool busy = false;
	uint32_t first = 0, count = 0, ml = 0;
	uint64_t dense_first = 0;  // DENSE: the chunk's first entry in the caller's array
	uint32_t dense_count = 0;
};

// memcpy split over persistent host threads (started with the host path, joined at pcppx_close): a single
// core copies ~8-10 GB/s, below what the PCIe link takes. The caller copies part 0 itself.
class CopyPool
{
public:
	static constexpr unsigned kThreads = 16;

	void start()
	{
		for (unsigned k = 1; k < kThreads; ++k)
			m_threads.emplace_back([this, k] { work(k); });
	}

	void stop()
	{
		{
			std::lock_guard<std::mutex> g(m_mu);
			m_quit = true;
		}
		m_cv.notify_all();
		for (auto& t : m_threads)
			t.join();
		m_threads.clear();
		m_quit = false;
	}

	// one part per >= 1 MiB, at most kThreads parts
	void copy(void* dst, const void* src, size_t bytes)
	{
		unsigned parts = (unsigned)(bytes >> 20);
		parts = parts < 1 ? 1 : (parts > kThreads ? kThreads : parts);
		if (parts == 1 || m_threads.empty())
		{
			std::memcpy(dst, src, bytes);
			return;
		}
		const size_t per = ((bytes + parts - 1) / parts + 63) & ~(size_t)63;
		{
			std::lock_guard<std::mutex> g(m_mu);
			m_dst = static_cast<uint8_t*>(dst);
			m_src = static_cast<const uint8_t*>(src);
			m_bytes = bytes;
			m_per = per;
			m_parts = parts;
			m_left = 0;
			for (unsigned k = 1; k < parts; ++k)
				m_left += k * per < bytes ? 1 : 0;
			++m_gen;
		}
		m_cv.notify_all();
		std::memcpy(dst, src, per < bytes ? per : bytes);
		std::unique_lock<std::mutex> g(m_mu);
		m_done.wait(g, [&] { return m_left == 0; });
	}

private:
	void work(unsigned k)
	{
		uint64_t seen = 0;
		for (;;)
		{
			uint8_t* d;
			const uint8_t* s;
			size_t lo, len;
			{
				std::unique_lock<std::mutex> g(m_mu);
				m_cv.wait(g, [&] { return m_quit || m_gen != seen; });
				if (m_quit)
					return;
				seen = m_gen;
				lo = k * m_per;
				if (k >= m_parts || lo >= m_bytes)
					continue;
				len = m_bytes - lo < m_per ? m_bytes - lo : m_per;
				d = m_dst + lo;
				s = m_src + lo;
			}
			std::memcpy(d, s, len);
			{
				std::lock_guard<std::mutex> g(m_mu);
				--m_left;
			}
			m_done.notify_one();
		}
	}

	std::vector<std::thread> m_threads;
	std::mutex m_mu;
	std::condition_variable m_cv, m_done;
	uint8_t* m_dst = nullptr;
	const uint8_t* m_src = nullptr;
	size_t m_bytes = 0, m_per = 0;
	unsigned m_parts = 0, m_left = 0;
	uint64_t m_gen = 0;
	bool m_quit = false;
};

constexpr uint32_t kDefaultFlowSlots = 1u << 22;  // 64 MiB of flow table in HBM
constexpr uint32_t kMaxSlots = 3;                   // host-path chunk slots in flight
}  // namespace

struct pcppx_ctx
{
	int device = 0;
	hipStream_t stream = nullptr;
	bool host_ready = false;
	Slot slots[kMaxSlots];
	uint32_t nslots = 0;  // slots allocated and used by the host paths
	CopyPool copier;      // staging and drain copies of the host paths
	// host filter path (pcppx_filter_reset / pcppx_filter_batch_host): the worker's flow table in HBM
	uint64_t* d_keys = nullptr;
	uint64_t* d_first = nullptr;
	pcppx_packet_stats* d_stats = nullptr;
	uint32_t flow_slots = 0;
	uint64_t seq = 0;
	// pcppx_flow_count_device: the partitioned flush's record queues and queue lengths (zero between calls), and
	// an event after each call's last kernel: the next call (on whatever stream) waits for it before touching
	// the scratch, so calls on one context are ordered even across streams
	void* d_flow_queues = nullptr;
	uint64_t flow_queue_recs = 0;
	uint32_t* d_flow_fill = nullptr;
	hipEvent_t flow_done = nullptr;
	bool flow_pending = false;
	// pcppx_records.proto_stats: the parse's per-wave collectStats records (16 B per 64 packets), summed into the
	// caller's counters by a second kernel; ordered across calls like the flow scratch
	void* d_wave_stats = nullptr;
	uint64_t wave_stats_bytes = 0;
	hipEvent_t stats_done = nullptr;
	bool stats_pending = false;
	// the engine's header-window choice for PCPPX_WINDOW_DEFAULT launches: a sampled parse (every launch until the first
	// decision, then one in kWinEvery) first adds the live packets and deep stacks of about 64 of its tiles to d_win (never
	// cleared); after it, a private stream copies the counters into a page-locked mirror, which a later launch reads once
	// the copy is done (no wait on any stream)
	unsigned long long* d_win = nullptr;
	unsigned long long* h_win = nullptr;
	hipStream_t win_stream = nullptr;
	hipEvent_t win_parsed = nullptr, win_copied = nullptr;
	bool win_ready = false, win_pending = false;
	unsigned long long win_live = 0, win_deep = 0;  // the mirror at the last decision
	int deep_traffic = -1;                            // -1: not known yet; 0: plain stacks; 1: deep stacks
	uint64_t win_launches = 0;                        // DEFAULT-window parses so far (the sampling schedule)
};

namespace
{
bool ok(hipError_t e)
{
	return e == hipSuccess;
}

// ---- the engine's header window (PCPPX_WINDOW_DEFAULT) ----
constexpr unsigned long long kWinMinSample = 2048;  // sampled packets per decision (a launch samples up to ~4096)
constexpr unsigned long long kWinDeepShare = 256;   // deep stacks above 1 in 256 sampled packets: deep traffic
constexpr uint64_t kWinEvery = 16;                  // once decided, one parse in 16 is sampled (the traffic may change)

bool ensure_win(pcppx_ctx* c)
{
	if (c->win_ready)
		return true;
	const bool good = ok(hipMalloc(reinterpret_cast<void**>(&c->d_win), 2 * sizeof(unsigned long long))) &&
	                  ok(hipMemset(c->d_win, 0, 2 * sizeof(unsigned long long))) &&
	                  ok(hipHostMalloc(reinterpret_cast<void**>(&c->h_win), 2 * sizeof(unsigned long long))) &&
	                  ok(hipStreamCreateWithFlags(&c->win_stream, hipStreamNonBlocking)) &&
	                  ok(hipEventCreateWithFlags(&c->win_parsed, hipEventDisableTiming)) &&
	                  ok(hipEventCreateWithFlags(&c->win_copied, hipEventDisableTiming));
	if (!good)
	{
		(void)hipGetLastError();
		return false;
	}
	c->h_win[0] = c->h_win[1] = 0;
	c->win_ready = true;
	return true;
}

// fold a finished counter copy into the decision (wait: block until the copy in flight is done)
void update_window(pcppx_ctx* c, bool wait)
{
	if (!c->win_pending)
		return;
	if (wait ? !ok(hipEventSynchronize(c->win_copied)) : hipEventQuery(c->win_copied) != hipSuccess)
		return;
	c->win_pending = false;
	const unsigned long long live = c->h_win[0] - c->win_live, deep = c->h_win[1] - c->win_deep;
	if (live < kWinMinSample)
		return;
	c->deep_traffic = deep * kWinDeepShare > live ? 1 : 0;
	c->win_live = c->h_win[0];
	c->win_deep = c->h_win[1];
}

// the window a launch runs with: an explicit DEEP / SHORT as asked; DEFAULT follows the traffic this context has seen
// (deep stacks: the two-round window for checksum launches too; plain stacks: one round for parse-only launches too).
// The records are the same whichever window runs.
pcppx_opts resolve_window(pcppx_ctx* c, const pcppx_opts* o)
{
	pcppx_opts e = *o;
	if (o->window != PCPPX_WINDOW_DEFAULT)
		return e;
	update_window(c, false);
	if (c->deep_traffic == 1 && o->want_checksums)
		e.window = PCPPX_WINDOW_DEEP;
	else if (c->deep_traffic == 0 && !o->want_checksums)
		e.window = PCPPX_WINDOW_SHORT;
	return e;
}

// the counters a parse samples into, or null: a PCPPX_WINDOW_DEFAULT parse every time until the first decision, then
// one in kWinEvery; a parse whose window the caller forced never (the choice follows the DEFAULT parses' traffic)
unsigned long long* window_sample(pcppx_ctx* c, const pcppx_opts* o)
{
	if (o->window != PCPPX_WINDOW_DEFAULT || !ensure_win(c))
		return nullptr;
	update_window(c, false);
	const uint64_t k = c->win_launches++;
	return (c->deep_traffic < 0 || k % kWinEvery == 0) ? c->d_win : nullptr;
}

// after a sampled parse on st (win: window_sample's counters): copy the counters out behind it on the private stream
// (one copy in flight)
void note_window(pcppx_ctx* c, hipStream_t st, const unsigned long long* win)
{
	if (win == nullptr || !c->win_ready || c->win_pending)
		return;
	if (ok(hipEventRecord(c->win_parsed, st)) && ok(hipStreamWaitEvent(c->win_stream, c->win_parsed, 0)) &&
	    ok(hipMemcpyAsync(c->h_win, c->d_win, 2 * sizeof(unsigned long long), hipMemcpyDeviceToHost, c->win_stream)) &&
	    ok(hipEventRecord(c->win_copied, c->win_stream)))
		c->win_pending = true;
	else
		(void)hipGetLastError();
}

int valid_opts(const pcppx_opts* o)
{
	if (o == nullptr || o->max_layers > PCPPX_MAX_LAYERS || o->window > PCPPX_WINDOW_SHORT ||
	    o->layout > PCPPX_LAYOUT_DENSE || (o->layout == PCPPX_LAYOUT_PACKED && o->max_layers > PCPPX_PACKED_MAX_LAYERS))
		return PCPPX_E_INVAL;
	return PCPPX_OK;
}

// the device path's record arguments: layers when max_layers > 0; a summary unless the caller wants only the
// summary-free outputs -- the 5-tuple extract, the dense flow-key column and / or the collectStats counters (a
// FilterTraffic-style consumer reads nothing else) -- with no layers (a PACKED layout is decoded through the summary's
// n_layers)
bool valid_device_records(const pcppx_opts* o, const pcppx_records* r)
{
	if (o->max_layers != 0 && r->layers == nullptr)
		return false;
	if (r->summary == nullptr && r->brief == nullptr &&
	    (o->max_layers != 0 || (r->tuples == nullptr && r->flow_keys == nullptr && r->proto_stats == nullptr)))
		return false;
	return o->layout != PCPPX_LAYOUT_DENSE;  // DENSE: the host path's layout
}

// Scratch owned by a context and shared by its calls: a call waits (on its own stream) for the previous call's
// `done` event before touching it, and a larger size is reallocated in stream order behind that wait -- no call
// stalls the device or another stream.
int ensure_scratch(hipStream_t st, void** ptr, uint64_t* have, uint64_t want, hipEvent_t* done, bool pending)
{
	if (*done == nullptr && !ok(hipEventCreateWithFlags(done, hipEventDisableTiming)))
		return PCPPX_E_HIP;
	if (pending && !ok(hipStreamWaitEvent(st, *done, 0)))
		return PCPPX_E_HIP;
	if (*have < want)
	{
		if (*ptr != nullptr && !ok(hipFreeAsync(*ptr, st)))
			return PCPPX_E_HIP;
		*ptr = nullptr;
		*have = 0;
		if (!ok(hipMallocAsync(ptr, want, st)))
			return PCPPX_E_NOMEM;
		*have = want;
	}
	return PCPPX_OK;
}

// launch a device parse (plain or with the fused reassembly output) with the collectStats reduction when
// r->proto_stats is set
int device_parse(pcppx_ctx* c, const pcppx_batch* b, const pcppx_opts* o, pcppx_records* r, pcppx_reasm_info* info,
                 hipStream_t st)
{
	void* ws = nullptr;
	if (r->proto_stats != nullptr)
	{
		const int rc = ensure_scratch(st, &c->d_wave_stats, &c->wave_stats_bytes, (uint64_t)pcppx::parse_waves(b->n) * 16,
		                              &c->stats_done, c->stats_pending);
		if (rc != PCPPX_OK)
			return rc;
		ws = c->d_wave_stats;
	}
	const pcppx_opts eo = resolve_window(c, o);
	unsigned long long* win = window_sample(c, o);
	int rc = info ? pcppx::launch_parse_reasm(b, &eo, r, info, st, ws, win) : pcppx::launch_parse(b, &eo, r, st, ws, win);
	if (rc == PCPPX_OK)
		note_window(c, st, win);
	if (rc != PCPPX_OK || ws == nullptr)
		return rc;
	rc = pcppx::launch_proto_stats_reduce(ws, b->n, r->proto_stats, st);
	if (rc != PCPPX_OK)
		return rc;
	if (!ok(hipEventRecord(c->stats_done, st)))
		return PCPPX_E_HIP;
	c->stats_pending = true;
	return PCPPX_OK;
}

void free_slot(Slot& s)
{
	if (s.st) (void)hipStreamDestroy(s.st);
	if (s.done) (void)hipEventDestroy(s.done);
	if (s.parsed) (void)hipEventDestroy(s.parsed);
	(void)hipHostFree(s.h_brief);
	(void)hipHostFree(s.h_total);
	(void)hipFree(s.d_brief);
	(void)hipFree(s.d_dense);
	(void)hipFree(s.d_dsum);
	(void)hipHostFree(s.h_data);
	(void)hipHostFree(s.h_off);
	(void)hipHostFree(s.h_cap);
	(void)hipHostFree(s.h_sum);
	(void)hipHostFree(s.h_lay);
	(void)hipFree(s.d_data);
	(void)hipFree(s.d_off);
	(void)hipFree(s.d_cap);
	(void)hipFree(s.d_sum);
	(void)hipFree(s.d_lay);
	(void)hipHostFree(s.h_match);
	(void)hipFree(s.d_match);
	s = Slot();
}

int init_host_path(pcppx_ctx* c)
{
	if (c->host_ready)
		return PCPPX_OK;
	// three slots: the H2D copy of chunk k+1 overlaps the kernel of chunk k and the drain of chunk k-1
	c->nslots = kMaxSlots;
	for (uint32_t si = 0; si < c->nslots; ++si)
	{
		Slot& s = c->slots[si];
		bool good = ok(hipStreamCreateWithFlags(&s.st, hipStreamNonBlocking)) && ok(hipEventCreate(&s.done)) &&
		            ok(hipHostMalloc(reinterpret_cast<void**>(&s.h_data), kChunkBytes + 16)) &&
		            ok(hipHostMalloc(reinterpret_cast<void**>(&s.h_off), kChunkPackets * sizeof(uint64_t))) &&
		            ok(hipHostMalloc(reinterpret_cast<void**>(&s.h_cap), kChunkPackets * sizeof(uint32_t))) &&
		            ok(hipHostMalloc(reinterpret_cast<void**>(&s.h_sum), kChunkPackets * sizeof(pcppx_summary))) &&
		            ok(hipHostMalloc(reinterpret_cast<void**>(&s.h_lay),
		                             (size_t)kChunkPackets * PCPPX_MAX_LAYERS * sizeof(pcppx_layer))) &&
		            ok(hipMalloc(reinterpret_cast<void**>(&s.d_data), kChunkBytes + 16)) &&
		            ok(hipMalloc(reinterpret_cast<void**>(&s.d_off), kChunkPackets * sizeof(uint64_t))) &&
		            ok(hipMalloc(reinterpret_cast<void**>(&s.d_cap), kChunkPackets * sizeof(uint32_t))) &&
		            ok(hipMalloc(reinterpret_cast<void**>(&s.d_sum), kChunkPackets * sizeof(pcppx_summary))) &&
		            ok(hipMalloc(reinterpret_cast<void**>(&s.d_lay),
		                         (size_t)kChunkPackets * PCPPX_MAX_LAYERS * sizeof(pcppx_layer))) &&
		            ok(hipHostMalloc(reinterpret_cast<void**>(&s.h_match), kChunkPackets)) &&
		            ok(hipMalloc(reinterpret_cast<void**>(&s.d_match), kChunkPackets)) &&
		            ok(hipEventCreateWithFlags(&s.parsed, hipEventDisableTiming)) &&
		            ok(hipHostMalloc(reinterpret_cast<void**>(&s.h_brief), kChunkPackets * sizeof(pcppx_brief))) &&
		            ok(hipHostMalloc(reinterpret_cast<void**>(&s.h_total), 2 * sizeof(uint32_t))) &&
		            ok(hipMalloc(reinterpret_cast<void**>(&s.d_brief), kChunkPackets * sizeof(pcppx_brief))) &&
		            ok(hipMalloc(reinterpret_cast<void**>(&s.d_dense),
		                         (size_t)kChunkPackets * PCPPX_MAX_LAYERS * sizeof(pcppx_layer))) &&
		            ok(hipMalloc(reinterpret_cast<void**>(&s.d_dsum),
		                         (pcppx::dense_blocks(kChunkPackets) + 2) * sizeof(uint32_t)));
		if (!good)
		{
			for (Slot& t : c->slots)
				free_slot(t);
			return PCPPX_E_NOMEM;
		}
	}
	c->copier.start();
	c->host_ready = true;
	return PCPPX_OK;
}

// true if p is page-locked host memory the GPU can DMA from directly
bool is_pinned(const void* p)
{
	hipPointerAttribute_t a;
	if (hipPointerGetAttributes(&a, p) != hipSuccess)
	{
		(void)hipGetLastError();  // pageable memory: clear the error so launch checks do not see it
		return false;
	}
	return a.type == hipMemoryTypeHost;
}

// the device mapping of page-locked host memory (kernels store into it directly), or null
void* mapped(void* p)
{
	hipPointerAttribute_t a;
	if (hipPointerGetAttributes(&a, p) != hipSuccess || a.type != hipMemoryTypeHost || a.devicePointer == nullptr)
	{
		(void)hipGetLastError();
		return nullptr;
	}
	return a.devicePointer;
}

// Packets [i, j) of a host batch as one byte range [*base, *base + *bytes): ascending, each starting at most kMaxGap
// bytes after the previous one ends (packed batches; a memory-mapped capture's packets with their record headers
// between them, pcppx_pcap_map_batch): returns j, or i if packet i does not start such a run.
constexpr uint64_t kMaxGap = 256;
uint32_t contiguous_chunk(const pcppx_batch* b, uint32_t i, uint64_t* base, size_t* bytes)
{
	uint64_t end = b->offsets[i];
	*base = end;
	uint32_t j = i;
	while (j < b->n && j - i < kChunkPackets)
	{
		const uint64_t off = b->offsets[j];
		const uint32_t cap = b->caplens[j];
		if (off < end || off - end > kMaxGap || off + cap > b->data_len || off + cap < off)
			break;
		if (off + cap - *base > kChunkBytes)
			break;
		end = off + cap;
		++j;
	}
	*bytes = (size_t)(end - *base);
	return j;
}
constexpr uint32_t kMinRun = 4096;  // a shorter run that stops at a discontinuity is gathered per packet instead

// gather packets [i, j) of a host batch into the slot's pinned staging, rebasing offsets; returns j.
// Contiguous runs are not staged: *direct is then the source of the H2D copy, page-locked or not (the runtime DMAs a
// pageable range as fast as a page-locked one, 56 GB/s from a file map, profiles/r04f_h2d_probe.txt, where a copy
// into staging first ran at 30 GB/s per thread); scattered packets are gathered into the staging.
uint32_t stage_chunk(Slot& s, const pcppx_batch* b, uint32_t i, size_t* pos_out, const uint8_t** direct)
{
	*direct = nullptr;
	{
		uint64_t base = 0;
		size_t bytes = 0;
		const uint32_t j = contiguous_chunk(b, i, &base, &bytes);
		// a run that ends the batch, a long run, or one that stops only because the next packet (ascending) would not fit
		// the chunk: copied straight from the caller's bytes. (A next packet below the run -- an unordered batch -- is
		// no such reason: its offset minus the run's base would wrap.)
		if (j > i && (j == b->n || j - i >= kMinRun ||
		              (b->offsets[j] >= base && b->offsets[j] + b->caplens[j] - base > kChunkBytes)))
		{
			for (uint32_t k = i; k < j; ++k)
			{
				s.h_off[k - i] = b->offsets[k] - base;
				s.h_cap[k - i] = b->caplens[k];
			}
			*direct = b->data + base;
			*pos_out = bytes;
			return j;
		}
	}
	size_t pos = 0;
	uint32_t j = i;
	while (j < b->n && j - i < kChunkPackets)
	{
		const uint64_t off = b->offsets[j];
		const uint32_t cap = b->caplens[j];
		const bool in_bounds = off + cap <= b->data_len && off + cap >= off;
		const size_t take = in_bounds ? cap : 0;
		if (pos + take > kChunkBytes && j > i)
			break;
		if (in_bounds && cap <= kChunkBytes)
		{
			std::memcpy(s.h_data + pos, b->data + off, cap);
			s.h_off[j - i] = pos;
			pos += cap;
		}
		else
			s.h_off[j - i] = ~0ull >> 1;  // kernel flags PCPPX_F_BAD_DESC
		s.h_cap[j - i] = cap;
		++j;
	}
	*pos_out = pos;
	return j;
}

bool upload_chunk(Slot& s, size_t pos, uint32_t cnt, const uint8_t* direct = nullptr)
{
	return ok(hipMemcpyAsync(s.d_data, direct ? direct : s.h_data, pos ? pos : 1, hipMemcpyHostToDevice, s.st)) &&
	       ok(hipMemcpyAsync(s.d_off, s.h_off, cnt * sizeof(uint64_t), hipMemcpyHostToDevice, s.st)) &&
	       ok(hipMemcpyAsync(s.d_cap, s.h_cap, cnt * sizeof(uint32_t), hipMemcpyHostToDevice, s.st));
}

void free_filter(pcppx_ctx* c)
{
	(void)hipFree(c->d_keys);
	(void)hipFree(c->d_first);
	(void)hipFree(c->d_stats);
	c->d_keys = c->d_first = nullptr;
	c->d_stats = nullptr;
	c->flow_slots = 0;
	c->seq = 0;
}

int flow_count(pcppx_ctx* c, const pcppx_summary* summary, const uint32_t* keys_in, const uint32_t* caplens, uint32_t n,
               uint32_t* keys, uint64_t* packets, uint64_t* bytes, uint32_t capacity, uint64_t* stats, void* hip_stream);

// forget every slot's chunk without copying it out: after an error mid-call, and at the start of each host
// call, so that a later call never drains a stale chunk into its own (possibly smaller) output arrays
void abandon_slots(pcppx_ctx* c)
{
	for (Slot& s : c->slots)
	{
		if (s.st)
			(void)hipStreamSynchronize(s.st);
		s.busy = false;
	}
	(void)hipGetLastError();
}

// copy a finished chunk's records from pinned memory to the caller's arrays (nothing to copy when the
// caller's arrays are pinned: the chunk's D2H wrote them directly)
// (dense_direct: the DENSE chains were pushed into the caller's array through its device mapping; otherwise they sit in
// the slot's staging buffer -- a pinned caller array without a device mapping takes this path too)
void drain(CopyPool& cp, Slot& s, pcppx_records* out, bool direct_out, bool dense, bool dense_direct, uint64_t* written)
{
	if (dense && s.ml && out->layers)  // the chunk's chains: [batch total up to its end - its own, batch total)
	{
		s.dense_count = s.h_total[0];
		s.dense_first = s.h_total[1] - s.h_total[0];
		*written = s.h_total[1] > *written ? s.h_total[1] : *written;
	}
	if (!direct_out)
	{
		if (out->summary)
			cp.copy(out->summary + s.first, s.h_sum, (size_t)s.count * sizeof(pcppx_summary));
		if (out->brief)
			cp.copy(out->brief + s.first, s.h_brief, (size_t)s.count * sizeof(pcppx_brief));
		if (s.ml && out->layers && !dense)
			cp.copy(out->layers + (size_t)s.first * s.ml, s.h_lay, (size_t)s.count * s.ml * sizeof(pcppx_layer));
	}
	if (s.ml && out->layers && dense && !dense_direct)
		cp.copy(out->layers + s.dense_first, s.h_lay, (size_t)s.dense_count * sizeof(pcppx_layer));
	if (out->flow_keys)  // the dense hash5 column, from the host copy of the summaries / briefs
		for (uint32_t k = 0; k < s.count; ++k)
			out->flow_keys[s.first + k] = out->summary ? out->summary[s.first + k].hash5 : out->brief[s.first + k].hash5;
	s.busy = false;
}

// pcppx_parse_batch_host's chunk pipeline (argument checks done; slots idle on entry)
int parse_host_run(pcppx_ctx* c, const pcppx_batch* b, const pcppx_opts* o, pcppx_records* r)
{
	int rc = PCPPX_OK;
	const uint32_t ml = o->max_layers;
	const bool rows = ml != 0 && r->layers != nullptr;
	const bool dense = rows && o->layout == PCPPX_LAYOUT_DENSE;
	// a NIC ring / pcppx_host_alloc result buffer: records come back by DMA straight into the caller's arrays
	const bool direct_out = (r->summary == nullptr || is_pinned(r->summary)) &&
	                        (r->brief == nullptr || is_pinned(r->brief)) && (!rows || is_pinned(r->layers));
	uint64_t written = 0;
	// DENSE: the chains are pushed by a kernel through the device mapping of page-locked memory (the caller's array, or
	// the slot's staging buffer), their positions chained on the device chunk after chunk -- no host round trip to learn
	// a chunk's count before its copy
	const uint32_t kTot = pcppx::dense_blocks(kChunkPackets);  // d_dsum[kTot]: the chunk's, [kTot + 1]: cumulative
	// a page-locked caller array without a device mapping (pinned by another runtime, say) is still filled: its chains
	// are staged like a pageable array's (the FIXED rows reach such an array by DMA)
	pcppx_layer* lay_map = dense && direct_out ? static_cast<pcppx_layer*>(mapped(r->layers)) : nullptr;
	const bool dense_direct = lay_map != nullptr;
	Slot* prev = nullptr;  // DENSE: the previous chunk (its cumulative count is this chunk's base)
	uint32_t i = 0, k = 0;
	while (i < b->n)
	{
		Slot& s = c->slots[k % c->nslots];
		if (s.busy)
		{
			if (!ok(hipEventSynchronize(s.done)))
				return PCPPX_E_HIP;
			drain(c->copier, s, r, direct_out, dense, dense_direct, &written);
		}
		size_t pos = 0;
		const uint8_t* direct = nullptr;
		const uint32_t j = stage_chunk(s, b, i, &pos, &direct);
		const uint32_t cnt = j - i;
		if (!upload_chunk(s, pos, cnt, direct))
			return PCPPX_E_HIP;
		pcppx_batch db{ s.d_data, s.d_off, s.d_cap, pos, cnt, b->linktype, 0 };
		pcppx_records dr{};
		dr.summary = r->summary ? s.d_sum : nullptr;
		dr.brief = r->brief ? s.d_brief : nullptr;
		dr.layers = ml ? s.d_lay : nullptr;
		pcppx_opts fo = resolve_window(c, o);
		fo.layout = PCPPX_LAYOUT_FIXED;  // DENSE is compacted from the chunk's FIXED rows below
		unsigned long long* win = window_sample(c, o);
		rc = pcppx::launch_parse(&db, &fo, &dr, s.st, nullptr, win);
		if (rc == PCPPX_OK)
			note_window(c, s.st, win);
		if (rc == PCPPX_OK && dense)
			rc = pcppx::launch_dense_compact(s.d_lay,
			                                 dr.brief ? reinterpret_cast<const uint8_t*>(s.d_brief) + 14
			                                          : reinterpret_cast<const uint8_t*>(s.d_sum) + 14,
			                                 dr.brief ? sizeof(pcppx_brief) : sizeof(pcppx_summary), cnt, ml, s.d_dense,
			                                 s.d_dsum, s.d_dsum + pcppx::dense_blocks(kChunkPackets), s.st);
		if (rc != PCPPX_OK)
			return rc;
		pcppx_summary* hs = direct_out && r->summary ? r->summary + i : s.h_sum;
		pcppx_brief* hb = direct_out && r->brief ? r->brief + i : s.h_brief;
		pcppx_layer* hl = direct_out && rows ? r->layers + (size_t)i * ml : s.h_lay;
		bool good = (!r->summary ||
		             ok(hipMemcpyAsync(hs, s.d_sum, cnt * sizeof(pcppx_summary), hipMemcpyDeviceToHost, s.st))) &&
		            (!r->brief || ok(hipMemcpyAsync(hb, s.d_brief, cnt * sizeof(pcppx_brief), hipMemcpyDeviceToHost, s.st)));
		if (dense)
		{
			pcppx_layer* to = dense_direct ? lay_map : static_cast<pcppx_layer*>(mapped(s.h_lay));
			good = good && to != nullptr && (prev == nullptr || ok(hipStreamWaitEvent(s.st, prev->parsed, 0))) &&
			       pcppx::launch_dense_push(s.d_dense, s.d_dsum + kTot, prev ? prev->d_dsum + kTot + 1 : nullptr, to,
			                                dense_direct, s.d_dsum + kTot + 1, s.st) == PCPPX_OK &&
			       ok(hipEventRecord(s.parsed, s.st)) &&
			       ok(hipMemcpyAsync(s.h_total, s.d_dsum + kTot, 2 * sizeof(uint32_t), hipMemcpyDeviceToHost, s.st)) &&
			       ok(hipEventRecord(s.done, s.st));
			prev = &s;
		}
		else
			good = good &&
			       (!rows ||
			        ok(hipMemcpyAsync(hl, s.d_lay, (size_t)cnt * ml * sizeof(pcppx_layer), hipMemcpyDeviceToHost, s.st))) &&
			       ok(hipEventRecord(s.done, s.st));
		if (!good)
			return PCPPX_E_HIP;
		s.busy = true;
		s.first = i;
		s.count = cnt;
		s.ml = ml;
		i = j;
		++k;
	}
	for (Slot& s : c->slots)
		if (s.busy)
		{
			if (!ok(hipEventSynchronize(s.done)))
				return PCPPX_E_HIP;
			drain(c->copier, s, r, direct_out, dense, dense_direct, &written);
		}
	r->layers_written = dense ? written : (rows ? (uint64_t)b->n * ml : 0);
	return PCPPX_OK;
}

// pcppx_filter_batch_host's chunk pipeline (argument checks done; slots idle on entry)
int filter_host_run(pcppx_ctx* c, const pcppx_batch* b, const pcppx_match_spec* spec, uint8_t* matched,
                    pcppx_packet_stats* stats)
{
	int rc = PCPPX_OK;
	pcppx_opts o;
	pcppx_default_opts(&o);
	o.want_checksums = 0;  // the worker reads addresses, ports and the protocol mask only
	const uint32_t ml = o.max_layers;
	uint32_t i = 0, k = 0;
	Slot* prev = nullptr;
	while (i < b->n)
	{
		Slot& s = c->slots[k % c->nslots];
		if (s.busy)
		{
			if (!ok(hipEventSynchronize(s.done)))
				return PCPPX_E_HIP;
			std::memcpy(matched + s.first, s.h_match, s.count);
			s.busy = false;
		}
		size_t pos = 0;
		const uint8_t* direct = nullptr;
		const uint32_t j = stage_chunk(s, b, i, &pos, &direct);
		const uint32_t cnt = j - i;
		if (!upload_chunk(s, pos, cnt, direct))
			return PCPPX_E_HIP;
		// the flow table is shared by consecutive chunks: chunk k's lookups run after chunk k-1's marks
		if (prev != nullptr && !ok(hipStreamWaitEvent(s.st, prev->done, 0)))
			return PCPPX_E_HIP;
		pcppx_batch db{ s.d_data, s.d_off, s.d_cap, pos, cnt, b->linktype, 0 };
		pcppx_records dr{};
		dr.summary = s.d_sum;
		dr.layers = s.d_lay;
		const pcppx_opts eo = resolve_window(c, &o);
		unsigned long long* win = window_sample(c, &o);
		rc = pcppx::launch_parse(&db, &eo, &dr, s.st, nullptr, win);
		if (rc == PCPPX_OK)
			note_window(c, s.st, win);
		if (rc == PCPPX_OK)
			rc = pcppx::launch_filter(&db, &dr, ml, spec, c->seq + i, c->d_keys, c->d_first, c->flow_slots,
			                          s.d_match, c->d_stats, s.st);
		if (rc != PCPPX_OK)
			return rc;
		if (!ok(hipMemcpyAsync(s.h_match, s.d_match, cnt, hipMemcpyDeviceToHost, s.st)) ||
		    !ok(hipEventRecord(s.done, s.st)))
			return PCPPX_E_HIP;
		s.busy = true;
		s.first = i;
		s.count = cnt;
		prev = &s;
		i = j;
		++k;
	}
	for (Slot& s : c->slots)
		if (s.busy)
		{
			if (!ok(hipEventSynchronize(s.done)))
				return PCPPX_E_HIP;
			std::memcpy(matched + s.first, s.h_match, s.count);
			s.busy = false;
		}
	c->seq += b->n;
	if (stats != nullptr &&
	    (!ok(hipMemcpy(stats, c->d_stats, sizeof(pcppx_packet_stats), hipMemcpyDeviceToHost))))
		return PCPPX_E_HIP;
	return PCPPX_OK;
}
}  // namespace

extern "C"
{
	int pcppx_abi_version(void)
	{
		return PCPPX_ABI_VERSION;
	}

	const char* pcppx_strerror(int err)
	{
		switch (err)
		{
		case PCPPX_OK: return "ok";
		case PCPPX_E_INVAL: return "invalid argument";
		case PCPPX_E_NODEV: return "no such HIP device";
		case PCPPX_E_HIP: return "HIP runtime error";
		case PCPPX_E_NOMEM: return "out of device or pinned memory";
		case PCPPX_E_LINKTYPE: return "link type not handled";
		default: return "unknown error";
		}
	}

	int pcppx_runtime_info(int device, char* buf, size_t len)
	{
		if (buf == nullptr || len == 0)
			return PCPPX_E_INVAL;
		int rt = 0, drv = 0;
		(void)hipRuntimeGetVersion(&rt);
		(void)hipDriverGetVersion(&drv);
		hipDeviceProp_t prop;
		if (!ok(hipGetDeviceProperties(&prop, device)))
		{
			snprintf(buf, len, "hip runtime %d driver %d, device %d unavailable", rt, drv, device);
			return PCPPX_E_NODEV;
		}
		snprintf(buf, len, "hip runtime %d driver %d, device %d: %s (%s), %d CUs, %.1f GiB", rt, drv, device,
		         prop.name, prop.gcnArchName, prop.multiProcessorCount,
		         (double)prop.totalGlobalMem / (1024.0 * 1024.0 * 1024.0));
		return PCPPX_OK;
	}

	int pcppx_device_count(int* out)
	{
		if (out == nullptr)
			return PCPPX_E_INVAL;
		int n = 0;
		if (!ok(hipGetDeviceCount(&n)))
			n = 0;
		*out = n;
		return PCPPX_OK;
	}

	void pcppx_default_opts(pcppx_opts* o)
	{
		if (o == nullptr)
			return;
		o->parse_until_family = 0;  // UnknownProtocol
		o->parse_until_osi = 8;     // OsiModelLayerUnknown
		o->want_checksums = 1;
		o->max_layers = PCPPX_MAX_LAYERS;
		o->window = PCPPX_WINDOW_DEFAULT;
		o->layout = PCPPX_LAYOUT_FIXED;
		o->reserved[0] = o->reserved[1] = o->reserved[2] = 0;
	}

	int pcppx_open(int device, pcppx_ctx** out)
	{
		if (out == nullptr)
			return PCPPX_E_INVAL;
		*out = nullptr;
		int n = 0;
		if (!ok(hipGetDeviceCount(&n)) || device < 0 || device >= n)
			return PCPPX_E_NODEV;
		if (!ok(hipSetDevice(device)))
			return PCPPX_E_HIP;
		pcppx_ctx* c = new (std::nothrow) pcppx_ctx();
		if (c == nullptr)
			return PCPPX_E_NOMEM;
		c->device = device;
		if (!ok(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking)))
		{
			delete c;
			return PCPPX_E_HIP;
		}
		*out = c;
		return PCPPX_OK;
	}

	void pcppx_close(pcppx_ctx* c)
	{
		if (c == nullptr)
			return;
		(void)hipSetDevice(c->device);
		(void)hipStreamSynchronize(c->stream);
		if (c->host_ready)
			c->copier.stop();
		for (Slot& s : c->slots)
		{
			if (s.st)
				(void)hipStreamSynchronize(s.st);
			free_slot(s);
		}
		free_filter(c);
		if (c->flow_pending)
			(void)hipEventSynchronize(c->flow_done);
		if (c->stats_pending)
			(void)hipEventSynchronize(c->stats_done);
		// the flow / stats scratch is stream-ordered memory (hipMallocAsync): released on the context's stream
		if (c->d_flow_queues)
			(void)hipFreeAsync(c->d_flow_queues, c->stream);
		if (c->d_flow_fill)
			(void)hipFreeAsync(c->d_flow_fill, c->stream);
		if (c->d_wave_stats)
			(void)hipFreeAsync(c->d_wave_stats, c->stream);
		(void)hipStreamSynchronize(c->stream);
		if (c->win_ready)
		{
			(void)hipStreamSynchronize(c->win_stream);
			(void)hipStreamDestroy(c->win_stream);
			(void)hipEventDestroy(c->win_parsed);
			(void)hipEventDestroy(c->win_copied);
			(void)hipFree(c->d_win);
			(void)hipHostFree(c->h_win);
		}
		if (c->flow_done)
			(void)hipEventDestroy(c->flow_done);
		if (c->stats_done)
			(void)hipEventDestroy(c->stats_done);
		(void)hipStreamDestroy(c->stream);
		delete c;
	}

	int pcppx_window_choice(pcppx_ctx* c, int want_checksums, int* window)
	{
		if (c == nullptr || window == nullptr)
			return PCPPX_E_INVAL;
		if (!ok(hipSetDevice(c->device)))
			return PCPPX_E_HIP;
		update_window(c, true);
		pcppx_opts o;
		pcppx_default_opts(&o);
		o.want_checksums = want_checksums ? 1 : 0;
		*window = resolve_window(c, &o).window;
		return PCPPX_OK;
	}

	void* pcppx_ctx_stream(pcppx_ctx* c)
	{
		return c ? static_cast<void*>(c->stream) : nullptr;
	}

	int pcppx_sync(pcppx_ctx* c)
	{
		if (c == nullptr)
			return PCPPX_E_INVAL;
		if (!ok(hipSetDevice(c->device)) || !ok(hipStreamSynchronize(c->stream)))
			return PCPPX_E_HIP;
		return PCPPX_OK;
	}

	int pcppx_parse_batch_device(pcppx_ctx* c, const pcppx_batch* b, const pcppx_opts* o, pcppx_records* r,
	                             void* hip_stream)
	{
		if (c == nullptr || b == nullptr || r == nullptr || valid_opts(o) != PCPPX_OK)
			return PCPPX_E_INVAL;
		r->layout = o->layout;  // set for an empty batch too: a reused records struct keeps no stale count
		r->layers_written = 0;
		if (b->n == 0)
			return PCPPX_OK;
		if (b->data == nullptr || b->offsets == nullptr || b->caplens == nullptr || !valid_device_records(o, r))
			return PCPPX_E_INVAL;
		if (!ok(hipSetDevice(c->device)))
			return PCPPX_E_HIP;
		r->layers_written = o->max_layers ? (uint64_t)b->n * o->max_layers : 0;
		return device_parse(c, b, o, r, nullptr, static_cast<hipStream_t>(hip_stream));
	}

	int pcppx_parse_batch_host(pcppx_ctx* c, const pcppx_batch* b, const pcppx_opts* o, pcppx_records* r)
	{
		if (c == nullptr || b == nullptr || r == nullptr || valid_opts(o) != PCPPX_OK)
			return PCPPX_E_INVAL;
		r->layout = o->layout;  // set for an empty batch too: a reused records struct keeps no stale count
		r->layers_written = 0;
		if (b->n == 0)
			return PCPPX_OK;
		if (b->data == nullptr || b->offsets == nullptr || b->caplens == nullptr ||
		    (r->summary == nullptr && r->brief == nullptr) || (o->max_layers != 0 && r->layers == nullptr))
			return PCPPX_E_INVAL;
		// device-path-only outputs
		if (r->tuples != nullptr || r->proto_stats != nullptr || o->layout == PCPPX_LAYOUT_PACKED)
			return PCPPX_E_INVAL;
		// DENSE positions are 32-bit (the device's running totals, the facade's per-page indexes): a batch whose
		// n * max_layers could exceed them is refused rather than wrapped
		if (o->layout == PCPPX_LAYOUT_DENSE && (uint64_t)b->n * o->max_layers > (uint64_t)UINT32_MAX)
			return PCPPX_E_INVAL;
		if (!ok(hipSetDevice(c->device)))
			return PCPPX_E_HIP;
		int rc = init_host_path(c);
		if (rc != PCPPX_OK)
			return rc;
		abandon_slots(c);
		rc = parse_host_run(c, b, o, r);
		if (rc != PCPPX_OK)
			abandon_slots(c);
		return rc;
	}

	int pcppx_filter_device(pcppx_ctx* c, const pcppx_batch* b, const pcppx_records* r, uint8_t max_layers,
	                        const pcppx_match_spec* spec, uint64_t seq_base, uint64_t* flow_keys, uint64_t* flow_first,
	                        uint32_t capacity, uint8_t* matched, pcppx_packet_stats* stats, void* hip_stream)
	{
		if (c == nullptr || b == nullptr || r == nullptr || spec == nullptr || max_layers == 0 ||
		    max_layers > PCPPX_MAX_LAYERS || capacity == 0 || (capacity & (capacity - 1)) != 0)
			return PCPPX_E_INVAL;
		if (b->n == 0)
			return PCPPX_OK;
		if (b->data == nullptr || b->offsets == nullptr || r->summary == nullptr || r->layers == nullptr ||
		    flow_keys == nullptr || flow_first == nullptr || matched == nullptr || stats == nullptr ||
		    r->layout != PCPPX_LAYOUT_FIXED)
			return PCPPX_E_INVAL;
		if (!ok(hipSetDevice(c->device)))
			return PCPPX_E_HIP;
		return pcppx::launch_filter(b, r, max_layers, spec, seq_base, flow_keys, flow_first, capacity, matched, stats,
		                            static_cast<hipStream_t>(hip_stream));
	}

	int pcppx_parse_batch_device_reasm(pcppx_ctx* c, const pcppx_batch* b, const pcppx_opts* o, pcppx_records* r,
	                                   pcppx_reasm_info* info, void* hip_stream)
	{
		if (c == nullptr || b == nullptr || r == nullptr || valid_opts(o) != PCPPX_OK || o->max_layers == 0 ||
		    o->layout != PCPPX_LAYOUT_FIXED)
			return PCPPX_E_INVAL;
		if (b->n == 0)
			return PCPPX_OK;
		if (b->data == nullptr || b->offsets == nullptr || b->caplens == nullptr || r->summary == nullptr ||
		    r->layers == nullptr || info == nullptr)
			return PCPPX_E_INVAL;
		if (!ok(hipSetDevice(c->device)))
			return PCPPX_E_HIP;
		r->layout = PCPPX_LAYOUT_FIXED;
		return device_parse(c, b, o, r, info, static_cast<hipStream_t>(hip_stream));
	}

	int pcppx_reasm_device(pcppx_ctx* c, const pcppx_batch* b, const pcppx_records* r, uint8_t max_layers,
	                       pcppx_reasm_info* info, void* hip_stream)
	{
		if (c == nullptr || b == nullptr || r == nullptr || max_layers == 0 || max_layers > PCPPX_MAX_LAYERS)
			return PCPPX_E_INVAL;
		if (b->n == 0)
			return PCPPX_OK;
		if (b->data == nullptr || b->offsets == nullptr || r->summary == nullptr || r->layers == nullptr ||
		    info == nullptr || r->layout != PCPPX_LAYOUT_FIXED)
			return PCPPX_E_INVAL;
		if (!ok(hipSetDevice(c->device)))
			return PCPPX_E_HIP;
		return pcppx::launch_reasm(b, r, max_layers, info, static_cast<hipStream_t>(hip_stream));
	}

	int pcppx_filter_reset(pcppx_ctx* c, uint32_t capacity)
	{
		if (c == nullptr || (capacity & (capacity - 1)) != 0)
			return PCPPX_E_INVAL;
		if (capacity == 0)
			capacity = kDefaultFlowSlots;
		if (!ok(hipSetDevice(c->device)))
			return PCPPX_E_HIP;
		for (Slot& s : c->slots)
			if (s.st && !ok(hipStreamSynchronize(s.st)))
				return PCPPX_E_HIP;
		if (capacity != c->flow_slots)
		{
			free_filter(c);
			if (!ok(hipMalloc(reinterpret_cast<void**>(&c->d_keys), (size_t)capacity * 8)) ||
			    !ok(hipMalloc(reinterpret_cast<void**>(&c->d_first), (size_t)capacity * 8)) ||
			    !ok(hipMalloc(reinterpret_cast<void**>(&c->d_stats), sizeof(pcppx_packet_stats))))
			{
				free_filter(c);
				return PCPPX_E_NOMEM;
			}
			c->flow_slots = capacity;
		}
		c->seq = 0;
		const bool good = ok(hipMemsetAsync(c->d_keys, 0, (size_t)capacity * 8, c->stream)) &&
		                  ok(hipMemsetAsync(c->d_first, 0, (size_t)capacity * 8, c->stream)) &&
		                  ok(hipMemsetAsync(c->d_stats, 0, sizeof(pcppx_packet_stats), c->stream)) &&
		                  ok(hipStreamSynchronize(c->stream));
		return good ? PCPPX_OK : PCPPX_E_HIP;
	}

	int pcppx_filter_batch_host(pcppx_ctx* c, const pcppx_batch* b, const pcppx_match_spec* spec, uint8_t* matched,
	                            pcppx_packet_stats* stats)
	{
		if (c == nullptr || b == nullptr || spec == nullptr)
			return PCPPX_E_INVAL;
		if (b->n != 0 && (b->data == nullptr || b->offsets == nullptr || b->caplens == nullptr || matched == nullptr))
			return PCPPX_E_INVAL;
		if (!ok(hipSetDevice(c->device)))
			return PCPPX_E_HIP;
		int rc = c->flow_slots ? PCPPX_OK : pcppx_filter_reset(c, 0);
		if (rc == PCPPX_OK)
			rc = init_host_path(c);
		if (rc != PCPPX_OK)
			return rc;
		abandon_slots(c);
		rc = filter_host_run(c, b, spec, matched, stats);
		if (rc != PCPPX_OK)
			abandon_slots(c);
		return rc;
	}

	int pcppx_flow_count_device(pcppx_ctx* c, const pcppx_summary* summary, const uint32_t* caplens, uint32_t n,
	                            uint32_t* keys, uint64_t* packets, uint64_t* bytes, uint32_t capacity,
	                            uint64_t* stats, void* hip_stream)
	{
		return flow_count(c, summary, nullptr, caplens, n, keys, packets, bytes, capacity, stats, hip_stream);
	}

	int pcppx_flow_count_keys_device(pcppx_ctx* c, const uint32_t* keys_in, const uint32_t* caplens, uint32_t n,
	                                 uint32_t* keys, uint64_t* packets, uint64_t* bytes, uint32_t capacity,
	                                 uint64_t* stats, void* hip_stream)
	{
		return flow_count(c, nullptr, keys_in, caplens, n, keys, packets, bytes, capacity, stats, hip_stream);
	}
}

namespace
{
// pcppx_flow_count_device / _keys_device: keys from the summaries or from a dense column (exactly one non-null)
int flow_count(pcppx_ctx* c, const pcppx_summary* summary, const uint32_t* keys_in, const uint32_t* caplens, uint32_t n,
               uint32_t* keys, uint64_t* packets, uint64_t* bytes, uint32_t capacity, uint64_t* stats, void* hip_stream)
{
		if (c == nullptr || capacity == 0 || (capacity & (capacity - 1)) != 0)
			return PCPPX_E_INVAL;
		if (n == 0)
			return PCPPX_OK;
		if ((summary == nullptr) == (keys_in == nullptr) || caplens == nullptr || keys == nullptr || packets == nullptr ||
		    bytes == nullptr || stats == nullptr)
			return PCPPX_E_INVAL;
		if (!ok(hipSetDevice(c->device)))
			return PCPPX_E_HIP;
		hipStream_t st = static_cast<hipStream_t>(hip_stream);
		const uint32_t parts = pcppx::flow_partitions(capacity);
		const uint32_t rec_cap = pcppx::flow_queue_capacity(n, capacity);
		// the context's previous flow work (possibly queued on another stream) owns the scratch until flow_done; a
		// larger one is allocated in stream order behind that wait
		uint64_t have = c->flow_queue_recs * 16;
		const int src = ensure_scratch(st, &c->d_flow_queues, &have, (uint64_t)parts * rec_cap * 16, &c->flow_done,
		                               c->flow_pending);
		c->flow_queue_recs = have / 16;
		if (src != PCPPX_OK)
			return src;
		if (c->d_flow_fill == nullptr)
		{
			if (!ok(hipMallocAsync(reinterpret_cast<void**>(&c->d_flow_fill), 1024 * sizeof(uint32_t), st)) ||
			    !ok(hipMemsetAsync(c->d_flow_fill, 0, 1024 * sizeof(uint32_t), st)))
				return PCPPX_E_NOMEM;
		}
		const int rc = pcppx::launch_flow_count_part(summary, keys_in, caplens, n, keys, packets, bytes, capacity, stats,
		                                             c->d_flow_queues, rec_cap, c->d_flow_fill, st);
		if (rc != PCPPX_OK)
			return rc;
		if (!ok(hipEventRecord(c->flow_done, st)))
			return PCPPX_E_HIP;
		c->flow_pending = true;
		return PCPPX_OK;
	}
}

namespace
{
// PCPPX_LAYOUT_PACKED -> FIXED, the chain lengths at n_layers[i * stride]
int unpack_packed(const uint8_t* n_layers, size_t stride, const pcppx_layer* packed, uint64_t n, uint32_t max_layers,
                  pcppx_layer* fixed)
{
	if (packed == nullptr || fixed == nullptr || max_layers == 0 || max_layers > PCPPX_PACKED_MAX_LAYERS)
		return PCPPX_E_INVAL;
	uint64_t pos = 0;
	for (uint64_t i = 0; i < n; ++i)
	{
		if (i % 64 == 0)
			pos = i * max_layers;  // tile t's run starts at entry 64 * t * max_layers
		const uint32_t nl = n_layers[i * stride];
		const uint32_t cnt = nl < max_layers ? nl : max_layers;
		for (uint32_t k = 0; k < max_layers; ++k)
			fixed[i * max_layers + k] = k < cnt ? packed[pos + k] : pcppx_layer{};
		pos += cnt;
	}
	return PCPPX_OK;
}
}  // namespace

extern "C"
{
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

	int pcppx_unpack_layers(const pcppx_summary* summary, const pcppx_layer* packed, uint64_t n, uint32_t max_layers,
	                        pcppx_layer* fixed)
	{
		if (n == 0)
			return PCPPX_OK;
		if (summary == nullptr)
			return PCPPX_E_INVAL;
		return unpack_packed(&summary->n_layers, sizeof(pcppx_summary), packed, n, max_layers, fixed);
	}

	int pcppx_unpack_layers_brief(const pcppx_brief* brief, const pcppx_layer* packed, uint64_t n, uint32_t max_layers,
	                              pcppx_layer* fixed)
	{
		if (n == 0)
			return PCPPX_OK;
		if (brief == nullptr)
			return PCPPX_E_INVAL;
		return unpack_packed(&brief->n_layers, sizeof(pcppx_brief), packed, n, max_layers, fixed);
	}
}
