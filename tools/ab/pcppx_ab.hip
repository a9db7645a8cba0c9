// pcppx_ab.hip — TOOLS ONLY: the A/B and diagnostic kernels of the parse path, built into
// tools/ab/libpcppx_ab.so (never into the product library pcapplusplus_amd/libpcppx.so).
//
// This translation unit includes the product kernels (pcapplusplus_amd/csrc/pcppx_kernels.hip) and adds
//   - the lane-per-packet parse kernel (the round-1 baseline: one lane streams one whole packet), used as an
//     independent cross-check of the tile kernel in tests/ and as the "before" leg of measurements;
//   - tile-kernel shape variants (occupancy, stream windows, cached vs non-temporal loads) and the
//     stream-only diagnostic, whose measurements chose the product shape (profiles/r01_ab_*.txt);
//   - read-ceiling diagnostics (tile-shaped and grid-stride streaming reads of the batch bytes);
//   - the flow-table shape variants (block threads / LDS slots / batch / hot-flow threshold / prefetch).
// Entry points are plain C; everything else is hidden.
#include "../../pcapplusplus_amd/csrc/pcppx_kernels.hip"

#define PCPPX_AB_API extern "C" __attribute__((visibility("default")))

namespace pcppx
{
namespace
{
constexpr int kSlotDw = 33;      // 32 dwords of staged bytes + 1 pad dword: consecutive lanes land on different banks
constexpr int kStageChunks = 8;  // 8 x 16 B = 128 B staged per packet

// ================= lane kernel: one lane streams one whole packet (reference / fallback) =================
__global__ __launch_bounds__(kBlock) void parse_lane_kernel(Params prm)
{
	__shared__ uint32_t stage[kBlock * kSlotDw];

	const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
	if (i >= prm.n)
		return;
	pcppx_summary* sum_out = prm.summary + i;
	const uint64_t off = prm.offsets[i];
	const uint32_t cap = prm.caplens[i];
	bool empty;
	uint32_t bad = desc_flags(off, cap, prm.data_len, &empty);
	if (bad || empty)
	{
		write_summary(sum_out, 0, 0, 0, bad, 0, -1, 0, 0, 0, 0, 0);
		return;
	}

	Pkt p;
	p.g = (gptr8)(prm.data + off);
	p.a0 = (uintptr_t)p.g & ~(uintptr_t)15;
	p.mis = (uint32_t)((uintptr_t)p.g - p.a0);
	{
		uint32_t need = (p.mis + cap + 15) >> 4;
		p.nch = need < kStageChunks ? need : kStageChunks;
		lptr32w slot = (lptr32w)(stage) + threadIdx.x * kSlotDw;
		uint4 v[kStageChunks];
#pragma unroll
		for (int c = 0; c < kStageChunks; ++c)
			if ((uint32_t)c < p.nch)
				v[c] = ld16(p.a0 + 16 * c);
#pragma unroll
		for (int c = 0; c < kStageChunks; ++c)
			if ((uint32_t)c < p.nch)
			{
				slot[4 * c + 0] = v[c].x;
				slot[4 * c + 1] = v[c].y;
				slot[4 * c + 2] = v[c].z;
				slot[4 * c + 3] = v[c].w;
			}
		p.s = reinterpret_cast<lptr8>(slot);
		uint32_t staged = 16 * p.nch - p.mis;
		p.lim = staged < cap ? staged : cap;
	}

	uint2* lay_out = prm.layers ? reinterpret_cast<uint2*>(prm.layers) + (size_t)i * prm.max_layers : nullptr;
	Walk w = walk_chain(p, cap, prm, lay_out);
	uint32_t h5, h5d, h2;
	hashes(p, w, h5, h5d, h2);
	uint32_t flags = w.flags, ipc = 0, ips = 0, l4c = 0, l4s = 0;
	if (prm.want_csum)
	{
		if (w.v4 >= 0)
		{
			ipc = ipv4_checksum(p, w, &ips);
			flags |= PCPPX_F_IP_CSUM | (ipc == ips ? PCPPX_F_IP_CSUM_OK : 0);
		}
		if (w.l4i >= 0)
		{
			l4c = l4_checksum(p, w, range_residue(p, w.l4o, w.l4o + w.l4dlen), &l4s);
			flags |= PCPPX_F_L4_CSUM | (l4c == l4s ? PCPPX_F_L4_CSUM_OK : 0);
		}
	}
	write_summary(sum_out, h5, h5d, h2, flags, w.n_layers, w.l4i, w.mask, ipc, ips, l4c, l4s);
}

// ---- diagnostic streaming kernels (opts.variant 3/4): the read ceiling of the access pattern ----
// variant 3: 64-lane blocks, each wave sums one contiguous tile-sized span (like the tile kernel);
// variant 4: 256-lane blocks, grid-stride over the whole buffer, 4 x 16 B per lane in flight.
__global__ __launch_bounds__(kTile) void diag_tile_read(const uint8_t* data, uint64_t len, uint32_t per_wave,
                                                         uint32_t* out)
{
	const uint64_t base = (uint64_t)blockIdx.x * per_wave;
	uint32_t acc = 0;
	for (uint32_t c = threadIdx.x; 16ull * c < per_wave; c += 4 * kTile)
	{
		uint4 v[4];
#pragma unroll
		for (int k = 0; k < 4; ++k)
		{
			const uint64_t a = base + 16ull * (c + k * kTile);
			v[k] = a + 16 <= len ? ld16((uintptr_t)data + a) : make_uint4(0, 0, 0, 0);
		}
#pragma unroll
		for (int k = 0; k < 4; ++k)
			acc += halves(v[k].x) + halves(v[k].y) + halves(v[k].z) + halves(v[k].w);
	}
	acc = wave_incl_scan(acc);
	if (threadIdx.x == 63)
		out[blockIdx.x] = acc;
}

// variant 7: the tile-shaped read of variant 3 plus the parse's record stores -- each wave also writes w_per_wave bytes of
// non-temporal 16-B stores (config 3: 65.6 B of records per 333-B packet, 0.195 of the bytes read): the traffic floor of
// the checksum kernel's read + write mix without its header gather and parse
__global__ __launch_bounds__(kTile) void diag_tile_rw(const uint8_t* data, uint64_t len, uint32_t per_wave,
                                                       uint8_t* wout, uint32_t w_per_wave, uint32_t* out)
{
	const uint64_t base = (uint64_t)blockIdx.x * per_wave;
	uint32_t acc = 0;
	for (uint32_t c = threadIdx.x; 16ull * c < per_wave; c += 4 * kTile)
	{
		uint4 v[4];
#pragma unroll
		for (int k = 0; k < 4; ++k)
		{
			const uint64_t a = base + 16ull * (c + k * kTile);
			v[k] = a + 16 <= len ? ld16((uintptr_t)data + a) : make_uint4(0, 0, 0, 0);
		}
#pragma unroll
		for (int k = 0; k < 4; ++k)
			acc += halves(v[k].x) + halves(v[k].y) + halves(v[k].z) + halves(v[k].w);
	}
	acc = wave_incl_scan(acc);
	typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
	u32x4* w = reinterpret_cast<u32x4*>(wout + (uint64_t)blockIdx.x * w_per_wave);
	for (uint32_t c = threadIdx.x; 16 * c < w_per_wave; c += kTile)
	{
		u32x4 x;
		x.x = acc + c; x.y = acc; x.z = c; x.w = blockIdx.x;
		__builtin_nontemporal_store(x, w + c);
	}
	if (threadIdx.x == 63)
		out[blockIdx.x] = acc;
}

// variants 120-125: diag_tile_rw with the record stores under other cache policies (round 5): 0 plain, 1 nt (as
// diag_tile_rw), 2 sc1, 3 sc0 sc1, 4 nt sc1, 5 nt sc0 sc1 -- what the read + write mix costs per store policy
template <int P>
__device__ __forceinline__ void store_policy(void* p, uint32_t a, uint32_t b, uint32_t c, uint32_t d)
{
	typedef uint32_t v4 __attribute__((ext_vector_type(4)));
	v4 x;
	x.x = a; x.y = b; x.z = c; x.w = d;
	if (P == 0)
		*reinterpret_cast<v4*>(p) = x;
	else if (P == 1)
		__builtin_nontemporal_store(x, reinterpret_cast<v4*>(p));
	else if (P == 2)
		asm volatile("global_store_dwordx4 %0, %1, off sc1" : : "v"(p), "v"(x) : "memory");
	else if (P == 3)
		asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" : : "v"(p), "v"(x) : "memory");
	else if (P == 4)
		asm volatile("global_store_dwordx4 %0, %1, off nt sc1" : : "v"(p), "v"(x) : "memory");
	else
		asm volatile("global_store_dwordx4 %0, %1, off nt sc0 sc1" : : "v"(p), "v"(x) : "memory");
}
template <int P>
__global__ __launch_bounds__(kTile) void diag_tile_rw_policy(const uint8_t* data, uint64_t len, uint32_t per_wave,
                                                              uint8_t* wout, uint32_t w_per_wave, uint32_t* out)
{
	const uint64_t base = (uint64_t)blockIdx.x * per_wave;
	uint32_t acc = 0;
	for (uint32_t c = threadIdx.x; 16ull * c < per_wave; c += 4 * kTile)
	{
		uint4 v[4];
#pragma unroll
		for (int k = 0; k < 4; ++k)
		{
			const uint64_t a = base + 16ull * (c + k * kTile);
			v[k] = a + 16 <= len ? ld16((uintptr_t)data + a) : make_uint4(0, 0, 0, 0);
		}
#pragma unroll
		for (int k = 0; k < 4; ++k)
			acc += halves(v[k].x) + halves(v[k].y) + halves(v[k].z) + halves(v[k].w);
	}
	acc = wave_incl_scan(acc);
	uint8_t* w = wout + (uint64_t)blockIdx.x * w_per_wave;
	for (uint32_t c = threadIdx.x; 16 * c < w_per_wave; c += kTile)
		store_policy<P>(w + 16 * c, acc + c, acc, c, blockIdx.x);
	if (threadIdx.x == 63)
		out[blockIdx.x] = acc;
}

__global__ __launch_bounds__(kBlock) void diag_grid_read(const uint8_t* data, uint64_t len, uint32_t* out)
{
	const uint64_t nch = len / 16;
	uint32_t acc = 0;
	const uint64_t stride = (uint64_t)gridDim.x * kBlock;
	for (uint64_t c = (uint64_t)blockIdx.x * kBlock + threadIdx.x; c < nch; c += 4 * stride)
	{
		uint4 v[4];
#pragma unroll
		for (int k = 0; k < 4; ++k)
			v[k] = c + k * stride < nch ? ld16((uintptr_t)data + 16 * (c + k * stride)) : make_uint4(0, 0, 0, 0);
#pragma unroll
		for (int k = 0; k < 4; ++k)
			acc += halves(v[k].x) + halves(v[k].y) + halves(v[k].z) + halves(v[k].w);
	}
	out[blockIdx.x * kBlock + threadIdx.x] = acc;
}

}  // namespace
}  // namespace pcppx

using namespace pcppx;

/* variant: 1 lane kernel; 2 stream-only diagnostic (no header gather / parse; L4 range = [14, caplen));
 * 3 / 4 tile-shaped / grid-stride read of the batch bytes (results written over summary[]); 7 tile-shaped read + the
 * parse's record stores; 29 gather-only diagnostic; 30 / 31 the checksum / parse-only instance marking fast-path
 * packets (flags bit 0x8000); 44 / 52 skip-generic diagnostics; 70 the DEEP checksum instance with the early second
 * stream window; 80 / 81 / 82 parse-only windows of 144 / 128 / 160 B gathered in one round; 83 a 96 + 32-B two-round
 * parse-only window; anything else: the product kernel. Records equal the product's for 1, 70, 80-83 (30 / 31 up to
 * the mark).
 * The shape variants measured in rounds 1-3 are in git history (profiles/r0*_ab_*.txt hold their results). */
PCPPX_AB_API int pcppx_ab_parse_device(const pcppx_batch* b, const pcppx_opts* o, pcppx_records* r, void* hip_stream,
                                       int variant)
{
	if (b == nullptr || o == nullptr || r == nullptr || o->max_layers > PCPPX_MAX_LAYERS)
		return PCPPX_E_INVAL;
	if (b->n == 0)
		return PCPPX_OK;
	hipStream_t stream = static_cast<hipStream_t>(hip_stream);
	const Params prm = make_params(b, o, r, nullptr);
	const dim3 grid((b->n + kTile - 1) / kTile);
	switch (variant)
	{
	case 1:
		hipLaunchKernelGGL(parse_lane_kernel, dim3((b->n + kBlock - 1) / kBlock), dim3(kBlock), 0, stream, prm);
		break;
	case 3:
	case 4:
	{
		uint32_t* out = reinterpret_cast<uint32_t*>(r->summary);  // n * 32 bytes is ample
		if (variant == 3)
		{
			const uint32_t per_wave = 21 * 1024;
			const uint32_t blocks = (uint32_t)((b->data_len + per_wave - 1) / per_wave);
			hipLaunchKernelGGL(diag_tile_read, dim3(blocks), dim3(kTile), 0, stream, b->data, b->data_len, per_wave, out);
		}
		else
			hipLaunchKernelGGL(diag_grid_read, dim3(256 * 8), dim3(kBlock), 0, stream, b->data, b->data_len, out);
		break;
	}
	case 7:
	{
		// writes over the layer-record buffer (n * max_layers * 8 B must hold 0.2 x the batch bytes)
		const uint32_t per_wave = 21 * 1024, w_per_wave = 4192;  // 64 packets x 65.5 B
		const uint32_t blocks = (uint32_t)((b->data_len + per_wave - 1) / per_wave);
		if ((uint64_t)blocks * w_per_wave > (uint64_t)b->n * o->max_layers * 8)
			return PCPPX_E_INVAL;
		hipLaunchKernelGGL(diag_tile_rw, dim3(blocks), dim3(kTile), 0, stream, b->data, b->data_len, per_wave,
		                   reinterpret_cast<uint8_t*>(r->layers), w_per_wave, reinterpret_cast<uint32_t*>(r->summary));
		break;
	}
	case 120:
	case 121:
	case 122:
	case 123:
	case 124:
	case 125:
	{
		// diag_tile_rw under six store policies (same read + write bytes as variant 7)
		const uint32_t per_wave = 21 * 1024, w_per_wave = 4192;
		const uint32_t blocks = (uint32_t)((b->data_len + per_wave - 1) / per_wave);
		if ((uint64_t)blocks * w_per_wave > (uint64_t)b->n * o->max_layers * 8)
			return PCPPX_E_INVAL;
		uint8_t* wo = reinterpret_cast<uint8_t*>(r->layers);
		uint32_t* so = reinterpret_cast<uint32_t*>(r->summary);
		const dim3 g(blocks), t(kTile);
		if (variant == 120) hipLaunchKernelGGL(diag_tile_rw_policy<0>, g, t, 0, stream, b->data, b->data_len, per_wave, wo, w_per_wave, so);
		if (variant == 121) hipLaunchKernelGGL(diag_tile_rw_policy<1>, g, t, 0, stream, b->data, b->data_len, per_wave, wo, w_per_wave, so);
		if (variant == 122) hipLaunchKernelGGL(diag_tile_rw_policy<2>, g, t, 0, stream, b->data, b->data_len, per_wave, wo, w_per_wave, so);
		if (variant == 123) hipLaunchKernelGGL(diag_tile_rw_policy<3>, g, t, 0, stream, b->data, b->data_len, per_wave, wo, w_per_wave, so);
		if (variant == 124) hipLaunchKernelGGL(diag_tile_rw_policy<4>, g, t, 0, stream, b->data, b->data_len, per_wave, wo, w_per_wave, so);
		if (variant == 125) hipLaunchKernelGGL(diag_tile_rw_policy<5>, g, t, 0, stream, b->data, b->data_len, per_wave, wo, w_per_wave, so);
		break;
	}
	// diagnostics over the product shapes (ParseShape<NT, FillTails, TightR2, Realign, EarlyB, StreamOnly, MarkFast,
	// GatherOnly, SkipGeneric>): stream only, gather only, fast-path marks, skip the generic walk
	case 2: hipLaunchKernelGGL((parse_tile_kernel<5, 128, 6, true, 6, ParseShape<true, true, true, true, true, true>>), grid, dim3(kTile), 0, stream, prm); break;
	case 29: hipLaunchKernelGGL((parse_tile_kernel<1, 64, 9, false, 6, ParseShape<true, true, true, true, true, false, false, true>>), grid, dim3(kTile), 0, stream, prm); break;
	case 30: hipLaunchKernelGGL((parse_tile_kernel<5, 128, 6, true, 6, ParseShape<true, true, true, true, true, false, true>>), grid, dim3(kTile), 0, stream, prm); break;
	case 31: hipLaunchKernelGGL((parse_tile_kernel<1, 64, 9, false, 6, ParseShape<true, true, true, true, true, false, true>>), grid, dim3(kTile), 0, stream, prm); break;
	// the PCPPX_WINDOW_DEEP checksum instance with the early second stream window (the product's runs it late)
	case 70: hipLaunchKernelGGL((parse_tile_kernel<4, 128, 9, true, 6>), grid, dim3(kTile), 0, stream, prm); break;
	// parse-only windows gathered in ONE round for every packet (no dependent second round): 144 B, 128 B, 160 B
	case 80: hipLaunchKernelGGL((parse_tile_kernel<1, 64, 9, false, 9>), grid, dim3(kTile), 0, stream, prm); break;
	case 81: hipLaunchKernelGGL((parse_tile_kernel<1, 64, 8, false, 8>), grid, dim3(kTile), 0, stream, prm); break;
	case 82: hipLaunchKernelGGL((parse_tile_kernel<1, 64, 10, false, 10>), grid, dim3(kTile), 0, stream, prm); break;
	// two rounds 128 B (96 + 32)
	case 83: hipLaunchKernelGGL((parse_tile_kernel<1, 64, 8, false, 6>), grid, dim3(kTile), 0, stream, prm); break;
	// round 6: the 144-B parse-only window with a larger first round (128 / 112 B), the rest only for the stacks that
	// end past it -- fewer waves with a dependent second round on deep traffic (config 5)
	case 240: hipLaunchKernelGGL((parse_tile_kernel<1, 64, 9, false, 8>), grid, dim3(kTile), 0, stream, prm); break;
	// round 6: the SHORT parse-only instance held to 6 waves per SIMD (<= 80 VGPRs; its 7 KiB of LDS allow 22 waves per CU)
	case 260: hipLaunchKernelGGL((parse_tile_kernel<6, 64, 6, false, 6>), grid, dim3(kTile), 0, stream, prm); break;
	case 241: hipLaunchKernelGGL((parse_tile_kernel<1, 64, 9, false, 7>), grid, dim3(kTile), 0, stream, prm); break;
	// round 6: the write-volume sensitivity -- the product instances storing only the first half of each PACKED run
	// (records wrong past it): 270 the checksum instance, 271 the two-round parse-only instance
	case 270: hipLaunchKernelGGL((parse_tile_kernel<5, 128, 6, true, 6, ParseShape<true, true, true, true, true, false, false, false, false, 64>>), grid, dim3(kTile), 0, stream, prm); break;
	case 271: hipLaunchKernelGGL((parse_tile_kernel<1, 64, 9, false, 8, ParseShape<true, true, true, true, true, false, false, false, false, 64>>), grid, dim3(kTile), 0, stream, prm); break;
	// round 6: the instances under combinations of the ParseShape R6 switches (bit 0 DPP span reductions, bit 1
	// wave-wide hashes, bit 2 L7 register tables, bit 3 IPv4-wave hash skip): 200 + R6 for R6 = 0, 1, 2 (the rejected
	// bits alone), 209: R6 = 12 (bits 2 + 3), 450: R6 = 28 (the product; other combinations measured in r06a-c are in git
	// history)
	// the checksum instance (450: R6 = 28), 210 + the two-round parse-only instance, 220 + the SHORT parse-only instance, 230 + the DEEP
	// checksum instance (its ParseShape with EarlyB, tools/ab variant 70's)
#define PCPPX_AB_SHAPE(r) ParseShape<true, true, true, true, true, false, false, false, false, 0, r>
#define PCPPX_AB_R6(base, W, SW, C, CS, C1)                                                                                \
	case base + 0: hipLaunchKernelGGL((parse_tile_kernel<W, SW, C, CS, C1, PCPPX_AB_SHAPE(0)>), grid, dim3(kTile), 0, stream, prm); break; \
	case base + 1: hipLaunchKernelGGL((parse_tile_kernel<W, SW, C, CS, C1, PCPPX_AB_SHAPE(1)>), grid, dim3(kTile), 0, stream, prm); break; \
	case base + 2: hipLaunchKernelGGL((parse_tile_kernel<W, SW, C, CS, C1, PCPPX_AB_SHAPE(2)>), grid, dim3(kTile), 0, stream, prm); break; \
	case base + 9: hipLaunchKernelGGL((parse_tile_kernel<W, SW, C, CS, C1, PCPPX_AB_SHAPE(12)>), grid, dim3(kTile), 0, stream, prm); break; \
	case base + 250: hipLaunchKernelGGL((parse_tile_kernel<W, SW, C, CS, C1, PCPPX_AB_SHAPE(28)>), grid, dim3(kTile), 0, stream, prm); break;
	PCPPX_AB_R6(200, 5, 128, 6, true, 6)
	PCPPX_AB_R6(210, 1, 64, 9, false, 6)
	PCPPX_AB_R6(220, 1, 64, 6, false, 6)
	PCPPX_AB_R6(230, 4, 128, 9, true, 6)
#undef PCPPX_AB_SHAPE
#undef PCPPX_AB_R6
	case 0: return launch_parse(b, o, r, stream);
	default: return PCPPX_E_INVAL;  // a variant this build does not hold (older ones: git history)
	}
	return check_launch("pcppx_ab_parse_device", stream);
}

/* The partitioned flow table over a dense key column with count-kernel shape `shape` (0: the product's
 * 1024 threads / 8192 LDS slots / 4096-packet batches / 256 blocks; 1: 512 / 4096 / 2048 / 768; 2: 256 / 2048 / 1024 /
 * 1536; 3: 1024 / 8192 / 6144 / 512; 12: the round-3 product, 4096-packet batches and a one-round-ahead merge), then the
 * product's merge (shapes 4-11: merge variants; 9: one round ahead). queues / fill: scratch as pcppx_capi.cpp sizes it. */
PCPPX_AB_API int pcppx_ab_flow_part(const uint32_t* dkeys, const uint32_t* caplens, uint32_t n, uint32_t* keys,
                                    uint64_t* packets, uint64_t* bytes, uint32_t capacity, uint64_t* stats, void* queues,
                                    uint32_t rec_cap, uint32_t* fill, void* hip_stream, int shape)
{
	hipStream_t stream = static_cast<hipStream_t>(hip_stream);
	auto* pk = reinterpret_cast<unsigned long long*>(packets);
	auto* by = reinterpret_cast<unsigned long long*>(bytes);
	auto* st = reinterpret_cast<unsigned long long*>(stats);
	// shapes 4-7: the product count kernel with 512 / 1024 partitions (regions) and smaller merge blocks
	const uint32_t want = shape == 6 ? 8u : (shape == 7 ? 10u : 9u);  // partitions (log2): tools/ab_flow_part.py PARTS
	const uint32_t l = log2u(capacity), lp = l < want ? l : want;
	const FlowPart fp{ static_cast<uint4*>(queues), rec_cap, fill, lp, l - lp };
	auto go = [&](auto kern, uint32_t threads, uint32_t batch, uint32_t blocks) {
		const uint32_t batches = (n + batch - 1) / batch;
		hipLaunchKernelGGL(kern, dim3(batches < blocks ? batches : blocks), dim3(threads), 0, stream, nullptr, caplens, n,
		                   keys, pk, by, capacity, st, nullptr, fp, dkeys);
	};
	if (shape == 20)  // no partitions: each batch's distinct keys go straight to the table (packed 64-bit atomics into
	{                 // `queues` taken as a zeroed u64[capacity] accumulator), then one unpack pass over the table
		const uint32_t batches = (n + kFlowBatchPk - 1) / kFlowBatchPk;
		auto* acc = static_cast<unsigned long long*>(queues);
		hipLaunchKernelGGL((flow_count_kernel<1024, 8192, kFlowBatchPk, kFlowHot, true, false, true>),
		                   dim3(batches < kFlowBlocks ? batches : kFlowBlocks), dim3(1024), 0, stream, nullptr, caplens, n, keys,
		                   pk, by, capacity, st, acc, FlowPart{}, dkeys);
		int rc = check_launch("pcppx_ab_flow_part(unpartitioned)", stream);
		if (rc != PCPPX_OK)
			return rc;
		const uint32_t ub = (capacity + kBlock - 1) / kBlock;
		hipLaunchKernelGGL(flow_unpack_kernel, dim3(ub < 2048 ? ub : 2048), dim3(kBlock), 0, stream, pk, by, acc, capacity);
		return check_launch("flow_unpack_kernel", stream);
	}
	switch (shape)
	{
	case 1: go(flow_count_kernel<512, 4096, 2048, kFlowHot, true, true, true>, 512, 2048, 768); break;
	case 2: go(flow_count_kernel<256, 2048, 1024, kFlowHot, true, true, true>, 256, 1024, 1536); break;
	case 3: go(PCPPX_FLOW_PART_DENSE_KERNEL, 1024, kFlowBatchPk, 512); break;
	case 12: go(flow_count_kernel<1024, 8192, 4096, kFlowHot, true, true, true>, 1024, 4096, 256); break;  // r03 batch
	case 13: go(flow_count_kernel<1024, 8192, kFlowBatchPk, kFlowHot, true, true, true, false>, 1024, kFlowBatchPk, 256); break;  // two-pass flush (r04 before r04r)
	case 14: go(flow_count_kernel<1024, 8192, kFlowBatchPk, 4, true, true, true, true>, 1024, kFlowBatchPk, 256); break;  // + hot above 4
	case 15: go(flow_count_kernel<1024, 8192, kFlowBatchPk, 1, true, true, true, true>, 1024, kFlowBatchPk, 256); break;  // + hot above 1
	default: go(PCPPX_FLOW_PART_DENSE_KERNEL, 1024, kFlowBatchPk, 256); break;
	}
	int rc = check_launch("pcppx_ab_flow_part", stream);
	if (rc != PCPPX_OK)
		return rc;
	if (shape == 4)
		hipLaunchKernelGGL((flow_merge_kernel<1024, 4096, 1>), dim3(1u << lp), dim3(1024), 0, stream, fp, keys, pk, by, st);
	else if (shape >= 5 && shape <= 7)
		hipLaunchKernelGGL((flow_merge_kernel<512, 4096, 2>), dim3(1u << lp), dim3(512), 0, stream, fp, keys, pk, by, st);
	else if (shape == 8)  // merge lookahead: 2 / 3 rounds of queue records in flight
		hipLaunchKernelGGL((flow_merge_kernel<512, 4096, 2, 2>), dim3(1u << lp), dim3(512), 0, stream, fp, keys, pk, by, st);
	else if (shape == 9 || shape == 12)  // 12: the r03 product merge (one round ahead)
		hipLaunchKernelGGL((flow_merge_kernel<512, 4096, 2, 1>), dim3(1u << lp), dim3(512), 0, stream, fp, keys, pk, by, st);
	else if (shape == 17)  // deeper merge lookahead: 4 / 6 rounds of queue records in flight
		hipLaunchKernelGGL((flow_merge_kernel<512, 4096, 2, 4>), dim3(1u << lp), dim3(512), 0, stream, fp, keys, pk, by, st);
	else if (shape == 18)
		hipLaunchKernelGGL((flow_merge_kernel<512, 4096, 2, 6>), dim3(1u << lp), dim3(512), 0, stream, fp, keys, pk, by, st);
	else if (shape == 19)  // 1 record per thread, 6 rounds ahead
		hipLaunchKernelGGL((flow_merge_kernel<512, 4096, 1, 6>), dim3(1u << lp), dim3(512), 0, stream, fp, keys, pk, by, st);
	else if (shape == 10)  // 256 threads x 4 records per round, 2 rounds ahead
		hipLaunchKernelGGL((flow_merge_kernel<256, 4096, 4, 2>), dim3(1u << lp), dim3(256), 0, stream, fp, keys, pk, by, st);
	else if (shape == 11)  // 512 threads x 4 records, 8192-slot LDS table
		hipLaunchKernelGGL((flow_merge_kernel<512, 8192, 4, 2>), dim3(1u << lp), dim3(512), 0, stream, fp, keys, pk, by, st);
	else
		hipLaunchKernelGGL(PCPPX_FLOW_MERGE_KERNEL, dim3(1u << lp), dim3(kFlowMergeThreads), 0, stream, fp, keys, pk, by, st);
	return check_launch("flow_merge_kernel", stream);
}

/* Flow-table shapes 0-12 of profiles/r01_ab_flow_shape.txt (9 = the product's); grid 0 = the shape's default
 * persistent grid. packed: zeroed u64[capacity] scratch (the product's packed accumulator) or NULL. */
PCPPX_AB_API int pcppx_ab_flow_count_device(const pcppx_summary* sum, const uint32_t* caplens, uint32_t n,
                                            uint32_t* keys, uint64_t* packets, uint64_t* bytes, uint32_t capacity,
                                            uint64_t* stats, uint64_t* packed, void* hip_stream, int shape,
                                            uint32_t grid)
{
	if (sum == nullptr || caplens == nullptr || keys == nullptr || capacity == 0 || (capacity & (capacity - 1)) != 0 ||
	    n > kPackedMax)
		return PCPPX_E_INVAL;
	if (n == 0)
		return PCPPX_OK;
	hipStream_t stream = static_cast<hipStream_t>(hip_stream);
	auto* pk = reinterpret_cast<unsigned long long*>(packets);
	auto* by = reinterpret_cast<unsigned long long*>(bytes);
	auto* pc = reinterpret_cast<unsigned long long*>(packed);
	auto* st = reinterpret_cast<unsigned long long*>(stats);
	auto go = [&](auto kern, uint32_t threads, uint32_t batch, uint32_t def_grid) {
		const uint32_t batches = (n + batch - 1) / batch;
		const uint32_t cap = grid ? grid : def_grid;
		hipLaunchKernelGGL(kern, dim3(batches < cap ? batches : cap), dim3(threads), 0, stream, sum, caplens, n, keys, pk,
		                   by, capacity, st, pc, FlowPart{}, nullptr);
	};
	switch (shape)
	{
	case 0: go(flow_count_kernel<256, 2048, 1024>, 256, 1024, 512); break;  // 512 persistent blocks (r01_ab_flow_grid.txt)
	case 1: go(flow_count_kernel<512, 4096, 2048>, 512, 2048, 512); break;
	case 2: go(flow_count_kernel<1024, 8192, 4096>, 1024, 4096, 256); break;
	case 3: go(flow_count_kernel<256, 4096, 2048>, 256, 2048, 512); break;
	case 4: go(flow_count_kernel<512, 8192, 4096>, 512, 4096, 256); break;
	case 5: go(flow_count_kernel<1024, 8192, 2048>, 1024, 2048, 256); break;
	case 6: go(flow_count_kernel<1024, 8192, 4096, 1>, 1024, 4096, 256); break;
	case 7: go(flow_count_kernel<1024, 8192, 4096, 4>, 1024, 4096, 256); break;
	case 8: go(flow_count_kernel<1024, 8192, 4096, 8>, 1024, 4096, 256); break;
	case 10: go(flow_count_kernel<512, 4096, 2048, kFlowHot, true>, 512, 2048, 512); break;
	case 11: go(flow_count_kernel<1024, 4096, 2048, kFlowHot, true>, 1024, 2048, 512); break;
	case 12: go(flow_count_kernel<1024, 8192, 6144, kFlowHot, true>, 1024, 6144, 256); break;
	default: go(PCPPX_FLOW_KERNEL, kFlowThreads, 4096, kFlowBlocks); break;
	}
	int rc = check_launch("pcppx_ab_flow_count_device", stream);
	if (rc != PCPPX_OK || pc == nullptr)
		return rc;
	const uint32_t ub = (capacity + kBlock - 1) / kBlock;
	hipLaunchKernelGGL(flow_unpack_kernel, dim3(ub < 2048 ? ub : 2048), dim3(kBlock), 0, stream, pk, by, pc, capacity);
	return check_launch("flow_unpack_kernel", stream);
}
