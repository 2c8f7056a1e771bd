// snp.hip -- all-pairs SNP distances on gfx950 (the `ccphylo dist` hot loop).
//
// Reference: fsacmp.c:552 fsacmp (count of included positions where the
// 2-bit codes differ), fsacmp.c:587 fsacmpair (same over inc_i & inc_j, plus
// the number of compared positions), driven by fsacmpthrd.c:108 cmpFsaThrd /
// :261 cmpairFsaThrd which store nFactor*dist (resp. the A7 epilogue) into
// LT cell (i, j).
//
// Data layout in HBM ("bit planes"): for taxon t and 32-position word w,
//   hi[t][w] = high code bits, lo[t][w] = low code bits, MSB = first position
// (the include-mask bit order of fsacmp.c:200).  Non-pair mode pre-applies
// the global include mask to both planes, so a pair's count is
//   sum_w popc((hi_a ^ hi_b) | (lo_a ^ lo_b))        -- 3 VALU ops / 32 nt
// (v_xor, v_bitop3, v_bcnt with accumulate).
// Pair mode keeps each taxon's mask m beside its planes:
//   d += popc(((hi_a ^ hi_b) | (lo_a ^ lo_b)) & m_a & m_b), n += popc(m_a & m_b).
// Two kernel families compute it:
//   - the default, k_snp_mfma3 (non-pair) / k_snp_mfma2_pair: the count as an
//     exact MX-fp4 dot product on the matrix cores (each code a +-1
//     tetrahedron vector, dist = (3 L - dot) / 4), 256x256 pair tiles,
//     MFMA-bound; k_snp_mfma3 stages its chunks by LDS-DMA and interleaves
//     the plane-to-fp4 spreads with the MFMAs, k_snp_mfma2 (CCG_DIST_GLDS=0)
//     is the register-staged form it replaced;
//   - k_snp_tile / k_snp_tile_pair (CCG_DIST_MFMA=0): the popcount form
//     above, VALU-integer-bound, 128x128 pair tiles, 8x8 pairs per thread in
//     registers.
// Both stage KC-word chunks of the two row panels through LDS.
#include <cstring>
#include <vector>
#include <type_traits>
#include "ccg_internal.h"
#include "ccg_shard_layout.h"

#define TILE 128
#define KC 16          // words per LDS chunk (non-pair)
#define KCP 8          // words per LDS chunk (pair)
#define RS 130         // LDS row stride in 8-byte units: 16-byte aligned, 2-way write conflicts at most
#define RSP 130        // pair: stride in 16-byte units

// (a ^ b) | c in one v_bitop3_b32 (truth table 0xBE, checked on gfx950 by
// tools/micro/bitop3_check.hip): a word pair costs xor + bitop3 + bcnt
__device__ __forceinline__ uint32_t xor_or(uint32_t a, uint32_t b, uint32_t c) {
	return __builtin_amdgcn_bitop3_b32(a, b, c, 0xBE);
}

__device__ __forceinline__ uint32_t compress_even(uint64_t x) {
	x &= 0x5555555555555555ull;
	x = (x | (x >> 1)) & 0x3333333333333333ull;
	x = (x | (x >> 2)) & 0x0F0F0F0F0F0F0F0Full;
	x = (x | (x >> 4)) & 0x00FF00FF00FF00FFull;
	x = (x | (x >> 8)) & 0x0000FFFF0000FFFFull;
	x = (x | (x >> 16)) & 0x00000000FFFFFFFFull;
	return (uint32_t) x;
}

// qseq2nibble word (position p at bits 63-2p..62-2p) -> (hi, lo) planes.
// Non-pair mode may compact the words: plane word w holds alignment word
// widx[w] (the words the global mask does not exclude entirely, in order), so
// W32 is then their count; widx = NULL keeps every word.
__global__ void k_planes(const uint64_t *__restrict__ seqs, const uint32_t *__restrict__ incs, int n, int stride,
                         int W32, int Wp, int pair, uint2 *__restrict__ out2, uint4 *__restrict__ out4,
                         const int *__restrict__ widx) {
	// grid-stride: n * Wp exceeds 2^32 work-items at config sizes (50k x 5M)
	const long long total = (long long) n * Wp;
	for(long long e = (long long) blockIdx.x * blockDim.x + threadIdx.x; e < total;
	    e += (long long) gridDim.x * blockDim.x) {
		const int t = (int) (e / Wp), w = (int) (e % Wp);
		uint32_t hi = 0, lo = 0, m = 0;
		if(w < W32) {
			const int ws = widx ? widx[w] : w;
			uint64_t x = seqs[(size_t) t * stride + ws];
			hi = compress_even(x >> 1);
			lo = compress_even(x);
			m = pair ? incs[(size_t) t * stride + ws] : incs[ws];
		}
		if(pair) {
			out4[e] = make_uint4(hi, lo, m, 0);
		} else {
			out2[e] = make_uint2(hi & m, lo & m);
		}
	}
}

__global__ void k_popsum(const uint32_t *__restrict__ inc, int W32, int *out) {
	int s = 0;
	for(int w = threadIdx.x; w < W32; w += blockDim.x) s += __popc(inc[w]);
	for(int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
	__shared__ int ws[16];
	if((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = s;
	__syncthreads();
	if(threadIdx.x == 0) {
		int t = 0;
		for(int k = 0; k < (int) (blockDim.x >> 6); ++k) t += ws[k];
		*out = t;
	}
}

// linear tile index -> (I, J), I >= J, row-major over the lower triangle
__device__ __forceinline__ void tile_ij(long long t, int &I, int &J) {
	long long r = (long long) ((sqrt(8.0 * (double) t + 1.0) - 1.0) * 0.5);
	while(r * (r + 1) / 2 > t) --r;
	while((r + 1) * (r + 2) / 2 <= t) ++r;
	I = (int) r;
	J = (int) (t - r * (r + 1) / 2);
}

// XCD-aware tile order: workgroups are dispatched round-robin over the 8
// XCDs, so give XCD x a contiguous run of row-major tiles (tiles (I, J),
// (I, J+1), ... share the I panel in that XCD's L2).  Bijective on [0, cnt).
__device__ __forceinline__ long long xcd_tile(long long b, long long cnt) {
	const long long x = b & 7, k = b >> 3, q = cnt >> 3, r = cnt & 7;
	return x < r ? x * (q + 1) + k : r * (q + 1) + (x - r) * q + k;
}

// Non-pair tiles: double-buffered KC-word chunks of both 128-row panels; the
// next chunk's global loads are in flight while the current one is consumed
// from LDS, one barrier per chunk.  Work item = (tile, word slice): with
// S > 1 slices (split-K, so small tile counts still fill the chip) the
// partial counts are summed exactly with u32 atomics into `cnt` and
// k_snp_finish writes D.
template <int ET, bool SPLIT>
__global__ __launch_bounds__(256, 2) void k_snp_tile(const uint2 *__restrict__ P, int Wp, int n, long long t0,
                                                     long long items, int S, int Wk, double nFactor, double bs,
                                                     typename Elem<ET>::T *__restrict__ D, long long rowBegin,
                                                     long long rowEnd, unsigned *__restrict__ cnt, long long cbase) {
	__shared__ __attribute__((aligned(16))) uint2 As[2][KC * RS];
	__shared__ __attribute__((aligned(16))) uint2 Bs[2][KC * RS];
	int I, J;
	const long long item = t0 + xcd_tile(blockIdx.x, items);
	tile_ij(item / S, I, J);
	const int wb = (int) (item % S) * Wk, we = wb + Wk < Wp ? wb + Wk : Wp;
	const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
	const uint2 *Ap = P + (size_t) I * TILE * Wp + wb;
	const uint2 *Bp = P + (size_t) J * TILE * Wp + wb;
	const int Wl = we - wb;   // words of this slice (a multiple of KC)
	uint32_t acc[8][8];
#pragma unroll
	for(int a = 0; a < 8; ++a)
#pragma unroll
		for(int c = 0; c < 8; ++c) acc[a][c] = 0;
	// this thread's staging slots: rows e>>3, word pairs 2*(e&7), e = q*256 + tid
	uint4 va[4], vb[4];
#pragma unroll
	for(int q = 0; q < 4; ++q) {
		const int e = q * 256 + threadIdx.x, row = e >> 3, wp = e & 7;
		va[q] = *(const uint4 *) (Ap + (size_t) row * Wp + 2 * wp);
		vb[q] = *(const uint4 *) (Bp + (size_t) row * Wp + 2 * wp);
	}
#pragma unroll
	for(int q = 0; q < 4; ++q) {
		const int e = q * 256 + threadIdx.x, row = e >> 3, wp = e & 7;
		As[0][(2 * wp) * RS + row] = make_uint2(va[q].x, va[q].y);
		As[0][(2 * wp + 1) * RS + row] = make_uint2(va[q].z, va[q].w);
		Bs[0][(2 * wp) * RS + row] = make_uint2(vb[q].x, vb[q].y);
		Bs[0][(2 * wp + 1) * RS + row] = make_uint2(vb[q].z, vb[q].w);
	}
	__syncthreads();
	int buf = 0;
	for(int w0 = 0; w0 < Wl; w0 += KC, buf ^= 1) {
		const bool more = w0 + KC < Wl;
		if(more) {
#pragma unroll
			for(int q = 0; q < 4; ++q) {
				const int e = q * 256 + threadIdx.x, row = e >> 3, wp = e & 7;
				va[q] = *(const uint4 *) (Ap + (size_t) row * Wp + w0 + KC + 2 * wp);
				vb[q] = *(const uint4 *) (Bp + (size_t) row * Wp + w0 + KC + 2 * wp);
			}
		}
		const uint2 *Ac = As[buf], *Bc = Bs[buf];
#pragma unroll 1
		for(int w = 0; w < KC; ++w) {
			uint4 a[4], b[4];
#pragma unroll
			for(int q = 0; q < 4; ++q) {
				a[q] = *(const uint4 *) &Ac[w * RS + 2 * ty + 32 * q];
				b[q] = *(const uint4 *) &Bc[w * RS + 2 * tx + 32 * q];
			}
#pragma unroll
			for(int qa = 0; qa < 4; ++qa) {
#pragma unroll
				for(int qb = 0; qb < 4; ++qb) {
					acc[2 * qa][2 * qb] += __popc(xor_or(a[qa].x, b[qb].x, a[qa].y ^ b[qb].y));
					acc[2 * qa][2 * qb + 1] += __popc(xor_or(a[qa].x, b[qb].z, a[qa].y ^ b[qb].w));
					acc[2 * qa + 1][2 * qb] += __popc(xor_or(a[qa].z, b[qb].x, a[qa].w ^ b[qb].y));
					acc[2 * qa + 1][2 * qb + 1] += __popc(xor_or(a[qa].z, b[qb].z, a[qa].w ^ b[qb].w));
				}
			}
		}
		if(more) {
			uint2 *An = As[buf ^ 1], *Bn = Bs[buf ^ 1];
#pragma unroll
			for(int q = 0; q < 4; ++q) {
				const int e = q * 256 + threadIdx.x, row = e >> 3, wp = e & 7;
				An[(2 * wp) * RS + row] = make_uint2(va[q].x, va[q].y);
				An[(2 * wp + 1) * RS + row] = make_uint2(va[q].z, va[q].w);
				Bn[(2 * wp) * RS + row] = make_uint2(vb[q].x, vb[q].y);
				Bn[(2 * wp + 1) * RS + row] = make_uint2(vb[q].z, vb[q].w);
			}
		}
		__syncthreads();
	}
	// epilogue: D[i][j] = nFactor * dist (fsacmpthrd.c:247-255), j < i only
#pragma unroll
	for(int a = 0; a < 8; ++a) {
		long long i = (long long) I * TILE + 2 * ty + 32 * (a >> 1) + (a & 1);
		if(i >= n || i < rowBegin || i >= rowEnd) continue;
		long long base = tri(i);
#pragma unroll
		for(int c = 0; c < 8; ++c) {
			long long j = (long long) J * TILE + 2 * tx + 32 * (c >> 1) + (c & 1);
			if(j < i) {
				if(SPLIT) {
					atomicAdd(&cnt[base + j - cbase], acc[a][c]);
				} else {
					double v = nFactor * (double) acc[a][c];
					D[base + j] = Elem<ET>::put(v, 0.5, bs);
				}
			}
		}
	}
}

// ------------------------------------------------------------------ MFMA tiles (non-pair)
// fsacmp's count as a dot product on the matrix cores, exactly.  A 2-bit code
// (hi, lo) becomes the tetrahedron vector (s_hi, s_lo, s_hi s_lo) of +-1
// (s = 1 - 2 bit): equal codes dot to 3, different ones to -1, so over the
// L positions of a word slice (padding and the pre-masked positions are code
// 0 in every row: "equal")  dist = (3 L - dot) / 4.  The three components are
// MX-fp4 operands of v_mfma_scale_f32_32x32x64_f8f6f4 (e2m1 +1 = 0x2,
// -1 = 0xA, unit scales); f32 accumulation of the +-1 products is exact while
// |dot| <= 3 L < 2^24 (the host splits K beyond that).  A lane's operand for
// one 32x32x64 step is one 32-position plane word expanded to 32 nibbles
// (tools/micro/mfma_fp4: row = lane & 31, and A's (lane, nibble) meets B's
// (lane, nibble), so any fixed spread of the word's bits over the nibbles
// works if both panels use it): dword q holds bits q, q+4, ..., q+28 at the
// nibbles' sign bits, (x << (3 - q)) & 0x88888888 | 0x22222222, 2 VALU ops.
// Block = 4 waves on a 128x128 pair tile, each wave 64x64 (2x2 MFMA tiles,
// 3 components x 2 words of 32 positions per step); raw words staged through
// LDS as in k_snp_tile (double-buffered KC-word chunks, XCD-contiguous tile
// order, split-K over word slices).
typedef int v8i_t __attribute__((ext_vector_type(8)));
typedef float v16f_t __attribute__((ext_vector_type(16)));
#define MFMA_FP4 4
#define MFMA_SCALE1 127
#define MFMA_KMAX 174762   // words per slice: 3 * 32 * Wk < 2^24
#ifndef MFMA_UNROLL
#define MFMA_UNROLL 2
#endif
// k_snp_mfma's LDS chunk (words) and blocks per CU: 8-word chunks keep a
// block's double-buffered panels at 33 KB, so 3 blocks fit a CU's LDS
#ifndef KCM
#define KCM 8
#endif
#ifndef MFMA_BLOCKS
#define MFMA_BLOCKS 3
#endif
#define QS (TILE * KCM / 2 / 256)   // uint4 staged per thread per panel

// (a & b) | c in one v_bitop3_b32 (truth table 0xEA in xor_or's convention)
__device__ __forceinline__ uint32_t and_or(uint32_t a, uint32_t b, uint32_t c) {
	return __builtin_amdgcn_bitop3_b32(a, b, c, 0xEA);
}

__device__ __forceinline__ v8i_t fp4_spread(uint32_t x) {
	v8i_t v;
	v[0] = (int) and_or(x << 3, 0x88888888u, 0x22222222u);
	v[1] = (int) and_or(x << 2, 0x88888888u, 0x22222222u);
	v[2] = (int) and_or(x << 1, 0x88888888u, 0x22222222u);
	v[3] = (int) and_or(x, 0x88888888u, 0x22222222u);
	v[4] = v[5] = v[6] = v[7] = 0;
	return v;
}

template <int ET, bool SPLIT>
__global__ __launch_bounds__(256, MFMA_BLOCKS) void k_snp_mfma(const uint2 *__restrict__ P, int Wp, int n, long long t0,
                                                     long long items, int S, int Wk, double nFactor, double bs,
                                                     typename Elem<ET>::T *__restrict__ D, long long rowBegin,
                                                     long long rowEnd, unsigned *__restrict__ cnt, long long cbase) {
	__shared__ __attribute__((aligned(16))) uint2 As[2][KCM * RS];
	__shared__ __attribute__((aligned(16))) uint2 Bs[2][KCM * RS];
	int I, J;
	const long long item = t0 + xcd_tile(blockIdx.x, items);
	tile_ij(item / S, I, J);
	const int wb = (int) (item % S) * Wk, we = wb + Wk < Wp ? wb + Wk : Wp;
	const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
	const int wr = wid >> 1, wc = wid & 1;   // this wave's 64x64 quarter
	const uint2 *Ap = P + (size_t) I * TILE * Wp + wb;
	const uint2 *Bp = P + (size_t) J * TILE * Wp + wb;
	const int Wl = we - wb;   // words of this slice (a multiple of KC)
	v16f_t acc[2][2];
#pragma unroll
	for(int a = 0; a < 2; ++a)
#pragma unroll
		for(int c = 0; c < 2; ++c)
#pragma unroll
			for(int r = 0; r < 16; ++r) acc[a][c][r] = 0.0f;
	uint4 va[QS], vb[QS];
#pragma unroll
	for(int q = 0; q < QS; ++q) {
		const int e = q * 256 + threadIdx.x, row = e / (KCM / 2), wp = e % (KCM / 2);
		va[q] = *(const uint4 *) (Ap + (size_t) row * Wp + 2 * wp);
		vb[q] = *(const uint4 *) (Bp + (size_t) row * Wp + 2 * wp);
	}
#pragma unroll
	for(int q = 0; q < QS; ++q) {
		const int e = q * 256 + threadIdx.x, row = e / (KCM / 2), wp = e % (KCM / 2);
		As[0][(2 * wp) * RS + row] = make_uint2(va[q].x, va[q].y);
		As[0][(2 * wp + 1) * RS + row] = make_uint2(va[q].z, va[q].w);
		Bs[0][(2 * wp) * RS + row] = make_uint2(vb[q].x, vb[q].y);
		Bs[0][(2 * wp + 1) * RS + row] = make_uint2(vb[q].z, vb[q].w);
	}
	__syncthreads();
	const int h = lane >> 5, l32 = lane & 31;
	const int ra0 = 64 * wr + l32, rb0 = 64 * wc + l32;
	int buf = 0;
	for(int w0 = 0; w0 < Wl; w0 += KCM, buf ^= 1) {
		const bool more = w0 + KCM < Wl;
		if(more) {
#pragma unroll
			for(int q = 0; q < QS; ++q) {
				const int e = q * 256 + threadIdx.x, row = e / (KCM / 2), wp = e % (KCM / 2);
				va[q] = *(const uint4 *) (Ap + (size_t) row * Wp + w0 + KCM + 2 * wp);
				vb[q] = *(const uint4 *) (Bp + (size_t) row * Wp + w0 + KCM + 2 * wp);
			}
		}
		const uint2 *Ac = As[buf], *Bc = Bs[buf];
#pragma unroll MFMA_UNROLL
		for(int s = 0; s < KCM / 2; ++s) {
			const int w = 2 * s + h;   // this lane's word: its half of the step's 64 positions
			uint2 a[2], b[2];
#pragma unroll
			for(int t = 0; t < 2; ++t) {
				a[t] = Ac[w * RS + ra0 + 32 * t];
				b[t] = Bc[w * RS + rb0 + 32 * t];
			}
#pragma unroll
			for(int comp = 0; comp < 3; ++comp) {
				v8i_t fa[2], fb[2];
#pragma unroll
				for(int t = 0; t < 2; ++t) {
					fa[t] = fp4_spread(comp == 0 ? a[t].x : comp == 1 ? a[t].y : a[t].x ^ a[t].y);
					fb[t] = fp4_spread(comp == 0 ? b[t].x : comp == 1 ? b[t].y : b[t].x ^ b[t].y);
				}
#pragma unroll
				for(int ta = 0; ta < 2; ++ta)
#pragma unroll
					for(int tb = 0; tb < 2; ++tb)
						acc[ta][tb] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(
						    fa[ta], fb[tb], acc[ta][tb], MFMA_FP4, MFMA_FP4, 0, MFMA_SCALE1, 0, MFMA_SCALE1);
			}
		}
		if(more) {
			uint2 *An = As[buf ^ 1], *Bn = Bs[buf ^ 1];
#pragma unroll
			for(int q = 0; q < QS; ++q) {
				const int e = q * 256 + threadIdx.x, row = e / (KCM / 2), wp = e % (KCM / 2);
				An[(2 * wp) * RS + row] = make_uint2(va[q].x, va[q].y);
				An[(2 * wp + 1) * RS + row] = make_uint2(va[q].z, va[q].w);
				Bn[(2 * wp) * RS + row] = make_uint2(vb[q].x, vb[q].y);
				Bn[(2 * wp + 1) * RS + row] = make_uint2(vb[q].z, vb[q].w);
			}
		}
		__syncthreads();
	}
	// epilogue: C/D of 32x32 (col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5));
	// dist = (3 L - dot) / 4 over the slice's L = 32 Wl positions
	const int L3 = 3 * 32 * Wl;
#pragma unroll
	for(int ta = 0; ta < 2; ++ta) {
#pragma unroll
		for(int r = 0; r < 16; ++r) {
			const long long i = (long long) I * TILE + 64 * wr + 32 * ta + (r & 3) + 8 * (r >> 2) + 4 * h;
			if(i >= n || i < rowBegin || i >= rowEnd) continue;
			const long long base = tri(i);
#pragma unroll
			for(int tb = 0; tb < 2; ++tb) {
				const long long j = (long long) J * TILE + 64 * wc + 32 * tb + l32;
				if(j < i) {
					const unsigned d = (unsigned) ((L3 - (int) acc[ta][tb][r]) >> 2);
					if(SPLIT) {
						atomicAdd(&cnt[base + j - cbase], d);
					} else {
						const double v = nFactor * (double) d;
						D[base + j] = Elem<ET>::put(v, 0.5, bs);
					}
				}
			}
		}
	}
}

// The same tiles for one rank of the row-sharded layout (ccg_shard.h): the A
// panel gathers the rank's owned rows, so a rank computes only its own rows
// and writes them where ccg_tree_shard_dev reads them.
template <int ET>
__global__ __launch_bounds__(256, 2) void k_snp_tile_band(const uint2 *__restrict__ P, int Wp, int n,
                                                          const long long *__restrict__ pfx, int npanels, long long t0,
                                                          long long items, double nFactor, double bs,
                                                          typename Elem<ET>::T *__restrict__ Dloc, int rank, int world) {
	__shared__ __attribute__((aligned(16))) uint2 As[2][KCM * RS];
	__shared__ __attribute__((aligned(16))) uint2 Bs[2][KCM * RS];
	// tile t of the rank's list: panel I = last with pfx[I] <= t, J = t - pfx[I]
	const long long t = t0 + xcd_tile(blockIdx.x, items);
	int lo = 0, hi = npanels - 1;
	while(lo < hi) {
		const int mid = (lo + hi + 1) >> 1;
		if(pfx[mid] <= t) lo = mid; else hi = mid - 1;
	}
	const int I = lo, J = (int) (t - pfx[lo]);
	const Shard sh{rank, world};
	const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
	// A panel: the rank's owned rows I*TILE .. I*TILE+127 in its own order
	// (band g = rows [SB g, SB g + SB) of rank g % world); rows past n read row 0
	const auto arow = [&](int l) -> long long {
		const long long L = (long long) I * TILE + l, lb = L / SB, g = lb * world + rank, r = g * SB + (L - lb * SB);
		return r < n ? r : 0;
	};
	const uint2 *Bp = P + (size_t) J * TILE * Wp;
	const int Wl = Wp;
	uint32_t acc[8][8];
#pragma unroll
	for(int a = 0; a < 8; ++a)
#pragma unroll
		for(int c = 0; c < 8; ++c) acc[a][c] = 0;
	// this thread's staging slots: rows e>>3, word pairs 2*(e&7), e = q*256 + tid
	uint4 va[QS], vb[QS];
#pragma unroll
	for(int q = 0; q < 4; ++q) {
		const int e = q * 256 + threadIdx.x, row = e >> 3, wp = e & 7;
		va[q] = *(const uint4 *) (P + (size_t) arow(row) * Wp + 2 * wp);
		vb[q] = *(const uint4 *) (Bp + (size_t) row * Wp + 2 * wp);
	}
#pragma unroll
	for(int q = 0; q < 4; ++q) {
		const int e = q * 256 + threadIdx.x, row = e >> 3, wp = e & 7;
		As[0][(2 * wp) * RS + row] = make_uint2(va[q].x, va[q].y);
		As[0][(2 * wp + 1) * RS + row] = make_uint2(va[q].z, va[q].w);
		Bs[0][(2 * wp) * RS + row] = make_uint2(vb[q].x, vb[q].y);
		Bs[0][(2 * wp + 1) * RS + row] = make_uint2(vb[q].z, vb[q].w);
	}
	__syncthreads();
	int buf = 0;
	for(int w0 = 0; w0 < Wl; w0 += KC, buf ^= 1) {
		const bool more = w0 + KC < Wl;
		if(more) {
#pragma unroll
			for(int q = 0; q < 4; ++q) {
				const int e = q * 256 + threadIdx.x, row = e >> 3, wp = e & 7;
				va[q] = *(const uint4 *) (P + (size_t) arow(row) * Wp + w0 + KC + 2 * wp);
				vb[q] = *(const uint4 *) (Bp + (size_t) row * Wp + w0 + KC + 2 * wp);
			}
		}
		const uint2 *Ac = As[buf], *Bc = Bs[buf];
#pragma unroll 1
		for(int w = 0; w < KC; ++w) {
			uint4 a[4], b[4];
#pragma unroll
			for(int q = 0; q < 4; ++q) {
				a[q] = *(const uint4 *) &Ac[w * RS + 2 * ty + 32 * q];
				b[q] = *(const uint4 *) &Bc[w * RS + 2 * tx + 32 * q];
			}
#pragma unroll
			for(int qa = 0; qa < 4; ++qa) {
#pragma unroll
				for(int qb = 0; qb < 4; ++qb) {
					acc[2 * qa][2 * qb] += __popc(xor_or(a[qa].x, b[qb].x, a[qa].y ^ b[qb].y));
					acc[2 * qa][2 * qb + 1] += __popc(xor_or(a[qa].x, b[qb].z, a[qa].y ^ b[qb].w));
					acc[2 * qa + 1][2 * qb] += __popc(xor_or(a[qa].z, b[qb].x, a[qa].w ^ b[qb].y));
					acc[2 * qa + 1][2 * qb + 1] += __popc(xor_or(a[qa].z, b[qb].z, a[qa].w ^ b[qb].w));
				}
			}
		}
		if(more) {
			uint2 *An = As[buf ^ 1], *Bn = Bs[buf ^ 1];
#pragma unroll
			for(int q = 0; q < QS; ++q) {
				const int e = q * 256 + threadIdx.x, row = e / (KCM / 2), wp = e % (KCM / 2);
				An[(2 * wp) * RS + row] = make_uint2(va[q].x, va[q].y);
				An[(2 * wp + 1) * RS + row] = make_uint2(va[q].z, va[q].w);
				Bn[(2 * wp) * RS + row] = make_uint2(vb[q].x, vb[q].y);
				Bn[(2 * wp + 1) * RS + row] = make_uint2(vb[q].z, vb[q].w);
			}
		}
		__syncthreads();
	}
	// epilogue: the rank's row i at Shard::off(i) (fsacmpthrd.c:247-255 values)
#pragma unroll
	for(int a = 0; a < 8; ++a) {
		const int l = 2 * ty + 32 * (a >> 1) + (a & 1);
		const long long L = (long long) I * TILE + l, lb = L / SB, i = (lb * world + rank) * SB + (L - lb * SB);
		if(i >= n) continue;
		const long long base = sh.off(i);
#pragma unroll
		for(int c = 0; c < 8; ++c) {
			long long j = (long long) J * TILE + 2 * tx + 32 * (c >> 1) + (c & 1);
			if(j < i) Dloc[base + j] = Elem<ET>::put(nFactor * (double) acc[a][c], 0.5, bs);
		}
	}
}

// k_snp_mfma for one rank of the row-sharded layout (as k_snp_tile_band):
// A panel = the rank's owned rows, rows stored at Shard::off(i).  SPLIT: word
// slice item % S of Wk (< MFMA_KMAX) words, u32 counts added by local element
// (k_snp_finish stores them), when the rank's tiles do not fill the chip or a
// row exceeds the f32-exact slice length.
template <int ET, bool SPLIT = false>
__global__ __launch_bounds__(256, 2) void k_snp_mfma_band(const uint2 *__restrict__ P, int Wp, int n,
                                                          const long long *__restrict__ pfx, int npanels, long long t0,
                                                          long long items, double nFactor, double bs,
                                                          typename Elem<ET>::T *__restrict__ Dloc, int rank, int world,
                                                          int S = 1, int Wk = 0, unsigned *__restrict__ cnt = nullptr) {
	__shared__ __attribute__((aligned(16))) uint2 As[2][KC * RS];
	__shared__ __attribute__((aligned(16))) uint2 Bs[2][KC * RS];
	const long long item = t0 + xcd_tile(blockIdx.x, items), t = SPLIT ? item / S : item;
	// SPLIT: word slice item % S of Wk words (counts added into cnt by local element)
	const int wb = SPLIT ? (int) (item % S) * Wk : 0;
	int lo = 0, hi = npanels - 1;
	while(lo < hi) {
		const int mid = (lo + hi + 1) >> 1;
		if(pfx[mid] <= t) lo = mid; else hi = mid - 1;
	}
	const int I = lo, J = (int) (t - pfx[lo]);
	const Shard sh{rank, world};
	const auto arow = [&](int l) -> long long {
		const long long L = (long long) I * TILE + l, lb = L / SB, g = lb * world + rank, r = g * SB + (L - lb * SB);
		return r < n ? r : 0;
	};
	const uint2 *Bp = P + (size_t) J * TILE * Wp + wb;
	const int Wl = SPLIT ? (wb + Wk < Wp ? Wk : Wp - wb) : Wp;
	const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
	const int wr = wid >> 1, wc = wid & 1;
	v16f_t acc[2][2];
#pragma unroll
	for(int a = 0; a < 2; ++a)
#pragma unroll
		for(int c = 0; c < 2; ++c)
#pragma unroll
			for(int r = 0; r < 16; ++r) acc[a][c][r] = 0.0f;
	uint4 va[4], vb[4];
	long long ar[4];
#pragma unroll
	for(int q = 0; q < 4; ++q) {
		const int e = q * 256 + threadIdx.x, row = e >> 3, wp = e & 7;
		ar[q] = arow(row);
		va[q] = *(const uint4 *) (P + (size_t) ar[q] * Wp + wb + 2 * wp);
		vb[q] = *(const uint4 *) (Bp + (size_t) row * Wp + 2 * wp);
	}
#pragma unroll
	for(int q = 0; q < 4; ++q) {
		const int e = q * 256 + threadIdx.x, row = e >> 3, wp = e & 7;
		As[0][(2 * wp) * RS + row] = make_uint2(va[q].x, va[q].y);
		As[0][(2 * wp + 1) * RS + row] = make_uint2(va[q].z, va[q].w);
		Bs[0][(2 * wp) * RS + row] = make_uint2(vb[q].x, vb[q].y);
		Bs[0][(2 * wp + 1) * RS + row] = make_uint2(vb[q].z, vb[q].w);
	}
	__syncthreads();
	const int h = lane >> 5, l32 = lane & 31;
	const int ra0 = 64 * wr + l32, rb0 = 64 * wc + l32;
	int buf = 0;
	for(int w0 = 0; w0 < Wl; w0 += KC, buf ^= 1) {
		const bool more = w0 + KC < Wl;
		if(more) {
#pragma unroll
			for(int q = 0; q < 4; ++q) {
				const int e = q * 256 + threadIdx.x, row = e >> 3, wp = e & 7;
				va[q] = *(const uint4 *) (P + (size_t) ar[q] * Wp + wb + w0 + KC + 2 * wp);
				vb[q] = *(const uint4 *) (Bp + (size_t) row * Wp + w0 + KC + 2 * wp);
			}
		}
		const uint2 *Ac = As[buf], *Bc = Bs[buf];
#pragma unroll 2
		for(int s = 0; s < KC / 2; ++s) {
			const int w = 2 * s + h;
			uint2 a[2], b[2];
#pragma unroll
			for(int tt = 0; tt < 2; ++tt) {
				a[tt] = Ac[w * RS + ra0 + 32 * tt];
				b[tt] = Bc[w * RS + rb0 + 32 * tt];
			}
#pragma unroll
			for(int comp = 0; comp < 3; ++comp) {
				v8i_t fa[2], fb[2];
#pragma unroll
				for(int tt = 0; tt < 2; ++tt) {
					fa[tt] = fp4_spread(comp == 0 ? a[tt].x : comp == 1 ? a[tt].y : a[tt].x ^ a[tt].y);
					fb[tt] = fp4_spread(comp == 0 ? b[tt].x : comp == 1 ? b[tt].y : b[tt].x ^ b[tt].y);
				}
#pragma unroll
				for(int ta = 0; ta < 2; ++ta)
#pragma unroll
					for(int tb = 0; tb < 2; ++tb)
						acc[ta][tb] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(
						    fa[ta], fb[tb], acc[ta][tb], MFMA_FP4, MFMA_FP4, 0, MFMA_SCALE1, 0, MFMA_SCALE1);
			}
		}
		if(more) {
			uint2 *An = As[buf ^ 1], *Bn = Bs[buf ^ 1];
#pragma unroll
			for(int q = 0; q < 4; ++q) {
				const int e = q * 256 + threadIdx.x, row = e >> 3, wp = e & 7;
				An[(2 * wp) * RS + row] = make_uint2(va[q].x, va[q].y);
				An[(2 * wp + 1) * RS + row] = make_uint2(va[q].z, va[q].w);
				Bn[(2 * wp) * RS + row] = make_uint2(vb[q].x, vb[q].y);
				Bn[(2 * wp + 1) * RS + row] = make_uint2(vb[q].z, vb[q].w);
			}
		}
		__syncthreads();
	}
	const int L3 = 3 * 32 * Wl;
#pragma unroll
	for(int ta = 0; ta < 2; ++ta) {
#pragma unroll
		for(int r = 0; r < 16; ++r) {
			const int l = 64 * wr + 32 * ta + (r & 3) + 8 * (r >> 2) + 4 * h;
			const long long L = (long long) I * TILE + l, lb = L / SB, i = (lb * world + rank) * SB + (L - lb * SB);
			if(i >= n) continue;
			const long long base = sh.off(i);
#pragma unroll
			for(int tb = 0; tb < 2; ++tb) {
				const long long j = (long long) J * TILE + 64 * wc + 32 * tb + l32;
				if(j < i) {
					const unsigned d = (unsigned) ((L3 - (int) acc[ta][tb][r]) >> 2);
					if(SPLIT) atomicAdd(&cnt[base + j], d);
					else Dloc[base + j] = Elem<ET>::put(nFactor * (double) d, 0.5, bs);
				}
			}
		}
	}
}

// ------------------------------------------------------------------ MFMA, 256 x 256 tiles
// k_snp_mfma2: the same exact MX-fp4 form on 256 x 256 pair tiles, one block of
// 4 waves per CU, each wave 128 x 128 (4 x 4 MFMA tiles, 256 accumulator
// VGPRs).  Per 64-position step a lane spreads its 4 A and 4 B plane words
// once per component and feeds 16 MFMAs with them (k_snp_mfma: 4 spreads per
// 4 MFMAs), and the third component (hi ^ lo) comes from the first two
// spreads in one v_bitop3 per dword ((a ^ b) | 0x22222222: the sign bits
// xor, the 0x2 exponent bits cancel and are set again), so the VALU work per
// MFMA drops about 3x and each staged panel byte feeds twice the position
// pairs (half the panel traffic into the CUs).  BAND: the A panel gathers
// one rank's owned rows of the band layout (k_snp_mfma_band), D indexed by
// Shard::off.  SPLIT: word slice item % S of Wk words, exact u32 counts.
#define TILE2 256
#define KC2 8                          // words per LDS chunk (the default; KC2L with CCG_DIST_KC=16)
#define KC2L 16
#define RS2 260                        // LDS row stride (uint2): 16-byte aligned rows of 256 + pad

// Super-tile order of the LT's 256 x 256 tiles (CCG_DIST_ORDER=1): super-rows
// of 4 panel rows; inside one, column chunks of 8 panels (4 x 8 = 32 tiles,
// one XCD's 32 CUs at a time under xcd_tile), row-major inside a chunk, then
// the diagonal remainder J in [8F, I] row-major.  A super-row starts at the
// same tile index as in row-major order (T(P) = 4P (4P + 1) / 2), so the
// row-major row of t names its super-row; a super-row cut by the last panel
// row Ihi (the end of the range) stays row-major.  The 32 tiles an XCD runs
// together then read 4 A + 8 B panels (row-major: 1 + 32), in step along K.
__device__ __forceinline__ void tile_ij_super(long long t, long long Ihi, int &I, int &J) {
	int r, c;
	tile_ij(t, r, c);
	const long long P = r >> 2, I0 = 4 * P;
	if(I0 + 3 > Ihi) {
		I = r;
		J = c;
		return;
	}
	const long long u = t - I0 * (I0 + 1) / 2, F = P >> 1;   // F full chunks: J < 8F <= I0
	if(u < 32 * F) {
		const int v = (int) (u & 31);
		I = (int) I0 + (v >> 3);
		J = 8 * (int) (u >> 5) + (v & 7);
		return;
	}
	long long w = u - 32 * F;
	int i = (int) I0;
	while(w >= i - 8 * F + 1) {
		w -= i - 8 * F + 1;
		++i;
	}
	I = i;
	J = (int) (8 * F + w);
}

__device__ __forceinline__ v8i_t fp4_xor_spread(const v8i_t &a, const v8i_t &b) {
	v8i_t v;
#pragma unroll
	for(int q = 0; q < 4; ++q) v[q] = (int) xor_or((uint32_t) a[q], (uint32_t) b[q], 0x22222222u);
	v[4] = v[5] = v[6] = v[7] = 0;
	return v;
}

template <int ET, bool SPLIT, bool BAND, int KCW = KC2>
__global__ __launch_bounds__(256, 1) void k_snp_mfma2(const uint2 *__restrict__ P, int Wp, int n, long long t0,
                                                      long long items, int S, int Wk, double nFactor, double bs,
                                                      typename Elem<ET>::T *__restrict__ D, long long rowBegin,
                                                      long long rowEnd, unsigned *__restrict__ cnt, long long cbase,
                                                      const long long *__restrict__ pfx, int npanels, int rank,
                                                      int world, int sorder) {
	constexpr int QS2 = TILE2 * KCW / 2 / 256, WPR = KCW / 2;   // uint4 staged per thread per panel; per row
	__shared__ __attribute__((aligned(16))) uint2 As[2][KCW * RS2];
	__shared__ __attribute__((aligned(16))) uint2 Bs[2][KCW * RS2];
	const long long item = t0 + xcd_tile(blockIdx.x, items), t = SPLIT ? item / S : item;
	int I, J;
	if(BAND) {   // tile t of the rank's list: panel I = last with pfx[I] <= t, J = t - pfx[I]
		int lo = 0, hi = npanels - 1;
		while(lo < hi) {
			const int mid = (lo + hi + 1) >> 1;
			if(pfx[mid] <= t) lo = mid; else hi = mid - 1;
		}
		I = lo;
		J = (int) (t - pfx[lo]);
	} else if(sorder) {
		tile_ij_super(t, (rowEnd - 1) / TILE2, I, J);
	} else {
		tile_ij(t, I, J);
	}
	const int wb = SPLIT ? (int) (item % S) * Wk : 0;
	const int Wl = SPLIT ? (wb + Wk < Wp ? Wk : Wp - wb) : Wp;
	const Shard sh{rank, world};
	// the A panel's row l: I * TILE2 + l, or the rank's owned row of that local
	// index (rows past n stage row 0 and are never stored)
	const auto arow = [&](int l) -> long long {
		const long long L = (long long) I * TILE2 + l;
		if(!BAND) return L;
		const long long lb = L / SB, r = (lb * world + rank) * SB + (L - lb * SB);
		return r < n ? r : 0;
	};
	const uint2 *Bp = P + (size_t) J * TILE2 * Wp + wb;
	long long ar[QS2];
	uint4 va[QS2], vb[QS2];
#pragma unroll
	for(int q = 0; q < QS2; ++q) {
		const int e = q * 256 + threadIdx.x, row = e / WPR, wp = e % WPR;
		ar[q] = arow(row);
		va[q] = *(const uint4 *) (P + (size_t) ar[q] * Wp + wb + 2 * wp);
		vb[q] = *(const uint4 *) (Bp + (size_t) row * Wp + 2 * wp);
	}
#pragma unroll
	for(int q = 0; q < QS2; ++q) {
		const int e = q * 256 + threadIdx.x, row = e / WPR, wp = e % WPR;
		As[0][(2 * wp) * RS2 + row] = make_uint2(va[q].x, va[q].y);
		As[0][(2 * wp + 1) * RS2 + row] = make_uint2(va[q].z, va[q].w);
		Bs[0][(2 * wp) * RS2 + row] = make_uint2(vb[q].x, vb[q].y);
		Bs[0][(2 * wp + 1) * RS2 + row] = make_uint2(vb[q].z, vb[q].w);
	}
	__syncthreads();
	const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
	const int wr = wid >> 1, wc = wid & 1;
	const int h = lane >> 5, l32 = lane & 31;
	const int ra0 = 128 * wr + l32, rb0 = 128 * wc + l32;
	v16f_t acc[4][4];
#pragma unroll
	for(int a = 0; a < 4; ++a)
#pragma unroll
		for(int c = 0; c < 4; ++c)
#pragma unroll
			for(int r = 0; r < 16; ++r) acc[a][c][r] = 0.0f;
	int buf = 0;
	for(int w0 = 0; w0 < Wl; w0 += KCW, buf ^= 1) {
		const bool more = w0 + KCW < Wl;
		if(more) {
#pragma unroll
			for(int q = 0; q < QS2; ++q) {
				const int e = q * 256 + threadIdx.x, row = e / WPR, wp = e % WPR;
				va[q] = *(const uint4 *) (P + (size_t) ar[q] * Wp + wb + w0 + KCW + 2 * wp);
				vb[q] = *(const uint4 *) (Bp + (size_t) row * Wp + w0 + KCW + 2 * wp);
			}
		}
		const uint2 *Ac = As[buf], *Bc = Bs[buf];
#pragma unroll
		for(int s = 0; s < KCW / 2; ++s) {
			const int w = 2 * s + h;   // this lane's word: its half of the step's 64 positions
			uint2 a[4], b[4];
#pragma unroll
			for(int x = 0; x < 4; ++x) {
				a[x] = Ac[w * RS2 + ra0 + 32 * x];
				b[x] = Bc[w * RS2 + rb0 + 32 * x];
			}
			v8i_t f0[4], g0[4], f1[4], g1[4];
#pragma unroll
			for(int x = 0; x < 4; ++x) {
				f0[x] = fp4_spread(a[x].x);
				g0[x] = fp4_spread(b[x].x);
			}
#pragma unroll
			for(int ta = 0; ta < 4; ++ta)
#pragma unroll
				for(int tb = 0; tb < 4; ++tb)
					acc[ta][tb] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(
					    f0[ta], g0[tb], acc[ta][tb], MFMA_FP4, MFMA_FP4, 0, MFMA_SCALE1, 0, MFMA_SCALE1);
#pragma unroll
			for(int x = 0; x < 4; ++x) {
				f1[x] = fp4_spread(a[x].y);
				g1[x] = fp4_spread(b[x].y);
			}
#pragma unroll
			for(int ta = 0; ta < 4; ++ta)
#pragma unroll
				for(int tb = 0; tb < 4; ++tb)
					acc[ta][tb] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(
					    f1[ta], g1[tb], acc[ta][tb], MFMA_FP4, MFMA_FP4, 0, MFMA_SCALE1, 0, MFMA_SCALE1);
#pragma unroll
			for(int x = 0; x < 4; ++x) {
				f0[x] = fp4_xor_spread(f0[x], f1[x]);
				g0[x] = fp4_xor_spread(g0[x], g1[x]);
			}
#pragma unroll
			for(int ta = 0; ta < 4; ++ta)
#pragma unroll
				for(int tb = 0; tb < 4; ++tb)
					acc[ta][tb] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(
					    f0[ta], g0[tb], acc[ta][tb], MFMA_FP4, MFMA_FP4, 0, MFMA_SCALE1, 0, MFMA_SCALE1);
		}
		if(more) {
			uint2 *An = As[buf ^ 1], *Bn = Bs[buf ^ 1];
#pragma unroll
			for(int q = 0; q < QS2; ++q) {
				const int e = q * 256 + threadIdx.x, row = e / WPR, wp = e % WPR;
				An[(2 * wp) * RS2 + row] = make_uint2(va[q].x, va[q].y);
				An[(2 * wp + 1) * RS2 + row] = make_uint2(va[q].z, va[q].w);
				Bn[(2 * wp) * RS2 + row] = make_uint2(vb[q].x, vb[q].y);
				Bn[(2 * wp + 1) * RS2 + row] = make_uint2(vb[q].z, vb[q].w);
			}
		}
		__syncthreads();
	}
	// epilogue: C/D of 32x32 (col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5));
	// dist = (3 L - dot) / 4 over the slice's L = 32 Wl positions
	const int L3 = 3 * 32 * Wl;
#pragma unroll
	for(int ta = 0; ta < 4; ++ta) {
#pragma unroll
		for(int r = 0; r < 16; ++r) {
			const int l = 128 * wr + 32 * ta + (r & 3) + 8 * (r >> 2) + 4 * h;
			const long long L = (long long) I * TILE2 + l;
			long long i = L;
			if(BAND) {
				const long long lb = L / SB;
				i = (lb * world + rank) * SB + (L - lb * SB);
			}
			if(i >= n || (!BAND && (i < rowBegin || i >= rowEnd))) continue;
			const long long base = BAND ? sh.off(i) : tri(i);
#pragma unroll
			for(int tb = 0; tb < 4; ++tb) {
				const long long j = (long long) J * TILE2 + 128 * wc + 32 * tb + l32;
				if(j < i) {
					const unsigned d = (unsigned) ((L3 - (int) acc[ta][tb][r]) >> 2);
					if(SPLIT) {
						atomicAdd(&cnt[base + j - cbase], d);
					} else {
						const double v = nFactor * (double) d;
						D[base + j] = Elem<ET>::put(v, 0.5, bs);
					}
				}
			}
		}
	}
}

// ------------------------------------------------------------------ MFMA, 256 x 256 tiles, LDS-DMA staged
// k_snp_mfma3: k_snp_mfma2's tile, its MX-fp4 steps and its epilogue, with the
// panels staged by global_load_lds (no VGPR staging, no ds_write) through
// NST3 stages of LDS, so that NST3 - 2 chunks stay in flight across each
// barrier (cdna_hip_programming.md, "Pipelining across barriers": counted
// vmcnt, raw s_barrier).  At one block per CU and 512 VGPRs the round-4/5
// kernel had one chunk of register staging in flight and waited for it
// before every barrier.  LDS image, one array: [stage][panel][slice][row] of
// 16 bytes (two plane words of one row), so one wave-instruction (64 lanes x
// 16 B, lane-linear) writes 64 consecutive rows of one slice, and a step's
// 8-byte reads (row ra0 + 32x, word 2s + h) are 512 contiguous bytes per
// wave.  Wave w stages slice w of both panels: 4 + 4 instructions per chunk.
#define NST3 4
#define KC3 8
template <int ET, bool SPLIT, bool BAND>
__global__ __launch_bounds__(256, 1) void k_snp_mfma3(const uint2 *__restrict__ P, int Wp, int n, long long t0,
                                                      long long items, int S, int Wk, double nFactor, double bs,
                                                      typename Elem<ET>::T *__restrict__ D, long long rowBegin,
                                                      long long rowEnd, unsigned *__restrict__ cnt, long long cbase,
                                                      const long long *__restrict__ pfx, int npanels, int rank,
                                                      int world, int sorder) {
	constexpr int NSL = KC3 / 2;   // 16-byte slices per chunk (one per wave)
	static_assert(NSL == 4, "one slice per wave");
	__shared__ __attribute__((aligned(16))) uint4 L[NST3 * 2 * NSL * TILE2];   // 128 KB
	const long long item = t0 + xcd_tile(blockIdx.x, items), t = SPLIT ? item / S : item;
	int I, J;
	if(BAND) {
		int lo = 0, hi = npanels - 1;
		while(lo < hi) {
			const int mid = (lo + hi + 1) >> 1;
			if(pfx[mid] <= t) lo = mid; else hi = mid - 1;
		}
		I = lo;
		J = (int) (t - pfx[lo]);
	} else if(sorder) {
		tile_ij_super(t, (rowEnd - 1) / TILE2, I, J);
	} else {
		tile_ij(t, I, J);
	}
	const int wb = SPLIT ? (int) (item % S) * Wk : 0;
	const int Wl = SPLIT ? (wb + Wk < Wp ? Wk : Wp - wb) : Wp;
	const Shard sh{rank, world};
	const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
	// this lane's staging sources: rows q 64 + lane of both panels, words 2 wid, 2 wid + 1 of each chunk
	const uint2 *srcA[4], *srcB[4];
#pragma unroll
	for(int q = 0; q < 4; ++q) {
		const long long Lr = (long long) I * TILE2 + q * 64 + lane;
		long long r = Lr;
		if(BAND) {
			const long long lb = Lr / SB;
			r = (lb * world + rank) * SB + (Lr - lb * SB);
			r = r < n ? r : 0;   // rows past n stage row 0 and are never stored
		}
		srcA[q] = P + (size_t) r * Wp + wb + 2 * wid;
		srcB[q] = P + ((size_t) J * TILE2 + q * 64 + lane) * Wp + wb + 2 * wid;
	}
	const int nch = Wl / KC3;
	// one LDS-DMA wave-instruction (64 lanes x 16 B, lane-linear at the
	// wave-uniform LDS byte address lds): in inline asm, so that the compiler
	// does not drain vmcnt(0) before every ds_read of the array (it cannot
	// tell the stages apart); the counted waits below order the reads
	const unsigned lbase = (unsigned) (uintptr_t) (__attribute__((address_space(3))) uint4 *) L;
	auto glds = [&](const uint2 *src, unsigned lds) {
		unsigned keep;
		asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
		             : "=&s"(keep)
		             : "v"(src), "s"(lds)
		             : "memory");
	};
	auto issue = [&](int c) {   // chunk c into stage c % NST3
		const int st = c % NST3, w0 = c * KC3;
#pragma unroll
		for(int q = 0; q < 4; ++q) {
			glds(srcA[q] + w0, __builtin_amdgcn_readfirstlane(lbase + (unsigned) ((((st * 2 + 0) * NSL + wid) * TILE2 + q * 64) * 16)));
			glds(srcB[q] + w0, __builtin_amdgcn_readfirstlane(lbase + (unsigned) ((((st * 2 + 1) * NSL + wid) * TILE2 + q * 64) * 16)));
		}
	};
	const int wr = wid >> 1, wc = wid & 1;
	const int h = lane >> 5, l32 = lane & 31;
	const int ra0 = 128 * wr + l32, rb0 = 128 * wc + l32;
	v16f_t acc[4][4];
#pragma unroll
	for(int ta = 0; ta < 4; ++ta)
#pragma unroll
		for(int tb = 0; tb < 4; ++tb)
#pragma unroll
			for(int r = 0; r < 16; ++r) acc[ta][tb][r] = 0.0f;
	// chunk c landed for every wave: this wave's counted wait (the later chunks
	// stay in flight), then the raw barrier
	auto land = [&](int c) {
		const int ahead = nch - 1 - c < NST3 - 2 ? nch - 1 - c : NST3 - 2;
		if(ahead >= 2) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
		else if(ahead == 1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
		else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
		asm volatile("" ::: "memory");
		__builtin_amdgcn_s_barrier();
		asm volatile("" ::: "memory");
	};
	// step gs (64 positions): word 2 (gs % 4) + h of chunk gs / 4, rows ra0 + 32 x / rb0 + 32 x
	auto rd = [&](int gs, uint2 (&a)[4], uint2 (&b)[4]) {
		const int st = (gs >> 2) % NST3, sl = gs & 3;
		const uint2 *Ac = (const uint2 *) &L[((st * 2 + 0) * NSL + sl) * TILE2];
		const uint2 *Bc = (const uint2 *) &L[((st * 2 + 1) * NSL + sl) * TILE2];
#pragma unroll
		for(int x = 0; x < 4; ++x) {
			a[x] = Ac[(ra0 + 32 * x) * 2 + h];
			b[x] = Bc[(rb0 + 32 * x) * 2 + h];
		}
	};
#define MF3(TA, TB, F, G)                                                                                         \
	acc[TA][TB] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(F, G, acc[TA][TB], MFMA_FP4, MFMA_FP4, 0, MFMA_SCALE1, \
	                                                              0, MFMA_SCALE1)
	for(int c = 0; c < NST3 - 1 && c < nch; ++c) issue(c);
	land(0);
	if(NST3 - 1 < nch) issue(NST3 - 1);
	uint2 a[4], b[4];
	v8i_t f0[4], g0[4];
	rd(0, a, b);
#pragma unroll
	for(int x = 0; x < 4; ++x) {
		f0[x] = fp4_spread(a[x].x);
		g0[x] = fp4_spread(b[x].x);
	}
	// Each component's 16 MFMAs carry the VALU work of the next component
	// (one spread or xor per MFMA slot, pinned by sched_group_barrier), so the
	// matrix pipe does not idle while a wave spreads (k_snp_mfma2: 16 MFMAs,
	// then the spreads; ~60% MFMA busy, profiles/r06_dist_clock.json):
	//   comp 0 (f0, g0) + the spreads of lo (f1, g1)
	//   comp 1 (f1, g1) + the xors (x0, y0) and the next step's LDS reads
	//   comp 2 (x0, y0) + the next step's spreads of hi (f0, g0)
	// A chunk's last step waits for the next chunk (counted vmcnt + barrier)
	// between comp 0 and comp 1, so its reads follow the barrier.
	auto step = [&](auto SI, int gs, bool more, bool open) {   // SI: the step's place in its chunk (sync group ids)
		constexpr int G0 = 3 * decltype(SI)::value;
		v8i_t f1[4], g1[4], x0[4], y0[4];
#pragma unroll
		for(int k = 0; k < 16; ++k) {
			MF3(k >> 2, k & 3, f0[k >> 2], g0[k & 3]);
			if(k < 8) {
				if(k & 1) g1[k >> 1] = fp4_spread(b[k >> 1].y);
				else f1[k >> 1] = fp4_spread(a[k >> 1].y);
			}
		}
		// one spread (3 shifts, 4 bitop3) per MFMA on the first 8.  Measured at 50k x 5 Mbp: 4 VALU per slot
		// on 14 slots was slower (6.43 against 6.26 s), 4 / 3 on all 16 slots (and 2 on component 1's) the
		// same (5.56 against 5.54 s, headline data)
#pragma unroll
		for(int k = 0; k < 8; ++k) {
			__builtin_amdgcn_sched_group_barrier(0x008, 1, G0);
			__builtin_amdgcn_sched_group_barrier(0x002, 7, G0);
		}
		__builtin_amdgcn_sched_group_barrier(0x008, 8, G0);
		if(open) {   // the next step opens chunk (gs + 1) / 4
			const int cn = (gs + 1) >> 2;
			land(cn);
			if(cn + NST3 - 1 < nch) issue(cn + NST3 - 1);
		}
		uint2 an[4], bn[4];
		if(more) rd(gs + 1, an, bn);
#pragma unroll
		for(int k = 0; k < 16; ++k) {
			MF3(k >> 2, k & 3, f1[k >> 2], g1[k & 3]);
			if(k < 8) {
				if(k & 1) y0[k >> 1] = fp4_xor_spread(g0[k >> 1], g1[k >> 1]);
				else x0[k >> 1] = fp4_xor_spread(f0[k >> 1], f1[k >> 1]);
			}
		}
		if(more) __builtin_amdgcn_sched_group_barrier(0x100, 8, G0 + 1);   // the next step's 8 LDS reads first
#pragma unroll
		for(int k = 0; k < 8; ++k) {
			__builtin_amdgcn_sched_group_barrier(0x008, 1, G0 + 1);
			__builtin_amdgcn_sched_group_barrier(0x002, 4, G0 + 1);   // one xor (4 bitop3)
		}
		__builtin_amdgcn_sched_group_barrier(0x008, 8, G0 + 1);
#pragma unroll
		for(int k = 0; k < 16; ++k) {
			MF3(k >> 2, k & 3, x0[k >> 2], y0[k & 3]);
			if(more && k < 8) {
				if(k & 1) g0[k >> 1] = fp4_spread(bn[k >> 1].x);
				else f0[k >> 1] = fp4_spread(an[k >> 1].x);
			}
		}
		if(more) {
#pragma unroll
			for(int k = 0; k < 8; ++k) {
				__builtin_amdgcn_sched_group_barrier(0x008, 1, G0 + 2);
				__builtin_amdgcn_sched_group_barrier(0x002, 7, G0 + 2);
			}
			__builtin_amdgcn_sched_group_barrier(0x008, 8, G0 + 2);
#pragma unroll
			for(int x = 0; x < 4; ++x) {
				a[x] = an[x];
				b[x] = bn[x];
			}
		}
	};
	for(int c = 0; c + 1 < nch; ++c) {   // every chunk but the last: 4 steps, the last one opens chunk c + 1
		step(std::integral_constant<int, 0>(), 4 * c + 0, true, false);
		step(std::integral_constant<int, 1>(), 4 * c + 1, true, false);
		step(std::integral_constant<int, 2>(), 4 * c + 2, true, false);
		step(std::integral_constant<int, 3>(), 4 * c + 3, true, true);
	}
	{   // the last chunk
		const int g = 4 * (nch - 1);
		step(std::integral_constant<int, 0>(), g + 0, true, false);
		step(std::integral_constant<int, 1>(), g + 1, true, false);
		step(std::integral_constant<int, 2>(), g + 2, true, false);
		step(std::integral_constant<int, 3>(), g + 3, false, false);
	}
#undef MF3
	// epilogue: k_snp_mfma2's
	const int L3 = 3 * 32 * Wl;
#pragma unroll
	for(int ta = 0; ta < 4; ++ta) {
#pragma unroll
		for(int r = 0; r < 16; ++r) {
			const int l = 128 * wr + 32 * ta + (r & 3) + 8 * (r >> 2) + 4 * h;
			const long long Lr = (long long) I * TILE2 + l;
			long long i = Lr;
			if(BAND) {
				const long long lb = Lr / SB;
				i = (lb * world + rank) * SB + (Lr - lb * SB);
			}
			if(i >= n || (!BAND && (i < rowBegin || i >= rowEnd))) continue;
			const long long base = BAND ? sh.off(i) : tri(i);
#pragma unroll
			for(int tb = 0; tb < 4; ++tb) {
				const long long j = (long long) J * TILE2 + 128 * wc + 32 * tb + l32;
				if(j < i) {
					const unsigned d = (unsigned) ((L3 - (int) acc[ta][tb][r]) >> 2);
					if(SPLIT) {
						atomicAdd(&cnt[base + j - cbase], d);
					} else {
						const double v = nFactor * (double) d;
						D[base + j] = Elem<ET>::put(v, 0.5, bs);
					}
				}
			}
		}
	}
}

// split-K epilogue: D[f] = nFactor * count (fsacmpthrd.c:247-255)
template <int ET>
__global__ void k_snp_finish(const unsigned *__restrict__ cnt, long long cbase, long long f0, long long f1,
                             double nFactor, double bs, typename Elem<ET>::T *__restrict__ D) {
	for(long long f = f0 + (long long) blockIdx.x * blockDim.x + threadIdx.x; f < f1;
	    f += (long long) gridDim.x * blockDim.x) {
		D[f] = Elem<ET>::put(nFactor * (double) cnt[f - cbase], 0.5, bs);
	}
}

// A7 epilogue (fsacmpthrd.c:420-475) for one pair
template <int ET>
__device__ __forceinline__ void pair_store(typename Elem<ET>::T *D, typename Elem<ET>::T *N, long long f, uint32_t dist,
                                           uint32_t inc, unsigned norm, unsigned minLength, double bs) {
	typedef typename Elem<ET>::T T;
	if(ET == 8) {
		double v;
		if(minLength <= inc) {
			v = norm ? (double) ((unsigned long long) dist * norm) / inc : (double) dist;
		} else {
			v = -1.0;
		}
		D[f] = (T) v;
		if(N) N[f] = (T) (double) inc;
	} else if(ET == 4) {
		float v;
		if(minLength <= inc) {
			if(norm) {
				v = (float) ((unsigned long long) dist * norm);
				v = v / (float) inc;
			} else {
				v = (float) dist;
			}
		} else {
			v = -1.0f;
		}
		D[f] = (T) v;
		if(N) N[f] = (T) (float) inc;
	} else {
		double v;
		if(minLength <= inc) {
			v = norm ? ((double) ((unsigned long long) dist * norm) * bs + 0.5) / inc : (double) dist * bs + 0.5;
		} else {
			v = -1.0 * bs + 0;
		}
		D[f] = (T) cvt_i32_x86(v);
		if(N) N[f] = (T) cvt_i32_x86(inc * bs + 0.5);
	}
}

// Pair tiles: as k_snp_tile, with each taxon's mask beside its planes
// (uint4 {hi, lo, m, 0} per word): double-buffered KCP-word chunks of both
// 128-row panels, XCD-contiguous tile order, and split-K over word slices when
// the tiles do not fill the chip (exact u32 atomics of dist and n, then
// k_snp_pair_finish applies the A7 epilogue).  BAND: one rank of the
// row-sharded layout, as k_snp_tile_band (A panel = the rank's owned rows,
// tile t of the rank's list found in pfx, rows stored at Shard::off(i), no
// N); split-K counts are indexed by the rank's local element.
template <int ET, bool SPLIT, bool BAND = false>
__global__ __launch_bounds__(256, 2) void k_snp_tile_pair(const uint4 *__restrict__ P, int Wp, int n, long long t0,
                                                          long long items, int S, int Wk, unsigned norm,
                                                          unsigned minLength, double bs,
                                                          typename Elem<ET>::T *__restrict__ D,
                                                          typename Elem<ET>::T *__restrict__ Nm, long long rowBegin,
                                                          long long rowEnd, unsigned *__restrict__ cd,
                                                          unsigned *__restrict__ cn, long long cbase,
                                                          const long long *__restrict__ pfx = nullptr, int npanels = 0,
                                                          int rank = 0, int world = 1) {
	__shared__ __attribute__((aligned(16))) uint4 As[2][KCP * RSP];
	__shared__ __attribute__((aligned(16))) uint4 Bs[2][KCP * RSP];
	int I, J;
	const long long item = t0 + xcd_tile(blockIdx.x, items);
	if(BAND) {
		const long long tile = item / S;
		int lo = 0, hi = npanels - 1;
		while(lo < hi) {
			const int mid = (lo + hi + 1) >> 1;
			if(pfx[mid] <= tile) lo = mid; else hi = mid - 1;
		}
		I = lo;
		J = (int) (tile - pfx[lo]);
	} else {
		tile_ij(item / S, I, J);
	}
	// global row of A-panel row l (band: the rank's owned row I*TILE + l; rows
	// past n read row 0)
	const auto arow = [&](int l) -> long long {
		const long long L = (long long) I * TILE + l;
		if(!BAND) return L;
		const long long lb = L / SB, r = (lb * world + rank) * SB + (L - lb * SB);
		return r < n ? r : 0;
	};
	const int wb = (int) (item % S) * Wk, we = wb + Wk < Wp ? wb + Wk : Wp;
	const int Wl = we - wb;   // a multiple of KCP
	const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
	const uint4 *Aq[4];
#pragma unroll
	for(int q = 0; q < 4; ++q) Aq[q] = P + (size_t) arow((q * 256 + threadIdx.x) >> 3) * Wp + wb;
	const uint4 *Bp = P + (size_t) J * TILE * Wp + wb;
	uint32_t ad[8][8], an[8][8];
#pragma unroll
	for(int a = 0; a < 8; ++a)
#pragma unroll
		for(int c = 0; c < 8; ++c) {
			ad[a][c] = 0;
			an[a][c] = 0;
		}
	uint4 va[4], vb[4];
#pragma unroll
	for(int q = 0; q < 4; ++q) {
		const int e = q * 256 + threadIdx.x, row = e >> 3, wp = e & 7;
		va[q] = Aq[q][wp];
		vb[q] = Bp[(size_t) row * Wp + wp];
	}
#pragma unroll
	for(int q = 0; q < 4; ++q) {
		const int e = q * 256 + threadIdx.x, row = e >> 3, wp = e & 7;
		As[0][wp * RSP + row] = va[q];
		Bs[0][wp * RSP + row] = vb[q];
	}
	__syncthreads();
	int buf = 0;
	for(int w0 = 0; w0 < Wl; w0 += KCP, buf ^= 1) {
		const bool more = w0 + KCP < Wl;
		if(more) {
#pragma unroll
			for(int q = 0; q < 4; ++q) {
				const int e = q * 256 + threadIdx.x, row = e >> 3, wp = e & 7;
				va[q] = Aq[q][w0 + KCP + wp];
				vb[q] = Bp[(size_t) row * Wp + w0 + KCP + wp];
			}
		}
		const uint4 *Ac = As[buf], *Bc = Bs[buf];
#pragma unroll 1
		for(int w = 0; w < KCP; ++w) {
			uint4 a[8], b[8];
#pragma unroll
			for(int q = 0; q < 4; ++q) {
				a[2 * q] = Ac[w * RSP + 2 * ty + 32 * q];
				a[2 * q + 1] = Ac[w * RSP + 2 * ty + 32 * q + 1];
				b[2 * q] = Bc[w * RSP + 2 * tx + 32 * q];
				b[2 * q + 1] = Bc[w * RSP + 2 * tx + 32 * q + 1];
			}
#pragma unroll
			for(int x = 0; x < 8; ++x) {
#pragma unroll
				for(int y = 0; y < 8; ++y) {
					const uint32_t m = a[x].z & b[y].z;
					ad[x][y] += __popc(xor_or(a[x].x, b[y].x, a[x].y ^ b[y].y) & m);
					an[x][y] += __popc(m);
				}
			}
		}
		if(more) {
			uint4 *An = As[buf ^ 1], *Bn = Bs[buf ^ 1];
#pragma unroll
			for(int q = 0; q < 4; ++q) {
				const int e = q * 256 + threadIdx.x, row = e >> 3, wp = e & 7;
				An[wp * RSP + row] = va[q];
				Bn[wp * RSP + row] = vb[q];
			}
		}
		__syncthreads();
	}
#pragma unroll
	for(int a = 0; a < 8; ++a) {
		const int l = 2 * ty + 32 * (a >> 1) + (a & 1);
		long long i = (long long) I * TILE + l;
		long long base;
		if(BAND) {
			const long long lb = i / SB;
			i = (lb * world + rank) * SB + (i - lb * SB);
			if(i >= n) continue;
			base = Shard{rank, world}.off(i);
		} else {
			if(i >= n || i < rowBegin || i >= rowEnd) continue;
			base = tri(i);
		}
#pragma unroll
		for(int c = 0; c < 8; ++c) {
			long long j = (long long) J * TILE + 2 * tx + 32 * (c >> 1) + (c & 1);
			if(j < i) {
				if(SPLIT) {
					atomicAdd(&cd[base + j - cbase], ad[a][c]);
					atomicAdd(&cn[base + j - cbase], an[a][c]);
				} else {
					pair_store<ET>(D, Nm, base + j, ad[a][c], an[a][c], norm, minLength, bs);
				}
			}
		}
	}
}

// Pair mode (fsacmpair fsacmp.c:587: dist and n over inc_a & inc_b) on the
// matrix cores: each component nibble is zeroed where the row's mask bit is
// 0, so over the positions both rows include, equal codes dot to 3 and
// different ones to -1 (dot = 3 n - 4 dist), and a fourth component, the
// mask itself (+1 / 0), dots to n = popc(m_a & m_b).  Same tiles, staging
// (uint4 {hi, lo, m, 0} words, KCP-word chunks) and split-K as
// k_snp_tile_pair; exact while 3 L < 2^24 per slice.
// one pair-mode operand: component comp (0 hi, 1 lo, 2 hi ^ lo: masked +-1;
// 3: the mask as +1 / 0) of a lane's word, from its mask spread mq
__device__ __forceinline__ v8i_t fp4_pair_comp(uint32_t hi, uint32_t lo, const uint32_t (&mq)[4], int comp) {
	v8i_t v;
#pragma unroll
	for(int q = 0; q < 4; ++q) {
		if(comp == 3) {
			v[q] = (int) (mq[q] >> 2);   // +1.0 where included
		} else {
			const uint32_t x = comp == 0 ? hi : comp == 1 ? lo : hi ^ lo;
			const uint32_t xs = q < 3 ? x << (3 - q) : x;
			const uint32_t mf = mq[q] | (mq[q] >> 1) | (mq[q] >> 2) | (mq[q] >> 3);   // 0xF where included
			v[q] = (int) (((xs & 0x88888888u) | 0x22222222u) & mf);
		}
	}
	v[4] = v[5] = v[6] = v[7] = 0;
	return v;
}

template <int ET, bool SPLIT, bool BAND = false>
__global__ __launch_bounds__(256, 2) void k_snp_mfma_pair(const uint4 *__restrict__ P, int Wp, int n, long long t0,
                                                          long long items, int S, int Wk, unsigned norm,
                                                          unsigned minLength, double bs,
                                                          typename Elem<ET>::T *__restrict__ D,
                                                          typename Elem<ET>::T *__restrict__ Nm, long long rowBegin,
                                                          long long rowEnd, unsigned *__restrict__ cd,
                                                          unsigned *__restrict__ cn, long long cbase,
                                                          const long long *__restrict__ pfx = nullptr, int npanels = 0,
                                                          int rank = 0, int world = 1) {
	__shared__ __attribute__((aligned(16))) uint4 As[2][KCP * RSP];
	__shared__ __attribute__((aligned(16))) uint4 Bs[2][KCP * RSP];
	int I, J;
	const long long item = t0 + xcd_tile(blockIdx.x, items);
	if(BAND) {   // as k_snp_tile_pair's band form
		const long long tile = item / S;
		int lo = 0, hi = npanels - 1;
		while(lo < hi) {
			const int mid = (lo + hi + 1) >> 1;
			if(pfx[mid] <= tile) lo = mid; else hi = mid - 1;
		}
		I = lo;
		J = (int) (tile - pfx[lo]);
	} else {
		tile_ij(item / S, I, J);
	}
	const auto arow = [&](int l) -> long long {
		const long long L = (long long) I * TILE + l;
		if(!BAND) return L;
		const long long lb = L / SB, r = (lb * world + rank) * SB + (L - lb * SB);
		return r < n ? r : 0;
	};
	const int wb = (int) (item % S) * Wk, we = wb + Wk < Wp ? wb + Wk : Wp;
	const int Wl = we - wb;   // a multiple of KCP
	const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
	const int wr = wid >> 1, wc = wid & 1;
	const uint4 *Aq[4];
#pragma unroll
	for(int q = 0; q < 4; ++q) Aq[q] = P + (size_t) arow((q * 256 + threadIdx.x) >> 3) * Wp + wb;
	const uint4 *Bp = P + (size_t) J * TILE * Wp + wb;
	v16f_t acc[2][2], accn[2][2];
#pragma unroll
	for(int a = 0; a < 2; ++a)
#pragma unroll
		for(int c = 0; c < 2; ++c)
#pragma unroll
			for(int r = 0; r < 16; ++r) acc[a][c][r] = accn[a][c][r] = 0.0f;
	uint4 va[4], vb[4];
#pragma unroll
	for(int q = 0; q < 4; ++q) {
		const int e = q * 256 + threadIdx.x, row = e >> 3, wp = e & 7;
		va[q] = Aq[q][wp];
		vb[q] = Bp[(size_t) row * Wp + wp];
	}
#pragma unroll
	for(int q = 0; q < 4; ++q) {
		const int e = q * 256 + threadIdx.x, row = e >> 3, wp = e & 7;
		As[0][wp * RSP + row] = va[q];
		Bs[0][wp * RSP + row] = vb[q];
	}
	__syncthreads();
	const int h = lane >> 5, l32 = lane & 31;
	const int ra0 = 64 * wr + l32, rb0 = 64 * wc + l32;
	int buf = 0;
	for(int w0 = 0; w0 < Wl; w0 += KCP, buf ^= 1) {
		const bool more = w0 + KCP < Wl;
		if(more) {
#pragma unroll
			for(int q = 0; q < 4; ++q) {
				const int e = q * 256 + threadIdx.x, row = e >> 3, wp = e & 7;
				va[q] = Aq[q][w0 + KCP + wp];
				vb[q] = Bp[(size_t) row * Wp + w0 + KCP + wp];
			}
		}
		const uint4 *Ac = As[buf], *Bc = Bs[buf];
#pragma unroll 1
		for(int s = 0; s < KCP / 2; ++s) {
			const int w = 2 * s + h;
			uint4 a[2], b[2];
			uint32_t ma[2][4], mb[2][4];
#pragma unroll
			for(int t = 0; t < 2; ++t) {
				a[t] = Ac[w * RSP + ra0 + 32 * t];
				b[t] = Bc[w * RSP + rb0 + 32 * t];
#pragma unroll
				for(int q = 0; q < 4; ++q) {
					ma[t][q] = (q < 3 ? a[t].z << (3 - q) : a[t].z) & 0x88888888u;
					mb[t][q] = (q < 3 ? b[t].z << (3 - q) : b[t].z) & 0x88888888u;
				}
			}
#pragma unroll
			for(int comp = 0; comp < 4; ++comp) {
				v8i_t fa[2], fb[2];
#pragma unroll
				for(int t = 0; t < 2; ++t) {
					fa[t] = fp4_pair_comp(a[t].x, a[t].y, ma[t], comp);
					fb[t] = fp4_pair_comp(b[t].x, b[t].y, mb[t], comp);
				}
#pragma unroll
				for(int ta = 0; ta < 2; ++ta)
#pragma unroll
					for(int tb = 0; tb < 2; ++tb) {
						if(comp < 3)
							acc[ta][tb] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(
							    fa[ta], fb[tb], acc[ta][tb], MFMA_FP4, MFMA_FP4, 0, MFMA_SCALE1, 0, MFMA_SCALE1);
						else
							accn[ta][tb] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(
							    fa[ta], fb[tb], accn[ta][tb], MFMA_FP4, MFMA_FP4, 0, MFMA_SCALE1, 0, MFMA_SCALE1);
					}
			}
		}
		if(more) {
			uint4 *An = As[buf ^ 1], *Bn = Bs[buf ^ 1];
#pragma unroll
			for(int q = 0; q < 4; ++q) {
				const int e = q * 256 + threadIdx.x, row = e >> 3, wp = e & 7;
				An[wp * RSP + row] = va[q];
				Bn[wp * RSP + row] = vb[q];
			}
		}
		__syncthreads();
	}
#pragma unroll
	for(int ta = 0; ta < 2; ++ta) {
#pragma unroll
		for(int r = 0; r < 16; ++r) {
			long long i = (long long) I * TILE + 64 * wr + 32 * ta + (r & 3) + 8 * (r >> 2) + 4 * h;
			long long base;
			if(BAND) {
				const long long lb = i / SB;
				i = (lb * world + rank) * SB + (i - lb * SB);
				if(i >= n) continue;
				base = Shard{rank, world}.off(i);
			} else {
				if(i >= n || i < rowBegin || i >= rowEnd) continue;
				base = tri(i);
			}
#pragma unroll
			for(int tb = 0; tb < 2; ++tb) {
				const long long j = (long long) J * TILE + 64 * wc + 32 * tb + l32;
				if(j < i) {
					const int nn = (int) accn[ta][tb][r];
					const unsigned d = (unsigned) ((3 * nn - (int) acc[ta][tb][r]) >> 2);
					if(SPLIT) {
						atomicAdd(&cd[base + j - cbase], d);
						atomicAdd(&cn[base + j - cbase], (unsigned) nn);
					} else {
						pair_store<ET>(D, Nm, base + j, d, (uint32_t) nn, norm, minLength, bs);
					}
				}
			}
		}
	}
}

// k_snp_mfma2_pair: pair mode on k_snp_mfma2's 256 x 256 tiles.  The mask
// enters the nibble's exponent instead of being and-ed in afterwards: a
// component nibble is (sign << 3) | (m << 1), +-1.0 where the row includes the
// position and +-0.0 where it does not, so one mask spread per word (the 0x2
// bits, itself the fourth operand: +1 / 0) serves all four components; hi and
// lo cost one and_or per dword on top of it and hi ^ lo one xor_or
// ((a ^ b) | msp: the shared exponent bits cancel and are set again).  Two
// accumulator sets (dot, n) per 32 x 32 tile, so a wave takes 128 x 64 and a
// block of 4 waves one column half of a 256 x 256 tile (items = 2 per tile):
// each step spreads 4 A and 2 B words (25 VALU each) for 32 MFMAs, against
// k_snp_mfma_pair's 384 VALU for 16.  Staging as k_snp_mfma2 with uint4
// {hi, lo, m, 0} words (99 KB of LDS at 8 words per chunk, one block per
// CU); BAND and SPLIT as k_snp_mfma2.
__device__ __forceinline__ v8i_t pair2_mask(uint32_t m) {
	v8i_t v;
	v[0] = (int) ((m << 1) & 0x22222222u);
	v[1] = (int) (m & 0x22222222u);
	v[2] = (int) ((m >> 1) & 0x22222222u);
	v[3] = (int) ((m >> 2) & 0x22222222u);
	v[4] = v[5] = v[6] = v[7] = 0;
	return v;
}

__device__ __forceinline__ v8i_t pair2_comp(uint32_t x, const v8i_t &m) {
	v8i_t v;
	v[0] = (int) and_or(x << 3, 0x88888888u, (uint32_t) m[0]);
	v[1] = (int) and_or(x << 2, 0x88888888u, (uint32_t) m[1]);
	v[2] = (int) and_or(x << 1, 0x88888888u, (uint32_t) m[2]);
	v[3] = (int) and_or(x, 0x88888888u, (uint32_t) m[3]);
	v[4] = v[5] = v[6] = v[7] = 0;
	return v;
}

__device__ __forceinline__ v8i_t pair2_xor(const v8i_t &h, const v8i_t &l, const v8i_t &m) {
	v8i_t v;
#pragma unroll
	for(int q = 0; q < 4; ++q) v[q] = (int) xor_or((uint32_t) h[q], (uint32_t) l[q], (uint32_t) m[q]);
	v[4] = v[5] = v[6] = v[7] = 0;
	return v;
}

#define RS2P 258   // pair LDS row strides (uint4): 256 A rows, 128 B rows, + pad
#define RS2B 130
template <int ET, bool SPLIT, bool BAND>
__global__ __launch_bounds__(256, 1) void k_snp_mfma2_pair(const uint4 *__restrict__ P, int Wp, int n, long long t0,
                                                           long long items, int S, int Wk, unsigned norm,
                                                           unsigned minLength, double bs,
                                                           typename Elem<ET>::T *__restrict__ D,
                                                           typename Elem<ET>::T *__restrict__ Nm, long long rowBegin,
                                                           long long rowEnd, unsigned *__restrict__ cd,
                                                           unsigned *__restrict__ cn, long long cbase,
                                                           const long long *__restrict__ pfx, int npanels, int rank,
                                                           int world) {
	constexpr int QA = TILE2 * KC2 / 256, QB = QA / 2;   // uint4 staged per thread: A panel, B half panel
	__shared__ __attribute__((aligned(16))) uint4 As[2][KC2 * RS2P];
	__shared__ __attribute__((aligned(16))) uint4 Bs[2][KC2 * RS2B];
	const long long item = t0 + xcd_tile(blockIdx.x, items), th = SPLIT ? item / S : item, t = th >> 1;
	const int half = (int) (th & 1);   // the tile's column half: B rows J * 256 + 128 half + [0, 128)
	int I, J;
	if(BAND) {
		int lo = 0, hi = npanels - 1;
		while(lo < hi) {
			const int mid = (lo + hi + 1) >> 1;
			if(pfx[mid] <= t) lo = mid; else hi = mid - 1;
		}
		I = lo;
		J = (int) (t - pfx[lo]);
	} else {
		tile_ij(t, I, J);
	}
	const int wb = SPLIT ? (int) (item % S) * Wk : 0;
	const int Wl = SPLIT ? (wb + Wk < Wp ? Wk : Wp - wb) : Wp;
	const auto arow = [&](int l) -> long long {
		const long long L = (long long) I * TILE2 + l;
		if(!BAND) return L;
		const long long lb = L / SB, r = (lb * world + rank) * SB + (L - lb * SB);
		return r < n ? r : 0;
	};
	const uint4 *Bp = P + ((size_t) J * TILE2 + 128 * half) * Wp + wb;
	const uint4 *Ap[QA];
	// (staging registers in arrays of 4 uint4: a larger array is left in scratch)
	// (staging registers as native 4-dword vectors: HIP's uint4 struct copies
	// become memcpys that keep the arrays in scratch)
	typedef unsigned u4v __attribute__((ext_vector_type(4)));
	u4v vaa[4], vab[4], vb[4];
	static_assert(QA == 8 && QB == 4, "staging registers: A in two arrays of 4, B in one");
	u4v *As4 = (u4v *) &As[0][0], *Bs4 = (u4v *) &Bs[0][0];
	const int srow = threadIdx.x / KC2, swp = threadIdx.x % KC2;   // staged element q: row srow + 32 q, word swp
#pragma unroll
	for(int q = 0; q < QA; ++q) Ap[q] = P + (size_t) arow(srow + 32 * q) * Wp + wb + swp;
#pragma unroll
	for(int q = 0; q < 4; ++q) {
		vaa[q] = *(const u4v *) Ap[q];
		vab[q] = *(const u4v *) Ap[q + 4];
	}
	Bp += (size_t) srow * Wp + swp;
#pragma unroll
	for(int q = 0; q < QB; ++q) vb[q] = *(const u4v *) (Bp + (size_t) 32 * q * Wp);
#pragma unroll
	for(int q = 0; q < 4; ++q) {
		As4[swp * RS2P + srow + 32 * q] = vaa[q];
		As4[swp * RS2P + srow + 32 * (q + 4)] = vab[q];
	}
#pragma unroll
	for(int q = 0; q < QB; ++q) Bs4[swp * RS2B + srow + 32 * q] = vb[q];
	__syncthreads();
	const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
	const int wr = wid >> 1, wc = wid & 1;
	const int h = lane >> 5, l32 = lane & 31;
	const int ra0 = 128 * wr + l32, rb0 = 64 * wc + l32;
	v16f_t acc[4][2], accn[4][2];
#pragma unroll
	for(int a = 0; a < 4; ++a)
#pragma unroll
		for(int c = 0; c < 2; ++c)
#pragma unroll
			for(int r = 0; r < 16; ++r) acc[a][c][r] = accn[a][c][r] = 0.0f;
	int buf = 0;
	for(int w0 = 0; w0 < Wl; w0 += KC2, buf ^= 1) {
		const bool more = w0 + KC2 < Wl;
		if(more) {
#pragma unroll
			for(int q = 0; q < 4; ++q) {
				vaa[q] = *(const u4v *) (Ap[q] + w0 + KC2);
				vab[q] = *(const u4v *) (Ap[q + 4] + w0 + KC2);
			}
#pragma unroll
			for(int q = 0; q < QB; ++q) vb[q] = *(const u4v *) (Bp + (size_t) 32 * q * Wp + w0 + KC2);
		}
		const uint4 *Ac = As[buf], *Bc = Bs[buf];
#pragma unroll
		for(int s = 0; s < KC2 / 2; ++s) {
			const int w = 2 * s + h;
			uint4 av[4], bv[2];
			v8i_t am[4], ah[4], al[4], bm[2], bh[2], bl[2];
#pragma unroll
			for(int x = 0; x < 4; ++x) {
				av[x] = Ac[w * RS2P + ra0 + 32 * x];
				am[x] = pair2_mask(av[x].z);
			}
#pragma unroll
			for(int y = 0; y < 2; ++y) {
				bv[y] = Bc[w * RS2B + rb0 + 32 * y];
				bm[y] = pair2_mask(bv[y].z);
			}
#pragma unroll
			for(int ta = 0; ta < 4; ++ta)
#pragma unroll
				for(int tb = 0; tb < 2; ++tb)
					accn[ta][tb] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(
					    am[ta], bm[tb], accn[ta][tb], MFMA_FP4, MFMA_FP4, 0, MFMA_SCALE1, 0, MFMA_SCALE1);
#pragma unroll
			for(int x = 0; x < 4; ++x) ah[x] = pair2_comp(av[x].x, am[x]);
#pragma unroll
			for(int y = 0; y < 2; ++y) bh[y] = pair2_comp(bv[y].x, bm[y]);
#pragma unroll
			for(int ta = 0; ta < 4; ++ta)
#pragma unroll
				for(int tb = 0; tb < 2; ++tb)
					acc[ta][tb] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(
					    ah[ta], bh[tb], acc[ta][tb], MFMA_FP4, MFMA_FP4, 0, MFMA_SCALE1, 0, MFMA_SCALE1);
#pragma unroll
			for(int x = 0; x < 4; ++x) al[x] = pair2_comp(av[x].y, am[x]);
#pragma unroll
			for(int y = 0; y < 2; ++y) bl[y] = pair2_comp(bv[y].y, bm[y]);
#pragma unroll
			for(int ta = 0; ta < 4; ++ta)
#pragma unroll
				for(int tb = 0; tb < 2; ++tb)
					acc[ta][tb] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(
					    al[ta], bl[tb], acc[ta][tb], MFMA_FP4, MFMA_FP4, 0, MFMA_SCALE1, 0, MFMA_SCALE1);
#pragma unroll
			for(int x = 0; x < 4; ++x) ah[x] = pair2_xor(ah[x], al[x], am[x]);
#pragma unroll
			for(int y = 0; y < 2; ++y) bh[y] = pair2_xor(bh[y], bl[y], bm[y]);
#pragma unroll
			for(int ta = 0; ta < 4; ++ta)
#pragma unroll
				for(int tb = 0; tb < 2; ++tb)
					acc[ta][tb] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(
					    ah[ta], bh[tb], acc[ta][tb], MFMA_FP4, MFMA_FP4, 0, MFMA_SCALE1, 0, MFMA_SCALE1);
		}
		if(more) {
			u4v *An = (u4v *) As[buf ^ 1], *Bn = (u4v *) Bs[buf ^ 1];
#pragma unroll
			for(int q = 0; q < 4; ++q) {
				An[swp * RS2P + srow + 32 * q] = vaa[q];
				An[swp * RS2P + srow + 32 * (q + 4)] = vab[q];
			}
#pragma unroll
			for(int q = 0; q < QB; ++q) Bn[swp * RS2B + srow + 32 * q] = vb[q];
		}
		__syncthreads();
	}
	// epilogue as k_snp_mfma2 (C/D row (r & 3) + 8 (r >> 2) + 4 h, column l32)
#pragma unroll
	for(int ta = 0; ta < 4; ++ta) {
#pragma unroll
		for(int r = 0; r < 16; ++r) {
			const long long L = (long long) I * TILE2 + 128 * wr + 32 * ta + (r & 3) + 8 * (r >> 2) + 4 * h;
			long long i = L;
			if(BAND) {
				const long long lb = L / SB;
				i = (lb * world + rank) * SB + (L - lb * SB);
			}
			if(i >= n || (!BAND && (i < rowBegin || i >= rowEnd))) continue;
			const long long base = BAND ? Shard{rank, world}.off(i) : tri(i);
#pragma unroll
			for(int tb = 0; tb < 2; ++tb) {
				const long long j = (long long) J * TILE2 + 128 * half + 64 * wc + 32 * tb + l32;
				if(j < i) {
					const int nn = (int) accn[ta][tb][r];
					const unsigned d = (unsigned) ((3 * nn - (int) acc[ta][tb][r]) >> 2);
					if(SPLIT) {
						atomicAdd(&cd[base + j - cbase], d);
						atomicAdd(&cn[base + j - cbase], (unsigned) nn);
					} else {
						pair_store<ET>(D, Nm, base + j, d, (uint32_t) nn, norm, minLength, bs);
					}
				}
			}
		}
	}
}

// split-K epilogue of pair mode: the A7 store of the summed (dist, n)
template <int ET>
__global__ void k_snp_pair_finish(const unsigned *__restrict__ cd, const unsigned *__restrict__ cn, long long f0,
                                  long long f1, unsigned norm, unsigned minLength, double bs,
                                  typename Elem<ET>::T *__restrict__ D, typename Elem<ET>::T *__restrict__ Nm) {
	for(long long f = f0 + (long long) blockIdx.x * blockDim.x + threadIdx.x; f < f1;
	    f += (long long) gridDim.x * blockDim.x) {
		pair_store<ET>(D, Nm, f, cd[f - f0], cn[f - f0], norm, minLength, bs);
	}
}

// ------------------------------------------------- pair mode with -P > 0
// maskProxi (fsacmp.c:355-485) followed by fsacmpair (fsacmp.c:587).  The
// reference walks the pair's SNPs (inc_i & inc_j set, codes differ) from the
// last position down; its counter i stands for position p + 1 (the "label"),
// and with lastSNP starting at len + proxi it clears include bits
// [label, lastSNP] whenever lastSNP - label <= proxi, then lastSNP = label.
// The cleared set is therefore the union of the closed intervals between
// consecutive labels (plus the sentinel len + proxi) that are at most proxi
// apart, and the pair's (dist, n) are the unmasked counts minus the counts
// over that union.  Consecutive intervals share one end point, which is
// added back once when both sides qualify.
//
// One wave per pair, 64 words per step (one per lane, coalesced): a max-scan
// of the lanes' highest labels gives every lane the label below its first
// SNP; a second scan over (label, qualified) carries whether that label's
// own lower gap qualified.  Interval counts re-read the (cached) words they
// cover.  The sequential dependency of maskProxi is only between consecutive
// SNPs, so the result is exact and independent of the lane split.
__device__ __forceinline__ int wave_scan_max_incl(int v, int lane) {
#pragma unroll
	for(int o = 1; o < 64; o <<= 1) {
		int t = __shfl_up(v, o, 64);
		if(lane >= o) v = v > t ? v : t;
	}
	return v;
}

// positions [s, e] (clipped to the W32 counted words) of pair rows A, B
__device__ __forceinline__ void range_counts(const uint4 *__restrict__ A, const uint4 *__restrict__ B, int W32, int s,
                                             int e, uint32_t &cm, uint32_t &cd) {
	cm = cd = 0;
	if(e > 32 * W32 - 1) e = 32 * W32 - 1;
	for(int w = s >> 5; w <= (e >> 5) && s <= e; ++w) {
		const int ks = w == (s >> 5) ? (s & 31) : 0, ke = w == (e >> 5) ? (e & 31) : 31;
		const uint32_t msk = (0xFFFFFFFFu >> ks) & (0xFFFFFFFFu << (31 - ke));
		const uint4 a = A[w], b = B[w];
		const uint32_t m = a.z & b.z & msk;
		cm += __popc(m);
		cd += __popc(xor_or(a.x, b.x, a.y ^ b.y) & m);
	}
}

template <int ET>
__global__ __launch_bounds__(256) void k_snp_pair_proxi(const uint4 *__restrict__ P, int Wp, int W32, int len, int proxi,
                                                        long long f0, long long f1, unsigned norm, unsigned minLength,
                                                        double bs, typename Elem<ET>::T *__restrict__ D,
                                                        typename Elem<ET>::T *__restrict__ Nm) {
	const int lane = threadIdx.x & 63;
	const long long stride = (long long) gridDim.x * 4;
	for(long long f = f0 + (long long) blockIdx.x * 4 + (threadIdx.x >> 6); f < f1; f += stride) {
		long long i = (long long) ((1.0 + sqrt(1.0 + 8.0 * (double) f)) * 0.5);
		while(tri(i) > f) --i;
		while(tri(i + 1) <= f) ++i;
		const long long j = f - tri(i);
		const uint4 *A = P + (size_t) i * Wp, *B = P + (size_t) j * Wp;
		int dist = 0, cnt = 0;
		int cL = -1, cQ = 0;                 // highest label so far, and whether its lower gap qualified
		for(int w0 = 0; w0 < W32; w0 += 64) {
			const int w = w0 + lane;
			uint32_t m = 0, d = 0;
			if(w < W32) {
				const uint4 a = A[w], b = B[w];
				m = a.z & b.z;
				d = xor_or(a.x, b.x, a.y ^ b.y) & m;
			}
			cnt += __popc(m);
			dist += __popc(d);
			// bit 31 - k <-> position 32w + k; label = position + 1
			const int hiL = d ? 32 * w + 32 - (__ffs(d)) + 1 : -1;
			int incl = wave_scan_max_incl(hiL, lane);
			int prevL = __shfl_up(incl, 1, 64);
			if(lane == 0) prevL = -1;
			if(cL > prevL) prevL = cL;
			// q of each own label: gap to the label below <= proxi
			int qhi = 0;
			{
				int prev = prevL;
				for(uint32_t x = d; x;) {
					const int k = __clz(x);
					x &= ~(0x80000000u >> k);
					const int cur = 32 * w + k + 1;
					qhi = prev >= 0 && cur - prev <= proxi;
					prev = cur;
				}
			}
			const int packed = hiL >= 0 ? 2 * hiL + qhi : -1;
			const int incl2 = wave_scan_max_incl(packed, lane);
			int prevP = __shfl_up(incl2, 1, 64);
			if(lane == 0) prevP = -1;
			const int cP = cL >= 0 ? 2 * cL + cQ : -1;
			if(cP > prevP) prevP = cP;
			// subtract the qualifying intervals ending at this lane's labels
			{
				int prev = prevL, qprev = prevP >= 0 ? (prevP & 1) : 0;
				for(uint32_t x = d; x;) {
					const int k = __clz(x);
					x &= ~(0x80000000u >> k);
					const int cur = 32 * w + k + 1;
					const int qc = prev >= 0 && cur - prev <= proxi;
					if(qc) {
						uint32_t rm, rd;
						range_counts(A, B, W32, prev, cur, rm, rd);
						cnt -= rm;
						dist -= rd;
						if(qprev) {
							range_counts(A, B, W32, prev, prev, rm, rd);
							cnt += rm;
							dist += rd;
						}
					}
					prev = cur;
					qprev = qc;
				}
			}
			const int top = __shfl(incl2, 63, 64);
			if(top >= 0 && (top >> 1) > cL) {
				cL = top >> 1;
				cQ = top & 1;
			}
		}
		// the highest SNP against the sentinel lastSNP = len + proxi (fsacmp.c:367)
		if(lane == 0 && cL >= 0 && (long long) len + proxi - cL <= proxi) {
			uint32_t rm, rd;
			const long long e = (long long) len + proxi;
			range_counts(A, B, W32, cL, e < 32LL * W32 ? (int) e : 32 * W32 - 1, rm, rd);
			cnt -= rm;
			dist -= rd;
			if(cQ) {
				range_counts(A, B, W32, cL, cL, rm, rd);
				cnt += rm;
				dist += rd;
			}
		}
#pragma unroll
		for(int o = 32; o > 0; o >>= 1) {
			dist += __shfl_xor(dist, o, 64);
			cnt += __shfl_xor(cnt, o, 64);
		}
		if(lane == 0) pair_store<ET>(D, Nm, f, (uint32_t) dist, (uint32_t) cnt, norm, minLength, bs);
	}
}

// ------------------------------------------------------------------ host
static inline long long cdivll(long long a, long long b) { return (a + b - 1) / b; }

// the non-pair dist kernel: 2 = k_snp_mfma2 (256 x 256 tiles, default),
// 1 = k_snp_mfma (128 x 128), 0 = the VALU tiles (CCG_DIST_MFMA)
static int dist_kernel_choice() {
	const char *mf = getenv("CCG_DIST_MFMA");
	return mf ? atoi(mf) : 2;
}

// k_snp_mfma2 over the LT rows [rb, re) (world == 0) or over one rank's rows
// of the band layout (world > 0), with split-K over word slices when the
// tiles do not fill the chip (one block per CU) or a row exceeds the
// f32-exact slice, counts finished by k_snp_finish
template <int ET, bool PAIR = false>
static int snp_launch_mfma2(ccg_ctx *ctx, const ccg_snp_args *a, const void *planes, int Wp, double nFactor, void *D,
                            long long rb, long long re, int rank, int world, void *N = NULL) {
	typedef typename Elem<ET>::T T;
	const long long n = a->n;
	long long t_begin = 0, t_end = 0, f0 = 0, f1 = 0;
	int npanels = 0;
	long long *d_pfx = NULL;
	if(world > 0) {
		const long long nb = (n + SB - 1) / SB;
		long long nloc = 0;   // owned rows below n
		if(rank < nb) {
			const long long owned = (nb - 1 - rank) / world + 1, last = (owned - 1) * world + rank;
			nloc = (owned - 1) * SB + (n - last * SB < SB ? n - last * SB : SB);
		}
		npanels = (int) cdivll(nloc, TILE2);
		if(npanels == 0) return CCG_OK;
		std::vector<long long> pfx(npanels + 1, 0);
		for(long long I = 0; I < npanels; ++I) {
			const long long Lmax = (I + 1) * TILE2 - 1 < nloc - 1 ? (I + 1) * TILE2 - 1 : nloc - 1;
			const long long lb = Lmax / SB, rmax = (lb * world + rank) * SB + (Lmax - lb * SB);
			pfx[I + 1] = pfx[I] + cdivll(rmax, TILE2);
		}
		CCG_CHECK(hipMalloc(&d_pfx, (size_t) (npanels + 1) * sizeof(long long)));
		if(hipMemcpyAsync(d_pfx, pfx.data(), (size_t) (npanels + 1) * sizeof(long long), hipMemcpyHostToDevice,
		                  ctx->stream) != hipSuccess) {
			hipFree(d_pfx);
			return CCG_EHIP;
		}
		t_end = pfx[npanels];
		f1 = ccg_shard_elems(n, rank, world);
	} else {
		const long long Ilo = rb / TILE2, Ihi = (re - 1) / TILE2;
		t_begin = Ilo * (Ilo + 1) / 2;
		t_end = (Ihi + 1) * (Ihi + 2) / 2;
		f0 = tri(rb);
		f1 = tri(re);
	}
	if(PAIR) {   // pair mode: items are tile column halves
		t_begin *= 2;
		t_end *= 2;
	}
	const long long tiles = t_end - t_begin;
	hipDeviceProp_t prop;
	if(hipGetDeviceProperties(&prop, ctx->device) != hipSuccess) {
		hipFree(d_pfx);
		return CCG_EHIP;
	}
	const long long slots = prop.multiProcessorCount;   // one block per CU
	// words per LDS chunk (CCG_DIST_KC=16: half the barriers, 133 KB of LDS)
	// and the tile order (CCG_DIST_ORDER=1: super-tiles, whole LT ranges from
	// a super-row start only)
	const char *kce = getenv("CCG_DIST_KC"), *ore = getenv("CCG_DIST_ORDER");
	const int kc = !PAIR && kce && atoi(kce) == KC2L && Wp % KC2L == 0 ? KC2L : KC2;
	// the LDS-DMA staged kernel (CCG_DIST_GLDS=0: k_snp_mfma2)
	const char *gle = getenv("CCG_DIST_GLDS");
	const bool glds = !PAIR && !(gle && atoi(gle) == 0) && kc == KC3;
	const int sorder = !PAIR && world == 0 && ore && atoi(ore) == 1 && (rb / TILE2) % 4 == 0;
	const int chunks = Wp / kc;
	int S = 1;
	if(tiles < 16 * slots) {
		S = (int) cdivll(16 * slots, tiles);
		if(S > chunks / 4) S = chunks / 4;
		if(S < 1) S = 1;
	}
	int Wk = (int) cdivll(chunks, S) * kc;
	if(Wk > MFMA_KMAX) Wk = (MFMA_KMAX / kc) * kc;
	S = (int) cdivll(Wp, Wk);
	const long long batch = 1 << 16;
	unsigned *cnt = NULL;
	int rc = CCG_OK;
	// every failure below leaves through `out`, which frees d_pfx and cnt
#define MF2_TRY(x) do { if((x) != hipSuccess) { rc = CCG_EHIP; goto out; } } while(0)
	if(S > 1) {   // pair mode: dist counts, then n counts
		const size_t cz = (size_t) (f1 - f0) * (PAIR ? 2 : 1) * sizeof(unsigned);
		if(hipMalloc(&cnt, cz) != hipSuccess) {
			cnt = NULL;
			rc = CCG_ENOMEM;
			goto out;
		}
		MF2_TRY(hipMemsetAsync(cnt, 0, cz, ctx->stream));
	}
	for(long long t = t_begin * S; t < t_end * S; t += batch) {
		const long long items = t_end * S - t < batch ? t_end * S - t : batch;
		const uint2 *pl = (const uint2 *) planes;
		if(PAIR) {
			typedef typename Elem<ET>::T T;
			const uint4 *pp = (const uint4 *) planes;
			unsigned *cn = cnt ? cnt + (f1 - f0) : NULL;
			T *Nn = world > 0 ? NULL : (T *) N;
			if(world > 0 && S > 1)
				k_snp_mfma2_pair<ET, true, true><<<(unsigned) items, 256, 0, ctx->stream>>>(
				    pp, Wp, (int) n, t, items, S, Wk, a->norm, a->minLength, a->byteScale, (T *) D, Nn, 0, n, cnt, cn, 0,
				    d_pfx, npanels, rank, world);
			else if(world > 0)
				k_snp_mfma2_pair<ET, false, true><<<(unsigned) items, 256, 0, ctx->stream>>>(
				    pp, Wp, (int) n, t, items, 1, Wp, a->norm, a->minLength, a->byteScale, (T *) D, Nn, 0, n, cnt, cn, 0,
				    d_pfx, npanels, rank, world);
			else if(S > 1)
				k_snp_mfma2_pair<ET, true, false><<<(unsigned) items, 256, 0, ctx->stream>>>(
				    pp, Wp, (int) n, t, items, S, Wk, a->norm, a->minLength, a->byteScale, (T *) D, Nn, rb, re, cnt, cn,
				    f0, NULL, 0, 0, 1);
			else
				k_snp_mfma2_pair<ET, false, false><<<(unsigned) items, 256, 0, ctx->stream>>>(
				    pp, Wp, (int) n, t, items, 1, Wp, a->norm, a->minLength, a->byteScale, (T *) D, Nn, rb, re, cnt, cn,
				    f0, NULL, 0, 0, 1);
			MF2_TRY(hipGetLastError());
			continue;
		}
#define MF2_LAUNCH(KCV)                                                                                              \
	if(world > 0) {                                                                                                  \
		if(S > 1)                                                                                                    \
			k_snp_mfma2<ET, true, true, KCV><<<(unsigned) items, 256, 0, ctx->stream>>>(                             \
			    pl, Wp, (int) n, t, items, S, Wk, nFactor, a->byteScale, (T *) D, 0, n, cnt, 0, d_pfx, npanels, rank,  \
			    world, 0);                                                                                           \
		else                                                                                                         \
			k_snp_mfma2<ET, false, true, KCV><<<(unsigned) items, 256, 0, ctx->stream>>>(                            \
			    pl, Wp, (int) n, t, items, 1, Wp, nFactor, a->byteScale, (T *) D, 0, n, cnt, 0, d_pfx, npanels, rank,  \
			    world, 0);                                                                                           \
	} else {                                                                                                         \
		if(S > 1)                                                                                                    \
			k_snp_mfma2<ET, true, false, KCV><<<(unsigned) items, 256, 0, ctx->stream>>>(                            \
			    pl, Wp, (int) n, t, items, S, Wk, nFactor, a->byteScale, (T *) D, rb, re, cnt, f0, NULL, 0, 0, 1,       \
			    sorder);                                                                                             \
		else                                                                                                         \
			k_snp_mfma2<ET, false, false, KCV><<<(unsigned) items, 256, 0, ctx->stream>>>(                           \
			    pl, Wp, (int) n, t, items, 1, Wp, nFactor, a->byteScale, (T *) D, rb, re, cnt, f0, NULL, 0, 0, 1,       \
			    sorder);                                                                                             \
	}
		if(glds) {   // k_snp_mfma3 (KC3-word chunks, LDS-DMA staged)
			if(world > 0) {
				if(S > 1)
					k_snp_mfma3<ET, true, true><<<(unsigned) items, 256, 0, ctx->stream>>>(
					    pl, Wp, (int) n, t, items, S, Wk, nFactor, a->byteScale, (T *) D, 0, n, cnt, 0, d_pfx, npanels,
					    rank, world, 0);
				else
					k_snp_mfma3<ET, false, true><<<(unsigned) items, 256, 0, ctx->stream>>>(
					    pl, Wp, (int) n, t, items, 1, Wp, nFactor, a->byteScale, (T *) D, 0, n, cnt, 0, d_pfx, npanels,
					    rank, world, 0);
			} else {
				if(S > 1)
					k_snp_mfma3<ET, true, false><<<(unsigned) items, 256, 0, ctx->stream>>>(
					    pl, Wp, (int) n, t, items, S, Wk, nFactor, a->byteScale, (T *) D, rb, re, cnt, f0, NULL, 0, 0, 1,
					    sorder);
				else
					k_snp_mfma3<ET, false, false><<<(unsigned) items, 256, 0, ctx->stream>>>(
					    pl, Wp, (int) n, t, items, 1, Wp, nFactor, a->byteScale, (T *) D, rb, re, cnt, f0, NULL, 0, 0, 1,
					    sorder);
			}
		} else if(kc == KC2L) {
			MF2_LAUNCH(KC2L)
		} else {
			MF2_LAUNCH(KC2)
		}
#undef MF2_LAUNCH
		MF2_TRY(hipGetLastError());
	}
	if(S > 1) {
		const long long g = cdivll(f1 - f0, 256);
		if(PAIR)
			k_snp_pair_finish<ET><<<(unsigned) (g < 65536 ? g : 65536), 256, 0, ctx->stream>>>(
			    cnt, cnt + (f1 - f0), f0, f1, a->norm, a->minLength, a->byteScale, (T *) D,
			    world > 0 ? (T *) NULL : (T *) N);
		else
			k_snp_finish<ET><<<(unsigned) (g < 65536 ? g : 65536), 256, 0, ctx->stream>>>(cnt, f0, f0, f1, nFactor,
			                                                                                a->byteScale, (T *) D);
		MF2_TRY(hipGetLastError());
	}
	MF2_TRY(hipStreamSynchronize(ctx->stream));
out:
#undef MF2_TRY
	if(rc != CCG_OK) hipStreamSynchronize(ctx->stream);   // no launch may still read cnt / d_pfx
	if(cnt && hipFree(cnt) != hipSuccess && rc == CCG_OK) rc = CCG_EHIP;
	if(d_pfx && hipFree(d_pfx) != hipSuccess && rc == CCG_OK) rc = CCG_EHIP;
	return rc;
}

template <int ET>
static int snp_launch(ccg_ctx *ctx, const ccg_snp_args *a, const void *planes, int Wp, double nFactor, void *D, void *N,
                      long long rb, long long re) {
	typedef typename Elem<ET>::T T;
	long long Ilo = rb / TILE, Ihi = (re - 1) / TILE;   // tile rows touching [rb, re)
	long long t_begin = Ilo * (Ilo + 1) / 2, t_end = (Ihi + 1) * (Ihi + 2) / 2;
	const long long batch = 1 << 14;
	if(a->pair && a->proxi) {
		const long long f0 = tri(rb), f1 = tri(re), g = cdivll(f1 - f0, 4);
		const int W32 = (a->len + 31) / 32;
		if(f1 > f0) {
			k_snp_pair_proxi<ET><<<(unsigned) (g < 16384 ? g : 16384), 256, 0, ctx->stream>>>(
			    (const uint4 *) planes, Wp, W32, a->len, (int) a->proxi, f0, f1, a->norm, a->minLength, a->byteScale,
			    (T *) D, (T *) N);
			CCG_CHECK(hipGetLastError());
		}
		return CCG_OK;
	}
	// split-K: enough (tile, slice) items that the tail round of resident
	// blocks (2 per CU) is small; each slice keeps >= 4 chunks
	hipDeviceProp_t prop;
	CCG_CHECK(hipGetDeviceProperties(&prop, ctx->device));
	const long long slots = 2LL * prop.multiProcessorCount;
	const long long tiles = t_end - t_begin;
	const int kc = a->pair ? KCP : KC;
	const int chunks = Wp / kc;
	int S = 1;
	if(tiles < 16 * slots) {
		S = (int) cdivll(16 * slots, tiles);
		if(S > chunks / 4) S = chunks / 4;
		if(S < 1) S = 1;
	}
	const int Wk = (int) cdivll(chunks, S) * kc;
	S = (int) cdivll(Wp, Wk);
	const long long f0 = tri(rb), f1 = tri(re);
	const long long i_begin = t_begin * S, i_end = t_end * S;
	if(a->pair && dist_kernel_choice() == 2)   // k_snp_mfma2_pair (CCG_DIST_MFMA=1: k_snp_mfma_pair, 0: VALU tiles)
		return snp_launch_mfma2<ET, true>(ctx, a, planes, Wp, nFactor, D, rb, re, 0, 0, N);
	if(a->pair) {
		unsigned *cd = NULL, *cn = NULL;
		if(S > 1) {
			CCG_CHECK(hipMalloc(&cd, (size_t) (f1 - f0) * 2 * sizeof(unsigned)));
			cn = cd + (f1 - f0);
			CCG_CHECK(hipMemsetAsync(cd, 0, (size_t) (f1 - f0) * 2 * sizeof(unsigned), ctx->stream));
		}
		// the MFMA form (default; CCG_DIST_MFMA=0: VALU tiles) while a slice is f32-exact
		const char *mfp = getenv("CCG_DIST_MFMA");
		const bool pmfma = (mfp ? atoi(mfp) : 1) && Wk < MFMA_KMAX;
		for(long long t = i_begin; t < i_end; t += batch) {
			long long items = i_end - t < batch ? i_end - t : batch;
			if(pmfma) {
				if(S > 1)
					k_snp_mfma_pair<ET, true><<<(unsigned) items, 256, 0, ctx->stream>>>(
					    (const uint4 *) planes, Wp, a->n, t, items, S, Wk, a->norm, a->minLength, a->byteScale, (T *) D,
					    (T *) N, rb, re, cd, cn, f0);
				else
					k_snp_mfma_pair<ET, false><<<(unsigned) items, 256, 0, ctx->stream>>>(
					    (const uint4 *) planes, Wp, a->n, t, items, 1, Wp, a->norm, a->minLength, a->byteScale, (T *) D,
					    (T *) N, rb, re, cd, cn, f0);
			} else if(S > 1) {
				k_snp_tile_pair<ET, true><<<(unsigned) items, 256, 0, ctx->stream>>>(
				    (const uint4 *) planes, Wp, a->n, t, items, S, Wk, a->norm, a->minLength, a->byteScale, (T *) D,
				    (T *) N, rb, re, cd, cn, f0);
			} else {
				k_snp_tile_pair<ET, false><<<(unsigned) items, 256, 0, ctx->stream>>>(
				    (const uint4 *) planes, Wp, a->n, t, items, 1, Wp, a->norm, a->minLength, a->byteScale, (T *) D,
				    (T *) N, rb, re, cd, cn, f0);
			}
			CCG_CHECK(hipGetLastError());
		}
		if(S > 1) {
			long long g = cdivll(f1 - f0, 256);
			k_snp_pair_finish<ET><<<(unsigned) (g < 65536 ? g : 65536), 256, 0, ctx->stream>>>(
			    cd, cn, f0, f1, a->norm, a->minLength, a->byteScale, (T *) D, (T *) N);
			CCG_CHECK(hipGetLastError());
			CCG_CHECK(hipStreamSynchronize(ctx->stream));
			CCG_CHECK(hipFree(cd));
		}
		return CCG_OK;
	}
	// MFMA forms (k_snp_mfma3 / k_snp_mfma2 the default, k_snp_mfma with CCG_DIST_MFMA=1,
	// the VALU tiles with 0): f32-exact while a slice holds < MFMA_KMAX words
	if(dist_kernel_choice() == 2) return snp_launch_mfma2<ET>(ctx, a, planes, Wp, nFactor, D, rb, re, 0, 0);
	const int use_mfma = dist_kernel_choice();
	int Sm = S, Wkm = Wk;
	if(use_mfma && Wkm > MFMA_KMAX) {
		Wkm = (MFMA_KMAX / kc) * kc;
		Sm = (int) cdivll(Wp, Wkm);
	}
	if(use_mfma) {
		S = Sm;
	}
	const long long mi_begin = t_begin * S, mi_end = t_end * S;
	unsigned *cnt = NULL;
	if(S > 1) {
		CCG_CHECK(hipMalloc(&cnt, (size_t) (f1 - f0) * sizeof(unsigned)));
		CCG_CHECK(hipMemsetAsync(cnt, 0, (size_t) (f1 - f0) * sizeof(unsigned), ctx->stream));
	}
	for(long long t = use_mfma ? mi_begin : i_begin; t < (use_mfma ? mi_end : i_end); t += batch) {
		const long long iend = use_mfma ? mi_end : i_end;
		long long items = iend - t < batch ? iend - t : batch;
		if(use_mfma) {
			if(S > 1)
				k_snp_mfma<ET, true><<<(unsigned) items, 256, 0, ctx->stream>>>((const uint2 *) planes, Wp, a->n, t, items,
				                                                             S, Wkm, nFactor, a->byteScale, (T *) D, rb,
				                                                             re, cnt, f0);
			else
				k_snp_mfma<ET, false><<<(unsigned) items, 256, 0, ctx->stream>>>((const uint2 *) planes, Wp, a->n, t,
				                                                              items, 1, Wp, nFactor, a->byteScale,
				                                                              (T *) D, rb, re, cnt, f0);
		} else if(S > 1) {
			k_snp_tile<ET, true><<<(unsigned) items, 256, 0, ctx->stream>>>((const uint2 *) planes, Wp, a->n, t, items, S,
			                                                             Wk, nFactor, a->byteScale, (T *) D, rb, re,
			                                                             cnt, f0);
		} else {
			k_snp_tile<ET, false><<<(unsigned) items, 256, 0, ctx->stream>>>((const uint2 *) planes, Wp, a->n, t, items,
			                                                              1, Wp, nFactor, a->byteScale, (T *) D, rb,
			                                                              re, cnt, f0);
		}
		CCG_CHECK(hipGetLastError());
	}
	if(S > 1) {
		long long g = cdivll(f1 - f0, 256);
		k_snp_finish<ET><<<(unsigned) (g < 65536 ? g : 65536), 256, 0, ctx->stream>>>(cnt, f0, f0, f1, nFactor,
		                                                                                a->byteScale, (T *) D);
		CCG_CHECK(hipGetLastError());
		CCG_CHECK(hipStreamSynchronize(ctx->stream));
		CCG_CHECK(hipFree(cnt));
	}
	return CCG_OK;
}

// the rank's owned rows of the band layout, in its own order: panels of TILE
// owned rows, each against the column tiles below its last row
template <int ET>
static int snp_launch_band(ccg_ctx *ctx, const ccg_snp_args *a, const void *planes, int Wp, double nFactor, void *D,
                           int rank, int world) {
	typedef typename Elem<ET>::T T;
	const long long n = a->n;
	auto row_of = [&](long long L) {
		const long long lb = L / SB;
		return (lb * world + rank) * SB + (L - lb * SB);
	};
	long long nloc = 0;   // owned rows below n
	const long long nb = (n + SB - 1) / SB;
	if(rank < nb) {
		const long long owned = (nb - 1 - rank) / world + 1, last = (owned - 1) * world + rank;
		nloc = (owned - 1) * SB + (n - last * SB < SB ? n - last * SB : SB);
	}
	if(a->pair && a->proxi) {
		// maskProxi pairs: an owned band's rows are contiguous in both the full
		// LT and the rank's buffer with the same relative offsets, so each run of
		// consecutive owned bands is k_snp_pair_proxi over its LT range with D
		// shifted by off(first row) - tri(first row)
		const int W32 = (a->len + 31) / 32;
		const Shard sh{rank, world};
		for(long long g = rank; g < nb;) {
			long long g2 = g;
			while(world == 1 && g2 + 1 < nb) ++g2;   // world 1 owns every band
			const long long r0 = g * SB, r1 = (g2 + 1) * SB < n ? (g2 + 1) * SB : n;
			const long long f0 = tri(r0), f1 = tri(r1), gr = cdivll(f1 - f0, 4);
			T *Dg = (T *) D + (sh.off(r0) - f0);
			if(f1 > f0) {
				k_snp_pair_proxi<ET><<<(unsigned) (gr < 16384 ? gr : 16384), 256, 0, ctx->stream>>>(
				    (const uint4 *) planes, Wp, W32, a->len, (int) a->proxi, f0, f1, a->norm, a->minLength,
				    a->byteScale, Dg, (T *) NULL);
				CCG_CHECK(hipGetLastError());
			}
			g = g2 + world;
		}
		CCG_CHECK(hipStreamSynchronize(ctx->stream));
		return CCG_OK;
	}
	// tiles per panel (column tiles with a cell j < i), prefix-summed so that a
	// launch spans many panels and fills the chip
	const int npanels = (int) cdivll(nloc, TILE);
	if(npanels == 0) return CCG_OK;
	std::vector<long long> pfx(npanels + 1, 0);
	for(long long I = 0; I < npanels; ++I) {
		const long long Lmax = (I + 1) * TILE - 1 < nloc - 1 ? (I + 1) * TILE - 1 : nloc - 1;
		pfx[I + 1] = pfx[I] + cdivll(row_of(Lmax), TILE);
	}
	long long *d_pfx = NULL;
	CCG_CHECK(hipMalloc(&d_pfx, (size_t) (npanels + 1) * sizeof(long long)));
	CCG_CHECK(hipMemcpyAsync(d_pfx, pfx.data(), (size_t) (npanels + 1) * sizeof(long long), hipMemcpyHostToDevice,
	                         ctx->stream));
	const long long total = pfx[npanels], batch = 1 << 16;
	// the MFMA form unless disabled (CCG_DIST_MFMA=0); a row longer than the
	// f32-exact slice is split over word slices
	const char *mf = getenv("CCG_DIST_MFMA");
	if(a->pair && dist_kernel_choice() == 2) {
		CCG_CHECK(hipFree(d_pfx));
		return snp_launch_mfma2<ET, true>(ctx, a, planes, Wp, nFactor, D, 0, n, rank, world);
	}
	if(a->pair) {
		// fsacmpair per cell, the pair tiles in the band form; split-K over word
		// slices (as snp_launch) when the rank's tiles do not fill the chip, the
		// u32 counts indexed by local element and finished in place
		hipDeviceProp_t prop;
		CCG_CHECK(hipGetDeviceProperties(&prop, ctx->device));
		const long long slots = 2LL * prop.multiProcessorCount;
		const int chunks = Wp / KCP;
		int S = 1;
		if(total < 16 * slots) {
			S = (int) cdivll(16 * slots, total);
			if(S > chunks / 4) S = chunks / 4;
			if(S < 1) S = 1;
		}
		const int Wk = (int) cdivll(chunks, S) * KCP;
		S = (int) cdivll(Wp, Wk);
		const bool pm = (mf ? atoi(mf) : 1) && Wk < MFMA_KMAX;
		const long long elems = ccg_shard_elems(n, rank, world);
		unsigned *cd = NULL, *cn = NULL;
		if(S > 1) {
			CCG_CHECK(hipMalloc(&cd, (size_t) elems * 2 * sizeof(unsigned)));
			cn = cd + elems;
			CCG_CHECK(hipMemsetAsync(cd, 0, (size_t) elems * 2 * sizeof(unsigned), ctx->stream));
		}
		for(long long t = 0; t < total * S; t += batch) {
			const long long items = total * S - t < batch ? total * S - t : batch;
			if(pm && S > 1)
				k_snp_mfma_pair<ET, true, true><<<(unsigned) items, 256, 0, ctx->stream>>>(
				    (const uint4 *) planes, Wp, (int) n, t, items, S, Wk, a->norm, a->minLength, a->byteScale, (T *) D,
				    (T *) NULL, 0, n, cd, cn, 0, d_pfx, npanels, rank, world);
			else if(pm)
				k_snp_mfma_pair<ET, false, true><<<(unsigned) items, 256, 0, ctx->stream>>>(
				    (const uint4 *) planes, Wp, (int) n, t, items, 1, Wp, a->norm, a->minLength, a->byteScale, (T *) D,
				    (T *) NULL, 0, n, NULL, NULL, 0, d_pfx, npanels, rank, world);
			else if(S > 1)
				k_snp_tile_pair<ET, true, true><<<(unsigned) items, 256, 0, ctx->stream>>>(
				    (const uint4 *) planes, Wp, (int) n, t, items, S, Wk, a->norm, a->minLength, a->byteScale, (T *) D,
				    (T *) NULL, 0, n, cd, cn, 0, d_pfx, npanels, rank, world);
			else
				k_snp_tile_pair<ET, false, true><<<(unsigned) items, 256, 0, ctx->stream>>>(
				    (const uint4 *) planes, Wp, (int) n, t, items, 1, Wp, a->norm, a->minLength, a->byteScale, (T *) D,
				    (T *) NULL, 0, n, NULL, NULL, 0, d_pfx, npanels, rank, world);
			CCG_CHECK(hipGetLastError());
		}
		if(S > 1) {
			const long long g = cdivll(elems, 256);
			k_snp_pair_finish<ET><<<(unsigned) (g < 65536 ? g : 65536), 256, 0, ctx->stream>>>(
			    cd, cn, 0, elems, a->norm, a->minLength, a->byteScale, (T *) D, (T *) NULL);
			CCG_CHECK(hipGetLastError());
		}
		CCG_CHECK(hipStreamSynchronize(ctx->stream));
		if(cd) CCG_CHECK(hipFree(cd));
		CCG_CHECK(hipFree(d_pfx));
		return CCG_OK;
	}
	if(dist_kernel_choice() == 2) {
		CCG_CHECK(hipFree(d_pfx));
		return snp_launch_mfma2<ET>(ctx, a, planes, Wp, nFactor, D, 0, n, rank, world);
	}
	if(mf ? atoi(mf) : 1) {
		// the MFMA form with snp_launch's split-K over word slices when the
		// rank's tiles do not fill the chip, or when a row exceeds the f32-exact
		// slice length; u32 counts by local element, k_snp_finish in place
		hipDeviceProp_t prop;
		CCG_CHECK(hipGetDeviceProperties(&prop, ctx->device));
		const long long slots = 2LL * prop.multiProcessorCount;
		const int chunks = Wp / KC;
		int S = 1;
		if(total < 16 * slots) {
			S = (int) cdivll(16 * slots, total);
			if(S > chunks / 4) S = chunks / 4;
			if(S < 1) S = 1;
		}
		int Wk = (int) cdivll(chunks, S) * KC;
		if(Wk > MFMA_KMAX) Wk = (MFMA_KMAX / KC) * KC;
		S = (int) cdivll(Wp, Wk);
		const long long elems = ccg_shard_elems(n, rank, world);
		unsigned *cnt = NULL;
		if(S > 1) {
			CCG_CHECK(hipMalloc(&cnt, (size_t) elems * sizeof(unsigned)));
			CCG_CHECK(hipMemsetAsync(cnt, 0, (size_t) elems * sizeof(unsigned), ctx->stream));
		}
		for(long long t = 0; t < total * S; t += batch) {
			const long long items = total * S - t < batch ? total * S - t : batch;
			if(S > 1)
				k_snp_mfma_band<ET, true><<<(unsigned) items, 256, 0, ctx->stream>>>(
				    (const uint2 *) planes, Wp, (int) n, d_pfx, npanels, t, items, nFactor, a->byteScale, (T *) D, rank,
				    world, S, Wk, cnt);
			else
				k_snp_mfma_band<ET><<<(unsigned) items, 256, 0, ctx->stream>>>((const uint2 *) planes, Wp, (int) n,
				                                                             d_pfx, npanels, t, items, nFactor,
				                                                             a->byteScale, (T *) D, rank, world);
			CCG_CHECK(hipGetLastError());
		}
		if(S > 1) {
			const long long g = cdivll(elems, 256);
			k_snp_finish<ET><<<(unsigned) (g < 65536 ? g : 65536), 256, 0, ctx->stream>>>(cnt, 0, 0, elems, nFactor,
			                                                                                a->byteScale, (T *) D);
			CCG_CHECK(hipGetLastError());
		}
		CCG_CHECK(hipStreamSynchronize(ctx->stream));
		if(cnt) CCG_CHECK(hipFree(cnt));
		CCG_CHECK(hipFree(d_pfx));
		return CCG_OK;
	}
	for(long long t = 0; t < total; t += batch) {
		const long long items = total - t < batch ? total - t : batch;
		k_snp_tile_band<ET><<<(unsigned) items, 256, 0, ctx->stream>>>((const uint2 *) planes, Wp, (int) n, d_pfx,
			                                                             npanels, t, items, nFactor, a->byteScale, (T *) D,
			                                                             rank, world);
		CCG_CHECK(hipGetLastError());
	}
	CCG_CHECK(hipStreamSynchronize(ctx->stream));
	CCG_CHECK(hipFree(d_pfx));
	return CCG_OK;
}

static int snp_run(ccg_ctx *ctx, const ccg_snp_args *a, void *D, void *N, int *inc_out, int rank, int world,
                   bool host_in);

int ccg_snp_dev_impl(ccg_ctx *ctx, const ccg_snp_args *a, void *D, void *N, int *inc_out, bool host_in) {
	return snp_run(ctx, a, D, N, inc_out, 0, 0, host_in);
}

int ccg_snp_shard_dev_impl(ccg_ctx *ctx, const ccg_snp_args *a, int rank, int world, void *Dloc, int *inc_out,
                           bool host_in) {
	if(!a || world < 1 || rank < 0 || rank >= world) return CCG_EINVAL;
	if(a->row_begin || a->row_end) return CCG_EINVAL;
	return snp_run(ctx, a, Dloc, NULL, inc_out, rank, world, host_in);
}

// the bit planes of every taxon.  host_in: a->seqs / a->incs are host memory,
// streamed through a bounded staging buffer, so HBM holds the planes and the
// LT only (configs[4]: 25 GB of planes beside a 250 GB shard, where a device
// copy of the packed MSA would add another 25 GB).  *mask = the device copy of
// the non-pair include mask (k_popsum reads it), or NULL.
static int snp_planes(ccg_ctx *ctx, const ccg_snp_args *a, int W32, int Wp, void *planes, bool host_in,
                      uint32_t **mask, const int *widx) {
	*mask = NULL;
	if(!host_in) {
		const long long total = (long long) a->n * Wp, pg = cdivll(total, 256);
		k_planes<<<(unsigned) (pg < 262144 ? pg : 262144), 256, 0, ctx->stream>>>(
		    a->seqs, a->incs, a->n, a->stride, W32, Wp, a->pair, (uint2 *) planes, (uint4 *) planes, widx);
		CCG_CHECK(hipGetLastError());
		return CCG_OK;
	}
	const size_t row_b = (size_t) a->stride * 8 + (a->pair ? (size_t) a->stride * 4 : 0);
	long long R = (long long) (((size_t) 256 << 20) / row_b);
	if(R < 1) R = 1;
	if(R > a->n) R = a->n;
	void *stage = NULL;
	CCG_CHECK(hipMalloc(&stage, (size_t) R * row_b));
	if(!a->pair) {
		if(hipMalloc((void **) mask, (size_t) a->stride * 4) != hipSuccess) {
			hipFree(stage);
			*mask = NULL;
			return CCG_ENOMEM;
		}
		if(hipMemcpyAsync(*mask, a->incs, (size_t) a->stride * 4, hipMemcpyHostToDevice, ctx->stream) != hipSuccess) {
			hipFree(stage);
			hipFree(*mask);
			*mask = NULL;
			return CCG_EHIP;
		}
	}
	uint64_t *sseq = (uint64_t *) stage;
	uint32_t *sinc = (uint32_t *) ((char *) stage + (size_t) R * a->stride * 8);
	int rc = CCG_OK;
	for(long long t0 = 0; t0 < a->n && rc == CCG_OK; t0 += R) {
		const long long rows = a->n - t0 < R ? a->n - t0 : R;
		// stream-ordered: the copy into the stage waits for the previous chunk's k_planes
		if(hipMemcpyAsync(sseq, a->seqs + (size_t) t0 * a->stride, (size_t) rows * a->stride * 8,
		                  hipMemcpyHostToDevice, ctx->stream) != hipSuccess ||
		   (a->pair && hipMemcpyAsync(sinc, a->incs + (size_t) t0 * a->stride, (size_t) rows * a->stride * 4,
		                              hipMemcpyHostToDevice, ctx->stream) != hipSuccess)) {
			rc = CCG_EHIP;
			break;
		}
		const long long pg = cdivll(rows * Wp, 256);
		k_planes<<<(unsigned) (pg < 262144 ? pg : 262144), 256, 0, ctx->stream>>>(
		    sseq, a->pair ? sinc : *mask, (int) rows, a->stride, W32, Wp, a->pair, (uint2 *) planes + t0 * Wp,
		    (uint4 *) planes + t0 * Wp, widx);
		if(hipGetLastError() != hipSuccess) rc = CCG_EHIP;
	}
	hipStreamSynchronize(ctx->stream);
	hipFree(stage);
	return rc;
}

static int snp_run(ccg_ctx *ctx, const ccg_snp_args *a, void *D, void *N, int *inc_out, int rank, int world,
                   bool host_in) {
	if(!a || a->n < 0 || a->len <= 0 || a->stride < (a->len + 31) / 32) return CCG_EINVAL;
	if(a->etype != 8 && a->etype != 4 && a->etype != 2 && a->etype != 1) return CCG_EINVAL;
	if(a->n < 2) {
		if(inc_out && !a->pair && host_in) {
			int s = 0;
			for(int w = 0; w < (a->len + 31) / 32; ++w) s += __builtin_popcount(a->incs[w]);
			*inc_out = s;
		} else if(inc_out && !a->pair) {
			int *d_inc;
			CCG_CHECK(hipMalloc(&d_inc, sizeof(int)));
			k_popsum<<<1, 256, 0, ctx->stream>>>(a->incs, (a->len + 31) / 32, d_inc);
			CCG_CHECK(hipMemcpyAsync(inc_out, d_inc, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
			CCG_CHECK(hipStreamSynchronize(ctx->stream));
			CCG_CHECK(hipFree(d_inc));
		}
		return CCG_OK;
	}
	const int W32 = (a->len + 31) / 32;
	const int kc = a->pair ? KCP : KC;
	// Non-pair mode: a word the global mask excludes entirely contributes to
	// no pair (fsacmp.c:552 counts included positions only), so the planes
	// keep only the other words (partial words stay masked); the pair kernels
	// then stream and multiply ~10% fewer words on the headline's alignment.
	// Pair mode's masks are per taxon and stay whole.
	std::vector<int> keep;
	int Wc = W32;
	if(!a->pair) {
		std::vector<uint32_t> hm((size_t) W32);
		if(host_in) std::memcpy(hm.data(), a->incs, (size_t) W32 * 4);
		else {
			CCG_CHECK(hipMemcpyAsync(hm.data(), a->incs, (size_t) W32 * 4, hipMemcpyDeviceToHost, ctx->stream));
			CCG_CHECK(hipStreamSynchronize(ctx->stream));
		}
		for(int w = 0; w < W32; ++w)
			if(hm[w]) keep.push_back(w);
		Wc = (int) keep.size();
		if(Wc == W32 || getenv("CCG_DIST_NOCOMPACT")) {
			keep.clear();
			Wc = W32;
		}
		if(Wc == 0) Wc = 1;   // nothing included: one all-zero word (every count 0)
	}
	const int Wp = (int) (cdivll(Wc, kc) * kc);
	const long long npad = cdivll(a->n, TILE2) * TILE2;   // whole panels of either tile size
	const size_t esz = a->pair ? sizeof(uint4) : sizeof(uint2);
	void *planes = NULL;
	int *d_inc = NULL, *d_widx = NULL;
	// a CCG_CTX_NOSYNC context (a pipeline's dist) keeps its planes in the
	// workspace cache: no hipMalloc / hipFree per matrix (hipFree waits for
	// every stream of the device, the other context's too)
	// (with the small buffers behind them: the count and the word list)
	const bool cached = (ctx->flags & CCG_CTX_NOSYNC) != 0;
	const size_t planes_b = ((size_t) npad * Wp * esz + 255) & ~(size_t) 255;
	auto free_bufs = [&]() {
		if(cached) return;
		hipFree(planes);
		hipFree(d_inc);
		hipFree(d_widx);
	};
	if(cached) {
		const int wrc = ccg_ctx_workspace(ctx, 2, planes_b + 256 + keep.size() * sizeof(int), &planes);
		if(wrc != CCG_OK) return wrc;
		d_inc = (int *) ((char *) planes + planes_b);
		if(!keep.empty()) d_widx = (int *) ((char *) planes + planes_b + 256);
	} else {
		CCG_CHECK(hipMalloc(&planes, planes_b));
		if(hipMalloc(&d_inc, sizeof(int)) != hipSuccess ||
		   (!keep.empty() && hipMalloc(&d_widx, keep.size() * sizeof(int)) != hipSuccess)) {
			hipFree(planes);
			hipFree(d_inc);
			return CCG_ENOMEM;
		}
	}
	uint32_t *mask = NULL;
	int prc = CCG_OK;
	// k_planes writes every word of rows < n: only the padding rows need zeros
	if(hipMemsetAsync((char *) planes + (size_t) a->n * Wp * esz, 0, (size_t) (npad - a->n) * Wp * esz,
	                  ctx->stream) != hipSuccess ||
	   (d_widx && hipMemcpyAsync(d_widx, keep.data(), keep.size() * sizeof(int), hipMemcpyHostToDevice,
	                             ctx->stream) != hipSuccess))
		prc = CCG_EHIP;
	if(!prc) {
		// the compacted word list, or every word (a mask with no included word: one zero word)
		const int *widx = d_widx;
		const int Wsrc = d_widx ? Wc : (a->pair || Wc == W32 ? W32 : 0);
		prc = snp_planes(ctx, a, Wsrc, Wp, planes, host_in, &mask, widx);
	}
	if(prc) {
		hipStreamSynchronize(ctx->stream);
		free_bufs();
		hipFree(mask);
		return prc;
	}
	int inc = 0;
	if(!a->pair) {
		k_popsum<<<1, 1024, 0, ctx->stream>>>(mask ? mask : a->incs, W32, d_inc);
		CCG_CHECK(hipMemcpyAsync(&inc, d_inc, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
		CCG_CHECK(hipStreamSynchronize(ctx->stream));
	}
	if(mask) CCG_CHECK(hipFree(mask));
	if(d_widx && !cached) CCG_CHECK(hipFree(d_widx));
	d_widx = NULL;
	double nFactor = 1.0;
	if(!a->pair && a->norm) {
		nFactor = a->norm;
		nFactor /= inc;   // fsacmpthrd.c:171-176
	}
	long long rb = a->row_begin, re = a->row_end;
	if(rb == 0 && re == 0) re = a->n;
	if(rb < 0 || re > a->n || rb > re) {
		free_bufs();
		return CCG_EINVAL;
	}
	int rc = CCG_OK;
	ctx->dist_ms = 0;
	CCG_CHECK(hipEventRecord(ctx->ev0, ctx->stream));
	if(world > 0) {
		switch(a->etype) {
			case 8: rc = snp_launch_band<8>(ctx, a, planes, Wp, nFactor, D, rank, world); break;
			case 4: rc = snp_launch_band<4>(ctx, a, planes, Wp, nFactor, D, rank, world); break;
			case 2: rc = snp_launch_band<2>(ctx, a, planes, Wp, nFactor, D, rank, world); break;
			default: rc = snp_launch_band<1>(ctx, a, planes, Wp, nFactor, D, rank, world); break;
		}
	} else if(re > rb) {
		switch(a->etype) {
			case 8: rc = snp_launch<8>(ctx, a, planes, Wp, nFactor, D, N, rb, re); break;
			case 4: rc = snp_launch<4>(ctx, a, planes, Wp, nFactor, D, N, rb, re); break;
			case 2: rc = snp_launch<2>(ctx, a, planes, Wp, nFactor, D, N, rb, re); break;
			default: rc = snp_launch<1>(ctx, a, planes, Wp, nFactor, D, N, rb, re); break;
		}
	}
	CCG_CHECK(hipEventRecord(ctx->ev1, ctx->stream));
	CCG_CHECK(hipStreamSynchronize(ctx->stream));
	if(rc == CCG_OK) CCG_CHECK(hipEventElapsedTime(&ctx->dist_ms, ctx->ev0, ctx->ev1));
	if(!cached) {
		CCG_CHECK(hipFree(planes));
		CCG_CHECK(hipFree(d_inc));
	}
	if(inc_out) *inc_out = inc;
	return rc;
}

extern "C" int ccg_last_dist_ms(ccg_ctx *ctx, double *ms) {
	if(!ctx || !ms) return CCG_EINVAL;
	*ms = ctx->dist_ms;
	return CCG_OK;
}

// ------------------------------------------------------------------ Phylip round trip
// `ccphylo dist -W ... | ccphylo tree` passes each cell through text: printphy
// (phy.c:59-123) writes an integral d as "%d" and any other as "%.*f" with -x
// digits, and loadPhy (phy.c:469) reads it back with strtod (then the cast to
// the matrix type).  The fused `dist --tree` stores the same values in place:
// K = round-half-even(d * 10^p) exactly (d * 10^p = hi + lo without error),
// then K / 10^p is one correctly rounded division of exact operands, which is
// strtod's result for the printed decimal.  Cells whose product reaches 2^53
// (more digits than a double carries) set *bad; the caller refuses them.
template <typename T>
__global__ void k_round_decimal(T *__restrict__ D, long long elems, double P, int *__restrict__ bad) {
	for(long long e = (long long) blockIdx.x * blockDim.x + threadIdx.x; e < elems;
	    e += (long long) gridDim.x * blockDim.x) {
		const double x = (double) D[e];
		if(x == trunc(x)) continue;   // "%d" or the integer's exact digits
		const double hi = x * P, lo = fma(x, P, -hi);
		const double ah = fabs(hi);
		if(!(ah < 9007199254740992.0)) {   // K itself may not be a double past 2^53
			atomicOr(bad, 1);
			continue;
		}
		double K;
		if(ah < 4503599627370496.0) {
			K = rint(hi);   // half-even on hi; the exact tie needs lo == 0
			const double d = hi - K;
			if(d == 0.5 && lo > 0) K += 1.0;
			else if(d == -0.5 && lo < 0) K -= 1.0;
		} else {
			// 2^52 <= |hi| < 2^53: hi is an integer and |lo| <= 1/2 (half an
			// ulp), so x P rounds to hi unless lo is an exact tie, which goes
			// to the even neighbour (|K| <= 2^53 stays exact)
			K = hi;
			if(lo == 0.5 || lo == -0.5) {
				const double other = hi + (lo > 0 ? 1.0 : -1.0);
				K = fmod(hi, 2.0) == 0.0 ? hi : other;
			}
		}
		D[e] = (T) (K / P);
	}
}

extern "C" int ccg_round_decimal_dev(ccg_ctx *ctx, void *D, int64_t elems, int etype, int precision) {
	if(!ctx || (!D && elems) || elems < 0 || precision < 0 || precision > 22) return CCG_EINVAL;
	if(etype != 8 && etype != 4) return CCG_EUNSUP;
	CCG_CHECK(hipSetDevice(ctx->device));
	CCG_DEVICE_SYNC(ctx);
	if(!elems) return CCG_OK;
	double P = 1.0;
	for(int k = 0; k < precision; ++k) P *= 10.0;   // exact up to 10^22
	int *d_bad = NULL, bad = 0;
	CCG_CHECK(hipMalloc(&d_bad, sizeof(int)));
	CCG_CHECK(hipMemsetAsync(d_bad, 0, sizeof(int), ctx->stream));
	const long long g = cdivll(elems, 256);
	const unsigned grid = (unsigned) (g < 65536 ? g : 65536);
	if(etype == 8) k_round_decimal<double><<<grid, 256, 0, ctx->stream>>>((double *) D, elems, P, d_bad);
	else k_round_decimal<float><<<grid, 256, 0, ctx->stream>>>((float *) D, elems, P, d_bad);
	CCG_CHECK(hipGetLastError());
	CCG_CHECK(hipMemcpyAsync(&bad, d_bad, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
	CCG_CHECK(hipStreamSynchronize(ctx->stream));
	CCG_CHECK(hipFree(d_bad));
	if(bad) {
		ccg_set_last_msg("ccg_round_decimal_dev: a cell needs more than 15 significant digits at this precision");
		return CCG_EUNSUP;
	}
	return CCG_OK;
}
