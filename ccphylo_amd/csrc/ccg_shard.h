// ccg_shard.h -- the row-sharded LT layout and what the sharded NJ
// (tree_shard.hip) and DNJ (tree_shard_dnj.hip) engines share: ownership and
// offsets, the argmin records, exact initSummaD over gathered column chunks,
// and the collective transport wrapper.
#pragma once
#include <stdio.h>
#include <string.h>
#include "ccg_tree_common.h"

#include "ccg_shard_layout.h"
static_assert(SB == NJ_RB, "a shard band is one NJ argmin row band");

struct ShRec {   // one rank's argmin record (q, flat index); zeros in other ranks' slots
	double q;
	long long f;
};

// q0: the fold's start (NJ's initQ: 1.0; HNJ's minQ: DBL_MAX)
__device__ __forceinline__ void rec_fold(const ShRec *__restrict__ rec, int world, double &bq, long long &bf,
                                         double q0 = 1.0) {
	bq = q0;
	bf = -1;
	for(int w = 0; w < world; ++w) {
		const double q = rec[w].q;
		const long long f = rec[w].f;
		if(f >= 0 && (q < bq || (q == bq && f > bf))) {
			bq = q;
			bf = f;
		}
	}
}

__device__ __forceinline__ void flat_to_ij(long long bf, int &i, int &j) {
	long long r = (long long) ((1.0 + sqrt(1.0 + 8.0 * (double) bf)) * 0.5);
	while(r > 1 && tri(r) > bf) --r;
	while(tri(r + 1) <= bf) ++r;
	i = (int) r;
	j = (int) (bf - tri(r));
}

// ------------------------------------------------------------------ init
// initSummaD row parts of the owned rows (the same wave-serial sum as
// tree.hip's k_init_rows); RP = [n f64 sums][n i32 counts][i32 missing]
template <int ET>
__global__ __launch_bounds__(TB) void k_sh_init_rows(const typename Elem<ET>::T *__restrict__ D, int n, double bs,
                                                     Shard sh, double *__restrict__ rp, int *__restrict__ rc,
                                                     int *__restrict__ miss_out) {
	__shared__ double buf[TB / 64][64];
	const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
	const int k = blockIdx.x * (TB / 64) + wid;
	if(k >= n) return;
	if(!sh.owns(k)) {
		if(lane == 0) {
			rp[k] = 0;
			rc[k] = 0;
		}
		return;
	}
	double s = 0;
	int c = 1, miss = 0;
	const typename Elem<ET>::T *row = D + sh.off(k);
	for(int m0 = 0; m0 < k; m0 += 64) {
		int m = m0 + lane;
		double d = m < k ? Elem<ET>::get(row[m], bs) : 0.0;
		bool ok = m < k && 0 <= d;
		miss |= m < k && !ok;
		c += __popcll(__ballot(ok));
		buf[wid][lane] = ok ? d : 0.0;
		__builtin_amdgcn_wave_barrier();
		if(lane == 0) {
			int lim = k - m0 < 64 ? k - m0 : 64;
			for(int u = 0; u < lim; ++u) s += buf[wid][u];
		}
		__builtin_amdgcn_wave_barrier();
	}
	miss = __any(miss);
	if(lane == 0) {
		rp[k] = s;
		rc[k] = c;
		if(miss) atomicOr(miss_out, 1);
	}
}

// ---- initSummaD's column parts, exact and O(n * world) bytes where possible
// The column part of sD[c] continues the row part s0 serially over
// D(c+1, c), D(c+2, c), ... (nj.c:111-180), and those cells are spread over
// every rank.  Every cell is >= 0 (a negative one makes the matrix "missing",
// which the shards refuse), so the running sum only grows.  If every cell and
// s0 are multiples of 2^G and the total stays below 2^(53+G), every partial
// sum of the serial order is representable: each add is exact and the serial
// result is the exact sum, which any rank can form in any order.  So each
// rank reports, per column, the sum of its own cells, their smallest
// granularity 2^g (lowest set bit) and their count (16 bytes; one allgather
// of n x 16 bytes), and only the columns that fail the test -- typically none
// for integer SNP counts (configs[4]) or float distances -- are gathered
// whole and summed serially (k_sh_pack_cols / k_sh_init_cols, in chunks).

// exponent of the lowest set bit of x > 0 (the granularity of its value)
__device__ __forceinline__ int dbl_gran(double x) {
	const unsigned long long u = (unsigned long long) __double_as_longlong(x);
	const int e = (int) ((u >> 52) & 0x7FF);
	const unsigned long long m = e ? (u & ((1ull << 52) - 1)) | (1ull << 52) : (u & ((1ull << 52) - 1));
	return (e ? e - 1075 : -1074) + __builtin_ctzll(m);
}

// per-rank column statistics, SoA: s[n] (f64 sum of the owned cells >= 0),
// g[n] (u32: 2048 + the smallest granularity exponent; 0xFFFFFFFF when none),
// c[n] (i32 count of the owned cells >= 0)
static __host__ __device__ inline size_t sh_cs_bytes(int n) { return (size_t) n * 16; }

#define CS_CHUNK 32   // owned bands per block (256 rows)
// grid (column tiles of TB, chunks of CS_CHUNK owned bands); block (x, y)
// folds the cells D(m, c), m > c, of its chunk's rows into its TB columns
template <int ET>
__global__ __launch_bounds__(TB) void k_sh_col_stats(const typename Elem<ET>::T *__restrict__ D, int n, double bs,
                                                     Shard sh, double *__restrict__ cs_s, unsigned *__restrict__ cs_g,
                                                     int *__restrict__ cs_c, int *__restrict__ miss_out) {
	const int c0 = blockIdx.x * TB, c = c0 + threadIdx.x;
	const long long lb0 = (long long) blockIdx.y * CS_CHUNK;
	// the chunk's last global row: nothing below the tile's first column + 1
	const long long lbl = lb0 + CS_CHUNK - 1;
	const long long rlast = (lbl * sh.world + sh.rank) * SB + SB - 1;
	if(rlast <= c0 || c >= n) return;
	double s = 0;
	int g = 0x7FFFFFFF, cnt = 0, miss = 0;
	for(int q = 0; q < CS_CHUNK; ++q) {
		const long long r0 = ((lb0 + q) * sh.world + sh.rank) * SB;
		if(r0 >= n) break;
		const long long base = sh.off(r0);
		long long rowoff = 0;
		for(int t = 0; t < SB; ++t) {
			const long long m = r0 + t;
			if(m >= n) break;
			if(m > c) {
				const double d = Elem<ET>::get(D[base + rowoff + c], bs);
				if(0 <= d) {
					s += d;
					++cnt;
					if(d > 0) {
						const int gd = dbl_gran(d);
						g = gd < g ? gd : g;
					}
				} else {
					miss = 1;
				}
			}
			rowoff += m;   // row m holds m cells
		}
	}
	if(cnt) {
		atomicAdd(cs_s + c, s);   // any order: used only where every partial sum is exact
		atomicAdd(cs_c + c, cnt);
		if(g != 0x7FFFFFFF) atomicMin(cs_g + c, (unsigned) (2048 + g));
	}
	if(__any(miss) && (threadIdx.x & 63) == 0) atomicOr(miss_out, 1);
}

// every rank, per column: the exact test over the gathered statistics (rank
// order); sD / N where it holds, else hard[c] = 1 for the serial gather
template <int UNUSED = 0>
__global__ __launch_bounds__(TB) void k_sh_init_exact(int n, int world, const unsigned char *__restrict__ cs_all,
                                                      const double *__restrict__ rp, const int *__restrict__ rc,
                                                      double *__restrict__ sD, int *__restrict__ N,
                                                      unsigned char *__restrict__ hard, int *__restrict__ nhard) {
	const int c = blockIdx.x * TB + threadIdx.x;
	if(c >= n) return;
	const double s0 = rp[c];
	int G = s0 > 0 ? dbl_gran(s0) : 0x7FFFFFFF, cnt = rc[c];
	double T = s0;
	bool any = false;
	for(int r = 0; r < world; ++r) {
		const unsigned char *b = cs_all + (size_t) r * sh_cs_bytes(n);
		const int cr = ((const int *) (b + (size_t) n * 12))[c];
		if(!cr) continue;
		const double sr = ((const double *) b)[c];
		const unsigned gr = ((const unsigned *) (b + (size_t) n * 8))[c];
		if(gr != 0xFFFFFFFFu) {
			const int gg = (int) gr - 2048;
			G = gg < G ? gg : G;
		}
		T += sr;
		cnt += cr;
		any = any || sr != 0;
	}
	// the total (approximate: relative error < n 2^-53 < 2^-20) below 2^(53+G)
	const bool ok = !any || (G != 0x7FFFFFFF && T < ldexp(1.0 - 0x1p-20, 53 + (G < 960 ? G : 960)));
	if(ok) {
		double t = s0;
		for(int r = 0; r < world; ++r) t += ((const double *) (cs_all + (size_t) r * sh_cs_bytes(n)))[c];
		sD[c] = t;
		N[c] = cnt;
		hard[c] = 0;
	} else {
		hard[c] = 1;
		atomicAdd(nhard, 1);
	}
}

// hard columns hc[0..K) (ascending), rows hc[0]+1 .. n-1:
// X[(m - hc[0] - 1) * K + q] = D(m, hc[q]) for the owned rows m > hc[q], zero elsewhere
template <int ET>
__global__ __launch_bounds__(TB) void k_sh_pack_cols(const typename Elem<ET>::T *__restrict__ D, int n, Shard sh,
                                                     const int *__restrict__ hc, int K,
                                                     typename Elem<ET>::T *__restrict__ X) {
	const int cf = hc[0];
	const long long total = (long long) (n - cf - 1) * K;
	for(long long e = (long long) blockIdx.x * TB + threadIdx.x; e < total; e += (long long) gridDim.x * TB) {
		const int m = cf + 1 + (int) (e / K), c = hc[(int) (e % K)];
		typename Elem<ET>::T v = 0;
		if(c < m && sh.owns(m)) v = D[sh.off(m) + c];
		X[e] = v;
	}
}

// the hard columns' parts, continued serially from the row parts in
// increasing m (tree.hip's k_init_cols order); 8 loads in flight per step
template <int ET>
__global__ __launch_bounds__(TB) void k_sh_init_cols(const typename Elem<ET>::T *__restrict__ X, int n, double bs,
                                                     const int *__restrict__ hc, int K, const double *__restrict__ rp,
                                                     const int *__restrict__ rc, double *__restrict__ sD,
                                                     int *__restrict__ N, TreeCtl *ctl) {
	const int q = blockIdx.x * TB + threadIdx.x;
	if(q >= K) return;
	const int cf = hc[0], c = hc[q];
	double s = rp[c];
	int cnt = rc[c], miss = 0;
	const typename Elem<ET>::T *col = X + q;
	constexpr int U = 8;
	for(int m = c + 1; m < n; m += U) {
		typename Elem<ET>::T v[U];
#pragma unroll
		for(int u = 0; u < U; ++u) {
			const int mm = m + u < n ? m + u : n - 1;
			v[u] = col[(long long) (mm - cf - 1) * K];
		}
#pragma unroll
		for(int u = 0; u < U; ++u) {
			if(m + u < n) {
				const double d = Elem<ET>::get(v[u], bs);
				if(0 <= d) {
					s += d;
					++cnt;
				} else {
					miss = 1;
				}
			}
		}
	}
	sD[c] = s;
	N[c] = cnt;
	if(miss) atomicOr(&ctl->has_missing, 1);
}

// ------------------------------------------------------------------ transports
static int coll_fail(const char *what) {
	char m[128];
	snprintf(m, sizeof(m), "collective transport failed in %s", what);
	ccg_set_last_msg(m);
	return CCG_EHIP;
}

// world == 1 without a transport: nothing to reduce, the broadcast is a copy
static int self_allreduce(void *, void *, size_t, void *) { return 0; }
static int self_bcast(void *, const void *send, void *recv, size_t bytes, int, void *stream) {
	if(send != recv && bytes) {
		if(hipMemcpyAsync(recv, send, bytes, hipMemcpyDeviceToDevice, (hipStream_t) stream) != hipSuccess) return -1;
	}
	return 0;
}

static int self_allgather(void *, const void *send, void *recv, size_t bytes, void *stream) {
	return self_bcast(nullptr, send, recv, bytes, 0, stream);
}

// world == 1 without a transport
static inline void sh_self_coll(ccg_coll *c) {
	memset(c, 0, sizeof(*c));
	c->world = 1;
	c->allreduce_sum_u8 = self_allreduce;
	c->broadcast = self_bcast;
	c->allgather = self_allgather;
}

struct CollRun {
	const ccg_coll *c;
	hipStream_t st;
	unsigned char *h;   // pinned staging buffer (host_staged transports)
	KTimer *kt;
	int allreduce(void *d, size_t bytes) {
		if(!c->host_staged) {
			if(c->allreduce_sum_u8(c->user, d, bytes, (void *) st)) return coll_fail("allreduce");
			kt->mark(CCG_K_COLL);
			return CCG_OK;
		}
		CCG_CHECK(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, st));
		CCG_CHECK(hipStreamSynchronize(st));
		if(c->allreduce_sum_u8(c->user, h, bytes, (void *) st)) return coll_fail("allreduce");
		CCG_CHECK(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, st));
		kt->mark(CCG_K_COLL);
		return CCG_OK;
	}
	int bcast(const void *dsend, void *drecv, size_t bytes, int root) {
		if(!c->host_staged) {
			if(c->broadcast(c->user, dsend, drecv, bytes, root, (void *) st)) return coll_fail("broadcast");
			kt->mark(CCG_K_COLL);
			return CCG_OK;
		}
		if(root == c->rank) CCG_CHECK(hipMemcpyAsync(h, dsend, bytes, hipMemcpyDeviceToHost, st));
		CCG_CHECK(hipStreamSynchronize(st));
		if(c->broadcast(c->user, h, h, bytes, root, (void *) st)) return coll_fail("broadcast");
		CCG_CHECK(hipMemcpyAsync(drecv, h, bytes, hipMemcpyHostToDevice, st));
		kt->mark(CCG_K_COLL);
		return CCG_OK;
	}
	// dsend's `bytes` of every rank r -> drecv + r * bytes (device buffers;
	// dsend may be this rank's slot of drecv); without a transport allgather,
	// the allreduce of a zeroed world x bytes buffer (a gather, twice the bytes)
	int allgather(const void *dsend, void *drecv, size_t bytes) {
		unsigned char *slot = (unsigned char *) drecv + (size_t) c->rank * bytes;
		if(!c->allgather) {
			if(slot != dsend) CCG_CHECK(hipMemcpyAsync(slot, dsend, bytes, hipMemcpyDeviceToDevice, st));
			if(c->rank) CCG_CHECK(hipMemsetAsync(drecv, 0, (size_t) c->rank * bytes, st));
			if(c->rank + 1 < c->world)
				CCG_CHECK(hipMemsetAsync(slot + bytes, 0, (size_t) (c->world - c->rank - 1) * bytes, st));
			return allreduce(drecv, (size_t) c->world * bytes);
		}
		if(!c->host_staged) {
			if(c->allgather(c->user, dsend, drecv, bytes, (void *) st)) return coll_fail("allgather");
			kt->mark(CCG_K_COLL);
			return CCG_OK;
		}
		unsigned char *hs = h + (size_t) c->rank * bytes;
		CCG_CHECK(hipMemcpyAsync(hs, dsend, bytes, hipMemcpyDeviceToHost, st));
		CCG_CHECK(hipStreamSynchronize(st));
		if(c->allgather(c->user, hs, h, bytes, (void *) st)) return coll_fail("allgather");
		CCG_CHECK(hipMemcpyAsync(drecv, h, (size_t) c->world * bytes, hipMemcpyHostToDevice, st));
		kt->mark(CCG_K_COLL);
		return CCG_OK;
	}
};

// ------------------------------------------------------------------ init
// Cells per chunk of the gathered hard columns: at most a quarter of free HBM
// (16 GB cap); host-staged transports move 64 MB at a time.
static int sh_init_chunk(int n0, int es, bool host_staged, long long *K) {
	size_t free_b = 0, total_b = 0;
	CCG_CHECK(hipMemGetInfo(&free_b, &total_b));
	const size_t budget =
	    host_staged ? ((size_t) 64 << 20) : (free_b / 4 < ((size_t) 16 << 30) ? free_b / 4 : ((size_t) 16 << 30));
	long long k = (long long) (budget / ((size_t) n0 * es));
	if(k < 256) k = 256;
	if(k > n0) k = n0;
	*K = k;
	return CCG_OK;
}

// bytes of the row-part gather buffer: n0 f64 sums, n0 i32 counts, i32 missing flag
static inline size_t sh_rp_bytes(int n0) { return (size_t) n0 * 12 + 16; }

// the pinned staging buffer a host-staged transport needs for the init: the
// gathered statistics, or one 64 MB chunk of hard columns
static inline size_t sh_init_host_bytes(int n0, int world) {
	size_t h = sh_cs_bytes(n0) * (size_t) world;
	const size_t chunk = (size_t) 64 << 20;
	if(h < chunk + (size_t) n0 * 8) h = chunk + (size_t) n0 * 8;
	return h > sh_rp_bytes(n0) ? h : sh_rp_bytes(n0);
}

// device scratch of sh_init_summad beyond the row parts: this rank's column
// statistics, every rank's (allgather), the hard flags / list and counter
static inline size_t sh_init_scratch_bytes(int n0, int world) {
	return sh_cs_bytes(n0) * (size_t) (world + 1) + (size_t) n0 * 5 + 256;
}

struct ShInitStat {
	long long coll_bytes;   // bytes this rank put into the init collectives
	int hard;               // columns summed through the serial gather
};

// initSummaD (nj.c:111), exact for every world size: the owners' row parts
// are gathered; each column part is the exact sum of the ranks' statistics
// where every partial sum is representable, else (hard columns) continued
// serially over the gathered column.  Leaves sD/N replicated in b and sets
// *missing when any entry is negative (the shards do not run updateD's
// missing-entry quirks).
template <int ET>
static int sh_init_summad(const typename Elem<ET>::T *D, int n0, double bs, const Shard &sh, CollRun &cr,
                          hipStream_t st, void *rp_buf, void *scratch, TreeBufs &b, long long *launches, int *missing,
                          ShInitStat *is) {
	double *rp = (double *) rp_buf;
	int *rcnt = (int *) ((char *) rp_buf + (size_t) n0 * 8);
	int *rmiss = rcnt + n0;
	unsigned char *cs = (unsigned char *) scratch, *cs_all = cs + sh_cs_bytes(n0);
	unsigned char *hard = cs_all + sh_cs_bytes(n0) * (size_t) sh.world;
	int *hlist = (int *) (((uintptr_t) (hard + n0) + 15) & ~(uintptr_t) 15);
	int *nhard = hlist + n0;
	is->coll_bytes = 0;
	is->hard = 0;
	k_sh_init_rows<ET><<<cdiv(n0, TB / 64), TB, 0, st>>>(D, n0, bs, sh, rp, rcnt, rmiss);
	CCG_CHECK(hipGetLastError());
	CCG_CHECK(hipMemsetAsync(cs, 0, (size_t) n0 * 8, st));
	CCG_CHECK(hipMemsetAsync(cs + (size_t) n0 * 8, 0xFF, (size_t) n0 * 4, st));
	CCG_CHECK(hipMemsetAsync(cs + (size_t) n0 * 12, 0, (size_t) n0 * 4, st));
	CCG_CHECK(hipMemsetAsync(nhard, 0, 4, st));
	{
		const int nb = (n0 + SB - 1) / SB;
		const int nlb = nb > sh.rank ? (nb - sh.rank + sh.world - 1) / sh.world : 0;
		const unsigned gy = (unsigned) cdiv(nlb, CS_CHUNK);
		if(gy) {
			dim3 g((unsigned) cdiv(n0, TB), gy);
			k_sh_col_stats<ET><<<g, TB, 0, st>>>(D, n0, bs, sh, (double *) cs, (unsigned *) (cs + (size_t) n0 * 8),
			                                     (int *) (cs + (size_t) n0 * 12), rmiss);
			CCG_CHECK(hipGetLastError());
		}
	}
	cr.kt->mark(CCG_K_INIT);
	int rc = cr.allreduce(rp, sh_rp_bytes(n0));
	if(rc) return rc;
	if((rc = cr.allgather(cs, cs_all, sh_cs_bytes(n0)))) return rc;
	is->coll_bytes += (long long) sh_rp_bytes(n0) + (long long) sh_cs_bytes(n0);
	k_sh_init_exact<><<<cdiv(n0, TB), TB, 0, st>>>(n0, sh.world, cs_all, rp, rcnt, b.sD, b.N, hard, nhard);
	CCG_CHECK(hipGetLastError());
	cr.kt->mark(CCG_K_INIT);
	*launches += 3;
	int hm = 0, nh = 0;
	CCG_CHECK(hipMemcpyAsync(&hm, rmiss, 4, hipMemcpyDeviceToHost, st));
	CCG_CHECK(hipMemcpyAsync(&nh, nhard, 4, hipMemcpyDeviceToHost, st));
	CCG_CHECK(hipStreamSynchronize(st));
	if(hm) {
		*missing = 1;
		return CCG_OK;
	}
	if(nh) {
		// the hard columns, ascending (the same list on every rank), gathered
		// in chunks of at most K * n0 cells through a buffer of their own
		long long K = 0;
		if((rc = sh_init_chunk(n0, ET, cr.c->host_staged != 0, &K))) return rc;
		typename Elem<ET>::T *Xc = NULL;
		if(hipMalloc((void **) &Xc, (size_t) K * n0 * ET) != hipSuccess) return CCG_ENOMEM;
		unsigned char *hh = (unsigned char *) malloc((size_t) n0);
		int *hl = (int *) malloc((size_t) nh * sizeof(int));
		if(!hh || !hl) {
			free(hh);
			free(hl);
			hipFree(Xc);
			return CCG_ENOMEM;
		}
		rc = hipMemcpy(hh, hard, (size_t) n0, hipMemcpyDeviceToHost) == hipSuccess ? CCG_OK : CCG_EHIP;
		int q = 0;
		for(int c = 0; c < n0 && q < nh; ++c)
			if(hh[c]) hl[q++] = c;
		if(!rc && hipMemcpy(hlist, hl, (size_t) nh * sizeof(int), hipMemcpyHostToDevice) != hipSuccess) rc = CCG_EHIP;
		// chunks of consecutive hard columns whose rows fit the buffer of K * n0 cells
		for(int q0 = 0; q0 < nh && !rc;) {
			const long long rows = n0 - hl[q0] - 1;
			long long kq = rows > 0 ? (K * (long long) n0) / rows : nh;
			if(kq < 1) kq = 1;
			if(kq > nh - q0) kq = nh - q0;
			const int Kc = (int) kq;
			const long long cells = rows * Kc;
			if(cells > 0) {
				long long g = (cells + TB - 1) / TB;
				if(g > 65536) g = 65536;
				k_sh_pack_cols<ET><<<(unsigned) g, TB, 0, st>>>(D, n0, sh, hlist + q0, Kc, Xc);
				cr.kt->mark(CCG_K_INIT);
				if((rc = cr.allreduce(Xc, (size_t) cells * ET))) break;
				is->coll_bytes += cells * ET;
			}
			k_sh_init_cols<ET><<<cdiv(Kc, TB), TB, 0, st>>>(Xc, n0, bs, hlist + q0, Kc, rp, rcnt, b.sD, b.N, b.ctl);
			cr.kt->mark(CCG_K_INIT);
			*launches += 2;
			q0 += Kc;
		}
		hipStreamSynchronize(st);
		hipFree(Xc);
		free(hh);
		free(hl);
		if(rc) return rc;
		is->hard = nh;
	}
	TreeCtl hc;
	CCG_CHECK(hipMemcpyAsync(&hc, b.ctl, sizeof(hc), hipMemcpyDeviceToHost, st));
	CCG_CHECK(hipStreamSynchronize(st));
	*missing = hc.has_missing || hm;
	return CCG_OK;
}
