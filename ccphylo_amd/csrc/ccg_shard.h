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

__device__ __forceinline__ void rec_fold(const ShRec *__restrict__ rec, int world, double &bq, long long &bf) {
	bq = 1.0;
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

// column chunk [c0, c0 + K): X[(m - c0 - 1) * K + (c - c0)] = D(m, c) for the
// owned rows m > c, zero elsewhere
template <int ET>
__global__ __launch_bounds__(TB) void k_sh_pack_cols(const typename Elem<ET>::T *__restrict__ D, int n, Shard sh,
                                                     int c0, int K, typename Elem<ET>::T *__restrict__ X) {
	const long long total = (long long) (n - c0 - 1) * K;
	for(long long e = (long long) blockIdx.x * TB + threadIdx.x; e < total; e += (long long) gridDim.x * TB) {
		const int m = c0 + 1 + (int) (e / K), c = c0 + (int) (e % K);
		typename Elem<ET>::T v = 0;
		if(c < m && sh.owns(m)) v = D[sh.off(m) + c];
		X[e] = v;
	}
}

// column parts, continued serially from the row parts in increasing m (the
// same order as tree.hip's k_init_cols); 8 loads in flight per step
template <int ET>
__global__ __launch_bounds__(TB) void k_sh_init_cols(const typename Elem<ET>::T *__restrict__ X, int n, double bs,
                                                     int c0, int K, const double *__restrict__ rp,
                                                     const int *__restrict__ rc, double *__restrict__ sD,
                                                     int *__restrict__ N, TreeCtl *ctl) {
	const int c = c0 + blockIdx.x * TB + threadIdx.x;
	if(c >= c0 + K || c >= n) return;
	double s = rp[c];
	int cnt = rc[c], miss = 0;
	const typename Elem<ET>::T *col = X + (c - c0);
	constexpr int U = 8;
	for(int m = c + 1; m < n; m += U) {
		typename Elem<ET>::T v[U];
#pragma unroll
		for(int u = 0; u < U; ++u) {
			const int mm = m + u < n ? m + u : n - 1;
			v[u] = col[(long long) (mm - c0 - 1) * K];
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

// world == 1 without a transport
static inline void sh_self_coll(ccg_coll *c) {
	memset(c, 0, sizeof(*c));
	c->world = 1;
	c->allreduce_sum_u8 = self_allreduce;
	c->broadcast = self_bcast;
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
};

// ------------------------------------------------------------------ init
// Columns per chunk of the gathered column parts: wide enough to keep the
// serial column sums parallel, at most a quarter of free HBM (16 GB cap);
// host-staged transports move 64 MB at a time.
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

// initSummaD (nj.c:111), exact for every world size: the owners' row parts
// are gathered, then the column parts continue serially in increasing m over
// chunks of K columns gathered the same way.  Leaves sD/N replicated in b and
// sets *missing when any entry is negative (the shards do not run updateD's
// missing-entry quirks).
template <int ET>
static int sh_init_summad(const typename Elem<ET>::T *D, int n0, double bs, const Shard &sh, CollRun &cr,
                          hipStream_t st, void *rp_buf, typename Elem<ET>::T *Xc, long long K, TreeBufs &b,
                          long long *launches, int *missing) {
	double *rp = (double *) rp_buf;
	int *rcnt = (int *) ((char *) rp_buf + (size_t) n0 * 8);
	int *rmiss = rcnt + n0;
	k_sh_init_rows<ET><<<cdiv(n0, TB / 64), TB, 0, st>>>(D, n0, bs, sh, rp, rcnt, rmiss);
	CCG_CHECK(hipGetLastError());
	cr.kt->mark(CCG_K_INIT);
	int rc = cr.allreduce(rp, sh_rp_bytes(n0));
	if(rc) return rc;
	for(int c0 = 0; c0 < n0 - 1; c0 += (int) K) {
		const int Kc = (int) (n0 - c0 < K ? n0 - c0 : K);
		const long long cells = (long long) (n0 - c0 - 1) * Kc;
		long long g = (cells + TB - 1) / TB;
		if(g > 65536) g = 65536;
		k_sh_pack_cols<ET><<<(unsigned) g, TB, 0, st>>>(D, n0, sh, c0, Kc, Xc);
		cr.kt->mark(CCG_K_INIT);
		if((rc = cr.allreduce(Xc, (size_t) cells * ET))) return rc;
		k_sh_init_cols<ET><<<cdiv(Kc, TB), TB, 0, st>>>(Xc, n0, bs, c0, Kc, rp, rcnt, b.sD, b.N, b.ctl);
		cr.kt->mark(CCG_K_INIT);
		*launches += 2;
	}
	// the last column (n0 - 1) has no column part
	CCG_CHECK(hipMemcpyAsync(b.sD + n0 - 1, rp + n0 - 1, 8, hipMemcpyDeviceToDevice, st));
	CCG_CHECK(hipMemcpyAsync(b.N + n0 - 1, rcnt + n0 - 1, 4, hipMemcpyDeviceToDevice, st));
	CCG_CHECK(hipGetLastError());
	*launches += 1;
	TreeCtl hc;
	int hm = 0;
	CCG_CHECK(hipMemcpyAsync(&hc, b.ctl, sizeof(hc), hipMemcpyDeviceToHost, st));
	CCG_CHECK(hipMemcpyAsync(&hm, rmiss, 4, hipMemcpyDeviceToHost, st));
	CCG_CHECK(hipStreamSynchronize(st));
	*missing = hc.has_missing || hm;
	return CCG_OK;
}
