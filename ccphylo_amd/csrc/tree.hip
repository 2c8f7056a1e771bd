// tree.hip -- neighbor joining (NJ) and dynamic NJ (DNJ) on an HBM-resident
// packed lower-triangular distance matrix, for gfx950.
//
// Reference semantics (ccphylo 0.8.5):
//   initSummaD nj.c:111, initQ nj.c:182, limbLength nj.c:42/:81, updateD nj.c:836,
//   ltdMatrix_popArrange matrix.c:518, nj loop nj.c:1560,
//   initHNJ hclust.c:56, minQ hclust.c:353, minQpair dnj.c:43, updateDNJ dnj.c:607,
//   DNJ_popArrange dnj.c:817, minPos dnj.c:977, dnj loop dnj.c:985.
//
// Layout in HBM: D is the reference's contiguous LT buffer (row r starts at
// r(r-1)/2, element type ET), plus n-vectors sD (f64), N (i32), Q (f64),
// P (i32).  All control state lives in a device TreeCtl; the host only
// enqueues kernels (n shrinks by exactly one per join, so every grid is known
// in advance) and reads the join list at the end.
//
// DNJ selection (minQpair) is a strict serial scan in the reference: row i is
// rescanned iff its stale bound Q[i] is below the running minimum m(i) of the
// rows above it.  Here:
//   k_dnj_top    rescans the top-B candidate rows (Q[i] < m0) in parallel;
//   k_dnj_rest   computes U = min(m0, min_{k in S} max(fresh_k, Q_k)), an upper
//                bound of m(i) for every row below S (a row k above i that the
//                serial scan rescans gives m(i) <= fresh_k, one it skips gives
//                m(i) <= m(k) <= Q_k), and rescans every row with Q[i] < U;
//   k_dnj_replay replays the reference's decisions serially over that set,
//                so Q/P and the chosen pair are identical to minQpair's.
#include <string.h>
#include "ccg_internal.h"

#define TB 256           // threads per block for the vector kernels
#define DNJ_B 64         // top candidates rescanned speculatively
#define REST_BLOCKS 128  // blocks of k_dnj_rest

struct TreeCtl {
	int done;            // the reference loop stopped (pos == 0)
	int final_n;         // n when done was set
	int njoins;
	int first;           // cand comes from minQ (first DNJ iteration)
	int cand;
	int mi, mj;
	int i, j;            // current join
	double Li, Lj, Dij;
	double m0;           // minQpair's initial min
	int pos_i, pos_j;    // minQpair's initial pos
	int nS;              // |S|
	int has_missing;     // D holds entries < 0 (or NaN): general updateD path
	unsigned counter;    // last-block ticket, reset by the last block
	int neg;             // limbLengthNeg
	int exact;
	int exact_fast;      // stats: exact sums resolved without the serial chain
	long long rows, cells;
};

struct TreeBufs {
	double *sD, *Q, *fq, *contrib;
	int *N, *P, *fj, *S, *seg, *segcnt;
	double *wsum;        // per-block partial sums
	int *wcnt;
	double *qpart;       // per-block QArg partials (4 per block)
	int *ipart;
	double *absb;        // per-block sum |c|, for the exactness test
	int *qmin;           // per-block minimum quantum exponent
	long long *fpart;
	ccg_join *joins;
	TreeCtl *ctl;
};

// ------------------------------------------------------------------ init
template <int ET>
__global__ void k_init_sums(const typename Elem<ET>::T *__restrict__ D, int n, double bs,
                            double *__restrict__ sD, int *__restrict__ N, TreeCtl *ctl) {
	int k = blockIdx.x * blockDim.x + threadIdx.x;
	if(k >= n) return;
	double s = 0;
	int c = 1, miss = 0;
	const typename Elem<ET>::T *row = D + tri(k);
	for(int m = 0; m < k; ++m) {        // row part: m < k, increasing m
		double d = Elem<ET>::get(row[m], bs);
		if(0 <= d) {
			s += d;
			++c;
		} else {
			miss = 1;
		}
	}
	for(int m = k + 1; m < n; ++m) {    // column part: m > k, increasing m
		double d = Elem<ET>::get(D[tri(m) + k], bs);
		if(0 <= d) {
			s += d;
			++c;
		} else {
			miss = 1;
		}
	}
	sD[k] = s;
	N[k] = c;
	if(miss) atomicOr(&ctl->has_missing, 1);
}

// hclust.c:56-130: per-row min with ties -> smaller D, then later j
template <int ET>
__global__ void k_init_hnj(const typename Elem<ET>::T *__restrict__ D, int n, double bs,
                           const double *__restrict__ sD, const int *__restrict__ N,
                           double *__restrict__ Q, int *__restrict__ P) {
	int i = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
	int lane = threadIdx.x & 63;
	if(i >= n) return;
	double bq = DBL_MAX, bd = DBL_MAX;
	int bj = 0;
	const typename Elem<ET>::T *row = D + tri(i);
	int Ni = N[i];
	double sDi = sD[i];
	for(int j = lane; j < i; j += 64) {
		double d = Elem<ET>::get(row[j], bs);
		if(0 <= d) {
			double q = qcrit(Ni, N[j], d, sDi, sD[j]);
			if(q < bq || (q == bq && (d < bd || (d == bd && j > bj)))) {
				bq = q;
				bd = d;
				bj = j;
			}
		}
	}
#pragma unroll
	for(int off = 32; off > 0; off >>= 1) {
		double oq = __shfl_xor(bq, off, 64), od = __shfl_xor(bd, off, 64);
		int oj = __shfl_xor(bj, off, 64);
		if(oq < bq || (oq == bq && (od < bd || (od == bd && oj > bj)))) {
			bq = oq;
			bd = od;
			bj = oj;
		}
	}
	if(lane == 0) {
		Q[i] = bq;
		P[i] = bj;
	}
}

// hclust.c:353 minQ -> the first candidate row of dnj.c:997-998
__global__ void k_min_q_row(const double *__restrict__ Q, int n, TreeCtl *ctl) {
	__shared__ double sq[TB / 64];
	__shared__ int si[TB / 64];
	double q = DBL_MAX;
	int idx = 0;
	for(int i = 1 + threadIdx.x; i < n; i += blockDim.x) {
		if(qarg_better(Q[i], i, q, idx)) {
			q = Q[i];
			idx = i;
		}
	}
	qarg_block_reduce(q, idx, sq, si);
	if(threadIdx.x == 0) {
		ctl->cand = idx;
		ctl->first = 1;
	}
}

// nj.c:42 limbLength / nj.c:81 limbLengthNeg
__device__ void limb_length(double *Li, double *Lj, int i, int j, const double *sD, const int *N,
                            double Dij, int neg) {
	int Ni = N[i] - 2, Nj = N[j] - 2;
	if(0 < Ni && 0 < Nj) {
		double delta = ((sD[i] - Dij) / Ni) - ((sD[j] - Dij) / Nj);
		*Li = (Dij + delta) / 2;
		*Lj = (Dij - delta) / 2;
		if(!neg) {
			if(*Li < 0) {
				*Lj = Dij;
				*Li = 0;
			} else if(*Lj < 0) {
				*Li = Dij;
				*Lj = 0;
			}
		}
	} else if(0 < Ni) {
		*Li = 0;
		*Lj = Dij;
	} else if(0 < Nj) {
		*Li = Dij;
		*Lj = 0;
	} else {
		*Li = *Lj = Dij / 2;
	}
}

template <int ET>
__device__ void record_join(const typename Elem<ET>::T *D, double bs, const TreeBufs &b, int i, int j) {
	TreeCtl *ctl = b.ctl;
	double Dij = Elem<ET>::get(D[tri(i) + j], bs), Li, Lj;
	limb_length(&Li, &Lj, i, j, b.sD, b.N, Dij, ctl->neg);
	ctl->i = i;
	ctl->j = j;
	ctl->Li = Li;
	ctl->Lj = Lj;
	ctl->Dij = Dij;
	ccg_join J;
	J.i = i;
	J.j = j;
	J.Li = Li;
	J.Lj = Lj;
	b.joins[ctl->njoins++] = J;
}

// fresh (q, j) min of LT row r over j < r, whole block (dnj.c:99-112)
template <int ET>
__device__ __forceinline__ void rescan_row(const typename Elem<ET>::T *__restrict__ D, double bs,
                                           const double *__restrict__ sD, const int *__restrict__ N,
                                           int r, double *sq, int *si, double &oq, int &oj) {
	const typename Elem<ET>::T *row = D + tri(r);
	int Nr = N[r];
	double sDr = sD[r];
	double q = DBL_MAX;
	int idx = 0;
	for(int j = threadIdx.x; j < r; j += blockDim.x) {
		double d = Elem<ET>::get(row[j], bs);
		if(0 <= d) {
			double v = qcrit(Nr, N[j], d, sDr, sD[j]);
			if(qarg_better(v, j, q, idx)) {
				q = v;
				idx = j;
			}
		}
	}
	qarg_block_reduce(q, idx, sq, si);
	oq = q;
	oj = idx;
}

// ------------------------------------------------------------------ DNJ
__device__ __forceinline__ int dnj_candidate(const TreeCtl *ctl, const double *Q, int n) {
	if(ctl->first) return ctl->cand;
	int mi = ctl->mi, mj = ctl->mj;
	if(mj == n) return mi;
	if(mi == n) return mj;
	// dnj.c:977 minPos
	return (Q[mj] < Q[mi] || (mi < mj && Q[mj] == Q[mi])) ? mj : mi;
}

// ordered block compaction of flags (descending row order = thread order)
__device__ __forceinline__ int block_compact(bool flag, int value, int *out, int base, int cap, int *wcount) {
	const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
	unsigned long long m = __ballot(flag);
	if(lane == 0) wcount[wid] = __popcll(m);
	__syncthreads();
	int off = 0, tot = 0;
	for(int w = 0; w < nw; ++w) {
		if(w < wid) off += wcount[w];
		tot += wcount[w];
	}
	if(flag) {
		int pos = base + off + __popcll(m & ((1ull << lane) - 1));
		if(pos < cap) out[pos] = value;
	}
	__syncthreads();
	return tot;
}

template <int ET>
__global__ __launch_bounds__(TB) void k_dnj_top(const typename Elem<ET>::T *__restrict__ D, int n, double bs,
                                                TreeBufs b) {
	__shared__ int list[DNJ_B + TB];
	__shared__ int wcount[TB / 64];
	__shared__ double sq[TB / 64];
	__shared__ int si[TB / 64];
	TreeCtl *ctl = b.ctl;
	if(ctl->done) return;
	int cand = dnj_candidate(ctl, b.Q, n);
	double m0 = DBL_MAX;
	if(cand && m0 != b.Q[cand]) m0 = b.Q[cand];
	// the first DNJ_B rows (descending) with Q[r] < m0
	int cnt = 0;
	for(int base = n - 1; base >= 1 && cnt < DNJ_B; base -= blockDim.x) {
		int r = base - (int) threadIdx.x;
		bool f = r >= 1 && b.Q[r] < m0;
		cnt += block_compact(f, r, list, cnt, DNJ_B, wcount);
	}
	int nS = cnt < DNJ_B ? cnt : DNJ_B;
	if(blockIdx.x == 0 && threadIdx.x == 0) {
		ctl->cand = cand;
		ctl->m0 = m0;
		ctl->pos_i = (cand && m0 != DBL_MAX) ? cand : 0;
		ctl->pos_j = (cand && m0 != DBL_MAX) ? b.P[cand] : 0;
		ctl->nS = nS;
	}
	if(blockIdx.x == 0) {
		for(int t = threadIdx.x; t < nS; t += blockDim.x) b.S[t] = list[t];
	}
	for(int t = blockIdx.x; t < nS; t += gridDim.x) {
		int r = list[t];
		double q;
		int j;
		rescan_row<ET>(D, bs, b.sD, b.N, r, sq, si, q, j);
		if(threadIdx.x == 0) {
			b.fq[r] = q;
			b.fj[r] = j;
		}
	}
}

template <int ET>
__global__ __launch_bounds__(TB) void k_dnj_rest(const typename Elem<ET>::T *__restrict__ D, int n, double bs,
                                                 TreeBufs b) {
	__shared__ int list[TB];
	__shared__ int wcount[TB / 64];
	__shared__ double sq[TB / 64];
	__shared__ int si[TB / 64];
	__shared__ double sU;
	TreeCtl *ctl = b.ctl;
	if(ctl->done) return;
	int nS = ctl->nS;
	int w = blockIdx.x;
	if(nS < DNJ_B) {
		if(threadIdx.x == 0) b.segcnt[w] = 0;
		return;
	}
	int smin = b.S[DNJ_B - 1];
	if(threadIdx.x < 64) {
		double U = ctl->m0;
		for(int t = threadIdx.x; t < DNJ_B; t += 64) {
			int k = b.S[t];
			double u = b.fq[k] > b.Q[k] ? b.fq[k] : b.Q[k];
			if(u < U) U = u;
		}
#pragma unroll
		for(int off = 32; off > 0; off >>= 1) {
			double o = __shfl_xor(U, off, 64);
			if(o < U) U = o;
		}
		if(threadIdx.x == 0) sU = U;
	}
	__syncthreads();
	double U = sU;
	// rows [1, smin) in gridDim.x slices; slice w covers [lo, hi)
	int rows = smin - 1;
	int lo = 1 + (int) ((long long) rows * w / gridDim.x);
	int hi = 1 + (int) ((long long) rows * (w + 1) / gridDim.x);
	int cnt = 0;
	for(int base = hi - 1; base >= lo; base -= blockDim.x) {
		int r = base - (int) threadIdx.x;
		bool f = r >= lo && b.Q[r] < U;
		int got = block_compact(f, r, list, 0, TB, wcount);
		for(int t = 0; t < got; ++t) {
			int rr = list[t];
			double q;
			int j;
			rescan_row<ET>(D, bs, b.sD, b.N, rr, sq, si, q, j);
			if(threadIdx.x == 0) {
				b.fq[rr] = q;
				b.fj[rr] = j;
				b.seg[lo + cnt] = rr;
			}
			++cnt;
		}
	}
	if(threadIdx.x == 0) b.segcnt[w] = cnt;
}

// serial replay of minQpair's decisions over S then the slices, descending
template <int ET>
__global__ __launch_bounds__(TB) void k_dnj_replay(const typename Elem<ET>::T *__restrict__ D, int n, double bs,
                                                   TreeBufs b, int nrest) {
	__shared__ int rr[TB], rj[TB];
	__shared__ double rq[TB], rf[TB];
	__shared__ double s_m;
	__shared__ int s_pi, s_pj, s_total;
	__shared__ int sl_base[REST_BLOCKS + 1];
	TreeCtl *ctl = b.ctl;
	if(ctl->done) return;
	const int nS = ctl->nS;
	const bool more = nS == DNJ_B;
	const int rows = (more ? b.S[DNJ_B - 1] : 1) - 1;   // rows [1, smin) went to k_dnj_rest
	if(threadIdx.x == 0) {
		s_m = ctl->m0;
		s_pi = ctl->pos_i;
		s_pj = ctl->pos_j;
		// slice t of the replay order is rest block w = nrest-1-t (higher rows first)
		int acc = nS;
		for(int t = 0; t < nrest; ++t) {
			sl_base[t] = acc;
			acc += more ? b.segcnt[nrest - 1 - t] : 0;
		}
		sl_base[nrest] = acc;
		s_total = acc;
	}
	__syncthreads();
	const int total = s_total;
	int nrows = 0;
	long long cells = 0;
	for(int c0 = 0; c0 < total; c0 += blockDim.x) {
		int e = c0 + threadIdx.x;
		if(e < total) {
			int r;
			if(e < nS) {
				r = b.S[e];
			} else {
				int lo_t = 0, hi_t = nrest - 1;   // last t with sl_base[t] <= e
				while(lo_t < hi_t) {
					int mid = (lo_t + hi_t + 1) >> 1;
					if(sl_base[mid] <= e) lo_t = mid; else hi_t = mid - 1;
				}
				int w = nrest - 1 - lo_t;
				int lo = 1 + (int) ((long long) rows * w / nrest);
				r = b.seg[lo + (e - sl_base[lo_t])];
			}
			rr[threadIdx.x] = r;
			rq[threadIdx.x] = b.Q[r];
			rf[threadIdx.x] = b.fq[r];
			rj[threadIdx.x] = b.fj[r];
			++nrows;
			cells += r;
		}
		__syncthreads();
		if(threadIdx.x == 0) {
			double m = s_m;
			int pi = s_pi, pj = s_pj;
			int lim = total - c0 < (int) blockDim.x ? total - c0 : (int) blockDim.x;
			for(int u = 0; u < lim; ++u) {
				if(rq[u] < m) {
					// the reference rescans this row (dnj.c:78-123)
					int r = rr[u];
					b.Q[r] = rf[u];
					b.P[r] = rj[u];
					if(rf[u] < m) {
						m = rf[u];
						pi = r;
						pj = rj[u];
					}
				}
			}
			s_m = m;
			s_pi = pi;
			s_pj = pj;
		}
		__syncthreads();
	}
	for(int off = 32; off > 0; off >>= 1) {
		nrows += __shfl_xor(nrows, off, 64);
		cells += __shfl_xor(cells, off, 64);
	}
	if((threadIdx.x & 63) == 0 && nrows) {
		atomicAdd((unsigned long long *) &ctl->rows, (unsigned long long) nrows);
		atomicAdd((unsigned long long *) &ctl->cells, (unsigned long long) cells);
	}
	if(threadIdx.x == 0) {
		ctl->first = 0;
		if(s_pi == 0 && s_pj == 0) {
			ctl->done = 1;
			ctl->final_n = n;
		} else {
			record_join<ET>(D, bs, b, s_pi, s_pj);
		}
	}
}

// ------------------------------------------------------------------ NJ argmin
// nj.c:182 initQ: min starts at 1, the last minimal cell in row-major order
template <int ET>
__global__ __launch_bounds__(TB) void k_nj_argmin(const typename Elem<ET>::T *__restrict__ D, int n, double bs,
                                                  TreeBufs b, long long chunk) {
	__shared__ double sq[TB / 64];
	__shared__ long long sf[TB / 64];
	TreeCtl *ctl = b.ctl;
	if(ctl->done) return;
	long long cells = tri(n);
	long long f0 = (long long) blockIdx.x * chunk;
	long long f1 = f0 + chunk < cells ? f0 + chunk : cells;
	double bq = 1.0;
	long long bf = -1;
	if(f0 < f1) {
		long long f = f0 + threadIdx.x;
		// row of f: largest r with r(r-1)/2 <= f
		long long r = (long long) ((1.0 + sqrt(1.0 + 8.0 * (double) f)) * 0.5);
		while(tri(r) > f) --r;
		while(tri(r + 1) <= f) ++r;
		long long c = f - tri(r);
		int Nr = b.N[r];
		double sDr = b.sD[r];
		for(; f < f1; f += blockDim.x) {
			double d = Elem<ET>::get(D[f], bs);
			if(0 <= d) {
				double q = qcrit(Nr, b.N[c], d, sDr, b.sD[c]);
				if(q < bq || (q == bq && f > bf)) {
					bq = q;
					bf = f;
				}
			}
			c += blockDim.x;
			if(c >= r) {
				do {
					c -= r;
					++r;
				} while(c >= r);
				if(r < n) {
					Nr = b.N[r];
					sDr = b.sD[r];
				}
			}
		}
	}
	// block reduce (min q, max f)
#pragma unroll
	for(int off = 32; off > 0; off >>= 1) {
		double oq = __shfl_xor(bq, off, 64);
		long long of = __shfl_xor(bf, off, 64);
		if(oq < bq || (oq == bq && of > bf)) {
			bq = oq;
			bf = of;
		}
	}
	int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
	if(lane == 0) {
		sq[wid] = bq;
		sf[wid] = bf;
	}
	__syncthreads();
	if(threadIdx.x == 0) {
		for(int w = 1; w < (int) (blockDim.x >> 6); ++w) {
			if(sq[w] < bq || (sq[w] == bq && sf[w] > bf)) {
				bq = sq[w];
				bf = sf[w];
			}
		}
		b.qpart[blockIdx.x] = bq;
		b.fpart[blockIdx.x] = bf;
	}
	if(last_block_arrive(&ctl->counter)) {
		if(threadIdx.x == 0) {
			ctl->counter = 0;
			double q = 1.0;
			long long f = -1;
			for(unsigned w = 0; w < gridDim.x; ++w) {
				double oq = __hip_atomic_load(&b.qpart[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
				long long of = __hip_atomic_load(&b.fpart[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
				if(oq < q || (oq == q && of > f)) {
					q = oq;
					f = of;
				}
			}
			if(f < 0) {
				ctl->done = 1;
				ctl->final_n = n;
			} else {
				long long r = (long long) ((1.0 + sqrt(1.0 + 8.0 * (double) f)) * 0.5);
				while(tri(r) > f) --r;
				while(tri(r + 1) <= f) ++r;
				record_join<ET>(D, bs, b, (int) r, (int) (f - tri(r)));
			}
		}
	}
}

// ------------------------------------------------------------------ updateD
// nj.c:836-1044 without missing entries: every k takes the (D_ik, D_kj >= 0)
// branch, so the sD/N cursor never lags.
template <int ET>
__global__ __launch_bounds__(TB) void k_update(typename Elem<ET>::T *__restrict__ D, int n, double bs, TreeBufs b) {
	__shared__ double ssum[TB / 64];
	__shared__ int scnt[TB / 64];
	TreeCtl *ctl = b.ctl;
	if(ctl->done) return;
	int i = ctl->i, j = ctl->j;
	double Dij = ctl->Dij;
	int k = blockIdx.x * blockDim.x + threadIdx.x;
	double d = 0;
	int cnt = 0;
	if(k < n && k != i && k != j) {
		long long fik = k < i ? tri(i) + k : tri(k) + i;
		long long fkj = k < j ? tri(j) + k : tri(k) + j;
		double Dik = Elem<ET>::get(D[fik], bs), Dkj = Elem<ET>::get(D[fkj], bs);
		d = (Dik + Dkj - Dij) / 2;
		d = d < 0 ? 0 : d;
		D[fkj] = Elem<ET>::put(d, 0.25, bs);
		b.sD[k] -= (Dik + Dkj - d);
		b.N[k] -= 1;
		cnt = 1;
	}
	if(ctl->exact && k < n) b.contrib[k] = d;
	// fixed-order block partials
	double s = d;
#pragma unroll
	for(int off = 32; off > 0; off >>= 1) {
		s += __shfl_down(s, off, 64);
		cnt += __shfl_down(cnt, off, 64);
	}
	int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
	if(lane == 0) {
		ssum[wid] = s;
		scnt[wid] = cnt;
	}
	__syncthreads();
	if(threadIdx.x == 0) {
		double t = 0;
		int c = 0;
		for(int w = 0; w < (int) (blockDim.x >> 6); ++w) {
			t += ssum[w];
			c += scnt[w];
		}
		b.wsum[blockIdx.x] = t;
		b.wcnt[blockIdx.x] = c;
	}
	if(last_block_arrive(&ctl->counter)) {
		__shared__ double buf[TB];
		int c = 0;
		for(unsigned w = threadIdx.x; w < gridDim.x; w += blockDim.x) {
			c += __hip_atomic_load(&b.wcnt[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		}
		for(int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off, 64);
		__shared__ int sc[TB / 64];
		if(lane == 0) sc[wid] = c;
		double sd = 0;
		if(ctl->exact) {
			// serial sum in increasing k (nj.c:911/:1002), staged through LDS
			for(int c0 = 0; c0 < n; c0 += blockDim.x) {
				int kk = c0 + threadIdx.x;
				buf[threadIdx.x] = kk < n ? __hip_atomic_load(&b.contrib[kk], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.0;
				__syncthreads();
				if(threadIdx.x == 0) {
					int lim = n - c0 < (int) blockDim.x ? n - c0 : (int) blockDim.x;
					for(int u = 0; u < lim; ++u) sd += buf[u];
				}
				__syncthreads();
			}
		} else if(threadIdx.x == 0) {
			for(unsigned w = 0; w < gridDim.x; ++w) {
				sd += __hip_atomic_load(&b.wsum[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
			}
		}
		__syncthreads();
		if(threadIdx.x == 0) {
			int tot = 0;
			for(int w = 0; w < (int) (blockDim.x >> 6); ++w) tot += sc[w];
			b.N[j] = 1 + tot;
			b.sD[j] = sd;
			ctl->counter = 0;
		}
	}
}

// nj.c:836-1044 general path (entries < 0 are "missing"): one block walks k
// in chunks, reproducing the lagging sD/N cursor and the out-of-row read
// D_j[k] of the D_kj-only column branch (nj.c:1022).
template <int ET>
__global__ __launch_bounds__(1024) void k_update_general(typename Elem<ET>::T *__restrict__ D, int n, double bs,
                                                         TreeBufs b) {
	typedef typename Elem<ET>::T T;
	__shared__ int wsc[16];
	__shared__ double sbuf[1024];
	__shared__ int s_carry, s_cnt;
	TreeCtl *ctl = b.ctl;
	if(ctl->done) return;
	const int i = ctl->i, j = ctl->j;
	const double Dij = ctl->Dij, Li = ctl->Li, Lj = ctl->Lj;
	const long long rj = tri(j), ri = tri(i);
	if(threadIdx.x == 0) {
		s_carry = 0;
		s_cnt = 0;
	}
	__syncthreads();
	double sd = 0;   // thread 0
	for(int c0 = 0; c0 < n; c0 += blockDim.x) {
		int k = c0 + threadIdx.x;
		int br = 0;               // 0 none, 1 both, 2 Dik only, 3 Dkj only
		double Dik = 0, Dkj = 0, dd = 0, dsd = 0;
		int dN = 0;
		long long fkj = 0;
		T newv = 0;
		if(k < n && k != i && k != j) {
			long long fik = k < i ? ri + k : tri(k) + i;
			fkj = k < j ? rj + k : tri(k) + j;
			Dik = Elem<ET>::get(D[fik], bs);
			Dkj = Elem<ET>::get(D[fkj], bs);
			if(0 <= Dik && 0 <= Dkj) {
				br = 1;
				dd = (Dik + Dkj - Dij) / 2;
				dd = dd < 0 ? 0 : dd;
				newv = Elem<ET>::put(dd, 0.25, bs);
				dsd = -(Dik + Dkj - dd);
				dN = -1;
			} else if(0 <= Dik) {
				br = 2;
				dd = Dik - Li;
				newv = Elem<ET>::put(dd, 0, bs);
				dsd = -Li;
			} else if(0 <= Dkj) {
				br = 3;
				// typed "D -= Lj" (nj.c:931-940 / :1021-1030)
				T old = D[fkj];
				if(ET == 8 || ET == 4) {
					newv = (T) ((double) old - Lj);
				} else {
					newv = (T) cvt_i32_x86((double) old - (Lj * bs + 0));
				}
				if(k < j) {
					dd = Elem<ET>::get(newv, bs);
					dsd = dd - Dkj;
				} else {
					// garbage operand D_j[k] = flat element rj + k, as of serial time k
					long long g = rj + k;
					long long r = (long long) ((1.0 + sqrt(1.0 + 8.0 * (double) g)) * 0.5);
					while(tri(r) > g) --r;
					while(tri(r + 1) <= g) ++r;
					T gv;
					if(g == fkj) {
						gv = newv;                       // read after the store
					} else if(g - tri(r) == j && r > j && r < k && r >= c0 && r != i) {
						// column-j cell already rewritten earlier in this pass
						long long fir = r < i ? ri + r : tri(r) + i;
						double a = Elem<ET>::get(D[fir], bs), c = Elem<ET>::get(D[g], bs);
						if(0 <= a && 0 <= c) {
							double x = (a + c - Dij) / 2;
							gv = Elem<ET>::put(x < 0 ? 0 : x, 0.25, bs);
						} else if(0 <= a) {
							gv = Elem<ET>::put(a - Li, 0, bs);
						} else if(0 <= c) {
							T o = D[g];
							gv = (ET == 8 || ET == 4) ? (T) ((double) o - Lj) : (T) cvt_i32_x86((double) o - (Lj * bs + 0));
						} else {
							gv = D[g];
						}
					} else {
						gv = D[g];
					}
					if(ET == 8) {
						dd = (double) newv - (double) gv;
					} else if(ET == 4) {
						dd = (double) (float) ((float) newv - (float) gv);
					} else {
						dd = ((int) newv - (int) gv) / bs;
					}
					dsd = dd;
				}
				dN = -1;
			}
		}
		// ordered scan of the cursor lag: every k (other than i, j) without a branch
		bool none = (k < n && k != i && k != j && br == 0);
		unsigned long long m = __ballot(none);
		int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
		if(lane == 0) wsc[wid] = __popcll(m);
		__syncthreads();
		int pre = s_carry;
		for(int w = 0; w < wid; ++w) pre += wsc[w];
		pre += __popcll(m & ((1ull << lane) - 1));
		int tot = 0;
		for(int w = 0; w < (int) (blockDim.x >> 6); ++w) tot += wsc[w];
		__syncthreads();   // every garbage read above happened before any store below
		if(br) {
			D[fkj] = newv;
			int idx = k - pre;
			b.sD[idx] += dsd;
			b.N[idx] += dN;
			atomicAdd(&s_cnt, 1);
		}
		sbuf[threadIdx.x] = br ? dd : 0.0;
		__syncthreads();
		if(threadIdx.x == 0) {
			int lim = n - c0 < (int) blockDim.x ? n - c0 : (int) blockDim.x;
			for(int u = 0; u < lim; ++u) sd += sbuf[u];
			s_carry += tot;
		}
		__syncthreads();
	}
	if(threadIdx.x == 0) {
		b.N[j] = 1 + s_cnt;
		b.sD[j] = sd;
	}
}

// ------------------------------------------------------------------ DNJ requeue
// updateDNJ's Q/P part (dnj.c:618-709) followed by DNJ_popArrange (dnj.c:817-975)
template <int ET>
__global__ __launch_bounds__(TB) void k_dnj_requeue(typename Elem<ET>::T *__restrict__ D, int n, double bs, TreeBufs b) {
	__shared__ double sq[TB / 64];
	__shared__ int si[TB / 64];
	TreeCtl *ctl = b.ctl;
	if(ctl->done) return;
	const int i = ctl->i, j = ctl->j, nn = n - 1;
	const int Nj = b.N[j];
	const double sDj = b.sD[j];
	const bool move = i != nn;
	const int Nm = move ? b.N[nn] : 0;
	const double sDm = move ? b.sD[nn] : 0;
	int k = blockIdx.x * blockDim.x + threadIdx.x;
	double rq = DBL_MAX, pq = DBL_MAX, r2q = DBL_MAX, p2q = DBL_MAX;
	int rj = 0, pk = -1, r2j = 0, p2k = -1;
	if(k < n) {
		int Nk = b.N[k];
		double sDk = b.sD[k];
		if(k < j) {
			double d = Elem<ET>::get(D[tri(j) + k], bs);
			if(0 <= d) {
				rq = qcrit(Nj, Nk, d, sDj, sDk);
				rj = k;
			}
		}
		if(k > j && k != i) {
			double qk = b.Q[k];
			int pkk = b.P[k];
			bool upd = false;
			double d = Elem<ET>::get(D[tri(k) + j], bs);
			if(0 <= d) {
				double q = qcrit(Nj, Nk, d, sDj, sDk);
				if(q <= qk) {
					qk = q;
					pkk = j;
					upd = true;
					pq = q;
					pk = k;
				}
			}
			if(move && k > i && k < nn) {
				typename Elem<ET>::T v = D[tri(nn) + k];
				D[tri(k) + i] = v;
				double dm = Elem<ET>::get(v, bs);
				if(0 <= dm) {
					double q = qcrit(Nm, Nk, dm, sDm, sDk);
					if(q <= qk) {
						qk = q;
						pkk = i;
						upd = true;
						p2q = q;
						p2k = k;
					}
				}
			}
			if(upd) {
				b.Q[k] = qk;
				b.P[k] = pkk;
			}
		}
		if(move && k < i) {
			typename Elem<ET>::T v = D[tri(nn) + k];
			D[tri(i) + k] = v;
			double dm = Elem<ET>::get(v, bs);
			if(0 <= dm) {
				r2q = qcrit(Nm, Nk, dm, sDm, sDk);
				r2j = k;
			}
		}
	}
	// four (q, idx) block reductions -> per-block partials
	qarg_block_reduce(rq, rj, sq, si);
	qarg_block_reduce(pq, pk, sq, si);
	qarg_block_reduce(r2q, r2j, sq, si);
	qarg_block_reduce(p2q, p2k, sq, si);
	if(threadIdx.x == 0) {
		double *qp = b.qpart + 4 * blockIdx.x;
		int *ip = b.ipart + 4 * blockIdx.x;
		qp[0] = rq; ip[0] = rj;
		qp[1] = pq; ip[1] = pk;
		qp[2] = r2q; ip[2] = r2j;
		qp[3] = p2q; ip[3] = p2k;
	}
	if(last_block_arrive(&ctl->counter)) {
		if(threadIdx.x == 0) {
			double q[4] = {DBL_MAX, DBL_MAX, DBL_MAX, DBL_MAX};
			int ix[4] = {0, -1, 0, -1};
			for(unsigned w = 0; w < gridDim.x; ++w) {
				for(int t = 0; t < 4; ++t) {
					double oq = __hip_atomic_load(&b.qpart[4 * w + t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
					int oi = __hip_atomic_load(&b.ipart[4 * w + t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
					if(qarg_better(oq, oi, q[t], ix[t])) {
						q[t] = oq;
						ix[t] = oi;
					}
				}
			}
			// row j (dnj.c:619-663) and p over the lowered column entries
			b.Q[j] = q[0];
			b.P[j] = ix[0];
			int p = j;
			if(ix[1] >= 0 && qarg_better(q[1], ix[1], q[0], j)) p = ix[1];
			int p2 = 0;
			if(move) {
				b.sD[i] = sDm;
				b.N[i] = Nm;
				b.Q[i] = q[2];
				b.P[i] = ix[2];
				p2 = i;
				if(ix[3] >= 0 && qarg_better(q[3], ix[3], q[2], i)) p2 = ix[3];
			}
			ctl->mi = p;
			ctl->mj = p2;
			ctl->counter = 0;
		}
	}
}

// ------------------------------------------------------------------ NJ pop
// matrix.c:518 ltdMatrix_popArrange + nj.c:1588-1589
template <int ET>
__global__ __launch_bounds__(TB) void k_nj_pop(typename Elem<ET>::T *__restrict__ D, int n, TreeBufs b) {
	TreeCtl *ctl = b.ctl;
	if(ctl->done) return;
	const int i = ctl->i, nn = n - 1;
	if(i == nn) return;
	int k = blockIdx.x * blockDim.x + threadIdx.x;
	if(k < i) {
		D[tri(i) + k] = D[tri(nn) + k];
	} else if(k > i && k < nn) {
		D[tri(k) + i] = D[tri(nn) + k];
	}
	if(k == 0) {
		b.sD[i] = b.sD[nn];
		b.N[i] = b.N[nn];
	}
}

// ------------------------------------------------------------------ host
static inline unsigned cdiv(long long a, long long b) { return (unsigned) ((a + b - 1) / b); }

struct TreeWork {
	TreeBufs b;
	void *mem;
};

static int tree_alloc(TreeWork *w, int n) {
	size_t nb = (size_t) cdiv(n, TB) + 1;
	size_t nq = 4096;   // NJ argmin partials
	size_t sz = 0;
	auto take = [&](size_t bytes) { size_t off = sz; sz += (bytes + 255) & ~(size_t) 255; return off; };
	size_t o_sD = take(n * 8), o_Q = take(n * 8), o_fq = take(n * 8), o_c = take(n * 8);
	size_t o_N = take(n * 4), o_P = take(n * 4), o_fj = take(n * 4), o_S = take(DNJ_B * 4);
	size_t o_seg = take((size_t) n * 4 + 64), o_segc = take(REST_BLOCKS * 4);
	size_t o_ws = take(nb * 8), o_wc = take(nb * 4);
	size_t o_qp = take((nb > nq ? nb : nq) * 4 * 8), o_ip = take((nb > nq ? nb : nq) * 4 * 4);
	size_t o_ab = take(nb * 8), o_qm = take(nb * 4), o_fp = take(nq * 8);
	size_t o_j = take((size_t) n * sizeof(ccg_join)), o_ctl = take(sizeof(TreeCtl));
	char *m;
	CCG_CHECK(hipMalloc((void **) &m, sz));
	CCG_CHECK(hipMemset(m, 0, sz));
	w->mem = m;
	TreeBufs &b = w->b;
	b.sD = (double *) (m + o_sD);
	b.Q = (double *) (m + o_Q);
	b.fq = (double *) (m + o_fq);
	b.contrib = (double *) (m + o_c);
	b.N = (int *) (m + o_N);
	b.P = (int *) (m + o_P);
	b.fj = (int *) (m + o_fj);
	b.S = (int *) (m + o_S);
	b.seg = (int *) (m + o_seg);
	b.segcnt = (int *) (m + o_segc);
	b.wsum = (double *) (m + o_ws);
	b.wcnt = (int *) (m + o_wc);
	b.qpart = (double *) (m + o_qp);
	b.ipart = (int *) (m + o_ip);
	b.absb = (double *) (m + o_ab);
	b.qmin = (int *) (m + o_qm);
	b.fpart = (long long *) (m + o_fp);
	b.joins = (ccg_join *) (m + o_j);
	b.ctl = (TreeCtl *) (m + o_ctl);
	return CCG_OK;
}

template <int ET>
static int tree_run_t(ccg_ctx *ctx, const ccg_tree_args *a, void *Dd, ccg_join *joins, int *njoins,
                      int *final_n, double *final_d, int64_t *stats) {
	typedef typename Elem<ET>::T T;
	T *D = (T *) Dd;
	const int n0 = a->n;
	const double bs = a->byteScale;
	hipStream_t st = ctx->stream;
	TreeWork w;
	int rc = tree_alloc(&w, n0);
	if(rc) return rc;
	TreeBufs b = w.b;
	TreeCtl init;
	memset(&init, 0, sizeof(init));
	init.neg = (a->flags & 2) != 0;
	init.exact = a->exact != 0;
	CCG_CHECK(hipMemcpyAsync(b.ctl, &init, sizeof(init), hipMemcpyHostToDevice, st));
	long long launches = 0;
	CCG_CHECK(hipEventRecord(ctx->ev0, st));
	k_init_sums<ET><<<cdiv(n0, TB), TB, 0, st>>>(D, n0, bs, b.sD, b.N, b.ctl);
	++launches;
	if(a->method == CCG_TREE_DNJ) {
		k_init_hnj<ET><<<cdiv(n0, TB / 64), TB, 0, st>>>(D, n0, bs, b.sD, b.N, b.Q, b.P);
		k_min_q_row<<<1, TB, 0, st>>>(b.Q, n0, b.ctl);
		launches += 2;
	}
	CCG_CHECK(hipGetLastError());
	TreeCtl h;
	CCG_CHECK(hipMemcpyAsync(&h, b.ctl, sizeof(h), hipMemcpyDeviceToHost, st));
	CCG_CHECK(hipStreamSynchronize(st));
	const bool general = h.has_missing != 0;
	int n = n0;
	int since_check = 0;
	while(n != 2) {
		if(a->method == CCG_TREE_DNJ) {
			k_dnj_top<ET><<<DNJ_B, TB, 0, st>>>(D, n, bs, b);
			k_dnj_rest<ET><<<REST_BLOCKS, TB, 0, st>>>(D, n, bs, b);
			k_dnj_replay<ET><<<1, TB, 0, st>>>(D, n, bs, b, REST_BLOCKS);
			launches += 3;
		} else {
			long long cells = tri(n);
			unsigned g = cdiv(cells, 4096);
			if(g > 2048) g = 2048;
			if(g < 1) g = 1;
			long long chunk = (cells + g - 1) / g;
			k_nj_argmin<ET><<<g, TB, 0, st>>>(D, n, bs, b, chunk);
			launches += 1;
		}
		if(general) {
			k_update_general<ET><<<1, 1024, 0, st>>>(D, n, bs, b);
		} else {
			k_update<ET><<<cdiv(n, TB), TB, 0, st>>>(D, n, bs, b);
		}
		++launches;
		if(a->method == CCG_TREE_DNJ) {
			k_dnj_requeue<ET><<<cdiv(n, TB), TB, 0, st>>>(D, n, bs, b);
		} else {
			k_nj_pop<ET><<<cdiv(n, TB), TB, 0, st>>>(D, n, b);
		}
		++launches;
		CCG_CHECK(hipGetLastError());
		--n;
		if(++since_check == 512) {
			since_check = 0;
			CCG_CHECK(hipMemcpyAsync(&h, b.ctl, sizeof(h), hipMemcpyDeviceToHost, st));
			CCG_CHECK(hipStreamSynchronize(st));
			if(h.done) break;
		}
	}
	CCG_CHECK(hipEventRecord(ctx->ev1, st));
	CCG_CHECK(hipMemcpyAsync(&h, b.ctl, sizeof(h), hipMemcpyDeviceToHost, st));
	CCG_CHECK(hipStreamSynchronize(st));
	float ms = 0;
	CCG_CHECK(hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
	*njoins = h.njoins;
	*final_n = h.done ? h.final_n : n;
	if(h.njoins) {
		CCG_CHECK(hipMemcpy(joins, b.joins, (size_t) h.njoins * sizeof(ccg_join), hipMemcpyDeviceToHost));
	}
	*final_d = -1.0;
	if(*final_n == 2) {
		T v;
		CCG_CHECK(hipMemcpy(&v, D, sizeof(T), hipMemcpyDeviceToHost));
		*final_d = (ET == 8 || ET == 4) ? (double) v : v / bs;
	}
	if(stats) {
		stats[0] = h.rows;
		stats[1] = h.cells;
		stats[2] = launches;
		stats[3] = (int64_t) (ms * 1000.0);
	}
	CCG_CHECK(hipFree(w.mem));
	return CCG_OK;
}

int ccg_tree_impl(ccg_ctx *ctx, const ccg_tree_args *a, void *Dd, ccg_join *joins, int *njoins, int *final_n,
                  double *final_d, int64_t *stats) {
	switch(a->etype) {
		case 8: return tree_run_t<8>(ctx, a, Dd, joins, njoins, final_n, final_d, stats);
		case 4: return tree_run_t<4>(ctx, a, Dd, joins, njoins, final_n, final_d, stats);
		case 2: return tree_run_t<2>(ctx, a, Dd, joins, njoins, final_n, final_d, stats);
		case 1: return tree_run_t<1>(ctx, a, Dd, joins, njoins, final_n, final_d, stats);
		default: return CCG_EINVAL;
	}
}
