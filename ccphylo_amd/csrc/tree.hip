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
// P (i32).  All loop state (n, the current join, the DNJ selection) lives in
// a device TreeCtl, so every per-iteration kernel takes the same arguments;
// each one finishes with a "last block" (agent-scope ticket) that folds the
// per-block partials in a fixed order and prepares the next kernel's input.
//
// DNJ selection (minQpair) is a serial scan in the reference: row i is
// rescanned iff its stale bound Q[i] is below the running minimum m(i) of
// the rows above it.  Here, per join:
//   k_dnj_top   rescans the top-B candidate rows S (Q[r] < m0) in 2048-cell
//               units spread over the whole GPU; its last block derives
//               U = min(m0, min_{k in S} max(fresh_k, Q_k)), an upper bound of
//               m(i) for every row below S (a row k above i that the serial
//               scan rescans gives m(i) <= fresh_k, one it skips gives
//               m(i) <= m(k) <= Q_k);
//   k_dnj_rest  rescans every row below S with Q[r] < U (any other row is
//               provably skipped by the reference); its last block replays
//               the reference's accept/reject decisions over S then C1 in
//               descending row order.  When every fresh min is >= its stale
//               bound the running minimum is exactly the prefix minimum of the
//               fresh values, so the replay is a parallel scan; otherwise it
//               runs serially.  Either way Q/P and the pair are minQpair's.
#include <string.h>
#include "ccg_internal.h"

#define TB 256           // threads per block of the vector kernels
#define DNJ_B 128        // |S|: top candidate rows rescanned speculatively
#define SEG 2048         // cells per rescan unit (8 per thread)
#define RPB 16           // rows per block slice in k_dnj_rest
#define TOP_BLOCKS 1024  // grid of k_dnj_top
#define REPLAY_CAP 2048  // entries replayed from LDS at once

struct TreeCtl {
	int n;               // current matrix size
	int done;            // the reference loop stopped (pos == 0)
	int final_n;
	int njoins;
	int i, j;            // current join
	double Li, Lj, Dij;
	int cand;            // minQpair's candidate row
	int pos_i, pos_j;    // minQpair's initial pos
	double m0;           // minQpair's initial min
	double U;            // bound for rows below S
	int nS, nunits, smin;
	int mi, mj;
	int neg, exact, method;
	int serial_sums, serial_replays;
	unsigned tick[4];    // last-block tickets (reset by their last block)
	long long rows, cells;
	long long cells_top, cells_rest;
	int has_missing;
};

struct TreeBufs {
	double *sD, *Q, *fq, *contrib;
	int *N, *P, *fj;
	int *S, *uoff;       // DNJ_B rows, DNJ_B+1 unit offsets
	double *uq;          // per-unit partial (q, j)
	int *uj;
	int *blk_rows, *blk_cnt;
	double *wsum, *wabs; // per-block partial sums / sum |c|
	int *wcnt, *wexp;    // per-block count / min exponent of the contributions
	double *qpart;       // 4 (q, idx) partials per block
	int *ipart;
	long long *fpart;
	ccg_join *joins;
	TreeCtl *ctl;
};

// ------------------------------------------------------------------ helpers
__device__ __forceinline__ double lds_min_reduce(double v, double *s) {
	for(int off = 32; off > 0; off >>= 1) {
		double o = __shfl_xor(v, off, 64);
		v = o < v ? o : v;
	}
	__syncthreads();
	if((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = v;
	__syncthreads();
	v = s[0];
	for(int w = 1; w < (int) (blockDim.x >> 6); ++w) v = s[w] < v ? s[w] : v;
	__syncthreads();
	return v;
}

// block-wide exclusive prefix sum of a per-thread int; *total receives the sum
__device__ __forceinline__ int block_excl_scan(int v, int *s, int *total) {
	const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
	int x = v;
	for(int off = 1; off < 64; off <<= 1) {
		int y = __shfl_up(x, off, 64);
		if(lane >= off) x += y;
	}
	__syncthreads();
	if(lane == 63) s[wid] = x;
	__syncthreads();
	int pre = 0, tot = 0;
	for(int w = 0; w < nw; ++w) {
		if(w < wid) pre += s[w];
		tot += s[w];
	}
	__syncthreads();
	*total = tot;
	return pre + x - v;
}

// nj.c:42 limbLength / nj.c:81 limbLengthNeg
__device__ void limb_length(double *Li, double *Lj, int i, int j, const double *sD, const int *N, double Dij,
                            int neg) {
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

// (q, j) min of LT row r over columns [c0, c1), whole block, 8 loads in flight
// per thread (dnj.c:99-112 with the `<=` last-wins rule)
template <int ET, int UNR = 8>
__device__ __forceinline__ void row_segment_min(const typename Elem<ET>::T *__restrict__ D, double bs,
                                                const double *__restrict__ sD, const int *__restrict__ N, int r,
                                                int c0, int c1, double &q, int &idx) {
	const typename Elem<ET>::T *row = D + tri(r);
	const int Nr = N[r];
	const double sDr = sD[r];
	for(int base = c0; base < c1; base += UNR * TB) {
		typename Elem<ET>::T v[UNR];
		int nk[UNR];
		double sk[UNR];
#pragma unroll
		for(int m = 0; m < UNR; ++m) {
			int c = base + m * TB + (int) threadIdx.x;
			if(c < c1) {
				v[m] = row[c];
				nk[m] = N[c];
				sk[m] = sD[c];
			}
		}
#pragma unroll
		for(int m = 0; m < UNR; ++m) {
			int c = base + m * TB + (int) threadIdx.x;
			if(c < c1) {
				double d = Elem<ET>::get(v[m], bs);
				if(0 <= d) {
					double x = qcrit(Nr, nk[m], d, sDr, sk[m]);
					if(qarg_better(x, c, q, idx)) {
						q = x;
						idx = c;
					}
				}
			}
		}
	}
}

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

// ------------------------------------------------------------------ DNJ selection setup
// Computes minQpair's starting point and the top-B candidate set S for the
// current n; run by ONE block (the last block of k_dnj_requeue, or k_dnj_prep).
__device__ void prepare_selection(const TreeBufs &b, int n, int cand) {
	__shared__ int s_scan[TB / 64];
	__shared__ int s_cnt;
	TreeCtl *ctl = b.ctl;
	double m0 = DBL_MAX;
	if(cand && m0 != ld_wt(&b.Q[cand])) m0 = ld_wt(&b.Q[cand]);
	if(threadIdx.x == 0) {
		ctl->cand = cand;
		ctl->m0 = m0;
		ctl->pos_i = (cand && m0 != DBL_MAX) ? cand : 0;
		ctl->pos_j = (cand && m0 != DBL_MAX) ? ld_wt(&b.P[cand]) : 0;
		s_cnt = 0;
	}
	__syncthreads();
	// rows n-1, n-2, ... with Q[r] < m0, 4 rows per thread per step
	for(int base = n - 1; base >= 1; base -= 4 * (int) blockDim.x) {
		int cnt = s_cnt;
		if(cnt >= DNJ_B) break;
		int rows[4], k = 0;
#pragma unroll
		for(int m = 0; m < 4; ++m) {
			int r = base - 4 * (int) threadIdx.x - m;
			if(r >= 1 && ld_wt(&b.Q[r]) < m0) rows[k++] = r;
		}
		int tot;
		int off = block_excl_scan(k, s_scan, &tot);
		for(int m = 0; m < k; ++m) {
			if(cnt + off + m < DNJ_B) b.S[cnt + off + m] = rows[m];
		}
		__syncthreads();
		if(threadIdx.x == 0) s_cnt = cnt + tot;
		__syncthreads();
	}
	__threadfence_block();
	__syncthreads();
	int nS = s_cnt < DNJ_B ? s_cnt : DNJ_B;
	// rescan units per row of S
	int t = threadIdx.x;
	int u = 0;
	if(t < nS) u = (b.S[t] + SEG - 1) / SEG;
	int tot;
	int off = block_excl_scan(u, s_scan, &tot);
	if(t < nS) b.uoff[t] = off;
	if(t == 0) {
		b.uoff[nS] = tot;
		ctl->nS = nS;
		ctl->nunits = tot;
	}
}

// hclust.c:353 minQ -> the first candidate (dnj.c:997-998), then selection setup
__global__ __launch_bounds__(TB) void k_dnj_prep(TreeBufs b) {
	__shared__ double sq[TB / 64];
	__shared__ int si[TB / 64];
	const int n = b.ctl->n;
	double q = DBL_MAX;
	int idx = 0;
	for(int i = 1 + threadIdx.x; i < n; i += blockDim.x) {
		if(qarg_better(b.Q[i], i, q, idx)) {
			q = b.Q[i];
			idx = i;
		}
	}
	qarg_block_reduce(q, idx, sq, si);
	prepare_selection(b, n, idx);
}

// ------------------------------------------------------------------ DNJ rescans
template <int ET>
__global__ __launch_bounds__(TB) void k_dnj_top(const typename Elem<ET>::T *__restrict__ D, double bs, TreeBufs b) {
	__shared__ int sS[DNJ_B], so[DNJ_B + 1];
	__shared__ double sq[TB / 64];
	__shared__ int si[TB / 64];
	TreeCtl *ctl = b.ctl;
	if(ctl->done) return;
	const int nS = ctl->nS, nunits = ctl->nunits;
	for(int t = threadIdx.x; t <= nS; t += blockDim.x) {
		if(t < nS) sS[t] = b.S[t];
		so[t] = b.uoff[t];
	}
	__syncthreads();
	for(int u = blockIdx.x; u < nunits; u += gridDim.x) {
		int lo = 0, hi = nS - 1;   // last t with so[t] <= u
		while(lo < hi) {
			int mid = (lo + hi + 1) >> 1;
			if(so[mid] <= u) lo = mid; else hi = mid - 1;
		}
		int r = sS[lo];
		int c0 = (u - so[lo]) * SEG, c1 = c0 + SEG < r ? c0 + SEG : r;
		double q = DBL_MAX;
		int idx = 0;
		row_segment_min<ET>(D, bs, b.sD, b.N, r, c0, c1, q, idx);
		qarg_block_reduce(q, idx, sq, si);
		if(threadIdx.x == 0) {
			st_wt(&b.uq[u], q);
			st_wt(&b.uj[u], idx);
		}
	}
	if(!last_block_arrive(&ctl->tick[0])) return;
	// fold the units of every row of S; derive U
	double U = ctl->m0;
	long long cells = 0;
	for(int t = threadIdx.x; t < nS; t += blockDim.x) {
		double q = DBL_MAX;
		int idx = 0;
		for(int u = so[t]; u < so[t + 1]; ++u) {
			double uq = ld_wt(&b.uq[u]);
			int uj = ld_wt(&b.uj[u]);
			if(qarg_better(uq, uj, q, idx)) {
				q = uq;
				idx = uj;
			}
		}
		int r = sS[t];
		b.fq[r] = q;
		b.fj[r] = idx;
		double Qr = b.Q[r];
		double v = q > Qr ? q : Qr;
		U = v < U ? v : U;
		cells += r;
	}
	U = lds_min_reduce(U, sq);
	for(int off = 32; off > 0; off >>= 1) cells += __shfl_xor(cells, off, 64);
	if((threadIdx.x & 63) == 0 && cells) {
		atomicAdd((unsigned long long *) &ctl->cells, (unsigned long long) cells);
		atomicAdd((unsigned long long *) &ctl->cells_top, (unsigned long long) cells);
	}
	if(threadIdx.x == 0) {
		ctl->U = U;
		ctl->smin = nS == DNJ_B ? sS[DNJ_B - 1] : 1;
		ctl->rows += nS;
		ctl->tick[0] = 0;
	}
}

template <int ET>
__global__ __launch_bounds__(TB) void k_dnj_rest(const typename Elem<ET>::T *__restrict__ D, double bs, TreeBufs b) {
	__shared__ double sq[TB / 64];
	__shared__ int si[TB / 64];
	__shared__ int scan[TB / 64];
	__shared__ double wmin[TB / 64];
	__shared__ int list[RPB];
	__shared__ int s_cnt;
	__shared__ int e_row[REPLAY_CAP], e_j[REPLAY_CAP];
	__shared__ double e_b[REPLAY_CAP], e_f[REPLAY_CAP];
	__shared__ int s_pi, s_pj;
	TreeCtl *ctl = b.ctl;
	if(ctl->done) return;
	const int smin = ctl->smin;
	const double U = ctl->U;
	const int nblk = (smin - 1 + RPB - 1) / RPB;   // slices of rows [1, smin)
	const int w = blockIdx.x;
	const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
	for(int sl = w; sl < nblk; sl += gridDim.x) {
		int lo = 1 + sl * RPB, hi = lo + RPB < smin ? lo + RPB : smin;
		if(threadIdx.x < 64) {
			int r = hi - 1 - (int) threadIdx.x;
			bool f = r >= lo && b.Q[r] < U;
			unsigned long long m = __ballot(f);
			if(f) list[__popcll(m & ((1ull << threadIdx.x) - 1))] = r;
			if(threadIdx.x == 0) s_cnt = __popcll(m);
		}
		__syncthreads();
		const int cnt = s_cnt;
		long long cells = 0;
		for(int t = 0; t < cnt; ++t) {
			int r = list[t];
			double q = DBL_MAX;
			int idx = 0;
			row_segment_min<ET, 16>(D, bs, b.sD, b.N, r, 0, r, q, idx);
			qarg_block_reduce(q, idx, sq, si);
			if(threadIdx.x == 0) {
				st_wt(&b.fq[r], q);
				st_wt(&b.fj[r], idx);
				st_wt(&b.blk_rows[sl * RPB + t], r);
			}
			cells += r;
		}
		if(threadIdx.x == 0) {
			st_wt(&b.blk_cnt[sl], cnt);
			if(cnt) {
				atomicAdd((unsigned long long *) &ctl->cells, (unsigned long long) cells);
				atomicAdd((unsigned long long *) &ctl->cells_rest, (unsigned long long) cells);
				atomicAdd((unsigned long long *) &ctl->rows, (unsigned long long) cnt);
			}
		}
		__syncthreads();
	}
	if(!last_block_arrive(&ctl->tick[1])) return;

	// ---- replay of minQpair's decisions: S (descending) then slices nblk-1 .. 0
	const int nS = ctl->nS;
	const double m0 = ctl->m0;
	if(threadIdx.x == 0) {
		s_pi = ctl->pos_i;
		s_pj = ctl->pos_j;
	}
	int carry = nS;
	for(int c0 = 0; c0 < nblk; c0 += blockDim.x) {
		int t = c0 + threadIdx.x;
		int c = t < nblk ? ld_wt(&b.blk_cnt[nblk - 1 - t]) : 0;
		int tot;
		int off = block_excl_scan(c, scan, &tot);
		for(int k = 0; k < c; ++k) {
			int e = carry + off + k;
			if(e < REPLAY_CAP) e_row[e] = ld_wt(&b.blk_rows[(nblk - 1 - t) * RPB + k]);
		}
		carry += tot;
	}
	for(int t = threadIdx.x; t < nS; t += blockDim.x) e_row[t] = b.S[t];
	const int total = carry;
	__syncthreads();
	if(total <= REPLAY_CAP) {
		// gather (bound, fresh, j) and test the prefix-min condition fresh >= bound
		int bad = 0;
		for(int e = threadIdx.x; e < total; e += blockDim.x) {
			int r = e_row[e];
			double bq = b.Q[r], fq = ld_wt(&b.fq[r]);
			e_b[e] = bq;
			e_f[e] = fq;
			e_j[e] = ld_wt(&b.fj[r]);
			bad |= !(fq >= bq);
		}
		bad = __syncthreads_or(bad);
		if(!bad) {
			// running min before entry e = min(m0, f[0..e-1]); accepted iff bound < it
			double carry_m = m0;
			for(int c0 = 0; c0 < total; c0 += blockDim.x) {
				int e = c0 + threadIdx.x;
				double f = e < total ? e_f[e] : DBL_MAX;
				double x = f;   // inclusive wave min-scan
				for(int off = 1; off < 64; off <<= 1) {
					double y = __shfl_up(x, off, 64);
					if(lane >= off) x = y < x ? y : x;
				}
				if(lane == 63) wmin[wid] = x;
				__syncthreads();
				double pre = carry_m;
				for(int k = 0; k < wid; ++k) pre = wmin[k] < pre ? wmin[k] : pre;
				double excl = __shfl_up(x, 1, 64);
				if(lane > 0) pre = excl < pre ? excl : pre;
				double chunk_min = carry_m;
				for(int k = 0; k < (int) (blockDim.x >> 6); ++k) chunk_min = wmin[k] < chunk_min ? wmin[k] : chunk_min;
				if(e < total && e_b[e] < pre) {
					int r = e_row[e];
					b.Q[r] = f;
					b.P[r] = e_j[e];
				}
				__syncthreads();
				carry_m = chunk_min;
			}
			// the pair: first entry reaching the final minimum, if below m0
			double q = DBL_MAX;
			int idx = 0x7fffffff;
			for(int e = threadIdx.x; e < total; e += blockDim.x) {
				double f = e_f[e];
				if(f < q || (f == q && e < idx)) {
					q = f;
					idx = e;
				}
			}
			for(int off = 32; off > 0; off >>= 1) {
				double oq = __shfl_xor(q, off, 64);
				int oi = __shfl_xor(idx, off, 64);
				if(oq < q || (oq == q && oi < idx)) {
					q = oq;
					idx = oi;
				}
			}
			if(lane == 0) {
				sq[wid] = q;
				si[wid] = idx;
			}
			__syncthreads();
			if(threadIdx.x == 0) {
				for(int k = 1; k < (int) (blockDim.x >> 6); ++k) {
					if(sq[k] < q || (sq[k] == q && si[k] < idx)) {
						q = sq[k];
						idx = si[k];
					}
				}
				if(total && q < m0) {
					s_pi = e_row[idx];
					s_pj = e_j[idx];
				}
			}
			__syncthreads();
		} else {
			if(threadIdx.x == 0) {
				double m = m0;
				int pi = s_pi, pj = s_pj;
				for(int e = 0; e < total; ++e) {
					if(e_b[e] < m) {
						int r = e_row[e];
						b.Q[r] = e_f[e];
						b.P[r] = e_j[e];
						if(e_f[e] < m) {
							m = e_f[e];
							pi = r;
							pj = e_j[e];
						}
					}
				}
				s_pi = pi;
				s_pj = pj;
				ctl->serial_replays++;
			}
			__syncthreads();
		}
	} else if(threadIdx.x == 0) {
		// very large candidate sets: serial replay straight from global memory
		double m = m0;
		int pi = s_pi, pj = s_pj;
		int t = 0, k = 0;
		for(int e = 0; e < total; ++e) {
			int r;
			if(e < nS) {
				r = b.S[e];
			} else {
				while(k >= ld_wt(&b.blk_cnt[nblk - 1 - t])) {
					++t;
					k = 0;
				}
				r = ld_wt(&b.blk_rows[(nblk - 1 - t) * RPB + k]);
				++k;
			}
			if(b.Q[r] < m) {
				double f = ld_wt(&b.fq[r]);
				int fj = ld_wt(&b.fj[r]);
				b.Q[r] = f;
				b.P[r] = fj;
				if(f < m) {
					m = f;
					pi = r;
					pj = fj;
				}
			}
		}
		s_pi = pi;
		s_pj = pj;
		ctl->serial_replays++;
	}
	__syncthreads();
	if(threadIdx.x == 0) {
		ctl->tick[1] = 0;
		if(s_pi == 0 && s_pj == 0) {
			ctl->done = 1;
			ctl->final_n = ctl->n;
		} else {
			record_join<ET>(D, bs, b, s_pi, s_pj);
		}
	}
}

// ------------------------------------------------------------------ NJ argmin
// nj.c:182 initQ: min starts at 1, the last minimal cell in row-major order
template <int ET>
__global__ __launch_bounds__(TB) void k_nj_argmin(const typename Elem<ET>::T *__restrict__ D, double bs, TreeBufs b) {
	__shared__ double sq[TB / 64];
	__shared__ long long sf[TB / 64];
	TreeCtl *ctl = b.ctl;
	if(ctl->done) return;
	const int n = ctl->n;
	const long long cells = tri(n);
	const long long chunk = (cells + gridDim.x - 1) / gridDim.x;
	const long long f0 = (long long) blockIdx.x * chunk;
	const long long f1 = f0 + chunk < cells ? f0 + chunk : cells;
	double bq = 1.0;
	long long bf = -1;
	if(f0 < f1) {
		long long f = f0 + threadIdx.x;
		long long r = (long long) ((1.0 + sqrt(1.0 + 8.0 * (double) f)) * 0.5);
		while(r > 1 && tri(r) > f) --r;
		while(tri(r + 1) <= f) ++r;
		long long c = f - tri(r);
		for(; f < f1; f += 4 * TB) {
			// four cells of this thread: f, f+TB, f+2TB, f+3TB
			typename Elem<ET>::T v[4];
			int nr[4], nc[4];
			double sr[4], sc[4];
#pragma unroll
			for(int m = 0; m < 4; ++m) {
				if(f + m * TB < f1) {
					v[m] = D[f + m * TB];
					nr[m] = b.N[r];
					sr[m] = b.sD[r];
					nc[m] = b.N[c];
					sc[m] = b.sD[c];
				}
				c += TB;
				while(c >= r && r < n) {
					c -= r;
					++r;
				}
			}
#pragma unroll
			for(int m = 0; m < 4; ++m) {
				long long fm = f + m * TB;
				if(fm < f1) {
					double d = Elem<ET>::get(v[m], bs);
					if(0 <= d) {
						double q = qcrit(nr[m], nc[m], d, sr[m], sc[m]);
						if(q < bq || (q == bq && fm > bf)) {
							bq = q;
							bf = fm;
						}
					}
				}
			}
		}
	}
	// block reduce (min q, max f)
	for(int off = 32; off > 0; off >>= 1) {
		double oq = __shfl_xor(bq, off, 64);
		long long of = __shfl_xor(bf, off, 64);
		if(oq < bq || (oq == bq && of > bf)) {
			bq = oq;
			bf = of;
		}
	}
	const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
	if(lane == 0) {
		sq[wid] = bq;
		sf[wid] = bf;
	}
	__syncthreads();
	if(threadIdx.x == 0) {
		for(int k = 1; k < (int) (blockDim.x >> 6); ++k) {
			if(sq[k] < bq || (sq[k] == bq && sf[k] > bf)) {
				bq = sq[k];
				bf = sf[k];
			}
		}
		st_wt(&b.qpart[blockIdx.x], bq);
		st_wt(&b.fpart[blockIdx.x], bf);
	}
	if(!last_block_arrive(&ctl->tick[1])) return;
	bq = 1.0;
	bf = -1;
	for(unsigned k = threadIdx.x; k < gridDim.x; k += blockDim.x) {
		double oq = ld_wt(&b.qpart[k]);
		long long of = ld_wt(&b.fpart[k]);
		if(oq < bq || (oq == bq && of > bf)) {
			bq = oq;
			bf = of;
		}
	}
	for(int off = 32; off > 0; off >>= 1) {
		double oq = __shfl_xor(bq, off, 64);
		long long of = __shfl_xor(bf, off, 64);
		if(oq < bq || (oq == bq && of > bf)) {
			bq = oq;
			bf = of;
		}
	}
	__syncthreads();
	if(lane == 0) {
		sq[wid] = bq;
		sf[wid] = bf;
	}
	__syncthreads();
	if(threadIdx.x == 0) {
		for(int k = 1; k < (int) (blockDim.x >> 6); ++k) {
			if(sq[k] < bq || (sq[k] == bq && sf[k] > bf)) {
				bq = sq[k];
				bf = sf[k];
			}
		}
		ctl->tick[1] = 0;
		if(bf < 0) {
			ctl->done = 1;
			ctl->final_n = n;
		} else {
			long long r = (long long) ((1.0 + sqrt(1.0 + 8.0 * (double) bf)) * 0.5);
			while(r > 1 && tri(r) > bf) --r;
			while(tri(r + 1) <= bf) ++r;
			record_join<ET>(D, bs, b, (int) r, (int) (bf - tri(r)));
		}
	}
}

// ------------------------------------------------------------------ updateD
// exponent e of the lowest set bit of x (x = odd * 2^e); INT32_MAX for 0,
// INT32_MIN for inf / NaN
__device__ __forceinline__ int low_exp(double x) {
	unsigned long long u = (unsigned long long) __double_as_longlong(x);
	int ex = (int) ((u >> 52) & 0x7FF);
	unsigned long long m = u & ((1ull << 52) - 1);
	if(ex == 0x7FF) return INT32_MIN;
	if(ex == 0) {
		if(m == 0) return INT32_MAX;
		return -1074 + __ffsll((long long) m) - 1;
	}
	m |= 1ull << 52;
	return ex - 1075 + __ffsll((long long) m) - 1;
}

// nj.c:836-1044 without missing entries: every k takes the (D_ik, D_kj >= 0)
// branch, so the sD/N cursor never lags.  The new row sum sD[j] is the
// reference's serial sum over k (exact mode) or a fixed-order tree sum; both
// are the same number whenever every partial sum is exactly representable
// (all terms multiples of 2^e and sum |c| < 2^53 * 2^e), e.g. integer SNP data.
template <int ET>
__global__ __launch_bounds__(TB) void k_update(typename Elem<ET>::T *__restrict__ D, double bs, TreeBufs b) {
	__shared__ double ssum[TB / 64], sabs[TB / 64];
	__shared__ int scnt[TB / 64], sexp[TB / 64];
	__shared__ double buf[8 * TB];
	__shared__ double red[1024];
	TreeCtl *ctl = b.ctl;
	if(ctl->done) return;
	const int n = ctl->n, i = ctl->i, j = ctl->j;
	const double Dij = ctl->Dij;
	const int k = blockIdx.x * blockDim.x + threadIdx.x;
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
	const bool exact = ctl->exact;
	if(exact && k < n) st_wt(&b.contrib[k], d);
	double s = d, a = fabs(d);
	int e = low_exp(d);
	for(int off = 32; off > 0; off >>= 1) {
		s += __shfl_down(s, off, 64);
		a += __shfl_down(a, off, 64);
		cnt += __shfl_down(cnt, off, 64);
		int oe = __shfl_down(e, off, 64);
		e = oe < e ? oe : e;
	}
	const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
	if(lane == 0) {
		ssum[wid] = s;
		sabs[wid] = a;
		scnt[wid] = cnt;
		sexp[wid] = e;
	}
	__syncthreads();
	if(threadIdx.x == 0) {
		double t = 0, ta = 0;
		int c = 0, te = INT32_MAX;
		for(int w = 0; w < (int) (blockDim.x >> 6); ++w) {
			t += ssum[w];
			ta += sabs[w];
			c += scnt[w];
			te = sexp[w] < te ? sexp[w] : te;
		}
		st_wt(&b.wsum[blockIdx.x], t);
		st_wt(&b.wabs[blockIdx.x], ta);
		st_wt(&b.wcnt[blockIdx.x], c);
		st_wt(&b.wexp[blockIdx.x], te);
	}
	if(!last_block_arrive(&ctl->tick[2])) return;
	// fixed-order fold of the block partials: 1024 leaves (block g -> leaf
	// g mod 1024, folded in order), then a pairwise tree
	const int G = gridDim.x;
	for(int leaf = threadIdx.x; leaf < 1024; leaf += blockDim.x) {
		double v = 0;
		for(int g = leaf; g < G; g += 1024) v += ld_wt(&b.wsum[g]);
		red[leaf] = v;
	}
	double tabs = 0;
	int tcnt = 0, texp = INT32_MAX;
	for(int g = threadIdx.x; g < G; g += blockDim.x) {
		tabs += ld_wt(&b.wabs[g]);
		tcnt += ld_wt(&b.wcnt[g]);
		int oe = ld_wt(&b.wexp[g]);
		texp = oe < texp ? oe : texp;
	}
	__syncthreads();
	for(int stride = 512; stride > 0; stride >>= 1) {
		for(int leaf = threadIdx.x; leaf < stride; leaf += blockDim.x) red[leaf] += red[leaf + stride];
		__syncthreads();
	}
	const double total = red[0];
	for(int off = 32; off > 0; off >>= 1) {
		tabs += __shfl_xor(tabs, off, 64);
		tcnt += __shfl_xor(tcnt, off, 64);
		int oe = __shfl_xor(texp, off, 64);
		texp = oe < texp ? oe : texp;
	}
	__syncthreads();
	if(lane == 0) {
		sabs[wid] = tabs;
		scnt[wid] = tcnt;
		sexp[wid] = texp;
	}
	__syncthreads();
	tabs = 0;
	tcnt = 0;
	texp = INT32_MAX;
	for(int w = 0; w < (int) (blockDim.x >> 6); ++w) {
		tabs += sabs[w];
		tcnt += scnt[w];
		texp = sexp[w] < texp ? sexp[w] : texp;
	}
	double sd = total;
	if(exact) {
		bool provable = texp != INT32_MIN &&
		                (texp == INT32_MAX || (texp > -1000 && tabs * (1.0 + 1e-9) < ldexp(1.0, 53 + texp)));
		if(!provable) {
			// the reference's serial sum in increasing k (nj.c:911 / :1002)
			sd = 0;
			double nxt[4];
#pragma unroll
			for(int m = 0; m < 4; ++m) {
				int kk = m * TB + threadIdx.x;
				buf[m * TB + threadIdx.x] = kk < n ? ld_wt(&b.contrib[kk]) : 0.0;
			}
			__syncthreads();
			for(int c0 = 0, p = 0; c0 < n; c0 += 4 * TB, p ^= 1) {
				// fetch the next chunk while thread 0 runs the serial chain
#pragma unroll
				for(int m = 0; m < 4; ++m) {
					int kk = c0 + 4 * TB + m * TB + threadIdx.x;
					nxt[m] = kk < n ? ld_wt(&b.contrib[kk]) : 0.0;
				}
				if(threadIdx.x == 0) {
					const double *cur = buf + p * 4 * TB;
					int lim = n - c0 < 4 * TB ? n - c0 : 4 * TB;
					for(int u = 0; u < lim; ++u) sd += cur[u];
				}
#pragma unroll
				for(int m = 0; m < 4; ++m) buf[(p ^ 1) * 4 * TB + m * TB + threadIdx.x] = nxt[m];
				__syncthreads();
			}
			if(threadIdx.x == 0) ctl->serial_sums++;
		}
	}
	if(threadIdx.x == 0) {
		b.N[j] = 1 + tcnt;
		b.sD[j] = sd;
		ctl->tick[2] = 0;
	}
}

// nj.c:836-1044 general path (entries < 0 are "missing"): one block walks k
// in chunks, reproducing the lagging sD/N cursor and the out-of-row read
// D_j[k] of the D_kj-only column branch (nj.c:1022).
template <int ET>
__global__ __launch_bounds__(1024) void k_update_general(typename Elem<ET>::T *__restrict__ D, double bs, TreeBufs b) {
	typedef typename Elem<ET>::T T;
	__shared__ int wsc[16];
	__shared__ double sbuf[1024];
	__shared__ int s_carry, s_cnt;
	TreeCtl *ctl = b.ctl;
	if(ctl->done) return;
	const int n = ctl->n;
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
// updateDNJ's Q/P part (dnj.c:618-709) followed by DNJ_popArrange
// (dnj.c:817-975) and minPos (dnj.c:1026-1032); the last block folds the four
// (q, idx) reductions, shrinks n and prepares the next minQpair.
template <int ET>
__global__ __launch_bounds__(TB) void k_dnj_requeue(typename Elem<ET>::T *__restrict__ D, double bs, TreeBufs b) {
	__shared__ double sq[TB / 64];
	__shared__ int si[TB / 64];
	__shared__ int s_cand;
	TreeCtl *ctl = b.ctl;
	if(ctl->done) return;
	const int n = ctl->n, i = ctl->i, j = ctl->j, nn = n - 1;
	const int Nj = b.N[j];
	const double sDj = b.sD[j];
	const bool move = i != nn;
	const int Nm = move ? b.N[nn] : 0;
	const double sDm = move ? b.sD[nn] : 0;
	const int k = blockIdx.x * blockDim.x + threadIdx.x;
	double rq = DBL_MAX, pq = DBL_MAX, r2q = DBL_MAX, p2q = DBL_MAX;
	int rj = 0, pk = -1, r2j = 0, p2k = -1;
	if(k < n) {
		const int Nk = b.N[k];
		const double sDk = b.sD[k];
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
				st_wt(&b.Q[k], qk);
				st_wt(&b.P[k], pkk);
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
	qarg_block_reduce(rq, rj, sq, si);
	qarg_block_reduce(pq, pk, sq, si);
	qarg_block_reduce(r2q, r2j, sq, si);
	qarg_block_reduce(p2q, p2k, sq, si);
	if(threadIdx.x == 0) {
		double *qp = b.qpart + 4 * blockIdx.x;
		int *ip = b.ipart + 4 * blockIdx.x;
		st_wt(&qp[0], rq); st_wt(&ip[0], rj);
		st_wt(&qp[1], pq); st_wt(&ip[1], pk);
		st_wt(&qp[2], r2q); st_wt(&ip[2], r2j);
		st_wt(&qp[3], p2q); st_wt(&ip[3], p2k);
	}
	if(!last_block_arrive(&ctl->tick[3])) return;
	double q[4] = {DBL_MAX, DBL_MAX, DBL_MAX, DBL_MAX};
	int ix[4] = {0, -1, 0, -1};
	for(unsigned w = threadIdx.x; w < gridDim.x; w += blockDim.x) {
#pragma unroll
		for(int t = 0; t < 4; ++t) {
			double oq = ld_wt(&b.qpart[4 * w + t]);
			int oi = ld_wt(&b.ipart[4 * w + t]);
			if(qarg_better(oq, oi, q[t], ix[t])) {
				q[t] = oq;
				ix[t] = oi;
			}
		}
	}
#pragma unroll
	for(int t = 0; t < 4; ++t) qarg_block_reduce(q[t], ix[t], sq, si);
	if(threadIdx.x == 0) {
		// row j (dnj.c:619-663) and p over the lowered column entries
		st_wt(&b.Q[j], q[0]);
		st_wt(&b.P[j], ix[0]);
		int p = j;
		if(ix[1] >= 0 && qarg_better(q[1], ix[1], q[0], j)) p = ix[1];
		int p2 = 0;
		if(move) {
			b.sD[i] = sDm;
			b.N[i] = Nm;
			st_wt(&b.Q[i], q[2]);
			st_wt(&b.P[i], ix[2]);
			p2 = i;
			if(ix[3] >= 0 && qarg_better(q[3], ix[3], q[2], i)) p2 = ix[3];
		}
		ctl->mi = p;
		ctl->mj = p2;
		ctl->n = nn;
		ctl->tick[3] = 0;
		// dnj.c:1026-1032: next candidate row
		int cand;
		if(p2 == nn) cand = p;
		else if(p == nn) cand = p2;
		else {
			double Qp = ld_wt(&b.Q[p]), Qp2 = ld_wt(&b.Q[p2]);
			cand = (Qp2 < Qp || (p < p2 && Qp2 == Qp)) ? p2 : p;
		}
		s_cand = cand;
	}
	asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
	__syncthreads();
	if(nn > 2) prepare_selection(b, nn, s_cand);
}

// ------------------------------------------------------------------ NJ pop
// matrix.c:518 ltdMatrix_popArrange + nj.c:1588-1589
template <int ET>
__global__ __launch_bounds__(TB) void k_nj_pop(typename Elem<ET>::T *__restrict__ D, TreeBufs b) {
	TreeCtl *ctl = b.ctl;
	if(ctl->done) return;
	const int n = ctl->n, i = ctl->i, nn = n - 1;
	const int k = blockIdx.x * blockDim.x + threadIdx.x;
	if(i != nn) {
		if(k < i) {
			D[tri(i) + k] = D[tri(nn) + k];
		} else if(k > i && k < nn) {
			D[tri(k) + i] = D[tri(nn) + k];
		}
	}
	if(!last_block_arrive(&ctl->tick[3])) return;
	if(threadIdx.x == 0) {
		if(i != nn) {
			b.sD[i] = b.sD[nn];
			b.N[i] = b.N[nn];
		}
		ctl->n = nn;
		ctl->tick[3] = 0;
	}
}

// ------------------------------------------------------------------ host
static inline unsigned cdiv(long long a, long long b) { return (unsigned) ((a + b - 1) / b); }

struct TreeWork {
	TreeBufs b;
	void *mem;
};

static int tree_alloc(TreeWork *w, int n, hipStream_t st) {
	const size_t nb = (size_t) cdiv(n, TB) + 1;
	const size_t maxunits = (size_t) DNJ_B * (cdiv(n, SEG) + 1);
	const size_t nslices = (size_t) cdiv(n, RPB) + 1;
	const size_t nq = 4096;
	size_t sz = 0;
	auto take = [&](size_t bytes) {
		size_t off = sz;
		sz += (bytes + 255) & ~(size_t) 255;
		return off;
	};
	size_t o_sD = take(n * 8), o_Q = take(n * 8), o_fq = take(n * 8), o_c = take(n * 8);
	size_t o_N = take(n * 4), o_P = take(n * 4), o_fj = take(n * 4);
	size_t o_S = take(DNJ_B * 4), o_uo = take((DNJ_B + 1) * 4);
	size_t o_uq = take(maxunits * 8), o_uj = take(maxunits * 4);
	size_t o_br = take(nslices * RPB * 4), o_bc = take(nslices * 4);
	size_t o_ws = take(nb * 8), o_wa = take(nb * 8), o_wc = take(nb * 4), o_we = take(nb * 4);
	size_t o_qp = take((nb > nq ? nb : nq) * 4 * 8), o_ip = take((nb > nq ? nb : nq) * 4 * 4);
	size_t o_fp = take(nq * 8);
	size_t o_j = take((size_t) n * sizeof(ccg_join)), o_ctl = take(sizeof(TreeCtl));
	char *m;
	CCG_CHECK(hipMalloc((void **) &m, sz));
	CCG_CHECK(hipMemsetAsync(m, 0, sz, st));
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
	b.uoff = (int *) (m + o_uo);
	b.uq = (double *) (m + o_uq);
	b.uj = (int *) (m + o_uj);
	b.blk_rows = (int *) (m + o_br);
	b.blk_cnt = (int *) (m + o_bc);
	b.wsum = (double *) (m + o_ws);
	b.wabs = (double *) (m + o_wa);
	b.wcnt = (int *) (m + o_wc);
	b.wexp = (int *) (m + o_we);
	b.qpart = (double *) (m + o_qp);
	b.ipart = (int *) (m + o_ip);
	b.fpart = (long long *) (m + o_fp);
	b.joins = (ccg_join *) (m + o_j);
	b.ctl = (TreeCtl *) (m + o_ctl);
	return CCG_OK;
}

// Per-kernel HIP-event timing (profile mode): one event after every launch,
// harvested in batches.
struct KTimer {
	bool on;
	hipStream_t st;
	hipEvent_t ev[1025];
	int cls[1025];
	int used;
	long long cnt[CCG_NKSTAT], ns[CCG_NKSTAT];
	void init(hipStream_t s, bool enable) {
		on = enable;
		st = s;
		used = 0;
		memset(cnt, 0, sizeof(cnt));
		memset(ns, 0, sizeof(ns));
		if(on) {
			for(int k = 0; k < 1025; ++k) hipEventCreate(&ev[k]);
			hipEventRecord(ev[0], st);
			used = 1;
		}
	}
	void harvest() {
		hipEventSynchronize(ev[used - 1]);
		for(int k = 1; k < used; ++k) {
			float ms = 0;
			hipEventElapsedTime(&ms, ev[k - 1], ev[k]);
			cnt[cls[k]] += 1;
			ns[cls[k]] += (long long) (ms * 1.0e6);
		}
		hipEvent_t t = ev[0];
		ev[0] = ev[used - 1];
		ev[used - 1] = t;
		used = 1;
	}
	void mark(int c) {
		if(!on) return;
		cls[used] = c;
		hipEventRecord(ev[used++], st);
		if(used == 1025) harvest();
	}
	void finish() {
		if(!on) return;
		harvest();
		for(int k = 0; k < 1025; ++k) hipEventDestroy(ev[k]);
	}
};

// One join's kernels, for a matrix of (at most) n taxa.
template <int ET>
static void enqueue_iteration(hipStream_t st, typename Elem<ET>::T *D, double bs, const TreeBufs &b, int n,
                              int method, bool general, KTimer &kt) {
	if(method == CCG_TREE_DNJ) {
		k_dnj_top<ET><<<TOP_BLOCKS, TB, 0, st>>>(D, bs, b);
		kt.mark(CCG_K_TOP);
		unsigned g2 = cdiv(n, RPB);
		if(g2 > 2048) g2 = 2048;
		k_dnj_rest<ET><<<g2, TB, 0, st>>>(D, bs, b);
		kt.mark(CCG_K_REST);
	} else {
		long long cells = tri(n);
		unsigned g = cdiv(cells, 8 * TB);
		if(g > 2048) g = 2048;
		if(g < 1) g = 1;
		k_nj_argmin<ET><<<g, TB, 0, st>>>(D, bs, b);
		kt.mark(CCG_K_ARGMIN);
	}
	if(general) {
		k_update_general<ET><<<1, 1024, 0, st>>>(D, bs, b);
	} else {
		k_update<ET><<<cdiv(n, TB), TB, 0, st>>>(D, bs, b);
	}
	kt.mark(CCG_K_UPDATE);
	if(method == CCG_TREE_DNJ) {
		k_dnj_requeue<ET><<<cdiv(n, TB), TB, 0, st>>>(D, bs, b);
		kt.mark(CCG_K_REQUEUE);
	} else {
		k_nj_pop<ET><<<cdiv(n, TB), TB, 0, st>>>(D, b);
		kt.mark(CCG_K_POP);
	}
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
	int rc = tree_alloc(&w, n0, st);
	if(rc) return rc;
	TreeBufs b = w.b;
	TreeCtl init;
	memset(&init, 0, sizeof(init));
	init.n = n0;
	init.neg = (a->flags & 2) != 0;
	init.exact = a->exact != 0;
	init.method = a->method;
	CCG_CHECK(hipMemcpyAsync(b.ctl, &init, sizeof(init), hipMemcpyHostToDevice, st));
	long long launches = 0;
	static KTimer kt;
	CCG_CHECK(hipEventRecord(ctx->ev0, st));
	kt.init(st, a->profile != 0);
	k_init_sums<ET><<<cdiv(n0, TB), TB, 0, st>>>(D, n0, bs, b.sD, b.N, b.ctl);
	++launches;
	if(a->method == CCG_TREE_DNJ) {
		k_init_hnj<ET><<<cdiv(n0, TB / 64), TB, 0, st>>>(D, n0, bs, b.sD, b.N, b.Q, b.P);
		k_dnj_prep<<<1, TB, 0, st>>>(b);
		launches += 2;
	}
	kt.mark(CCG_K_INIT);
	CCG_CHECK(hipGetLastError());
	TreeCtl h;
	CCG_CHECK(hipMemcpyAsync(&h, b.ctl, sizeof(h), hipMemcpyDeviceToHost, st));
	CCG_CHECK(hipStreamSynchronize(st));
	const bool general = h.has_missing != 0;
	int n = n0;
	int since_check = 0;
	while(n != 2) {
		enqueue_iteration<ET>(st, D, bs, b, n, a->method, general, kt);
		launches += a->method == CCG_TREE_DNJ ? 4 : 3;
		CCG_CHECK(hipGetLastError());
		--n;
		if(++since_check == 1024) {
			since_check = 0;
			CCG_CHECK(hipMemcpyAsync(&h, b.ctl, sizeof(h), hipMemcpyDeviceToHost, st));
			CCG_CHECK(hipStreamSynchronize(st));
			if(h.done) break;
		}
	}
	CCG_CHECK(hipEventRecord(ctx->ev1, st));
	kt.finish();
	CCG_CHECK(hipMemcpyAsync(&h, b.ctl, sizeof(h), hipMemcpyDeviceToHost, st));
	CCG_CHECK(hipStreamSynchronize(st));
	float ms = 0;
	CCG_CHECK(hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
	*njoins = h.njoins;
	*final_n = h.done ? h.final_n : h.n;
	if(h.njoins) {
		CCG_CHECK(hipMemcpyAsync(joins, b.joins, (size_t) h.njoins * sizeof(ccg_join), hipMemcpyDeviceToHost, st));
	}
	*final_d = -1.0;
	if(*final_n == 2) {
		T v;
		CCG_CHECK(hipMemcpyAsync(&v, D, sizeof(T), hipMemcpyDeviceToHost, st));
		CCG_CHECK(hipStreamSynchronize(st));
		*final_d = (ET == 8 || ET == 4) ? (double) v : v / bs;
	}
	if(stats) {
		stats[0] = h.rows;
		stats[1] = h.cells;
		stats[2] = launches;
		stats[3] = (int64_t) (ms * 1000.0);
		if(a->profile) {
			for(int c = 0; c < CCG_NKSTAT; ++c) {
				stats[4 + 2 * c] = kt.cnt[c];
				stats[5 + 2 * c] = kt.ns[c];
			}
			stats[4 + 2 * CCG_NKSTAT] = h.cells_top;
			stats[5 + 2 * CCG_NKSTAT] = h.cells_rest;
		}
	}
	CCG_CHECK(hipStreamSynchronize(st));
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
