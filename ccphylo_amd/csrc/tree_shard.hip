// tree_shard.hip -- NJ (nj.c:1560 loop, -t 1 semantics) over an LT matrix
// whose rows are split across ranks, one process per GPU.
//
// Ownership: bands of CCG_SHARD_BAND (= NJ_RB) rows dealt round-robin; a rank
// keeps its rows back to back (Shard::off).  sD and N are replicated and every
// rank updates them identically, so the only exchanges per join are two
// allreduces:
//   1. the per-rank argmin records (initQ nj.c:182): a world x 16-byte array
//      in which each rank fills its own slot; every rank folds the records in
//      rank order with initQ's total order (smaller q, then larger flat
//      index), so all ranks pick the same (i, j).  Row n-1 (it moves to slot
//      i in the pop, matrix.c:518) rides behind the records: its owner copies
//      it there, the other ranks write zeros (k_sh_xm);
//   3. lines i and j (D_ik, D_jk for every k): each rank contributes the
//      entries its rows hold and zeros elsewhere, so the bytewise sum is a
//      gather.  Every rank then computes the whole updated line j
//      (updateD nj.c:836) and the new row sum of j itself -- with the same
//      fixed-order partials as the single-GPU engine (ccg_tree_common.h) --
//      and stores the entries of its own rows.
// The initial row sums (initSummaD nj.c:111, serial in increasing m) are
// exact too: owners sum their rows' row parts, and the column parts are
// continued serially from column chunks gathered the same way.  The joins are
// therefore bit-identical to ccg_tree's for every world size.
#include <dlfcn.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <rccl/rccl.h>
#define CCG_DNJ_NO_TRACE
#include "ccg_tree_common.h"
#include "ccg_shard.h"
#include "ccg_dnj_search.h"   // k_init_hnj (initHNJ over the owned rows)

#define SH_GRID 8192         // max argmin blocks (grid-stride over the tiles)


// ------------------------------------------------------------------ per join
// row n-1 behind the argmin records: the owner's cells, zeros elsewhere
template <int ET>
__global__ __launch_bounds__(TB) void k_sh_xm(const typename Elem<ET>::T *__restrict__ D, int n, Shard sh,
                                              typename Elem<ET>::T *__restrict__ xm) {
	const int k = blockIdx.x * TB + threadIdx.x;
	if(k >= n - 1) return;
	const bool own = sh.owns(n - 1);
	xm[k] = own ? D[sh.off(n - 1) + k] : (typename Elem<ET>::T) 0;
}

// initQ over the rank's tiles: NJ_SEG-column segments x one band, segment-
// major.  Segment s holds the local bands from global band 256 s on:
// first(s) = ceil((256 s - rank) / world), F = prefix sums of first, so the
// tiles before segment s number P(s) = s * nlb - F[s].
template <int ET>
__global__ __launch_bounds__(TB) void k_sh_argmin(const typename Elem<ET>::T *__restrict__ D, double bs, TreeBufs b,
                                                  int n, Shard sh, const long long *__restrict__ F, int nlb,
                                                  int sstar, long long tiles) {
	__shared__ double sq[TB / 64];
	__shared__ long long sf[TB / 64];
	if(b.ctl->done) return;
	constexpr int M = NJ_SEG / TB;
	double bq = 1.0;
	long long bf = -1;
	for(long long idx = blockIdx.x; idx < tiles; idx += gridDim.x) {
		int lo = 0, hi = sstar - 1;
		while(lo < hi) {
			const int mid = (lo + hi + 1) >> 1;
			if((long long) mid * nlb - F[mid] <= idx) lo = mid;
			else hi = mid - 1;
		}
		const int s = lo;
		const long long lb = (F[s + 1] - F[s]) + (idx - ((long long) s * nlb - F[s]));
		const int r0 = (int) ((lb * sh.world + sh.rank) * SB), r1 = r0 + SB < n ? r0 + SB : n;
		const int c0 = s * NJ_SEG;
		double sc[M];
#pragma unroll
		for(int m = 0; m < M; ++m) {
			int c = c0 + m * TB + (int) threadIdx.x;
			c = c < n ? c : n - 1;
			sc[m] = b.sD[c];
		}
		constexpr int G = 4;
		for(int rg = r0; rg < r1; rg += G) {
			typename Elem<ET>::T v[G][M];
			double sr[G];
#pragma unroll
			for(int g = 0; g < G; ++g) {
				const int r = rg + g < r1 ? rg + g : r1 - 1;
				const long long base = sh.off(r);
				sr[g] = b.sD[r];
#pragma unroll
				for(int m = 0; m < M; ++m) {
					const int c = c0 + m * TB + (int) threadIdx.x;
					v[g][m] = D[base + (c < r ? c : 0)];
				}
			}
#pragma unroll
			for(int g = 0; g < G; ++g) {
				const int r = rg + g;
				const long long fb = tri(r);
#pragma unroll
				for(int m = 0; m < M; ++m) {
					const int c = c0 + m * TB + (int) threadIdx.x;
					const double d = Elem<ET>::get(v[g][m], bs);
					const double q = qcrit(n, n, d, sr[g], sc[m]);
					const long long f = fb + c;
					const bool take = r < r1 && c < r && 0 <= d && (q < bq || (q == bq && f > bf));
					bq = take ? q : bq;
					bf = take ? f : bf;
				}
			}
		}
	}
	qf_wave_reduce(bq, bf);
	const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
	if(lane == 0) {
		sq[wid] = bq;
		sf[wid] = bf;
	}
	__syncthreads();
	if(threadIdx.x == 0) {
		for(int k = 1; k < TB / 64; ++k) {
			if(sq[k] < bq || (sq[k] == bq && sf[k] > bf)) {
				bq = sq[k];
				bf = sf[k];
			}
		}
		b.qpart[blockIdx.x] = bq;
		b.fpart[blockIdx.x] = bf;
	}
}

// this rank's record (G argmin partials; G = 0 when it owns no tile)
__global__ __launch_bounds__(TB) void k_sh_fold(TreeBufs b, int G, Shard sh, ShRec *__restrict__ rec,
                                                double q0 = 1.0) {
	__shared__ double sq[TB / 64];
	__shared__ long long sf[TB / 64];
	double fq = q0;
	long long ff = -1;
	for(int g = threadIdx.x; g < G; g += TB) {
		const double oq = b.qpart[g];
		const long long of = b.fpart[g];
		if(oq < fq || (oq == fq && of > ff)) {
			fq = oq;
			ff = of;
		}
	}
	qf_wave_reduce(fq, ff);
	const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
	if(lane == 0) {
		sq[wid] = fq;
		sf[wid] = ff;
	}
	__syncthreads();
	if(threadIdx.x == 0) {
		for(int w = 1; w < TB / 64; ++w) {
			if(sq[w] < fq || (sq[w] == fq && sf[w] > ff)) {
				fq = sq[w];
				ff = sf[w];
			}
		}
	}
	ShRec z;
	z.q = 0;
	z.f = 0;
	for(int w = threadIdx.x; w < sh.world; w += TB) {
		if(w != sh.rank) rec[w] = z;
	}
	if(threadIdx.x == 0) {
		ShRec r = z;
		if(!b.ctl->done) {
			r.q = fq;
			r.f = ff;
		}
		rec[sh.rank] = r;
	}
}

// the pieces of lines i and j this rank's rows hold: X[k] = D(i, k),
// X[n + k] = D(j, k) (raw elements; zeros where another rank owns the cell)
template <int ET>
__global__ __launch_bounds__(TB) void k_sh_lines(const typename Elem<ET>::T *__restrict__ D, TreeBufs b, int n,
                                                 Shard sh, const ShRec *__restrict__ rec,
                                                 typename Elem<ET>::T *__restrict__ X, double q0) {
	const int k = blockIdx.x * TB + threadIdx.x;
	if(b.ctl->done) return;
	double bq;
	long long bf;
	rec_fold(rec, sh.world, bq, bf, q0);
	if(bf < 0) {
		if(blockIdx.x == 0 && threadIdx.x == 0) {
			b.ctl->done = 1;
			b.ctl->final_n = n;
		}
		return;
	}
	int i, j;
	flat_to_ij(bf, i, j);
	if(k >= n) return;
	typename Elem<ET>::T xi = 0, xj = 0;
	if(k > i) {
		if(sh.owns(k)) xi = D[sh.off(k) + i];
	} else if(k < i && sh.owns(i)) {
		xi = D[sh.off(i) + k];
	}
	if(k > j) {
		if(sh.owns(k)) xj = D[sh.off(k) + j];
	} else if(k < j && sh.owns(j)) {
		xj = D[sh.off(j) + k];
	}
	X[k] = xi;
	X[n + k] = xj;
}

// limbLength, the join record and updateD (nj.c:836) over the gathered lines;
// every rank computes the whole new line j and stores its own cells (hnj:
// also into X[n + k], thread k's own slot, for k_sh_hnj's row-j minimum and
// column-j rule)
template <int ET>
__global__ __launch_bounds__(TB) void k_sh_join(typename Elem<ET>::T *__restrict__ D, double bs, TreeBufs b, int n,
                                                Shard sh, const ShRec *__restrict__ rec,
                                                typename Elem<ET>::T *__restrict__ X,
                                                typename Elem<ET>::T *__restrict__ Xm, double q0, int hnj) {
	__shared__ int s_stop, s_nj, s_neg, s_exact;
	TreeCtl *ctl = b.ctl;
	const int tid = threadIdx.x;
	const int k = blockIdx.x * TB + tid;
	double sDk = 0, Dik = 0, Dkj = 0;
	int Nk = 0;
	if(k < n) {
		sDk = b.sD[k];
		Nk = b.N[k];
		Dik = Elem<ET>::get(X[k], bs);
		Dkj = Elem<ET>::get(X[n + k], bs);
	}
	if(tid == 0) {
		s_stop = ctl->done;
		s_nj = ctl->njoins;
		s_neg = ctl->neg;
		s_exact = ctl->exact;
	}
	__syncthreads();
	if(s_stop) return;
	double bq;
	long long bf;
	rec_fold(rec, sh.world, bq, bf, q0);
	int i, j;
	flat_to_ij(bf, i, j);
	const double Dij = Elem<ET>::get(X[j], bs);
	if(blockIdx.x == 0 && tid == 0) {
		double Li, Lj;
		limb_length(&Li, &Lj, b.sD[i], b.sD[j], b.N[i], b.N[j], Dij, s_neg);
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
		b.joins[s_nj] = J;
		ctl->njoins = s_nj + 1;
	}
	double d = 0;
	int cnt = 0;
	if(k < n && k != i && k != j) {
		d = (Dik + Dkj - Dij) / 2;
		d = d < 0 ? 0 : d;
		const typename Elem<ET>::T v = Elem<ET>::put(d, 0.25, bs);
		if(k > j) {
			if(sh.owns(k)) D[sh.off(k) + j] = v;
		} else if(sh.owns(j)) {
			D[sh.off(j) + k] = v;
		}
		if(k == n - 1) Xm[j] = v;   // row n-1 moves to slot i in the pop
		if(hnj) X[n + k] = v;       // (this thread read its old value above)
		b.sD[k] = sDk - (Dik + Dkj - d);
		b.N[k] = Nk - 1;
		cnt = 1;
	}
	update_partials(b, n, s_exact, k, d, cnt, blockIdx.x);
	// exact mode: this block's row of the serial row sum (every rank holds
	// the whole new line j, so every rank computes the same rows)
	if(s_exact) xs_join_row(b, n, blockIdx.x, d, xs_tag(n));
}

// row sum of j, then ltdMatrix_popArrange (matrix.c:518) + nj.c:1588-1589:
// row n-1 (broadcast into Xm) becomes row/column i
template <int ET>
__global__ __launch_bounds__(TB) void k_sh_pop(typename Elem<ET>::T *__restrict__ D, TreeBufs b, int n, Shard sh,
                                               const typename Elem<ET>::T *__restrict__ Xm) {
	__shared__ double s_sd;
	__shared__ int s_nj, s_i, s_j, s_stop, s_serial, s_chain;
	TreeCtl *ctl = b.ctl;
	const int nn = n - 1;
	const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
	const int k = blockIdx.x * TB + tid;
	typename Elem<ET>::T vm = 0;
	if(k < nn) vm = Xm[k];
	const double sDm = b.sD[nn];
	const int Nm = b.N[nn];
	if(wid == 0) {
		const int done = ctl->done;
		const bool exact = ctl->exact;
		if(lane == 0) {
			s_i = ctl->i;
			s_j = ctl->j;
			s_stop = done;
		}
		if(!done) {
			double sd;
			int nj;
			bool need, chain;
			row_sum_j_wave(b, n, exact, false, &sd, &nj, &need, &chain);
			if(lane == 0) {
				s_sd = sd;
				s_nj = nj;
				s_serial = need;
				s_chain = chain;
			}
		}
	}
	__syncthreads();
	if(s_stop) return;
	const int i = s_i, j = s_j;
	// exact mode, a failed check of the parallel form: the serial chain (all threads)
	if(s_chain) {
		const double r = serial_sum_t<TB>(b.contrib, n);
		if(tid == 0) s_sd = r;
		if(blockIdx.x == 0 && tid == 0) ctl->chain_sums++;
		__syncthreads();
	}
	const double sdj = s_sd;
	if(blockIdx.x == 0 && tid == 0) {
		b.sD[j] = sdj;
		b.N[j] = s_nj;
		if(i != nn) {
			b.sD[i] = sDm;
			b.N[i] = Nm;
		}
		if(s_serial) ctl->serial_sums++;
	}
	if(i != nn) {
		if(k < i) {
			if(sh.owns(i)) D[sh.off(i) + k] = vm;
		} else if(k > i && k < nn && sh.owns(k)) {
			D[sh.off(k) + i] = vm;
		}
	}
}


// ------------------------------------------------------------------ HNJ
// hclust.c:1671 (-m hnj) over the row shards, tree.hip's k_hnj_argmin /
// k_nj_join / k_hnj_update split the sharded NJ way.  Q and P are indexed by
// global row; a row's (Q, P) is kept by its owner (updatePrevQ, the column-j
// and column-i rules read the row's own cells), while the two minima a join
// creates (row j from the new line j, row i from row n-1 moving into it) come
// from the gathered lines, so every rank computes them alike.  Per join:
//   k_sh_hnj_argmin  folds the last join's row-j / row-i minima into Q / P,
//                    then this rank's owned rows into argmin partials
//                    (minQ, hclust.c:353: smaller q, then the larger flat
//                    index tri(r) + P[r]); k_sh_fold makes the record; the
//                    records are allreduced with row n-1 behind them, as NJ;
//   k_sh_lines / allreduce / k_sh_join  as NJ (fold start DBL_MAX), the new
//                    line j kept in X[n + k];
//   k_sh_hnj         the row sum of j (k_sh_pop's), updateHNJ's Q / P pass on
//                    the owned rows, the row-j and row-i minima as partials,
//                    and HNJ_popArrange's stores (hclust.c:1308).
template <int UNUSED = 0>
__global__ __launch_bounds__(TB) void k_sh_hnj_argmin(TreeBufs b, int n, Shard sh) {
	__shared__ double sq[TB / 64], fq[2];
	__shared__ long long sf[TB / 64];
	__shared__ int fk[2];
	const TreeCtl *ctl = b.ctl;
	const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
	if(ctl->done) {
		if(tid == 0) {
			b.qpart[blockIdx.x] = DBL_MAX;
			b.fpart[blockIdx.x] = -1;
		}
		return;
	}
	const int r = (int) blockIdx.x * TB + tid;
	const int hj = ctl->hj, hi = ctl->hi;
	const bool own_j = hj >= 0 && hj / TB == (int) blockIdx.x, own_i = hi >= 0 && hi / TB == (int) blockIdx.x;
	if(blockIdx.x == 0 && tid == 0 && hi >= 0) {   // the pop's sD / N of row i (row n before the join)
		b.sD[hi] = b.sD[n];
		b.N[hi] = b.N[n];
	}
	if(own_j || own_i) {
		if(wid < 2 && ((wid == 0 && own_j) || (wid == 1 && own_i))) {
			double q;
			int k;
			if(wid == 0) qk_fold_wave(b.bmq, b.bmr, ctl->hjb, q, k);
			else qk_fold_wave(b.cfq, b.cfp, ctl->hib, q, k);
			if(lane == 0) {
				fq[wid] = q;
				fk[wid] = k;
			}
		}
		__syncthreads();
	}
	double q = DBL_MAX;
	long long f = -1;
	if(r < n) {
		double qr = b.Q[r];
		int pr = b.P[r];
		const int w = own_j && r == hj ? 0 : own_i && r == hi ? 1 : -1;
		if(w >= 0) {
			qr = fq[w];
			pr = fk[w] < 0 ? 0 : fk[w];
			b.Q[r] = qr;
			b.P[r] = pr;
		}
		if(r >= 1 && sh.owns(r) && qr <= DBL_MAX) {
			q = qr;
			f = tri(r) + pr;
		}
	}
	qf_wave_reduce(q, f);
	if(lane == 0) {
		sq[wid] = q;
		sf[wid] = f;
	}
	__syncthreads();
	if(tid == 0) {
		for(int k = 1; k < TB / 64; ++k) {
			if(sq[k] < q || (sq[k] == q && sf[k] > f)) {
				q = sq[k];
				f = sf[k];
			}
		}
		b.qpart[blockIdx.x] = q;
		b.fpart[blockIdx.x] = f;
	}
}

template <int ET>
__global__ __launch_bounds__(TB) void k_sh_hnj(typename Elem<ET>::T *__restrict__ D, double bs, TreeBufs b, int n,
                                               Shard sh, const typename Elem<ET>::T *__restrict__ X,
                                               const typename Elem<ET>::T *__restrict__ Xm) {
	__shared__ double s_sd, sq[TB / 64], sq2[TB / 64];
	__shared__ int s_nj, s_i, s_j, s_stop, s_serial, s_chain, sk[TB / 64], sk2[TB / 64];
	TreeCtl *ctl = b.ctl;
	const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
	const int k = (int) blockIdx.x * TB + tid;
	if(wid == 0) {
		const int done = ctl->done;
		const bool exact = ctl->exact;
		if(lane == 0) {
			s_i = ctl->i;
			s_j = ctl->j;
			s_stop = done;
		}
		if(!done) {
			double sd;
			int nj;
			bool need, chain;
			row_sum_j_wave(b, n, exact, false, &sd, &nj, &need, &chain);
			if(lane == 0) {
				s_sd = sd;
				s_nj = nj;
				s_serial = need;
				s_chain = chain;
			}
		}
	}
	__syncthreads();
	if(s_stop) return;
	const int i = s_i, j = s_j;
	if(s_chain) {   // exact mode, a failed check of the parallel form: the serial chain (all threads)
		const double r = serial_sum_t<TB>(b.contrib, n);
		if(tid == 0) s_sd = r;
		if(blockIdx.x == 0 && tid == 0) ctl->chain_sums++;
		__syncthreads();
	}
	const double sdj = s_sd;
	const int nj = s_nj;
	const int nn = n - 1;
	const bool move = i != nn;
	if(blockIdx.x == 0 && tid == 0) {
		b.sD[j] = sdj;
		b.N[j] = nj;
		ctl->hj = j;
		ctl->hjb = (int) cdiv(j, TB);
		// row i's sD / N (row nn's) wait for the next k_sh_hnj_argmin: sD[i]
		// is still read below as a partner's sum
		ctl->hi = move ? i : -1;
		ctl->hib = (int) cdiv(i, TB);
		if(s_serial) ctl->serial_sums++;
	}
	double rq = DBL_MAX, pq = DBL_MAX;
	int rk = -1, pk2 = -1;
	if(k < n) {
		const bool own = sh.owns(k);
		const int Nk = k == j ? nj : b.N[k];
		const double sDk = k == j ? sdj : b.sD[k];
		double Qk = b.Q[k];
		int Pk = b.P[k];
		if(own && k <= n - 2) {   // updatePrevQ (hclust.c:441-449): the row's own cell
			const int pk = Pk;
			const double d = Elem<ET>::get(D[sh.off(k) + pk], bs);
			if(0 <= d) {
				const int Np = pk == j ? nj : b.N[pk];
				const double sDp = pk == j ? sdj : b.sD[pk];
				Qk = ((Nk + Np - 4) >> 1) * d - sDk - sDp;
			}
		}
		if(own && k > j && k != i) {   // column j (hclust.c:530-556): the new D(k, j)
			const double d = Elem<ET>::get(X[n + k], bs);
			if(0 <= d) {
				const double q = ((nj + Nk - 4) >> 1) * d - sdj - sDk;
				if(Pk == i || Pk == j) {
					Qk = q;
					Pk = j;
				} else if(q <= Qk) {
					Qk = q;
					if(Pk < j) Pk = j;
				}
			}
		}
		if(k < j) {   // row j (hclust.c:497-511), from the gathered new line j
			const double d = Elem<ET>::get(X[n + k], bs);
			if(0 <= d) {
				rq = ((nj + Nk - 4) >> 1) * d - sdj - sDk;
				rk = k;
			}
		}
		// HNJ_popArrange (hclust.c:1308): row nn (gathered in Xm) moves to row
		// i (cells k < i: its minimum, on every rank) and column i (owned rows
		// i < k < nn: `q <= Q && (P < pos || q < Q)`)
		if(move && k < nn && k != i) {
			const typename Elem<ET>::T vm = Xm[k];
			const double d = Elem<ET>::get(vm, bs);
			const double sDi = b.sD[nn];
			const int Ni = b.N[nn];
			const double q = 0 <= d ? d * ((Ni + Nk - 4) >> 1) - sDi - sDk : 0.0;
			if(k < i) {
				if(sh.owns(i)) D[sh.off(i) + k] = vm;
				if(0 <= d) {
					pq = q;
					pk2 = k;
				}
			} else if(own) {
				D[sh.off(k) + i] = vm;
				if(0 <= d && q <= Qk && (Pk < i || q < Qk)) {
					Qk = q;
					Pk = i;
				}
			}
		}
		if(own && k != j) {
			b.Q[k] = Qk;
			b.P[k] = Pk;
		}
	}
	if((int) blockIdx.x * TB < j) {
		qk_block_reduce<TB>(rq, rk, sq, sk);
		if(tid == 0) {
			b.bmq[blockIdx.x] = rq;
			b.bmr[blockIdx.x] = rk;
		}
	}
	if(move && (int) blockIdx.x * TB < i) {
		qk_block_reduce<TB>(pq, pk2, sq2, sk2);
		if(tid == 0) {
			b.cfq[blockIdx.x] = pq;
			b.cfp[blockIdx.x] = pk2;
		}
	}
}

// RCCL, resolved with dlopen so the engine has no link-time dependency on it
struct RcclApi {
	void *h;
	ncclResult_t (*get_id)(ncclUniqueId *);
	ncclResult_t (*init_rank)(ncclComm_t *, int, ncclUniqueId, int);
	ncclResult_t (*all_reduce)(const void *, void *, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t);
	ncclResult_t (*bcast)(const void *, void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t);
	ncclResult_t (*all_gather)(const void *, void *, size_t, ncclDataType_t, ncclComm_t, hipStream_t);
	ncclResult_t (*abort_comm)(ncclComm_t);
	ncclResult_t (*destroy)(ncclComm_t);
	const char *(*err)(ncclResult_t);
};
static RcclApi g_rccl;

static int rccl_load() {
	if(g_rccl.h) return CCG_OK;
	const char *names[] = {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"};
	void *h = NULL;
	for(int k = 0; k < 3 && !h; ++k) h = dlopen(names[k], RTLD_NOW | RTLD_GLOBAL);
	if(!h) return CCG_EUNSUP;
	RcclApi a;
	a.h = h;
	a.get_id = (decltype(a.get_id)) dlsym(h, "ncclGetUniqueId");
	a.init_rank = (decltype(a.init_rank)) dlsym(h, "ncclCommInitRank");
	a.all_reduce = (decltype(a.all_reduce)) dlsym(h, "ncclAllReduce");
	a.bcast = (decltype(a.bcast)) dlsym(h, "ncclBroadcast");
	a.all_gather = (decltype(a.all_gather)) dlsym(h, "ncclAllGather");
	a.abort_comm = (decltype(a.abort_comm)) dlsym(h, "ncclCommAbort");
	a.destroy = (decltype(a.destroy)) dlsym(h, "ncclCommDestroy");
	a.err = (decltype(a.err)) dlsym(h, "ncclGetErrorString");
	if(!a.get_id || !a.init_rank || !a.all_reduce || !a.bcast || !a.all_gather || !a.destroy || !a.err)
		return CCG_EUNSUP;
	g_rccl = a;
	return CCG_OK;
}

// A rank's communicator.  ccg_rccl_abort may run on another thread (the
// multi-GPU CLI aborts every rank's communicator when one rank fails): `mu`
// serialises it against this rank's own collective calls, and once `aborted`
// is set the calls fail without touching the (freed) communicator; the
// owner's ccg_rccl_close then only frees this struct.
struct RcclUser {
	ncclComm_t comm;
	pthread_mutex_t mu;
	int aborted;
};

static int rccl_gone(RcclUser *u, const char *what) {
	char m[160];
	snprintf(m, sizeof(m), "%s: the communicator was aborted (a peer rank failed)", what);
	ccg_set_last_msg(m);
	return 1;
}

// widest element that tiles the byte range (the sum is a gather either way)
static void rccl_type(const void *p, size_t bytes, ncclDataType_t *t, size_t *count) {
	const uintptr_t a = (uintptr_t) p;
	if(bytes % 8 == 0 && a % 8 == 0) {
		*t = ncclUint64;
		*count = bytes / 8;
	} else if(bytes % 4 == 0 && a % 4 == 0) {
		*t = ncclUint32;
		*count = bytes / 4;
	} else {
		*t = ncclUint8;
		*count = bytes;
	}
}

static int rccl_allreduce(void *user, void *buf, size_t bytes, void *stream) {
	ncclDataType_t t;
	size_t cnt;
	rccl_type(buf, bytes, &t, &cnt);
	RcclUser *u = (RcclUser *) user;
	pthread_mutex_lock(&u->mu);
	if(u->aborted) {
		pthread_mutex_unlock(&u->mu);
		return rccl_gone(u, "ncclAllReduce");
	}
	ncclResult_t r = g_rccl.all_reduce(buf, buf, cnt, t, ncclSum, u->comm, (hipStream_t) stream);
	pthread_mutex_unlock(&u->mu);
	if(r != ncclSuccess) {
		char m[160];
		snprintf(m, sizeof(m), "ncclAllReduce: %s", g_rccl.err(r));
		ccg_set_last_msg(m);
	}
	return r != ncclSuccess;
}

static int rccl_bcast(void *user, const void *send, void *recv, size_t bytes, int root, void *stream) {
	RcclUser *u = (RcclUser *) user;
	pthread_mutex_lock(&u->mu);
	if(u->aborted) {
		pthread_mutex_unlock(&u->mu);
		return rccl_gone(u, "ncclBroadcast");
	}
	ncclResult_t r = g_rccl.bcast(send ? send : recv, recv, bytes, ncclUint8, root, u->comm, (hipStream_t) stream);
	pthread_mutex_unlock(&u->mu);
	if(r != ncclSuccess) {
		char m[160];
		snprintf(m, sizeof(m), "ncclBroadcast: %s", g_rccl.err(r));
		ccg_set_last_msg(m);
	}
	return r != ncclSuccess;
}

static int rccl_allgather(void *user, const void *send, void *recv, size_t bytes, void *stream) {
	ncclDataType_t t;
	size_t cnt;
	// the widest element tiling both buffers and the slot size
	rccl_type((const void *) ((uintptr_t) send | (uintptr_t) recv), bytes, &t, &cnt);
	RcclUser *u = (RcclUser *) user;
	pthread_mutex_lock(&u->mu);
	if(u->aborted) {
		pthread_mutex_unlock(&u->mu);
		return rccl_gone(u, "ncclAllGather");
	}
	ncclResult_t r = g_rccl.all_gather(send, recv, cnt, t, u->comm, (hipStream_t) stream);
	pthread_mutex_unlock(&u->mu);
	if(r != ncclSuccess) {
		char m[160];
		snprintf(m, sizeof(m), "ncclAllGather: %s", g_rccl.err(r));
		ccg_set_last_msg(m);
	}
	return r != ncclSuccess;
}

// ------------------------------------------------------------------ host driver
static long long sh_first(int s, const Shard &sh) {
	if(s == 0) return 0;
	const long long a = (long long) (NJ_SEG / NJ_RB) * s - sh.rank;
	return (a + sh.world - 1) / sh.world;
}

static int sh_nlb(int n, const Shard &sh) {
	const int nb = (n + SB - 1) / SB;
	return nb > sh.rank ? (nb - sh.rank + sh.world - 1) / sh.world : 0;
}

// the sharded NJ's device state (one allocation): the TreeBufs subset its
// loop uses, the argmin records with row n-1 behind them, lines i / j, the
// exact row sums' records and the init gathers
struct ShnLayout {
	size_t o_sD, o_c, o_N, o_ws, o_wa, o_wc, o_we, o_qp, o_fp, o_j, o_ctl, o_F, o_rec, o_X, o_Xm;
	size_t o_xa, o_xb, o_xcr, o_xt, o_rp, o_is, rec_b, sz = 0;
	size_t o_Q = 0, o_P = 0, o_bq = 0, o_br = 0, o_cq = 0, o_cp = 0;   // HNJ: Q / P and the row-minimum partials
	ShnLayout(int n0, int world, int es, bool hnj = false) {
		auto take = [&](size_t bytes) {
			size_t off = sz;
			sz += (bytes + 255) & ~(size_t) 255;
			return off;
		};
		const size_t nb = (size_t) cdiv(n0, TB) + 1;
		const int nseg0 = (int) cdiv(n0 - 1, NJ_SEG);
		o_sD = take(((size_t) n0 + 1) * 8);
		o_c = take(((size_t) n0 + 1) * 8);
		o_N = take(((size_t) n0 + 1) * 4);
		o_ws = take(nb * 8);
		o_wa = take(nb * 8);
		o_wc = take(nb * 4);
		o_we = take(nb * 4);
		o_qp = take(SH_GRID * 8);
		o_fp = take(SH_GRID * 8);
		o_j = take((size_t) n0 * sizeof(ccg_join));
		o_ctl = take(sizeof(TreeCtl));
		rec_b = ((size_t) world * sizeof(ShRec) + 15) & ~(size_t) 15;
		o_F = take((size_t) (nseg0 + 2) * 8);
		o_rec = take(rec_b + (size_t) n0 * es + 16);
		o_X = take((size_t) 2 * n0 * es);
		o_Xm = take((size_t) n0 * es + 8);
		o_xa = take(nb * 8);
		o_xb = take(nb * sizeof(XsBlk));
		o_xcr = take(nb * XB_CAP * sizeof(XsCross));
		o_xt = take(nb * XB_CAP_T * sizeof(XsTie));
		o_rp = take(sh_rp_bytes(n0));
		o_is = take(sh_init_scratch_bytes(n0, world));
		if(hnj) {
			o_Q = take(((size_t) n0 + 1) * 8);
			o_P = take(((size_t) n0 + 1) * 4);
			o_bq = take(nb * 8);
			o_br = take(nb * 4);
			o_cq = take(nb * 8);
			o_cp = take(nb * 4);
		}
	}
};

template <int ET>
static int tree_shard_run_t(ccg_ctx *ctx, const ccg_tree_args *a, const ccg_coll *coll_in, void *Dd,
                            ccg_join *joins, int *njoins, int *final_n, double *final_d, int64_t *stats) {
	typedef typename Elem<ET>::T T;
	T *D = (T *) Dd;
	const int n0 = a->n;
	const double bs = a->byteScale;
	hipStream_t st = ctx->stream;
	ccg_coll self;
	if(!coll_in) {
		sh_self_coll(&self);
		coll_in = &self;
	}
	const Shard sh = {coll_in->rank, coll_in->world};
	// device state: the single-GPU TreeBufs subset this loop uses
	const int nseg0 = (int) cdiv(n0 - 1, NJ_SEG);
	const bool hnj = a->method == CCG_TREE_HNJ;
	if(hnj && cdiv(n0, TB) > SH_GRID) return CCG_EINVAL;   // the minQ partials (one per 256 rows)
	const ShnLayout L(n0, coll_in->world, ET, hnj);
	const size_t rec_b = L.rec_b, sz = L.sz;
	const size_t o_sD = L.o_sD, o_c = L.o_c, o_N = L.o_N, o_ws = L.o_ws, o_wa = L.o_wa, o_wc = L.o_wc, o_we = L.o_we;
	const size_t o_qp = L.o_qp, o_fp = L.o_fp, o_j = L.o_j, o_ctl = L.o_ctl, o_F = L.o_F, o_rec = L.o_rec;
	const size_t o_X = L.o_X, o_Xm = L.o_Xm, o_xa = L.o_xa, o_xb = L.o_xb, o_xcr = L.o_xcr, o_xt = L.o_xt;
	const size_t o_rp = L.o_rp, o_is = L.o_is;
	char *m;
	if(hipMalloc((void **) &m, sz) != hipSuccess) return CCG_ENOMEM;
	size_t hcap = sh_init_host_bytes(n0, coll_in->world);
	if((size_t) 2 * n0 * ET > hcap) hcap = (size_t) 2 * n0 * ET;
	if(rec_b + (size_t) n0 * ET + 16 > hcap) hcap = rec_b + (size_t) n0 * ET + 16;
	unsigned char *h = NULL;
	if(coll_in->host_staged && hipHostMalloc((void **) &h, hcap) != hipSuccess) {
		hipFree(m);
		return CCG_ENOMEM;
	}
	int rc = CCG_OK;
	static thread_local KTimer kt;   // one per host thread (the CLI runs one rank per thread)
	CollRun cr = {coll_in, st, h, &kt};
	TreeBufs b;
	memset(&b, 0, sizeof(b));
	b.sD = (double *) (m + o_sD);
	b.contrib = (double *) (m + o_c);
	b.N = (int *) (m + o_N);
	b.wsum = (double *) (m + o_ws);
	b.wabs = (double *) (m + o_wa);
	b.wcnt = (int *) (m + o_wc);
	b.wexp = (int *) (m + o_we);
	b.qpart = (double *) (m + o_qp);
	b.fpart = (long long *) (m + o_fp);
	b.joins = (ccg_join *) (m + o_j);
	b.ctl = (TreeCtl *) (m + o_ctl);
	b.xagg = (unsigned long long *) (m + o_xa);
	b.xblk = (XsBlk *) (m + o_xb);
	b.xcr = (XsCross *) (m + o_xcr);
	b.xti = (XsTie *) (m + o_xt);
	if(hnj) {
		b.Q = (double *) (m + L.o_Q);
		b.P = (int *) (m + L.o_P);
		b.bmq = (double *) (m + L.o_bq);
		b.bmr = (int *) (m + L.o_br);
		b.cfq = (double *) (m + L.o_cq);
		b.cfp = (int *) (m + L.o_cp);
	}
	long long *F = (long long *) (m + o_F);
	ShRec *rec = (ShRec *) (m + o_rec);
	T *X = (T *) (m + o_X), *Xm = (T *) (m + o_Xm);
	void *rp = m + o_rp;
	ShInitStat istat = {0, 0};
	long long *hF = (long long *) malloc((size_t) (nseg0 + 2) * 8);
	TreeCtl init, hc;
	long long launches = 0;
	int n = n0;
	float ms = 0;
	memset(&init, 0, sizeof(init));
	init.neg = (a->flags & 2) != 0;
	init.exact = a->exact != 0;
	init.method = a->method;
	init.hj = init.hi = -1;
#define SH_TRY(x)                    \
	do {                             \
		if((rc = (x)) != CCG_OK) goto out; \
	} while(0)
#define SH_HIP(x)                                                     \
	do {                                                              \
		hipError_t e_ = (x);                                          \
		if(e_ != hipSuccess) {                                        \
			ccg_set_last_error(e_, #x, __FILE__, __LINE__);          \
			rc = e_ == hipErrorOutOfMemory ? CCG_ENOMEM : CCG_EHIP;  \
			goto out;                                                 \
		}                                                             \
	} while(0)
	if(!hF) {
		rc = CCG_ENOMEM;
		goto out;
	}
	hF[0] = 0;
	for(int s = 0; s <= nseg0; ++s) hF[s + 1] = hF[s] + sh_first(s, sh);
	SH_HIP(hipMemsetAsync(m, 0, sz, st));
	SH_HIP(hipMemcpyAsync(F, hF, (size_t) (nseg0 + 2) * 8, hipMemcpyHostToDevice, st));
	SH_HIP(hipMemcpyAsync(b.ctl, &init, sizeof(init), hipMemcpyHostToDevice, st));
	SH_HIP(hipEventRecord(ctx->ev0, st));
	kt.init(st, a->profile != 0);
	{
		int missing = 0;
		SH_TRY(sh_init_summad<ET>(D, n0, bs, sh, cr, st, rp, m + o_is, b, &launches, &missing, &istat));
		if(missing) {
			rc = CCG_EUNSUP;   // the missing-entry quirks of updateD run on one GPU only
			goto out;
		}
	}
	if(hnj) {   // initHNJ (hclust.c:56) over the owned rows
		k_init_hnj<ET><<<cdiv(n0, TB / 64), TB, 0, st>>>(sh, D, n0, bs, b.sD, b.N, b.Q, b.P);
		SH_HIP(hipGetLastError());
		++launches;
	}
	{
		int since_check = 0;
		const int stop_n = a->max_joins > 0 && a->max_joins < n0 - 2 ? n0 - a->max_joins : 2;
		while(n > stop_n) {
			T *Xmr = (T *) ((char *) rec + rec_b);   // row n-1, gathered with the records
			k_sh_xm<ET><<<cdiv(n - 1, TB), TB, 0, st>>>(D, n, sh, Xmr);
			const unsigned gn = cdiv(n, TB);
			int G = 0;
			if(hnj) {   // minQ over the owned rows' (Q, P)
				G = (int) gn;
				k_sh_hnj_argmin<><<<gn, TB, 0, st>>>(b, n, sh);
			} else {
				const int nlb = sh_nlb(n, sh), nseg = (int) cdiv(n - 1, NJ_SEG);
				int sstar = 0;
				while(sstar < nseg && hF[sstar + 1] - hF[sstar] < nlb) ++sstar;
				const long long tiles = (long long) sstar * nlb - hF[sstar];
				G = (int) (tiles < SH_GRID ? tiles : SH_GRID);
				if(G > 0) k_sh_argmin<ET><<<G, TB, 0, st>>>(D, bs, b, n, sh, F, nlb, sstar, tiles);
			}
			const double q0 = hnj ? DBL_MAX : 1.0;   // HNJ's minQ starts at DBL_MAX, NJ's initQ at 1
			k_sh_fold<<<1, TB, 0, st>>>(b, G, sh, rec, q0);
			kt.mark(CCG_K_ARGMIN);
			SH_TRY(cr.allreduce(rec, rec_b + (size_t) (n - 1) * ET));
			k_sh_lines<ET><<<gn, TB, 0, st>>>(D, b, n, sh, rec, X, q0);
			kt.mark(CCG_K_UPDATE);
			SH_TRY(cr.allreduce(X, (size_t) 2 * n * ET));
			k_sh_join<ET><<<gn, TB, 0, st>>>(D, bs, b, n, sh, rec, X, Xmr, q0, hnj);
			kt.mark(CCG_K_UPDATE);
			if(hnj) k_sh_hnj<ET><<<gn, TB, 0, st>>>(D, bs, b, n, sh, X, Xmr);
			else k_sh_pop<ET><<<gn, TB, 0, st>>>(D, b, n, sh, Xmr);
			kt.mark(CCG_K_POP);
			SH_HIP(hipGetLastError());
			launches += (G > 0) + 5;   // k_sh_xm, fold, lines, join, pop
			--n;
			if(++since_check == 1024) {
				since_check = 0;
				SH_HIP(hipMemcpyAsync(&hc, b.ctl, sizeof(hc), hipMemcpyDeviceToHost, st));
				SH_HIP(hipStreamSynchronize(st));
				if(hc.done) break;
			}
		}
	}
	SH_HIP(hipEventRecord(ctx->ev1, st));
	kt.finish();
	SH_HIP(hipMemcpyAsync(&hc, b.ctl, sizeof(hc), hipMemcpyDeviceToHost, st));
	SH_HIP(hipStreamSynchronize(st));
	SH_HIP(hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
	*njoins = hc.njoins;
	*final_n = hc.done ? hc.final_n : n;
	if(hc.njoins) {
		SH_HIP(hipMemcpyAsync(joins, b.joins, (size_t) hc.njoins * sizeof(ccg_join), hipMemcpyDeviceToHost, st));
	}
	*final_d = -1.0;
	if(*final_n == 2) {
		// D(1, 0): row 1 is in band 0, owned by rank 0
		SH_TRY(cr.bcast(sh.rank == 0 ? (const void *) (D + sh.off(1)) : NULL, Xm, ET, 0));
		T v;
		SH_HIP(hipMemcpyAsync(&v, Xm, sizeof(T), hipMemcpyDeviceToHost, st));
		SH_HIP(hipStreamSynchronize(st));
		*final_d = (ET == 8 || ET == 4) ? (double) v : v / bs;
	}
	if(stats) {
		stats[0] = 0;
		stats[1] = 0;
		stats[2] = launches;
		stats[3] = (int64_t) (ms * 1000.0);
		if(a->profile) {
			for(int c = 0; c < CCG_NKSTAT; ++c) {
				stats[4 + 2 * c] = kt.cnt[c];
				stats[5 + 2 * c] = kt.ns[c];
			}
			stats[4 + 2 * CCG_NKSTAT] = 0;
			stats[5 + 2 * CCG_NKSTAT] = 0;
			stats[6 + 2 * CCG_NKSTAT] = 0;
			stats[7 + 2 * CCG_NKSTAT] = 0;
			stats[8 + 2 * CCG_NKSTAT] = istat.coll_bytes;
			stats[9 + 2 * CCG_NKSTAT] = istat.hard;
			stats[10 + 2 * CCG_NKSTAT] = 0;
			stats[11 + 2 * CCG_NKSTAT] = 0;
		}
	}
out:
#undef SH_TRY
#undef SH_HIP
	if(rc != CCG_OK) kt.on = false;
	hipStreamSynchronize(st);
	free(hF);
	if(h) hipHostFree(h);
	hipFree(m);
	return rc;
}

// tree_shard_dnj.hip
size_t ccg_shard_dnj_bytes(int n, int world, int es);
int ccg_tree_shard_dnj_impl(ccg_ctx *c, const ccg_tree_args *a, const ccg_coll *coll, void *Dloc, ccg_join *joins,
                            int *njoins, int *final_n, double *final_d, int64_t *stats);

// tree.hip: the single-GPU engine
int ccg_tree_impl(ccg_ctx *ctx, const ccg_tree_args *a, void *Dd, ccg_join *joins, int *njoins, int *final_n,
                  double *final_d, int64_t *stats, const ccg_dnj_state *sin, ccg_dnj_state *sout);

// world 1 holds the whole matrix in the band layout, which is the packed LT
// the single-GPU engine consumes: with nothing to exchange it runs that engine
// (missing entries and -m hnj included).  CCG_SHARD_FORCE=1 keeps the sharded
// kernels at world 1 (their tests compare them with the single engine).
static bool shard_world1_single(const ccg_coll *coll) {
	if(coll && coll->world != 1) return false;
	const char *f = getenv("CCG_SHARD_FORCE");
	return !(f && atoi(f));
}

// ------------------------------------------------------------------ C ABI
extern "C" {

int ccg_shard_owner(int64_t row, int world) { return world > 0 ? (int) ((row / SB) % world) : -1; }

int64_t ccg_shard_row_offset(int64_t row, int rank, int world) {
	const Shard sh = {rank, world};
	return sh.off(row);
}

int64_t ccg_shard_elems(int64_t n, int rank, int world) {
	if(n <= 0 || world <= 0 || rank < 0 || rank >= world) return 0;
	const Shard sh = {rank, world};
	const int64_t gb = n / SB;
	if(n % SB && sh.owns(n)) return sh.off(n);   // n falls inside an owned band
	// first owned band at or above ceil(n / SB)
	int64_t g = (n + SB - 1) / SB;
	g += ((rank - g % world) % world + world) % world;
	(void) gb;
	return sh.off(g * SB);
}

int ccg_rccl_unique_id(void *id) {
	if(!id) return CCG_EINVAL;
	int rc = rccl_load();
	if(rc) return rc;
	ncclUniqueId u;
	if(g_rccl.get_id(&u) != ncclSuccess) return CCG_EHIP;
	memcpy(id, &u, sizeof(u));
	return CCG_OK;
}

int ccg_rccl_open(ccg_ctx *ctx, const void *id, int rank, int world, ccg_coll *out) {
	if(!ctx || !id || !out || world < 1 || rank < 0 || rank >= world) return CCG_EINVAL;
	int rc = rccl_load();
	if(rc) return rc;
	CCG_CHECK(hipSetDevice(ctx->device));
	RcclUser *u = (RcclUser *) calloc(1, sizeof(RcclUser));
	if(!u) return CCG_ENOMEM;
	pthread_mutex_init(&u->mu, NULL);
	ncclUniqueId uid;
	memcpy(&uid, id, sizeof(uid));
	ncclResult_t r = g_rccl.init_rank(&u->comm, world, uid, rank);
	if(r != ncclSuccess) {
		char m[160];
		snprintf(m, sizeof(m), "ncclCommInitRank: %s", g_rccl.err(r));
		ccg_set_last_msg(m);
		pthread_mutex_destroy(&u->mu);
		free(u);
		return CCG_EHIP;
	}
	memset(out, 0, sizeof(*out));
	out->user = u;
	out->rank = rank;
	out->world = world;
	out->host_staged = 0;
	out->allreduce_sum_u8 = rccl_allreduce;
	out->broadcast = rccl_bcast;
	out->allgather = rccl_allgather;
	return CCG_OK;
}

int ccg_tree_shard_bytes(int64_t n, int etype, int method, int world, int64_t *device_bytes, int64_t *gather_bytes) {
	if(!device_bytes || n < 3 || n > INT32_MAX - 512 || world < 1) return CCG_EINVAL;
	if(etype != 8 && etype != 4 && etype != 2 && etype != 1) return CCG_EINVAL;
	if(method != CCG_TREE_NJ && method != CCG_TREE_DNJ && method != CCG_TREE_HNJ) return CCG_EINVAL;
	const int n0 = (int) n;
	*device_bytes = (int64_t) (method == CCG_TREE_DNJ ? ccg_shard_dnj_bytes(n0, world, etype)
	                                                  : ShnLayout(n0, world, etype, method == CCG_TREE_HNJ).sz);
	// sh_init_chunk's bound on the hard-column gather buffer (a quarter of the
	// free memory, at most 16 GB, at least 256 columns)
	if(gather_bytes) {
		int64_t g = (int64_t) 16 << 30, mn = (int64_t) 256 * n0 * etype;
		*gather_bytes = g > mn ? g : mn;
	}
	return CCG_OK;
}

int ccg_rccl_abort(ccg_coll *c) {
	if(!c || !c->user) return CCG_EINVAL;
	if(!g_rccl.abort_comm) return CCG_EUNSUP;
	RcclUser *u = (RcclUser *) c->user;
	pthread_mutex_lock(&u->mu);   // waits for an enqueue in progress on the owner's thread
	int rc = CCG_OK;
	if(!u->aborted) {
		u->aborted = 1;
		rc = g_rccl.abort_comm(u->comm) == ncclSuccess ? CCG_OK : CCG_EHIP;
		u->comm = NULL;
	}
	pthread_mutex_unlock(&u->mu);
	return rc;
}

// the owner's call: destroys the communicator (or, after an abort, only
// frees what is left of it)
int ccg_rccl_close(ccg_coll *c) {
	if(!c || !c->user) return CCG_EINVAL;
	RcclUser *u = (RcclUser *) c->user;
	ncclResult_t r = ncclSuccess;
	if(!u->aborted) r = g_rccl.destroy(u->comm);
	pthread_mutex_destroy(&u->mu);
	free(u);
	c->user = NULL;
	return r == ncclSuccess ? CCG_OK : CCG_EHIP;
}

static int shard_check(ccg_ctx *c, const ccg_tree_args *a, const ccg_coll *coll) {
	if(!c || !a) return CCG_EINVAL;
	if(a->n < 3 || (a->method != CCG_TREE_NJ && a->method != CCG_TREE_DNJ && a->method != CCG_TREE_HNJ))
		return CCG_EINVAL;
	if(a->etype != 8 && a->etype != 4 && a->etype != 2 && a->etype != 1) return CCG_EINVAL;
	if((a->etype == 2 || a->etype == 1) && !(a->byteScale != 0)) return CCG_EINVAL;
	if(coll && (coll->world < 1 || coll->rank < 0 || coll->rank >= coll->world || !coll->allreduce_sum_u8 ||
	            !coll->broadcast))
		return CCG_EINVAL;
	return CCG_OK;
}

int ccg_tree_shard_dev(ccg_ctx *c, const ccg_tree_args *a, const ccg_coll *coll, void *Dloc, ccg_join *joins,
                       int *njoins, int *final_n, double *final_d, int64_t *stats) {
	if(c && a && shard_world1_single(coll) && (!coll || coll->rank == 0)) {
		if(!Dloc || !joins || !njoins || !final_n || !final_d) return CCG_EINVAL;
		if(a->n < 3 || (a->method != CCG_TREE_NJ && a->method != CCG_TREE_DNJ && a->method != CCG_TREE_HNJ))
			return CCG_EINVAL;
		if(a->etype != 8 && a->etype != 4 && a->etype != 2 && a->etype != 1) return CCG_EINVAL;
		if((a->etype == 2 || a->etype == 1) && !(a->byteScale != 0)) return CCG_EINVAL;
		CCG_CHECK(hipSetDevice(c->device));
		CCG_DEVICE_SYNC(c);
		return ccg_tree_impl(c, a, Dloc, joins, njoins, final_n, final_d, stats, NULL, NULL);
	}
	int rc = shard_check(c, a, coll);
	if(rc) return rc;
	if(!Dloc || !joins || !njoins || !final_n || !final_d) return CCG_EINVAL;
	CCG_CHECK(hipSetDevice(c->device));
	CCG_DEVICE_SYNC(c);   // inputs may come from other streams (e.g. torch's)
	if(a->method == CCG_TREE_DNJ) {
		ccg_coll self;
		if(!coll) {
			sh_self_coll(&self);
			coll = &self;
		}
		return ccg_tree_shard_dnj_impl(c, a, coll, Dloc, joins, njoins, final_n, final_d, stats);
	}
	switch(a->etype) {
		case 8: return tree_shard_run_t<8>(c, a, coll, Dloc, joins, njoins, final_n, final_d, stats);
		case 4: return tree_shard_run_t<4>(c, a, coll, Dloc, joins, njoins, final_n, final_d, stats);
		case 2: return tree_shard_run_t<2>(c, a, coll, Dloc, joins, njoins, final_n, final_d, stats);
		default: return tree_shard_run_t<1>(c, a, coll, Dloc, joins, njoins, final_n, final_d, stats);
	}
}

int ccg_tree_shard(ccg_ctx *c, const ccg_tree_args *a, const ccg_coll *coll, const void *D, ccg_join *joins,
                   int *njoins, int *final_n, double *final_d, int64_t *stats) {
	int rc = c && a && shard_world1_single(coll) ? CCG_OK : shard_check(c, a, coll);
	if(rc) return rc;
	if(!D) return CCG_EINVAL;
	const int rank = coll ? coll->rank : 0, world = coll ? coll->world : 1;
	const int64_t n = a->n, es = a->etype;
	const int64_t elems = ccg_shard_elems(n, rank, world);
	// the rank's bands are contiguous row runs of the full LT: copy band by band
	char *hbuf = (char *) malloc((size_t) (elems ? elems : 1) * es);
	if(!hbuf) return CCG_ENOMEM;
	const char *src = (const char *) D;
	for(int64_t g = rank; g * SB < n; g += world) {
		const int64_t r0 = g * SB, r1 = r0 + SB < n ? r0 + SB : n;
		memcpy(hbuf + ccg_shard_row_offset(r0, rank, world) * es, src + tri(r0) * es, (size_t) (tri(r1) - tri(r0)) * es);
	}
	CCG_CHECK(hipSetDevice(c->device));
	void *d = NULL;
	if(hipMalloc(&d, (size_t) (elems ? elems : 1) * es) != hipSuccess) {
		free(hbuf);
		return CCG_ENOMEM;
	}
	if(hipMemcpy(d, hbuf, (size_t) elems * es, hipMemcpyHostToDevice) != hipSuccess) {
		rc = CCG_EHIP;
	} else {
		rc = ccg_tree_shard_dev(c, a, coll, d, joins, njoins, final_n, final_d, stats);
	}
	free(hbuf);
	hipStreamSynchronize(c->stream);
	hipFree(d);
	return rc;
}

}   // extern "C"
