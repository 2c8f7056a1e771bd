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
// P (i32).  The matrix size n of a join is a launch argument; the join and
// the DNJ selection live in a device TreeCtl.
//
// Pipeline without in-kernel grid synchronisation.  A dependent global round
// trip costs ~1 us on MI355X (coherent traffic crosses XCDs), so no kernel
// ends in a "last block" ticket: every kernel writes per-block partials, and
// the NEXT kernel folds them redundantly in each of its blocks (identical,
// fixed-order, hence deterministic), substituting locally the few values its
// block 0 persists for the kernels after it.  Per DNJ join
// (ccg_dnj_search.h has the search kernels):
//   k_dnj_plan    one block: folds the previous requeue (updateDNJ +
//                 DNJ_popArrange partials, minPos), picks the top rows S
//                 (Q[r] < m0, scanning down from n-1), bounds the rows below
//                 S by max(q(k, P[k]), Q_k) over the S rows k above them (the
//                 Q criterion at k's stored partner cell is >= k's fresh min,
//                 so this bounds minQpair's running min as max(fresh_k, Q_k)
//                 does) and lists S and every row under its bound, descending,
//                 with unit offsets (any unlisted row is provably skipped);
//   k_dnj_scan    rescans the listed rows in SEG-cell units over the grid
//                 (k_dnj_fold folds each entry's units once for large n);
//   k_dnj_join    replays minQpair's accept/reject decisions over the entries
//                 in descending row order (a parallel prefix-min when every
//                 fresh min is >= its stale bound, pass by pass otherwise),
//                 records the join, runs updateD and, in exact mode, its
//                 blocks' part of the serial row sum (xs_join_row);
//   k_dnj_requeue takes the new row sum of j (tree sum, or the exact walk of
//                 the join blocks' records) and runs updateDNJ's Q/P part
//                 plus DNJ_popArrange.
// NJ: k_nj_argmin (initQ over all cells), k_nj_join (fold + updateD),
// k_nj_pop (row sum + ltdMatrix_popArrange).
#include <string.h>
#include <stdio.h>
#include <vector>
#include <stdlib.h>
#include "ccg_tree_common.h"

#include "ccg_dnj_search.h"

static thread_local DnjGrid g_grid;   // loaded per tree run (per host thread: tree_run_t adapts it per window)

// ------------------------------------------------------------------ init
// nj.c:111 initSummaD: per row, the row part (m < k) then the column part
// (m > k), each in increasing m, summed serially.  k_init_rows: one wave per
// row stages 64 contiguous cells at a time and lane 0 accumulates them in
// order; k_init_cols: one thread per row continues over the column part,
// coalesced across the wave (threads k..k+63 read row m at columns k..k+63).
template <int ET>
__global__ __launch_bounds__(TB) void k_init_rows(const typename Elem<ET>::T *__restrict__ D, int n, double bs,
                                                  double *__restrict__ sD, int *__restrict__ N, TreeCtl *ctl) {
	__shared__ double buf[TB / 64][64];
	const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
	const int k = blockIdx.x * (TB / 64) + wid;
	if(k >= n) return;
	double s = 0;
	int c = 1, miss = 0;
	const typename Elem<ET>::T *row = D + tri(k);
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
		sD[k] = s;
		N[k] = c;
		if(miss) atomicOr(&ctl->has_missing, 1);
	}
}

template <int ET>
__global__ __launch_bounds__(TB) void k_init_cols(const typename Elem<ET>::T *__restrict__ D, int n, double bs,
                                                  double *__restrict__ sD, int *__restrict__ N, TreeCtl *ctl) {
	const int k = blockIdx.x * TB + threadIdx.x;
	if(k >= n) return;
	double s = sD[k];
	int c = N[k], miss = 0;
	for(int m = k + 1; m < n; ++m) {
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

// nj.c:836-1044 without missing entries: every k takes the (D_ik, D_kj >= 0)
// branch, so the sD/N cursor never lags.  Writes the per-block partials of
// the new row sum of j (sum, sum |c|, count, min exponent) and, in exact mode,
// each contribution.
template <int ET>
__device__ __forceinline__ void update_body(typename Elem<ET>::T *__restrict__ D, double bs, const TreeBufs &b, int n,
                                            int i, int j, double Dij, bool exact, int k, double Dik, double Dkj,
                                            double sDk, int Nk, int slot) {
	double d = 0;
	int cnt = 0;
	typename Elem<ET>::T v = 0;
	if(k < n && k != i && k != j) {
		d = (Dik + Dkj - Dij) / 2;
		d = d < 0 ? 0 : d;
		v = Elem<ET>::put(d, 0.25, bs);
		D[k < j ? tri(j) + k : tri(k) + j] = v;
		b.sD[k] = sDk - (Dik + Dkj - d);
		b.N[k] = Nk - 1;
		cnt = 1;
	}
	if(b.lbm) {   // (uniform) block bounds: row j rewritten (exact per wave), column j lowered where written
		const bool rowj = k < j;   // k < j < i: a cell of row j
		const unsigned x = lb_bits(Elem<ET>::get(v, bs));
		const unsigned mn = wave_min_u32(rowj ? x : 0xFFFFFFFFu);
		if((threadIdx.x & 63) == 0 && k < j) b.lbm[(long long) j * b.lbs + (k >> 6)] = mn;
		if(k > j && k < n && k != i) __hip_atomic_fetch_min(b.lbm + (long long) k * b.lbs + (j >> 6), x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
	}
	update_partials(b, n, exact, k, d, cnt, slot);
	// exact mode: this block's row of the serial row sum (xs_join_row; the
	// consumer walks the rows' records)
	if(exact) xs_join_row(b, n, slot, d, xs_tag(n));   // tag: the matrix size, one per join and uniform over the grid
}


// limbLength (nj.c:42), the join record and updateD (nj.c:836) of the pair
// (i, j); (ci, cj) is the plan's candidate pair, whose operands the caller
// loaded at entry (pij, pik, pkj)
template <int ET>
__device__ __forceinline__ void join_tail(typename Elem<ET>::T *__restrict__ D, double bs, const TreeBufs &b, int n,
                                          int general, int i, int j, int ci, int cj, typename Elem<ET>::T pij,
                                          typename Elem<ET>::T pik, typename Elem<ET>::T pkj, double sDk, int Nk,
                                          int neg, int nj, int exact) {
	TreeCtl *ctl = b.ctl;
	const int tid = threadIdx.x, k = blockIdx.x * TB + tid;
	const bool writer = blockIdx.x == 0;
	if(i == 0 && j == 0) {
		if(writer && tid == 0) {
			ctl->done = 1;
			ctl->final_n = n;
		}
		return;
	}
	// ---- join: limbLength (nj.c:42) and updateD (nj.c:836)
	const bool hit = i == ci && j == cj;   // uniform
	const double Dij = Elem<ET>::get(hit ? pij : D[tri(i) + j], bs);
	double Dik = 0, Dkj = 0;
	if(!general && k < n && k != i && k != j) {
		Dik = Elem<ET>::get(hit ? pik : D[k < i ? tri(i) + k : tri(k) + i], bs);
		Dkj = Elem<ET>::get(hit ? pkj : D[k < j ? tri(j) + k : tri(k) + j], bs);
	}
	if(writer && tid == 0) {
		double Li, Lj;
		limb_length(&Li, &Lj, b.sD[i], b.sD[j], b.N[i], b.N[j], Dij, neg);
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
		b.joins[nj] = J;
		ctl->njoins = nj + 1;
	}
	TS(3, 4);
	if(general) return;
	update_body<ET>(D, bs, b, n, i, j, Dij, exact, k, Dik, Dkj, sDk, Nk, blockIdx.x);
	TS(3, 5);
}

// ------------------------------------------------------------------ block lower bounds
// TreeBufs::lbm / msd from the matrix and sD as they are (the first join, or a
// resumed state): one wave per row, BB blocks in flight per lane; one wave per
// 64 columns for the sD maxima
template <int ET>
__global__ __launch_bounds__(TB) void k_lb_init(const typename Elem<ET>::T *__restrict__ D, int n, double bs,
                                                TreeBufs b) {
	constexpr int BB = 8;
	const int lane = threadIdx.x & 63;
	const int r = blockIdx.x * (TB / 64) + (threadIdx.x >> 6);
	if(r >= n) return;   // (wave-uniform)
	if(r < (n + LBW - 1) / LBW) {   // the sD maxima of block r
		const int c = r * LBW + lane;
		const double mx = wave_max_d(c < n ? b.sD[c] : -DBL_MAX);
		if(lane == 0) b.msd[r] = mx;
	}
	if(lane == 0) b.ubq[r] = INFINITY;   // no partner-cell threshold yet: the first scan reads every block
	const typename Elem<ET>::T *row = D + tri(r);
	const int nbk = (r + LBW - 1) / LBW;
	for(int u0 = 0; u0 < nbk; u0 += BB) {
		unsigned x[BB];
#pragma unroll
		for(int m = 0; m < BB; ++m) {
			const int c = (u0 + m) * LBW + lane;
			x[m] = u0 + m < nbk && c < r ? lb_bits(Elem<ET>::get(row[c], bs)) : 0xFFFFFFFFu;
		}
#pragma unroll
		for(int m = 0; m < BB; ++m) {
			const unsigned mn = wave_min_u32(x[m]);
			if(lane == 0 && u0 + m < nbk) b.lbm[(long long) r * b.lbs + u0 + m] = mn;
		}
	}
}

// ------------------------------------------------------------------ DNJ join
// Wave 0: fresh mins of the rest entries (fold of their units), minQpair's
// replay; then limbLength, the join record and updateD with the whole grid.
// (n <= prefold_n; larger matrices use k_dnj_join_pf below.)
template <int ET, bool GEN>
__global__ __launch_bounds__(TB) void k_dnj_join(typename Elem<ET>::T *__restrict__ D, double bs, TreeBufs b, int n,
                                                 int general, int prefold, int seg) {
	__shared__ int e_row[DNJ_B + REPLAY_CAP], e_j[DNJ_B + REPLAY_CAP];
	__shared__ double e_b[DNJ_B + REPLAY_CAP], e_f[DNJ_B + REPLAY_CAP];
	__shared__ unsigned char e_acc[DNJ_B + REPLAY_CAP];
	__shared__ int s_pi, s_pj, s_stop, s_nj, s_neg, s_exact, s_nS, s_merged;
	__shared__ double s_m0;
	__shared__ double lq[JOIN_UPRE];
	__shared__ int lj[JOIN_UPRE];
	TreeCtl *ctl = b.ctl;
	const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
	const bool writer = blockIdx.x == 0;
	TS_ENTRY(3);
	TS(3, 0);
	// updateD's operands for the plan's candidate pair (pos_i, pos_j), loaded
	// now: when the replay keeps that pair (no rescanned row improves on m0)
	// the update needs no dependent load after it; sD / N of k in any case
	const int k = blockIdx.x * TB + tid;
	int ci = ctl->pos_i, cj = ctl->pos_j;
	ci = ci < 0 || ci >= n ? 0 : ci;
	cj = cj < 0 || cj >= ci ? 0 : cj;
	typename Elem<ET>::T pik = 0, pkj = 0;
	double sDk = 0;
	int Nk = 0;
	if(!general && k < n) {
		sDk = b.sD[k];
		Nk = b.N[k];
		if(k != ci && k != cj) {
			pik = D[k < ci ? tri(ci) + k : tri(k) + ci];
			pkj = D[k < cj ? tri(cj) + k : tri(k) + cj];
		}
	}
	const typename Elem<ET>::T pij = D[tri(ci) + cj];
	// every thread prefetches rest-unit partials (their count is not known yet);
	// with k_dnj_fold (prefold) the entries' folded pairs instead
	if(prefold) {
#pragma unroll
		for(int m = 0; m < JOIN_UPRE / TB; ++m) {
			lq[tid + m * TB] = b.rf[tid + m * TB];
			lj[tid + m * TB] = b.rj[tid + m * TB];
		}
	} else {
#pragma unroll
		for(int m = 0; m < JOIN_UPRE / TB; ++m) {
			lq[tid + m * TB] = b.cq[tid + m * TB];
			lj[tid + m * TB] = b.cj[tid + m * TB];
		}
	}
	__syncthreads();
	if(wid == 0) {
		// ---- loads independent of the outcome
		const int done = ctl->done, nS = ctl->nS, T = ctl->T;
		const bool merged = ctl->ntop != nS;   // band rows of S interleave with the rest
		const int pos_i = ctl->pos_i, pos_j = ctl->pos_j;
		const double m0 = ctl->m0;   // read early (independent of the outcome)
		Entry se0, se1;
		se0 = b.Sent[lane];
		se1 = b.Sent[lane + 64];
		const int sp0 = merged ? b.Spos[lane] : lane, sp1 = merged ? b.Spos[lane + 64] : lane + 64;
		int rr[4], cs[4];
		double bb[4];
#pragma unroll
		for(int m = 0; m < 4; ++m) {
			cs[m] = merged ? b.cslot[lane + 64 * m] : nS + lane + 64 * m;
			rr[m] = b.crow[lane + 64 * m];
			bb[m] = b.cbnd[lane + 64 * m];
		}
		const int umax = dnj_umax(n, seg);   // entry e's units: [e umax, e umax + dcdiv(row, seg))
		if(lane == 0) {
			s_nj = ctl->njoins;
			s_neg = ctl->neg;
			s_exact = ctl->exact;
		}
		if(done) {
			if(lane == 0) s_stop = 1;
		} else {
			TS(3, 1);
			int pi = pos_i, pj = pos_j;
			// entries in LDS, or in HBM when more rows qualified than LDS holds
			const bool lds = T <= REPLAY_CAP;
			int *x_row = lds ? e_row : b.erow, *x_j = lds ? e_j : b.ej;
			double *x_b = lds ? e_b : b.eb, *x_f = lds ? e_f : b.ef;
			// entries in scan order: S rows and rest rows interleave below the
			// top part of S (slots from k_dnj_find)
			if(lane < nS) {
				x_row[sp0] = se0.row;
				x_j[sp0] = se0.j;
				x_b[sp0] = se0.bnd;
				x_f[sp0] = se0.f;
			}
			if(lane + 64 < nS) {
				x_row[sp1] = se1.row;
				x_j[sp1] = se1.j;
				x_b[sp1] = se1.bnd;
				x_f[sp1] = se1.f;
			}
			// fresh (q, j) of the first 256 rest entries: fold of their units
			// (entries past 256 are folded by the whole block below)
#pragma unroll
			for(int m = 0; m < 4; ++m) {
				const int e = lane + 64 * m;
				if(e >= T) continue;
				const int ua = e * umax, ub = ua + dcdiv(rr[m], seg);
				double q = DBL_MAX;
				int idx = 0;
				if(prefold) {
					q = lq[e];   // e < 256 <= JOIN_UPRE
					idx = lj[e];
				} else if(ub <= JOIN_UPRE) {
					for(int u = ua; u < ub; ++u) {
						if(qarg_better(lq[u], lj[u], q, idx)) {
							q = lq[u];
							idx = lj[u];
						}
					}
				} else {
					fold_units(b.cq, b.cj, ua, ub, q, idx);
				}
				x_row[cs[m]] = rr[m];
				x_j[cs[m]] = idx;
				x_b[cs[m]] = bb[m];
				x_f[cs[m]] = q;
			}
			wave_sync();
			if(lane == 0) {
				s_stop = 0;
				s_merged = merged;
				s_pi = pi;
				s_pj = pj;
				s_nS = nS;
				s_m0 = m0;
			}
		}
	}
	// entries past the first 256: the whole block folds them (T is uniform)
	const int T = ctl->T;
	if(T > 256) {
		__syncthreads();
		if(!s_stop) {
			const bool lds = T <= REPLAY_CAP;
			int *x_row = lds ? e_row : b.erow, *x_j = lds ? e_j : b.ej;
			double *x_b = lds ? e_b : b.eb, *x_f = lds ? e_f : b.ef;
			// prefolded (large n, many entries): 8 entries per thread per step, all
			// of their loads in flight together
			for(int e0 = 256 + tid; prefold && e0 < T; e0 += 8 * TB) {
				int r[8], idx[8], sl[8];
				double bnd[8], q[8];
#pragma unroll
				for(int m = 0; m < 8; ++m) {
					const int e = e0 + m * TB < T ? e0 + m * TB : e0;
					r[m] = b.crow[e];
					bnd[m] = b.cbnd[e];
					q[m] = e < JOIN_UPRE ? lq[e] : b.rf[e];
					idx[m] = e < JOIN_UPRE ? lj[e] : b.rj[e];
					sl[m] = s_merged ? b.cslot[e] : s_nS + e;
				}
#pragma unroll
				for(int m = 0; m < 8; ++m) {
					if(e0 + m * TB >= T) continue;
					x_row[sl[m]] = r[m];
					x_j[sl[m]] = idx[m];
					x_b[sl[m]] = bnd[m];
					x_f[sl[m]] = q[m];
				}
			}
			for(int e = 256 + tid; !prefold && e < T; e += TB) {
				const int r = b.crow[e];
				const double bnd = b.cbnd[e];
				double q = DBL_MAX;
				int idx = 0;
				if(e * dnj_umax(n, seg) + dcdiv(r, seg) <= JOIN_UPRE) {
					const int ua = e * dnj_umax(n, seg), ub = ua + dcdiv(r, seg);
					for(int u = ua; u < ub; ++u) {
						if(qarg_better(lq[u], lj[u], q, idx)) {
							q = lq[u];
							idx = lj[u];
						}
					}
				} else {
					fold_units(b.cq, b.cj, e * dnj_umax(n, seg), e * dnj_umax(n, seg) + dcdiv(r, seg), q, idx);
				}
				const int s = s_merged ? b.cslot[e] : s_nS + e;
				x_row[s] = r;
				x_j[s] = idx;
				x_b[s] = bnd;
				x_f[s] = q;
			}
		}
	}
	__syncthreads();
	if(s_stop) return;
	{
		TS(3, 2);
		const int nS = s_nS, total = nS + T;
		const double m0 = s_m0;
		const bool lds = T <= REPLAY_CAP;
		const double *x_b = lds ? e_b : b.eb, *x_f = lds ? e_f : b.ef;
		// minQpair's replay.  Without "bad" entries (fresh < stale bound, rare)
		// every entry contributes its fresh value to the running min, so the
		// decisions are a prefix min over the entries in scan order: the whole
		// block folds it (contiguous entries per thread, one block scan); the
		// pair is the first entry reaching the overall minimum.  Only the
		// writer block needs the per-entry accept decisions (its (Q, P) writes).
		// each thread's contiguous chunk [e0, e1): in registers up to RP entries
		// (one round trip when the entries are in HBM), else in steps of 8
		constexpr int RP = 16;
		const int per = (total + TB - 1) / TB, e0 = tid * per, e1 = e0 + per < total ? e0 + per : total;
		const bool inreg = per >= 2 && per <= RP;   // uniform (one entry per thread: the plain loops)
		double rf[RP], rb[RP];
		int bad = 0;
		double tmin = DBL_MAX;
		if(inreg) {
#pragma unroll
			for(int m = 0; m < RP; ++m) {
				rf[m] = DBL_MAX;
				rb[m] = 0;
				if(m < per) {   // uniform
					const int e = e0 + m < e1 ? e0 + m : 0;
					rf[m] = x_f[e];
					rb[m] = x_b[e];
				}
			}
#pragma unroll
			for(int m = 0; m < RP; ++m) {
				if(e0 + m >= e1) continue;
				bad |= !(rf[m] >= rb[m]);
				tmin = rf[m] < tmin ? rf[m] : tmin;
			}
		} else {
			for(int e = e0; e < e1; e += 8) {
				double f8[8], b8[8];
#pragma unroll
				for(int m = 0; m < 8; ++m) {
					f8[m] = DBL_MAX;
					b8[m] = 0;
					if(e + m < e1) {
						f8[m] = x_f[e + m];
						b8[m] = x_b[e + m];
					}
				}
#pragma unroll
				for(int m = 0; m < 8; ++m) {
					if(e + m >= e1) continue;
					bad |= !(f8[m] >= b8[m]);
					tmin = f8[m] < tmin ? f8[m] : tmin;
				}
			}
		}
		if(__syncthreads_or(bad)) {
			if(wid == 0) {
				int pi = s_pi, pj = s_pj;
				bool had_bad;
				// two calls so the LDS case keeps ds_* accesses (no flat addressing)
				if(lds) replay_wave(total, m0, e_row, e_j, e_b, e_f, e_acc, writer, b, pi, pj, &had_bad, n);
				else replay_wave(total, m0, b.erow, b.ej, b.eb, b.ef, b.eacc, writer, b, pi, pj, &had_bad, n);
				if(writer && lane == 0 && had_bad) ctl->serial_replays++;
				if(lane == 0) {
					s_pi = pi;
					s_pj = pj;
				}
			}
		} else {
			__shared__ double s_wm[TB / 64];
			__shared__ int s_we[TB / 64];
			const double inc = wave_incl_min(tmin);
			if(lane == 63) s_wm[wid] = inc;
			__syncthreads();
			double carry = m0, cm = m0;
#pragma unroll
			for(int w = 0; w < TB / 64; ++w) {
				if(w < wid) carry = s_wm[w] < carry ? s_wm[w] : carry;
				cm = s_wm[w] < cm ? s_wm[w] : cm;
			}
			// the first entry reaching cm (only when it improves on m0)
			int first = 0x7fffffff;
			if(cm < m0) {
				if(inreg) {
#pragma unroll
					for(int m = RP - 1; m >= 0; --m)
						if(e0 + m < e1 && rf[m] == cm) first = e0 + m;
				} else {
					for(int e = e0; e < e1; ++e) {
						if(x_f[e] == cm) {
							first = e;
							break;
						}
					}
				}
			}
			first = wave_min_int(first);
			if(lane == 0) s_we[wid] = first;
			if(writer) {
				// accept decisions of this thread's entries: b_e < the running min before e
				double run = dpp_d<DPP_WAVE_SHR1, 0xF>(DBL_MAX, inc);
				run = run < carry ? run : carry;
				const int *x_row = lds ? e_row : b.erow, *x_j = lds ? e_j : b.ej;
				long long nacc = 0, cacc = 0;   // minQpair's own rescans (ctl->ref_rows / ref_cells)
				if(inreg) {
					int rr[RP], rj[RP];
#pragma unroll
					for(int m = 0; m < RP; ++m) {
						rr[m] = rj[m] = 0;
						if(m < per) {   // uniform
							const int e = e0 + m < e1 ? e0 + m : 0;
							rr[m] = x_row[e];
							rj[m] = x_j[e];
						}
					}
#pragma unroll
					for(int m = 0; m < RP; ++m) {
						if(e0 + m >= e1) continue;
						if(rb[m] < run) {
							b.Q[rr[m]] = rf[m];
							b.P[rr[m]] = rj[m];
							++nacc;
							cacc += rr[m];
						}
						run = rf[m] < run ? rf[m] : run;
					}
				} else {
					for(int e = e0; e < e1; ++e) {
						const double f = x_f[e];
						if(x_b[e] < run) {
							b.Q[x_row[e]] = f;
							b.P[x_row[e]] = x_j[e];
							++nacc;
							cacc += x_row[e];
						}
						run = f < run ? f : run;
					}
				}
				nacc = wave_sum_int(nacc);
				cacc = wave_sum_int(cacc);
				if(lane == 0 && nacc) {
					atomicAdd((unsigned long long *) &ctl->ref_rows, (unsigned long long) nacc);
					atomicAdd((unsigned long long *) &ctl->ref_cells, (unsigned long long) cacc);
				}
			}
			__syncthreads();
			if(tid == 0 && cm < m0) {
				int fe = s_we[0];
#pragma unroll
				for(int w = 1; w < TB / 64; ++w) fe = s_we[w] < fe ? s_we[w] : fe;
				s_pi = lds ? e_row[fe] : b.erow[fe];
				s_pj = lds ? e_j[fe] : b.ej[fe];
			}
		}
	}
	__syncthreads();
	TS(3, 3);
	join_tail<ET>(D, bs, b, n, general, s_pi, s_pj, ci, cj, pij, pik, pkj, sDk, Nk, s_neg, s_nj, s_exact);
	TS_EXIT(3);
}

// ------------------------------------------------------------------ DNJ join, large n
// With k_dnj_fold (n > prefold_n) the entries' fresh values and the 64-entry
// chunk summaries are in HBM, in scan order.  Without a "bad" entry minQpair's
// running min is a prefix min (replay_wave's comment), so every block finds
// the pair from the chunk summaries alone: the overall minimum cm and, when it
// improves on m0, the first chunk reaching it.  Each wave then applies its own
// chunk's accept decisions (an entry is accepted iff its stale bound is below
// the running min before it: the owner's prefix over the chunks before, then
// the chunk's own prefix).  Nothing is copied, and no block reads every entry
// (at n = 200k late in configs[3] a join lists ~28k rows).  With a bad entry
// (or force_replay) block 0 runs replay_wave over the entries in HBM and
// publishes the pair (tagged with n); the other blocks wait for it (block 0 is
// dispatched first and waits on no other block).
template <int ET, bool GEN>
__global__ __launch_bounds__(TB) void k_dnj_join_pf(typename Elem<ET>::T *__restrict__ D, double bs, TreeBufs b, int n,
                                                    int general, int force_replay) {
	__shared__ double s_wm[TB / 64], s_tpre[TB];
	__shared__ int s_wi[TB / 64], s_pi, s_pj;
	TreeCtl *ctl = b.ctl;
	const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
	const bool writer = blockIdx.x == 0;
	TS_ENTRY(3);
	TS(3, 0);
	const int k = blockIdx.x * TB + tid;
	const int pos_i = ctl->pos_i, pos_j = ctl->pos_j;
	int ci = pos_i, cj = pos_j;
	ci = ci < 0 || ci >= n ? 0 : ci;
	cj = cj < 0 || cj >= ci ? 0 : cj;
	typename Elem<ET>::T pik = 0, pkj = 0;
	double sDk = 0;
	int Nk = 0;
	if(!general && k < n) {
		sDk = b.sD[k];
		Nk = b.N[k];
		if(k != ci && k != cj) {
			pik = D[k < ci ? tri(ci) + k : tri(k) + ci];
			pkj = D[k < cj ? tri(cj) + k : tri(k) + cj];
		}
	}
	const typename Elem<ET>::T pij = D[tri(ci) + cj];
	const int done = ctl->done, T = ctl->T, nj = ctl->njoins, neg = ctl->neg, exact = ctl->exact;
	const double m0 = ctl->m0;
	if(done) return;
	const int nc = (T + 63) >> 6;
	// this wave's chunk of the accept pass: its loads go out now
	const int cw = (int) blockIdx.x * (TB / 64) + wid, ea = (cw << 6) + lane;
	const bool va = ea < T;
	double af = DBL_MAX, ab = 0;
	int ar = 0, aj = 0;
	if(va) {
		af = b.rf[ea];
		ab = b.cbnd[ea];
		ar = b.crow[ea];
		aj = b.rj[ea];
	}
	// every chunk's minimum and bad flag: thread t holds chunks [t per, (t + 1) per)
	const int per = (nc + TB - 1) / TB, c0 = tid * per, c1 = c0 + per < nc ? c0 + per : nc;
	double tmin = DBL_MAX;
	int bad = force_replay && T > 0;
	for(int c = c0; c < c1; c += 8) {
		double g[8];
		int f[8];
#pragma unroll
		for(int m = 0; m < 8; ++m) {
			const int cc = c + m < c1 ? c + m : c0;
			g[m] = b.chg[cc];
			f[m] = b.chb[cc];
		}
#pragma unroll
		for(int m = 0; m < 8; ++m) {
			if(c + m >= c1) continue;
			tmin = g[m] < tmin ? g[m] : tmin;
			bad |= f[m];
		}
	}
	TS(3, 1);
	if(__syncthreads_or(bad)) {
		// minQpair's serial replay (rare): block 0, entries in HBM
		if(writer) {
			if(wid == 0) {
				int pi = pos_i, pj = pos_j;
				bool had_bad;
				replay_wave(T, m0, b.crow, b.rj, b.cbnd, b.rf, b.eacc, true, b, pi, pj, &had_bad, n);
				if(lane == 0) {
					s_pi = pi;
					s_pj = pj;
					if(had_bad) ctl->serial_replays++;
					__hip_atomic_store(b.jpub, ((unsigned long long) n << 42) | ((unsigned long long) pi << 21) |
					                           (unsigned) pj, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
				}
			}
		} else if(tid == 0) {
			unsigned long long u = 0;
			bool ok = false;
			for(int spin = 0; spin <= (1 << 24) && !ok; ++spin) {
				u = __hip_atomic_load(b.jpub, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
				ok = (int) (u >> 42) == n;
				if(!ok) __builtin_amdgcn_s_sleep(1);
			}
			s_pi = ok ? (int) ((u >> 21) & 0x1fffff) : 0;
			s_pj = ok ? (int) (u & 0x1fffff) : 0;
			if(!ok) {   // never expected: stop the loop and report it (tree_run_t)
				ctl->final_n = -1;
				ctl->done = 1;
			}
		}
		__syncthreads();
		TS(3, 3);
		join_tail<ET>(D, bs, b, n, general, s_pi, s_pj, ci, cj, pij, pik, pkj, sDk, Nk, neg, nj, exact);
		TS_EXIT(3);
		return;   // replay_wave applied the accept decisions
	}
	// the running min is a prefix min: block scan over the slices
	const double inc = wave_incl_min(tmin);
	if(lane == 63) s_wm[wid] = inc;
	__syncthreads();
	double carry = m0, cm = m0;
#pragma unroll
	for(int w = 0; w < TB / 64; ++w) {
		if(w < wid) carry = s_wm[w] < carry ? s_wm[w] : carry;
		cm = s_wm[w] < cm ? s_wm[w] : cm;
	}
	double ex = dpp_d<DPP_WAVE_SHR1, 0xF>(DBL_MAX, inc);   // before this thread's slice
	s_tpre[tid] = ex < carry ? ex : carry;
	// the pair: the first entry reaching cm, when it improves on m0
	int first = 0x7fffffff;
	if(cm < m0 && tmin == cm) {
		for(int c = c0; c < c1; ++c) {
			if(b.chg[c] == cm) {
				first = c;
				break;
			}
		}
	}
	first = wave_min_int(first);
	if(lane == 0) s_wi[wid] = first;
	__syncthreads();
	int i = pos_i, j = pos_j;
	if(cm < m0) {
		int fc = s_wi[0];
#pragma unroll
		for(int w = 1; w < TB / 64; ++w) fc = s_wi[w] < fc ? s_wi[w] : fc;
		i = b.chr[fc];
		j = b.chj[fc];
	}
	TS(3, 3);
	join_tail<ET>(D, bs, b, n, general, i, j, ci, cj, pij, pik, pkj, sDk, Nk, neg, nj, exact);
	// accept decisions of this wave's chunk
	if(cw < nc) {   // uniform per wave
		const int t = cw / per, cs = t * per;
		double pc = s_tpre[t];
		for(int x0 = cs; x0 < cw; x0 += 64) {   // the owner's chunks before cw
			const double g = x0 + lane < cw ? b.chg[x0 + lane] : DBL_MAX;
			pc = g < pc ? g : pc;
		}
		pc = readlane_d(wave_incl_min(pc), 63);
		double run = dpp_d<DPP_WAVE_SHR1, 0xF>(DBL_MAX, wave_incl_min(af));
		run = run < pc ? run : pc;
		const bool acc = va && ab < run;
		if(acc) {
			b.Q[ar] = af;
			b.P[ar] = aj;
		}
		const long long nacc = __popcll(__ballot(acc)), cacc = wave_sum_int((long long) (acc ? ar : 0));
		if(lane == 0 && nacc) {
			atomicAdd((unsigned long long *) &ctl->ref_rows, (unsigned long long) nacc);
			atomicAdd((unsigned long long *) &ctl->ref_cells, (unsigned long long) cacc);
		}
	}
	TS_EXIT(3);
}

// ------------------------------------------------------------------ general updateD
// nj.c:836-1044 with entries < 0 ("missing"): one block walks k in chunks,
// reproducing the lagging sD/N cursor and the out-of-row read D_j[k] of the
// D_kj-only column branch (nj.c:1022).  Leaves the serial row sum in wsum[0]
// and the count in wcnt[0] for the fold that follows.
template <int ET>
__global__ __launch_bounds__(1024) void k_update_general(typename Elem<ET>::T *__restrict__ D, double bs, TreeBufs b,
                                                         int n) {
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
		b.wsum[0] = sd;
		b.wcnt[0] = s_cnt;
	}
}

// ------------------------------------------------------------------ DNJ requeue
// Row sum of j, then updateDNJ's Q/P part (dnj.c:618-709) and DNJ_popArrange
// (dnj.c:817-975); the four (q, idx) reductions go to per-block partials that
// the next k_dnj_select folds.
template <int ET, bool BANDS, bool VBLK = false>
__global__ __launch_bounds__(TB) void k_dnj_requeue(typename Elem<ET>::T *__restrict__ D, double bs, TreeBufs b,
                                                    int n, int general, int exact_arg) {
	__shared__ double sq[5][TB / 64], sfq[TB / 64];
	__shared__ int si[5][TB / 64], sfp[TB / 64], sbp[TB / 64];
	__shared__ double sfv[TB / 64], sbq[TB / 64];
	__shared__ double s_sd;
	__shared__ int s_nj, s_i, s_j, s_stop, s_serial, s_chain;
	TreeCtl *ctl = b.ctl;
	const int nn = n - 1;
	const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
	const int k = blockIdx.x * TB + tid;
	TS_ENTRY(4);
	TS(4, 0);
	int Nk = 0, pkk0 = 0;
	double sDk = 0, qk0 = 0;
	typename Elem<ET>::T vm = 0;
	if(k < n) {
		Nk = b.N[k];
		sDk = b.sD[k];
		qk0 = b.Q[k];
		pkk0 = b.P[k];
	}
	if(k < nn) vm = D[tri(nn) + k];   // row nn, moved to i
	// VBLK: the cell at the row's partner and the partner's row sum, for the
	// row's bound V_k of the next join's scan (prefetched: usually unchanged)
	typename Elem<ET>::T vp = 0;
	double sdp0 = 0.0;
	const bool PV = VBLK || b.ubq;   // (uniform) the partner cells are wanted
	if(PV && k >= 1 && k < n) {
		const int p0 = pkk0 >= 0 && pkk0 < k ? pkk0 : 0;
		vp = D[tri(k) + p0];
		sdp0 = b.sD[p0];
	}
	const int Nm0 = b.N[nn];
	const double sDm0 = b.sD[nn];
	// column j of the joined pair, read by every thread (not through wave 0's
	// LDS copy), so these loads overlap wave 0's row sum; row i's writes below
	// never touch column j
	int jq = ctl->j;
	jq = jq < 0 || jq >= n ? 0 : jq;
	typename Elem<ET>::T vj = 0;
	if(k < n && k != jq) vj = k < jq ? D[tri(jq) + k] : D[tri(k) + jq];
	if(wid == 0) {
		const int done = ctl->done;
		const bool exact = exact_arg != 0;   // a launch argument: the row sum's loads wait for no ctl load
		if(lane == 0) {
			s_i = ctl->i;
			s_j = ctl->j;
			s_stop = done;
		}
		{   // also once the loop stopped (the result is unused then): nothing waits for `done`
			double sd;
			int nj;
			bool need, chain;
			row_sum_j_wave(b, n, exact, general, &sd, &nj, &need, &chain);
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
	const int i = s_i, j = s_j, Nj = s_nj;
	// exact mode, a failed check of the parallel form: the serial chain (all threads)
	if(s_chain) {
		const double r = serial_sum_t<TB>(b.contrib, n);
		if(tid == 0) s_sd = r;
		if(blockIdx.x == 0 && tid == 0) ctl->chain_sums++;
		__syncthreads();
	}
	const double sdj = s_sd;
	TS(4, 1);
	if(blockIdx.x == 0 && tid == 0) {
		b.sD[j] = sdj;
		b.N[j] = Nj;
		if(s_serial) ctl->serial_sums++;
	}
	const bool move = i != nn;
	const int Nm = move ? Nm0 : 0;
	const double sDm = move ? sDm0 : 0;
	if(k == j) {
		Nk = Nj;
		sDk = sdj;
	}
	double rq = DBL_MAX, pq = DBL_MAX, r2q = DBL_MAX, p2q = DBL_MAX, fq = DBL_MAX;
	int rj = 0, pk = -1, r2j = 0, p2k = -1, fp = 0;
	if(k < n) {
		if(k < j) {
			double d = Elem<ET>::get(vj, bs);   // j == jq (ctl->j, read twice)
			if(0 <= d) {
				rq = qcrit(Nj, Nk, d, sdj, sDk);
				rj = k;
			}
		}
		if(k > j && k != i) {
			double qk = qk0;
			int pkk = pkk0;
			bool upd = false;
			double d = Elem<ET>::get(vj, bs);
			if(0 <= d) {
				double q = qcrit(Nj, Nk, d, sdj, sDk);
				if(q <= qk) {
					qk = q;
					pkk = j;
					upd = true;
					pq = q;
					pk = k;
				}
			}
			if(move && k > i && k < nn) {
				D[tri(k) + i] = vm;
				double dm = Elem<ET>::get(vm, bs);
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
			fq = qk;    // the row's final (Q, P), carried with (pq, pk)
			fp = pkk;
		}
		if(move && k < i) {
			D[tri(i) + k] = vm;
			double dm = Elem<ET>::get(vm, bs);
			if(0 <= dm) {
				r2q = qcrit(Nm, Nk, dm, sDm, sDk);
				r2j = k;
			}
		}
	}
	if(b.lbm) {   // (uniform) block bounds of the next join: row i = the moved row, column i; sD maxima
		const unsigned x = lb_bits(Elem<ET>::get(vm, bs));
		if(move) {
			const unsigned mn = wave_min_u32(k < i ? x : 0xFFFFFFFFu);
			if(lane == 0 && k < i) b.lbm[(long long) i * b.lbs + (k >> 6)] = mn;
			if(k > i && k < nn) __hip_atomic_fetch_min(b.lbm + (long long) k * b.lbs + (i >> 6), x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		}
		const double sf = k < nn ? (move && k == i ? sDm : sDk) : -DBL_MAX;   // sD of column k at the next join
		const double mx = wave_max_d(sf);
		if(lane == 0 && k < nn) b.msd[k >> 6] = mx;
	}
	// VBLK: V_k = max(q at the row's partner cell, Q_k) in the next join's
	// state, a bound of minQpair's running min below row k whatever the
	// reference does with it (a cell of row k is >= its fresh minimum); the
	// block minimum, for the next scan's suffix bound over the rows above
	// ubq (block bounds): the same q, the next scan's threshold for row k
	double vk = DBL_MAX, qpc = INFINITY;
	if(PV && k >= 1 && k < nn && k != i && k != j) {
		const bool later = k > j;   // rows above j may have a new partner (j or the moved i)
		const int pf = later ? fp : pkk0;
		const double qf = later ? fq : qk0;
		double d = -1.0, sp = 0.0;
		if(pf == j && later) {
			d = Elem<ET>::get(vj, bs);
			sp = sdj;
		} else if(pf == i && move && later) {
			d = Elem<ET>::get(vm, bs);
			sp = sDm;
		} else if(pf == pkk0 && pkk0 >= 0 && pkk0 < k && pkk0 != i && pkk0 != j) {
			d = Elem<ET>::get(vp, bs);
			sp = sdp0;
		}
		if(0 <= d) {
			const double q = qcrit(nn, nn, d, sDk, sp);
			qpc = q;
			vk = q > qf ? q : qf;
		}
		if(b.ubq) b.ubq[k] = qpc;
	}
	if(VBLK) {
		vk = readlane_d(wave_incl_min(vk), 63);
		if(lane == 0) sfv[wid] = vk;
	}
	// the row's bound for the next join: each block's min-Q row becomes a
	// candidate of the next S (rows j and i take theirs from k_dnj_select's
	// fold); only when the next S has a band part
	// (with ubq, also the q at that partner cell: the plan then needs no load for it)
	double bq = DBL_MAX, bqc = INFINITY;
	int bk = 0, bp = 0;
	if(BANDS) {
		if(k >= 1 && k < nn && k != i && k != j) {
			bq = k > j ? fq : qk0;
			bk = k;
			bp = k > j ? fp : pkk0;   // its partner, for k_dnj_plan's partner-cell bound
			bqc = qpc;
		}
		qarg_wave_reduce_carry(bq, bk, bqc, bp);
	}
	qarg_wave_reduce(rq, rj);
	qarg_wave_reduce_carry(pq, pk, fq, fp);
	qarg_wave_reduce(r2q, r2j);
	qarg_wave_reduce(p2q, p2k);
	if(lane == 0) {
		sq[0][wid] = rq;
		si[0][wid] = rj;
		sq[1][wid] = pq;
		si[1][wid] = pk;
		sfq[wid] = fq;
		sfp[wid] = fp;
		sq[2][wid] = r2q;
		si[2][wid] = r2j;
		sq[3][wid] = p2q;
		si[3][wid] = p2k;
		if(BANDS) {
			sq[4][wid] = bq;
			si[4][wid] = bk;
			sbp[wid] = bp;
			sbq[wid] = bqc;
		}
	}
	__syncthreads();
	if(tid < (BANDS ? 5 : 4)) {
		double q = sq[tid][0], cq = sfq[0], xq = BANDS ? sbq[0] : 0.0;
		int ix = si[tid][0], cp = sfp[0], xp = BANDS ? sbp[0] : 0;
		for(int w = 1; w < TB / 64; ++w) {
			if(qarg_better(sq[tid][w], si[tid][w], q, ix)) {
				q = sq[tid][w];
				ix = si[tid][w];
				cq = sfq[w];
				cp = sfp[w];
				if(BANDS) {
					xp = sbp[w];
					xq = sbq[w];
				}
			}
		}
		if(tid == 4) {
			b.bmq[blockIdx.x] = q;
			b.bmr[blockIdx.x] = ix;
			b.bmp[blockIdx.x] = xp;
			b.bmqp[blockIdx.x] = xq;
		} else {
			b.qpart[4 * blockIdx.x + tid] = q;
			b.ipart[4 * blockIdx.x + tid] = ix;
		}
		if(tid == 1) {
			b.cfq[blockIdx.x] = cq;
			b.cfp[blockIdx.x] = cp;
		}
	}
	if(VBLK && tid == 0) {
		double v = sfv[0];
		for(int w = 1; w < TB / 64; ++w) v = sfv[w] < v ? sfv[w] : v;
		b.bmv[blockIdx.x] = v;
		if(blockIdx.x == 0) ctl->vtag = nn;   // the join these minima serve
	}
	TS(4, 2);
	TS_EXIT(4);
}


// ------------------------------------------------------------------ NJ argmin
// nj.c:182 initQ: min starts at 1, the last minimal cell in row-major order
// (larger flat index wins ties).  Blocks tile the triangle in NJ_SEG-column
// segments x NJ_RB-row bands, enumerated segment-major: segment s holds the
// bands from row s*NJ_SEG on, so block -> (s, band) is closed-form.  A thread
// keeps its 8 columns' sD in registers for all the band's rows (sD[r] is one
// scalar per row), so D is the only per-cell stream.
__host__ __device__ __forceinline__ long long nj_prefix(long long s, long long nb) {
	return s * nb - (long long) (NJ_SEG / NJ_RB) * s * (s - 1) / 2;
}
__host__ __device__ __forceinline__ long long nj_blocks(int n) {
	const long long nb = (n + NJ_RB - 1) / NJ_RB, nseg = (n - 1 + NJ_SEG - 1) / NJ_SEG;
	return nj_prefix(nseg, nb);
}

template <int ET, bool GEN>
__global__ __launch_bounds__(TB) void k_nj_argmin(const typename Elem<ET>::T *__restrict__ D, double bs, TreeBufs b,
                                                  int n) {
	__shared__ double sq[TB / 64];
	__shared__ long long sf[TB / 64];
	if(b.ctl->done) return;
	const long long nb = (n + NJ_RB - 1) / NJ_RB;
	const long long idx = blockIdx.x;
	long long s = 0;
	while(nj_prefix(s + 1, nb) <= idx) ++s;
	const int band = (int) ((NJ_SEG / NJ_RB) * s + (idx - nj_prefix(s, nb)));
	const int c0 = (int) s * NJ_SEG;
	constexpr int M = NJ_SEG / TB;
	double sc[M];
	int nc[M];
#pragma unroll
	for(int m = 0; m < M; ++m) {
		int c = c0 + m * TB + (int) threadIdx.x;
		c = c < n ? c : n - 1;
		sc[m] = b.sD[c];
		nc[m] = GEN ? b.N[c] : n;
	}
	double bq = 1.0;
	long long bf = -1;
	const int r0 = band * NJ_RB, r1 = r0 + NJ_RB < n ? r0 + NJ_RB : n;
	constexpr int G = 4;   // rows per step: G*M loads in flight
	for(int rg = r0; rg < r1; rg += G) {
		typename Elem<ET>::T v[G][M];
		double sr[G];
		int nr[G];
#pragma unroll
		for(int g = 0; g < G; ++g) {
			const int r = rg + g < r1 ? rg + g : r1 - 1;
			const long long base = tri(r);
			sr[g] = b.sD[r];
			nr[g] = GEN ? b.N[r] : n;
#pragma unroll
			for(int m = 0; m < M; ++m) {
				const int c = c0 + m * TB + (int) threadIdx.x;
				v[g][m] = D[base + (c < r ? c : 0)];
			}
		}
#pragma unroll
		for(int g = 0; g < G; ++g) {
			const int r = rg + g;
			const long long base = tri(r);
#pragma unroll
			for(int m = 0; m < M; ++m) {
				const int c = c0 + m * TB + (int) threadIdx.x;
				const double d = Elem<ET>::get(v[g][m], bs);
				const double q = qcrit(nr[g], nc[m], d, sr[g], sc[m]);
				const long long f = base + c;
				const bool take = r < r1 && c < r && 0 <= d && (q < bq || (q == bq && f > bf));
				bq = take ? q : bq;
				bf = take ? f : bf;
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

// fold of the argmin partials (wave 0), limbLength, the join record and updateD
template <int ET>
__global__ __launch_bounds__(TB) void k_nj_join(typename Elem<ET>::T *__restrict__ D, double bs, TreeBufs b, int n,
                                                int G, int general, double q0) {
	__shared__ long long s_bf, s_wf[TB / 64];
	__shared__ double s_wq[TB / 64];
	__shared__ int s_stop, s_nj, s_neg, s_exact;
	TreeCtl *ctl = b.ctl;
	const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
	const int k = blockIdx.x * TB + tid;
	double sDk = 0;
	int Nk = 0;
	if(k < n) {
		sDk = b.sD[k];
		Nk = b.N[k];
	}
	// fold of the argmin partials by the whole block (G grows as n^2)
	double fq = q0;
	long long ff = -1;
	for(int g = tid; g < G; g += TB) {
		double oq = b.qpart[g];
		long long of = b.fpart[g];
		if(oq < fq || (oq == fq && of > ff)) {
			fq = oq;
			ff = of;
		}
	}
	qf_wave_reduce(fq, ff);
	if(lane == 0) {
		s_wq[wid] = fq;
		s_wf[wid] = ff;
	}
	if(tid == 0) {
		s_stop = ctl->done;
		s_nj = ctl->njoins;
		s_neg = ctl->neg;
		s_exact = ctl->exact;
	}
	__syncthreads();
	if(tid == 0) {
		for(int w = 1; w < TB / 64; ++w) {
			if(s_wq[w] < fq || (s_wq[w] == fq && s_wf[w] > ff)) {
				fq = s_wq[w];
				ff = s_wf[w];
			}
		}
		s_bf = ff;
	}
	__syncthreads();
	if(s_stop) return;
	const bool writer = blockIdx.x == 0 && tid == 0;
	const long long bf = s_bf;
	if(bf < 0) {
		if(writer) {
			ctl->done = 1;
			ctl->final_n = n;
		}
		return;
	}
	long long r = (long long) ((1.0 + sqrt(1.0 + 8.0 * (double) bf)) * 0.5);
	while(r > 1 && tri(r) > bf) --r;
	while(tri(r + 1) <= bf) ++r;
	const int i = (int) r, j = (int) (bf - tri(r));
	const double Dij = Elem<ET>::get(D[bf], bs);
	double Dik = 0, Dkj = 0;
	if(!general && k < n && k != i && k != j) {
		Dik = Elem<ET>::get(D[k < i ? tri(i) + k : tri(k) + i], bs);
		Dkj = Elem<ET>::get(D[k < j ? tri(j) + k : tri(k) + j], bs);
	}
	if(writer) {
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
	if(general) return;
	update_body<ET>(D, bs, b, n, i, j, Dij, s_exact, k, Dik, Dkj, sDk, Nk, blockIdx.x);
}

// row sum of j, then matrix.c:518 ltdMatrix_popArrange + nj.c:1588-1589
template <int ET>
__global__ __launch_bounds__(TB) void k_nj_pop(typename Elem<ET>::T *__restrict__ D, TreeBufs b, int n, int general, int exact_arg) {
	__shared__ double s_sd;
	__shared__ int s_nj, s_i, s_j, s_stop, s_serial, s_chain;
	TreeCtl *ctl = b.ctl;
	const int nn = n - 1;
	const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
	const int k = blockIdx.x * TB + tid;
	typename Elem<ET>::T vm = 0;
	if(k < nn) vm = D[tri(nn) + k];
	const double sDm = b.sD[nn];
	const int Nm = b.N[nn];
	if(wid == 0) {
		const int done = ctl->done;
		const bool exact = exact_arg != 0;   // a launch argument: the row sum's loads wait for no ctl load
		if(lane == 0) {
			s_i = ctl->i;
			s_j = ctl->j;
			s_stop = done;
		}
		{   // also once the loop stopped (the result is unused then): nothing waits for `done`
			double sd;
			int nj;
			bool need, chain;
			row_sum_j_wave(b, n, exact, general, &sd, &nj, &need, &chain);
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
			D[tri(i) + k] = vm;
		} else if(k > i && k < nn) {
			D[tri(k) + i] = vm;
		}
	}
}


// ------------------------------------------------------------------ HNJ
// hclust.c:1671 hclust with initHNJ / minQ / updateHNJ / HNJ_popArrange
// (-m hnj).  Every step is O(n) per join; per join:
//   k_hnj_argmin  folds the last join's two row minima (row j from
//                 k_hnj_update, row i from its pop) into Q/P, then per-block
//                 minQ partials (q, tri(r) + P[r]) over rows 1..n-1: P[r] < r,
//                 so the larger flat index is the later row, minQ's `<=` rule
//                 (hclust.c:353);
//   k_nj_join     (shared with NJ, fold start DBL_MAX) limbLength, the join
//                 record and updateD;
//   k_hnj_update  per row k: updatePrevQ (hclust.c:413, rows 0..n-2, row 0
//                 reading flat element P[0]) then updateHNJ's column-j rule
//                 (hclust.c:516-558), the row-j minimum as per-block partials,
//                 and HNJ_popArrange (hclust.c:1308) in the same pass: row
//                 n-1 into row i (its minimum as partials) and column i with
//                 `P < pos || q < Q`.

// (qk_take, qk_block_reduce, qk_fold_wave: ccg_tree_common.h, shared with the sharded HNJ)

template <int UNUSED = 0>
__global__ __launch_bounds__(TB) void k_hnj_argmin(TreeBufs b, int n) {
	__shared__ double sq[TB / 64], fq[2];
	__shared__ long long sf[TB / 64];
	__shared__ int fk[2];
	const TreeCtl *ctl = b.ctl;
	if(ctl->done) return;
	const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
	const int r = (int) blockIdx.x * TB + tid;
	const int hj = ctl->hj, hi = ctl->hi;
	const bool own_j = hj >= 0 && hj / TB == (int) blockIdx.x, own_i = hi >= 0 && hi / TB == (int) blockIdx.x;
	if(blockIdx.x == 0 && tid == 0 && hi >= 0) {   // the pop's sD/N of row i (row n before the join)
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
		if(r >= 1 && qr <= DBL_MAX) {
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
__global__ __launch_bounds__(TB) void k_hnj_update(typename Elem<ET>::T *__restrict__ D, double bs, TreeBufs b,
                                                   int n, int general, int exact_arg) {
	__shared__ double s_sd, sq[TB / 64], sq2[TB / 64];
	__shared__ int s_nj, s_i, s_j, s_stop, s_serial, s_chain, sk[TB / 64], sk2[TB / 64];
	TreeCtl *ctl = b.ctl;
	const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
	const int k = (int) blockIdx.x * TB + tid;
	if(wid == 0) {
		const int done = ctl->done;
		const bool exact = exact_arg != 0;   // a launch argument: the row sum's loads wait for no ctl load
		if(lane == 0) {
			s_i = ctl->i;
			s_j = ctl->j;
			s_stop = done;
		}
		{   // also once the loop stopped (the result is unused then): nothing waits for `done`
			double sd;
			int nj;
			bool need, chain;
			row_sum_j_wave(b, n, exact, general, &sd, &nj, &need, &chain);
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
	const int nj = s_nj;
	const int nn = n - 1;
	const bool move = i != nn;
	if(blockIdx.x == 0 && tid == 0) {
		b.sD[j] = sdj;
		b.N[j] = nj;
		ctl->hj = j;
		ctl->hjb = (int) cdiv(j, TB);
		// row i of the pop: its minimum is in this kernel's partials; its sD/N
		// (row nn's) are persisted by the next k_hnj_argmin (sD[i] is still
		// read here as a partner's sum)
		ctl->hi = move ? i : -1;
		ctl->hib = (int) cdiv(i, TB);
		if(s_serial) ctl->serial_sums++;
	}
	double rq = DBL_MAX, pq = DBL_MAX;
	int rk = -1, pk2 = -1;
	if(k < n) {
		const int Nk = k == j ? nj : b.N[k];
		const double sDk = k == j ? sdj : b.sD[k];
		double Qk = b.Q[k];
		int Pk = b.P[k];
		if(k <= n - 2) {   // updatePrevQ (hclust.c:441-449)
			const int pk = Pk;
			const double d = Elem<ET>::get(D[tri(k) + pk], bs);
			if(0 <= d) {
				const int Np = pk == j ? nj : b.N[pk];
				const double sDp = pk == j ? sdj : b.sD[pk];
				Qk = ((Nk + Np - 4) >> 1) * d - sDk - sDp;
			}
		}
		if(k > j && k != i) {   // column j (hclust.c:530-556)
			const double d = Elem<ET>::get(D[tri(k) + j], bs);
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
		if(k < j) {   // row j (hclust.c:497-511)
			const double d = Elem<ET>::get(D[tri(j) + k], bs);
			if(0 <= d) {
				rq = ((nj + Nk - 4) >> 1) * d - sdj - sDk;
				rk = k;
			}
		}
		// HNJ_popArrange (hclust.c:1308) in the same pass: row nn moves to row
		// i (cells k < i; its minimum as partials) and column i (rows i < k < nn,
		// `q <= Q && (P < pos || q < Q)`).  Thread k read its own cells of row /
		// column i above; row nn is not written by this kernel.
		if(move && k < nn && k != i) {
			const typename Elem<ET>::T vm = D[tri(nn) + k];
			const double d = Elem<ET>::get(vm, bs);
			const double sDi = b.sD[nn];
			const int Ni = b.N[nn];
			const double q = 0 <= d ? d * ((Ni + Nk - 4) >> 1) - sDi - sDk : 0.0;
			if(k < i) {
				D[tri(i) + k] = vm;
				if(0 <= d) {
					pq = q;
					pk2 = k;
				}
			} else {
				D[tri(k) + i] = vm;
				if(0 <= d && q <= Qk && (Pk < i || q < Qk)) {
					Qk = q;
					Pk = i;
				}
			}
		}
		if(k != j) {
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

// ------------------------------------------------------------------ host
// The device layout of one tree run (one allocation), sized for n taxa:
// returns its bytes, and with m != NULL points b's arrays into it.
static size_t tree_layout(TreeBufs *bp, int n, char *m) {
	const size_t nb = (size_t) cdiv(n, TB) + 1;
	const size_t maxu = cdiv(n, SEG_S) + 1;   // S rows' units (SEG_S cells)
	// every row below S may qualify: room for n entries and their units
	const size_t ncand = (size_t) n + 257;
	// entry e's rescan units are [e umax, (e + 1) umax) (k_dnj_scan): room for
	// ncand entries at the largest umax of the run (seg grows with n in steps
	// at n = 16384 m, so the maximum is at n or just below a step)
	DnjGrid g;
	g.load();
	int umax = dnj_umax(n, g.seg(n));
	for(int mm = 2; mm <= 9; ++mm) {
		const int k = 16384 * mm - 1;
		if(k <= n && dnj_umax(k, g.seg(k)) > umax) umax = dnj_umax(k, g.seg(k));
	}
	size_t cunits = ncand * (size_t) umax;
	if(cunits < JOIN_UPRE) cunits = JOIN_UPRE;
	const size_t nq = (size_t) nj_blocks(n) + 1;
	size_t sz = 0;
	auto take = [&](size_t bytes) {
		size_t off = sz;
		sz += (bytes + 255) & ~(size_t) 255;
		return off;
	};
	size_t o_sD = take((n + 1) * 8), o_Q = take((n + 1) * 8), o_c = take((n + 1) * 8);
	size_t o_N = take((n + 1) * 4), o_P = take((n + 1) * 4);
	size_t o_S = take(DNJ_B * 4), o_uo = take((DNJ_B + 1) * 4), o_Sb = take(DNJ_B * 8);
	size_t o_uq = take(DNJ_B * maxu * 8), o_uj = take(DNJ_B * maxu * 4);
	size_t o_Se = take(DNJ_B * sizeof(Entry));
	const size_t nent = (size_t) DNJ_B + ncand;
	size_t o_ef = take(nent * 8), o_eb = take(nent * 8), o_er = take(nent * 4), o_ej = take(nent * 4);
	size_t o_ea = take(nent);
	size_t o_cr = take(ncand * 4), o_cb = take(ncand * 8), o_co = take(ncand * 4);
	size_t o_cq = take(cunits * 8), o_cj = take(cunits * 4);
	size_t o_ws = take(nb * 8), o_wa = take(nb * 8), o_wc = take(nb * 4), o_we = take(nb * 4);
	size_t o_qp = take((nb > nq ? nb : nq) * 4 * 8), o_ip = take((nb > nq ? nb : nq) * 4 * 4);
	size_t o_fp = take(nq * 8), o_cfq = take(nb * 8), o_cfp = take(nb * 4);
	size_t o_j = take((size_t) n * sizeof(ccg_join)), o_ctl = take(sizeof(TreeCtl));
	const size_t nrf = ncand > JOIN_UPRE ? ncand : JOIN_UPRE;   // k_dnj_join prefetches JOIN_UPRE
	size_t o_bp = take(nb * 4), o_bqp = take(nb * 8);
	size_t o_bq = take(nb * 8), o_br = take(nb * 4), o_sp = take((DNJ_B + 1) * 4), o_cs = take(ncand * 4);
	size_t o_rf = take(nrf * 8), o_rj = take(nrf * 4);
	size_t o_xa = take(nb * 8), o_xb = take(nb * sizeof(XsBlk)), o_xc = take(nb * XB_CAP * sizeof(XsCross));
	size_t o_xt = take(nb * XB_CAP_T * sizeof(XsTie));
	size_t o_pp = take(PLAN_MAXB * 8), o_jp = take(8);
	const size_t nch = ncand / 64 + 2;   // k_dnj_fold's chunk summaries
	size_t o_hg = take(nch * 8), o_hr = take(nch * 4), o_hj = take(nch * 4), o_hb = take(nch * 4);
	size_t o_ec = take(nent * 4), o_cc = take(nch * 4);
	size_t o_pr = take(DNJ_B * 4), o_pe = take(DNJ_B * 4), o_pu = take((DNJ_B + 1) * 4), o_pq = take(DNJ_B * 8);
	size_t o_pb = take(DNJ_B * 8), o_eS = take(nent), o_bv = take(nb * 8), o_vs = take(nb * 8);
	size_t o_sr = take(SRDY_REP * 128), o_uh = take((size_t) PLAN_MAXB * UHIST * 4);
	size_t o_bc = take(UHIST * 4), o_bl = take(ncand * 4), o_ep = take(nent);
	size_t o_sh = take(128), o_sf = take(DNJ_B * 8), o_sj = take(DNJ_B * 4), o_es = take(DNJ_B * 4);
	if(!m) return sz;
	TreeBufs &b = *bp;
	b.sD = (double *) (m + o_sD);
	b.Q = (double *) (m + o_Q);
	b.contrib = (double *) (m + o_c);
	b.N = (int *) (m + o_N);
	b.P = (int *) (m + o_P);
	b.S = (int *) (m + o_S);
	b.uoff = (int *) (m + o_uo);
	b.Sb = (double *) (m + o_Sb);
	b.uq = (double *) (m + o_uq);
	b.uj = (int *) (m + o_uj);
	b.Sent = (Entry *) (m + o_Se);
	b.ef = (double *) (m + o_ef);
	b.eb = (double *) (m + o_eb);
	b.erow = (int *) (m + o_er);
	b.ej = (int *) (m + o_ej);
	b.eacc = (unsigned char *) (m + o_ea);
	b.crow = (int *) (m + o_cr);
	b.cbnd = (double *) (m + o_cb);
	b.cq = (double *) (m + o_cq);
	b.coff = (int *) (m + o_co);
	b.cj = (int *) (m + o_cj);
	b.wsum = (double *) (m + o_ws);
	b.wabs = (double *) (m + o_wa);
	b.wcnt = (int *) (m + o_wc);
	b.wexp = (int *) (m + o_we);
	b.qpart = (double *) (m + o_qp);
	b.ipart = (int *) (m + o_ip);
	b.fpart = (long long *) (m + o_fp);
	b.cfq = (double *) (m + o_cfq);
	b.cfp = (int *) (m + o_cfp);
	b.joins = (ccg_join *) (m + o_j);
	b.bmq = (double *) (m + o_bq);
	b.bmr = (int *) (m + o_br);
	b.bmp = (int *) (m + o_bp);
	b.bmqp = (double *) (m + o_bqp);
	b.Spos = (int *) (m + o_sp);
	b.cslot = (int *) (m + o_cs);
	b.rf = (double *) (m + o_rf);
	b.rj = (int *) (m + o_rj);
	b.ctl = (TreeCtl *) (m + o_ctl);
	b.xagg = (unsigned long long *) (m + o_xa);
	b.xblk = (XsBlk *) (m + o_xb);
	b.xcr = (XsCross *) (m + o_xc);
	b.xti = (XsTie *) (m + o_xt);
	b.ppub = (unsigned long long *) (m + o_pp);
	b.jpub = (unsigned long long *) (m + o_jp);
	b.chg = (double *) (m + o_hg);
	b.chr = (int *) (m + o_hr);
	b.chj = (int *) (m + o_hj);
	b.chb = (int *) (m + o_hb);
	b.ecnt = (unsigned *) (m + o_ec);
	b.ccnt = (unsigned *) (m + o_cc);
	b.pS_row = (int *) (m + o_pr);
	b.pS_ent = (int *) (m + o_pe);
	b.pS_uo = (int *) (m + o_pu);
	b.pS_q = (double *) (m + o_pq);
	b.pS_bnd = (double *) (m + o_pb);
	b.eS = (unsigned char *) (m + o_eS);
	b.bmv = (double *) (m + o_bv);
	b.vsuf = (double *) (m + o_vs);
	b.srdy = (unsigned *) (m + o_sr);
	b.uhist = (int *) (m + o_uh);
	b.bcnt = (int *) (m + o_bc);
	b.blist = (int *) (m + o_bl);
	b.ePr = (unsigned char *) (m + o_ep);
	b.shdr = (unsigned long long *) (m + o_sh);
	b.sfq = (double *) (m + o_sf);
	b.sfj = (int *) (m + o_sj);
	b.ecS = (unsigned *) (m + o_es);
	b.maxu = (int) maxu;
	b.lbm = NULL;   // the block bounds: tree_run_t's own allocation (single engine, DNJ)
	b.msd = NULL;
	b.ubq = NULL;
	b.lbs = 0;
	b.lbw = 0;
	b.lbskip = NULL;
	// the all-records walk (CCG_XS_ALLPRE=1): configs[1] 22.3k joins/s against 22.5k block by block, the
	// headline tree the same (round 5, measured): off by default
	b.xs_allpre = getenv("CCG_XS_ALLPRE") && atoi(getenv("CCG_XS_ALLPRE")) != 0;
	return sz;
}

size_t ccg_tree_bytes(int n) { return tree_layout(NULL, n, NULL); }

int ccg_tree_alloc(TreeWork *w, int n, hipStream_t st) {
	const size_t sz = tree_layout(NULL, n, NULL);
	char *m;
	CCG_CHECK(hipMalloc((void **) &m, sz));
	CCG_CHECK(hipMemsetAsync(m, 0, sz, st));
	w->mem = m;
	tree_layout(&w->b, n, m);
	return CCG_OK;
}

// the single engine's workspace: the context's cached slot 0 (no hipFree per run)
static int tree_alloc_ctx(ccg_ctx *c, TreeWork *w, int n) {
	const size_t sz = tree_layout(NULL, n, NULL);
	void *m;
	const int rc = ccg_ctx_workspace(c, 0, sz, &m);
	if(rc) return rc;
	CCG_CHECK(hipMemsetAsync(m, 0, sz, c->stream));
	w->mem = m;
	tree_layout(&w->b, n, (char *) m);
	return CCG_OK;
}

// DNJ: k_dnj_plan of the join at matrix size n (first: the run's first join,
// whose candidate k_dnj_prep or a resumed state left in ctl)
// the scan rescans S first and prunes the other entries under S's exact
// fresh minima: band mode, the wave scans with the fold at their last
// arrivals, no missing entries
// (scan_prune 1: the S phase inside the scan, with FoldTail; 2: S rescanned by
// k_dnj_sphase, its own launch, then the wave scan with k_dnj_fold)
static int dnj_prune(int n, int et, bool gen) {
	const int sm = g_grid.scan_mode(n, et);
	if(gen || !g_grid.bands(n) || !g_grid.prefold(n)) return 0;
	if(g_grid.scan_prune == 1 && g_grid.scan_fold && ((sm >= 4 && sm < 20) || (sm >= 20 && sm <= 23))) return 1;
	// prune 2 with the row groups: the compacted group scan (k_dnj_scan_gc) enumerates the survivors
	const bool gcmp = sm >= 20 && sm <= 23 && g_grid.scan_cmp && dnj_umax(n, g_grid.seg(n)) < UHIST;
	if(g_grid.scan_prune == 2 && g_grid.prune_on && !g_grid.scan_fold && ((sm >= 4 && sm < 20) || gcmp)) return 2;
	return 0;
}

template <int ET, bool GEN>
static void enqueue_plan(hipStream_t st, typename Elem<ET>::T *D, double bs, const TreeBufs &b, int n, int first) {
	const int seg = g_grid.seg(n);
	const unsigned gp = g_grid.plan_blocks(n);
	const int prune = dnj_prune(n, ET, GEN);
	const int nh = prune == 2 && g_grid.plan_help ? g_grid.plan_help : 0;   // S's rescans by helper blocks
	if(g_grid.bands(n)) k_dnj_plan<ET, GEN, DenseRows, true><<<gp + nh, TBF, 0, st>>>(D, bs, b, n, first, DenseRows(), seg, g_grid.top(n), g_grid.bands(n), g_grid.plan_flags(prune != 0, nh));
	else k_dnj_plan<ET, GEN, DenseRows, false><<<gp, TBF, 0, st>>>(D, bs, b, n, first, DenseRows(), seg, g_grid.top(n), 0, g_grid.plan_flags());
}

// One join's kernels for a matrix of n taxa; returns the launch count.
template <int ET, bool GEN>
static int enqueue_iteration(hipStream_t st, typename Elem<ET>::T *D, double bs, const TreeBufs &b, int n, int first,
                             int method, int exact, KTimer &kt) {
	const unsigned gn = cdiv(n, TB);
	const int general = GEN;
	const int xs = 0;   // exact row sums: split over the join kernel and its consumer (xs_join_row, xs_walk_blocks)
	if(method == CCG_TREE_DNJ) {
		const unsigned gc = g_grid.scan(n);
		const int seg = g_grid.seg(n), prefold = g_grid.prefold(n);
		// one-phase search: k_dnj_plan lists S and the rows below it under the
		// partner-cell bound, k_dnj_scan rescans them all
		enqueue_plan<ET, GEN>(st, D, bs, b, n, first);
		kt.mark(CCG_K_FIND);
		const int sm = g_grid.scan_mode(n, ET);
		// the wave-per-unit scans fold the entries at their last arrivals
		// (FoldTail) instead of a k_dnj_fold pass
		const bool tfold = prefold && g_grid.scan_fold && sm >= 1;
		const int prune = dnj_prune(n, ET, GEN);
		if(prune == 2 && g_grid.plan_help) k_dnj_sphase<ET, false><<<g_grid.sphase_blocks(), TB, 0, st>>>(D, bs, b, n, seg);
		else if(prune == 2) k_dnj_sphase<ET><<<g_grid.sphase_blocks(), TB, 0, st>>>(D, bs, b, n, seg);
		if(b.lbm && !GEN && sm >= 20 && sm <= 23 && g_grid.lb_groups && g_grid.scan_cmp && !tfold && prune == 0 &&
		   dnj_umax(n, seg) < UHIST) {
			// bounded row groups (float / u16 / u8 rows): 4 rows per wave share each column-sum load
			const unsigned gcc = gc < (unsigned) g_grid.cmp_blocks ? gc : (unsigned) g_grid.cmp_blocks;
			k_dnj_scan_gc<ET, 4, 8, false, true><<<gcc, TB, 0, st>>>(D, bs, b, n, seg);
		} else if(b.lbm && !GEN && sm >= 4 && g_grid.scan_cmp && !tfold && prune != 1 && dnj_umax(n, seg) < UHIST) {
			// the compacted wave scan under the block lower bounds (every element type)
			const unsigned gcc = gc < (unsigned) g_grid.cmp_blocks ? gc : (unsigned) g_grid.cmp_blocks;
			if(prune == 2) k_dnj_scan_v<ET, DenseRows, NoTail, 0, 2, true, true><<<gcc, TB, 0, st>>>(D, bs, b, n, DenseRows(), seg);
			else k_dnj_scan_v<ET, DenseRows, NoTail, 0, 0, true, true><<<gcc, TB, 0, st>>>(D, bs, b, n, DenseRows(), seg);
		} else if(sm >= 20 && sm <= 23 && !GEN && g_grid.scan_cmp && !tfold && prune != 1 && dnj_umax(n, seg) < UHIST) {
			// row groups over the dense (group, unit) enumeration; with pruning, the survivors only
			const unsigned gcc = gc < (unsigned) g_grid.cmp_blocks ? gc : (unsigned) g_grid.cmp_blocks;
			if(prune == 2) {
				if(sm == 20) k_dnj_scan_gc<ET, 4, 8, true><<<gcc, TB, 0, st>>>(D, bs, b, n, seg);
				else if(sm == 21) k_dnj_scan_gc<ET, 8, 4, true><<<gcc, TB, 0, st>>>(D, bs, b, n, seg);
				else if(sm == 22) k_dnj_scan_gc<ET, 4, 4, true><<<gcc, TB, 0, st>>>(D, bs, b, n, seg);
				else k_dnj_scan_gc<ET, 2, 8, true><<<gcc, TB, 0, st>>>(D, bs, b, n, seg);
			} else {
				if(sm == 20) k_dnj_scan_gc<ET, 4, 8, false><<<gcc, TB, 0, st>>>(D, bs, b, n, seg);
				else if(sm == 21) k_dnj_scan_gc<ET, 8, 4, false><<<gcc, TB, 0, st>>>(D, bs, b, n, seg);
				else if(sm == 22) k_dnj_scan_gc<ET, 4, 4, false><<<gcc, TB, 0, st>>>(D, bs, b, n, seg);
				else k_dnj_scan_gc<ET, 2, 8, false><<<gcc, TB, 0, st>>>(D, bs, b, n, seg);
			}
		} else if(sm >= 20 && sm <= 23 && !GEN) {
			if(prune) {
				if(sm == 20) k_dnj_scan_g<ET, 4, 8, true, true><<<gc, TB, 0, st>>>(D, bs, b, n, seg);
				else if(sm == 21) k_dnj_scan_g<ET, 8, 4, true, true><<<gc, TB, 0, st>>>(D, bs, b, n, seg);
				else if(sm == 22) k_dnj_scan_g<ET, 4, 4, true, true><<<gc, TB, 0, st>>>(D, bs, b, n, seg);
				else k_dnj_scan_g<ET, 2, 8, true, true><<<gc, TB, 0, st>>>(D, bs, b, n, seg);
			} else if(tfold) {
				if(sm == 20) k_dnj_scan_g<ET, 4, 8, true><<<gc, TB, 0, st>>>(D, bs, b, n, seg);
				else if(sm == 21) k_dnj_scan_g<ET, 8, 4, true><<<gc, TB, 0, st>>>(D, bs, b, n, seg);
				else if(sm == 22) k_dnj_scan_g<ET, 4, 4, true><<<gc, TB, 0, st>>>(D, bs, b, n, seg);
				else k_dnj_scan_g<ET, 2, 8, true><<<gc, TB, 0, st>>>(D, bs, b, n, seg);
			} else {
				if(sm == 20) k_dnj_scan_g<ET, 4, 8><<<gc, TB, 0, st>>>(D, bs, b, n, seg);
				else if(sm == 21) k_dnj_scan_g<ET, 8, 4><<<gc, TB, 0, st>>>(D, bs, b, n, seg);
				else if(sm == 22) k_dnj_scan_g<ET, 4, 4><<<gc, TB, 0, st>>>(D, bs, b, n, seg);
				else k_dnj_scan_g<ET, 2, 8><<<gc, TB, 0, st>>>(D, bs, b, n, seg);
			}
		} else if(sm >= 4 && !GEN) {
			// the compacted form (the plan's unit histogram; umax within its bins)
			const bool cmp = g_grid.scan_cmp && prune != 1 && !tfold && dnj_umax(n, seg) < UHIST;
			const unsigned gcc = gc < (unsigned) g_grid.cmp_blocks ? gc : (unsigned) g_grid.cmp_blocks;
			if(cmp && prune == 2) {
				switch(sm) {
#define SV_(M) case 4 + M: k_dnj_scan_v<ET, DenseRows, NoTail, M, 2, true><<<gcc, TB, 0, st>>>(D, bs, b, n, DenseRows(), seg); break;
					SV_(1) SV_(5) SV_(7) SV_(13)
#undef SV_
					default: k_dnj_scan_v<ET, DenseRows, NoTail, 0, 2, true><<<gcc, TB, 0, st>>>(D, bs, b, n, DenseRows(), seg);
				}
			} else if(cmp) {
				switch(sm) {
#define SV_(M) case 4 + M: k_dnj_scan_v<ET, DenseRows, NoTail, M, 0, true><<<gcc, TB, 0, st>>>(D, bs, b, n, DenseRows(), seg); break;
					SV_(1) SV_(5) SV_(7) SV_(13)
#undef SV_
					default: k_dnj_scan_v<ET, DenseRows, NoTail, 0, 0, true><<<gcc, TB, 0, st>>>(D, bs, b, n, DenseRows(), seg);
				}
			} else if(prune == 2) {
				switch(sm) {
#define SV_(M) case 4 + M: k_dnj_scan_v<ET, DenseRows, NoTail, M, 2><<<gc, TB, 0, st>>>(D, bs, b, n, DenseRows(), seg); break;
					SV_(1) SV_(5)
#undef SV_
					default: k_dnj_scan_v<ET, DenseRows, NoTail, 0, 2><<<gc, TB, 0, st>>>(D, bs, b, n, DenseRows(), seg);
				}
			} else if(prune) {
				switch(sm) {
#define SV_(M) case 4 + M: k_dnj_scan_v<ET, DenseRows, FoldTail, M, true><<<gc, TB, 0, st>>>(D, bs, b, n, DenseRows(), seg); break;
					SV_(1) SV_(5)
#undef SV_
					default: k_dnj_scan_v<ET, DenseRows, FoldTail, 0, true><<<gc, TB, 0, st>>>(D, bs, b, n, DenseRows(), seg);
				}
			} else if(tfold) {
				switch(sm) {
#define SV_(M) case 4 + M: k_dnj_scan_v<ET, DenseRows, FoldTail, M><<<gc, TB, 0, st>>>(D, bs, b, n, DenseRows(), seg); break;
					SV_(1) SV_(5)
#undef SV_
					default: k_dnj_scan_v<ET, DenseRows, FoldTail><<<gc, TB, 0, st>>>(D, bs, b, n, DenseRows(), seg);
				}
			} else {
				switch(sm) {
#define SV_(M) case 4 + M: k_dnj_scan_v<ET, DenseRows, NoTail, M><<<gc, TB, 0, st>>>(D, bs, b, n, DenseRows(), seg); break;
					SV_(1) SV_(2) SV_(3) SV_(4) SV_(5) SV_(6) SV_(7) SV_(13) SV_(15)
#undef SV_
					default: k_dnj_scan_v<ET, DenseRows><<<gc, TB, 0, st>>>(D, bs, b, n, DenseRows(), seg);
				}
			}
		} else if(sm >= 1) {
			if(tfold) k_dnj_scan_w<ET, GEN, DenseRows, FoldTail><<<gc, TB, 0, st>>>(D, bs, b, n, DenseRows(), seg);
			else k_dnj_scan_w<ET, GEN><<<gc, TB, 0, st>>>(D, bs, b, n, DenseRows(), seg);
		} else k_dnj_scan<ET, GEN><<<gc, TB, 0, st>>>(D, bs, b, n, DenseRows(), seg);
		if(prefold && !tfold) k_dnj_fold<><<<FOLD_BLOCKS, TB, 0, st>>>(b, n, seg, prune == 2);
		kt.mark(CCG_K_REST);
		if(prefold && g_grid.join_pf) k_dnj_join_pf<ET, GEN><<<gn, TB, 0, st>>>(D, bs, b, n, general, g_grid.join_pf == 2);
		else k_dnj_join<ET, GEN><<<gn, TB, 0, st>>>(D, bs, b, n, general, prefold, seg);
		if(GEN) k_update_general<ET><<<1, 1024, 0, st>>>(D, bs, b, n);
		kt.mark(CCG_K_UPDATE);
		if(xs) {
			k_exact_sum<><<<1, XS_NT, 0, st>>>(b, n, (int) gn);
			kt.mark(CCG_K_XSUM);
		}
		if(g_grid.bands(n - 1) && g_grid.scan_vblk && dnj_prune(n - 1, ET, GEN))
			k_dnj_requeue<ET, true, true><<<gn, TB, 0, st>>>(D, bs, b, n, general, exact);
		else if(g_grid.bands(n - 1)) k_dnj_requeue<ET, true><<<gn, TB, 0, st>>>(D, bs, b, n, general, exact);
		else k_dnj_requeue<ET, false><<<gn, TB, 0, st>>>(D, bs, b, n, general, exact);
		kt.mark(CCG_K_REQUEUE);
		return (GEN ? 5 : 4) + (prefold && !tfold) + (prune == 2) + xs;
	}
	if(method == CCG_TREE_HNJ) {
		k_hnj_argmin<><<<gn, TB, 0, st>>>(b, n);
		kt.mark(CCG_K_ARGMIN);
		k_nj_join<ET><<<gn, TB, 0, st>>>(D, bs, b, n, (int) gn, general, DBL_MAX);
		if(GEN) k_update_general<ET><<<1, 1024, 0, st>>>(D, bs, b, n);
		kt.mark(CCG_K_UPDATE);
		if(xs) {
			k_exact_sum<><<<1, XS_NT, 0, st>>>(b, n, (int) gn);
			kt.mark(CCG_K_XSUM);
		}
		k_hnj_update<ET><<<gn, TB, 0, st>>>(D, bs, b, n, general, exact);   // updateHNJ's Q/P pass + HNJ_popArrange
		kt.mark(CCG_K_POP);
		return (GEN ? 4 : 3) + xs;
	}
	const unsigned g = (unsigned) nj_blocks(n);
	k_nj_argmin<ET, GEN><<<g, TB, 0, st>>>(D, bs, b, n);
	kt.mark(CCG_K_ARGMIN);
	k_nj_join<ET><<<gn, TB, 0, st>>>(D, bs, b, n, (int) g, general, 1.0);
	if(GEN) k_update_general<ET><<<1, 1024, 0, st>>>(D, bs, b, n);
	kt.mark(CCG_K_UPDATE);
	if(xs) {
		k_exact_sum<><<<1, XS_NT, 0, st>>>(b, n, (int) gn);
		kt.mark(CCG_K_XSUM);
	}
	k_nj_pop<ET><<<gn, TB, 0, st>>>(D, b, n, general, exact);
	kt.mark(CCG_K_POP);
	return (GEN ? 4 : 3) + xs;
}

static bool g_progress = false;

template <int ET>
static int tree_run_t(ccg_ctx *ctx, const ccg_tree_args *a, void *Dd, ccg_join *joins, int *njoins,
                      int *final_n, double *final_d, int64_t *stats, const ccg_dnj_state *sin,
                      ccg_dnj_state *sout) {
	typedef typename Elem<ET>::T T;
	T *D = (T *) Dd;
	const int n0 = a->n;
	const double bs = a->byteScale;
	hipStream_t st = ctx->stream;
	TreeWork w;
	g_grid = DnjGrid();
	g_grid.load();
	g_progress = getenv("CCG_PROGRESS") != nullptr;
	// the compacted scans deal their units over a grid meant to be resident at
	// once (cmp_blocks per 256 CUs): a CU-masked context sizes it to its CUs
	const bool cmp_env = getenv("CCG_SCAN_CMPB") != nullptr;
	auto cmp_share = [&](int blocks) {
		return ctx->cus > 0 && ctx->cus < ctx->ncu ? (blocks * ctx->cus / ctx->ncu > 64 ? blocks * ctx->cus / ctx->ncu : 64)
		                                           : blocks;
	};
	if(!cmp_env) g_grid.cmp_blocks = cmp_share(g_grid.cmp_blocks);
	int rc = tree_alloc_ctx(ctx, &w, n0);
	if(rc) return rc;
	TreeBufs b = w.b;
	TreeCtl init;
	memset(&init, 0, sizeof(init));
	init.neg = (a->flags & 2) != 0;
	init.exact = a->exact != 0;
	init.method = a->method;
	init.hj = init.hi = -1;
	if(sin) {   // a resumed DNJ state: its candidate takes k_dnj_prep's place
		init.cand = sin->cand;
		init.cand_q = sin->Q[sin->cand];
		init.cand_p = sin->P[sin->cand];
	}
	CCG_CHECK(hipMemcpyAsync(b.ctl, &init, sizeof(init), hipMemcpyHostToDevice, st));
	long long launches = 0;
	static thread_local KTimer kt;   // one per host thread (the CLI runs one rank per thread)
	CCG_CHECK(hipEventRecord(ctx->ev0, st));
	kt.init(st, a->profile != 0);
	k_init_rows<ET><<<cdiv(n0, TB / 64), TB, 0, st>>>(D, n0, bs, b.sD, b.N, b.ctl);
	k_init_cols<ET><<<cdiv(n0, TB), TB, 0, st>>>(D, n0, bs, b.sD, b.N, b.ctl);
	launches += 2;
	bool resumed_counts = false;   // a resumed state whose N differs from the matrix size somewhere
	if(sin) {
		// initSummaD above only detected missing entries (ctl->has_missing);
		// the state's own vectors replace its sums
		CCG_CHECK(hipMemcpyAsync(b.sD, sin->sD, (size_t) n0 * 8, hipMemcpyHostToDevice, st));
		CCG_CHECK(hipMemcpyAsync(b.Q, sin->Q, (size_t) n0 * 8, hipMemcpyHostToDevice, st));
		CCG_CHECK(hipMemcpyAsync(b.N, sin->N, (size_t) n0 * 4, hipMemcpyHostToDevice, st));
		CCG_CHECK(hipMemcpyAsync(b.P, sin->P, (size_t) n0 * 4, hipMemcpyHostToDevice, st));
		for(int k = 0; k < n0 && !resumed_counts; ++k) resumed_counts = sin->N[k] != n0;
	} else if(a->method == CCG_TREE_DNJ) {
		k_init_hnj<ET><<<cdiv(n0, TB / 64), TB, 0, st>>>(DenseRows(), D, n0, bs, b.sD, b.N, b.Q, b.P);
		k_dnj_prep<><<<1, TB, 0, st>>>(b, n0);
		launches += 2;
	} else if(a->method == CCG_TREE_HNJ) {
		k_init_hnj<ET><<<cdiv(n0, TB / 64), TB, 0, st>>>(DenseRows(), D, n0, bs, b.sD, b.N, b.Q, b.P);   // hclust.c:56
		launches += 1;
	}
	kt.mark(CCG_K_INIT);
	CCG_CHECK(hipGetLastError());
	TreeCtl h;
	CCG_CHECK(hipMemcpyAsync(&h, b.ctl, sizeof(h), hipMemcpyDeviceToHost, st));
	CCG_CHECK(hipStreamSynchronize(st));
	// GEN = false assumes N[k] == n for every row (no missing entries ever)
	const bool general = h.has_missing != 0 || resumed_counts;
	// the block lower bounds (DnjGrid::lb): one allocation beside the run's
	void *lbmem = NULL;
	if(a->method == CCG_TREE_DNJ && !general && g_grid.lb && n0 > g_grid.lb_min_n) {
		const long long LS = (n0 + LBW - 1) / LBW;
		const size_t lbb = ((size_t) n0 * LS * 4 + 255) & ~(size_t) 255;
		const size_t msb = ((size_t) (LS + 1) * 8 + 255) & ~(size_t) 255;
		const size_t ubb = ((size_t) n0 * 8 + 255) & ~(size_t) 255, skb = (size_t) (LB_SCAN + LB_HELP) * LB_SLOT * 8;
		if(ccg_ctx_workspace(ctx, 1, lbb + msb + ubb + skb, &lbmem) == CCG_OK) {
			b.lbm = (unsigned *) lbmem;
			b.msd = (double *) ((char *) lbmem + lbb);
			b.ubq = (double *) ((char *) lbmem + lbb + msb);
			b.lbs = LS;
			b.lbskip = (long long *) ((char *) lbmem + lbb + msb + ubb);
			CCG_CHECK(hipMemsetAsync(b.lbskip, 0, skb, st));
			k_lb_init<ET><<<cdiv(n0, TB / 64), TB, 0, st>>>(D, n0, bs, b);
			launches += 1;
			CCG_CHECK(hipGetLastError());
			// S-bound pruning no longer pays beside the bounded scan (headline tree, profiled: 4.61 s
			// without, 4.78 s with the plan's helpers and the compaction); CCG_SCAN_PRUNE still forces it
			if(!getenv("CCG_SCAN_PRUNE")) g_grid.scan_prune = 0;
			// the bounded units are short: twice the waves (headline tree 4.84 -> 4.74 s, profiled)
			if(!cmp_env) g_grid.cmp_blocks = cmp_share(2048);
		} else {
			(void) hipGetLastError();   // no room: the run goes without (the same joins)
			lbmem = NULL;
		}
	}
#ifdef CCG_TRACE
	const char *tn = getenv("CCG_TRACE_N");
	int trace_hi = tn ? atoi(tn) : n0 / 2;
	CCG_CHECK(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_trace_hi), &trace_hi, sizeof(int), 0, hipMemcpyHostToDevice, st));
	static unsigned long long zero_tr[256 * 4 * 16];
	CCG_CHECK(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_trace), zero_tr, sizeof(zero_tr), 0, hipMemcpyHostToDevice, st));
#endif
	int n = n0;
	int since_check = 0;
	long long win_rows = h.rows, win_cells = h.cells;   // ctl->rows / cells at the last check
	bool stopped = false;
	const int stop_n = a->max_joins > 0 && a->max_joins < n0 - 2 ? n0 - a->max_joins : 2;
	while(n > stop_n) {
		launches += general ? enqueue_iteration<ET, true>(st, D, bs, b, n, n == n0, a->method, a->exact, kt)
		                    : enqueue_iteration<ET, false>(st, D, bs, b, n, n == n0, a->method, a->exact, kt);
		CCG_CHECK(hipGetLastError());
		--n;
		if(++since_check == 1024) {
			since_check = 0;
			CCG_CHECK(hipMemcpyAsync(&h, b.ctl, sizeof(h), hipMemcpyDeviceToHost, st));
			CCG_CHECK(hipStreamSynchronize(st));
			// the next window's scan form below 16384 taxa (DnjGrid::small_wave)
			g_grid.small_wave = g_grid.adapt_rows && h.rows - win_rows > 1024LL * g_grid.adapt_rows;
			g_grid.prune_on = !g_grid.prune_cells || h.cells - win_cells > 1024LL * g_grid.prune_cells;
			win_rows = h.rows;
			win_cells = h.cells;
			if(g_progress && (n0 - n) % (16 * 1024) == 0)   // long trees (CCG_PROGRESS=1): a line per 16384 joins
				fprintf(stderr, "ccg_tree: %d joins, n = %d, rows %lld cells %lld (reference rule %lld / %lld)\n", n0 - n,
				        n, h.rows, h.cells, h.ref_rows, h.ref_cells);
			if(h.done) {
				stopped = true;
				break;
			}
		}
	}
	(void) stopped;
	CCG_CHECK(hipEventRecord(ctx->ev1, st));
	kt.finish();
	CCG_CHECK(hipMemcpyAsync(&h, b.ctl, sizeof(h), hipMemcpyDeviceToHost, st));
	CCG_CHECK(hipStreamSynchronize(st));
	if(b.lbskip) {   // the bounded-out cells, from the per-wave slots
		std::vector<long long> sl((size_t) (LB_SCAN + LB_HELP) * LB_SLOT);
		// on the context's stream (a null-stream copy would wait for every blocking stream of the device)
		CCG_CHECK(hipMemcpyAsync(sl.data(), b.lbskip, sl.size() * 8, hipMemcpyDeviceToHost, st));
		CCG_CHECK(hipStreamSynchronize(st));
		for(size_t x = 0; x < (size_t) LB_SCAN + LB_HELP; ++x) {
			h.cells_lbskip += sl[x * LB_SLOT];
			h.cells_help -= sl[x * LB_SLOT + 1];
		}
	}
	float ms = 0;
	CCG_CHECK(hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
	if(getenv("CCG_XS_WHY"))   // diagnostics: why exact row sums fell back to the serial chain
		fprintf(stderr, "xs_why: value %d nc %d nt %d stuck %d ex0 %d cap %d walk %d (chain sums %d of %d)\n",
		        h.xs_why[0], h.xs_why[1], h.xs_why[2], h.xs_why[3], h.xs_why[4], h.xs_why[5], h.xs_why[6],
		        h.chain_sums, h.serial_sums);
#ifdef CCG_TRACE
	{
		static unsigned long long tr[256 * NKT * 16];
		CCG_CHECK(hipMemcpyFromSymbol(tr, HIP_SYMBOL(g_trace), sizeof(tr), 0, hipMemcpyDeviceToHost));
		const int nk = a->method == CCG_TREE_DNJ ? NKT : 0;   // NJ kernels are not stamped
		// per kernel: min block entry (15, stored inverted), block-0 phases (0..8), max block exit (14);
		// times in us relative to the kernel's first block entry, averaged over joins
		double acc[NKT][16] = {{0}}, gap[NKT] = {0}, itv = 0;
		int cnt = 0;
		bool present[NKT] = {false};   // kernels launched in this pipeline (k_dnj_select is not)
		for(int s = 0; s < 256; ++s)
			for(int k = 0; k < nk; ++k) present[k] = present[k] || tr[(s * NKT + k) * 16 + 15];
		for(int s = 0; s < 256; ++s) {
			const unsigned long long *e = tr + s * NKT * 16;
			bool ok = true;
			for(int k = 0; k < nk; ++k) ok = ok && (!present[k] || (e[k * 16 + 15] && e[k * 16 + 14]));
			if(!ok) continue;
			++cnt;
			int k0 = 0, prev = -1;
			while(k0 < nk && !present[k0]) ++k0;
			for(int k = k0; k < nk; ++k) {
				if(!present[k]) continue;
				unsigned long long t0 = ~e[k * 16 + 15];
				for(int p = 0; p < 15; ++p)
					if(e[k * 16 + p]) acc[k][p] += ((double) e[k * 16 + p] - (double) t0) / 100.0;
				if(prev >= 0) gap[k] += ((double) t0 - (double) e[prev * 16 + 14]) / 100.0;
				prev = k;
			}
			if(s + 1 < 256 && tr[((s + 1) * NKT + k0) * 16 + 15]) {
				gap[k0] += ((double) ~tr[((s + 1) * NKT + k0) * 16 + 15] - (double) e[(nk - 1) * 16 + 14]) / 100.0;
				itv += ((double) ~tr[((s + 1) * NKT + k0) * 16 + 15] - (double) ~e[k0 * 16 + 15]) / 100.0;
			}
		}
		const char *kn[NKT] = {"select", "plan/find", "scan", "join", "requeue"};
		fprintf(stderr, "trace: %d joins at n <= %d; iteration %.2f us; serial replays %d, serial sums %d\n", cnt,
		        trace_hi, cnt ? itv / (cnt - 1) : 0, h.serial_replays, h.serial_sums);
		{
			// sampled scan blocks (every 32nd): start and end relative to the kernel's first entry
			static unsigned long long sp[256 * 64 * 3];
			CCG_CHECK(hipMemcpyFromSymbol(sp, HIP_SYMBOL(g_samp), sizeof(sp), 0, hipMemcpyDeviceToHost));
			double st_max = 0, en_max = 0, dur = 0, st_med = 0, stg = 0;
			int sc = 0, jc = 0;
			for(int s = 0; s < 256; ++s) {
				const unsigned long long t0 = ~tr[(s * NKT + 2) * 16 + 15];
				if(!tr[(s * NKT + 2) * 16 + 15]) continue;
				double smax = 0, emax = 0;
				int any = 0;
				for(int q = 0; q < 64; ++q) {
					const unsigned long long *e = sp + (s * 64 + q) * 3;
					if(!e[0] || !e[2] || e[0] < t0) continue;
					const double a = (e[0] - t0) / 100.0, z = (e[2] - t0) / 100.0;
					smax = a > smax ? a : smax;
					emax = z > emax ? z : emax;
					dur += z - a;
					if(e[1] >= e[0]) stg += (e[1] - e[0]) / 100.0;
					st_med += a;
					++sc;
					any = 1;
				}
				if(any) {
					st_max += smax;
					en_max += emax;
					++jc;
				}
			}
			{
				static unsigned long long ua[256 * 64 * 8];
				CCG_CHECK(hipMemcpyFromSymbol(ua, HIP_SYMBOL(g_uamp), sizeof(ua), 0, hipMemcpyDeviceToHost));
				double ud[4] = {0}, ug[4] = {0}, us0 = 0;
				int uc[4] = {0}, gc[4] = {0}, s0c = 0;
				for(int s = 0; s < 256; ++s) {
					const unsigned long long t0 = ~tr[(s * NKT + 2) * 16 + 15];
					if(!tr[(s * NKT + 2) * 16 + 15]) continue;
					for(int q = 0; q < 64; ++q) {
						const unsigned long long *e = ua + (s * 64 + q) * 8;
						const unsigned long long *sp0 = sp + (s * 64 + q) * 3;
						if(e[0] && e[0] >= t0 && sp0[0] && e[0] >= sp0[0]) {
							us0 += (e[0] - sp0[0]) / 100.0;   // block entry -> first unit
							++s0c;
						}
						for(int k = 0; k < 4; ++k) {
							if(e[2 * k] && e[2 * k + 1] >= e[2 * k] && e[2 * k] >= t0) {
								ud[k] += (e[2 * k + 1] - e[2 * k]) / 100.0;
								++uc[k];
							}
							if(k && e[2 * k] && e[2 * k - 1] && e[2 * k] >= e[2 * k - 1] && e[2 * k] >= t0) {
								ug[k] += (e[2 * k] - e[2 * k - 1]) / 100.0;
								++gc[k];
							}
						}
					}
				}
				fprintf(stderr, "  scan units (wave 0 of sampled blocks): entry->first unit %.2f us;", s0c ? us0 / s0c : 0.0);
				for(int k = 0; k < 4; ++k)
					fprintf(stderr, " unit%d n=%d dur %.2f gap %.2f;", k, uc[k], uc[k] ? ud[k] / uc[k] : 0.0, gc[k] ? ug[k] / gc[k] : 0.0);
				fprintf(stderr, "\n");
				memset(ua, 0, sizeof(ua));
				CCG_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_uamp), ua, sizeof(ua), 0, hipMemcpyHostToDevice));
			}
			if(jc) fprintf(stderr, "  scan samples: %d joins, %.1f working blocks sampled/join; last start %.2f us, last end %.2f us, mean start %.2f, mean duration %.2f us (setup %.2f)\n",
			                jc, (double) sc / jc, st_max / jc, en_max / jc, st_med / sc, dur / sc, stg / sc);
		}
		for(int k = 0; k < nk && cnt; ++k) {
			if(!present[k]) continue;
			fprintf(stderr, "  %-14s gap-before %6.2f  span %6.2f  block0:", kn[k], gap[k] / cnt, acc[k][14] / cnt);
			for(int p = 0; p < 14; ++p) fprintf(stderr, " %6.2f", acc[k][p] / cnt);
			fprintf(stderr, "\n");
		}
	}
#endif
	if(h.done && h.final_n < 0) {   // k_dnj_plan's look-back timed out (never expected)
		ccg_set_last_msg("k_dnj_plan / k_dnj_join: a block's bounded wait on another block timed out");
		return CCG_EHIP;
	}
	*njoins = h.njoins;
	*final_n = h.done ? h.final_n : n;
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
	if(sout) {   // the loop state after the last join, as the next minQpair reads it
		// (a finished tree, n == 2, has no next join: n = 0 as for a stopped one)
		const bool over = h.done || n <= 2;
		sout->n = over ? 0 : n;
		sout->cand = 0;
		if(!over) {
			if(n != n0) {
				// the next join's plan prologue folds the last requeue's partials
				// into Q/P of rows j and i (and moves row n's sD/N to i) and
				// picks the candidate (minPos, dnj.c:1026-1032); nothing after
				// it in this run reads what else it lists
				if(general) enqueue_plan<ET, true>(st, D, bs, b, n, 0);
				else enqueue_plan<ET, false>(st, D, bs, b, n, 0);
				CCG_CHECK(hipGetLastError());
			}
			TreeCtl h2;   // h keeps the run's counters (the extra plan adds its S cells)
			CCG_CHECK(hipMemcpyAsync(&h2, b.ctl, sizeof(h2), hipMemcpyDeviceToHost, st));
			CCG_CHECK(hipMemcpyAsync(sout->sD, b.sD, (size_t) n * 8, hipMemcpyDeviceToHost, st));
			CCG_CHECK(hipMemcpyAsync(sout->Q, b.Q, (size_t) n * 8, hipMemcpyDeviceToHost, st));
			CCG_CHECK(hipMemcpyAsync(sout->N, b.N, (size_t) n * 4, hipMemcpyDeviceToHost, st));
			CCG_CHECK(hipMemcpyAsync(sout->P, b.P, (size_t) n * 4, hipMemcpyDeviceToHost, st));
			CCG_CHECK(hipStreamSynchronize(st));
			sout->cand = h2.cand;
		}
	}
	if(stats) {
		stats[0] = h.rows;
		stats[1] = h.cells - h.cells_pruned - h.cells_lbskip;   // cells the scans loaded (listed, less the pruned / bounded-out ones)
		stats[2] = launches;
		stats[3] = (int64_t) (ms * 1000.0);
		if(a->profile) {
			for(int c = 0; c < CCG_NKSTAT; ++c) {
				stats[4 + 2 * c] = kt.cnt[c];
				stats[5 + 2 * c] = kt.ns[c];
			}
			stats[4 + 2 * CCG_NKSTAT] = h.cells_top;
			stats[5 + 2 * CCG_NKSTAT] = h.cells_rest - h.cells_pruned - h.cells_lbskip;
			stats[6 + 2 * CCG_NKSTAT] = h.serial_sums;
			stats[7 + 2 * CCG_NKSTAT] = h.chain_sums;
			stats[8 + 2 * CCG_NKSTAT] = h.cells_help;
			stats[9 + 2 * CCG_NKSTAT] = 0;
			stats[10 + 2 * CCG_NKSTAT] = h.ref_rows;
			stats[11 + 2 * CCG_NKSTAT] = h.ref_cells;
		}
	}
	CCG_CHECK(hipStreamSynchronize(st));
	return CCG_OK;   // the workspaces stay with the context (ccg_ctx_workspace)
}

// ------------------------------------------------------------------ self-test of the exact row sum
template <int NT>
__global__ __launch_bounds__(NT) void k_selftest_row_sum(TreeBufs b, int n, double *out, int *par,
                                                        unsigned long long *stamps) {
	double s;
	if(stamps && threadIdx.x == 0) stamps[15] = __builtin_amdgcn_s_memrealtime();
	// NT = TB: 4 waves, rows reloaded past n = 6144 (the second-pass path)
	const bool ok = exact_sum_w<NT, XS_RB>(b.contrib, n, &s, stamps);
	if(!ok) s = serial_sum_t<NT>(b.contrib, n);
	if(threadIdx.x == 0) {
		out[0] = s;
		par[0] = ok;
	}
}

int ccg_selftest_row_sum_impl(ccg_ctx *ctx, const double *c, int n, double *out, int *parallel) {
	hipStream_t st = ctx->stream;
	char *m;
	CCG_CHECK(hipMalloc((void **) &m, (size_t) (n + 1) * 8 + 64 + 64 * 8));
	TreeBufs b;
	memset(&b, 0, sizeof(b));
	b.contrib = (double *) m;
	double *dout = (double *) (m + (size_t) (n + 1) * 8);
	int *dpar = (int *) (dout + 1);
	unsigned long long *dst = (unsigned long long *) (m + (size_t) (n + 1) * 8 + 64);
	CCG_CHECK(hipMemcpyAsync(b.contrib, c, (size_t) n * 8, hipMemcpyHostToDevice, st));
	const bool small = getenv("CCG_SELFTEST_TB256") != nullptr;   // 4 waves: exercises the reload path
	auto launch = [&](unsigned long long *stp) {
		if(small) k_selftest_row_sum<TB><<<1, TB, 0, st>>>(b, n, dout, dpar, stp);
		else k_selftest_row_sum<XS_NT><<<1, XS_NT, 0, st>>>(b, n, dout, dpar, stp);
	};
	launch(nullptr);
	CCG_CHECK(hipGetLastError());
	if(const char *e = getenv("CCG_SELFTEST_REPS")) {   // development timing
		const int reps = atoi(e);
		CCG_CHECK(hipEventRecord(ctx->ev0, st));
		for(int r = 0; r < reps; ++r) launch(nullptr);
		CCG_CHECK(hipEventRecord(ctx->ev1, st));
		CCG_CHECK(hipEventSynchronize(ctx->ev1));
		float ms = 0;
		CCG_CHECK(hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
		fprintf(stderr, "selftest_row_sum n=%d: %.2f us per launch\n", n, 1000.0 * ms / (reps > 0 ? reps : 1));
		unsigned long long hs[64] = {0};
		CCG_CHECK(hipMemsetAsync(dst, 0, 64 * 8, st));
		launch(dst);
		CCG_CHECK(hipMemcpyAsync(hs, dst, 64 * 8, hipMemcpyDeviceToHost, st));
		CCG_CHECK(hipStreamSynchronize(st));
		for(int w = 0; w < 4; ++w) {
			fprintf(stderr, "  wave %d phases (us from entry):", w);
			for(int i = 0; i < 15; ++i)
				fprintf(stderr, " %d:%.2f", i, hs[16 * w + i] ? (double) (hs[16 * w + i] - hs[15]) / 100.0 : -1.0);
			fprintf(stderr, "\n");
		}
	}
	CCG_CHECK(hipMemcpyAsync(out, dout, 8, hipMemcpyDeviceToHost, st));
	CCG_CHECK(hipMemcpyAsync(parallel, dpar, 4, hipMemcpyDeviceToHost, st));
	CCG_CHECK(hipStreamSynchronize(st));
	CCG_CHECK(hipFree(m));
	return CCG_OK;
}

int ccg_tree_impl(ccg_ctx *ctx, const ccg_tree_args *a, void *Dd, ccg_join *joins, int *njoins, int *final_n,
                  double *final_d, int64_t *stats, const ccg_dnj_state *sin, ccg_dnj_state *sout) {
	switch(a->etype) {
		case 8: return tree_run_t<8>(ctx, a, Dd, joins, njoins, final_n, final_d, stats, sin, sout);
		case 4: return tree_run_t<4>(ctx, a, Dd, joins, njoins, final_n, final_d, stats, sin, sout);
		case 2: return tree_run_t<2>(ctx, a, Dd, joins, njoins, final_n, final_d, stats, sin, sout);
		case 1: return tree_run_t<1>(ctx, a, Dd, joins, njoins, final_n, final_d, stats, sin, sout);
		default: return CCG_EINVAL;
	}
}
