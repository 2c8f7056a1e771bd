// tree_shard_dnj.hip -- DNJ (dnj.c:985 loop, the reference's default tree
// method) over an LT matrix whose rows are split across ranks, one process
// per GPU.  Same layout as the sharded NJ (ccg_shard.h):
// bands of CCG_SHARD_BAND rows dealt round-robin, a rank's rows back to back;
// sD, N, Q, P and the join list are replicated and every rank updates them
// with the same arithmetic.
//
// Per join at matrix size n: five kernels, two collectives.  (Round 5: row
// n-1 travels in the lines' allreduce instead of a broadcast of its own --
// one collective latency fewer per join)
//   1. k_dnj_plan (ccg_dnj_search.h, Shard row policy): minPos, m0 and the
//      top rows S depend on the replicated Q only, so every rank computes the
//      same ones.  Each rank bounds minQpair's serial running min with the
//      S rows it owns alone: max(q(k, P[k]), Q_k) over its own k in S is an
//      upper bound of that running min for ANY subset of S (a rescanned k
//      gives m <= fresh_k <= q(k, P[k]), a skipped one m <= Q_k).  It lists
//      its own S rows and its own rows below S with Q under the bound; any
//      other row is provably skipped by dnj.c:88;
//   2. k_dnj_scan rescans the listed units; its tail (RecTail) folds each
//      row's units into a record of the rank's own rows, indexed by the
//      row's position among them -- one bit byte per owned band, f64 fresh
//      q, i32 j;
//      -> allgather of the ranks' record slots (each rank sends only its own
//      rows' records: half the ring bytes of the round-2 allreduce-as-gather
//      over dense row-indexed arrays);
//   3. k_shd_pick: every block replays minQpair's accept/reject decisions
//      over the listed rows in descending order (replay_wave); rows that the
//      serial scan would skip have bound >= running min, so the replay
//      rejects them and (i, j) is the single-GPU engine's on every rank.
//      Then each rank's pieces of lines i and j, and row n-1 from its owner
//      (the pop moves it to slot i, dnj.c:817 / matrix.c:518);
//      -> allreduce-sum of lines i and j and row n-1 (a gather again);
//   4. k_shd_join: the accepted (Q, P) updates, limbLength, updateD
//      (nj.c:836) on every rank for every k, own cells stored, the new line j
//      kept whole (its exact row sum: xs_join_row);
//   5. k_shd_requeue: updateDNJ's Q/P pass (dnj.c:618-709) and
//      DNJ_popArrange (dnj.c:817) over the replicated lines, own cells
//      stored; the records are zeroed for the next join.
// Hence the joins are bit-identical to ccg_tree's DNJ for every world size.
#define CCG_DNJ_NO_TRACE
#include <stdio.h>
#include <string.h>
#include <stdlib.h>
#include <vector>
#include "ccg_dnj_search.h"
#include "ccg_shard.h"

// ------------------------------------------------------------------ records
// Per join, one rank's slot: [a bit byte per owned band (row r of band g is
// bit r % 8 of byte g / world)][f64 fresh q][i32 fresh j] of its owned rows
// by position (g / world) * 8 + r % 8, sized for the rank that owns the most
// bands at size n; the allgather lays the slots side by side, rank order.
static_assert(SB == 8, "one bit byte per shard band");
struct RecSlot {
	size_t f_off, j_off, bytes;
};
static __host__ __device__ inline RecSlot rec_slot(int n, int world) {
	const int nb = (n + SB - 1) / SB, omb = (nb + world - 1) / world;
	RecSlot s;
	s.f_off = ((size_t) omb + 15) & ~(size_t) 15;
	s.j_off = s.f_off + (size_t) omb * SB * 8;
	s.bytes = (s.j_off + (size_t) omb * SB * 4 + 15) & ~(size_t) 15;
	return s;
}
// a row's owner and position among the owner's rows
static __host__ __device__ inline int rec_owner(int r, int world) { return (r / SB) % world; }
static __host__ __device__ inline int rec_pos(int r, int world) { return (r / SB) / world * SB + r % SB; }

// initHNJ's gather (once): [bitmap of rows (u64 words)][f64 q][i32 j], dense
static __host__ __device__ inline size_t rec_bits_bytes(int n) { return (size_t) ((n + 63) / 64) * 8; }
static __host__ __device__ inline size_t rec_bytes(int n) { return rec_bits_bytes(n) + (size_t) n * 12; }

struct RecView {
	unsigned *bits;
	double *f;
	int *j;
};
static __host__ __device__ inline RecView rec_view(void *R, int n) {
	RecView v;
	v.bits = (unsigned *) R;
	v.f = (double *) ((char *) R + rec_bits_bytes(n));
	v.j = (int *) ((char *) R + rec_bits_bytes(n) + (size_t) n * 8);
	return v;
}

// own rescans -> records, as k_dnj_scan's tail: every scan block first copies
// a slice of row n-1 behind the records (the owner's cells, zeros on the
// other ranks); the thread that stores a row's last unit partial folds the
// row's units and fills its record and bit.  The hand-off needs no L2
// write-back or invalidate (an agent-scope release / acquire costs both on
// the per-XCD L2s): the partials are stored write-through (sc1) and drained
// (s_waitcnt vmcnt(0)) before the relaxed per-row arrival count, and the
// last arriver reads them with sc1 loads (cdna_hip_programming.md G16, R1
// with sc1 loads).  The count goes back to 0 for the next join.
template <int ET>
struct RecTail {
	const typename Elem<ET>::T *D;
	Shard sh;
	void *R;                          // this rank's record slot
	unsigned *cnt;   // n0 zeros
	__device__ void begin(const TreeBufs &, int) const {}
	__device__ void unit(const TreeBufs &b, int n, int u, int ua, int ub, int r, double q, int j) const {
		if(ub - ua > 1) {
			__hip_atomic_store(b.cq + u, q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
			__hip_atomic_store(b.cj + u, j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
			asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
			const unsigned seen = __hip_atomic_fetch_add(cnt + r, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
			if((int) seen != ub - ua - 1) return;
			__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
			for(int x = ua; x < ub; ++x) {
				if(x == u) continue;
				const double oq = __hip_atomic_load(b.cq + x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
				const int oi = __hip_atomic_load(b.cj + x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
				if(qarg_better(oq, oi, q, j)) {
					q = oq;
					j = oi;
				}
			}
			__hip_atomic_store(cnt + r, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		}
		const RecSlot s = rec_slot(n, sh.world);
		const int o = rec_pos(r, sh.world), ob = o / SB;
		((double *) ((char *) R + s.f_off))[o] = q;
		((int *) ((char *) R + s.j_off))[o] = j;
		atomicOr((unsigned *) R + (ob >> 2), 1u << ((ob & 3) * 8 + (r & 7)));
	}
};

// minQpair's replay (dnj.c:76-125) fused with the gather of lines i and j.
// Every block builds the entries in scan order from the gathered records --
// the rows with their bit set, descending (with the one-phase plan S rows are
// listed like any other row) -- and replays them itself, so that no block
// waits for another: the inputs (records, Q, m0, pos) are the same in every
// block and so are the decisions.  Q/P are not written here (another block
// may still be reading Q as a bound): block 0 leaves the entries and their
// accept flags for k_shd_join.  Entries live in LDS up to PICK_CAP; beyond,
// every block writes the same values into the shared HBM arrays and keeps
// its accept scratch in its own slice of pacc.
#define PICK_T 1024
#define PICK_CAP 2048
#define PICK_MAXB 256
template <int ET>
__global__ __launch_bounds__(PICK_T) void k_shd_pick(const typename Elem<ET>::T *__restrict__ D, TreeBufs b, int n,
                                                     Shard sh, void *R, typename Elem<ET>::T *__restrict__ X,
                                                     unsigned char *pacc, unsigned char *acc_out, int pstride,
                                                     unsigned long long *dbg) {
#define PTS(ph)                                                                                  \
	do {                                                                                         \
		if(dbg && blockIdx.x == 0 && threadIdx.x == 0) {                                         \
			unsigned long long t_;                                                               \
			asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");     \
			dbg[(n & 1023) * 8 + (ph)] = t_;                                                     \
		}                                                                                        \
	} while(0)
	PTS(0);
	__shared__ int s_scan[PICK_T / 64];
	__shared__ int e_row[PICK_CAP], e_j[PICK_CAP];
	__shared__ double e_b[PICK_CAP], e_f[PICK_CAP];
	__shared__ unsigned char e_acc[PICK_CAP];
	__shared__ int s_i, s_j;
	TreeCtl *ctl = b.ctl;
	const int tid = threadIdx.x;
	// the gathered slots (R: world x rs.bytes)
	const int W = sh.world;
	const RecSlot rs = rec_slot(n, W);
	const int nbands = (n + SB - 1) / SB;
	auto rbits = [&](int w) -> unsigned {   // rows 32w .. 32w + 31: bands 4w .. 4w + 3
		unsigned x = 0;
#pragma unroll
		for(int t = 0; t < 4; ++t) {
			const int g = 4 * w + t;
			if(g < nbands) x |= (unsigned) ((const unsigned char *) R)[(size_t) (g % W) * rs.bytes + g / W] << (8 * t);
		}
		return x;
	};
	auto rf = [&](int r) {
		return ((const double *) ((const char *) R + (size_t) rec_owner(r, W) * rs.bytes + rs.f_off))[rec_pos(r, W)];
	};
	auto rj = [&](int r) {
		return ((const int *) ((const char *) R + (size_t) rec_owner(r, W) * rs.bytes + rs.j_off))[rec_pos(r, W)];
	};
	// rows [1, n) with their bit set; thread t owns a contiguous run of
	// bitmap words, the highest runs first (the first word and the replay's
	// inputs are loaded before the stop test: one round trip fewer)
	const int nw = n > 1 ? ((n - 1) >> 5) + 1 : 0;
	const int per = (nw + PICK_T - 1) / PICK_T;
	auto word = [&](int w, unsigned x) -> unsigned {
		if(w == 0) x &= ~1u;                                          // row 0 never qualifies
		if(w == nw - 1 && (n & 31)) x &= (1u << (n & 31)) - 1u;       // rows >= n
		return x;
	};
	const int wfirst = nw - 1 - tid * per;
	const unsigned x0 = wfirst >= 0 ? rbits(wfirst) : 0u;
	const int pos_i = ctl->pos_i, pos_j = ctl->pos_j;
	const double m0 = ctl->m0;
	if(ctl->done) return;
	PTS(1);
	int cnt = 0;
	for(int q = 0; q < per; ++q) {
		const int w = nw - 1 - (tid * per + q);
		if(w >= 0) cnt += __popc(word(w, q == 0 ? x0 : rbits(w)));
	}
	int total;
	int pos = block_excl_scan(cnt, s_scan, &total);
	PTS(2);
	const bool lds = total <= PICK_CAP;
	int *x_row = lds ? e_row : b.erow, *x_j = lds ? e_j : b.ej;
	double *x_b = lds ? e_b : b.eb, *x_f = lds ? e_f : b.ef;
	for(int q = 0; q < per; ++q) {
		const int w = nw - 1 - (tid * per + q);
		if(w < 0) break;
		unsigned x = word(w, q == 0 ? x0 : rbits(w));
		while(x) {
			const int bit = 31 - __clz((int) x);
			x &= ~(1u << bit);
			x_row[pos++] = w * 32 + bit;
		}
	}
	__syncthreads();
	// then every entry's loads at once (the top rows of S fill whole bitmap
	// words: loading per bit would chain 32 round trips in one thread)
	for(int e = tid; e < total; e += PICK_T) {
		const int r = x_row[e];
		x_b[e] = b.Q[r];
		x_f[e] = rf(r);
		x_j[e] = rj(r);
	}
	__syncthreads();
	PTS(3);
	const bool writer = blockIdx.x == 0;
	// Without a "bad" entry (fresh below its stale bound) minQpair's running
	// min is a prefix min (replay_wave's comment), so the whole block decides
	// at once from per-thread summaries of contiguous entry runs (minimum
	// fresh value, any bad), as k_dnj_join_pf does from k_dnj_fold's 64-entry
	// chunk summaries: a block prefix-min gives each run its running min on
	// entry, the accept decisions follow in the run, and the pair is the
	// first entry reaching the overall minimum.  With a bad entry wave 0
	// replays serially (replay_wave).
	const int per2 = (total + PICK_T - 1) / PICK_T, a0 = tid * per2, a1 = a0 + per2 < total ? a0 + per2 : total;
	double tmin = DBL_MAX;
	int tbad = 0;
	for(int e = a0; e < a1; ++e) {
		const double f = x_f[e];
		tbad |= !(f >= x_b[e]);
		tmin = f < tmin ? f : tmin;
	}
	if(!__syncthreads_or(tbad)) {
		__shared__ double s_wm[PICK_T / 64];
		__shared__ int s_wf[PICK_T / 64];
		__shared__ long long s_na[PICK_T / 64], s_ca[PICK_T / 64];
		const int lane = tid & 63, wid = tid >> 6;
		const double inc = wave_incl_min(tmin);
		if(lane == 63) s_wm[wid] = inc;
		__syncthreads();
		double carry = m0, cm = m0;
#pragma unroll
		for(int w = 0; w < PICK_T / 64; ++w) {
			if(w < wid) carry = s_wm[w] < carry ? s_wm[w] : carry;
			cm = s_wm[w] < cm ? s_wm[w] : cm;
		}
		const double ex = dpp_d<DPP_WAVE_SHR1, 0xF>(DBL_MAX, inc);
		double run = ex < carry ? ex : carry;   // the running min before this thread's run
		long long nacc = 0, cacc = 0;
		int first = 0x7fffffff;
		for(int e = a0; e < a1; ++e) {
			const double f = x_f[e];
			const bool acc = x_b[e] < run;
			if(acc) {
				++nacc;
				cacc += x_row[e];
			}
			if(writer) acc_out[e] = acc;   // applied by k_shd_join
			if(f == cm && e < first) first = e;
			run = f < run ? f : run;
		}
		first = wave_min_int(cm < m0 ? first : 0x7fffffff);
		nacc = wave_sum_int(nacc);
		cacc = wave_sum_int(cacc);
		if(lane == 0) {
			s_wf[wid] = first;
			s_na[wid] = nacc;
			s_ca[wid] = cacc;
		}
		__syncthreads();
		if(tid == 0) {
			int fe = 0x7fffffff;
			long long na = 0, ca = 0;
			for(int w = 0; w < PICK_T / 64; ++w) {
				fe = s_wf[w] < fe ? s_wf[w] : fe;
				na += s_na[w];
				ca += s_ca[w];
			}
			const int pi = fe < 0x7fffffff ? x_row[fe] : pos_i, pj = fe < 0x7fffffff ? x_j[fe] : pos_j;
			s_i = pi;
			s_j = pj;
			if(writer) {
				if(na) {   // minQpair's own rescans (ctl->ref_rows / ref_cells)
					atomicAdd((unsigned long long *) &ctl->ref_rows, (unsigned long long) na);
					atomicAdd((unsigned long long *) &ctl->ref_cells, (unsigned long long) ca);
				}
				if(pi == 0 && pj == 0) {
					ctl->done = 1;
					ctl->final_n = n;
				} else {
					ctl->i = pi;
					ctl->j = pj;
				}
				ctl->rtotal = total;
			}
		}
	} else if(tid < 64) {
		int pi = pos_i, pj = pos_j;
		bool had_bad;
		if(lds) replay_wave(total, m0, e_row, e_j, e_b, e_f, e_acc, writer, b, pi, pj, &had_bad, n, acc_out);
		else replay_wave(total, m0, b.erow, b.ej, b.eb, b.ef, pacc + (size_t) blockIdx.x * pstride, writer, b, pi, pj,
		                 &had_bad, n, acc_out);
		if(tid == 0) {
			s_i = pi;
			s_j = pj;
			if(writer) {
				if(pi == 0 && pj == 0) {
					ctl->done = 1;
					ctl->final_n = n;
				} else {
					ctl->i = pi;
					ctl->j = pj;
				}
				ctl->rtotal = total;
				ctl->serial_replays += had_bad;
			}
		}
	}
	__syncthreads();
	PTS(4);
	const int i = s_i, j = s_j;
	if(i == 0 && j == 0) return;
	// block 0: the entries behind the accept flags, for k_shd_join
	if(writer && lds) {
		for(int e = tid; e < total; e += PICK_T) {
			b.erow[e] = e_row[e];
			b.ef[e] = e_f[e];
			b.ej[e] = e_j[e];
		}
	}
	// the pieces of lines i and j this rank's rows hold: X[k] = D(i, k),
	// X[n + k] = D(j, k), and row n-1, X[2n + k] = D(n-1, k) (raw elements;
	// zeros where another rank owns the cell)
	const bool own_m = sh.owns(n - 1);
	const typename Elem<ET>::T *rowm = D + (own_m ? sh.off(n - 1) : 0);
	for(int k = blockIdx.x * PICK_T + tid; k < n; k += gridDim.x * PICK_T) {
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
		X[2 * n + k] = own_m && k < n - 1 ? rowm[k] : (typename Elem<ET>::T) 0;
	}
	PTS(5);
	if(dbg && blockIdx.x == 0 && threadIdx.x == 0) dbg[(n & 1023) * 8 + 6] = total;
#undef PTS
}

// limbLength (nj.c:42/:81), the join record and updateD (nj.c:836) over the
// gathered lines: every rank computes the whole new line j (kept in Xj and,
// at k = n-1, patched into the gathered row Xm) and stores its own cells
template <int ET>
__global__ __launch_bounds__(TB) void k_shd_join(typename Elem<ET>::T *__restrict__ D, double bs, TreeBufs b, int n,
                                                 Shard sh, const typename Elem<ET>::T *__restrict__ X,
                                                 typename Elem<ET>::T *__restrict__ Xm,
                                                 typename Elem<ET>::T *__restrict__ Xj,
                                                 const unsigned char *__restrict__ acc) {
	__shared__ int s_stop, s_nj, s_neg, s_exact, s_i, s_j;
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
		s_i = ctl->i;
		s_j = ctl->j;
	}
	__syncthreads();
	if(s_stop) return;
	// minQpair's accepted (Q, P) updates (dnj.c:94-99), flagged by k_shd_pick
	for(int e = k, tot = ctl->rtotal; e < tot; e += gridDim.x * TB) {
		if(acc[e]) {
			b.Q[b.erow[e]] = b.ef[e];
			b.P[b.erow[e]] = b.ej[e];
		}
	}
	const int i = s_i, j = s_j;
	const double Dij = Elem<ET>::get(X[j], bs);
	if(blockIdx.x == 0 && tid == 0) {
		double Li, Lj;
		limb_length(&Li, &Lj, b.sD[i], b.sD[j], b.N[i], b.N[j], Dij, s_neg);
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
	typename Elem<ET>::T v = 0;
	if(k < n && k != i && k != j) {
		d = (Dik + Dkj - Dij) / 2;
		d = d < 0 ? 0 : d;
		v = Elem<ET>::put(d, 0.25, bs);
		if(k > j) {
			if(sh.owns(k)) D[sh.off(k) + j] = v;
		} else if(sh.owns(j)) {
			D[sh.off(j) + k] = v;
		}
		Xj[k] = v;
		if(k == n - 1) Xm[j] = v;   // row n-1 moves to slot i in the pop
		b.sD[k] = sDk - (Dik + Dkj - d);
		b.N[k] = Nk - 1;
		cnt = 1;
	}
	if(b.lbm) {   // (uniform) block bounds of the owned rows: row j rewritten, column j lowered where written
		const unsigned x = lb_bits(Elem<ET>::get(v, bs));
		if(sh.owns(j)) {
			const unsigned mn = wave_min_u32(k < j ? x : 0xFFFFFFFFu);
			if((tid & 63) == 0 && k < j) lb_line(b, j)[k >> 6] = mn;
		}
		if(k > j && k < n && k != i && sh.owns(k))
			__hip_atomic_fetch_min(lb_line(b, k) + (j >> 6), x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
	}
	update_partials(b, n, s_exact, k, d, cnt, blockIdx.x);
	// exact mode: this block's row of the serial row sum (every rank holds
	// the whole new line j, so every rank computes the same rows)
	if(s_exact) xs_join_row(b, n, blockIdx.x, d, xs_tag(n));
}

// Row sum of j, updateDNJ's Q/P part (dnj.c:618-709) and DNJ_popArrange
// (dnj.c:817-975) over the replicated lines Xj (new line j) and Xm (row n-1,
// moved to i), in the partial format k_dnj_select folds (tree.hip's
// k_dnj_requeue, without missing entries); then the records are zeroed in
// the layout of size n-1.
template <int ET, bool BANDS>
__global__ __launch_bounds__(TB) void k_shd_requeue(typename Elem<ET>::T *__restrict__ D, double bs, TreeBufs b,
                                                    int n, Shard sh, const typename Elem<ET>::T *__restrict__ Xm,
                                                    const typename Elem<ET>::T *__restrict__ Xj, void *R) {
	__shared__ double sq[5][TB / 64], sfq[TB / 64];
	__shared__ int si[5][TB / 64], sfp[TB / 64], sbp[TB / 64];
	__shared__ double s_sd;
	__shared__ int s_nj, s_i, s_j, s_stop, s_serial, s_chain;
	TreeCtl *ctl = b.ctl;
	const int nn = n - 1;
	const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
	const int k = blockIdx.x * TB + tid;
	int Nk = 0, pkk0 = 0;
	double sDk = 0, qk0 = 0;
	typename Elem<ET>::T vm = 0, vj = 0;
	if(k < n) {
		Nk = b.N[k];
		sDk = b.sD[k];
		qk0 = b.Q[k];
		pkk0 = b.P[k];
		vj = Xj[k];
	}
	if(k < nn) vm = Xm[k];
	// block bounds: the owned row's partner cell and the partner's row sum,
	// for the row's threshold in the next scan (ubq, as k_dnj_requeue)
	typename Elem<ET>::T vp = 0;
	double sdp0 = 0.0;
	const bool PV = b.ubq != nullptr;   // (uniform)
	if(PV && k >= 1 && k < n && sh.owns(k)) {
		const int p0 = pkk0 >= 0 && pkk0 < k ? pkk0 : 0;
		vp = D[sh.off(k) + p0];
		sdp0 = b.sD[p0];
	}
	const int Nm0 = b.N[nn];
	const double sDm0 = b.sD[nn];
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
	const int i = s_i, j = s_j, Nj = s_nj;
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
			const double d = Elem<ET>::get(vj, bs);
			if(0 <= d) {
				rq = qcrit(Nj, Nk, d, sdj, sDk);
				rj = k;
			}
		}
		if(k > j && k != i) {
			double qk = qk0;
			int pkk = pkk0;
			bool upd = false;
			const double d = Elem<ET>::get(vj, bs);
			if(0 <= d) {
				const double q = qcrit(Nj, Nk, d, sdj, sDk);
				if(q <= qk) {
					qk = q;
					pkk = j;
					upd = true;
					pq = q;
					pk = k;
				}
			}
			if(move && k > i && k < nn) {
				if(sh.owns(k)) D[sh.off(k) + i] = vm;
				const double dm = Elem<ET>::get(vm, bs);
				if(0 <= dm) {
					const double q = qcrit(Nm, Nk, dm, sDm, sDk);
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
			if(sh.owns(i)) D[sh.off(i) + k] = vm;
			const double dm = Elem<ET>::get(vm, bs);
			if(0 <= dm) {
				r2q = qcrit(Nm, Nk, dm, sDm, sDk);
				r2j = k;
			}
		}
	}
	// this rank's record slot for the next join: its bit bytes (q and j are
	// read only where a bit is set)
	if((size_t) k * 4 < rec_slot(n, sh.world).f_off) ((unsigned *) R)[k] = 0;
	if(b.lbm) {   // (uniform) block bounds of the owned rows: row i = the moved row, column i; sD maxima
		const unsigned x = lb_bits(Elem<ET>::get(vm, bs));
		if(move) {
			if(sh.owns(i)) {
				const unsigned mn = wave_min_u32(k < i ? x : 0xFFFFFFFFu);
				if(lane == 0 && k < i) lb_line(b, i)[k >> 6] = mn;
			}
			if(k > i && k < nn && sh.owns(k))
				__hip_atomic_fetch_min(lb_line(b, k) + (i >> 6), x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		}
		const double sf = k < nn ? (move && k == i ? sDm : sDk) : -DBL_MAX;   // sD of column k at the next join
		const double mx = wave_max_d(sf);
		if(lane == 0 && k < nn) b.msd[k >> 6] = mx;
	}
	// ubq: the q at the owned row's partner cell in the next join's state (the
	// next scan's threshold for the row); +inf for the other ranks' rows
	double qpc = INFINITY;
	if(PV && k >= 1 && k < nn && k != i && k != j && sh.owns(k)) {
		const bool later = k > j;   // rows above j may have a new partner (j or the moved i)
		const int pf = later ? fp : pkk0;
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
		if(0 <= d) qpc = qcrit(nn, nn, d, sDk, sp);
		b.ubq[k] = qpc;
	}
	// the row's bound for the next join: each block's min-Q row becomes a
	// candidate of the next S (rows j and i take theirs from k_dnj_select's
	// fold); only when the next S has a band part (with ubq also the q at its
	// partner cell, k_dnj_plan's partner-cell bound: +inf for another rank's row)
	double bq = DBL_MAX, bqc = INFINITY;
	int bk = 0, bp = 0;
	__shared__ double sbq[TB / 64];
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
			if(PV) b.bmqp[blockIdx.x] = xq;
		} else {
			b.qpart[4 * blockIdx.x + tid] = q;
			b.ipart[4 * blockIdx.x + tid] = ix;
		}
		if(tid == 1) {
			b.cfq[blockIdx.x] = cq;
			b.cfp[blockIdx.x] = cp;
		}
	}
}

// the block lower bounds of the owned rows (k_lb_init's sharded form): wave
// w takes the rank's w-th own row, and (replicated) the sD maxima of block w
// and the threshold +inf of row w
template <int ET>
__global__ __launch_bounds__(TB) void k_shd_lb_init(const typename Elem<ET>::T *__restrict__ D, int n, double bs,
                                                    TreeBufs b, Shard sh) {
	constexpr int BB = 8;
	const int lane = threadIdx.x & 63;
	const int w = blockIdx.x * (TB / 64) + (threadIdx.x >> 6);
	if(w >= n) return;   // (wave-uniform)
	if(w < (n + LBW - 1) / LBW) {
		const int c = w * LBW + lane;
		const double mx = wave_max_d(c < n ? b.sD[c] : -DBL_MAX);
		if(lane == 0) b.msd[w] = mx;
	}
	if(lane == 0) b.ubq[w] = INFINITY;
	const int r = ((w >> 3) * sh.world + sh.rank) * 8 + (w & 7);
	if(r >= n) return;
	const typename Elem<ET>::T *row = D + sh.off(r);
	unsigned *line = lb_line(b, r);
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
			if(lane == 0 && u0 + m < nbk) line[u0 + m] = mn;
		}
	}
}

// initHNJ's (Q, P) of the owned rows into the zeroed records' q/j arrays
template <int ET>
static int shd_init_hnj(const typename Elem<ET>::T *D, int n0, double bs, const Shard &sh, CollRun &cr,
                        hipStream_t st, TreeBufs &b, void *R) {
	const RecView v = rec_view(R, n0);
	CCG_CHECK(hipMemsetAsync(R, 0, rec_bytes(n0), st));
	k_init_hnj<ET><<<cdiv(n0, TB / 64), TB, 0, st>>>(sh, D, n0, bs, b.sD, b.N, v.f, v.j);
	CCG_CHECK(hipGetLastError());
	cr.kt->mark(CCG_K_INIT);
	int rc = cr.allreduce(v.f, (size_t) n0 * 12);
	if(rc) return rc;
	CCG_CHECK(hipMemcpyAsync(b.Q, v.f, (size_t) n0 * 8, hipMemcpyDeviceToDevice, st));
	CCG_CHECK(hipMemcpyAsync(b.P, v.j, (size_t) n0 * 4, hipMemcpyDeviceToDevice, st));
	CCG_CHECK(hipMemsetAsync(R, 0, rec_bytes(n0), st));
	k_dnj_prep<><<<1, TB, 0, st>>>(b, n0);
	CCG_CHECK(hipGetLastError());
	cr.kt->mark(CCG_K_INIT);
	return CCG_OK;
}

// ------------------------------------------------------------------ host driver
// the sharded DNJ's buffers beyond ccg_tree_alloc's (one allocation): the
// records, lines i / j, row n-1, the new line j, the replay's scratch and the
// init gathers
struct ShdLayout {
	size_t o_R, o_X, o_Xm, o_Sl, o_G, o_Xj, o_pf, o_pa, o_pc, o_rp, o_is, sz = 0;
	ShdLayout(int n0, int world, int es) {
		auto take = [&](size_t bytes) {
			size_t off = sz;
			sz += (bytes + 255) & ~(size_t) 255;
			return off;
		};
		const RecSlot rs0 = rec_slot(n0, world);
		o_R = take(rec_bytes(n0));
		o_X = take((size_t) 3 * n0 * es);
		o_Xm = take((size_t) n0 * es + 8);
		o_Sl = take(rs0.bytes);
		o_G = take((size_t) world * rs0.bytes);
		o_Xj = take((size_t) n0 * es + 8);
		o_pf = take((size_t) n0);
		o_pa = take((size_t) PICK_MAXB * n0);
		o_pc = take((size_t) n0 * 4);
		o_rp = take(sh_rp_bytes(n0));
		o_is = take(sh_init_scratch_bytes(n0, world));
	}
};

size_t ccg_shard_dnj_bytes(int n, int world, int es) { return ccg_tree_bytes(n) + ShdLayout(n, world, es).sz; }

template <int ET>
static int tree_shard_dnj_run_t(ccg_ctx *ctx, const ccg_tree_args *a, const ccg_coll *coll, void *Dd,
                                ccg_join *joins, int *njoins, int *final_n, double *final_d, int64_t *stats) {
	typedef typename Elem<ET>::T T;
	T *D = (T *) Dd;
	const int n0 = a->n;
	const double bs = a->byteScale;
	hipStream_t st = ctx->stream;
	const Shard sh = {coll->rank, coll->world};
	int rc;
	TreeWork w;
	if((rc = ccg_tree_alloc(&w, n0, st))) return rc;
	TreeBufs b = w.b;
	const ShdLayout L(n0, coll->world, ET);
	const RecSlot rs0 = rec_slot(n0, coll->world);
	const size_t o_R = L.o_R, o_X = L.o_X, o_Xm = L.o_Xm, o_Sl = L.o_Sl, o_G = L.o_G, o_Xj = L.o_Xj, o_pf = L.o_pf;
	const size_t o_pa = L.o_pa, o_pc = L.o_pc, o_rp = L.o_rp, o_is = L.o_is, sz = L.sz;
	char *m = NULL;
	unsigned char *h = NULL;
	if(hipMalloc((void **) &m, sz) != hipSuccess) {
		hipFree(w.mem);
		return CCG_ENOMEM;
	}
	size_t hcap = sh_init_host_bytes(n0, coll->world);
	if((size_t) 3 * n0 * ET > hcap) hcap = (size_t) 3 * n0 * ET;
	if(rec_bytes(n0) > hcap) hcap = rec_bytes(n0);
	if((size_t) coll->world * rs0.bytes > hcap) hcap = (size_t) coll->world * rs0.bytes;
	if(coll->host_staged && hipHostMalloc((void **) &h, hcap) != hipSuccess) {
		hipFree(m);
		hipFree(w.mem);
		return CCG_ENOMEM;
	}
	static thread_local KTimer kt;   // one per host thread (the CLI runs one rank per thread)
	CollRun cr = {coll, st, h, &kt};
	DnjGrid grid;
	grid.load();
	void *R = m + o_R, *Sl = m + o_Sl, *G = m + o_G;   // initHNJ's gather; this rank's record slot; the gathered slots
	T *X = (T *) (m + o_X), *Xm = (T *) (m + o_Xm), *Xj = (T *) (m + o_Xj);
	ShInitStat istat = {0, 0};
	unsigned char *pflag = (unsigned char *) (m + o_pf), *pacc = (unsigned char *) (m + o_pa);
	unsigned *pcnt = (unsigned *) (m + o_pc);
	unsigned long long *dbg = NULL;
	void *lbmem = NULL;
	// diagnostic: k_shd_pick's phase stamps (s_memrealtime), averaged to stderr
	if(getenv("CCG_PICK_TS")) {
		if(hipMalloc((void **) &dbg, 1024 * 8 * 8) != hipSuccess) dbg = NULL;
		else if(hipMemsetAsync(dbg, 0, 1024 * 8 * 8, st) != hipSuccess) {
			hipFree(dbg);
			dbg = NULL;
		}
	}
	TreeCtl init, hc;
	long long launches = 0;
	int n = n0;
	float ms = 0;
	memset(&init, 0, sizeof(init));
	init.neg = (a->flags & 2) != 0;
	init.exact = a->exact != 0;
	init.method = a->method;
#define SD_TRY(x)                          \
	do {                                   \
		if((rc = (x)) != CCG_OK) goto out; \
	} while(0)
#define SD_HIP(x)                                                    \
	do {                                                             \
		hipError_t e_ = (x);                                         \
		if(e_ != hipSuccess) {                                       \
			ccg_set_last_error(e_, #x, __FILE__, __LINE__);         \
			rc = e_ == hipErrorOutOfMemory ? CCG_ENOMEM : CCG_EHIP; \
			goto out;                                                \
		}                                                            \
	} while(0)
	SD_HIP(hipMemsetAsync(m, 0, sz, st));
	SD_HIP(hipMemcpyAsync(b.ctl, &init, sizeof(init), hipMemcpyHostToDevice, st));
	SD_HIP(hipEventRecord(ctx->ev0, st));
	kt.init(st, a->profile != 0);
	{
		int missing = 0;
		SD_TRY(sh_init_summad<ET>(D, n0, bs, sh, cr, st, m + o_rp, m + o_is, b, &launches, &missing, &istat));
		if(missing) {
			rc = CCG_EUNSUP;   // the missing-entry quirks of updateD run on one GPU only
			goto out;
		}
	}
	SD_TRY(shd_init_hnj<ET>(D, n0, bs, sh, cr, st, b, R));
	launches += 2;
	// the block lower bounds (DnjGrid::lb, as the single engine): a line per
	// owned row, the sD maxima and the thresholds replicated
	if(grid.lb && n0 > grid.lb_min_n) {
		const long long LS = (n0 + LBW - 1) / LBW, own = (long long) cdiv(cdiv(n0, 8), sh.world) * 8;
		const size_t lbb = ((size_t) own * LS * 4 + 255) & ~(size_t) 255;
		const size_t msb = ((size_t) (LS + 1) * 8 + 255) & ~(size_t) 255;
		const size_t ubb = ((size_t) n0 * 8 + 255) & ~(size_t) 255, skb = (size_t) (LB_SCAN + LB_HELP) * LB_SLOT * 8;
		if(hipMalloc(&lbmem, lbb + msb + ubb + skb) == hipSuccess) {
			b.lbm = (unsigned *) lbmem;
			b.msd = (double *) ((char *) lbmem + lbb);
			b.ubq = (double *) ((char *) lbmem + lbb + msb);
			b.lbs = LS;
			b.lbw = sh.world;
			b.lbskip = (long long *) ((char *) lbmem + lbb + msb + ubb);
			SD_HIP(hipMemsetAsync(b.lbskip, 0, skb, st));
			k_shd_lb_init<ET><<<cdiv(n0, TB / 64), TB, 0, st>>>(D, n0, bs, b, sh);
			SD_HIP(hipGetLastError());
			launches += 1;
		} else {
			(void) hipGetLastError();   // no room: the run goes without (the same joins)
			lbmem = NULL;
		}
	}
	{
		int since_check = 0;
		const int stop_n = a->max_joins > 0 && a->max_joins < n0 - 2 ? n0 - a->max_joins : 2;
		while(n > stop_n) {
			const unsigned gn = cdiv(n, TB), gp = cdiv(n, PICK_T) < PICK_MAXB ? cdiv(n, PICK_T) : PICK_MAXB;
			T *Xmr = X + 2 * (size_t) n;   // row n-1, gathered with lines i and j
			const unsigned gc = grid.scan(n);
			const int seg = grid.seg(n);
			// one-phase search (k_dnj_plan): each rank lists the S rows and the
			// rows below S it owns, under the bound of its own S rows' partner
			// cells (a subset of S: looser, still exact after the replay)
			// the listing over a grid of blocks with the decoupled look-back past 15361 taxa, as on one GPU:
			// every rank walks all n rows for its owned ones (round 6: one block took 140 us per join at
			// 200k, tools/shard_cost.py)
			const unsigned gpl = grid.plan_blocks(n);
			if(grid.bands(n)) k_dnj_plan<ET, false, Shard, true><<<gpl, TBF, 0, st>>>(D, bs, b, n, n == n0, sh, seg, grid.top(n), grid.bands(n), grid.plan_flags());
			else k_dnj_plan<ET, false, Shard, false><<<gpl, TBF, 0, st>>>(D, bs, b, n, n == n0, sh, seg, grid.top(n), 0, grid.plan_flags());
			kt.mark(CCG_K_FIND);
			if(b.lbm && grid.scan_mode(n, ET) == 9) k_dnj_scan_v<ET, Shard, RecTail<ET>, 5, 0, false, true><<<gc, TB, 0, st>>>(D, bs, b, n, sh, seg, RecTail<ET>{D, sh, Sl, pcnt});
			else if(b.lbm && grid.scan_mode(n, ET) >= 4) k_dnj_scan_v<ET, Shard, RecTail<ET>, 0, 0, false, true><<<gc, TB, 0, st>>>(D, bs, b, n, sh, seg, RecTail<ET>{D, sh, Sl, pcnt});
			else if(grid.scan_mode(n, ET) == 9) k_dnj_scan_v<ET, Shard, RecTail<ET>, 5><<<gc, TB, 0, st>>>(D, bs, b, n, sh, seg, RecTail<ET>{D, sh, Sl, pcnt});
			else if(grid.scan_mode(n, ET) >= 4) k_dnj_scan_v<ET, Shard, RecTail<ET>><<<gc, TB, 0, st>>>(D, bs, b, n, sh, seg, RecTail<ET>{D, sh, Sl, pcnt});
			else if(grid.scan_mode(n, ET)) k_dnj_scan_w<ET, false, Shard, RecTail<ET>><<<gc, TB, 0, st>>>(D, bs, b, n, sh, seg, RecTail<ET>{D, sh, Sl, pcnt});
			else k_dnj_scan<ET, false><<<gc, TB, 0, st>>>(D, bs, b, n, sh, seg, RecTail<ET>{D, sh, Sl, pcnt});
			kt.mark(CCG_K_REST);
			SD_TRY(cr.allgather(Sl, G, rec_slot(n, sh.world).bytes));
			k_shd_pick<ET><<<gp, PICK_T, 0, st>>>(D, b, n, sh, G, X, pacc, pflag, n0, dbg);
			kt.mark(CCG_K_UPDATE);
			SD_TRY(cr.allreduce(X, (size_t) 3 * n * ET));
			k_shd_join<ET><<<gn, TB, 0, st>>>(D, bs, b, n, sh, X, Xmr, Xj, pflag);
			kt.mark(CCG_K_UPDATE);
			if(grid.bands(n - 1)) k_shd_requeue<ET, true><<<gn, TB, 0, st>>>(D, bs, b, n, sh, Xmr, Xj, Sl);
			else k_shd_requeue<ET, false><<<gn, TB, 0, st>>>(D, bs, b, n, sh, Xmr, Xj, Sl);
			kt.mark(CCG_K_REQUEUE);
			SD_HIP(hipGetLastError());
			launches += 5;
			--n;
			if(++since_check == 1024) {
				since_check = 0;
				SD_HIP(hipMemcpyAsync(&hc, b.ctl, sizeof(hc), hipMemcpyDeviceToHost, st));
				SD_HIP(hipStreamSynchronize(st));
				if(hc.done) break;
			}
		}
	}
	SD_HIP(hipEventRecord(ctx->ev1, st));
	kt.finish();
	if(dbg) {
		static thread_local unsigned long long hd[1024 * 8];
		if(hipMemcpyAsync(hd, dbg, sizeof(hd), hipMemcpyDeviceToHost, st) != hipSuccess ||
		   hipStreamSynchronize(st) != hipSuccess)
			memset(hd, 0, sizeof(hd));
		double acc[8] = {0};
		int cnt = 0;
		for(int s_ = 0; s_ < 1024; ++s_) {
			const unsigned long long *t_ = hd + s_ * 8;
			if(!t_[0] || !t_[5]) continue;
			for(int p_ = 1; p_ < 6; ++p_) acc[p_] += (double) (t_[p_] - t_[p_ - 1]) * 10.0;
			acc[6] += (double) t_[6];
			++cnt;
		}
		if(cnt)
			fprintf(stderr, "pick phases over %d joins (ns): entry->loads %.0f, count+scan %.0f, entries %.0f, replay %.0f, gather %.0f; total entries %.1f\n",
			        cnt, acc[1] / cnt, acc[2] / cnt, acc[3] / cnt, acc[4] / cnt, acc[5] / cnt, acc[6] / cnt);
		hipFree(dbg);
	}
	SD_HIP(hipMemcpyAsync(&hc, b.ctl, sizeof(hc), hipMemcpyDeviceToHost, st));
	SD_HIP(hipStreamSynchronize(st));
	SD_HIP(hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
	*njoins = hc.njoins;
	*final_n = hc.done ? hc.final_n : n;
	if(hc.njoins) {
		SD_HIP(hipMemcpyAsync(joins, b.joins, (size_t) hc.njoins * sizeof(ccg_join), hipMemcpyDeviceToHost, st));
	}
	*final_d = -1.0;
	if(*final_n == 2) {
		// D(1, 0): row 1 is in band 0, owned by rank 0
		SD_TRY(cr.bcast(sh.rank == 0 ? (const void *) (D + sh.off(1)) : NULL, Xm, ET, 0));
		T v;
		SD_HIP(hipMemcpyAsync(&v, Xm, sizeof(T), hipMemcpyDeviceToHost, st));
		SD_HIP(hipStreamSynchronize(st));
		*final_d = (ET == 8 || ET == 4) ? (double) v : v / bs;
	}
	if(b.lbskip) {   // the bounded-out cells, from the per-wave slots
		std::vector<long long> sl((size_t) LB_SCAN * LB_SLOT);
		SD_HIP(hipMemcpyAsync(sl.data(), b.lbskip, sl.size() * 8, hipMemcpyDeviceToHost, st));
		SD_HIP(hipStreamSynchronize(st));
		for(size_t x = 0; x < (size_t) LB_SCAN; ++x) hc.cells_lbskip += sl[x * LB_SLOT];
	}
	if(stats) {
		stats[0] = hc.rows;
		stats[1] = hc.cells - hc.cells_lbskip;   // cells the scans loaded
		stats[2] = launches;
		stats[3] = (int64_t) (ms * 1000.0);
		if(a->profile) {
			for(int c = 0; c < CCG_NKSTAT; ++c) {
				stats[4 + 2 * c] = kt.cnt[c];
				stats[5 + 2 * c] = kt.ns[c];
			}
			stats[4 + 2 * CCG_NKSTAT] = hc.cells_top;
			stats[5 + 2 * CCG_NKSTAT] = hc.cells_rest - hc.cells_lbskip;
			stats[6 + 2 * CCG_NKSTAT] = hc.serial_sums;
			stats[7 + 2 * CCG_NKSTAT] = hc.chain_sums;
			stats[8 + 2 * CCG_NKSTAT] = istat.coll_bytes;
			stats[9 + 2 * CCG_NKSTAT] = istat.hard;
			stats[10 + 2 * CCG_NKSTAT] = hc.ref_rows;
			stats[11 + 2 * CCG_NKSTAT] = hc.ref_cells;
		}
	}
out:
#undef SD_TRY
#undef SD_HIP
	if(rc != CCG_OK && kt.on) {   // the profiled run ended early: release its events
		for(int k = 0; k < 1025; ++k) hipEventDestroy(kt.ev[k]);
		kt.on = false;
	}
	hipStreamSynchronize(st);
	if(h) hipHostFree(h);
	if(lbmem) hipFree(lbmem);
	hipFree(m);
	hipFree(w.mem);
	return rc;
}

// called by ccg_tree_shard_dev (tree_shard.hip) for method CCG_TREE_DNJ;
// arguments already checked there, coll non-null
int ccg_tree_shard_dnj_impl(ccg_ctx *c, const ccg_tree_args *a, const ccg_coll *coll, void *Dloc, ccg_join *joins,
                            int *njoins, int *final_n, double *final_d, int64_t *stats) {
	switch(a->etype) {
		case 8: return tree_shard_dnj_run_t<8>(c, a, coll, Dloc, joins, njoins, final_n, final_d, stats);
		case 4: return tree_shard_dnj_run_t<4>(c, a, coll, Dloc, joins, njoins, final_n, final_d, stats);
		case 2: return tree_shard_dnj_run_t<2>(c, a, coll, Dloc, joins, njoins, final_n, final_d, stats);
		default: return tree_shard_dnj_run_t<1>(c, a, coll, Dloc, joins, njoins, final_n, final_d, stats);
	}
}
