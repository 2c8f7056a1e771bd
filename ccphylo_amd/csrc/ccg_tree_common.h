// ccg_tree_common.h -- device state and helpers shared by the single-GPU tree
// engine (tree.hip) and the row-sharded one (tree_shard.hip).  Both sum the
// new row of j and fold the argmin partials with exactly these functions, so
// their joins are bit-identical.
#pragma once
#include <string.h>
#include "ccg_internal.h"

#define TB 256           // threads per block
#define NJ_RB 8          // NJ argmin tile: rows
#define NJ_SEG (TB * 8)  // NJ argmin tile: columns

// one candidate row of minQpair: fresh (q, j) and its stale bound Q[row]
struct Entry {
	double f, bnd;
	int row, j;
};

struct TreeCtl {
	int done;            // the reference loop stopped (pos == 0)
	int final_n;
	int njoins;
	int i, j;            // current join
	double Li, Lj, Dij;
	int cand;            // minQpair's candidate row
	double cand_q;       // Q/P of the first candidate (k_dnj_prep)
	int cand_p;
	int pos_i, pos_j;    // minQpair's initial pos
	int nS, smin;        // |S| and the lowest row of its top part (1: no rows below S)
	int ntop;            // S = ntop top rows (descending), then band-minimum rows below them
	int T;               // rows found below S
	double m0;           // minQpair's initial min
	unsigned tick;       // k_dnj_select's last-block ticket
	int neg, exact, method, has_missing;
	int serial_sums, serial_replays;
	int chain_sums;      // exact row sums the parallel form declined (serial chain)
	int xnj;             // k_exact_sum: count and row sum of the new row j
	double xsum;
	long long rows, cells, cells_top, cells_rest;
	long long ref_rows, ref_cells;  // rows / cells minQpair's own rule rescans (dnj.c:78: Q[r] < running min)
	int hj, hi, hjb, hib;  // HNJ: rows j / i of the last join whose minima are still in partials (-1: none)
	int rtotal;          // sharded DNJ: replay entries whose accept flags k_shd_join applies
	int pS;              // S rows whose exact fresh minima prune the scan (0: no pruning this join)
	unsigned scnt;       // the scan's S entries folded so far (reset by the last)
	long long cells_pruned;  // listed cells the scan skipped under the S bound table
	long long cells_help;    // S cells rescanned inside k_dnj_plan by its helper blocks (scan_prune 2)
	long long cells_lbskip;  // listed cells the scan skipped under the block lower bounds
	int vtag;            // VBLK: the matrix size whose join the requeue's bmv minima serve
	int pblk;            // k_dnj_plan's block count (rows of uhist this join)
	int xs_why[8];       // exact row sums sent to the chain, by reason (XS_WHY_*)
};

struct XsBlk;
struct XsCross;
struct XsTie;

struct TreeBufs {
	double *sD, *Q, *contrib;
	int *N, *P;
	int *S, *uoff;       // DNJ_B rows, DNJ_B+1 unit offsets
	double *Sb;          // Q[S[t]] at selection time
	double *uq;          // per-unit (q, j) of the S rescans, by unit (uoff[t]..uoff[t+1])
	int *uj;
	Entry *Sent;         // folded S rows
	double *ef, *eb;     // replay entries in HBM when more than REPLAY_CAP rows
	int *erow, *ej;      // qualified below S (S first, then the rest)
	unsigned char *eacc;
	int *crow;           // rows found below S with Q < U, descending (k_dnj_select)
	double *cbnd;        // their bounds Q[row]
	int *coff;           // and SEG-cell unit offsets (REPLAY_CAP + 1)
	double *cq;          // per-unit (q, j) of the rest rescans, by unit (coff[e]..coff[e+1])
	int *cj;
	double *wsum, *wabs; // per-block partial sums / sum |c|
	int *wcnt, *wexp;    // per-block count / min exponent of the contributions
	double *qpart;       // 4 (q, idx) partials per block
	int *ipart;
	double *cfq;         // requeue: final (Q, P) of the row of each block's
	int *cfp;            // column-j (q, idx) partial, carried to the fold
	long long *fpart;
	double *bmq;         // requeue: each block's min-Q row (candidates of the next S)
	int *bmr, *bmp;      // and its partner P
	double *bmqp;        // and (with ubq) the Q criterion at that partner cell in the next join's state
	int *Spos;           // entry slot of each S row in the descending scan order
	int *cslot;          // and of each rest entry (k_dnj_find)
	double *rf;          // per rest entry: fresh (q, j) folded once by k_dnj_fold
	int *rj;             // (rows with many units)
	ccg_join *joins;
	TreeCtl *ctl;
	unsigned long long *xagg;   // exact row sum over the join blocks: tagged block sums (look-back)
	XsBlk *xblk;                // and each block's summary, crossing and tie records
	XsCross *xcr;
	XsTie *xti;
	unsigned long long *ppub;   // k_dnj_plan with several blocks: each block's tagged entry count (look-back)
	unsigned long long *jpub;   // k_dnj_join_pf, replay path: the pair block 0 chose, tagged with n (n, i, j: 21 bits each)
	double *chg;                // k_dnj_fold: per 64-entry chunk, the minimum fresh value,
	int *chr, *chj, *chb;       // the row and partner of its first entry reaching it, and whether any entry is "bad"
	unsigned *ecnt, *ccnt;      // the scan's fold at its last arrivals: units arrived per entry / entries per
	                            // 64-entry chunk (zero between joins: each last arriver resets its counter)
	int *pS_row, *pS_ent, *pS_uo;   // S for the scan's pruning: rows (descending), entry index, unit prefix
	double *pS_q, *pS_bnd;          // their Q (stale bounds), and the bound table the scan builds
	unsigned char *eS;              // per entry: 1 for an S row
	double *bmv, *vsuf;             // VBLK: per requeue block the minimum of V_k = max(q at the partner cell, Q_k),
	                                // and the scan's suffix minima of them (bounds from every row above)
	int *bcnt, *blist;              // k_dnj_sphase: surviving entries per unit-count bucket (zeroed by k_dnj_fold)
	                                // and their indices, bucket u at [entries with more than u units, ...)
	unsigned char *ePr;             // per entry: pruned by the S bound table this join (k_dnj_sphase)
	unsigned long long *shdr;       // k_dnj_plan's S header for its helper blocks: m0, sD of the moved row i,
	                                // (i << 32 | |S|), then the tag n (written last, write-through)
	double *sfq;                    // S rows' fresh minima by S index (the plan's helpers), and their
	int *sfj;                       // partners; ecS counts each S row's arrived units
	unsigned *ecS;
	int *uhist;                     // k_dnj_plan: per plan block, its entries by rescan-unit count (UHIST bins);
	                                // the compacted wave scan enumerates the real units from it
	unsigned *srdy;                 // SRDY_REP copies (one 128-B line each) of the tag n the scan's S bound
	                                // table is published with; block b polls copy b % SRDY_REP
	int maxu;
	// block lower bounds (DNJ, single engine, no missing entries; NULL when
	// off): lbm[r * lbs + u] = the bits of a float <= every cell of row r in
	// columns [64u, 64u + 64) (non-negative, so the bits order as the values;
	// kept conservative by atomicMin where a cell of a column changes),
	// msd[u] >= sD of every column there (the next join's, left by the
	// requeue).  The scan skips a 64-column block whose bound of the Q
	// criterion exceeds the q at the row's partner cell.
	unsigned *lbm;
	double *msd;
	double *ubq;         // per row: the Q criterion at its partner cell in this join's state (an upper bound
	                     // of its fresh minimum, left by the previous requeue; +inf: unknown, rows j and i)
	long long lbs;
	int lbw;             // 0: lbm rows are the matrix rows; w > 0: the sharded engine's, a rank's own rows
	                     // by position among them (bands of 8 rows dealt over w ranks, ccg_shard.h)
	int xs_allpre;       // the exact walk loads every block's records at once (CCG_XS_ALLPRE=1; default block by block)
	long long *lbskip;   // cells skipped under the block bounds (stats): per-wave slots of LB_SLOT longs --
	                     // field 0 the cells not loaded, field 1 those of them in S rows (the plan's helpers);
	                     // scan waves [0, LB_SCAN), helper waves after (no same-address atomics: thousands
	                     // of waves adding to one counter serialise at its L2 channel)
};

#define LBW 64   // columns per block of the lower bounds (one wave)
#define LB_SLOT 16      // longs per stats slot (one 128-B line)
#define LB_SCAN 4096    // scan wave slots
#define LB_HELP 8192    // helper wave slots

// row r's line of the block bounds
__device__ __forceinline__ unsigned *lb_line(const TreeBufs &b, int r) {
	const long long p = b.lbw ? (long long) ((r >> 3) / b.lbw) * 8 + (r & 7) : r;
	return b.lbm + p * b.lbs;
}

// a float <= x (x >= 0: a cell value) as order-preserving bits
__device__ __forceinline__ unsigned lb_bits(double x) {
	return x > 0.0 ? __float_as_uint(__double2float_rd(x)) : 0u;
}


// the device state of one tree run (one hipMalloc), sized for n taxa
struct TreeWork {
	TreeBufs b;
	void *mem;
};
int ccg_tree_alloc(TreeWork *w, int n, hipStream_t st);
size_t ccg_tree_bytes(int n);   // what ccg_tree_alloc allocates

// ------------------------------------------------------------------ helpers
__host__ __device__ static inline unsigned cdiv(long long a, long long b) { return (unsigned) ((a + b - 1) / b); }
__device__ __forceinline__ int dcdiv(int a, int b) { return (a + b - 1) / b; }

// block-wide exclusive prefix sum of a per-thread int; *total receives the sum
// (two barriers; `s` holds blockDim/64 ints)
__device__ __forceinline__ int block_excl_scan(int v, int *s, int *total) {
	const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
	const int x = wave_incl_sum(v);
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

// ---- wave-level building blocks (no block barriers)
// orders the wave's own LDS accesses (they complete in issue order per wave)
__device__ __forceinline__ void wave_sync() {
	__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
	__builtin_amdgcn_wave_barrier();
	__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ int wave_excl_scan(int v, int *total) {
	const int inc = wave_incl_sum(v);
	*total = __builtin_amdgcn_readlane(inc, 63);
	return inc - v;
}

// fixed-order wave sum (DPP scan order); the same value in every lane
__device__ __forceinline__ double wave_sum_fixed(double x) {
#define S_(C, R) x += dpp_d<C, R>(0.0, x);
	CCG_DPP_STEPS(S_)
#undef S_
	return readlane_d(x, 63);
}

__device__ __forceinline__ int wave_sum_int(int v) { return __builtin_amdgcn_readlane(wave_incl_sum(v), 63); }
__device__ __forceinline__ long long wave_sum_int(long long v) { return readlane_l(wave_incl_sum_l(v), 63); }
__device__ __forceinline__ int wave_min_int(int v) { return __builtin_amdgcn_readlane(wave_incl_min_i(v), 63); }
// wave minimum of u32 / maximum of f64, the same value in every lane (all lanes active)
__device__ __forceinline__ unsigned wave_min_u32(unsigned v) {
#define S_(C, R)                                                          \
	{                                                                     \
		const unsigned t_ = (unsigned) dpp_i<C, R>((int) 0xFFFFFFFFu, (int) v); \
		v = t_ < v ? t_ : v;                                              \
	}
	CCG_DPP_STEPS(S_)
#undef S_
	return (unsigned) __builtin_amdgcn_readlane((int) v, 63);
}
__device__ __forceinline__ double wave_max_d(double x) {
#define S_(C, R)                                   \
	{                                              \
		const double t_ = dpp_d<C, R>(-DBL_MAX, x); \
		x = t_ > x ? t_ : x;                       \
	}
	CCG_DPP_STEPS(S_)
#undef S_
	return readlane_d(x, 63);
}

// nj.c:42 limbLength / nj.c:81 limbLengthNeg
static __device__ void limb_length(double *Li, double *Lj, double sDi, double sDj, int Ni_, int Nj_, double Dij, int neg) {
	int Ni = Ni_ - 2, Nj = Nj_ - 2;
	if(0 < Ni && 0 < Nj) {
		double delta = ((sDi - Dij) / Ni) - ((sDj - Dij) / Nj);
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

// ------------------------------------------------------------------ updateD body
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

// The per-block partials of the new row sum of j (sum, sum |c|, count, min
// exponent) and, in exact mode, each contribution; thread k of the grid holds
// contribution d of row k (0 for k in {i, j} or k >= n).
__device__ __forceinline__ void update_partials(const TreeBufs &b, int n, bool exact, int k, double d, int cnt,
                                                int slot) {
	__shared__ double ssum[TB / 64], sabs[TB / 64];
	__shared__ int scnt[TB / 64], sexp[TB / 64];
	if(exact && k < n) b.contrib[k] = d;
	const double s = wave_sum_fixed(d), a = wave_sum_fixed(fabs(d));
	cnt = wave_sum_int(cnt);
	const int e = wave_min_int(low_exp(d));
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
		for(int w = 0; w < TB / 64; ++w) {
			t += ssum[w];
			ta += sabs[w];
			c += scnt[w];
			te = sexp[w] < te ? sexp[w] : te;
		}
		b.wsum[slot] = t;
		b.wabs[slot] = ta;
		b.wcnt[slot] = c;
		b.wexp[slot] = te;
	}
}


// Wave 0: fold of the updateD partials of G blocks into the new row sum of j
// and its count (fixed order: lane l sums blocks l, l+64, ... in order, then
// a shfl_down tree), identical in every block.  In exact mode this is the
// reference's serial sum whenever that is provable (all contributions
// multiples of 2^e, sum |c| < 2^53 * 2^e, e.g. integer SNP distances);
// otherwise *need_serial asks for the serial order (k_exact_sum).  General (missing data):
// k_update_general left the serial sum in wsum[0].
static __device__ void fold_update_wave(const TreeBufs &b, int G, bool exact, bool general, double *sd_out, int *nj_out,
                                 bool *need_serial) {
	const int lane = threadIdx.x & 63;
	*need_serial = false;
	if(general) {
		*sd_out = b.wsum[0];
		*nj_out = 1 + b.wcnt[0];
		return;
	}
	double s = 0, a = 0;
	int c = 0, e = INT32_MAX;
	for(int g = lane; g < G; g += 64) {
		s += b.wsum[g];
		a += b.wabs[g];
		c += b.wcnt[g];
		int oe = b.wexp[g];
		e = oe < e ? oe : e;
	}
	const double sd = wave_sum_fixed(s);
	a = wave_sum_fixed(a);
	c = wave_sum_int(c);
	e = wave_min_int(e);
	if(exact) {
		bool provable = e != INT32_MIN && (e == INT32_MAX || (e > -1000 && a * (1.0 + 1e-9) < ldexp(1.0, 53 + e)));
		*need_serial = !provable;
	}
	*sd_out = sd;
	*nj_out = 1 + c;
}

// the reference's serial sum of the contributions in increasing k (nj.c:911 /
// :1002); thread 0 runs the chain while the block stages the next chunk of
// XC_CH elements (NT threads, NT <= XC_CH)
#define XC_CH 1024
template <int NT>
static __device__ double serial_sum_t(const double *__restrict__ c, int n) {
	constexpr int PER = XC_CH / NT;
	__shared__ __attribute__((aligned(16))) double buf[2 * XC_CH];
	__shared__ double s_sd;
	double sd = 0;
	double nxt[PER];
#pragma unroll
	for(int m = 0; m < PER; ++m) {
		int kk = m * NT + threadIdx.x;
		buf[m * NT + threadIdx.x] = kk < n ? c[kk] : 0.0;
	}
	__syncthreads();
	for(int c0 = 0, p = 0; c0 < n; c0 += XC_CH, p ^= 1) {
#pragma unroll
		for(int m = 0; m < PER; ++m) {
			int kk = c0 + XC_CH + m * NT + threadIdx.x;
			nxt[m] = kk < n ? c[kk] : 0.0;
		}
		if(threadIdx.x == 0) {
			const double *cur = buf + p * XC_CH;
			const int lim = n - c0 < XC_CH ? n - c0 : XC_CH;
			// one dependent add per element; the 16-byte LDS loads of the next
			// 16 elements are issued ahead of the chain
			int u = 0;
			for(; u + 16 <= lim; u += 16) {
				double2 v[8];
#pragma unroll
				for(int q = 0; q < 8; ++q) v[q] = *(const double2 *) (cur + u + 2 * q);
#pragma unroll
				for(int q = 0; q < 8; ++q) {
					sd += v[q].x;
					sd += v[q].y;
				}
			}
			for(; u < lim; ++u) sd += cur[u];
		}
#pragma unroll
		for(int m = 0; m < PER; ++m) buf[(p ^ 1) * XC_CH + m * NT + threadIdx.x] = nxt[m];
		__syncthreads();
	}
	if(threadIdx.x == 0) s_sd = sd;
	__syncthreads();
	return s_sd;
}

// ---- diagnostic build only (make trace): s_memrealtime stamps (100 MHz) of
// block 0's entry and phases and of the last block exit, for the joins at
// n in (g_trace_hi - 256, g_trace_hi]; dumped to stderr by tree_run_t.
#if defined(CCG_TRACE) && !defined(CCG_DNJ_NO_TRACE)
#define NKT 5
__device__ unsigned long long g_trace[256 * NKT * 16];
__device__ int g_trace_hi;
__device__ __forceinline__ unsigned long long rt_stamp() {
	unsigned long long t;
	__builtin_amdgcn_sched_barrier(0);
	asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
	__builtin_amdgcn_sched_barrier(0);
	return t;
}
#define TS(kern, ph)                                                                  \
	do {                                                                              \
		if(blockIdx.x == 0 && threadIdx.x == 0) {                                     \
			int s_ = g_trace_hi - n;                                                  \
			if(s_ >= 0 && s_ < 256) g_trace[(s_ * NKT + (kern)) * 16 + (ph)] = rt_stamp(); \
		}                                                                             \
	} while(0)
#define TSW(kern, ph, th)                                                             \
	do {                                                                              \
		if(blockIdx.x == 0 && threadIdx.x == (th)) {                                  \
			int s_ = g_trace_hi - n;                                                  \
			if(s_ >= 0 && s_ < 256) g_trace[(s_ * NKT + (kern)) * 16 + (ph)] = rt_stamp(); \
		}                                                                             \
	} while(0)
#define TS_ENTRY(kern)                                                                \
	do {                                                                              \
		if(blockIdx.x == 0 && threadIdx.x == 0) {                                     \
			int s_ = g_trace_hi - n;                                                  \
			if(s_ >= 0 && s_ < 256) g_trace[(s_ * NKT + (kern)) * 16 + 15] = ~rt_stamp(); \
		}                                                                             \
	} while(0)
// every 32nd block of the scan: entry / table staged / exit stamps (no atomics)
__device__ unsigned long long g_samp[256 * 64 * 3];
#define TS_SAMP(ph)                                                                   \
	do {                                                                              \
		if(threadIdx.x == 0 && (blockIdx.x & 31) == 0 && (blockIdx.x >> 5) < 64) {    \
			int s_ = g_trace_hi - n;                                                  \
			if(s_ >= 0 && s_ < 256) g_samp[(s_ * 64 + (blockIdx.x >> 5)) * 3 + (ph)] = rt_stamp(); \
		}                                                                             \
	} while(0)
// wave 0 of every 32nd scan block: start / end stamps of its first 4 units (slots 0..7)
__device__ unsigned long long g_uamp[256 * 64 * 8];
#define TS_U(slot)                                                                    \
	do {                                                                              \
		if(threadIdx.x == 0 && (blockIdx.x & 31) == 0 && (blockIdx.x >> 5) < 64 && (slot) < 8) { \
			int s_ = g_trace_hi - n;                                                  \
			if(s_ >= 0 && s_ < 256) g_uamp[(s_ * 64 + (blockIdx.x >> 5)) * 8 + (slot)] = rt_stamp(); \
		}                                                                             \
	} while(0)
#define TS_EXIT(kern)                                                                 \
	do {                                                                              \
		if(threadIdx.x == 0) {                                                        \
			int s_ = g_trace_hi - n;                                                  \
			if(s_ >= 0 && s_ < 256) atomicMax(&g_trace[(s_ * NKT + (kern)) * 16 + 14], rt_stamp()); \
		}                                                                             \
	} while(0)
#else
#define TS_U(slot)
#define TS_EXIT(kern)
#define TS(kern, ph)
#define TSW(kern, ph, th)
#define TS_SAMP(ph)
#define TS_ENTRY(kern)
#endif

// ------------------------------------------------------------------ exact row sum, in parallel
// The reference's serial sum s_k = fl(s_{k-1} + c_k) (nj.c:911 / :1002) of
// the new row of j, computed without its dependent chain.  Every c_k >= 0
// (updateD clamps d at 0), so s only grows and stays in one binade
// [2^e, 2^(e+1)) for long runs of k.  Inside such a run every s is a multiple
// of u = 2^(e-52), so fl(s + c) = s + RN_u(c): c rounded to a multiple of u,
// a tie (remainder exactly u/2) going to the even total.  The sum of a run is
// then an exact integer sum of its increments (any order), and only the few
// elements where s changes binade ("crossings", ~log2 of the sum's growth)
// need the true floating-point add, in order.
//   pass 1: per-thread sums -> an approximate prefix P (only a prediction);
//   pass 2: per element, the binade of P before it predicts the run; a change
//           of binade is a crossing (listed); otherwise the increment in
//           units of u (integer-valued doubles, summed exactly); ties listed
//           with the parity of their run prefix;
//   walk:   one lane, per run in order: total = start/u + sum + tie round-ups
//           (each tie makes the running total even), then the crossing's
//           real add.
// Every prediction is verified (start and crossing binades, totals < 2^53,
// the binade each thread's first run assumed); any failure, a negative or
// non-finite c, or more crossings / ties than the lists hold returns false
// and the caller runs the serial chain.  Validated against the serial sum on
// 3000 random, dyadic tie-heavy and wide-range inputs (tools/sim_exact_sum.py).
#define XS_CAP 128                // crossings / ties listed per sum (xs_walk_blocks: crossings)
#define XS_CAP_T 512              // xs_walk_blocks: ties listed per sum (one per run and join block)
#define XS_HEAD 64                // elements summed serially first

struct XsCross {
	double v, run;   // c_k; provisional sum (units of its run's u) of the chunk's run before it
	int k, x;        // element; biased exponent of s after it
	int R, tb;       // last-run parities of the chunks before its chunk; ties before it
};
struct XsTie {
	int k, pi;       // element; parity of its run prefix (within the chunk) + floor(c/u)
	int R, first;    // as XsCross.R; 1: in its chunk's first run
};

// biased exponent field of x >= 0 (0 for zeros and subnormals, 0x7FF for inf / NaN)
__device__ __forceinline__ int xs_bexp(double x) {
	return (int) (((unsigned) ((unsigned long long) __double_as_longlong(x) >> 32) >> 20) & 0x7FF);
}

// parity of an integer-valued double 0 <= y < 2^53
__device__ __forceinline__ int xs_par(double y) {
	if(y < 1.0) return 0;
	const unsigned long long u = (unsigned long long) __double_as_longlong(y);
	const int sh = 1075 - (int) ((u >> 52) & 0x7FF);   // bit of the units digit in the mantissa
	const unsigned long long m = (u & ((1ull << 52) - 1)) | (1ull << 52);
	return (int) ((m >> sh) & 1ull);
}

#define XS_STAMP(i)                                                                 \
	do {                                                                            \
		if(stamps && (threadIdx.x & 63) == 0 && threadIdx.x < 256) stamps[i + 16 * (threadIdx.x >> 6)] = __builtin_amdgcn_s_memrealtime(); \
	} while(0)

// whole block of NT threads; true and *out = the serial sum, or false.  Wave w owns
// a contiguous range of rows of 256 elements (lane l: elements 4l .. 4l+3),
// walks them in order with wave-level scans only, and keeps its crossing and
// tie records, in element order, in its own lists; one block barrier then
// joins the waves.  The binade of the running sum is predicted per element
// from one approximate prefix chain (each lane continues the lane before it,
// each row the row before it); a crossing is an element whose predicted
// binade differs from its predecessor's, so every run uses one unit.
#define XW_CAP 32                 // crossing / tie records per wave
#define XW_EL 4                   // elements per lane per row

template <int NT, int RB>
static __device__ bool exact_sum_w(const double *__restrict__ c, int n, double *out,
                                   unsigned long long *stamps = nullptr) {
	constexpr int NW = NT / 64, RE = 64 * XW_EL;
	__shared__ XsCross xw[NW][XW_CAP];
	__shared__ XsTie tw[NW][XW_CAP];
	__shared__ double s_wt[NW], s_tail[NW], s_seg[XS_CAP + 1], s_out, s_head;
	__shared__ int s_nc[NW], s_nt[NW], s_tp[NW], s_ex0[NW], s_bad, s_eh;
	__shared__ __attribute__((aligned(16))) double s_hb[XS_HEAD];
	const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
	if(tid == 0) s_bad = 0;
	for(int q = tid; q <= XS_CAP; q += NT) s_seg[q] = 0.0;
	XS_STAMP(0);
	const int rows = (n + RE - 1) / RE, rpw = (rows + NW - 1) / NW;
	const int r0 = w * rpw, r1 = r0 + rpw < rows ? r0 + rpw : rows;
	const bool inreg = rpw <= RB;   // uniform
	double x[RB][XW_EL];
	auto load = [&](int rb) {   // rows rb .. rb + RB - 1 of this wave (clamped)
#pragma unroll
		for(int q = 0; q < RB; ++q)
#pragma unroll
			for(int e = 0; e < XW_EL; ++e) {
				const int k = (rb + q) * RE + XW_EL * lane + e;
				const double v = c[k < n && rb + q < r1 ? k : n - 1];
				x[q][e] = k < n && k >= XS_HEAD && rb + q < r1 ? v : 0.0;
			}
	};
	// ---- pass 1: the wave's total (approximate prefixes of the waves)
	double wt = 0;
	bool bad = false;
	for(int rb = r0; rb < r1; rb += RB) {
		load(rb);
#pragma unroll
		for(int q = 0; q < RB; ++q)
#pragma unroll
			for(int e = 0; e < XW_EL; ++e) {
				bad |= !(x[q][e] >= 0.0 && x[q][e] <= DBL_MAX);
				wt += x[q][e];
			}
	}
	// the head: the first XS_HEAD elements summed serially (wave 0, one
	// dependent add each; most binade changes of s happen while s is small)
	if(w == 0) {
		s_hb[lane] = lane < n ? c[lane] : 0.0;
		wave_sync();
		if(lane == 0) {   // 16-byte LDS loads ahead of one dependent add each
			double S = 0;
#pragma unroll
			for(int l = 0; l < XS_HEAD; l += 2) {
				const double2 v = *(const double2 *) (s_hb + l);
				S += v.x;
				S += v.y;
			}
			s_head = S;
			s_eh = xs_bexp(S);
		}
	}
	wt = wave_sum_fixed(wt);
	if(lane == 0) s_wt[w] = wt;
	__syncthreads();
	XS_STAMP(9);
	const double SH = s_head;
	const int eH = s_eh;
	double P = SH;
	for(int q = 0; q < w; ++q) P += s_wt[q];
	int ep_c = xs_bexp(P);   // predicted binade before the wave's first element
	if(lane == 0) s_ex0[w] = ep_c;
	bad |= P != 0.0 && ep_c == 0;
	// ---- pass 2: rows in order
	int nc = 0, nt = 0;      // the wave's records so far (uniform)
	double acc = 0;          // provisional sum of the current run in this wave (units of its u)
	for(int rb = r0; rb < r1; rb += RB) {
		if(!inreg) load(rb);
#pragma unroll
		for(int q = 0; q < RB; ++q) {
			if(rb + q >= r1) break;   // uniform
			// lane prefix within the row (approximate), continuing the chain
			const double cs = x[q][0] + x[q][1] + x[q][2] + x[q][3];
			double xs = cs;
#define S_(C, R_) xs += dpp_d<C, R_>(0.0, xs);
			CCG_DPP_STEPS(S_)
#undef S_
			double Pl = P + (xs - cs);
			double Pn[XW_EL];
			int en[XW_EL];
#pragma unroll
			for(int e = 0; e < XW_EL; ++e) {
				Pl += x[q][e];
				Pn[e] = Pl;
				en[e] = xs_bexp(Pl);
			}
			// binade before the lane's first element: the previous lane's last
			int epl = dpp_i<DPP_WAVE_SHR1, 0xF>(ep_c, en[XW_EL - 1]);
			unsigned cm = 0, tm = 0;
			double fl[XW_EL], run = 0;
#pragma unroll
			for(int e = 0; e < XW_EL; ++e) {
				const int ep = e ? en[e - 1] : epl;
				const double t = ldexp(x[q][e], 1075 - ep) + 0.5;
				fl[e] = floor(t);
				cm |= (unsigned) (ep != en[e]) << e;
				tm |= (unsigned) (t == fl[e]) << e;
				run += fl[e];
			}
			tm &= ~cm;
			ep_c = __builtin_amdgcn_readlane(en[XW_EL - 1], 63);
			P = readlane_d(Pn[XW_EL - 1], 63);
			const unsigned long long fm = __ballot((cm | tm) != 0u);
			if(fm == 0ull) {
				acc += wave_sum_fixed(run);   // integers below 2^53: exact in any order
				continue;
			}
			// a row with crossings or ties (few): flagged lanes in order, the
			// complete chunks between them as masked sums
			int from = 0;
			for(unsigned long long f = fm; f; f &= f - 1) {
				const int L = __ffsll((long long) f) - 1;
				acc += wave_sum_fixed(lane >= from && lane < L ? run : 0.0);
				const unsigned cmL = __builtin_amdgcn_readlane(cm, L), tmL = __builtin_amdgcn_readlane(tm, L);
#pragma unroll
				for(int e = 0; e < XW_EL; ++e) {
					const double fe = readlane_d(fl[e], L);
					const int k = (rb + q) * RE + XW_EL * L + e;
					if((cmL >> e) & 1u) {
						if(nc < XW_CAP && lane == 0) {
							XsCross r;
							r.v = readlane_d(x[q][e], L);
							r.run = acc;
							r.k = k;
							r.x = __builtin_amdgcn_readlane(en[e], L);
							r.R = 0;
							r.tb = nt;
							xw[w][nc] = r;
						}
						++nc;
						acc = 0;
					} else {
						if((tmL >> e) & 1u) {
							if(nt < XW_CAP && lane == 0) {
								XsTie r;
								r.k = k;
								r.pi = (xs_par(acc) + xs_par(fe) + 1) & 1;   // floor = fl - 1
								r.R = nc;                                    // local run of the tie
								r.first = nc == 0;
								tw[w][nt] = r;
							}
							++nt;
						}
						acc += fe;
					}
				}
				from = L + 1;
			}
			acc += wave_sum_fixed(lane >= from ? run : 0.0);
		}
	}
	bad |= ep_c == 0x7FF || nc > XW_CAP || nt > XW_CAP;
	if(lane == 0) {
		s_tail[w] = acc;
		s_nc[w] = nc;
		s_nt[w] = nt;
		s_tp[w] = xs_par(acc);
	}
	if(bad) s_bad = 1;
	XS_STAMP(3);
	__syncthreads();
	XS_STAMP(5);
	// ---- join the waves: global record indices, segment sums, checks
	int co[NW + 1], to[NW + 1], Rw[NW + 1];
	co[0] = to[0] = Rw[0] = 0;
#pragma unroll
	for(int q = 0; q < NW; ++q) {
		co[q + 1] = co[q] + s_nc[q];
		to[q + 1] = to[q] + s_nt[q];
		Rw[q + 1] = Rw[q] + s_tp[q];
	}
	const int nx = co[NW], ntot = to[NW];
	if(s_bad || nx > XS_CAP - 1 || ntot > XS_CAP) return false;
	auto cross_at = [&](int g, int *wv) -> const XsCross & {   // global crossing g -> its record
		int q = 0;
#pragma unroll
		for(int z = 1; z < NW; ++z) q += g >= co[z];
		*wv = q;
		return xw[q][g - co[q]];
	};
	auto tie_at = [&](int g, int *wv) -> const XsTie & {
		int q = 0;
#pragma unroll
		for(int z = 1; z < NW; ++z) q += g >= to[z];
		*wv = q;
		return tw[q][g - to[q]];
	};
	// each wave's first run must have assumed its segment's binade; its last
	// run's sum goes to its segment
	if(tid < NW) {
		int wc;
		const int want = co[tid] == 0 ? eH : cross_at(co[tid] - 1, &wc).x;
		if(s_ex0[tid] != want) s_bad = 1;
		atomicAdd(&s_seg[co[tid] + s_nc[tid]], s_tail[tid]);   // integer-valued: exact in any order
	}
	__syncthreads();
	if(s_bad) return false;
	// ---- walk (wave 0)
	if(w == 0) {
		double A0[2], A1[2], cvA[2];
		int exA[2], cxA[2];
#pragma unroll
		for(int h = 0; h < 2; ++h) {
			const int s = lane + 64 * h;
			A0[h] = A1[h] = cvA[h] = 0.0;
			exA[h] = cxA[h] = 0;
			if(s <= nx) {
				int wc = 0, wn = 0;
				double seg = s_seg[s];
				int ta = 0, tz = ntot;
				if(s) {
					const XsCross &p = cross_at(s - 1, &wc);
					exA[h] = p.x;
					ta = to[wc] + p.tb;
				} else {
					exA[h] = eH;
				}
				if(s < nx) {
					const XsCross &q = cross_at(s, &wn);
					cvA[h] = q.v;
					cxA[h] = q.x;
					seg += q.run;
					tz = to[wn] + q.tb;
				}
				int dn0 = 0, dn1 = 0;
				for(int g = ta; g < tz; ++g) {
					int wt2;
					const XsTie &t = tie_at(g, &wt2);
					int pi = t.pi;
					// a run that began in an earlier wave: the parities of the last
					// runs of the waves from the crossing's on come before it
					if(t.first) pi ^= (Rw[wt2] - Rw[wc]) & 1;
					dn0 += 1 - ((pi + dn0) & 1);
					dn1 += 1 - ((1 + pi + dn1) & 1);
				}
				A0[h] = seg - (double) dn0;
				A1[h] = seg - (double) dn1;
			}
		}
		XS_STAMP(6);
		double S = SH;
		bool ok = (eH > 0 && eH < 0x7FF) || (SH == 0.0 && s_seg[0] == 0.0);
		for(int s = 0; s <= nx; ++s) {
			const int h = s >> 6, l = s & 63;
			if(s > 0 || eH > 0) {
				const int exs = __builtin_amdgcn_readlane(h ? exA[1] : exA[0], l);
				const double a0 = readlane_d(h ? A0[1] : A0[0], l), a1 = readlane_d(h ? A1[1] : A1[0], l);
				const int ue = exs - 1075;   // u = 2^ue
				ok = ok && exs > 0 && exs < 0x7FF && xs_bexp(S) == exs;
				const double T0 = ldexp(S, -ue);   // in [2^52, 2^53): its units bit is the mantissa's last
				const double T = T0 + (((unsigned) __double_as_longlong(T0) & 1u) ? a1 : a0);
				ok = ok && T < 9007199254740992.0;
				S = ldexp(T, ue);
			}
			if(s < nx) {
				const double Sn = S + readlane_d(h ? cvA[1] : cvA[0], l);
				ok = ok && xs_bexp(Sn) == __builtin_amdgcn_readlane(h ? cxA[1] : cxA[0], l);
				S = Sn;
			}
		}
		if(lane == 0) {
			s_out = S;
			s_bad = !ok;
		}
		XS_STAMP(7);
	}
	__syncthreads();
	XS_STAMP(8);
	*out = s_out;
	return !s_bad;
}

// ------------------------------------------------------------------ exact row sum, over the join blocks
// The single-GPU engine splits exact_sum_w over the kernels that already
// exist, so no kernel of its own sits between updateD and its consumers:
//   the join kernel (k_dnj_join / k_nj_join), block g holding the
//   contributions of elements 256g .. 256g+255 after its updateD:
//     1. publishes its (fixed-order) block sum as a tagged 8-byte granule;
//     2. block 0 sums the head serially; block g > 0 takes the approximate
//        prefix from the granules of blocks 0 .. g-1 (a decoupled look-back:
//        a block only waits on lower-indexed blocks, which are dispatched
//        before it and never wait on it; the spin is bounded);
//     3. runs pass 2 of exact_sum_w over its row (wave 0, 4 elements per
//        lane) and stores its crossing / tie records and tail in HBM;
//   the consumer (k_dnj_requeue / k_nj_pop / k_hnj_update), wave 0 of every
//   block: joins the rows' records (prefixes over the blocks, checks) and
//   walks the crossings (xs_walk_blocks), exactly as exact_sum_w's wave 0 does.
// Any failed check falls back to the serial chain, in the consumer.
#define XB_CAP 8                  // crossing records per join block
#define XB_CAP_T (XB_CAP + 1)     // tie records per join block: one per run (a run's later ties are resolved in place)
// why the parallel form declined (TreeCtl::xs_why counts, CCG_XS_WHY=1 prints them)
#define XS_WHY_VALUE 1    // a negative / non-finite contribution, a subnormal or infinite prefix
#define XS_WHY_NC 2       // more than XB_CAP crossings in one join block
#define XS_WHY_NT 4       // more than XB_CAP ties in one join block
#define XS_WHY_STUCK 8    // the look-back for the block's prefix timed out
#define XS_WHY_EX0 16     // a block's assumed start binade was not the walk's
#define XS_WHY_CAP 32     // more than XS_CAP crossings / ties in the row
#define XS_WHY_WALK 64    // the walk's own checks (binade, < 2^53)
#define XS_NWHY 7
#define XS_TAG_BITS 20

struct XsBlk {
	double tail, head;   // provisional sum of the block's last run (units of its u); block 0: the head's serial sum
	int nc, nt, tp, ex0; // records, parity of tail, predicted binade before the block's first element
	int eh, bad, pad0, pad1;
};

__device__ __forceinline__ unsigned long long xs_granule(double a, unsigned tag) {
	return ((unsigned long long) __double_as_longlong(a) & ~((1ull << XS_TAG_BITS) - 1)) | tag;
}
// tag of the join at matrix size n (consecutive joins differ; never 0, the
// value of the zeroed buffer)
__device__ __forceinline__ unsigned xs_tag(int n) { return (unsigned) (n % ((1 << XS_TAG_BITS) - 1)) + 1u; }

// all threads of a TB-thread join block; d = contribution of element
// TB * blk + threadIdx.x (0 where none)
__device__ void xs_join_row(const TreeBufs &b, int n, int blk, double d, unsigned tag) {
	__shared__ __attribute__((aligned(16))) double s_row[TB];
	const int tid = threadIdx.x, lane = tid & 63;
	s_row[tid] = d;
	__syncthreads();
	if(tid >= 64) return;
	double x[XW_EL];
#pragma unroll
	for(int e = 0; e < XW_EL; ++e) x[e] = s_row[XW_EL * lane + e];
	// 1. publish the block sum (approximate: only predicts binades)
	const double A = wave_sum_fixed(x[0] + x[1] + x[2] + x[3]);
	if(lane == 0) __hip_atomic_store(b.xagg + blk, xs_granule(A, tag), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
	const int k0 = TB * blk + XW_EL * lane;
	bool bad = false, stuck = false;   // (reasons for the consumer's diagnostics: XS_WHY_*)
#pragma unroll
	for(int e = 0; e < XW_EL; ++e) {
		bad |= !(x[e] >= 0.0 && x[e] <= DBL_MAX);
		if(k0 + e < XS_HEAD) x[e] = 0.0;   // the head is summed serially
	}
	// 2. prefix before the row
	double P = 0, SH = 0;
	int eH = 0;
	if(blk == 0) {
		if(lane == 0) {
			double S = 0;
#pragma unroll
			for(int l = 0; l < XS_HEAD; l += 2) {
				const double2 v = *(const double2 *) (s_row + l);
				S += v.x;
				S += v.y;
			}
			SH = S;
		}
		SH = readlane_d(SH, 0);
		eH = xs_bexp(SH);
		P = SH;
	} else {
		for(int g0 = 0; g0 < blk; g0 += 64) {
			const int g = g0 + lane;
			unsigned long long u = 0;
			bool ok = g >= blk;
			for(int spin = 0;; ++spin) {
				if(!ok) {
					u = __hip_atomic_load(b.xagg + g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
					ok = (unsigned) (u & ((1u << XS_TAG_BITS) - 1)) == tag;
				}
				if(__all(ok)) break;
				if(spin > (1 << 22)) {   // bounded: a stuck predecessor costs the serial chain, never a hang
					stuck = true;
					break;
				}
				__builtin_amdgcn_s_sleep(2);
			}
			const double a = g < blk && ok ? __longlong_as_double((long long) (u & ~((1ull << XS_TAG_BITS) - 1))) : 0.0;
			P += wave_sum_fixed(a);
		}
	}
	int ep_c = xs_bexp(P);
	const int ex0 = ep_c;
	bad |= P != 0.0 && ep_c == 0;
	// 3. pass 2 over the row (exact_sum_w's row body)
	int nc = 0, nt = 0;
	double acc = 0;
	{
		const double cs = x[0] + x[1] + x[2] + x[3];
		double xs = cs;
#define S_(C, R_) xs += dpp_d<C, R_>(0.0, xs);
		CCG_DPP_STEPS(S_)
#undef S_
		double Pl = P + (xs - cs);
		double Pn[XW_EL];
		int en[XW_EL];
#pragma unroll
		for(int e = 0; e < XW_EL; ++e) {
			Pl += x[e];
			Pn[e] = Pl;
			en[e] = xs_bexp(Pl);
		}
		const int epl = dpp_i<DPP_WAVE_SHR1, 0xF>(ep_c, en[XW_EL - 1]);
		unsigned cm = 0, tm = 0;
		double fl[XW_EL], run = 0;
#pragma unroll
		for(int e = 0; e < XW_EL; ++e) {
			const int ep = e ? en[e - 1] : epl;
			const double t = ldexp(x[e], 1075 - ep) + 0.5;
			fl[e] = floor(t);
			cm |= (unsigned) (ep != en[e]) << e;
			tm |= (unsigned) (t == fl[e]) << e;
			run += fl[e];
		}
		tm &= ~cm;
		ep_c = __builtin_amdgcn_readlane(en[XW_EL - 1], 63);
		const unsigned long long fm = __ballot((cm | tm) != 0u);
		if(fm == 0ull) {
			acc = wave_sum_fixed(run);   // integers below 2^53: exact in any order
		} else {
			XsCross *xc = b.xcr + (size_t) blk * XB_CAP;
			XsTie *xt = b.xti + (size_t) blk * XB_CAP_T;
			int from = 0;
			// a run's first tie in this block is a record (its rounding depends on
			// the parity of the sum before the block); after any tie the sum is
			// even (round half to even), so each later tie of the run rounds up
			// iff the increments since the previous tie plus floor(c/u) are odd,
			// known here: its true increment goes into the run sum directly
			bool tied = false;
			double acc_t = 0;
			for(unsigned long long f = fm; f; f &= f - 1) {
				const int L = __ffsll((long long) f) - 1;
				acc += wave_sum_fixed(lane >= from && lane < L ? run : 0.0);
				const unsigned cmL = __builtin_amdgcn_readlane(cm, L), tmL = __builtin_amdgcn_readlane(tm, L);
#pragma unroll
				for(int e = 0; e < XW_EL; ++e) {
					const double fe = readlane_d(fl[e], L);
					const int k = TB * blk + XW_EL * L + e;
					if((cmL >> e) & 1u) {
						if(nc < XB_CAP && lane == 0) {
							XsCross r;
							r.v = readlane_d(x[e], L);
							r.run = acc;
							r.k = k;
							r.x = __builtin_amdgcn_readlane(en[e], L);
							r.R = 0;
							r.tb = nt;
							xc[nc] = r;
						}
						++nc;
						acc = 0;
						tied = false;
					} else if((tmL >> e) & 1u) {
						if(!tied) {
							if(nt < XB_CAP_T && lane == 0) {
								XsTie r;
								r.k = k;
								r.pi = (xs_par(acc) + xs_par(fe) + 1) & 1;
								r.R = nc;
								r.first = nc == 0;
								xt[nt] = r;
							}
							++nt;
							tied = true;
							acc += fe;
						} else {
							const bool up = xs_par(acc - acc_t + (fe - 1.0)) != 0;
							acc += up ? fe : fe - 1.0;
						}
						acc_t = acc;
					} else {
						acc += fe;
					}
				}
				from = L + 1;
			}
			acc += wave_sum_fixed(lane >= from ? run : 0.0);
		}
	}
	bad |= ep_c == 0x7FF;
	const int why = (__any(bad) ? XS_WHY_VALUE : 0) | (__any(stuck) ? XS_WHY_STUCK : 0) |
	                (nc > XB_CAP ? XS_WHY_NC : 0) | (nt > XB_CAP_T ? XS_WHY_NT : 0);   // nc, nt: uniform
	if(lane == 0) {
		XsBlk s;
		s.tail = acc;
		s.head = SH;
		s.nc = nc;
		s.nt = nt;
		s.tp = xs_par(acc);
		s.ex0 = ex0;
		s.eh = eH;
		s.bad = why;
		s.pad0 = s.pad1 = 0;
		b.xblk[blk] = s;
	}
	(void) n;
}

// wave 0 of a consumer block: the serial sum from the G join blocks'
// records; false when a check fails (the caller then runs the chain)
// the walk's first loads, issued before the consumer knows it needs them
// (with the fold's partials, one round trip instead of three): lane g < 64
// holds block g's summary, its first XS_PRE_C crossings and first tie
#define XS_PRE_C 2
#define XS_PRE_H 4   // blocks' summaries prefetched per lane: every join block up to G = 256 (n = 65536)
struct XsPre {
	XsBlk blk, bh[XS_PRE_H - 1];   // blocks lane, lane + 64 h
	XsCross cr[XS_PRE_C];
	XsTie ti;
};
__device__ __forceinline__ void xs_prefetch(const TreeBufs &b, int G, XsPre &p) {
	const int g = threadIdx.x & 63;
	if(g < G) {
		p.blk = b.xblk[g];
#pragma unroll
		for(int c = 0; c < XS_PRE_C; ++c) p.cr[c] = b.xcr[(size_t) g * XB_CAP + c];
		p.ti = b.xti[(size_t) g * XB_CAP_T];
	}
#pragma unroll
	for(int h = 1; h < XS_PRE_H; ++h)
		if(g + 64 * h < G) p.bh[h - 1] = b.xblk[g + 64 * h];
}

__device__ bool xs_walk_blocks(const TreeBufs &b, int G, double *out, const XsPre *pre, int n, int *why_out) {
	(void) n;   // trace stamps only
	__shared__ XsCross lc[XS_CAP];
	__shared__ int lcR[XS_CAP], lcT[XS_CAP];   // the crossing's block: Rw, global index of its first tie
	__shared__ XsTie lt[XS_CAP_T];
	__shared__ int ltR[XS_CAP_T];              // the tie's block: Rw
	__shared__ double lseg[XS_CAP + 1];
	const int lane = threadIdx.x & 63;
	for(int q = lane; q <= XS_CAP; q += 64) lseg[q] = 0.0;
	const double SH = b.xblk[0].head;
	const int eH = b.xblk[0].eh;
	int cob = 0, tob = 0, Rwb = 0;
	int why = 0;
	wave_sync();
	// every block's summary is in registers (pre, G <= 256): the record loads
	// of all blocks are issued together below, one round trip (round 5);
	// otherwise block by block as they come
	const bool allpre = pre && G <= 64 * XS_PRE_H && b.xs_allpre;
	__shared__ int bco[64 * XS_PRE_H], bto[64 * XS_PRE_H], bRw[64 * XS_PRE_H], bex[64 * XS_PRE_H];
	__shared__ short cown[XS_CAP], town[XS_CAP_T];   // the block of each crossing / tie record
	for(int g0 = 0; g0 < G; g0 += 64) {
		const int g = g0 + lane, ph = g0 >> 6;
		XsBlk s;
		if(g < G) {
			s = pre && g0 == 0 ? pre->blk
			    : allpre       ? pre->bh[ph >= 1 && ph < XS_PRE_H ? ph - 1 : 0]
			                   : b.xblk[g];
		} else {
			s.tail = 0;
			s.nc = s.nt = s.tp = s.ex0 = s.bad = 0;
		}
		why |= s.bad | (s.nc > XB_CAP ? XS_WHY_NC : 0) | (s.nt > XB_CAP_T ? XS_WHY_NT : 0);
		int tc, tt, tr;
		const int co = cob + wave_excl_scan(s.nc, &tc);
		const int to = tob + wave_excl_scan(s.nt, &tt);
		const int Rw = Rwb + wave_excl_scan(s.tp, &tr);
		if(allpre) {   // the block's place in the record lists; the records come after the loop
			bco[g0 + lane] = co;
			bto[g0 + lane] = to;
			bRw[g0 + lane] = Rw;
			bex[g0 + lane] = s.ex0;
			if(g < G) {
				for(int c = 0; c < s.nc && c < XB_CAP && co + c < XS_CAP; ++c) cown[co + c] = (short) g;
				for(int t = 0; t < s.nt && t < XB_CAP_T && to + t < XS_CAP_T; ++t) town[to + t] = (short) g;
			}
		} else {
			for(int c = 0; c < s.nc && c < XB_CAP; ++c) {
				if(co + c < XS_CAP) {
					lc[co + c] = pre && g0 == 0 && c < XS_PRE_C ? pre->cr[c < XS_PRE_C ? c : 0] : b.xcr[(size_t) g * XB_CAP + c];
					lcR[co + c] = Rw;
					lcT[co + c] = to;
				}
			}
			for(int t = 0; t < s.nt && t < XB_CAP_T; ++t) {
				if(to + t < XS_CAP_T) {
					lt[to + t] = pre && g0 == 0 && t == 0 ? pre->ti : b.xti[(size_t) g * XB_CAP_T + t];
					ltR[to + t] = Rw;
				}
			}
		}
		wave_sync();
		if(g < G) {
			// the block's first run must have assumed its segment's binade (checked
			// after the records with allpre); its last run's sum goes to its segment
			// (integer-valued: exact in any order)
			if(!allpre) {
				const int want = co == 0 ? eH : co - 1 < XS_CAP ? lc[co - 1].x : -1;
				why |= s.ex0 != want ? XS_WHY_EX0 : 0;
			}
			if(co + s.nc <= XS_CAP) atomicAdd(&lseg[co + s.nc], s.tail);
			else why |= XS_WHY_CAP;
		}
		cob += tc;
		tob += tt;
		Rwb += tr;
	}
	const int nx = cob, ntot = tob;
	if(allpre) {
		// record q of the crossing (tie) list belongs to block cown[q] (town[q]):
		// every lane loads its records at once, then stores them
		auto owner = [&](const short *own, int q) { return (int) own[q]; };
		XsCross cv[2];
		int cg[2];
#pragma unroll
		for(int m = 0; m < 2; ++m) {   // XS_CAP = 128 crossings: two per lane
			const int q = lane + 64 * m;
			cg[m] = -1;
			if(q < nx && q < XS_CAP) {
				const int g = owner(cown, q);
				cg[m] = g;
				cv[m] = b.xcr[(size_t) g * XB_CAP + (q - bco[g])];
			}
		}
		XsTie tv[XS_CAP_T / 64];
		int tg[XS_CAP_T / 64];
#pragma unroll
		for(int m = 0; m < XS_CAP_T / 64; ++m) {
			const int q = lane + 64 * m;
			tg[m] = -1;
			if(q < ntot && q < XS_CAP_T) {
				const int g = owner(town, q);
				tg[m] = g;
				tv[m] = b.xti[(size_t) g * XB_CAP_T + (q - bto[g])];
			}
		}
#pragma unroll
		for(int m = 0; m < 2; ++m) {
			const int q = lane + 64 * m;
			if(cg[m] >= 0) {
				lc[q] = cv[m];
				lcR[q] = bRw[cg[m]];
				lcT[q] = bto[cg[m]];
			}
		}
#pragma unroll
		for(int m = 0; m < XS_CAP_T / 64; ++m) {
			const int q = lane + 64 * m;
			if(tg[m] >= 0) {
				lt[q] = tv[m];
				ltR[q] = bRw[tg[m]];
			}
		}
		wave_sync();
		for(int g = lane; g < G; g += 64) {   // the start-binade checks of the loop above
			const int co = bco[g];
			const int want = co == 0 ? eH : co - 1 < XS_CAP ? lc[co - 1].x : -1;
			why |= bex[g] != want ? XS_WHY_EX0 : 0;
		}
	}
	why |= nx > XS_CAP - 1 || ntot > XS_CAP_T ? XS_WHY_CAP : 0;
#pragma unroll
	for(int q = 0; q < XS_NWHY; ++q) why |= __any((why >> q) & 1) ? 1 << q : 0;
	*why_out = why;
	if(why) return false;
	wave_sync();
	TS(4, 7);
	// ---- per segment: its increment for an even / odd start (ties rounded to even)
	double A0[2], A1[2], cvA[2];
	int exA[2], cxA[2];
#pragma unroll
	for(int h = 0; h < 2; ++h) {
		const int s = lane + 64 * h;
		A0[h] = A1[h] = cvA[h] = 0.0;
		exA[h] = cxA[h] = 0;
		if(s <= nx) {
			double seg = lseg[s];
			int ta = 0, tz = ntot, Rc = 0;
			if(s) {
				const XsCross &p = lc[s - 1];
				exA[h] = p.x;
				ta = lcT[s - 1] + p.tb;
				Rc = lcR[s - 1];
			} else {
				exA[h] = eH;
			}
			if(s < nx) {
				const XsCross &q = lc[s];
				cvA[h] = q.v;
				cxA[h] = q.x;
				seg += q.run;
				tz = lcT[s] + q.tb;
			}
			int dn0 = 0, dn1 = 0;
			for(int g = ta; g < tz; ++g) {
				const XsTie &t = lt[g];
				int pi = t.pi;
				// a run that began in an earlier block: the parities of the last runs
				// of the blocks from the crossing's on come before it
				if(t.first) pi ^= (ltR[g] - Rc) & 1;
				dn0 += 1 - ((pi + dn0) & 1);
				dn1 += 1 - ((1 + pi + dn1) & 1);
			}
			A0[h] = seg - (double) dn0;
			A1[h] = seg - (double) dn1;
		}
	}
	TS(4, 8);
	// ---- the walk
	double S = SH;
	bool ok = (eH > 0 && eH < 0x7FF) || (SH == 0.0 && lseg[0] == 0.0);
	for(int s = 0; s <= nx; ++s) {
		const int h = s >> 6, l = s & 63;
		if(s > 0 || eH > 0) {
			const int exs = __builtin_amdgcn_readlane(h ? exA[1] : exA[0], l);
			const double a0 = readlane_d(h ? A0[1] : A0[0], l), a1 = readlane_d(h ? A1[1] : A1[0], l);
			const int ue = exs - 1075;
			ok = ok && exs > 0 && exs < 0x7FF && xs_bexp(S) == exs;
			const double T0 = ldexp(S, -ue);
			const double T = T0 + (((unsigned) __double_as_longlong(T0) & 1u) ? a1 : a0);
			ok = ok && T < 9007199254740992.0;
			S = ldexp(T, ue);
		}
		if(s < nx) {
			const double Sn = S + readlane_d(h ? cvA[1] : cvA[0], l);
			ok = ok && xs_bexp(Sn) == __builtin_amdgcn_readlane(h ? cxA[1] : cxA[0], l);
			S = Sn;
		}
	}
	TS(4, 9);
#if defined(CCG_TRACE) && !defined(CCG_DNJ_NO_TRACE)
	if(blockIdx.x == 0 && threadIdx.x == 0) {   // counts in the stamp columns 10 / 11 (printed as "us")
		const int s_ = g_trace_hi - n;
		if(s_ >= 0 && s_ < 256) {
			const unsigned long long t0 = ~g_trace[(s_ * NKT + 4) * 16 + 15];
			g_trace[(s_ * NKT + 4) * 16 + 10] = t0 + (unsigned long long) nx * 100;     // crossings
			g_trace[(s_ * NKT + 4) * 16 + 11] = t0 + (unsigned long long) ntot * 100;   // ties
		}
	}
#endif
	*out = S;
	if(!ok) *why_out = XS_WHY_WALK;
	return ok;
}

// wave 0 of a consumer (k_dnj_requeue / k_nj_pop / k_hnj_update): the new
// row sum of j and its count.  *chain: the whole block must run the serial
// chain over b.contrib (rare: a failed check of the parallel form).
__device__ void row_sum_j_wave(const TreeBufs &b, int n, bool exact, bool general, double *sd, int *nj, bool *need,
                               bool *chain) {
	const int G = (int) cdiv(n, TB);
	XsPre pre;
	if(exact) xs_prefetch(b, G, pre);
	TS(4, 5);
	fold_update_wave(b, G, exact, general, sd, nj, need);
	TS(4, 6);
	*chain = false;
	if(*need) {
		double r;
		int why = 0;
		if(xs_walk_blocks(b, G, &r, exact ? &pre : nullptr, n, &why)) {
			*sd = r;
		} else {
			*chain = true;
			if(blockIdx.x == 0 && (threadIdx.x & 63) == 0)
				for(int q = 0; q < XS_NWHY; ++q)
					if((why >> q) & 1) atomicAdd(&b.ctl->xs_why[q], 1);
		}
	}
}

// ------------------------------------------------------------------ exact row sum of j
// Exact mode (the default): the reference's serial sum of the new row of j
// (nj.c:911 / :1002), once per join by one 512-thread block between updateD
// and its consumers (k_dnj_requeue, k_nj_pop, k_hnj_update and the sharded
// engines' k_sh_pop / k_shd_requeue read ctl->xsum; every rank holds the whole
// new line j, so every rank runs it identically):
// the fixed-order fold when that is provably the serial sum (integer-like
// data), else the parallel binade-segmented form, else the chain.
#define XS_NT 512
#define XS_RB 6        // rows (of 256) per wave held in registers: one load up to n = 12288 at 512 threads
template <int UNUSED = 0>
__global__ __launch_bounds__(XS_NT) void k_exact_sum(TreeBufs b, int n, int G) {
	__shared__ double s_sd;
	__shared__ int s_nj, s_need, s_stop;
	TreeCtl *ctl = b.ctl;
	if(threadIdx.x < 64) {
		const int done = ctl->done;
		double sd = 0;
		int nj = 0;
		bool need = false;
		if(!done) fold_update_wave(b, G, true, false, &sd, &nj, &need);
		if(threadIdx.x == 0) {
			s_stop = done;
			s_sd = sd;
			s_nj = nj;
			s_need = need;
		}
	}
	__syncthreads();
	if(s_stop) return;
	double r = s_sd;
	bool chain = false;
	if(s_need && !exact_sum_w<XS_NT, XS_RB>(b.contrib, n, &r)) {
		r = serial_sum_t<XS_NT>(b.contrib, n);
		chain = true;
	}
	if(threadIdx.x == 0) {
		ctl->xsum = r;
		ctl->xnj = s_nj;
		ctl->serial_sums += s_need;
		ctl->chain_sums += chain;
	}
}

// (q, f) cells of initQ: smaller q wins, equal q -> larger flat index f
// ------------------------------------------------------------------ HNJ row minima (tree.hip, tree_shard.hip)
// (q, k) `<=` rule over ascending k: smaller q, then the later k
__device__ __forceinline__ void qk_take(double &bq, int &bk, double q, int k) {
	if(q < bq || (q == bq && k > bk)) {
		bq = q;
		bk = k;
	}
}

template <int NT>
__device__ __forceinline__ void qk_block_reduce(double &bq, int &bk, double *sq, int *sk) {
	for(int o = 32; o > 0; o >>= 1) {
		const double oq = __shfl_xor(bq, o, 64);
		const int ok = __shfl_xor(bk, o, 64);
		qk_take(bq, bk, oq, ok);
	}
	const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
	if(lane == 0) {
		sq[wid] = bq;
		sk[wid] = bk;
	}
	__syncthreads();
	if(threadIdx.x == 0) {
		for(int w = 1; w < NT / 64; ++w) qk_take(bq, bk, sq[w], sk[w]);
	}
}

// one wave: fold of G row-minimum partials (blocks in ascending k order)
__device__ __forceinline__ void qk_fold_wave(const double *pq, const int *pk, int G, double &bq, int &bk) {
	const int lane = threadIdx.x & 63;
	bq = DBL_MAX;
	bk = -1;
	for(int g = lane; g < G; g += 64) qk_take(bq, bk, pq[g], pk[g]);
	for(int o = 32; o > 0; o >>= 1) {
		const double oq = __shfl_xor(bq, o, 64);
		const int ok = __shfl_xor(bk, o, 64);
		qk_take(bq, bk, oq, ok);
	}
}

__device__ __forceinline__ void qf_wave_reduce(double &q, long long &f) {
#define S_(C, R)                                          \
	{                                                     \
		const double oq_ = dpp_d<C, R>(DBL_MAX, q);       \
		const long long of_ = dpp_l<C, R>(-2, f);         \
		if(oq_ < q || (oq_ == q && of_ > f)) {            \
			q = oq_;                                      \
			f = of_;                                      \
		}                                                 \
	}
	CCG_DPP_STEPS(S_)
#undef S_
	q = readlane_d(q, 63);
	f = readlane_l(f, 63);
}


// ------------------------------------------------------------------ host
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
		if(on)   // a previous profiled run that ended early (an error return) still holds its events
			for(int k = 0; k < 1025; ++k) hipEventDestroy(ev[k]);
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
		on = false;   // later marks (e.g. a final collective) are not timed
	}
};

