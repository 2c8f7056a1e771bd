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
	long long rows, cells, cells_top, cells_rest;
	int hj, hi, hjb, hib;  // HNJ: rows j / i of the last join whose minima are still in partials (-1: none)
};

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
	int *bmr;
	int *Spos;           // entry slot of each S row in the descending scan order
	int *cslot;          // and of each rest entry (k_dnj_find)
	double *rf;          // per rest entry: fresh (q, j) folded once by k_dnj_fold
	int *rj;             // (rows with many units)
	ccg_join *joins;
	TreeCtl *ctl;
	int maxu;
};


// the device state of one tree run (one hipMalloc), sized for n taxa
struct TreeWork {
	TreeBufs b;
	void *mem;
};
int ccg_tree_alloc(TreeWork *w, int n, hipStream_t st);

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
// otherwise *need_serial asks for serial_sum_block.  General (missing data):
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
// :1002); thread 0 runs the chain while the block stages the next chunk
static __device__ double serial_sum_block(const TreeBufs &b, int n) {
	__shared__ __attribute__((aligned(16))) double buf[8 * TB];
	__shared__ double s_sd;
	double sd = 0;
	double nxt[4];
#pragma unroll
	for(int m = 0; m < 4; ++m) {
		int kk = m * TB + threadIdx.x;
		buf[m * TB + threadIdx.x] = kk < n ? b.contrib[kk] : 0.0;
	}
	__syncthreads();
	for(int c0 = 0, p = 0; c0 < n; c0 += 4 * TB, p ^= 1) {
#pragma unroll
		for(int m = 0; m < 4; ++m) {
			int kk = c0 + 4 * TB + m * TB + threadIdx.x;
			nxt[m] = kk < n ? b.contrib[kk] : 0.0;
		}
		if(threadIdx.x == 0) {
			const double *cur = buf + p * 4 * TB;
			const int lim = n - c0 < 4 * TB ? n - c0 : 4 * TB;
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
		for(int m = 0; m < 4; ++m) buf[(p ^ 1) * 4 * TB + m * TB + threadIdx.x] = nxt[m];
		__syncthreads();
	}
	if(threadIdx.x == 0) s_sd = sd;
	__syncthreads();
	return s_sd;
}

// (q, f) cells of initQ: smaller q wins, equal q -> larger flat index f
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

