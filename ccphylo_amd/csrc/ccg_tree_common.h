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
#define XS_CAP 128                // crossings / ties listed per sum
#define XS_HEAD 64                // elements summed serially first
// a tile: NT chunks of ET consecutive elements (exact_sum_t<NT, ET>)

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

// whole block (blockDim = TB); true and *out = the serial sum, or false.
// Tiles of XS_TILE elements are staged through LDS with coalesced loads (the
// next tile's loads in flight during the current one); thread t then owns
// the chunk [t XS_ET, (t + 1) XS_ET) of the tile, chunks in element order.
// Increments are taken provisionally as RN_u(c) with ties rounded up,
// floor(c/u + 1/2); the walk takes back the ties that go down.
template <int NT, int XS_ET>
static __device__ bool exact_sum_t(const double *__restrict__ c, int n, double *out,
                                   unsigned long long *stamps = nullptr) {
	constexpr int XS_TILE = NT * XS_ET;
	__shared__ double s_tile[XS_TILE + NT];   // chunk t at t (XS_ET + 1): padded against bank conflicts
	__shared__ XsCross xe[XS_CAP];
	__shared__ XsTie te[XS_CAP];
	__shared__ double s_seg[XS_CAP + 1], s_wd[NT / 64], s_out;
	__shared__ long long s_wl[NT / 64];
	__shared__ int s_bad, s_eh;
	__shared__ double s_head;
	const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
	if(tid == 0) s_bad = 0;
	for(int s = tid; s <= XS_CAP; s += NT) s_seg[s] = 0.0;
	XS_STAMP(0);
	const int ntiles = (n + XS_TILE - 1) / XS_TILE;
	double r[XS_ET];
#pragma unroll
	for(int i = 0; i < XS_ET; ++i) {
		const int k = tid + NT * i;
		r[i] = c[k < n ? k : n - 1];
	}
	// the head: the first XS_HEAD elements summed serially (wave 0, one
	// dependent add each; most binade changes of s happen here, while s is
	// small), so the parallel part starts from an exact s_H with few crossings
	if(wid == 0) {
		const double hx = lane < n ? c[lane] : 0.0;
		double S = 0;
		for(int l = 0; l < XS_HEAD; ++l) S += readlane_d(hx, l);
		if(lane == 0) {
			s_head = S;
			s_eh = xs_bexp(S);
		}
	}
	__syncthreads();
	const double SH = s_head;
	const int eH = s_eh;
	double tileP = SH;          // approximate prefix before the tile (uniform)
	int X = 0, NTIE = 0, RP = 0;  // crossings, ties, last-run parities before the tile (uniform)
	bool bad = false;
	for(int tile = 0; tile < ntiles; ++tile) {
		const int base = tile * XS_TILE;
		__syncthreads();   // the previous tile's LDS reads are done
#pragma unroll
		for(int i = 0; i < XS_ET; ++i) {
			const int e = tid + NT * i;   // element of the tile; chunk e / XS_ET
			s_tile[e + e / XS_ET] = base + e < n && base + e >= XS_HEAD ? r[i] : 0.0;
		}
		__syncthreads();
		if(tile == 0) XS_STAMP(9);
		if(tile + 1 < ntiles) {
#pragma unroll
			for(int i = 0; i < XS_ET; ++i) {
				const int k = base + XS_TILE + tid + NT * i;
				r[i] = c[k < n ? k : n - 1];
			}
		}
		double v[XS_ET];
		double cs = 0;
#pragma unroll
		for(int m = 0; m < XS_ET; ++m) {
			v[m] = s_tile[tid * (XS_ET + 1) + m];   // elements past n are 0: no effect
			bad |= !(v[m] >= 0.0 && v[m] <= DBL_MAX);
			cs += v[m];
		}
		// approximate exclusive prefix of the chunk sums
		double x = cs;
#define S_(C, R_) x += dpp_d<C, R_>(0.0, x);
		CCG_DPP_STEPS(S_)
#undef S_
		if(lane == 63) s_wd[wid] = x;
		__syncthreads();
		double P = tileP + (x - cs);
		double tot = 0;
#pragma unroll
		for(int w = 0; w < NT / 64; ++w) {
			if(w < wid) P += s_wd[w];
			tot += s_wd[w];
		}
		tileP += tot;
		if(tile == 0) XS_STAMP(10);
		// ---- branch-free pass: crossing and tie masks, provisional increments
		const double P0 = P;
		const int ep0 = xs_bexp(P);
		bad |= P0 != 0.0 && ep0 == 0;   // subnormal running sum
		int ep = ep0;
		unsigned cm = 0, tm = 0;
		double inc[XS_ET];
		double run = 0;
#pragma unroll
		for(int m = 0; m < XS_ET; ++m) {
			const double Pn = P + v[m];
			const int en = xs_bexp(Pn);
			cm |= (unsigned) (ep != en) << m;          // (x = 0 keeps P, so a change means x > 0)
			const double t = ldexp(v[m], 1075 - ep) + 0.5;   // c / u + 1/2 (< 2^52 off crossings)
			const double fl = floor(t);
			tm |= (unsigned) (t == fl) << m;          // remainder exactly u / 2
			inc[m] = fl;
			run += fl;
			P = Pn;
			ep = en;
		}
		bad |= ep == 0x7FF;
		tm &= ~cm;
		const int nc = __popc(cm), ntl = __popc(tm);
		if(cm) {   // the last run starts after the last crossing
			const int lc = 31 - __clz(cm);
			run = 0;
#pragma unroll
			for(int m = 0; m < XS_ET; ++m) run += m > lc ? inc[m] : 0.0;
		}
		if(tile == 0) XS_STAMP(11);
		// ---- positions: crossings, ties and last-run parities before the chunk
		const long long pk = ((long long) nc << 40) | ((long long) ntl << 20) | (long long) xs_par(run);
		const long long incl = wave_incl_sum_l(pk);
		if(lane == 63) s_wl[wid] = incl;
		__syncthreads();
		long long pre = incl - pk, ttot = 0;
#pragma unroll
		for(int w = 0; w < NT / 64; ++w) {
			if(w < wid) pre += s_wl[w];
			ttot += s_wl[w];
		}
		const int cb = X + (int) (pre >> 40), tb = NTIE + (int) ((pre >> 20) & 0xFFFFF),
		          Rc = RP + (int) (pre & 0xFFFFF);
		const int tx = (int) (ttot >> 40), tt = (int) ((ttot >> 20) & 0xFFFFF);
		if(X + tx > XS_CAP - 1 || NTIE + tt > XS_CAP) {
			bad = true;   // uniform
			break;
		}
		if(tile == 0) XS_STAMP(12);
		// ---- chunks with crossings or ties (few): list them, in element order
		if(cm | tm) {
			double Pw = P0;
			int ci = 0, ti = 0;
			double rw = 0;
#pragma unroll
			for(int m = 0; m < XS_ET; ++m) {
				Pw += v[m];
				if((cm >> m) & 1u) {
					XsCross q;
					q.v = v[m];
					q.run = rw;
					q.k = base + tid * XS_ET + m;
					q.x = xs_bexp(Pw);
					q.R = Rc;
					q.tb = tb + ti;
					xe[cb + ci] = q;
					++ci;
					rw = 0;
				} else {
					if((tm >> m) & 1u) {
						XsTie q;
						q.k = base + tid * XS_ET + m;
						q.pi = (xs_par(rw) + xs_par(inc[m]) + 1) & 1;   // floor = inc - 1
						q.R = Rc;
						q.first = ci == 0;
						te[tb + ti] = q;
						++ti;
					}
					rw += inc[m];
				}
			}
		}
		if(tile == 0) XS_STAMP(13);
		// the chunk's last run: segment cb + nc (atomics on integer-valued
		// doubles below 2^53 are exact in any order; one per wave when the
		// wave's last runs share a segment)
		const int seg_last = cb + nc;
		{
			const int s0 = __builtin_amdgcn_readfirstlane(seg_last);
			if(__ballot(seg_last != s0) == 0ull) {
				const double ws = wave_sum_fixed(run);
				if(lane == 0) atomicAdd(&s_seg[s0], ws);
			} else {
				atomicAdd(&s_seg[seg_last], run);
			}
		}
		__syncthreads();
		if(tile == 0) XS_STAMP(14);
		// the binade the chunk's first run assumed must be its segment's
		bad |= ep0 != (cb == 0 ? eH : xe[cb - 1].x);
		X += tx;
		NTIE += tt;
		RP += (int) (ttot & 0xFFFFF);
	}
	XS_STAMP(3);
	if(bad) s_bad = 1;
	__syncthreads();
	XS_STAMP(5);
	if(s_bad) return false;
	const int nx = X, nt = NTIE;
	// ---- walk (wave 0).  Lane l prepares segments l and l + 64: start binade
	// and provisional run sum less the ties that round down, for either parity
	// of the start (A0 / A1), and the crossing that ends it; then the chain
	// over the segments reads them with readlane (no memory on the dependent path).
	if(wid == 0) {
		double A0[2], A1[2], cvA[2];
		int exA[2], cxA[2];
#pragma unroll
		for(int h = 0; h < 2; ++h) {
			const int s = lane + 64 * h;
			A0[h] = A1[h] = cvA[h] = 0.0;
			exA[h] = cxA[h] = 0;
			if(s <= nx) {
				const double seg = s_seg[s] + (s < nx ? xe[s].run : 0.0);
				exA[h] = s ? xe[s - 1].x : eH;
				const int R0 = s ? xe[s - 1].R : 0;
				if(s < nx) {
					cvA[h] = xe[s].v;
					cxA[h] = xe[s].x;
				}
				int dn0 = 0, dn1 = 0;
				const int ta = s ? xe[s - 1].tb : 0, tz = s < nx ? xe[s].tb : nt;
				for(int q = ta; q < tz; ++q) {
					int pi = te[q].pi;
					// a run that began in an earlier chunk: the parities of the
					// runs of the chunks from the crossing's on come before it
					if(te[q].first) pi ^= (te[q].R - R0) & 1;
					dn0 += 1 - ((pi + dn0) & 1);        // round up iff start + prefix + floor is odd
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

// the reference's serial row sum: the parallel form above, the chain when it declines


// ------------------------------------------------------------------ exact row sum of j
// Exact mode (the default): the reference's serial sum of the new row of j
// (nj.c:911 / :1002), once per join by one 512-thread block between updateD
// and its consumers (k_dnj_requeue, k_nj_pop, k_hnj_update and the sharded
// engines' k_sh_pop / k_shd_requeue read ctl->xsum; every rank holds the whole
// new line j, so every rank runs it identically):
// the fixed-order fold when that is provably the serial sum (integer-like
// data), else the parallel binade-segmented form, else the chain.
#define XS_NT 512
#define XS_ET_BIG 16   // LDS tiles of 8192 elements
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
	if(s_need && !exact_sum_t<XS_NT, XS_ET_BIG>(b.contrib, n, &r)) {
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

