// ccg_dnj_search.h -- minQpair's search kernels (dnj.c:43), shared by the
// single-GPU DNJ engine (tree.hip) and the row-sharded one (tree_shard_dnj.hip).
//
// The kernels are templated on a row policy `Rows`: rows.owns(r) says whether
// this rank holds LT row r, rows.row(r) where its cells start in the local
// buffer.  DenseRows (one GPU) owns every row at tri(r); Shard (ccg_shard.h)
// owns bands of rows dealt round-robin.  Rows a rank does not own contribute
// no rescan units, so a sharded rank rescans only its own candidates.
#pragma once
#include <stdlib.h>
#include "ccg_tree_common.h"

struct DenseRows {
	__host__ __device__ __forceinline__ bool owns(long long) const { return true; }
	__host__ __device__ __forceinline__ long long row(long long r) const { return tri(r); }
};

#define DNJ_B 128        // capacity of S, the candidate rows rescanned speculatively
#define DNJ_BANDS 64     // S: the top rows with Q < m0, then the min-Q row of each
                         // of this many bands below them (DnjGrid::top/bands)
#define DNJ_BANDS_MAX 128  // CCG_S_BANDS up to this (two bands per lane of k_dnj_plan's wave 0)
#define SEG 2048         // cells per rescan unit (TB threads x 8)
#define SEG_S 1024       // cells per rescan unit of S's rows (pruning's S phase: shorter chains, more waves)
#define SEL_RPL 8        // rows per lane per step of the S scan (<= 32)
#define SEL_STEPS 8      // steps of the S scan at most (then the listing takes over)
#define TBF 1024         // threads of k_dnj_plan (one block)
#define FIND_RPT 16      // rows per thread per step of k_dnj_plan's listing (one step up to n = 15361)
#define FIND_CHUNKS 2048  // 64-row chunks of k_dnj_plan's S-rank table (n <= 131072; else binary searches)
#define REPLAY_CAP 2048  // rest entries staged in LDS
#define JOIN_UPRE 2048   // rest-unit partials k_dnj_join prefetches into LDS
#define FOLD_BLOCKS 256  // grid of k_dnj_fold (one wave per entry, grid-stride)
#define PLAN_MAXB 256    // blocks of k_dnj_plan (one listing step of LT * FR rows each)
#define SRDY_REP 64      // copies of the scan's S-table ready tag (pollers spread over lines)
#define UHIST 64         // bins of k_dnj_plan's per-block histogram of entries by unit count (umax < UHIST)

// Grid of k_dnj_scan: min(ceil(n / scan_div), scan_max).  CCG_SCAN_DIV and
// CCG_SCAN_MAX override it (tests shrink the grid so that several grid
// waves of units run at small n).
struct DnjGrid {
	// prefold_n: every n folds each entry's units once (k_dnj_fold + k_dnj_join_pf); round 4, measured: the
	// headline's tree 6.61 -> 6.36 s (profiled), configs[1] 24.7k -> 25.0k joins/s, 4k Euclidean unchanged
	int scan_div = 4, scan_max = 2048, seg_mul = 0, prefold_n = 0;
	// below 16384 taxa the wave scan replaces the block scan while the joins list many rows: tree_run_t
	// sets small_wave from the rows listed per join over its last 1024-join window (> adapt_rows;
	// CCG_SCAN_ADAPT, 0: never; headline tree 6.23 -> 6.16 s at 1000, 6.11 at 500).  Clade SNP data (the headline) lists thousands of rows per join there,
	// Euclidean matrices a few hundred (configs[1]: 246), where the block scan is 2-3 % faster
	int small_wave = 0, adapt_rows = 500;
	int sphase_b = 512;   // CCG_SPHASE_BLOCKS
	// scan_prune 2: k_dnj_plan's helper blocks rescan S while the plan lists (CCG_PLAN_HELP; 0: S in
	// k_dnj_sphase after the plan): headline tree 5.96 -> 5.71 (128) / 5.67 s (256), profiled
	int plan_help = 256;
	int scan_cmp = 1, cmp_blocks = 1024;   // the compacted wave scan (CCG_SCAN_CMP=0: off) and its grid
	// scan_prune 2 pays while the joins list many cells: tree_run_t keeps it on (prune_on) while the last
	// 1024-join window listed more than prune_cells cells per join (CCG_PRUNE_CELLS; 0: always)
	long long prune_cells = 20000000;
	int prune_on = 1;
	// plan_qdelay: the listing waves hold their Q loads back by qdelay x 32 x 64 cycles so that wave 0's fold
	// loads go first (round 6, profiles/r06_config1_sweep.txt: 0 -> 2 gives configs[1] 23.5k -> 23.9k joins/s,
	// the headline tree 12.79k -> 12.90k; 4 and above lose at 10k)
	int s_top = 0, s_bands = -1, s_split_n = 16384, plan_qdelay = 2, scan_wave = -1, plan_multi = 1;
	int plan_regsel = 0, plan_fr = FIND_RPT;   // measured at 10k: S from registers 13.2 -> 15.4 us (Q arrives late), FR 1-8 within noise
	// tests only (CCG_TEST_WITHHOLD): bit 0, k_dnj_plan's block 0 never publishes its entry count (the
	// listing blocks' look-back must time out into an error); bit 1, it never tags the S header (the
	// helper blocks' wait must); either shortens the bounded spins so that the error comes quickly
	int test_withhold = 0;
	int join_pf = 1;   // with k_dnj_fold: k_dnj_join_pf (0: k_dnj_join; 2: its block-0 replay path always)
	// measured at the headline (configs[2], 50k, profiled tree; round 4): scan + fold per join 68.3 us with
	// k_dnj_fold, 72.4 with FoldTail, 84.2 with FoldTail + pruning (cells 2.12x -> 1.27x the reference's:
	// the S phase and the wait for its table lengthen every wave's chain more than the pruned loads save)
	int scan_fold = 0; // the fold at the scan's last arrivals (FoldTail) instead of k_dnj_fold (CCG_SCAN_FOLD=1)
	// band mode: the S rows' exact fresh minima bound the other entries, and an entry whose stale Q is not
	// below the bound at its row is one minQpair skips (dnj.c:78): 2 (default) k_dnj_sphase rescans S,
	// builds the table and keeps only the surviving entries for the compacted wave scan; 1: the S phase
	// inside the scan (with FoldTail, CCG_SCAN_FOLD=1); 0: off.  Headline tree (profiled, round 4):
	// 6.29 s off, 5.86-5.89 s with 2 while the joins list > 15-30M cells, 6.05 s with 2 throughout
	int scan_prune = 2;
	// the block lower bounds (TreeBufs::lbm, lb_unit): kept by the join and the requeue from the first join
	// of a matrix larger than lb_min_n on (CCG_SCAN_LB=0: off; CCG_LB_MIN_N), used by the compacted wave scan
	int lb = 1, lb_min_n = 16384;
	// with the bounds, the row-group scan modes (20-23: float / u16 / u8 rows) may rescan bounded row groups
	// (CCG_LB_GROUPS=1: k_dnj_scan_gc<LB>, lb_unit_g: one column-sum load per lane for the group's rows
	// needing a block) instead of one bounded row per wave.  Measured (round 6, configs[3] on round 4's
	// cdist matrix, first 40k joins, the same cells): scan 40.9 s against 17.2 s for one row per wave --
	// the bounded scan is latency-bound, and the group form has a quarter of the units at 131 VGPRs
	// (3 waves/SIMD) against 68 (7): off by default
	int lb_groups = 0;
	int scan_vblk = 1;  // with pruning: also the bound from every row above (the requeue's per-block
	                    // minima of V_k = max(q at the partner cell, Q_k)) (CCG_SCAN_VBLK=0: off)
	void load() {
		if(const char *e = getenv("CCG_JOIN_PF")) join_pf = atoi(e);
		if(const char *e = getenv("CCG_SCAN_FOLD")) scan_fold = atoi(e);
		if(const char *e = getenv("CCG_SCAN_PRUNE")) scan_prune = atoi(e);
		if(const char *e = getenv("CCG_SCAN_VBLK")) scan_vblk = atoi(e);
		if(const char *e = getenv("CCG_S_TOP")) s_top = atoi(e) > 0 ? atoi(e) : 0;
		if(const char *e = getenv("CCG_S_BANDS")) s_bands = atoi(e) >= 0 ? atoi(e) : -1;
		if(const char *e = getenv("CCG_S_SPLIT_N")) s_split_n = atoi(e);
		if(const char *e = getenv("CCG_SCAN_DIV")) scan_div = atoi(e) > 0 ? atoi(e) : 4;
		if(const char *e = getenv("CCG_SCAN_MAX")) scan_max = atoi(e) > 0 ? atoi(e) : 2048;
		if(const char *e = getenv("CCG_SEG_MUL")) seg_mul = atoi(e) > 0 ? atoi(e) : 0;
		if(const char *e = getenv("CCG_PREFOLD_N")) prefold_n = atoi(e) >= 0 ? atoi(e) : 0;
		if(const char *e = getenv("CCG_SCAN_ADAPT")) adapt_rows = atoi(e) > 0 ? atoi(e) : 0;
		if(const char *e = getenv("CCG_SPHASE_BLOCKS")) sphase_b = atoi(e) > 0 ? atoi(e) : 512;
		if(const char *e = getenv("CCG_PLAN_HELP")) plan_help = atoi(e) >= 0 && atoi(e) < 512 ? atoi(e) : 256;
		if(const char *e = getenv("CCG_SCAN_CMP")) scan_cmp = atoi(e);
		if(const char *e = getenv("CCG_PRUNE_CELLS")) prune_cells = atoll(e) > 0 ? atoll(e) : 0;
		prune_on = 1;
		if(const char *e = getenv("CCG_SCAN_CMPB")) cmp_blocks = atoi(e) > 0 ? atoi(e) : 1024;
		if(const char *e = getenv("CCG_PLAN_QDELAY")) plan_qdelay = atoi(e) >= 0 ? atoi(e) : 2;
		if(const char *e = getenv("CCG_SCAN_WAVE")) scan_wave = atoi(e);
		if(const char *e = getenv("CCG_PLAN_MULTI")) plan_multi = atoi(e);
		if(const char *e = getenv("CCG_PLAN_REGSEL")) plan_regsel = atoi(e);
		if(const char *e = getenv("CCG_PLAN_FR")) plan_fr = atoi(e) < 1 ? 1 : atoi(e) > FIND_RPT ? FIND_RPT : atoi(e);
		if(const char *e = getenv("CCG_TEST_WITHHOLD")) test_withhold = atoi(e) & 3;
		if(const char *e = getenv("CCG_SCAN_LB")) lb = atoi(e);
		if(const char *e = getenv("CCG_LB_MIN_N")) lb_min_n = atoi(e);
		if(const char *e = getenv("CCG_LB_GROUPS")) lb_groups = atoi(e);
	}
	// k_dnj_plan's last argument: the Q-load delay (low 14 bits), bits 14-15 the
	// test knob test_withhold, bit 16 turns
	// the register S selection off (on with CCG_PLAN_REGSEL=1)
	// and bits 17-20 the rows per thread per listing step less one (CCG_PLAN_FR)
	int plan_flags(bool prune = false, int helpers = 0) const {
		return (plan_qdelay & 0x3fff) | (test_withhold & 3) << 14 | (plan_regsel ? 0 : 1 << 16) | ((plan_fr - 1) & 15) << 17 | (prune ? 1 << 21 : 0) |
		       (helpers & 511) << 22;
	}
	// k_dnj_plan's grid: one listing step of (TBF - 64) FIND_RPT rows per block
	// (CCG_PLAN_MULTI=0: one block walks every step, the round-2 form)
	unsigned plan_blocks(int n) const {
		if(!plan_multi) return 1;
		const int step = (TBF - 64) * plan_fr;
		const int g = (n - 1 + step - 1) / step;
		return (unsigned) (g < 1 ? 1 : g > PLAN_MAXB ? PLAN_MAXB : g);
	}
	// rescans one unit per wave past 16384 taxa, where the units are long:
	// 16-byte row loads (k_dnj_scan_v, mode 4; the GEN form k_dnj_scan_w,
	// mode 1); one unit per block below (k_dnj_scan, mode 0).  Measured per
	// join at 50k (headline data): 88.4 (block) -> 72.0 (wave) -> 66.7 us
	// (wave, 16-byte loads) -> 65.2 us (+ nontemporal row loads and 16-byte
	// sD loads where aligned, mode 9; 8433 -> 8920 joins/s); 10k: 9.4 (block)
	// against 9.8 us (wave).  Float rows take the row-group form (mode 20,
	// k_dnj_scan_g, 4 rows per wave sharing the sD loads): configs[3]'s first
	// 30k joins rescan in 34.0 s against 47.0 s with mode 4 on the same box
	// (mode 4 41.7-47.0 s over boxes; 9: 46.0, 11: 46.8, 13: 47.0, 15: 47.5);
	// double rows gain nothing from it at 50k (joins/s: G4/UC8 8472, G4/UC4
	// 8453, G2/UC8 8656 against 8901 for mode 9; modes 20, 22, 23).
	// In the sharded engine (no row groups) modes >= 4 run k_dnj_scan_v.
	// CCG_SCAN_WAVE=0/1/4..19/20/21 forces a form.
	// past 16384 taxa: double rows (the headline) stream with the 16-byte
	// nontemporal wave scan (9); narrower rows (float -p, u16 -s, u8 -b) in row
	// groups (20), where the 8-byte sD load per cell outweighs the row bytes
	// and one sD load serves 4 rows
	int scan_mode(int n, int et = 8) const {
		return scan_wave >= 0 ? scan_wave : n > 16384 || small_wave ? (et == 8 ? 9 : 20) : 0;
	}
	// cells per rescan unit: SEG up to 8 units per row, then growing with n
	// (at most 8 SEG) so that a unit's fixed cost stays small beside its bytes
	int seg(int n) const {
		int m = seg_mul ? seg_mul : n / (8 * SEG);
		m = m < 1 ? 1 : m > 8 ? 8 : m;
		return m * SEG;
	}
	// rows with many units: fold each row's unit partials once (k_dnj_fold)
	// instead of in every block of k_dnj_join
	bool prefold(int n) const { return n > prefold_n; }
	// S: `top` rows from the top, then up to `bands` band-minimum rows.  Small
	// matrices are latency-bound: 128 top rows, no bands; beyond s_split_n the
	// bands cut the rescanned cells several-fold (tools/sim_stages.c)
	int top(int n) const {
		// (round 4: 8 top rows in band mode measured the same as 16 at the headline; band mode with pruning
		// below 16384 taxa -- CCG_S_TOP=8 CCG_S_BANDS=64 -- took its tree 5.64 -> 5.43-5.51 s profiled, engine
		// cells 1.31 -> 1.16x, but costs configs[1]'s Euclidean trees, and switching band mode per window
		// needs the requeue and the next plan to agree; not done)
		const int t = s_top ? s_top : n > s_split_n ? 16 : DNJ_B;
		return t < 1 ? 1 : t > DNJ_B ? DNJ_B : t;
	}
	int bands(int n) const {
		int b = s_bands >= 0 ? s_bands : n > s_split_n ? DNJ_BANDS : 0;
		b = b > DNJ_BANDS_MAX ? DNJ_BANDS_MAX : b;
		return top(n) + b > DNJ_B ? DNJ_B - top(n) : b;
	}
	// k_dnj_sphase's grid (one wave per S unit, grid-stride)
	unsigned sphase_blocks() const { return sphase_b; }
	unsigned scan(int n) const {
		const long long g = (n + scan_div - 1) / scan_div;
		return (unsigned) (g < scan_max ? g : scan_max);
	}
};

// (trace stamps TS / TSW / TS_ENTRY / TS_EXIT / TS_SAMP: ccg_tree_common.h)

// ------------------------------------------------------------------ helpers
// (q, j) min of LT row r over columns [c0, c1), whole block of NT threads,
// UNR cells in flight per thread (dnj.c:99-112, `<=` last-wins rule).  Column
// isub (the row moved by the previous join, not yet persisted) reads (Nm, sDm).
// Without missing entries (GEN = false) every N[k] equals the matrix size n
// (initSummaD counts n - 1 entries + 1; updateD and the pop keep that), so
// the N gathers are skipped and Nr = Nm = n is passed in.
template <int ET, bool GEN, int NT, int UNR, class Rows>
__device__ __forceinline__ void row_segment_min(const Rows &rows, const typename Elem<ET>::T *__restrict__ D, double bs,
                                                const double *__restrict__ sD, const int *__restrict__ N, int r,
                                                int c0, int c1, int Nr, double sDr, int isub, int Nm, double sDm,
                                                double &q, int &idx) {
	const typename Elem<ET>::T *row = D + rows.row(r);
	typename Elem<ET>::T v[UNR];
	int nk[UNR];
	double sk[UNR];
	// clamped (always valid) addresses: no branches between the loads, so all
	// of them are in flight before the first wait
	auto load = [&](int base, typename Elem<ET>::T (&lv)[UNR], int (&lk)[UNR], double (&ls)[UNR]) {
#pragma unroll
		for(int m = 0; m < UNR; ++m) {
			int c = base + m * NT + (int) threadIdx.x;
			c = c < c1 ? c : c1 - 1;
			lv[m] = row[c];
			lk[m] = GEN ? N[c] : Nr;
			ls[m] = sD[c];
		}
	};
	load(c0, v, nk, sk);
	for(int base = c0; base < c1; base += UNR * NT) {
		// software pipeline (segments of several UNR * NT cells, large n): the
		// next step's loads are in flight while this step's cells are compared
		typename Elem<ET>::T vn[UNR];
		int nkn[UNR];
		double skn[UNR];
		const bool more = base + UNR * NT < c1;   // uniform
		if(more) load(base + UNR * NT, vn, nkn, skn);
		// branch-free (no use of a loaded value under a condition, so the
		// compiler cannot sink a load behind the first wait)
#pragma unroll
		for(int m = 0; m < UNR; ++m) {
			const int c = base + m * NT + (int) threadIdx.x;
			const double d = Elem<ET>::get(v[m], bs);
			const int Nc = c == isub ? Nm : nk[m];
			const double sc = c == isub ? sDm : sk[m];
			const double x = qcrit(Nr, Nc, d, sDr, sc);
			const bool take = c < c1 && 0 <= d && qarg_better(x, c, q, idx);
			q = take ? x : q;
			idx = take ? c : idx;
		}
		if(more) {
#pragma unroll
			for(int m = 0; m < UNR; ++m) {
				v[m] = vn[m];
				nk[m] = nkn[m];
				sk[m] = skn[m];
			}
		}
	}
}

// fold of the (q, j) unit partials [ua, ub), 4 branch-free loads in flight
__device__ __forceinline__ void fold_units(const double *__restrict__ uq, const int *__restrict__ uj, int ua, int ub,
                                           double &q, int &idx) {
	for(int u = ua; u < ub; u += 4) {
		double oq[4];
		int oi[4];
#pragma unroll
		for(int m = 0; m < 4; ++m) {
			const int v = u + m < ub ? u + m : ub - 1;
			oq[m] = uq[v];
			oi[m] = uj[v];
		}
#pragma unroll
		for(int m = 0; m < 4; ++m) {
			if(u + m < ub && qarg_better(oq[m], oi[m], q, idx)) {
				q = oq[m];
				idx = oi[m];
			}
		}
	}
}

// block (q, idx) reduce with one barrier; the result is valid in thread 0.
// The caller separates two uses with a barrier.
__device__ __forceinline__ void qarg_block_reduce1(double &q, int &idx, double *sq, int *si) {
	qarg_wave_reduce(q, idx);
	const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
	if(lane == 0) {
		sq[wid] = q;
		si[wid] = idx;
	}
	__syncthreads();
	if(threadIdx.x == 0) {
		for(int w = 1; w < nw; ++w) {
			if(qarg_better(sq[w], si[w], q, idx)) {
				q = sq[w];
				idx = si[w];
			}
		}
	}
}

// ------------------------------------------------------------------ DNJ init
// hclust.c:56-130: per-row min with ties -> smaller D, then later j
// (rows this rank does not own are skipped: their owner writes them)
template <int ET, class Rows>
__global__ void k_init_hnj(Rows rows, const typename Elem<ET>::T *__restrict__ D, int n, double bs,
                           const double *__restrict__ sD, const int *__restrict__ N,
                           double *__restrict__ Q, int *__restrict__ P) {
	int i = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
	int lane = threadIdx.x & 63;
	if(i >= n || !rows.owns(i)) return;
	double bq = DBL_MAX, bd = DBL_MAX;
	int bj = 0;
	const typename Elem<ET>::T *row = D + rows.row(i);
	int Ni = N[i];
	double sDi = sD[i];
	for(int j = lane; j < i; j += 64) {
		double d = Elem<ET>::get(row[j], bs);
		// non-short-circuit condition and selects: ROCm 7.2's compiler dropped
		// the bj update of the tie branch of the if-form for ET = 1 (a
		// matrix of equal u8 entries then picked P = 63 for every row >= 64)
		const double q = qcrit(Ni, N[j], d, sDi, sD[j]);
		const bool take = (0 <= d) & ((q < bq) | ((q == bq) & ((d < bd) | ((d == bd) & (j > bj)))));
		bq = take ? q : bq;
		bd = take ? d : bd;
		bj = take ? j : bj;
	}
#pragma unroll
	for(int off = 32; off > 0; off >>= 1) {
		const double oq = __shfl_xor(bq, off, 64), od = __shfl_xor(bd, off, 64);
		const int oj = __shfl_xor(bj, off, 64);
		const bool take = (oq < bq) | ((oq == bq) & ((od < bd) | ((od == bd) & (oj > bj))));
		bq = take ? oq : bq;
		bd = take ? od : bd;
		bj = take ? oj : bj;
	}
	if(lane == 0) {
		Q[i] = bq;
		P[i] = bj;
	}
}

// hclust.c:353 minQ -> the first candidate row (dnj.c:997-998)
template <int UNUSED = 0>
__global__ __launch_bounds__(TB) void k_dnj_prep(TreeBufs b, int n) {
	__shared__ double sq[TB / 64];
	__shared__ int si[TB / 64];
	double q = DBL_MAX;
	int idx = 0;
	for(int i = 1 + threadIdx.x; i < n; i += blockDim.x) {
		if(qarg_better(b.Q[i], i, q, idx)) {
			q = b.Q[i];
			idx = i;
		}
	}
	qarg_block_reduce(q, idx, sq, si);
	if(threadIdx.x == 0) {
		b.ctl->cand = idx;
		b.ctl->cand_q = b.Q[idx];
		b.ctl->cand_p = b.P[idx];
	}
}

// ------------------------------------------------------------------ DNJ plan (one-phase search)
// One block of TBF threads, before any rescan of the join, so S and the rows
// below it are rescanned in ONE phase (k_dnj_scan):
//   wave 0: the previous join's updateDNJ / DNJ_popArrange fold, minPos and
//   minQpair's start (dnj.c:1026-1032, :55-60), S: the top rows with Q < m0,
//   plus band-minimum rows for large n;
//   the bound of the rows below S, from each S row k's Q criterion at its
//   stored partner column P[k] evaluated now: fresh_k is the minimum over all
//   of row k's columns, so q(k, P[k]) >= fresh_k and max(q(k, P[k]), Q_k)
//   bounds minQpair's running min below row k as max(fresh_k, Q_k) does (a
//   rescanned row leaves m <= fresh_k, a skipped one m <= Q_k; any subset of
//   S gives a looser, still valid bound).  The partner is the fresh minimum
//   in ~94% of S rows and the same rows qualify (tools/sim_bound.c, N=10k:
//   120.0 rest rows per join either way);
//   the entry list in scan order (descending rows: S, then the rows below
//   with Q < their bound, band rows of S merged in: crow / cbnd, ctl->T),
//   read by k_dnj_scan and k_dnj_join (which sees nS = 0: every entry is a
//   "rest" entry); entry e's rescan units are [e umax, (e + 1) umax).
// Rows j and i of the previous join have their Q/P in the requeue partials
// (substituted here, persisted by thread 0); the moved row i's sD/N (row n's)
// are substituted as column and persisted for the kernels after.
// The plan's helper blocks (scan_prune 2): once block 0 has published S
// (shdr tagged n), S's rows are rescanned in SEG-cell units, one wave each,
// with the moved row i's sD substituted (block 0 persists it in this very
// launch); each S row is folded at its last unit (sfq / sfj by S index), and
// the last S row builds the bound table (s_table's content, from sfq) and
// publishes it (srdy).  The listing blocks never wait for them; k_dnj_compact
// reads the table after the launch.
__device__ __forceinline__ void s_table_h(const TreeBufs &b, int n, int nS, double m0) {
	const int lane = threadIdx.x & 63;
	double v[2];
#pragma unroll
	for(int h = 0; h < 2; ++h) {
		const int t = lane + 64 * h;
		v[h] = DBL_MAX;
		if(t < nS) {
			const double f = __hip_atomic_load(b.sfq + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
			const double qt = __hip_atomic_load(b.pS_q + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
			v[h] = f > qt ? f : qt;
		}
	}
	double x0 = wave_incl_min(v[0]);
	x0 = x0 < m0 ? x0 : m0;
	const double c = readlane_d(x0, 63);
	double x1 = wave_incl_min(v[1]);
	x1 = x1 < c ? x1 : c;
	if(lane < nS) __hip_atomic_store(b.pS_bnd + lane, x0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
	if(lane + 64 < nS) __hip_atomic_store(b.pS_bnd + lane + 64, x1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
	if(b.ctl->vtag == n) {   // the requeue's V block minima: suffix minima (written by an earlier launch)
		const int G = (int) cdiv(n + 1, TB);
		double carry = DBL_MAX;
		for(int g1 = ((G - 1) / 64) * 64; g1 >= 0; g1 -= 64) {
			const int g = g1 + 63 - lane;
			double x = g < G ? b.bmv[g] : DBL_MAX;
			x = wave_incl_min(x);
			x = x < carry ? x : carry;
			if(g < G) __hip_atomic_store(b.vsuf + g, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
			carry = readlane_d(x, 63);
		}
		if(lane == 0) __hip_atomic_store(b.vsuf + G, DBL_MAX, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
	}
	asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
	if(lane < SRDY_REP)
		__hip_atomic_store(b.srdy + 32 * lane, (unsigned) n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

#ifndef LB_BB_D
#define LB_BB_D 8    // lb_unit's blocks in flight per lane, double rows
#endif
#ifndef LB_BB_N
#define LB_BB_N 8    // and narrower rows (float, u16, u8)
#endif
template <int ET>   // (below, with the scan)
__device__ __forceinline__ int lb_unit(const typename Elem<ET>::T *__restrict__ row, double bs, const TreeBufs &b, int n,
                                       int r, int c0, int c1, double sDr, double &q, int &idx, int isub = -1,
                                       double sDm = 0.0, bool ubinf = false);

template <int ET>
__device__ __forceinline__ void plan_s_helper(const typename Elem<ET>::T *__restrict__ D, double bs,
                                                        TreeBufs b, int n, int hb, int nh, bool tshort) {
	typedef typename Elem<ET>::T T;
	constexpr int UC = 8;   // (16: the plan kernel's registers spill further, 30.8 -> 33.4 us per plan at 50k)
	__shared__ int h_ok, h_nS, h_isub, h_jsub;
	__shared__ double h_m0, h_sDm;
	__shared__ int h_uo[DNJ_B + 1], h_row[DNJ_B];
	const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
	if(b.ctl->done) return;   // (block-uniform; the plan's blocks return too)
	if(tid == 0) {
		bool ok = false;
		for(int spin = 0; spin < (tshort ? 1 << 10 : 1 << 18); ++spin) {
			if(__hip_atomic_load(b.shdr + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned long long) n) {
				ok = true;
				break;
			}
			__builtin_amdgcn_s_sleep(4);
		}
		h_ok = ok;
		if(!ok) {
			// never expected (block 0 runs before its helpers): other helpers may
			// already have counted S units in (ecS, scnt) that this block's units
			// will never complete, so the bound table of this join and the
			// counters of the next would be wrong; stop the loop with an error
			// (tree_run_t) as k_dnj_plan's own look-back does
			b.ctl->final_n = -1;
			b.ctl->done = 1;
		}
		if(ok) {
			h_m0 = __longlong_as_double(
			    (long long) __hip_atomic_load(b.shdr + 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
			h_sDm = __longlong_as_double(
			    (long long) __hip_atomic_load(b.shdr + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
			const unsigned long long w = __hip_atomic_load(b.shdr + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
			h_nS = (int) (unsigned) (w & 0xffffffffu);
			h_isub = (int) (unsigned) (w >> 32);
			h_jsub = (int) (unsigned) __hip_atomic_load(b.shdr + 4, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		}
	}
	__syncthreads();
	if(!h_ok || h_nS <= 0) return;
	const int nS = h_nS, isub = h_isub, jsub = h_jsub;
	const double sDm = h_sDm;
	for(int t = tid; t <= nS; t += blockDim.x) {
		h_uo[t] = __hip_atomic_load(b.pS_uo + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		if(t < nS) h_row[t] = __hip_atomic_load(b.pS_row + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
	}
	__syncthreads();
	const int su = h_uo[nS];
	const int nwv = blockDim.x >> 6;
	for(int v = hb * nwv + wid; v < su; v += nh * nwv) {
		int lo = 0, hi = nS;
		while(hi - lo > 1) {
			const int mid = (lo + hi) >> 1;
			if(h_uo[mid] <= v) lo = mid; else hi = mid;
		}
		const int r = h_row[lo], c0 = (v - h_uo[lo]) * SEG_S;
		const int c1 = c0 + SEG_S < r ? c0 + SEG_S : r;
		const double sDr = r == isub ? sDm : b.sD[r];
		const T *row = D + tri(r);
		double q = DBL_MAX;
		int idx = 0;
		if(b.lbm) {   // under the block bounds (rows j and i: no threshold yet)
			const long long sk = lb_unit<ET>(row, bs, b, n, r, c0, c1, sDr, q, idx, isub, sDm, r == isub || r == jsub);
			if(lane == 0 && sk) {   // the cells the helpers did not load (stats; cells_help counted whole S rows)
				long long *slot = b.lbskip + (long long) (LB_SCAN + (hb * nwv + wid) % LB_HELP) * LB_SLOT;
				atomicAdd((unsigned long long *) slot, (unsigned long long) sk);
				atomicAdd((unsigned long long *) (slot + 1), (unsigned long long) sk);
			}
		} else {
			for(int base = c0; base < c1; base += 64 * UC) {
				double sk[UC];
				T vv[UC];
#pragma unroll
				for(int m = 0; m < UC; ++m) {
					const int c = base + 64 * m + lane;
					const int cc = c < c1 ? c : c1 - 1;
					sk[m] = b.sD[cc];
					vv[m] = row[cc];
				}
#pragma unroll
				for(int m = 0; m < UC; ++m) {
					const int c = base + 64 * m + lane;
					const double d = Elem<ET>::get(vv[m], bs);
					const double x = qcrit(n, n, d, sDr, c == isub ? sDm : sk[m]);
					const bool take = c < c1 && 0 <= d && qarg_better(x, c, q, idx);
					q = take ? x : q;
					idx = take ? c : idx;
				}
			}
		}
		qarg_wave_reduce(q, idx);
		// fold S row lo at its last unit; the last S row builds the table
		int s_done = 0;
		const int ua = h_uo[lo], ub = h_uo[lo + 1];
		int last = 1;
		if(ub - ua > 1) {
			if(lane == 0) {
				__hip_atomic_store(b.uq + v, q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
				__hip_atomic_store(b.uj + v, idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
				asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
				const unsigned seen = __hip_atomic_fetch_add(b.ecS + lo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
				last = (int) seen == ub - ua - 1;
				if(last) __hip_atomic_store(b.ecS + lo, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
			}
			last = __shfl(last, 0);
			if(last) {
				// the row's partials, one per lane (a top row of S has up to
				// n / SEG_S of them): one round trip, then the wave's reduce (the
				// total order of qarg_better makes the fold order free)
				for(int x = ua + lane; x < ub; x += 64) {
					const double oq = __hip_atomic_load(b.uq + x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
					const int oi = __hip_atomic_load(b.uj + x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
					if(qarg_better(oq, oi, q, idx)) {
						q = oq;
						idx = oi;
					}
				}
				qarg_wave_reduce(q, idx);
			}
		}
		if(lane == 0) {
			if(last) {
				__hip_atomic_store(b.sfq + lo, q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
				__hip_atomic_store(b.sfj + lo, idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
				asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
				const unsigned sseen = __hip_atomic_fetch_add(&b.ctl->scnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
				s_done = (int) sseen == nS - 1;
				if(s_done) __hip_atomic_store(&b.ctl->scnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
			}
		}
		if(__shfl(s_done, 0)) s_table_h(b, n, nS, h_m0);
	}
}

template <int ET, bool GEN, class Rows, bool BANDS>
__global__ __launch_bounds__(TBF) void k_dnj_plan(const typename Elem<ET>::T *__restrict__ D, double bs, TreeBufs b,
                                                  int n, int first, Rows rows, int seg, int ktop, int kbands,
                                                  int qdelay) {
	// wave 0 folds and selects S; waves 1.. (LT threads) hold the rows of the
	// listing and the speculative partner cells (their loads sit in the other
	// branch of wave 0's prologue, so the two share registers)
	constexpr int NW = TBF / 64, FR = FIND_RPT, NSP = TBF - 64, LT = TBF - 64, LW = NW - 1;
	__shared__ int sS[DNJ_B];
	__shared__ double sQS[DNJ_B], sQP[DNJ_B];   // S rows: Q, and the Q criterion at the partner cell (band rows)
	__shared__ double spq[NSP];                 // the Q criterion at the partner cell of row top - t
	__shared__ double spm[DNJ_B + 2];           // bound below S row t (prefix over S in scan order)
	__shared__ int s_mw[FR * LW], s_cnt;
	__shared__ double s_sb[LW * FR];          // band mode: the bound of slot (wave, m)'s 64 rows ...
	__shared__ __attribute__((aligned(16))) unsigned char s_sf[LW * FR];   // ... unless an S row falls among them
	__shared__ int sch[FIND_CHUNKS];
	__shared__ int s_done, s_isub, s_jsub, s_nS, s_ntop, s_smin, s_Nm;
	__shared__ double s_m0, s_Qj, s_Qi, s_sDm;
	TreeCtl *ctl = b.ctl;
	const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
	const int top = n - 1;
	// several blocks (large n): block b lists the rows of step b (LT FR rows
	// from top - b LT FR down); every block runs the prologue itself, block 0
	// persists it; entry positions follow from a decoupled look-back over the
	// lower blocks' counts (ppub, tagged with n)
	// fr (<= FR): rows per thread per listing step, from the flags (small n:
	// fewer rows per block, more blocks to pull Q in)
	const int fr = ((qdelay >> 17) & 15) + 1;
	// helper blocks (the last (qdelay >> 22) & 511 of the grid, scan_prune 2):
	// S's rescans and the bound table while the listing blocks list
	const int nhelp = (qdelay >> 22) & 511;
	if((int) blockIdx.x >= (int) gridDim.x - nhelp) {
		plan_s_helper<ET>(D, bs, b, n, (int) blockIdx.x - ((int) gridDim.x - nhelp), nhelp, (qdelay >> 14) & 3);
		return;
	}
	const int nblk = gridDim.x - nhelp, bid = blockIdx.x, bstep = bid * (LT * fr), stride = nblk * (LT * fr);
	__shared__ int s_off;
	__shared__ int s_uh[UHIST];   // this block's entries by rescan-unit count (the compacted scan's enumeration)
	TS_ENTRY(1);
	TS(1, 0);
	if(tid < UHIST) s_uh[tid] = 0;   // wave 0: before its own top-part counts; the others after the barrier
	const int lt = tid - 64;   // listing thread (waves 1..)
	// every row of the matrix sits in the listing's registers (one block, one
	// step, no bands: n <= 15361): S is selected from them after the fold, by
	// the whole block, instead of by wave 0 in dependent steps of loads
	const bool regsel = !BANDS && nblk == 1 && top <= LT * fr && !((qdelay >> 16) & 1);   // (off by default)
	// S for the scan's pruning (band mode): its rows, Q and unit prefix persisted,
	// every entry flagged (eS) and each S row's entry index recorded
	const bool prune = BANDS && ((qdelay >> 21) & 1);
	const int nhelp_ = (qdelay >> 22) & 511;
	// tests (DnjGrid::test_withhold): block 0 withholds its count (bit 14) or the
	// S header's tag (bit 15); the bounded spins are then short
	const bool wh_cnt = (qdelay >> 14) & 1, wh_hdr = (qdelay >> 15) & 1;
	const int spin_max = wh_cnt || wh_hdr ? 1 << 12 : 1 << 24;
	qdelay &= 0x3fff;
	double qv[FR];
	const int rt = top - lt;
	bool have_rt = false;
	int pr = 0, nr = n, np = n;
	double dpr = -1.0, sdr = 0.0, sdp = 0.0;
	if(wid > 0) {
		// ---- loads that do not depend on the fold: the partner cell of the
		// top LT rows (speculative: S is not known yet), and Q of the listed
		// rows in descending (m, lt) order, the bulk, held back by qdelay x 32 x
		// 64 cycles so that wave 0's fold loads are not queued behind them
		// (issue order: the partner index, then Q, then the cells that wait for
		// the index; loads return in order, so Q issued behind the dependent
		// cell loads would arrive a round trip later)
		have_rt = rt >= 1 && rows.owns(rt);
		if(have_rt) {
			pr = b.P[rt];
			sdr = b.sD[rt];
			if(GEN) nr = b.N[rt];
		}
		for(int d = 0; d < qdelay; ++d) __builtin_amdgcn_s_sleep(32);
#pragma unroll
		for(int m = 0; m < FR; ++m) {
			const int r = top - bstep - (m * LT + lt);
			const bool v = m < fr && r >= 1;
			const double x = b.Q[v ? r : 1];
			qv[m] = v ? x : DBL_MAX;
		}
		if(have_rt) {
			pr = pr >= 0 && pr < rt ? pr : 0;
			dpr = Elem<ET>::get(D[rows.row(rt) + pr], bs);
			sdp = b.sD[pr];
			if(GEN) np = b.N[pr];
		}
	} else {
		// ---- prologue: fold, minPos, m0, S
		const int done = ctl->done;
		const int i = first ? -1 : ctl->i, j = first ? -1 : ctl->j;
		const int cand0 = first ? ctl->cand : 0;
		const double cand0_q = first ? ctl->cand_q : 0.0;
		const int cand0_p = first ? ctl->cand_p : 0;
		double q[4] = {DBL_MAX, DBL_MAX, DBL_MAX, DBL_MAX}, cq1 = DBL_MAX;
		int ix[4] = {0, -1, 0, -1}, cp1 = 0;
		__builtin_amdgcn_s_setprio(3);   // wave 0's loads first: the fold is the critical path
		// the band candidates' first four requeue blocks (every block of a band
		// up to G = 256), loaded before the fold's partials so that both share
		// one round trip; with ubq the requeue also left each block minimum's
		// partner-cell q (bmqp), so no dependent load for it follows (round 5)
		const bool lbq = b.ubq != nullptr;
		double bo_q[2][4], bo_c[2][4];
		int bo_r[2][4], bo_p[2][4];
#pragma unroll
		for(int h = 0; h < 2; ++h) {
			const int k = lane + 64 * h;
			const bool act = BANDS && !first && k < kbands;
			const int G = (int) cdiv(n + 1, TB);
			const int ga = act ? k * G / kbands : 0, gz = act ? (k + 1) * G / kbands : 0;
#pragma unroll
			for(int m = 0; m < 4; ++m) {
				const int g = ga + m < gz ? ga + m : (gz > ga ? gz - 1 : 0);
				bo_q[h][m] = act ? b.bmq[g] : DBL_MAX;
				bo_r[h][m] = act ? b.bmr[g] : 0;
				bo_p[h][m] = act ? b.bmp[g] : 0;
				bo_c[h][m] = act && lbq ? b.bmqp[g] : INFINITY;
			}
		}
		if(!first) {
			const int G = (int) cdiv(n + 1, TB);   // k_dnj_requeue's grid at size n + 1
			// FU requeue blocks per lane per round trip: every load of a step is
			// issued before the first compare (the winner is unique under
			// qarg_better's total order, so the fold order is free)
			constexpr int FU = 4;
			for(int w0 = lane; w0 < G; w0 += 64 * FU) {
				double oq[FU][4], ocq[FU];
				int oi[FU][4], ocp[FU];
#pragma unroll
				for(int u = 0; u < FU; ++u) {
					const int w = w0 + 64 * u < G ? w0 + 64 * u : w0;
#pragma unroll
					for(int t = 0; t < 4; ++t) {
						oq[u][t] = b.qpart[4 * w + t];
						oi[u][t] = b.ipart[4 * w + t];
					}
					ocq[u] = b.cfq[w];
					ocp[u] = b.cfp[w];
				}
#pragma unroll
				for(int u = 0; u < FU; ++u) {
					if(w0 + 64 * u >= G) continue;
#pragma unroll
					for(int t = 0; t < 4; ++t) {
						if(qarg_better(oq[u][t], oi[u][t], q[t], ix[t])) {
							q[t] = oq[u][t];
							ix[t] = oi[u][t];
							if(t == 1) {
								cq1 = ocq[u];
								cp1 = ocp[u];
							}
						}
					}
				}
			}
		}
		// band candidates: lane l holds the min-Q row of the requeue blocks
		// [k G / kbands, (k + 1) G / kbands) of bands k = l and l + 64 (h = 0, 1)
		// with its partner, and loads that partner's cell right away
		double bcq[2] = {DBL_MAX, DBL_MAX}, bd[2] = {-1.0, -1.0}, bsr[2] = {0.0, 0.0}, bsp[2] = {0.0, 0.0};
		double bcc[2] = {INFINITY, INFINITY};   // (with ubq) the winner's partner-cell q
		int bcr[2] = {0, 0}, bcp[2] = {0, 0}, bnr[2] = {n, n}, bnp[2] = {n, n};
#pragma unroll
		for(int h = 0; h < 2; ++h) {
			const int k = lane + 64 * h;
			if(!(BANDS && !first && k < kbands)) continue;
			const int G = (int) cdiv(n + 1, TB);
			const int ga = k * G / kbands, gz = (k + 1) * G / kbands;
			for(int g0 = ga; g0 < gz; g0 += 4) {
				double oq[4], oc[4];
				int orr[4], op[4];
#pragma unroll
				for(int m = 0; m < 4; ++m) {   // 4 loads in flight per array (the first four prefetched)
					const int g = g0 + m < gz ? g0 + m : gz - 1;
					oq[m] = g0 == ga ? bo_q[h][m] : b.bmq[g];
					orr[m] = g0 == ga ? bo_r[h][m] : b.bmr[g];
					op[m] = g0 == ga ? bo_p[h][m] : b.bmp[g];
					oc[m] = g0 == ga ? bo_c[h][m] : lbq ? b.bmqp[g] : INFINITY;
				}
#pragma unroll
				for(int m = 0; m < 4; ++m) {
					if(g0 + m < gz && qarg_better(oq[m], orr[m], bcq[h], bcr[h])) {
						bcq[h] = oq[m];
						bcr[h] = orr[m];
						bcp[h] = op[m];
						bcc[h] = oc[m];
					}
				}
			}
			if(!lbq && bcr[h] >= 1 && rows.owns(bcr[h])) {
				bcp[h] = bcp[h] >= 0 && bcp[h] < bcr[h] ? bcp[h] : 0;
				bd[h] = Elem<ET>::get(D[rows.row(bcr[h]) + bcp[h]], bs);
				bsr[h] = b.sD[bcr[h]];
				bsp[h] = b.sD[bcp[h]];
				if(GEN) {
					bnr[h] = b.N[bcr[h]];
					bnp[h] = b.N[bcp[h]];
				}
			}
		}
		double topQ[SEL_RPL];
#pragma unroll
		for(int m = 0; m < SEL_RPL; ++m) {
			const int r = n - 1 - (m * 64 + lane);
			topQ[m] = r >= 1 && !regsel ? b.Q[r] : DBL_MAX;
		}
		// band mode: the requeue's per-256-row-block minimum Q (rows i and j
		// excluded) of the top blocks; the S steps skip blocks whose minimum is
		// not below m0 (no row there can qualify) and load nothing for them
		const int gtop = (n - 1) >> 8;
		const double gbq = BANDS && !first && lane <= 2 * SEL_STEPS && gtop - lane >= 0 ? b.bmq[gtop - lane] : -DBL_MAX;
		const double sDm = first ? 0.0 : b.sD[n];   // row n moves to i (matrix.c:518 semantics)
		const int Nm = first ? 0 : b.N[n];
		if(done) {
			if(lane == 0) s_done = 1;
		} else {
			
			qarg_wave_reduce4(q, ix, cq1, cp1);
			const int nn = n;
			const bool move = !first && i != nn;
			const int isub = move ? i : -1, jsub = first ? -1 : j;
			const double Qj = q[0], Qi = q[2];
			const int Pj = ix[0], Pi = ix[2];
#define QSUB(r) ((r) == jsub ? Qj : (r) == isub ? Qi : (r) == ix[1] ? cq1 : (r) == ix[3] ? q[3] : DBL_MAX)
#define PSUB(r) ((r) == jsub ? Pj : (r) == isub ? Pi : (r) == ix[1] ? cp1 : (r) == ix[3] ? i : 0)
			int cand;
			if(first) {
				cand = cand0;
			} else {
				int p = j;
				if(ix[1] >= 0 && qarg_better(q[1], ix[1], q[0], j)) p = ix[1];
				int p2 = 0;
				if(move) {
					p2 = i;
					if(ix[3] >= 0 && qarg_better(q[3], ix[3], q[2], i)) p2 = ix[3];
				}
				if(p2 == nn) {
					cand = p;
				} else if(p == nn) {
					cand = p2;
				} else {
					double Qp = QSUB(p), Qp2 = QSUB(p2);
					cand = (Qp2 < Qp || (p < p2 && Qp2 == Qp)) ? p2 : p;
				}
			}
			const double Qc = !cand ? DBL_MAX : first ? cand0_q : QSUB(cand);
			double m0 = DBL_MAX;
			if(cand && m0 != Qc) m0 = Qc;
			const int pos_i = (cand && m0 != DBL_MAX) ? cand : 0;
			const int pos_j = (cand && m0 != DBL_MAX) ? (first ? cand0_p : PSUB(cand)) : 0;
#undef QSUB
#undef PSUB
			
			// ---- S, top part: ktop rows with Q < m0 from the top, examining at
			// most SEL_STEPS steps of 64 SEL_RPL rows (any S is exact: when the
			// scan stops short, the rows below the examined ones are left to the
			// listing under its bound, which never exceeds m0)
			TS(1, 9);
			int cnt = 0, low = n;   // rows >= low examined
			// bit l: block gtop - l may hold a row with Q < m0 (its minimum, or row j / i in it)
			const int gl = gtop - lane;
			const unsigned long long live =
			    __ballot(gl >= 0 && (gbq < m0 || (jsub >= 0 && (jsub >> 8) == gl) || (isub >= 0 && (isub >> 8) == gl))) |
			    ~((2ull << (2 * SEL_STEPS)) - 1);
			for(int base = n - 1, step = 0; !regsel && base >= 1 && cnt < ktop && step < SEL_STEPS;
			    base -= 64 * SEL_RPL, ++step) {
				{   // the step's rows [lo, base] lie in blocks gtop - b0 .. gtop - b1
					const int lo = base - (64 * SEL_RPL - 1) > 1 ? base - (64 * SEL_RPL - 1) : 1;
					const int b0 = gtop - (base >> 8), b1 = gtop - (lo >> 8);
					if(!(live & (((2ull << b1) - 1) & ~((1ull << b0) - 1)))) {   // uniform
						low = lo;
						continue;
					}
				}
				if(step) {
#pragma unroll
					for(int m = 0; m < SEL_RPL; ++m) {   // all of the step's loads in flight at once
						const int r = base - (m * 64 + lane);
						topQ[m] = b.Q[r >= 1 ? r : 1];
					}
				}
#pragma unroll
				for(int m = 0; m < SEL_RPL; ++m) {
					if(cnt >= ktop) continue;   // uniform
					const int r = base - (m * 64 + lane);
					const double v = r == jsub ? Qj : r == isub ? Qi : topQ[m];
					const bool f = r >= 1 && v < m0;
					const unsigned long long bm = __ballot(f);
					const int pos = cnt + (int) __builtin_amdgcn_mbcnt_hi((unsigned) (bm >> 32),
					                                                     __builtin_amdgcn_mbcnt_lo((unsigned) bm, 0));
					if(f && pos < ktop) {
						sS[pos] = r;
						sQS[pos] = v;
					}
					cnt += __popcll(bm);
					low = base - (m * 64 + 63) > 1 ? base - (m * 64 + 63) : 1;
				}
			}
			const int ntop = cnt < ktop ? cnt : ktop;
			int nS = ntop;
			// full: below S's last row; short: below the examined rows (1: all)
			const int smin = ntop == ktop ? sS[ktop - 1] : low;
			// ---- S, band part (large n): each band's min-Q row below the top
			// part, with the Q criterion at its partner cell (rows j and i of the
			// previous join are never band candidates)
			if(BANDS && smin > 1 && kbands) {
				// descending rows: bands 127..64 (h = 1), then 63..0
				int base_pos = ntop;
#pragma unroll
				for(int h = 1; h >= 0; --h) {
					const bool f = bcr[h] >= 1 && bcr[h] < smin && bcq[h] < m0;
					const unsigned long long bm = __ballot(f);
					const int pos = base_pos + __popcll(lane == 63 ? 0ull : bm >> (lane + 1));
					if(f) {
						const bool pm = bcp[h] == isub;
						sS[pos] = bcr[h];
						sQS[pos] = bcq[h];
						// (with ubq: the requeue's value of the same cell; +inf -> DBL_MAX, no bound)
						sQP[pos] = lbq ? (bcc[h] < DBL_MAX ? bcc[h] : DBL_MAX)
						           : 0 <= bd[h] ? qcrit(GEN ? bnr[h] : n, GEN ? (pm ? Nm : bnp[h]) : n, bd[h], bsr[h],
						                                pm ? sDm : bsp[h])
						                        : DBL_MAX;
					}
					base_pos += __popcll(bm);
				}
				nS = base_pos;
			}
			wave_sync();
			
			// ---- the top part is the head of the entry list: rows, bounds, units
			const int t0 = 2 * lane, t1 = 2 * lane + 1;
			const int r0 = t0 < ntop ? sS[t0] : 0, r1 = t1 < ntop ? sS[t1] : 0;
			const bool o0 = t0 < ntop && rows.owns(r0), o1 = t1 < ntop && rows.owns(r1);
			if(t0 < ntop && bid == 0) {
				b.crow[t0] = r0;
				b.cbnd[t0] = sQS[t0];
				atomicAdd(&s_uh[dcdiv(r0, seg) < UHIST ? dcdiv(r0, seg) : UHIST - 1], 1);
			}
			if(t1 < ntop && bid == 0) {
				b.crow[t1] = r1;
				b.cbnd[t1] = sQS[t1];
				atomicAdd(&s_uh[dcdiv(r1, seg) < UHIST ? dcdiv(r1, seg) : UHIST - 1], 1);
			}
			const long long ctop = wave_sum_int((long long) (o0 ? r0 : 0) + (o1 ? r1 : 0));
			
			if(lane == 0 && bid == 0) {
				if(!first) {   // persist the fold for the kernels after
					b.Q[j] = Qj;
					b.P[j] = Pj;
					if(b.ubq) b.ubq[j] = INFINITY;   // new partners: the scan's threshold is unknown
					if(move) {
						b.Q[i] = Qi;
						b.P[i] = Pi;
						b.sD[i] = sDm;
						b.N[i] = Nm;
						if(b.ubq) b.ubq[i] = INFINITY;
					}
				}
				ctl->cand = cand;
				ctl->m0 = m0;
				ctl->pos_i = pos_i;
				ctl->pos_j = pos_j;
				ctl->nS = 0;     // k_dnj_join: every entry is in the list
				ctl->ntop = 0;
				ctl->smin = smin;
				ctl->pS = prune ? nS : 0;
				if(ctop) {
					atomicAdd((unsigned long long *) &ctl->cells, (unsigned long long) ctop);
					atomicAdd((unsigned long long *) &ctl->cells_top, (unsigned long long) ctop);
				}
			}
			if(prune && bid == 0) {
				// S in scan order (top rows, then band rows: descending), the
				// top part's entries are the list's head; its SEG-cell rescan
				// units prefixed for the scan's S phase
				const int ta = lane, tb = lane + 64;
				const int ua = ta < nS ? (int) dcdiv(sS[ta], SEG_S) : 0, ub = tb < nS ? (int) dcdiv(sS[tb], SEG_S) : 0;
				int tota, totb;
				const int pa = wave_excl_scan(ua, &tota), pb = wave_excl_scan(ub, &totb);
				// (write-through: the helper blocks read them in this launch)
				if(ta < nS) {
					__hip_atomic_store(b.pS_row + ta, sS[ta], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
					__hip_atomic_store(b.pS_q + ta, sQS[ta], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
					__hip_atomic_store(b.pS_uo + ta, pa, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
					if(ta < ntop) {
						b.pS_ent[ta] = ta;
						b.eS[ta] = 1;
					}
				}
				if(tb < nS) {
					__hip_atomic_store(b.pS_row + tb, sS[tb], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
					__hip_atomic_store(b.pS_q + tb, sQS[tb], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
					__hip_atomic_store(b.pS_uo + tb, tota + pb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
					if(tb < ntop) {
						b.pS_ent[tb] = tb;
						b.eS[tb] = 1;
					}
				}
				if(lane == 0)
					__hip_atomic_store(b.pS_uo + nS, tota + totb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
				if(nhelp_) {   // the S header, then its tag, for the helper blocks
					// (S's cells, which the helpers rescan: the plan's bytes in the roofline)
					const long long hc = wave_sum_int((long long) (ta < nS ? sS[ta] : 0) + (tb < nS ? sS[tb] : 0));
					if(lane == 0 && hc) atomicAdd((unsigned long long *) &ctl->cells_help, (unsigned long long) hc);
					asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
					if(lane == 0) {
						__hip_atomic_store(b.shdr + 0, (unsigned long long) __double_as_longlong(m0), __ATOMIC_RELAXED,
						                   __HIP_MEMORY_SCOPE_AGENT);
						__hip_atomic_store(b.shdr + 1, (unsigned long long) __double_as_longlong(sDm), __ATOMIC_RELAXED,
						                   __HIP_MEMORY_SCOPE_AGENT);
						__hip_atomic_store(b.shdr + 2, ((unsigned long long) (unsigned) isub << 32) | (unsigned) nS,
						                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
						__hip_atomic_store(b.shdr + 4, (unsigned long long) (unsigned) jsub, __ATOMIC_RELAXED,
						                   __HIP_MEMORY_SCOPE_AGENT);
						asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
						if(!wh_hdr)
							__hip_atomic_store(b.shdr + 3, (unsigned long long) n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
					}
				}
			}
			if(lane == 0) {
				s_done = 0;
				s_nS = nS;
				s_ntop = ntop;
				s_smin = smin;
				s_isub = isub;
				s_jsub = jsub;
				s_Qj = Qj;
				s_Qi = Qi;
				s_m0 = m0;
				s_Nm = Nm;
				s_sDm = sDm;
			}
			
		}
		__builtin_amdgcn_s_setprio(0);
#pragma unroll
		for(int m = 0; m < FR; ++m) qv[m] = DBL_MAX;   // wave 0 lists no rows
	}
	TSW(1, 10, 64);
	__syncthreads();
	TS(1, 1);
	if(s_done) return;
	// per (slot, wave) counts in s_mw -> exclusive prefix in scan order, the
	// total in s_cnt (wave 0; the caller syncs before and after)
	auto count_prefix = [&]() {
		constexpr int NC = FR * LW, PER = (NC + 63) / 64;
		int c[PER], sum = 0;
#pragma unroll
		for(int k = 0; k < PER; ++k) {
			const int x = lane * PER + k;
			c[k] = x < NC ? s_mw[x] : 0;
			sum += c[k];
		}
		int tot;
		int pre = wave_excl_scan(sum, &tot);
#pragma unroll
		for(int k = 0; k < PER; ++k) {
			const int x = lane * PER + k;
			if(x < NC) s_mw[x] = pre;
			pre += c[k];
		}
		if(lane == 0) s_cnt = tot;
		return tot;
	};
	if(regsel) {
		// ---- S from the registers: the first ktop rows in descending order with
		// Q < m0 (rows j and i with the fold's values), as wave 0's steps would
		// find them, every row examined (so a short S leaves nothing to list)
		const int jsub = s_jsub, isub = s_isub;
		const double m0 = s_m0;
		unsigned long long bs_[FR];
#pragma unroll
		for(int m = 0; m < FR; ++m) {
			bs_[m] = 0ull;
			if(wid > 0) {
				const int r = top - (m * LT + lt);
				qv[m] = r == jsub ? s_Qj : r == isub ? s_Qi : qv[m];
				bs_[m] = __ballot(r >= 1 && qv[m] < m0);
				if(lane == 0) s_mw[m * LW + wid - 1] = __popcll(bs_[m]);
			}
		}
		__syncthreads();
		if(wid == 0) count_prefix();
		__syncthreads();
		const int tot = s_cnt, nt = tot < ktop ? tot : ktop;
		long long ctop = 0;
#pragma unroll
		for(int m = 0; m < FR; ++m) {
			if(bs_[m] == 0ull) continue;   // uniform (always for wave 0)
			const int r = top - (m * LT + lt);
			const int pos = s_mw[m * LW + wid - 1] + (int) __builtin_amdgcn_mbcnt_hi(
			                    (unsigned) (bs_[m] >> 32), __builtin_amdgcn_mbcnt_lo((unsigned) bs_[m], 0));
			if(((bs_[m] >> lane) & 1ull) && pos < ktop) {
				sS[pos] = r;
				sQS[pos] = qv[m];
				b.crow[pos] = r;
				b.cbnd[pos] = qv[m];
				if(bid == 0) atomicAdd(&s_uh[dcdiv(r, seg) < UHIST ? dcdiv(r, seg) : UHIST - 1], 1);
				ctop += rows.owns(r) ? r : 0;
			}
		}
		ctop = wave_sum_int(ctop);
		if(lane == 0 && ctop) {
			atomicAdd((unsigned long long *) &ctl->cells, (unsigned long long) ctop);
			atomicAdd((unsigned long long *) &ctl->cells_top, (unsigned long long) ctop);
		}
		__syncthreads();
		if(tid == 0) {
			const int sm = nt == ktop ? sS[ktop - 1] : 1;
			s_nS = s_ntop = nt;
			s_smin = sm;
			ctl->smin = sm;
		}
		__syncthreads();
	}
	const int nS = s_nS, ntop = s_ntop, smin = s_smin, isub = s_isub, jsub = s_jsub;
	const double m0 = s_m0;
	// ---- the Q criterion at the partner cell of the top rows, with the fold's
	// substitutions (rows j and i have a new partner in the partials: left
	// out, which only loosens the bound)
	if(wid > 0) {
		double qp = DBL_MAX;
		if(have_rt && rt != isub && rt != jsub && 0 <= dpr) {
			const bool pm = pr == isub;
			qp = qcrit(GEN ? nr : n, GEN ? (pm ? s_Nm : np) : n, dpr, sdr, pm ? s_sDm : sdp);
		}
		spq[lt] = qp;
	}
	TSW(1, 11, 64);
	__syncthreads();
	// ---- the bound below each S row: prefix min over S in scan order of
	// max(q at the partner, Q), starting at m0 (S spans at most 2 waves)
	double U;
	{
		double v = DBL_MAX;
		if(tid < nS) {
			const int r = sS[tid];
			const double qk = tid >= ntop ? sQP[tid] : top - r < NSP ? spq[top - r] : DBL_MAX;
			const double Qk = sQS[tid];
			v = qk > Qk ? qk : Qk;
		}
		const double x = wave_incl_min(v);
		if(wid < 2 && lane == 63) spm[DNJ_B + wid] = x;
		__syncthreads();
		double c = m0;
		if(wid == 1) c = spm[DNJ_B] < c ? spm[DNJ_B] : c;
		if(tid < nS) spm[tid] = x < c ? x : c;
		__syncthreads();
		U = ntop ? spm[ntop - 1] : m0;   // every row below the top part is under it
	}
	TS(1, 2);
	// ---- S rows above row r (band mode): chunk table
	const bool bands = BANDS && nS > ntop;
	const int nch0 = smin > 1 && bands ? ((smin - 1) >> 6) + 1 : 0;
	const bool table = nch0 <= FIND_CHUNKS;
	const int nch = table ? nch0 : 0;
	for(int c = tid; c < nch; c += TBF) {
		int lo = ntop, hi = nS;
		while(lo < hi) {
			const int mid = (lo + hi) >> 1;
			if(sS[mid] >= 64 * (c + 1)) lo = mid + 1; else hi = mid;
		}
		sch[c] = lo;
	}
	if(nch) __syncthreads();
	auto s_above = [&](int r) {
		int k;
		if(table) {
			k = sch[r >> 6];
			while(k < nS && sS[k] > r) ++k;
		} else {
			int lo = ntop, hi = nS;
			while(lo < hi) {
				const int mid = (lo + hi) >> 1;
				if(sS[mid] > r) lo = mid + 1; else hi = mid;
			}
			k = lo;
		}
		return k;
	};
	// ---- the rest of the entry list, after the top part: rows [1, smin) that
	// are band rows of S or have Q < their bound, with positions and unit
	// offsets from one prefix over (step, wave) counts
	int T = ntop, listed = 0;
	long long mycells = 0;
	if(smin > 1 && top - bstep >= 1) {
		double qn[FR];   // the next step's Q, loaded while this step runs
		for(int base = top - bstep; base >= 1; base -= stride) {
			if(base != top - bstep && wid > 0) {
#pragma unroll
				for(int m = 0; m < FR; ++m) qv[m] = qn[m];
			}
			if(bands) {
				// each slot's bound with one S search per slot, not per row
				if(tid < FR * LW) {   // slot (wave w + 1, m) at w FR + m: a wave reads its flags in one 16-byte load
					const int w = tid / FR, m = tid - (tid / FR) * FR;
					// rows >= smin are S's top part (never listed; s_above's chunk
					// table covers rows < smin only): the slot's highest listable row
					const int rh0 = base - (m * LT + w * 64), rhi = rh0 < smin - 1 ? rh0 : smin - 1;
					const int t0 = rhi >= 1 ? s_above(rhi) : nS;
					s_sb[tid] = t0 ? spm[t0 - 1] : m0;
					s_sf[tid] = t0 < nS && sS[t0] >= rh0 - 63;
				}
				__syncthreads();
			}
			unsigned sfm = 0;   // bit m: slot m of this wave holds an S row
			if(bands && wid > 0) {
				const uint4 f4 = *(const uint4 *) (s_sf + (wid - 1) * FR);
				const unsigned fw[4] = {f4.x, f4.y, f4.z, f4.w};
#pragma unroll
				for(int m = 0; m < FR; ++m) sfm |= ((fw[m >> 2] >> (8 * (m & 3))) & 1u) << m;
			}
			if(base == top) TS(1, 5);
			unsigned long long bm[FR];
			unsigned sbm = 0;   // bit m: this lane's slot-m row is a band row of S
#pragma unroll
			for(int m = 0; m < FR; ++m) bm[m] = 0ull;
			const int mlim = (base - 1) / LT + 1 < fr ? (base - 1) / LT + 1 : fr;   // slots holding rows >= 1
#pragma unroll
			for(int m = 0; m < FR; ++m) {
				if(m >= mlim) continue;   // uniform; no break: the loop stays unrolled (registers, not scratch)
				const int r = wid > 0 ? base - (m * LT + lt) : 0;
				const int rhi = base - (m * LT + (wid - 1) * 64);   // the wave's rows: [rhi - 63, rhi]
				if((jsub <= rhi && jsub >= rhi - 63) || (isub <= rhi && isub >= rhi - 63))   // uniform, rare
					qv[m] = r == jsub ? s_Qj : r == isub ? s_Qi : qv[m];
				// band mode: the wave's 64 rows [rhi - 63, rhi] mostly hold no S
				// row, so one wave-uniform lookup gives every lane's bound
				// (the per-row search only where an S row falls inside)
				double bnd = U;
				bool srow = false;
				if(bands && wid > 0) {
					if((sfm >> m) & 1u) {   // uniform branch (rare)
						const int t = s_above(r);
						srow = t < nS && sS[t] == r;
						bnd = t ? spm[t - 1] : m0;
					} else {
						bnd = s_sb[(wid - 1) * FR + m];
					}
				}
				bool f = false;
				if(r >= 1 && r < smin && rows.owns(r)) f = srow || qv[m] < bnd;
				sbm |= (f && srow ? 1u : 0u) << m;
				bm[m] = __ballot(f);
				if(lane == 0 && wid > 0) s_mw[m * LW + wid - 1] = __popcll(bm[m]);
			}
			if(lane == 0 && wid > 0) {
#pragma unroll
				for(int m = 0; m < FR; ++m)
					if(m >= mlim) s_mw[m * LW + wid - 1] = 0;
			}
			// the next step's Q, issued after this step's compares (a wait for
			// them must not hold up the compares) and in flight through the
			// prefix and the writes
			if(wid > 0 && base - stride >= 1) {
#pragma unroll
				for(int m = 0; m < FR; ++m) {
					const int r = base - stride - (m * LT + lt);
					qn[m] = m < fr && r >= 1 ? b.Q[r] : DBL_MAX;
				}
			}
			TSW(1, 12, 64);
			if(base == top) TSW(1, 6, 64);
			__syncthreads();
			if(wid == 0) {
				const int tot = count_prefix();
				if(nblk > 1) {
					// publish this block's count, then the lower blocks' counts
					// (dispatched before this block, they never wait on it)
					if(lane == 0 && !(wh_cnt && bid == 0))
						__hip_atomic_store(b.ppub + bid, ((unsigned long long) n << 32) | (unsigned) tot,
						                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
					int off = 0;
					bool stuck = false;
					for(int g0 = 0; g0 < bid; g0 += 64) {
						const int g = g0 + lane;
						unsigned long long u = 0;
						bool ok = g >= bid;
						for(int spin = 0;; ++spin) {
							if(!ok) {
								u = __hip_atomic_load(b.ppub + g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
								ok = (int) (u >> 32) == n;
							}
							if(__all(ok)) break;
							if(spin > spin_max) {
								stuck = true;
								break;
							}
							__builtin_amdgcn_s_sleep(1);
						}
						off += wave_sum_int(g < bid && ok ? (int) (u & 0xffffffffu) : 0);
					}
					if(lane == 0) {
						s_off = off;
						if(stuck) {   // never expected: stop the loop and report it (tree_run_t)
							ctl->final_n = -1;
							ctl->done = 1;
						}
					}
				}
				TS(1, 13);
				if(base == top) TS(1, 7);
			}
			__syncthreads();
			if(nblk > 1 && base == top - bstep) T += s_off;
#pragma unroll
			for(int m = 0; m < FR; ++m) {
				if(bm[m] == 0ull) continue;   // uniform (always for wave 0)
				const int r = base - (m * LT + lt);
				const bool f = (bm[m] >> lane) & 1ull;
				mycells += f ? r : 0;
				{   // the unit-count histogram: this wave's 64 consecutive rows span at most two counts
					const int rh = base - (m * LT + (wid - 1) * 64), bh0 = dcdiv(rh, seg);
					const int bh = bh0 < UHIST ? bh0 : UHIST - 1;
					const int ch = __popcll(__ballot(f && dcdiv(r, seg) == bh0)), ct = __popcll(bm[m]);
					if(lane == 0) {
						atomicAdd(&s_uh[bh], ch);
						if(ct > ch) atomicAdd(&s_uh[bh0 - 1 < UHIST ? bh0 - 1 : UHIST - 1], ct - ch);
					}
				}
				if(f) {
					const int pos = T + s_mw[m * LW + wid - 1] +
					                (int) __builtin_amdgcn_mbcnt_hi((unsigned) (bm[m] >> 32),
					                                                __builtin_amdgcn_mbcnt_lo((unsigned) bm[m], 0));
					b.crow[pos] = r;
					b.cbnd[pos] = qv[m];
					if(prune) {
						const bool isS = (sbm >> m) & 1u;
						b.eS[pos] = isS;
						if(isS) b.pS_ent[s_above(r)] = pos;
					}
				}
			}
			T += s_cnt;
			listed += s_cnt;
			if(base == top) TSW(1, 8, 64);
			if(base - stride < 1) break;
			__syncthreads();   // s_mw is reused by the next step
		}
	}
	// (nothing to list: smin <= 1.  Every block took the same branch -- smin
	// comes from the prologue every block runs on identical inputs, and
	// plan_blocks keeps top - bstep >= 1 for every block -- so every block's
	// count is 0 and the last block's T = ntop needs no look-back)
	TS(1, 3);
	mycells = wave_sum_int(mycells);
	if(lane == 0 && mycells) {
		atomicAdd((unsigned long long *) &ctl->cells, (unsigned long long) mycells);
		atomicAdd((unsigned long long *) &ctl->cells_rest, (unsigned long long) mycells);
	}
	__syncthreads();
	if(tid < UHIST) b.uhist[bid * UHIST + tid] = s_uh[tid];
	if(tid == 0) {
		if(bid == 0) ctl->pblk = nblk;
		if(bid == nblk - 1) ctl->T = T;   // every entry up to the last block's
		// the rows this block listed (block 0 also the top part of S)
		atomicAdd((unsigned long long *) &ctl->rows, (unsigned long long) (listed + (bid == 0 ? ntop : 0)));   // no read: nothing waits
	}
	TS(1, 4);
	TS_EXIT(1);
}

// ------------------------------------------------------------------ DNJ scan
// Rescans of the rows listed by k_dnj_plan, in seg-cell units spread over the
// whole grid.  Entry e owns the fixed unit range [e umax, (e + 1) umax) (umax
// = dnj_umax(n, seg), the units of the longest row); a row of r cells uses
// the first dcdiv(r, seg) of them, so no prefix over the entries is needed
// anywhere (the plan lists rows only).  Tail: work every block does first
// (begin) and the store of each unit's partial (unit, thread 0), for the
// sharded engine's records.
__host__ __device__ __forceinline__ int dnj_umax(int n, int seg) { return n > 2 ? (n - 2) / seg + 1 : 1; }

struct NoTail {
	__device__ __forceinline__ void begin(const TreeBufs &, int) const {}
	__device__ __forceinline__ void unit(const TreeBufs &b, int, int u, int, int, int, double q, int j) const {
		b.cq[u] = q;
		b.cj[u] = j;
	}
};
// k_dnj_fold's work done by the scan itself (no kernel boundary, no extra
// pass over the partials): a unit's wave stores its partial and counts itself
// in per entry; the entry's last unit folds the entry (rf, rj), counts the
// entry in per 64-entry chunk, and the chunk's last entry writes the chunk
// summary k_dnj_join_pf replays from.  Partials are stored write-through and
// drained (s_waitcnt) before the relaxed count, read back with agent-scope
// loads (the pattern of the sharded engine's RecTail); each last arriver
// resets its counter, so they are zero between joins.
struct FoldTail {
	__device__ __forceinline__ void begin(const TreeBufs &, int) const {}
};

template <class Tail>
__device__ __forceinline__ void tail_unit(const Tail &t, const TreeBufs &b, int n, int u, int ua, int ub, int r,
                                          double q, int j, int e, int T, bool sent = false) {
	(void) e;
	(void) T;
	(void) sent;
	if((threadIdx.x & 63) == 0) t.unit(b, n, u, ua, ub, r, q, j);
}

// the scan's S phase is complete (every S entry folded): the bound table, by
// one wave.  Row pS_row[t] leaves minQpair's running min at most
// max(fresh, Q) whether or not the reference rescans it (a rescanned row
// lowers it to <= fresh, a skipped one had it <= Q), so below S row t the
// running min is at most pS_bnd[t] = min(m0, min over S rows t' <= t of
// max(fresh_t', Q_t')); published with sready = n
__device__ __forceinline__ void s_table(const TreeBufs &b, int n) {
	const int lane = threadIdx.x & 63, nS = b.ctl->pS;
	const double m0 = b.ctl->m0;
	double v[2];
#pragma unroll
	for(int h = 0; h < 2; ++h) {
		const int t = lane + 64 * h;
		v[h] = DBL_MAX;
		if(t < nS) {
			const double f = __hip_atomic_load(b.rf + b.pS_ent[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
			const double qt = b.pS_q[t];
			v[h] = f > qt ? f : qt;
		}
	}
	double x0 = wave_incl_min(v[0]);
	x0 = x0 < m0 ? x0 : m0;
	const double c = readlane_d(x0, 63);
	double x1 = wave_incl_min(v[1]);
	x1 = x1 < c ? x1 : c;
	if(lane < nS) __hip_atomic_store(b.pS_bnd + lane, x0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
	if(lane + 64 < nS) __hip_atomic_store(b.pS_bnd + lane + 64, x1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
	// the requeue's V block minima (when they serve this join): suffix minima
	// over the blocks, vsuf[g] = min over rows >= 256 g (rows of the
	// requeue at size n + 1; row n is gone, its V never counted)
	if(b.ctl->vtag == n) {
		const int G = (int) cdiv(n + 1, TB);
		double carry = DBL_MAX;
		for(int g1 = ((G - 1) / 64) * 64; g1 >= 0; g1 -= 64) {   // 64 blocks per step, from the top
			const int g = g1 + 63 - lane;   // lane 0 the highest block of the step
			double x = g < G ? b.bmv[g] : DBL_MAX;
			x = wave_incl_min(x);   // lanes 0..l: blocks g1 + 63 - l .. g1 + 63
			x = x < carry ? x : carry;
			if(g < G) __hip_atomic_store(b.vsuf + g, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
			carry = readlane_d(x, 63);
		}
		if(lane == 0) __hip_atomic_store(b.vsuf + G, DBL_MAX, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
	}
	asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
	if(lane == 0) __hip_atomic_store(&b.ctl->scnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
	// the ready tag in SRDY_REP lines: thousands of waiting waves polling ONE
	// line cut the chip's bandwidth (MI355X_MICROARCH.md, polling-cost)
	if(lane < SRDY_REP)
		__hip_atomic_store(b.srdy + 32 * lane, (unsigned) n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// the S bound table of this join is published (bounded wait; false: never
// expected, the units then run unpruned, still exact).  ONE lane per block
// polls (its block's copy of the tag); the block's other waves read the
// table after a barrier this lane joins.
__device__ __forceinline__ bool s_table_wait(const TreeBufs &b, int n) {
	const unsigned *f = b.srdy + 32 * (blockIdx.x % SRDY_REP);
	for(int spin = 0; spin < (1 << 18); ++spin) {
		if(__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned) n) return true;
		__builtin_amdgcn_s_sleep(4);
	}
	return false;
}

// The S bound table in a wave's registers (lanes t and t + 64), and the
// bound below row r: the entry at the number of S rows above r
struct SBound {
	int ra, rb;
	double ba, bb, m0;
	int nS, G;
	bool ok, vb;
	const double *vsuf;
	// ready: s_table_wait's answer for this block (after a barrier)
	__device__ __forceinline__ bool load(const TreeBufs &b, int n, bool ready) {
		const int lane = threadIdx.x & 63;
		nS = b.ctl->pS;
		m0 = b.ctl->m0;
		ok = ready && nS > 0;
		if(!ok) return false;
		vb = b.ctl->vtag == n;
		G = (int) cdiv(n + 1, TB);
		vsuf = b.vsuf;
		ra = lane < nS ? b.pS_row[lane] : -1;
		rb = lane + 64 < nS ? b.pS_row[lane + 64] : -1;
		ba = lane < nS ? __hip_atomic_load(b.pS_bnd + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : m0;
		bb = lane + 64 < nS ? __hip_atomic_load(b.pS_bnd + lane + 64, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : m0;
		return true;
	}
	__device__ __forceinline__ double at(int r) const {
		const int t = __popcll(__ballot(ra > r)) + __popcll(__ballot(rb > r));
		const double xa = __shfl(ba, t - 1 < 63 ? (t - 1 < 0 ? 0 : t - 1) : 63);
		const double xb = __shfl(bb, t - 65 < 0 ? 0 : t - 65);
		double x = t == 0 ? m0 : t <= 64 ? xa : xb;
		if(vb) {   // every row of the blocks above r's
			const int g = (r >> 8) + 1;
			const double v = __hip_atomic_load(vsuf + (g < G ? g : G), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
			x = v < x ? v : x;
		}
		return x;
	}
};

// all lanes of the wave, with the wave's (q, j) of unit u of entry e, whose
// partials are pq / pj [ua, ub); sent: entry e is an S row of the scan's S
// phase (its partials then live in uq / uj, indexed by the S unit)
// CHUNKS = false (k_dnj_sphase): the entry is folded and counted into S only;
// k_dnj_fold summarises the chunks after the scan
template <bool CHUNKS = true>
__device__ __forceinline__ void fold_arrive(const TreeBufs &b, int n, double *pq, int *pj, int u, int ua, int ub,
                                            double q, int j, int e, int T, bool sent) {
	const int lane = threadIdx.x & 63;
	int chunk_done = 0, s_done = 0;
	if(lane == 0) {
		bool last = true;
		if(ub - ua > 1) {
			__hip_atomic_store(pq + u, q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
			__hip_atomic_store(pj + u, j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
			asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
			const unsigned seen = __hip_atomic_fetch_add(b.ecnt + e, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
			last = (int) seen == ub - ua - 1;
			if(last) {
				__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
				for(int x0 = ua; x0 < ub; x0 += 4) {   // 4 partials' loads in flight
					double oq[4];
					int oi[4];
#pragma unroll
					for(int m = 0; m < 4; ++m) {
						const int x = x0 + m < ub ? x0 + m : ub - 1;
						oq[m] = __hip_atomic_load(pq + x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
						oi[m] = __hip_atomic_load(pj + x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
					}
#pragma unroll
					for(int m = 0; m < 4; ++m) {
						if(x0 + m < ub && qarg_better(oq[m], oi[m], q, j)) {
							q = oq[m];
							j = oi[m];
						}
					}
				}
				__hip_atomic_store(b.ecnt + e, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
			}
		}
		if(last) {
			__hip_atomic_store(b.rf + e, q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
			__hip_atomic_store(b.rj + e, j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
			asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
			if(CHUNKS) {
				const int c = e >> 6, ce = T - (c << 6) < 64 ? T - (c << 6) : 64;
				const unsigned seen = __hip_atomic_fetch_add(b.ccnt + c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
				if((int) seen == ce - 1) {
					chunk_done = 1;
					__hip_atomic_store(b.ccnt + c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
				}
			}
			if(sent) {
				const unsigned sseen = __hip_atomic_fetch_add(&b.ctl->scnt, 1u, __ATOMIC_RELAXED,
				                                              __HIP_MEMORY_SCOPE_AGENT);
				s_done = (int) sseen == b.ctl->pS - 1;
			}
		}
	}
	if(__shfl(s_done, 0)) {
		__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
		s_table(b, n);
	}
	if(!CHUNKS || !__shfl(chunk_done, 0)) return;
	__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
	// the chunk summary, as k_dnj_fold leaves it
	const int c = e >> 6, e2 = (c << 6) + lane;
	const bool valid = e2 < T;
	const int rr = valid ? b.crow[e2] : 0;
	const double bnd = valid ? b.cbnd[e2] : 0.0;
	const double f = valid ? __hip_atomic_load(b.rf + e2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : DBL_MAX;
	const int fj = valid ? __hip_atomic_load(b.rj + e2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
	const double mq = readlane_d(wave_incl_min(f), 63);
	const unsigned long long hm = __ballot(valid && f == mq);
	const unsigned long long bm = __ballot(valid && !(f >= bnd));
	const int first = hm ? __ffsll((long long) hm) - 1 : 0;
	const int fr = __shfl(rr, first), fjj = __shfl(fj, first);
	if(lane == 0) {
		b.chg[c] = mq;
		b.chr[c] = fr;
		b.chj[c] = fjj;
		b.chb[c] = bm != 0ull;
	}
}

__device__ __forceinline__ void tail_unit(const FoldTail &, const TreeBufs &b, int n, int u, int ua, int ub, int r,
                                          double q, int j, int e, int T, bool sent = false) {
	(void) r;
	fold_arrive(b, n, b.cq, b.cj, u, ua, ub, q, j, e, T, sent);
}

template <int ET, bool GEN, class Rows, class Tail = NoTail>
__global__ __launch_bounds__(TB) void k_dnj_scan(const typename Elem<ET>::T *__restrict__ D, double bs, TreeBufs b,
                                                 int n, Rows rows, int seg, Tail tail = Tail()) {
	__shared__ int erow[REPLAY_CAP];
	__shared__ double sq[TB / 64];
	__shared__ int si[TB / 64];
	TreeCtl *ctl = b.ctl;
	const int tid = threadIdx.x;
	TS_ENTRY(2);
	TS(2, 0);
	TS_SAMP(0);
	// speculative first TB entries, then the rest once T is known
	const int r0 = b.crow[tid];
	const int done = ctl->done, T = ctl->T;
	if(done) return;
	tail.begin(b, n);
	if(T == 0) return;
	const int umax = dnj_umax(n, seg), nunits = T * umax;
	// blocks beyond the unit count leave before staging the table
	if((int) blockIdx.x >= nunits) return;
	// the entry rows in LDS when they fit, else read from HBM (L2-resident)
	const bool lds = T <= REPLAY_CAP;
	if(lds) {
		if(tid < T) erow[tid] = r0;
		for(int e = TB + tid; e < T; e += TB) erow[e] = b.crow[e];
	}
	__syncthreads();
	TS(2, 1);
	TS_SAMP(1);
	for(int u = blockIdx.x; u < nunits; u += gridDim.x) {
		const int e = u / umax, ua = e * umax;
		const int r = lds ? erow[e] : b.crow[e];
		const int c0 = (u - ua) * seg;
		if(c0 >= r || !rows.owns(r)) continue;   // past the row's end, or another rank's S row (uniform)
		const int c1 = c0 + seg < r ? c0 + seg : r;
		const int Nr = GEN ? b.N[r] : n;
		double qq = DBL_MAX;
		int idx = 0;
		row_segment_min<ET, GEN, TB, SEG / TB / 2>(rows, D, bs, b.sD, b.N, r, c0, c1, Nr, b.sD[r], -1, 0, 0.0, qq, idx);
		qarg_block_reduce1(qq, idx, sq, si);
		if(tid == 0) tail.unit(b, n, u, ua, ua + dcdiv(r, seg), r, qq, idx);
		if(u + (int) gridDim.x < nunits) __syncthreads();
	}
	TS(2, 2);
	TS_SAMP(2);
	TS_EXIT(2);
}

// The same rescans with one WAVE per unit (CCG_SCAN_WAVE=1): no block
// reduce or barrier per unit, and a wave's next unit starts loading while
// the current one reduces (the units of a wave are independent).  Lane l
// takes the unit's columns c0 + l, c0 + l + 64, ...; UW loads of the row
// (and of sD) in flight per lane.
template <int ET, bool GEN, class Rows, class Tail = NoTail, int SCAN_UW = 8>
__global__ __launch_bounds__(TB) void k_dnj_scan_w(const typename Elem<ET>::T *__restrict__ D, double bs, TreeBufs b,
                                                   int n, Rows rows, int seg, Tail tail = Tail()) {
	__shared__ int erow[REPLAY_CAP];
	TreeCtl *ctl = b.ctl;
	const int tid = threadIdx.x, lane = tid & 63;
	const int r0 = b.crow[tid];
	const int done = ctl->done, T = ctl->T;
	if(done) return;
	tail.begin(b, n);
	if(T == 0) return;
	const int umax = dnj_umax(n, seg), nunits = T * umax;
	if((int) blockIdx.x * (TB / 64) >= nunits) return;
	const bool lds = T <= REPLAY_CAP;
	if(lds) {
		if(tid < T) erow[tid] = r0;
		for(int e = TB + tid; e < T; e += TB) erow[e] = b.crow[e];
	}
	__syncthreads();
	const int gw = blockIdx.x * (TB / 64) + (tid >> 6), nw = gridDim.x * (TB / 64);
	for(int u = gw; u < nunits; u += nw) {
		const int e = u / umax, ua = e * umax;
		const int r = lds ? erow[e] : b.crow[e];
		const int c0 = (u - ua) * seg;
		if(c0 >= r || !rows.owns(r)) continue;   // wave-uniform
		const int c1 = c0 + seg < r ? c0 + seg : r;
		const int Nr = GEN ? b.N[r] : n;
		const double sDr = b.sD[r];
		const typename Elem<ET>::T *row = D + rows.row(r);
		double q = DBL_MAX;
		int idx = 0;
		for(int base = c0; base < c1; base += 64 * SCAN_UW) {
			typename Elem<ET>::T v[SCAN_UW];
			double sk[SCAN_UW];
			int nk[SCAN_UW];
#pragma unroll
			for(int m = 0; m < SCAN_UW; ++m) {
				int c = base + 64 * m + lane;
				c = c < c1 ? c : c1 - 1;
				v[m] = row[c];
				sk[m] = b.sD[c];
				nk[m] = GEN ? b.N[c] : Nr;
			}
#pragma unroll
			for(int m = 0; m < SCAN_UW; ++m) {
				const int c = base + 64 * m + lane;
				const double d = Elem<ET>::get(v[m], bs);
				const double x = qcrit(Nr, nk[m], d, sDr, sk[m]);
				const bool take = c < c1 && 0 <= d && qarg_better(x, c, q, idx);
				q = take ? x : q;
				idx = take ? c : idx;
			}
		}
		qarg_wave_reduce(q, idx);
		tail_unit(tail, b, n, u, ua, ua + dcdiv(r, seg), r, q, idx, e, T);
	}
}

// k_dnj_scan_w with 16-byte row loads (no missing entries): a lane reads
// VEC = 16 / sizeof(element) consecutive cells per load (4 floats, 2 doubles),
// so a float row streams at 1 KB per wave load instead of 256 B; the unit's
// unaligned head and its tail (fewer than VEC cells each) are scalar.  sD is
// gathered per cell.  UV vector loads in flight per lane (about 16 cells).
// MODE (measurement variants, CCG_SCAN_WAVE = 4 + MODE): bit 0 streams the
// row with nontemporal loads (read once; sD keeps the caches), bit 1
// software-pipelines the unit: the next UV loads are issued before the
// current ones are compared (half UV, two register sets), bit 2 loads sD
// 16 bytes at a time where the unit's aligned start is even (sD + ca 16-byte
// aligned; uniform per unit), bit 3 doubles the loads in flight per lane.
// CMP (single engine, NoTail): the real units enumerated densely from the
// plan's histogram of entries by unit count, slot-major (slot k: the E_k
// entries with more than k units, a prefix of the descending list), and dealt
// round-robin over a grid that is resident at once, so every wave gets the
// same number of units to within one (grid-stride over T umax slots left
// waves with 1 to 4+ units and a second round of blocks).
// One rescan unit, columns [c0, c1) of row r (c0 a multiple of LBW), under
// the block lower bounds (TreeBufs::lbm / msd): the threshold is the Q
// criterion at the row's partner cell P[r] in this join's state (ubq, left by
// the previous requeue) -- a cell of row r, so >= the row's fresh minimum
// f_r; +inf where unknown -- and a 64-column block whose bound
//     lb = ((n - 2) * m_d - sD_r) - M_sD    (qcrit's operation order)
// exceeds it holds no cell with q <= f_r (rounding is monotone, m_d <= every
// cell, M_sD >= every column's sD), so neither the minimum nor a tie the
// index rule could pick: it is skipped.  The other blocks are rescanned one
// cell per lane, BB blocks in flight.  Returns the cells skipped.
// (k_dnj_plan's helper blocks run while block 0 persists row i's sD and the
// thresholds of rows j and i: isub / sDm substitute the column, ubinf the
// threshold)
// a unit spans at most DnjGrid::seg's cap of 8 SEG cells (or SEG_S): lb_unit's
// four 64-lane bound loads must cover all of its blocks
static_assert(8 * SEG <= 4 * 64 * LBW && SEG_S <= 4 * 64 * LBW, "lb_unit loads at most 256 block bounds per unit");
template <int ET>
__device__ __forceinline__ int lb_unit(const typename Elem<ET>::T *__restrict__ row, double bs, const TreeBufs &b, int n,
                                       int r, int c0, int c1, double sDr, double &q, int &idx, int isub,
                                       double sDm, bool ubinf) {
	typedef typename Elem<ET>::T T;
	constexpr int BB = ET == 8 ? LB_BB_D : LB_BB_N;   // blocks in flight per lane
	const int lane = threadIdx.x & 63;
	const int bl0 = c0 / LBW, nbk = (c1 - c0 + LBW - 1) / LBW;   // <= seg / 64 <= 256 blocks
	// the unit's bounds (one or more per lane), loaded with the threshold
	const double ub = ubinf ? INFINITY : b.ubq[r];
	unsigned lbb[4];
	double msb[4];
	const unsigned *line = lb_line(b, r);
#pragma unroll
	for(int h = 0; h < 4; ++h) {
		const int t = lane + 64 * h;
		lbb[h] = t < nbk ? line[bl0 + t] : 0u;
		msb[h] = t < nbk ? b.msd[bl0 + t] : 0.0;
	}
	unsigned long long need[4];
#pragma unroll
	for(int h = 0; h < 4; ++h) {
		const int t = lane + 64 * h;
		const double lb = qcrit(n, n, (double) __uint_as_float(lbb[h]), sDr, msb[h]);
		need[h] = __ballot(t < nbk && !(lb > ub));
	}
	int loaded = 0;
	// the needed blocks, BB at a time (wave-uniform walk of the ballot masks)
	int h = 0;
	while(true) {
		int blk[BB], nb = 0;
		while(nb < BB && h < 4) {
			if(!need[h]) {
				++h;
				continue;
			}
			const int bit = __ffsll((long long) need[h]) - 1;
			need[h] &= need[h] - 1;
			blk[nb++] = bl0 + 64 * h + bit;
		}
		if(!nb) break;
		T v[BB];
		double sk[BB];
#pragma unroll
		for(int m = 0; m < BB; ++m) {
			int c = (m < nb ? blk[m] : blk[0]) * LBW + lane;
			c = c < c1 ? c : c1 - 1;
			v[m] = row[c];
			sk[m] = b.sD[c];
		}
#pragma unroll
		for(int m = 0; m < BB; ++m) {
			const int c = (m < nb ? blk[m] : blk[0]) * LBW + lane;
			const double d = Elem<ET>::get(v[m], bs);
			const double x = qcrit(n, n, d, sDr, c == isub ? sDm : sk[m]);
			if(m < nb && c < c1 && 0 <= d && qarg_better(x, c, q, idx)) {
				q = x;
				idx = c;
			}
		}
		for(int m = 0; m < nb; ++m) loaded += (blk[m] + 1) * LBW < c1 ? LBW : c1 - blk[m] * LBW;
	}
	return (c1 - c0) - loaded;
}

// lb_unit over a row group: the same column range [c0, c1_k)
// of G rows, each row's 64-column blocks tested against its own threshold
// exactly as lb_unit does, and the union of the rows' needed blocks walked BB
// at a time: one 8-byte column-sum load per lane serves every row of the
// group that needs the block, and a row loads its cells only in the blocks it
// needs itself.  So each row's fresh minimum (and the cells it counts as
// loaded) equals lb_unit's for that row, while the column sums cost 8 / (rows
// needing the block) bytes per cell instead of 8.  Returns the cells skipped
// over the group's active rows.
template <int ET, int G>
__device__ __forceinline__ long long lb_unit_g(const typename Elem<ET>::T *const (&row)[G], double bs, const TreeBufs &b,
                                               int n, const int (&r)[G], const bool (&act)[G], int c0,
                                               const int (&c1)[G], int cmax, const double (&sDr)[G], double (&q)[G],
                                               int (&idx)[G]) {
	typedef typename Elem<ET>::T T;
	constexpr int BB = ET == 8 ? LB_BB_D : LB_BB_N;
	const int lane = threadIdx.x & 63;
	const int bl0 = c0 / LBW, nbkm = (cmax - c0 + LBW - 1) / LBW;   // <= seg / 64 <= 256 blocks
	double msb[4];
#pragma unroll
	for(int h = 0; h < 4; ++h) {
		const int t = lane + 64 * h;
		msb[h] = t < nbkm ? b.msd[bl0 + t] : 0.0;
	}
	unsigned long long need[G][4], any[4] = {0, 0, 0, 0};
#pragma unroll
	for(int k = 0; k < G; ++k) {
		const int nbk = act[k] ? (c1[k] - c0 + LBW - 1) / LBW : 0;
		const double ub = act[k] ? b.ubq[r[k]] : 0.0;
		const unsigned *line = lb_line(b, act[k] ? r[k] : 1);
#pragma unroll
		for(int h = 0; h < 4; ++h) {
			const int t = lane + 64 * h;
			const unsigned lbv = t < nbk ? line[bl0 + t] : 0u;
			const double lb = qcrit(n, n, (double) __uint_as_float(lbv), sDr[k], msb[h]);
			need[k][h] = __ballot(t < nbk && !(lb > ub));
			any[h] |= need[k][h];
		}
	}
	long long loaded = 0;
	int h = 0;
	while(true) {
		int blk[BB], nb = 0;
		while(nb < BB && h < 4) {
			if(!any[h]) {
				++h;
				continue;
			}
			const int bit = __ffsll((long long) any[h]) - 1;
			any[h] &= any[h] - 1;
			blk[nb++] = 64 * h + bit;   // relative to bl0
		}
		if(!nb) break;
		double sk[BB];
		T v[G][BB];
#pragma unroll
		for(int m = 0; m < BB; ++m) {
			const int t = m < nb ? blk[m] : blk[0];
			int c = (bl0 + t) * LBW + lane;
			sk[m] = b.sD[c < cmax ? c : cmax - 1];
#pragma unroll
			for(int k = 0; k < G; ++k) {
				v[k][m] = 0;
				if((need[k][t >> 6] >> (t & 63)) & 1)   // (uniform) row k needs this block
					v[k][m] = row[k][c < c1[k] ? c : c1[k] - 1];
			}
		}
#pragma unroll
		for(int m = 0; m < BB; ++m) {
			const int t = m < nb ? blk[m] : blk[0];
			const int c = (bl0 + t) * LBW + lane;
#pragma unroll
			for(int k = 0; k < G; ++k) {
				if(m >= nb || !((need[k][t >> 6] >> (t & 63)) & 1)) continue;   // uniform
				const double d = Elem<ET>::get(v[k][m], bs);
				const double x = qcrit(n, n, d, sDr[k], sk[m]);
				if(c < c1[k] && 0 <= d && qarg_better(x, c, q[k], idx[k])) {
					q[k] = x;
					idx[k] = c;
				}
			}
		}
		for(int m = 0; m < nb; ++m) {
			const int c = (bl0 + blk[m]) * LBW;
#pragma unroll
			for(int k = 0; k < G; ++k)
				if((need[k][blk[m] >> 6] >> (blk[m] & 63)) & 1) loaded += c + LBW < c1[k] ? LBW : c1[k] - c;
		}
	}
	long long span = 0;
#pragma unroll
	for(int k = 0; k < G; ++k) span += act[k] ? c1[k] - c0 : 0;
	return span - loaded;
}

template <int ET, class Rows, class Tail = NoTail, int MODE = 0, int PRUNE = 0, bool CMP = false, bool LB = false>
__global__ __launch_bounds__(TB) void k_dnj_scan_v(const typename Elem<ET>::T *__restrict__ D, double bs, TreeBufs b,
                                                   int n, Rows rows, int seg, Tail tail = Tail()) {
	typedef typename Elem<ET>::T T;
	static_assert(!(LB && PRUNE == 1), "the block bounds serve the compacted scan (its S units fold elsewhere)");
	constexpr bool NTL = MODE & 1, PIPE = (MODE & 2) != 0, SDV = (MODE & 4) != 0;
	constexpr int VEC = 16 / (int) sizeof(T), UV0 = (VEC >= 16 ? 1 : 16 / VEC) * (MODE & 8 ? 2 : 1);
	constexpr int UV = PIPE && UV0 > 1 ? UV0 / 2 : UV0;
	__shared__ int erow[REPLAY_CAP];
	TreeCtl *ctl = b.ctl;
	const int tid = threadIdx.x, lane = tid & 63;
	TS_ENTRY(2);
	TS(2, 0);
	TS_SAMP(0);
	const int r0 = b.crow[tid];
	const int done = ctl->done, Tn = ctl->T;
	if(done) return;
	tail.begin(b, n);
	if(Tn == 0) return;
	const int umax = dnj_umax(n, seg), nunits = Tn * umax;
	const int nSp = PRUNE ? ctl->pS : 0;
	// (the S phase's SEG-cell units may outnumber the entries' units)
	const int su0 = PRUNE == 1 && nSp ? b.pS_uo[nSp] : 0;
	if((int) blockIdx.x * (TB / 64) >= (nunits > su0 ? nunits : su0)) return;
	const bool lds = Tn <= REPLAY_CAP;
	if(lds) {
		if(tid < Tn) erow[tid] = r0;
		for(int e = TB + tid; e < Tn; e += TB) erow[e] = b.crow[e];
	}
	__syncthreads();
	const int gw = blockIdx.x * (TB / 64) + (tid >> 6), nw = gridDim.x * (TB / 64);
	TS(2, 1);
	TS_SAMP(1);
	// PRUNE (band mode): the S entries' units first (the lowest waves), their
	// exact fresh minima then bound every other entry (SBound), and an entry
	// whose stale Q is not below the bound at its row is one minQpair skips
	// (dnj.c:78): its units load nothing and leave DBL_MAX, which the replay
	// neither accepts nor lets into the running min
	__shared__ int s_uo[DNJ_B + 1];
	int su = 0;
	if(PRUNE == 1 && nSp) {
		for(int t = tid; t <= nSp; t += TB) s_uo[t] = b.pS_uo[t];
		__syncthreads();
		su = s_uo[nSp];
	}
	long long pruned = 0, lbskip = 0;
	// one unit: columns [c0, c1) of entry e's row r; S-phase units (sent) are
	// SEG cells with their partials in uq / uj at the S unit index
	auto unit = [&](int u, int e, int r, int c0, int c1, bool skip, bool sent, int sua, int sub) {
		const int ua = e * umax;
		if(skip) {
			pruned += c1 - c0;
			tail_unit(tail, b, n, u, ua, ua + dcdiv(r, seg), r, DBL_MAX, 0, e, Tn);
			return;
		}
		const double sDr = b.sD[r];
		const long long ro = rows.row(r);
		const T *row = D + ro;
		if(LB) {   // the block lower bounds (single engine)
			double q = DBL_MAX;
			int idx = 0;
			lbskip += lb_unit<ET>(row, bs, b, n, r, c0, c1, sDr, q, idx);
			qarg_wave_reduce(q, idx);
			tail_unit(tail, b, n, u, ua, ua + dcdiv(r, seg), r, q, idx, e, Tn);
			return;
		}
		const int a = (int) ((VEC - (ro + c0) % VEC) % VEC);
		const int ca = c0 + a < c1 ? c0 + a : c1;
		const int nv = (c1 - ca) / VEC, ce = ca + nv * VEC;
		double q = DBL_MAX;
		int idx = 0;
		auto cell = [&](int c) {
			const double d = Elem<ET>::get(row[c], bs);
			const double x = qcrit(n, n, d, sDr, b.sD[c]);
			if(0 <= d && qarg_better(x, c, q, idx)) {
				q = x;
				idx = c;
			}
		};
		if(lane < ca - c0) cell(c0 + lane);   // the unaligned head
		if(lane < c1 - ce) cell(ce + lane);   // the tail
		uint4 w[2][UV];
		double sk[2][UV][VEC];
		const bool sda = SDV && (ca & 1) == 0;   // uniform
		auto load = [&](int buf, int v0) {
#pragma unroll
			for(int m = 0; m < UV; ++m) {
				int k = v0 + 64 * m + lane;
				k = k < nv ? k : nv - 1;
				const uint4 *src = (const uint4 *) (row + ca + VEC * k);
				if(NTL) {
					typedef unsigned u4v __attribute__((ext_vector_type(4)));
					const u4v x = __builtin_nontemporal_load((const u4v *) src);
					w[buf][m] = make_uint4(x.x, x.y, x.z, x.w);
				} else {
					w[buf][m] = *src;
				}
				if(sda) {
#pragma unroll
					for(int t = 0; t < VEC; t += 2) {
						const double2 x = *(const double2 *) (b.sD + ca + VEC * k + t);
						sk[buf][m][t] = x.x;
						sk[buf][m][t + 1] = x.y;
					}
				} else {
#pragma unroll
					for(int t = 0; t < VEC; ++t) sk[buf][m][t] = b.sD[ca + VEC * k + t];
				}
			}
		};
		auto compare = [&](int buf, int v0) {
#pragma unroll
			for(int m = 0; m < UV; ++m) {
				const int k = v0 + 64 * m + lane;
				const T *ev = (const T *) &w[buf][m];
#pragma unroll
				for(int t = 0; t < VEC; ++t) {
					const int c = ca + VEC * k + t;
					const double d = Elem<ET>::get(ev[t], bs);
					const double x = qcrit(n, n, d, sDr, sk[buf][m][t]);
					const bool take = k < nv && 0 <= d && qarg_better(x, c, q, idx);
					q = take ? x : q;
					idx = take ? c : idx;
				}
			}
		};
		if(PIPE) {
			if(nv > 0) load(0, 0);
			int v0 = 0;
			for(; v0 + 64 * UV < nv; v0 += 128 * UV) {
				load(1, v0 + 64 * UV);
				compare(0, v0);
				if(v0 + 128 * UV < nv) load(0, v0 + 128 * UV);
				compare(1, v0 + 64 * UV);
			}
			if(v0 < nv) compare(0, v0);
		} else {
			for(int v0 = 0; v0 < nv; v0 += 64 * UV) {
				load(0, v0);
				compare(0, v0);
			}
		}
		qarg_wave_reduce(q, idx);
		if(PRUNE == 1 && sent) fold_arrive(b, n, b.uq, b.uj, u, sua, sub, q, idx, e, Tn, true);
		else tail_unit(tail, b, n, u, ua, ua + dcdiv(r, seg), r, q, idx, e, Tn);
	};
	for(int v = gw; v < su; v += nw) {   // the S phase: SEG-cell units (short, so the phase is)
		int lo = 0, hi = nSp;   // the S row t with s_uo[t] <= v < s_uo[t + 1]
		while(hi - lo > 1) {
			const int mid = (lo + hi) >> 1;
			if(s_uo[mid] <= v) lo = mid; else hi = mid;
		}
		const int r = b.pS_row[lo], c0 = (v - s_uo[lo]) * SEG_S;
		unit(v, b.pS_ent[lo], r, c0, c0 + SEG_S < r ? c0 + SEG_S : r, false, true, s_uo[lo], s_uo[lo + 1]);
	}
	SBound sb;
	bool have_sb = false, ready = false;
	if(PRUNE == 1 && nSp && (int) blockIdx.x * (TB / 64) < nunits) {   // block-uniform: one poller per block
		__shared__ int s_ready;
		__syncthreads();
		if(tid == 0) s_ready = s_table_wait(b, n);
		__syncthreads();
		ready = s_ready;
	}
	// PRUNE == 2: k_dnj_sphase (the launch before) rescanned S, folded its
	// entries and left the table tagged n (plain loads after the boundary)
	if(PRUNE == 2 && nSp) ready = b.srdy[0] == (unsigned) n;
	int nu = 0;   // (trace: units of this wave so far)
	(void) nu;
	if(CMP && PRUNE == 2 && nSp) {
		// k_dnj_sphase left only the surviving entries, by unit-count bucket
		// u at blist[Eall(u) ...): slot k's units are the survivors with more
		// than k units, buckets in descending u
		int H = 0;
		const int pb = ctl->pblk;
		for(int g = 0; g < pb; ++g) H += b.uhist[g * UHIST + lane];
		const int inch = wave_incl_sum(H), Eall = __builtin_amdgcn_readlane(inch, 63) - inch;
		const int cnt = b.bcnt[lane];
		const int incc = wave_incl_sum(cnt), totc = __builtin_amdgcn_readlane(incc, 63);
		const int Es = totc - incc;          // survivors with more than `lane` units
		const int C = totc - incc + cnt;     // survivors with at least `lane` units
		int R;
		const int P = wave_excl_scan(Es, &R);
		for(int v = gw; v < R; v += nw) {
			const int k = 63 - __clzll((long long) __ballot(Es > 0 && P <= v));
			const int j = v - __shfl(P, k);
			const int ub = 63 - __clzll((long long) __ballot(lane > k && C > j));
			const int p = j - (__shfl(C, ub) - __shfl(cnt, ub));
			const int e = b.blist[__shfl(Eall, ub) + p];
			const int r = lds ? erow[e] : b.crow[e];
			const int c0 = k * seg;
			TS_U(2 * nu);
			unit(e * umax + k, e, r, c0, c0 + seg < r ? c0 + seg : r, false, false, 0, 0);
			TS_U(2 * nu + 1);
			++nu;
		}
	} else if(CMP) {
		int H = 0;   // lane k: entries with exactly k units, summed over the plan's blocks
		const int pb = ctl->pblk;
		for(int g = 0; g < pb; ++g) H += b.uhist[g * UHIST + lane];
		int tot;
		const int inc = wave_incl_sum(H);
		tot = __builtin_amdgcn_readlane(inc, 63);
		const int E = tot - inc;   // entries with more than `lane` units: slot `lane`'s real units
		int R;
		const int P = wave_excl_scan(E, &R);
		for(int v = gw; v < R; v += nw) {
			const unsigned long long mk = __ballot(E > 0 && P <= v);
			const int k = 63 - __clzll((long long) mk);
			const int e = v - __shfl(P, k);
			const int r = lds ? erow[e] : b.crow[e];
			const int c0 = k * seg;
			bool skip = false;
			if(PRUNE == 2 && nSp) {
				if(b.eS[e]) continue;   // rescanned by k_dnj_sphase
				if(!have_sb) {
					sb.load(b, n, ready);
					have_sb = true;
				}
				skip = sb.ok && !(b.cbnd[e] < sb.at(r));
			}
			TS_U(2 * nu);
			unit(e * umax + k, e, r, c0, c0 + seg < r ? c0 + seg : r, skip, false, 0, 0);
			TS_U(2 * nu + 1);
			++nu;
		}
	}
	for(int u = CMP ? nunits : gw; u < nunits; u += nw) {
		const int e = u / umax, ua = e * umax;
		const int r = lds ? erow[e] : b.crow[e];
		const int c0 = (u - ua) * seg;
		if(c0 >= r || !rows.owns(r)) continue;   // wave-uniform
		bool skip = false;
		if(PRUNE && nSp) {
			if(b.eS[e]) continue;   // ran in the S phase
			if(!have_sb) {
				sb.load(b, n, ready);
				have_sb = true;
			}
			skip = sb.ok && !(b.cbnd[e] < sb.at(r));
		}
		TS_U(2 * nu);
		unit(u, e, r, c0, c0 + seg < r ? c0 + seg : r, skip, false, 0, 0);
		TS_U(2 * nu + 1);
		++nu;
	}
	// (uniform: every lane counted the same units; with PRUNE 2 k_dnj_sphase
	// already counted the pruned entries' whole rows)
	if(PRUNE == 1 && pruned && lane == 0)
		atomicAdd((unsigned long long *) &ctl->cells_pruned, (unsigned long long) pruned);
	if(LB && lbskip && lane == 0)   // this wave's slot (no contention)
		atomicAdd((unsigned long long *) (b.lbskip + (long long) ((blockIdx.x * (TB / 64) + (tid >> 6)) % LB_SCAN) * LB_SLOT),
		          (unsigned long long) lbskip);
	TS(2, 2);
	TS_SAMP(2);
	TS_EXIT(2);
}

// S's rescans in a launch of their own before the scan (CCG_SCAN_PRUNE=2):
// S rows (the plan's top and band rows, pS_*) in SEG-cell units, one wave per
// unit, each S entry folded at its last unit and the bound table built by the
// last S entry (fold_arrive without chunk accounting, s_table), so the scan
// that follows prunes with the table from its first unit and never waits.
// Column/row values are those the scan would read (the plan persisted row
// i's sD / N before this launch).
// SLOOP = false (k_dnj_compact, the default): the plan's helper blocks
// already rescanned S and built the table; this launch copies S's fresh
// minima to their entries and compacts the rest.  If the table is missing
// (a helper's bounded wait gave up: never expected) every entry, S's too,
// survives and is rescanned.
template <int ET, bool SLOOP = true>
__global__ __launch_bounds__(TB) void k_dnj_sphase(const typename Elem<ET>::T *__restrict__ D, double bs, TreeBufs b,
                                                   int n, int seg) {
	typedef typename Elem<ET>::T T;
	constexpr int UC = 16;   // a SEG-cell unit in two steps of loads
	__shared__ int s_uo[DNJ_B + 1];
	const TreeCtl *ctl = b.ctl;
	const int tid = threadIdx.x, lane = tid & 63;
	if(ctl->done) return;   // (block-uniform)
	const int nSp = ctl->pS, Tn = ctl->T;
	if(nSp <= 0) return;    // (block-uniform) no S this join: the scan enumerates every entry
	for(int t = tid; t <= nSp; t += TB) s_uo[t] = b.pS_uo[t];
	__syncthreads();
	const int su = SLOOP ? s_uo[nSp] : 0;
	const int gw = blockIdx.x * (TB / 64) + (tid >> 6), nw = gridDim.x * (TB / 64);
	for(int v = gw; v < su; v += nw) {
		int lo = 0, hi = nSp;   // the S row t with s_uo[t] <= v < s_uo[t + 1]
		while(hi - lo > 1) {
			const int mid = (lo + hi) >> 1;
			if(s_uo[mid] <= v) lo = mid; else hi = mid;
		}
		const int e = b.pS_ent[lo], r = b.pS_row[lo], c0 = (v - s_uo[lo]) * SEG_S;
		const int c1 = c0 + SEG_S < r ? c0 + SEG_S : r;
		const double sDr = b.sD[r];
		const T *row = D + tri(r);
		double q = DBL_MAX;
		int idx = 0;
		for(int base = c0; base < c1; base += 64 * UC) {
			double sk[UC];
			T vv[UC];
#pragma unroll
			for(int m = 0; m < UC; ++m) {
				const int c = base + 64 * m + lane;
				const int cc = c < c1 ? c : c1 - 1;
				sk[m] = b.sD[cc];
				vv[m] = row[cc];
			}
#pragma unroll
			for(int m = 0; m < UC; ++m) {
				const int c = base + 64 * m + lane;
				const double d = Elem<ET>::get(vv[m], bs);
				const double x = qcrit(n, n, d, sDr, sk[m]);
				const bool take = c < c1 && 0 <= d && qarg_better(x, c, q, idx);
				q = take ? x : q;
				idx = take ? c : idx;
			}
		}
		qarg_wave_reduce(q, idx);
		fold_arrive<false>(b, n, b.uq, b.uj, v, s_uo[lo], s_uo[lo + 1], q, idx, e, Tn, true);
	}
	// ---- the other entries under the table (one lane per entry): pruned ones
	// flagged (ePr, k_dnj_fold folds them as DBL_MAX), survivors appended to
	// their unit-count bucket (the scan enumerates only those).  A block whose
	// wait gives up keeps all its entries (still exact).
	__shared__ int s_ready, s_prow[DNJ_B];
	__shared__ double s_pbnd[DNJ_B];
	// this wave's first 64 entries, loaded before the wait (they do not depend on the table)
	const int ef = gw * 64 + lane;
	const bool vf = ef < Tn;
	const int rf0 = vf ? b.crow[ef] : 1;
	const bool sf0 = vf && b.eS[ef];
	const double cbf = vf ? b.cbnd[ef] : 0.0;
	__syncthreads();
	if(tid == 0) s_ready = SLOOP ? s_table_wait(b, n) : b.srdy[0] == (unsigned) n;
	__syncthreads();
	const bool ready = s_ready;
	if(!SLOOP && ready && blockIdx.x == 0)   // S's fresh minima to their entries (k_dnj_fold keeps them)
		for(int t = tid; t < nSp; t += TB) {
			const int e = b.pS_ent[t];
			b.rf[e] = b.sfq[t];
			b.rj[e] = b.sfj[t];
		}
	const double m0 = ctl->m0;
	if(ready) {
		for(int t = tid; t < nSp; t += TB) {
			s_prow[t] = b.pS_row[t];
			s_pbnd[t] = __hip_atomic_load(b.pS_bnd + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		}
	}
	__syncthreads();
	const bool vb = ready && ctl->vtag == n;
	const int G = (int) cdiv(n + 1, TB);
	int H = 0;   // lane u: entries with exactly u units (the plan's histogram); bucket u starts at E (u)
	for(int g = 0; g < ctl->pblk; ++g) H += b.uhist[g * UHIST + lane];
	const int inc = wave_incl_sum(H), E = __builtin_amdgcn_readlane(inc, 63) - inc;
	long long pcells = 0;   // cells of the pruned entries (stats: the scan never loads them)
	for(int e0 = gw * 64; e0 < Tn; e0 += nw * 64) {
		const int e = e0 + lane;
		const bool first = e0 == gw * 64, valid = e < Tn;
		const int r = first ? rf0 : valid ? b.crow[e] : 1;
		bool sE = first ? sf0 : valid && b.eS[e];
		if(!SLOOP && !ready && sE) {   // no table: S's entries are rescanned as any other
			b.eS[e] = 0;
			sE = false;
		}
		const double cb = first ? cbf : valid ? b.cbnd[e] : 0.0;
		bool pr = false;
		if(ready && valid && !sE) {
			int lo = 0, hi = nSp;   // S rows above r (descending rows)
			while(lo < hi) {
				const int mid = (lo + hi) >> 1;
				if(s_prow[mid] > r) lo = mid + 1; else hi = mid;
			}
			double bnd = lo ? s_pbnd[lo - 1] : m0;
			if(vb) {
				const int g = (r >> 8) + 1;
				const double vv = __hip_atomic_load(b.vsuf + (g < G ? g : G), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
				bnd = vv < bnd ? vv : bnd;
			}
			pr = !(cb < bnd);
		}
		if(valid) b.ePr[e] = pr;
		pcells += pr ? r : 0;
		const bool surv = valid && !sE && !pr;
		const int u0 = dcdiv(r, seg), u = u0 < UHIST ? u0 : UHIST - 1;
		unsigned long long rem = __ballot(surv);
		while(rem) {   // one atomic per bucket present in the wave
			const int ld = __ffsll((long long) rem) - 1;
			const int ub = __shfl(u, ld);
			const unsigned long long mk = __ballot(surv && u == ub);
			int base = 0;
			if(lane == ld) base = atomicAdd(b.bcnt + ub, __popcll(mk));
			base = __shfl(base, ld) + __shfl(E, ub);
			if(surv && u == ub)
				b.blist[base + (int) __builtin_amdgcn_mbcnt_hi((unsigned) (mk >> 32),
				                                               __builtin_amdgcn_mbcnt_lo((unsigned) mk, 0))] = e;
			rem &= ~mk;
		}
	}
	pcells = wave_sum_int(pcells);
	if(lane == 0 && pcells) atomicAdd((unsigned long long *) &b.ctl->cells_pruned, (unsigned long long) pcells);
}

// Row groups (the default rescan past 16384 taxa for every element type but
// double, scan_mode 20; 21-23 are other (G, UC) forms for measurement,
// CCG_SCAN_WAVE): one wave rescans
// the same seg-cell column range of G consecutive entries, so each sD load
// serves G rows (sD bytes per cell / G) and the wave holds G row streams in
// flight; rows are read one cell per lane (4- or 8-byte loads, coalesced per
// row), each row's (q, j) reduced and stored as its own unit partial, so the
// fold and the join read the layout of k_dnj_scan_v.  UC columns per lane per
// step.
template <int ET, int G, int UC, bool FOLD = false, bool PRUNE = false>
__global__ __launch_bounds__(TB) void k_dnj_scan_g(const typename Elem<ET>::T *__restrict__ D, double bs, TreeBufs b,
                                                   int n, int seg) {
	typedef typename Elem<ET>::T T;
	__shared__ int erow[REPLAY_CAP];
	__shared__ int s_uo[DNJ_B + 1];
	TreeCtl *ctl = b.ctl;
	const int tid = threadIdx.x, lane = tid & 63;
	const int r0 = b.crow[tid];
	const int done = ctl->done, Tn = ctl->T;
	if(done) return;
	if(Tn == 0) return;
	const int umax = dnj_umax(n, seg), ngroups = (Tn + G - 1) / G, nunits = ngroups * umax;
	const int nSp = PRUNE ? ctl->pS : 0;
	// (the S phase may hold more units than the groups: S rows one per wave)
	const int su0 = PRUNE && nSp ? b.pS_uo[nSp] : 0;
	if((int) blockIdx.x * (TB / 64) >= (nunits > su0 ? nunits : su0)) return;
	const bool lds = Tn <= REPLAY_CAP;
	if(lds) {
		if(tid < Tn) erow[tid] = r0;
		for(int e = TB + tid; e < Tn; e += TB) erow[e] = b.crow[e];
	}
	// PRUNE (band mode, with FOLD): the S entries' units first, one row per
	// wave, then the groups, whose entries below the S bound table's value at
	// their row (k_dnj_scan_v) load nothing and leave DBL_MAX
	int su = 0;
	if(PRUNE && nSp)
		for(int t = tid; t <= nSp; t += TB) s_uo[t] = b.pS_uo[t];
	__syncthreads();
	if(PRUNE && nSp) su = s_uo[nSp];
	const int gw = blockIdx.x * (TB / 64) + (tid >> 6), nw = gridDim.x * (TB / 64);
	long long pruned = 0;
	for(int v = gw; v < su; v += nw) {   // the S phase (PRUNE only)
		int lo = 0, hi = nSp;
		while(hi - lo > 1) {
			const int mid = (lo + hi) >> 1;
			if(s_uo[mid] <= v) lo = mid; else hi = mid;
		}
		const int e = b.pS_ent[lo], r = b.pS_row[lo], c0 = (v - s_uo[lo]) * SEG_S;   // SEG-cell S units
		const int c1 = c0 + SEG_S < r ? c0 + SEG_S : r;
		const double sDr = b.sD[r];
		const T *row = D + tri(r);
		double q = DBL_MAX;
		int idx = 0;
		for(int base = c0; base < c1; base += 64 * UC) {
			double sk[UC];
			T vv[UC];
#pragma unroll
			for(int m = 0; m < UC; ++m) {
				const int c = base + 64 * m + lane;
				const int cc = c < c1 ? c : c1 - 1;
				sk[m] = b.sD[cc];
				vv[m] = row[cc];
			}
#pragma unroll
			for(int m = 0; m < UC; ++m) {
				const int c = base + 64 * m + lane;
				const double d = Elem<ET>::get(vv[m], bs);
				const double x = qcrit(n, n, d, sDr, sk[m]);
				const bool take = c < c1 && 0 <= d && qarg_better(x, c, q, idx);
				q = take ? x : q;
				idx = take ? c : idx;
			}
		}
		qarg_wave_reduce(q, idx);
		fold_arrive(b, n, b.uq, b.uj, v, s_uo[lo], s_uo[lo + 1], q, idx, e, Tn, true);
	}
	SBound sb;
	bool have_sb = false, ready = false;
	if(PRUNE && nSp && (int) blockIdx.x * (TB / 64) < nunits) {   // block-uniform: one poller per block
		__shared__ int s_ready;
		__syncthreads();
		if(tid == 0) s_ready = s_table_wait(b, n);
		__syncthreads();
		ready = s_ready;
	}
	for(int u = gw; u < nunits; u += nw) {
		const int g = u / umax, s = u - g * umax, c0 = s * seg;
		int r[G], c1[G];
		bool act[G], skip[G];
		int cmax = c0;
#pragma unroll
		for(int k = 0; k < G; ++k) {
			const int e = g * G + k;
			r[k] = e < Tn ? (lds ? erow[e] : b.crow[e]) : 0;
			act[k] = e < Tn && c0 < r[k];
			skip[k] = false;
			if(PRUNE && nSp && act[k] && b.eS[e]) act[k] = false;   // ran in the S phase: no arrival here
		}
		if(PRUNE && nSp) {
			bool any = false;
#pragma unroll
			for(int k = 0; k < G; ++k) any = any || act[k];
			if(any && !have_sb) {   // uniform
				sb.load(b, n, ready);
				have_sb = true;
			}
			if(any && sb.ok) {
#pragma unroll
				for(int k = 0; k < G; ++k) {
					if(act[k] && !(b.cbnd[g * G + k] < sb.at(r[k]))) {   // uniform
						skip[k] = true;
						act[k] = false;
					}
				}
			}
		}
#pragma unroll
		for(int k = 0; k < G; ++k) {
			c1[k] = act[k] ? (c0 + seg < r[k] ? c0 + seg : r[k]) : c0;
			cmax = c1[k] > cmax ? c1[k] : cmax;
		}
		if(PRUNE) {
#pragma unroll
			for(int k = 0; k < G; ++k) {
				if(!skip[k]) continue;   // uniform
				const int e = g * G + k;
				pruned += (c0 + seg < r[k] ? c0 + seg : r[k]) - c0;
				tail_unit(FoldTail(), b, n, e * umax + s, e * umax, e * umax + dcdiv(r[k], seg), r[k], DBL_MAX, 0, e,
				          Tn);
			}
		}
		if(cmax == c0) continue;   // wave-uniform
		double sDr[G], q[G];
		int idx[G];
		const T *row[G];
#pragma unroll
		for(int k = 0; k < G; ++k) {
			sDr[k] = act[k] ? b.sD[r[k]] : 0.0;
			row[k] = D + tri(act[k] ? r[k] : 1);
			q[k] = DBL_MAX;
			idx[k] = 0;
		}
		for(int base = c0; base < cmax; base += 64 * UC) {
			double sk[UC];
			T v[G][UC];
#pragma unroll
			for(int m = 0; m < UC; ++m) {
				const int c = base + 64 * m + lane;
				sk[m] = b.sD[c < cmax ? c : cmax - 1];
#pragma unroll
				for(int k = 0; k < G; ++k) v[k][m] = row[k][c < c1[k] ? c : (act[k] ? c1[k] - 1 : 0)];
			}
#pragma unroll
			for(int m = 0; m < UC; ++m) {
				const int c = base + 64 * m + lane;
#pragma unroll
				for(int k = 0; k < G; ++k) {
					const double d = Elem<ET>::get(v[k][m], bs);
					const double x = qcrit(n, n, d, sDr[k], sk[m]);
					const bool take = c < c1[k] && 0 <= d && qarg_better(x, c, q[k], idx[k]);
					q[k] = take ? x : q[k];
					idx[k] = take ? c : idx[k];
				}
			}
		}
#pragma unroll
		for(int k = 0; k < G; ++k) {
			if(!act[k]) continue;   // wave-uniform
			double qq = q[k];
			int ii = idx[k];
			qarg_wave_reduce(qq, ii);
			const int e = g * G + k;
			if(FOLD) {
				tail_unit(FoldTail(), b, n, e * umax + s, e * umax, e * umax + dcdiv(r[k], seg), r[k], qq, ii, e, Tn);
			} else if(lane == 0) {
				b.cq[e * umax + s] = qq;
				b.cj[e * umax + s] = ii;
			}
		}
	}
	if(PRUNE && pruned && lane == 0)
		atomicAdd((unsigned long long *) &ctl->cells_pruned, (unsigned long long) pruned);
}

// Row groups over a dense enumeration (scan_mode 20-23 with the compacted
// form, the single engine's default for float / u16 / u8 rows past 16384
// taxa): the entries to rescan -- every listed entry, or with pruning
// (PRUNE2, k_dnj_sphase ran) only the survivors k_dnj_sphase appended to
// their unit-count buckets -- are taken in descending unit count (bucket u
// holds the entries with exactly u units; entry order inside a bucket is
// free) and cut into groups of G consecutive ones.  Slot k of the
// enumeration holds the groups whose first entry has more than k units
// (ceil(E_k / G) of them, E_k = the entries with more than k units, a prefix
// of the order), so the real (group, unit) pairs are numbered densely,
// slot-major, and dealt round-robin over a grid that is resident at once.
// One wave rescans the same seg-cell column range of its group's rows
// (k_dnj_scan_g's body: one sD load serves G rows); each row's (q, j) goes
// to its unit partial, which k_dnj_fold folds (pruned entries and S's, which
// k_dnj_sphase / the plan's helpers settled, have no units here).
// LB: each group's unit under the block lower bounds (lb_unit_g; the single
// engine with TreeBufs::lbm, no pruning)
template <int ET, int G, int UC, bool PRUNE2, bool LB = false>
__global__ __launch_bounds__(TB) void k_dnj_scan_gc(const typename Elem<ET>::T *__restrict__ D, double bs, TreeBufs b,
                                                    int n, int seg) {
	typedef typename Elem<ET>::T T;
	static_assert(!(LB && PRUNE2), "the bounded row groups run without S-bound pruning");
	const TreeCtl *ctl = b.ctl;
	const int tid = threadIdx.x, lane = tid & 63;
	const int done = ctl->done, Tn = ctl->T;
	if(done || Tn == 0) return;   // (block-uniform)
	const int umax = dnj_umax(n, seg);
	const int nSp = PRUNE2 ? ctl->pS : 0;
	const bool surv = PRUNE2 && nSp > 0;   // k_dnj_sphase left the survivors in blist (else: every entry, e = p)
	const int gw = blockIdx.x * (TB / 64) + (tid >> 6), nw = gridDim.x * (TB / 64);
	// lane u: H = listed entries with exactly u units (the plan's histogram, summed over its blocks);
	// bucket u's survivors sit at blist[Eall(u) ...), cnt(u) of them (k_dnj_sphase)
	int H = 0;
	const int pb = ctl->pblk;
	for(int g = 0; g < pb; ++g) H += b.uhist[g * UHIST + lane];
	const int inch = wave_incl_sum(H), Eall = __builtin_amdgcn_readlane(inch, 63) - inch;
	const int cnt = surv ? b.bcnt[lane] : H;
	const int incc = wave_incl_sum(cnt), totc = __builtin_amdgcn_readlane(incc, 63);
	const int Es = totc - incc;        // entries (survivors) with more than `lane` units: a prefix of the order
	const int C = Es + cnt;            // ... with at least `lane` units
	const int NG = (Es + G - 1) / G;   // slot `lane`'s groups
	int R;
	const int PG = wave_excl_scan(NG, &R);
	long long lbskip = 0;
	for(int v = gw; v < R; v += nw) {
		const int k = 63 - __clzll((long long) __ballot(NG > 0 && PG <= v));   // the slot (uniform)
		const int grp = v - __shfl(PG, k), EsK = __shfl(Es, k);
		const int c0 = k * seg;
		int r[G], e[G], c1[G];
		bool act[G];
		int cmax = c0;
#pragma unroll
		for(int t = 0; t < G; ++t) {
			const int pos = grp * G + t;
			act[t] = pos < EsK;   // (uniform) this member has unit k
			e[t] = 0;
			r[t] = 1;
			if(act[t]) {
				if(surv) {
					// the bucket: the highest u > k with C(u) > pos (C non-increasing in u)
					const int ub = 63 - __clzll((long long) __ballot(lane > k && C > pos));
					const int pin = pos - (__shfl(C, ub) - __shfl(cnt, ub));
					e[t] = b.blist[__shfl(Eall, ub) + pin];
				} else {
					e[t] = pos;   // the entry list is in descending rows: already in bucket order
				}
				r[t] = b.crow[e[t]];
			}
			c1[t] = act[t] ? (c0 + seg < r[t] ? c0 + seg : r[t]) : c0;
			cmax = c1[t] > cmax ? c1[t] : cmax;
		}
		double sDr[G], q[G];
		int idx[G];
		const T *row[G];
#pragma unroll
		for(int t = 0; t < G; ++t) {
			sDr[t] = act[t] ? b.sD[r[t]] : 0.0;
			row[t] = D + tri(act[t] ? r[t] : 1);
			q[t] = DBL_MAX;
			idx[t] = 0;
		}
		if(LB) lbskip += lb_unit_g<ET, G>(row, bs, b, n, r, act, c0, c1, cmax, sDr, q, idx);
		for(int base = c0; !LB && base < cmax; base += 64 * UC) {
			double sk[UC];
			T vv[G][UC];
#pragma unroll
			for(int m = 0; m < UC; ++m) {
				const int c = base + 64 * m + lane;
				sk[m] = b.sD[c < cmax ? c : cmax - 1];
#pragma unroll
				for(int t = 0; t < G; ++t) vv[t][m] = row[t][c < c1[t] ? c : (act[t] ? c1[t] - 1 : 0)];
			}
#pragma unroll
			for(int m = 0; m < UC; ++m) {
				const int c = base + 64 * m + lane;
#pragma unroll
				for(int t = 0; t < G; ++t) {
					const double d = Elem<ET>::get(vv[t][m], bs);
					const double x = qcrit(n, n, d, sDr[t], sk[m]);
					const bool take = c < c1[t] && 0 <= d && qarg_better(x, c, q[t], idx[t]);
					q[t] = take ? x : q[t];
					idx[t] = take ? c : idx[t];
				}
			}
		}
#pragma unroll
		for(int t = 0; t < G; ++t) {
			if(!act[t]) continue;   // wave-uniform
			double qq = q[t];
			int ii = idx[t];
			qarg_wave_reduce(qq, ii);
			if(lane == 0) {
				b.cq[e[t] * umax + k] = qq;
				b.cj[e[t] * umax + k] = ii;
			}
		}
	}
	if(LB && lbskip && lane == 0)   // this wave's slot (no contention), as k_dnj_scan_v
		atomicAdd((unsigned long long *) (b.lbskip + (long long) ((blockIdx.x * (TB / 64) + (tid >> 6)) % LB_SCAN) * LB_SLOT),
		          (unsigned long long) lbskip);
}

// ------------------------------------------------------------------ DNJ fold
// Rows with many units (large n): each entry's unit partials folded once into
// (rf, rj), one lane per entry and one wave per 64-entry chunk (scan order),
// and per chunk the summary k_dnj_join_pf replays from: the minimum fresh
// value, the row and partner of the first entry reaching it, and whether any
// entry is "bad" (fresh below its stale bound: minQpair's running min is then
// not a prefix min).
// sfold: this join's S entries (eS) were folded by k_dnj_sphase (rf / rj kept).
template <int UNUSED = 0>
__global__ __launch_bounds__(TB) void k_dnj_fold(TreeBufs b, int n, int seg, int sfold = 0) {
	const TreeCtl *ctl = b.ctl;
	if(ctl->done) return;
	const int T = ctl->T, lane = threadIdx.x & 63, umax = dnj_umax(n, seg);
	sfold = sfold && ctl->pS > 0;
	// k_dnj_sphase's bucket counts, consumed by the scan: zero for the next join
	if(blockIdx.x == 0 && threadIdx.x < UHIST) b.bcnt[threadIdx.x] = 0;
	const int nc = (T + 63) >> 6;
	const int w0 = (int) (blockIdx.x * (TB / 64) + (threadIdx.x >> 6)), nw = (int) (gridDim.x * (TB / 64));
	for(int c = w0; c < nc; c += nw) {
		const int e = (c << 6) + lane;
		const bool valid = e < T;
		const int r = valid ? b.crow[e] : 0;
		const double bnd = valid ? b.cbnd[e] : 0.0;
		const bool sdone = sfold && valid && b.eS[e], pruned = sfold && valid && !sdone && b.ePr[e];
		const int ua = e * umax, ub = ua + (valid && !sdone && !pruned ? dcdiv(r, seg) : 0);
		double q = sdone ? b.rf[e] : DBL_MAX;
		int idx = sdone ? b.rj[e] : 0;
		int u = ua;
		for(; u + 4 <= ub; u += 4) {   // 4 units' loads in flight
			double oq[4];
			int oi[4];
#pragma unroll
			for(int m = 0; m < 4; ++m) {
				oq[m] = b.cq[u + m];
				oi[m] = b.cj[u + m];
			}
#pragma unroll
			for(int m = 0; m < 4; ++m) {
				if(qarg_better(oq[m], oi[m], q, idx)) {
					q = oq[m];
					idx = oi[m];
				}
			}
		}
		for(; u < ub; ++u) {
			const double oq = b.cq[u];
			const int oi = b.cj[u];
			if(qarg_better(oq, oi, q, idx)) {
				q = oq;
				idx = oi;
			}
		}
		if(valid && !sdone) {
			b.rf[e] = q;
			b.rj[e] = idx;
		}
		const double mq = readlane_d(wave_incl_min(valid ? q : DBL_MAX), 63);
		const unsigned long long hm = __ballot(valid && q == mq);
		const unsigned long long bm = __ballot(valid && !(q >= bnd));
		const int first = hm ? __ffsll((long long) hm) - 1 : 0;
		const int fr = __shfl(r, first), fj = __shfl(idx, first);
		if(lane == 0) {
			b.chg[c] = mq;
			b.chr[c] = fr;
			b.chj[c] = fj;
			b.chb[c] = bm != 0ull;
		}
	}
}

// ------------------------------------------------------------------ minQpair replay
// dnj.c:88-112 decisions over the candidate entries in scan order (S, then
// the rest, descending rows), wave 0 only.  Entry e has its stale bound b_e
// = Q[row] and fresh min (f_e, j_e); the serial running min m_e starts at m0,
// entry e is accepted iff b_e < m_e, and then m_{e+1} = min(m_e, f_e).
//   A "good" entry (f_e >= b_e) gives m_{e+1} = min(m_e, f_e) whether or not
//   it is accepted (rejected means f_e >= b_e >= m_e), so over good entries
//   m is a prefix min.  A "bad" entry (f_e < b_e) lowers m only if accepted.
// So: prefix-min passes that treat the undecided bad entries as rejected;
// the first bad entry found accepted (b_e < m_e) is certainly accepted, fixes
// m_{e+1} = f_e, and the next pass starts after it.  Without bad entries this
// is one pass.  Accepted (Q, P) updates are applied by the writer block only,
// or, with acc_out, flagged per entry for a later kernel to apply.
__device__ __forceinline__ void replay_wave(int total, double m0, const int *e_row, const int *e_j, const double *e_b,
                            const double *e_f, unsigned char *e_acc, bool writer, const TreeBufs &b, int &pi,
                            int &pj, bool *had_bad, int n, unsigned char *acc_out = nullptr) {
	(void) n;   // trace stamps only
	const int lane = threadIdx.x & 63;
	int bad = 0;
	// 4 chunks of loads in flight (the entries may live in HBM)
	for(int e0 = lane; e0 < total; e0 += 256) {
		double f[4], bb[4];
#pragma unroll
		for(int k = 0; k < 4; ++k) {
			const int e = e0 + 64 * k < total ? e0 + 64 * k : total - 1;
			f[k] = e_f[e];
			bb[k] = e_b[e];
		}
#pragma unroll
		for(int k = 0; k < 4; ++k) {
			if(e0 + 64 * k < total) {
				bad |= !(f[k] >= bb[k]);
				e_acc[e0 + 64 * k] = 0;
			}
		}
	}
	const bool any_bad = __any(bad);
	*had_bad = any_bad;
	wave_sync();
	TS(3, 6);
	if(any_bad) {
		double m = m0;
		int start = 0;
		for(;;) {
			int hit = -1;
			double cm = m;
			for(int c0 = start; c0 < total; c0 += 64) {
				const int e = c0 + lane;
				const bool valid = e < total;
				const double f = valid ? e_f[e] : DBL_MAX, bb = valid ? e_b[e] : DBL_MAX;
				const bool good = valid && f >= bb;
				const double x = wave_incl_min(good ? f : DBL_MAX);
				double pre = dpp_d<DPP_WAVE_SHR1, 0xF>(DBL_MAX, x);
				pre = pre < cm ? pre : cm;
				const unsigned long long hm = __ballot(valid && !good && bb < pre);
				if(hm) {
					hit = c0 + __ffsll((long long) hm) - 1;
					break;
				}
				const double last = readlane_d(x, 63);
				cm = last < cm ? last : cm;
			}
			if(hit < 0) break;
			if(lane == 0) e_acc[hit] = 1;
			m = e_f[hit];
			start = hit + 1;
			wave_sync();
		}
	}
	// final pass: decisions, writes and the pair (the first contributor that
	// reaches the final minimum, if it is below m0)
	double cm = m0;
	long long nacc = 0, cacc = 0;   // minQpair's own rescans (ctl->ref_rows / ref_cells)
	for(int g0 = 0; g0 < total; g0 += 256) {
		double fv[4], bv[4];
		int rv[4], jv[4], av[4];
#pragma unroll
		for(int k = 0; k < 4; ++k) {
			const int e = g0 + 64 * k + lane < total ? g0 + 64 * k + lane : total - 1;
			fv[k] = e_f[e];
			bv[k] = e_b[e];
			rv[k] = e_row[e];
			jv[k] = e_j[e];
			av[k] = e_acc[e];
		}
#pragma unroll
		for(int k = 0; k < 4; ++k) {
			const int c0 = g0 + 64 * k;
			if(c0 >= total) break;
			const bool valid = c0 + lane < total;
			const double f = valid ? fv[k] : DBL_MAX, bb = valid ? bv[k] : DBL_MAX;
			const bool good = valid && f >= bb;
			const bool contrib = good || (valid && av[k]);
			const double x = wave_incl_min(contrib ? f : DBL_MAX);
			double pre = dpp_d<DPP_WAVE_SHR1, 0xF>(DBL_MAX, x);
			pre = pre < cm ? pre : cm;
			const bool accepted = good ? bb < pre : contrib;
			if(accepted) {
				++nacc;
				cacc += rv[k];
			}
			if(writer && acc_out) {
				if(valid) acc_out[c0 + lane] = accepted;   // applied later (k_shd_join)
			} else if(writer && accepted) {
				b.Q[rv[k]] = f;
				b.P[rv[k]] = jv[k];
			}
			const double last = readlane_d(x, 63);
			cm = last < cm ? last : cm;
		}
	}
	TS(3, 7);
	if(writer) {
		nacc = wave_sum_int(nacc);
		cacc = wave_sum_int(cacc);
		if(lane == 0 && nacc) {
			atomicAdd((unsigned long long *) &b.ctl->ref_rows, (unsigned long long) nacc);
			atomicAdd((unsigned long long *) &b.ctl->ref_cells, (unsigned long long) cacc);
		}
	}
	if(total && cm < m0) {
		int first_e = 0x7fffffff;
		for(int e0 = lane; e0 < total; e0 += 256) {
			double f[4], bb[4];
			int a[4];
#pragma unroll
			for(int k = 0; k < 4; ++k) {
				const int e = e0 + 64 * k < total ? e0 + 64 * k : total - 1;
				f[k] = e_f[e];
				bb[k] = e_b[e];
				a[k] = e_acc[e];
			}
#pragma unroll
			for(int k = 0; k < 4; ++k) {
				const int e = e0 + 64 * k;
				const bool contrib = f[k] >= bb[k] || a[k];
				if(e < total && contrib && f[k] == cm && e < first_e) first_e = e;
			}
		}
		first_e = wave_min_int(first_e);
		pi = e_row[first_e];
		pj = e_j[first_e];
	}
}
