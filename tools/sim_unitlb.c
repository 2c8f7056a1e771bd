/* sim_unitlb.c -- development aid: how many cells would minQpair's rescans
 * need if each row kept per-unit lower bounds of the Q criterion?  On the
 * serial DNJ of oracle/ccoracle.c: at every `every`-th join, for each row the
 * reference rescans (Q[r] < running min, dnj.c:78), the fresh minimum f_r and,
 * per unit of U consecutive columns, the bound
 *     lb(u) = (n - 2) * min_{c in u} d(r, c) - sD_r - max_{c in u} sD_c
 * (no missing entries: N == n).  A unit with lb(u) > f_r cannot hold the
 * row's minimum (nor a tie, which the index rule could pick), so an ideal
 * branch-and-bound rescans only the units with lb(u) <= f_r.  Exact per-unit
 * minima here (an engine would keep conservative ones, refreshed by every
 * full rescan), so the ratios are the idea's limit.
 * Build: gcc -O2 -std=gnu99 -ffp-contract=off -Ioracle tools/sim_unitlb.c -lm -o /tmp/sim_unitlb
 *        /tmp/sim_unitlb N [every] [maxjoins] [matrix.bin] */
#include "../oracle/ccoracle.c"
#include <stdio.h>
static const int32_t *g_P;

#define NU 4
static const int Us[NU] = {64, 256, 1024, 4096};
static double cref, cneed[NU], its;
/* maintained per-64-column bounds (the engine's form): exact at init and at
 * each refresh (every R joins), rows j and i (rewritten / moved) exact after
 * each join, and a cell written into column j or i of another row only
 * lowers that row's unit bound (min with the new value); rescans use the
 * threshold of the row's partner cell q(r, P[r]) instead of f_r */
#define LU 64
static double *LB, cmaint, cmaint_ideal;
static int LS;
static void lb_row(const Ltd *D, int r) {
	for(int u = 0; u * LU < r; ++u) {
		double md = DBL_MAX;
		for(int c = u * LU; c < (u + 1) * LU && c < r; ++c) md = at(D, r, c) < md ? at(D, r, c) : md;
		LB[(size_t) r * LS + u] = md;
	}
}
static void lb_col(const Ltd *D, int n, int c) {
	for(int k = c + 1; k < n; ++k) {
		double *x = LB + (size_t) k * LS + c / LU;
		if(at(D, k, c) < *x) *x = at(D, k, c);
	}
}

static void sim_iter(const Ltd *D, int n, const double *sD, const int32_t *N, const double *Q, int cand) {
	double m0 = DBL_MAX;
	if(cand && m0 != Q[cand]) m0 = Q[cand];
	double m = m0;
	for(int r = n - 1; r >= 1; --r) {
		if(!(Q[r] < m)) continue;
		int mj;
		const double f = row_min(D, r, sD, N, &mj, 0);
		cref += r;
		for(int k = 0; k < NU; ++k) {
			const int U = Us[k];
			for(int c0 = 0; c0 < r; c0 += U) {
				const int c1 = c0 + U < r ? c0 + U : r;
				double md = DBL_MAX, ms = -DBL_MAX;
				for(int c = c0; c < c1; ++c) {
					const double d = at(D, r, c);
					if(d < md) md = d;
					if(sD[c] > ms) ms = sD[c];
				}
				const double lb = (double) (n - 2) * md - sD[r] - ms;
				if(lb <= f) cneed[k] += c1 - c0;
			}
		}
		{   /* maintained bounds, partner-cell threshold */
			double ub = DBL_MAX;
			const int32_t pr = g_P[r] >= 0 && g_P[r] < r ? g_P[r] : 0;
			ub = qval(N[r], N[pr], at(D, r, pr), sD[r], sD[pr]);
			for(int c0 = 0, u = 0; c0 < r; c0 += LU, ++u) {
				const int c1 = c0 + LU < r ? c0 + LU : r;
				double ms = -DBL_MAX;
				for(int c = c0; c < c1; ++c) ms = sD[c] > ms ? sD[c] : ms;
				const double lb = (double) (n - 2) * LB[(size_t) r * LS + u] - sD[r] - ms;
				if(lb <= ub) cmaint += c1 - c0;
				if(lb <= f) cmaint_ideal += c1 - c0;
			}
		}
		if(f < m) m = f;
	}
	its += 1;
}
static const int32_t *g_P_dummy;

int main(int argc, char **argv) {
	int n = argc > 1 ? atoi(argv[1]) : 2000;
	int every = argc > 2 ? atoi(argv[2]) : 1;
	const int maxj = argc > 3 ? atoi(argv[3]) : 1 << 30;
	double *Dm = malloc((size_t) n * (n - 1) / 2 * sizeof(double));
	if(argc > 4) {
		FILE *f = fopen(argv[4], "rb");
		if(!f || fread(Dm, sizeof(double), (size_t) n * (n - 1) / 2, f) != (size_t) n * (n - 1) / 2) return 1;
		fclose(f);
	} else {
		srand(1);
		double *pts = malloc((size_t) n * 8 * sizeof(double));
		for(int k = 0; k < n * 8; ++k) pts[k] = rand() / (RAND_MAX + 1.0);
		for(int i = 1; i < n; ++i)
			for(int j = 0; j < i; ++j) {
				double s = 0;
				for(int d = 0; d < 8; ++d) s += (pts[i * 8 + d] - pts[j * 8 + d]) * (pts[i * 8 + d] - pts[j * 8 + d]);
				Dm[tri(i) + j] = round(sqrt(s) * 1e9) / 1e9;
			}
	}
	Ltd D = {8, 1.0, Dm};
	double *sD = malloc(n * sizeof(double)), *Q = malloc(n * sizeof(double));
	int32_t *N = malloc(n * sizeof(int32_t)), *P = malloc(n * sizeof(int32_t));
	init_sums(&D, n, sD, N);
	init_hnj(&D, n, sD, N, Q, P);
	g_P = P;
	const int R = getenv("REFRESH") ? atoi(getenv("REFRESH")) : 1 << 30;
	LS = (n + LU - 1) / LU;
	LB = malloc((size_t) n * LS * sizeof(double));
	for(int r = 1; r < n; ++r) lb_row(&D, r);
	int j = min_q_row(Q, n);
	uint64_t pos;
	int joins = 0;
	const int n0 = n;
	while(n != 2) {
		if(joins % every == 0) sim_iter(&D, n, sD, N, Q, j);
		if(!(pos = min_q_pair(&D, n, sD, N, Q, P, j, 0))) break;
		j = (int) (pos & 0xFFFFFFFFu);
		int i = (int) (pos >> 32);
		double Li, Lj;
		limb_length(&Li, &Lj, i, j, sD, N, ld(&D, tri(i) + j), 0);
		update_d(&D, n, sD, N, i, j, Li, Lj);
		int mi = update_dnj_q(&D, n, sD, N, Q, P, i, j);
		int mj = dnj_pop_arrange(&D, &n, sD, N, Q, P, i);
		/* bounds: row j rewritten, column j; row i = old row n-1 (moved), column i */
		lb_row(&D, j);
		lb_col(&D, n, j);
		if(i < n) {
			lb_row(&D, i);
			lb_col(&D, n, i);
		}
		if((joins + 1) % R == 0)
			for(int r = 1; r < n; ++r) lb_row(&D, r);
		j = mj == n ? mi : mi == n ? mj : min_pos(Q, mi, mj);
		++joins;
		if(joins % (n0 / 8) == 0 || joins == maxj) {
			printf("after %d joins: reference cells/join %.0f;", joins, cref / its);
			for(int k = 0; k < NU; ++k) printf(" U=%d needs %.3f", Us[k], cneed[k] / cref);
			printf(" | maintained U=%d: partner threshold %.3f, exact f %.3f", LU, cmaint / cref, cmaint_ideal / cref);
			printf("\n");
			fflush(stdout);
		}
		if(joins == maxj) break;
	}
	return 0;
}
