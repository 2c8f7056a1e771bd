/* sim_stages.c -- development aid: rescanned cells of the GPU engine's DNJ
 * candidate selection strategies against the serial reference (minQpair
 * dnj.c:43), on the serial DNJ of oracle/ccoracle.c (Euclidean U[0,1)^8):
 *   CUR   S = top-B rows with Q < m0, U from S, every row below S with Q < U
 *   MS(K) the same S, then stages of up to K rows below the previous stage
 *         with Q < U_k, U_{k+1} tightened by each stage, until no row is left
 * Build: gcc -O2 -std=gnu99 -ffp-contract=off -Ioracle tools/sim_stages.c -lm -o /tmp/sim_stages
 *        /tmp/sim_stages N [every] */
#include "../oracle/ccoracle.c"
#include <stdio.h>

#define NK 6
/* stage-size sequences: stage k takes up to seq[k] rows (the last repeats) */
static const int Seqs[NK][6] = {{128, 1 << 30}, {128, 256}, {8, 32, 128, 1 << 30}, {4, 16, 64, 256, 1 << 30},
                                {16, 64, 256, 1 << 30}, {32, 1 << 30}};
static double cref, ccur[NK], stages[NK], maxst[NK], its;
#define NH 4
static const int HA[NH] = {32, 16, 16, 8}, HB[NH] = {-64, -64, -112, -120};   /* -k: minima of k equal row blocks */
static double chyb[NH];
/* H1 (16 top + 64 band rows) with, in addition, the bound from every row
 * above r's 256-row block: V_k = max(q at k's partner cell, Q_k) (a cell of
 * row k bounds its fresh minimum), block minima of V (the requeue could
 * publish them); VB[1]: the same with every row above r (the idea's limit) */
static double cvb[4];
static const int32_t *g_P;
static int cmpq_desc_rows;   /* unused */
static const double *g_Q;
static int by_q(const void *a, const void *b) {
	double x = g_Q[*(const int *) a], y = g_Q[*(const int *) b];
	return x < y ? -1 : x > y ? 1 : (*(const int *) b - *(const int *) a);
}

static double fresh_of(const Ltd *D, int r, const double *sD, const int32_t *N, double *memo, char *have) {
	if(!have[r]) {
		int mj;
		memo[r] = row_min(D, r, sD, N, &mj, 0);
		have[r] = 1;
	}
	return memo[r];
}

static void sim_iter(const Ltd *D, int n, const double *sD, const int32_t *N, const double *Q, int cand) {
	const int32_t *P = g_P;
	double m0 = DBL_MAX;
	if(cand && m0 != Q[cand]) m0 = Q[cand];
	double *memo = malloc(n * sizeof(double));
	char *have = calloc(n, 1);
	/* reference */
	double m = m0;
	for(int r = n - 1; r >= 1; --r) {
		if(Q[r] < m) {
			double f = fresh_of(D, r, sD, N, memo, have);
			cref += r;
			if(f < m) m = f;
		}
	}
	for(int k = 0; k < NK; ++k) {
		double U = m0, cells = 0;
		int r = n - 1, st = 0, si = 0;
		while(r >= 1) {
			const int lim = Seqs[k][si];
			if(si < 5 && Seqs[k][si + 1]) ++si;
			double U2 = U;
			int taken = 0;
			for(; r >= 1 && taken < lim; --r) {
				if(Q[r] < U) {
					double f = fresh_of(D, r, sD, N, memo, have);
					double v = f > Q[r] ? f : Q[r];
					U2 = v < U2 ? v : U2;
					cells += r;
					++taken;
				}
			}
			++st;
			U = U2;
			if(taken < lim) break;   /* every row below was under test */
		}
		ccur[k] += cells;
		stages[k] += st;
		if(st > maxst[k]) maxst[k] = st;
	}
	/* hybrid: S = top-A rows with Q < m0 plus the B smallest-Q rows below them
	 * (Q < m0); every other row r with Q < m0 is rescanned iff Q[r] < bound(r)
	 * = min(m0, min over S rows above r of max(fresh, Q)) */
	{
		int *cand = malloc(n * sizeof(int)), nc = 0;
		for(int r = n - 1; r >= 1; --r) if(Q[r] < m0) cand[nc++] = r;
		char *inS = calloc(n, 1);
		for(int h = 0; h < NH; ++h) {
			memset(inS, 0, n);
			double cells = 0;
			int A = HA[h] < nc ? HA[h] : nc;
			for(int k = 0; k < A; ++k) inS[cand[k]] = 1;
			int rem = nc - A;
			if(rem > 0 && HB[h] < 0) {
				const int lowest = A ? cand[A - 1] : n;
				const int g = (lowest + (-HB[h]) - 1) / (-HB[h]);
				for(int b0 = 0; b0 < lowest; b0 += g) {
					int best = -1;
					for(int r = b0; r < b0 + g && r < lowest; ++r)
						if(r >= 1 && Q[r] < m0 && (best < 0 || Q[r] < Q[best])) best = r;
					if(best >= 0) inS[best] = 1;
				}
			}
			if(rem > 0 && HB[h] > 0) {
				int *tmp = malloc(rem * sizeof(int));
				memcpy(tmp, cand + A, rem * sizeof(int));
				g_Q = Q;
				qsort(tmp, rem, sizeof(int), by_q);
				for(int k = 0; k < HB[h] && k < rem; ++k) inS[tmp[k]] = 1;
				free(tmp);
			}
			double bound = m0;
			for(int k = 0; k < nc; ++k) {   /* descending rows */
				int r = cand[k];
				if(inS[r]) {
					double f = fresh_of(D, r, sD, N, memo, have);
					double v = f > Q[r] ? f : Q[r];
					cells += r;
					if(v < bound) bound = v;
				} else if(Q[r] < bound) {
					double f = fresh_of(D, r, sD, N, memo, have);
					(void) f;
					cells += r;
				}
			}
			chyb[h] += cells;
		}
		free(inS);
		free(cand);
	}
	/* H1 + V block minima / every row above */
	{
		double *V = malloc(n * sizeof(double)), *bmin = malloc(((n >> 8) + 2) * sizeof(double));
		for(int k = 0; k < n; ++k) {
			V[k] = DBL_MAX;
			if(k >= 1 && P[k] >= 0 && P[k] < k) {
				const double d = at(D, k, P[k]);
				if(d >= 0) {
					const double q = qval(N[k], N[P[k]], d, sD[k], sD[P[k]]);
					V[k] = q > Q[k] ? q : Q[k];
				}
			}
		}
		const int nb = (n >> 8) + 1;
		for(int g = 0; g <= nb; ++g) bmin[g] = DBL_MAX;
		for(int k = 0; k < n; ++k) if(V[k] < bmin[k >> 8]) bmin[k >> 8] = V[k];
		for(int g = nb - 1; g >= 0; --g) if(bmin[g + 1] < bmin[g]) bmin[g] = bmin[g + 1];   /* suffix min: blocks >= g */
		int *cand = malloc(n * sizeof(int)), nc = 0;
		for(int r = n - 1; r >= 1; --r) if(Q[r] < m0) cand[nc++] = r;
		char *inS = calloc(n, 1);
		for(int mode = 0; mode < 4; ++mode) {   /* 2: S by partner cells, no V (the engine); 3: + Vblk */
			memset(inS, 0, n);
			double cells = 0;
			int A = 16 < nc ? 16 : nc;
			for(int k = 0; k < A; ++k) inS[cand[k]] = 1;
			if(nc - A > 0) {
				const int lowest = A ? cand[A - 1] : n, g = (lowest + 63) / 64;
				for(int b0 = 0; b0 < lowest; b0 += g) {
					int best = -1;
					for(int r = b0; r < b0 + g && r < lowest; ++r)
						if(r >= 1 && Q[r] < m0 && (best < 0 || Q[r] < Q[best])) best = r;
					if(best >= 0) inS[best] = 1;
				}
			}
			double bound = m0, vrun = DBL_MAX;
			int prev = n;
			for(int k = 0; k < nc; ++k) {
				int r = cand[k];
				if(mode == 1) for(int x = prev - 1; x > r; --x) if(V[x] < vrun) vrun = V[x];   /* every row above r */
				prev = r;
				double bb = bound;
				const double vb = mode == 0 || mode == 3 ? bmin[(r >> 8) + 1] : mode == 1 ? vrun : DBL_MAX;
				if(vb < bb) bb = vb;
				if(inS[r]) {
					double f = fresh_of(D, r, sD, N, memo, have);
					double v = mode >= 2 ? V[r] : f > Q[r] ? f : Q[r];
					cells += r;
					if(v < bound) bound = v;
				} else if(Q[r] < bb) {
					cells += r;
				}
			}
			cvb[mode] += cells;
		}
		free(inS);
		free(cand);
		free(V);
		free(bmin);
	}
	its += 1;
	free(memo);
	free(have);
}

int main(int argc, char **argv) {
	int n = argc > 1 ? atoi(argv[1]) : 2000;
	int every = argc > 2 ? atoi(argv[2]) : 1;
	const int maxj = argc > 3 ? atoi(argv[3]) : 1 << 30;   /* stop (and print) after this many joins */
	double *Dm = malloc((size_t) n * (n - 1) / 2 * sizeof(double));
	if(argc > 4) {   /* a matrix from a file: n(n-1)/2 raw doubles (e.g. clade SNP counts) */
		FILE *f = fopen(argv[4], "rb");
		if(!f || fread(Dm, sizeof(double), (size_t) n * (n - 1) / 2, f) != (size_t) n * (n - 1) / 2) return 1;
		fclose(f);
		goto loaded;
	}
	srand(1);
	double *pts = malloc((size_t) n * 8 * sizeof(double));
	for(int k = 0; k < n * 8; ++k) pts[k] = rand() / (RAND_MAX + 1.0);
	for(int i = 1; i < n; ++i)
		for(int j = 0; j < i; ++j) {
			double s = 0;
			for(int d = 0; d < 8; ++d) s += (pts[i * 8 + d] - pts[j * 8 + d]) * (pts[i * 8 + d] - pts[j * 8 + d]);
			Dm[tri(i) + j] = round(sqrt(s) * 1e9) / 1e9;
		}
loaded:;
	Ltd D = {8, 1.0, Dm};
	double *sD = malloc(n * sizeof(double)), *Q = malloc(n * sizeof(double));
	int32_t *N = malloc(n * sizeof(int32_t)), *P = malloc(n * sizeof(int32_t));
	g_P = P;
	init_sums(&D, n, sD, N);
	init_hnj(&D, n, sD, N, Q, P);
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
		j = mj == n ? mi : mi == n ? mj : min_pos(Q, mi, mj);
		++joins;
		if(joins % (n0 / 8) == 0 || joins == maxj) {
			printf("  after %d joins: ref cells/join %.0f", joins, cref / its);
			for(int k = 0; k < NK; ++k) printf(" | %d,%d,%d x%.2f st %.2f (max %.0f)", Seqs[k][0], Seqs[k][1], Seqs[k][2], ccur[k] / cref, stages[k] / its, maxst[k]);
			for(int h = 0; h < NH; ++h) printf(" | H%d+%d x%.2f", HA[h], HB[h], chyb[h] / cref);
			printf(" | H16+64+Vblk x%.2f | H16+64+Vall x%.2f | H16+64 partner x%.2f | partner+Vblk x%.2f", cvb[0] / cref,
			       cvb[1] / cref, cvb[2] / cref, cvb[3] / cref);
			printf("\n");
			fflush(stdout);
		}
		if(joins == maxj) break;
	}
	return 0;
}
