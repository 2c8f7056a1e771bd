/* sim_dnj.c -- development aid: statistics of the GPU engine's DNJ selection
 * (top-B rows S of {Q < m0}, bound U, rows T below S with Q < U) on the
 * serial DNJ of oracle/ccoracle.c, for several B.  Build:
 *   gcc -O2 -std=gnu99 -ffp-contract=off -Ioracle tools/sim_dnj.c -lm -o /tmp/sim_dnj
 *   /tmp/sim_dnj N [snp]          (Euclidean U[0,1)^8 or integer SNP-like matrix) */
#include "../oracle/ccoracle.c"
#include <stdio.h>

#define NB 7
static const int Bs[NB] = {32, 64, 128, 192, 256, 384, 512};
static double sumT[NB], sumT0[NB], sumS[NB], sumCells[NB], its;
static long long hist[NB][8];

static void sim_iter(const Ltd *D, int n, const double *sD, const int32_t *N, const double *Q, const int32_t *P,
                     int cand) {
	double m0 = DBL_MAX;
	if(cand && m0 != Q[cand]) m0 = Q[cand];
	int *rows = malloc(n * sizeof(int));
	int c0 = 0;
	for(int r = n - 1; r >= 1; --r) if(Q[r] < m0) rows[c0++] = r;
	double *fresh = malloc((c0 ? c0 : 1) * sizeof(double));
	int nf = 0;
	for(int b = 0; b < NB; ++b) {
		int B = Bs[b];
		int nS = c0 < B ? c0 : B;
		while(nf < nS) {
			int mj;
			fresh[nf] = row_min(D, rows[nf], sD, N, &mj, 0);
			++nf;
		}
		double U = m0;
		double cells = 0;
		for(int t = 0; t < nS; ++t) {
			double v = fresh[t] > Q[rows[t]] ? fresh[t] : Q[rows[t]];
			U = v < U ? v : U;
			cells += rows[t];
		}
		int T = 0;
		if(nS == B) {
			int smin = rows[B - 1];
			for(int r = smin - 1; r >= 1; --r) if(Q[r] < U) { ++T; cells += r; }
		}
		sumT[b] += T;
		sumT0[b] += T == 0;
		sumS[b] += nS;
		sumCells[b] += cells;
		int h = T == 0 ? 0 : T < 4 ? 1 : T < 16 ? 2 : T < 64 ? 3 : T < 128 ? 4 : T < 256 ? 5 : T < 1024 ? 6 : 7;
		hist[b][h]++;
	}
	its += 1;
	free(rows);
	free(fresh);
}

int main(int argc, char **argv) {
	int n = argc > 1 ? atoi(argv[1]) : 2000;
	int snp = argc > 2;
	double *Dm = malloc((size_t) n * (n - 1) / 2 * sizeof(double));
	srand(1);
	if(!snp) {
		double *pts = malloc((size_t) n * 8 * sizeof(double));
		for(int k = 0; k < n * 8; ++k) pts[k] = rand() / (RAND_MAX + 1.0);
		for(int i = 1; i < n; ++i)
			for(int j = 0; j < i; ++j) {
				double s = 0;
				for(int d = 0; d < 8; ++d) s += (pts[i * 8 + d] - pts[j * 8 + d]) * (pts[i * 8 + d] - pts[j * 8 + d]);
				Dm[tri(i) + j] = round(sqrt(s) * 1e9) / 1e9;
			}
	} else {
		/* tree-like integer distances: random binary-ish clusters + noise */
		int *g = malloc(n * sizeof(int));
		for(int k = 0; k < n; ++k) g[k] = rand() % 50;
		for(int i = 1; i < n; ++i)
			for(int j = 0; j < i; ++j) Dm[tri(i) + j] = (g[i] == g[j] ? 20 : 200) + rand() % 40;
	}
	Ltd D = {8, 1.0, Dm};
	double *sD = malloc(n * sizeof(double)), *Q = malloc(n * sizeof(double));
	int32_t *N = malloc(n * sizeof(int32_t)), *P = malloc(n * sizeof(int32_t));
	init_sums(&D, n, sD, N);
	init_hnj(&D, n, sD, N, Q, P);
	int j = min_q_row(Q, n);
	uint64_t pos;
	int joins = 0;
	while(n != 2) {
		sim_iter(&D, n, sD, N, Q, P, j);
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
	}
	printf("joins %d\n   B   mean|S|   meanT  P(T=0)  cells/join   T hist [0,1-3,4-15,16-63,64-127,128-255,256-1023,1024+]\n", joins);
	for(int b = 0; b < NB; ++b) {
		printf("%4d %8.1f %8.1f %7.3f %11.0f  ", Bs[b], sumS[b] / its, sumT[b] / its, sumT0[b] / its, sumCells[b] / its);
		for(int h = 0; h < 8; ++h) printf(" %lld", hist[b][h]);
		printf("\n");
	}
	return 0;
}
