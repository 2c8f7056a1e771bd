/* sim_bound.c -- development aid: a cheaper bound for DNJ's second rescan
 * phase.  The engine's bound U = min(m0, min over S rows k of max(fresh_k,
 * Q_k)) needs S's rescans first (k_dnj_select -> k_dnj_find).  Any upper bound
 * of fresh_k keeps the rest list exact (a superset), e.g. the row's Q
 * criterion at its stored partner P[k] evaluated NOW (one cell per row):
 * U2 = min(m0, min_k max(q(k, P[k]), Q_k)).  With U2 the rest rows are known
 * before any rescan, so S and the rest could be rescanned in one phase.
 * Prints rows / cells per join rescanned by the reference, by the engine's
 * two-phase search (top-128 S + rest under U) and by the one-phase search
 * (top-128 S + rest under U2), on the serial DNJ of oracle/ccoracle.c
 * (Euclidean U[0,1)^8, %.9f).
 * Build: gcc -O2 -std=gnu99 -ffp-contract=off -Ioracle tools/sim_bound.c -lm -lpthread -o /tmp/sim_bound
 *        /tmp/sim_bound N [top] */
#include "../oracle/ccoracle.c"
#include <stdio.h>

int main(int argc, char **argv) {
	int n = argc > 1 ? atoi(argv[1]) : 2000;
	const int top = argc > 2 ? atoi(argv[2]) : 128;
	double *Dm = malloc((size_t) n * (n - 1) / 2 * sizeof(double));
	srand(1);
	double *pts = malloc((size_t) n * 8 * sizeof(double));
	for(int k = 0; k < n * 8; ++k) pts[k] = rand() / (RAND_MAX + 1.0);
	for(int i = 1; i < n; ++i)
		for(int j = 0; j < i; ++j) {
			double s = 0;
			for(int d = 0; d < 8; ++d) s += (pts[i * 8 + d] - pts[j * 8 + d]) * (pts[i * 8 + d] - pts[j * 8 + d]);
			Dm[tri(i) + j] = round(sqrt(s) * 1e9) / 1e9;
		}
	Ltd D = {8, 1.0, Dm};
	double *sD = malloc(n * sizeof(double)), *Q = malloc(n * sizeof(double));
	int32_t *N = malloc(n * sizeof(int32_t)), *P = malloc(n * sizeof(int32_t));
	init_sums(&D, n, sD, N);
	init_hnj(&D, n, sD, N, Q, P);
	int j = min_q_row(Q, n);
	uint64_t pos;
	int joins = 0;
	double ref_r = 0, ref_c = 0, two_r = 0, two_c = 0, one_r = 0, one_c = 0, same = 0, rest1 = 0, rest2 = 0;
	int *S = malloc(n * sizeof(int));
	while(n != 2) {
		double m0 = DBL_MAX;
		if(j && m0 != Q[j]) m0 = Q[j];
		int nS = 0, smin = 1;
		for(int r = n - 1; r >= 1 && nS < top; --r)
			if(Q[r] < m0) S[nS++] = r;
		if(nS == top) smin = S[top - 1];
		double U = m0, U2 = m0, sc = 0;
		for(int t = 0; t < nS; ++t) {
			int k = S[t], mj;
			double f = row_min(&D, k, sD, N, &mj, 0);
			double v = f > Q[k] ? f : Q[k];
			U = v < U ? v : U;
			double d = ld(&D, tri(k) + P[k]);
			double qp = 0 <= d ? qval(N[k], N[P[k]], d, sD[k], sD[P[k]]) : DBL_MAX;
			double v2 = qp > Q[k] ? qp : Q[k];
			U2 = v2 < U2 ? v2 : U2;
			same += qp == f;
			sc += k;
		}
		double r1 = 0, c1 = 0, r2 = 0, c2 = 0;
		for(int r = smin - 1; r >= 1 && smin > 1; --r) {
			if(Q[r] < U) {
				r1 += 1;
				c1 += r;
			}
			if(Q[r] < U2) {
				r2 += 1;
				c2 += r;
			}
		}
		two_r += nS + r1;
		two_c += sc + c1;
		one_r += nS + r2;
		one_c += sc + c2;
		rest1 += r1;
		rest2 += r2;
		double m = m0;
		for(int r = n - 1; r >= 1; --r) {
			if(Q[r] < m) {
				int mj;
				double f = row_min(&D, r, sD, N, &mj, 0);
				ref_r += 1;
				ref_c += r;
				if(f < m) m = f;
			}
		}
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
	printf("joins %d, S = top %d rows with Q < m0\n", joins, top);
	printf("reference        : %8.1f rows %12.0f cells per join\n", ref_r / joins, ref_c / joins);
	printf("two-phase (U)    : %8.1f rows %12.0f cells per join (x%.2f), rest %.1f rows\n", two_r / joins, two_c / joins,
	       two_c / ref_c, rest1 / joins);
	printf("one-phase (U2)   : %8.1f rows %12.0f cells per join (x%.2f), rest %.1f rows\n", one_r / joins, one_c / joins,
	       one_c / ref_c, rest2 / joins);
	printf("S rows whose partner cell is their fresh min: %.3f\n", same / (two_r - rest1));
	return 0;
}
