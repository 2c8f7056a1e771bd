/* sim_allq.c -- development aid: how many rows a one-phase DNJ search would
 * rescan.  minQpair (dnj.c:43) can only rescan rows with Q[r] < m0 (its start
 * min), so rescanning ALL of them speculatively in one phase (no bound, no
 * second scan) is exact after the replay.  Per join this prints the
 * distribution of that row count and of its cells, beside the serial
 * reference's rescans, on the serial DNJ of oracle/ccoracle.c (Euclidean
 * U[0,1)^8, %.9f).
 * Build: gcc -O2 -std=gnu99 -ffp-contract=off -Ioracle tools/sim_allq.c -lm -lpthread -o /tmp/sim_allq
 *        /tmp/sim_allq N */
#include "../oracle/ccoracle.c"
#include <stdio.h>

static int cmp_d(const void *a, const void *b) {
	double x = *(const double *) a, y = *(const double *) b;
	return x < y ? -1 : x > y;
}

int main(int argc, char **argv) {
	int n = argc > 1 ? atoi(argv[1]) : 2000;
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
	const int n0 = n;
	double *rows = malloc(n0 * sizeof(double)), *cells = malloc(n0 * sizeof(double)), *frac = malloc(n0 * sizeof(double));
	double ref_rows = 0, ref_cells = 0, all_cells = 0, all_rows = 0, lt_cells = 0;
	while(n != 2) {
		double m0 = DBL_MAX;
		if(j && m0 != Q[j]) m0 = Q[j];
		double rr = 0, cc = 0;
		for(int r = n - 1; r >= 1; --r)
			if(Q[r] < m0) {
				rr += 1;
				cc += r;
			}
		/* the reference's rescans */
		double m = m0;
		for(int r = n - 1; r >= 1; --r) {
			if(Q[r] < m) {
				int mj;
				double f = row_min(&D, r, sD, N, &mj, 0);
				ref_rows += 1;
				ref_cells += r;
				if(f < m) m = f;
			}
		}
		rows[joins] = rr;
		cells[joins] = cc;
		frac[joins] = cc / ((double) n * (n - 1) / 2);
		all_rows += rr;
		all_cells += cc;
		lt_cells += (double) n * (n - 1) / 2;
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
	printf("n=%d joins=%d\n", n0, joins);
	printf("reference rescans: %.1f rows/join, %.0f cells/join\n", ref_rows / joins, ref_cells / joins);
	printf("Q<m0 (one phase): %.1f rows/join, %.0f cells/join (x%.2f the reference's cells, %.3f of the LT)\n",
	       all_rows / joins, all_cells / joins, all_cells / ref_cells, all_cells / lt_cells);
	qsort(rows, joins, sizeof(double), cmp_d);
	qsort(cells, joins, sizeof(double), cmp_d);
	qsort(frac, joins, sizeof(double), cmp_d);
	const double ps[] = {0.5, 0.9, 0.99, 0.999, 1.0};
	for(int k = 0; k < 5; ++k) {
		int x = (int) (ps[k] * (joins - 1));
		printf("  p%-5g rows %8.0f cells %12.0f LT-frac %.4f\n", ps[k] * 100, rows[x], cells[x], frac[x]);
	}
	return 0;
}
