/*
 * kma_oracle.c -- plain-C restatement of ccphylo 0.8.5's count-matrix
 * (KMA *.mat) distance path, SURVEY rows B1/B2.
 *
 * TEST INFRASTRUCTURE ONLY (see ccoracle.h): the checker of the GPU engine's
 * ccg_kma_ltd and of the host loader; pinned by golden vectors of the
 * reference binary (tests/golden/gen_golden.py, "kma_*" cases).
 *
 * Restated behaviour, including the reference's quirks:
 *   - row parsing (matparse.c:45 FileBuffGetRow, :213 FileBuffLoadMat):
 *     fields after the ref byte are A C G T N -, stored as A C G T - N;
 *     counts truncate to u16, the total keeps the full sum;
 *   - stripMat (matcmp.c:27) compacts a row-sample's buffer with a 7-short
 *     stride although rows are 8 shorts, and without insertion rows it leaves
 *     len = rows + 1;
 *   - the metrics (matcmp.c:63-446) in their exact operation order, with int
 *     products that wrap (x86), nlinf comparing component 0 only, nln raising
 *     the first difference without |.|, nc resetting its denominator;
 *   - cmpMats (matcmp.c:448) and the inclusion rules of ltdMatrixThrd
 *     (ltdmatrixthrd.c:376-562): the first sample is checked over its rows
 *     with ref != '-', later ones over all rows.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>
#include "ccoracle.h"

/* ------------------------------------------------------------------ */
/* input: whole decompressed file                                      */
/* ------------------------------------------------------------------ */
typedef struct {
	unsigned char *p;
	size_t n;
} Blob;

static int blob_load(const char *path, Blob *b) {
	gzFile g = gzopen(path, "rb");
	size_t cap = 1 << 20;
	b->n = 0;
	b->p = NULL;
	if(!g) return -1;
	b->p = malloc(cap);
	for(;;) {
		if(b->n == cap) {
			cap *= 2;
			b->p = realloc(b->p, cap);
		}
		int got = gzread(g, b->p + b->n, (unsigned) (cap - b->n));
		if(got <= 0) break;
		b->n += (size_t) got;
	}
	gzclose(g);
	return 0;
}

/* FileBuffSkipTemplate (matparse.c:142) + name compare: offset of the first
 * row of template `tmpl`, or -1 */
static long find_template(const Blob *b, const char *tmpl) {
	size_t k = 0;
	const size_t tl = strlen(tmpl);
	while(k < b->n) {
		while(k < b->n && b->p[k] != '#') ++k;
		if(k >= b->n) return -1;
		size_t s = ++k;
		while(k < b->n && b->p[k] != '\n') ++k;
		if(k >= b->n) return -1;
		if(k - s == tl && memcmp(b->p + s, tmpl, tl) == 0) return (long) (k + 1);
		++k;
	}
	return -1;
}

typedef struct {
	unsigned char ref;
	uint16_t c[6];     /* A C G T - N */
	uint32_t tot;
} Row;

/* one row at *pos; 0 at a blank line, a '#' line or EOF */
static int next_row(const Blob *b, size_t *pos, Row *r) {
	size_t k = *pos;
	if(k >= b->n) return 0;
	if(b->p[k] == '\n' || b->p[k] == '#') return 0;
	r->ref = b->p[k++];
	uint32_t f[8] = {0};
	int nf = -1;
	int num = 0;
	while(k < b->n && b->p[k] != '\n') {
		const unsigned char ch = b->p[k++];
		if(ch == '\t') {
			if(nf >= 0 && nf < 8) f[nf] = (uint32_t) num;
			++nf;
			num = 0;
		} else {
			num = 10 * num + (ch - '0');
		}
	}
	if(nf >= 0 && nf < 8) f[nf] = (uint32_t) num;
	++k;   /* the '\n' */
	r->tot = f[0] + f[1] + f[2] + f[3] + f[4] + f[5];
	r->c[0] = (uint16_t) f[0];
	r->c[1] = (uint16_t) f[1];
	r->c[2] = (uint16_t) f[2];
	r->c[3] = (uint16_t) f[3];
	r->c[4] = (uint16_t) f[5];
	r->c[5] = (uint16_t) f[4];
	*pos = k;
	return 1;
}

/* ------------------------------------------------------------------ */
/* metrics (matcmp.c), each in the reference's operation order          */
/* ------------------------------------------------------------------ */
static inline int imul(int a, int b) { return (int) ((unsigned) a * (unsigned) b); }

static double m_cos(const uint16_t *x, const uint16_t *y) {   /* matcmp.c:420 */
	int a = x[0], b = y[0];
	unsigned long c1 = (unsigned long) (long) imul(a, a), c2 = (unsigned long) (long) imul(b, b);
	double d = imul(a, b);
	for(int k = 1; k < 5; ++k) {
		a = x[k];
		b = y[k];
		d += imul(a, b);
		c1 += (unsigned long) (long) imul(a, a);
		c2 += (unsigned long) (long) imul(b, b);
	}
	if(!c1 || !c2) return -1;
	d = 1 - d / (sqrt((double) c1) * sqrt((double) c2));
	return d < 0 ? 0 : d;
}

static double m_l1(const uint16_t *x, const uint16_t *y) {    /* matcmp.c:143 */
	int s = abs(x[0] - y[0]);
	for(int k = 1; k < 5; ++k) s += abs(x[k] - y[k]);
	return s;
}

static double m_l2(const uint16_t *x, const uint16_t *y) {    /* matcmp.c:158 */
	int t = x[0] - y[0], s = imul(t, t);
	for(int k = 1; k < 5; ++k) {
		t = x[k] - y[k];
		s += imul(t, t);
	}
	return sqrt(s);
}

static double m_ln(const uint16_t *x, const uint16_t *y, unsigned n) {   /* matcmp.c:173 */
	double d = pow(abs(x[0] - y[0]), n);
	for(int k = 1; k < 5; ++k) d += pow(abs(x[k] - y[k]), n);
	d = pow(d, 1.0 / n);
	return d < 0 ? 0 : d;
}

static double m_linf(const uint16_t *x, const uint16_t *y) {  /* matcmp.c:193 */
	int m = abs(x[0] - y[0]);
	for(int k = 1; k < 5; ++k) {
		if(m < abs(x[k] - y[k])) m = abs(x[k] - y[k]);
	}
	return m;
}

/* the "normalized" metrics divide by the total without N (slot 5) */
static double m_nl1(const uint16_t *x, const uint16_t *y, int t1, int t2) {   /* matcmp.c:63 */
	t1 -= x[5];
	t2 -= y[5];
	double d = 0;
	for(int k = 0; k < 5; ++k) {
		double t = (double) x[k] / t1 - (double) y[k] / t2;
		t = t < 0 ? -t : t;
		d = k ? d + t : t;
	}
	return d;
}

static double m_nl2(const uint16_t *x, const uint16_t *y, int t1, int t2) {   /* matcmp.c:81 */
	t1 -= x[5];
	t2 -= y[5];
	double d = 0;
	for(int k = 0; k < 5; ++k) {
		double t = (double) x[k] / t1 - (double) y[k] / t2;
		d = k ? d + t * t : t * t;
	}
	return sqrt(d);
}

static double m_nln(const uint16_t *x, const uint16_t *y, int t1, int t2, unsigned n) {   /* matcmp.c:98 */
	t1 -= x[5];
	t2 -= y[5];
	double d = pow((double) x[0] / t1 - (double) y[0] / t2, n);   /* no |.| on the first term */
	for(int k = 1; k < 5; ++k) {
		double t = (double) x[k] / t1 - (double) y[k] / t2;
		t = t < 0 ? -t : t;
		d += pow(t, n);
	}
	d = pow(d, 1.0 / n);
	return d < 0 ? 0 : d;
}

static double m_nlinf(const uint16_t *x, const uint16_t *y, int t1, int t2) {   /* matcmp.c:122 */
	t1 -= x[5];
	t2 -= y[5];
	/* the loop compares component 0 again each time: |x0/t1 - y0/t2| */
	double t = (double) x[0] / t1 - (double) y[0] / t2;
	return t < 0 ? -t : t;
}

static double m_nbc(const uint16_t *x, const uint16_t *y, int t1, int t2) {    /* matcmp.c:206 */
	t1 -= x[5];
	t2 -= y[5];
	double d = 0;
	for(int k = 0; k < 5; ++k) {
		const double a = (double) x[k] / t1, b = (double) y[k] / t2;
		d = k ? d + (a < b ? a : b) : (a < b ? a : b);
	}
	d = 1 - d;
	return d < 0 ? 0 : d;
}

static double m_bc(const uint16_t *x, const uint16_t *y, int t1, int t2) {     /* matcmp.c:227 */
	double d = x[0] < y[0] ? x[0] : y[0];
	for(int k = 1; k < 5; ++k) d += x[k] < y[k] ? x[k] : y[k];
	d /= (t1 - x[5] + t2 - y[5]);
	d = 1 - 2 * d;
	return d < 0 ? 0 : d;
}

static double m_nc(const uint16_t *x, const uint16_t *y, int t1, int t2) {     /* matcmp.c:243 */
	t1 -= x[5];
	t2 -= y[5];
	double a = (double) x[0] / t1, b = (double) y[0] / t2, d, T;
	if(a < b) {
		d = a;
		T = b;
	} else {
		d = b;
		T = a;
	}
	for(int k = 1; k < 5; ++k) {
		a = (double) x[k] / t1;
		b = (double) y[k] / t2;
		T = 1;   /* reset every step */
		if(a < b) {
			d += a;
			T += b;
		} else {
			d += b;
			T += a;
		}
	}
	d = 1 - d / T;
	return d < 0 ? 0 : d;
}

static double m_c(const uint16_t *x, const uint16_t *y) {     /* matcmp.c:278 */
	double d;
	int T;
	if(x[0] < y[0]) {
		d = x[0];
		T = y[0];
	} else {
		d = y[0];
		T = x[0];
	}
	for(int k = 1; k < 5; ++k) {
		if(x[k] < y[k]) {
			d += x[k];
			T += y[k];
		} else {
			d += y[k];
			T += x[k];
		}
	}
	if(!T) return -1;
	d = 1 - d / T;
	return d < 0 ? 0 : d;
}

static double m_chi2(const uint16_t *x, const uint16_t *y) {  /* matcmp.c:381 */
	double d = 0;
	for(int k = 0; k < 5; ++k) {
		const double T = x[k] - y[k];
		if(T != 0) d = k ? d + T * T / (x[k] + y[k]) : T * T / (x[k] + y[k]);
	}
	return sqrt(d);
}

static double m_nchi2(const uint16_t *x, const uint16_t *y, int t1, int t2) {  /* matcmp.c:396 */
	t1 -= x[5];
	t2 -= y[5];
	double d = 0;
	for(int k = 0; k < 5; ++k) {
		const double a = (double) x[k] / t1, b = (double) y[k] / t2, df = a - b;
		if(df != 0) d = k ? d + df * df / (a + b) : df * df / (a + b);
	}
	return sqrt(d);
}

static double metric(int m, unsigned lnorm, const uint16_t *x, const uint16_t *y, int t1, int t2) {
	switch(m) {
		case ORC_KMA_COS: return m_cos(x, y);
		case ORC_KMA_CHI2: return m_chi2(x, y);
		case ORC_KMA_NCHI2: return m_nchi2(x, y, t1, t2);
		case ORC_KMA_NC: return m_nc(x, y, t1, t2);
		case ORC_KMA_C: return m_c(x, y);
		case ORC_KMA_NBC: return m_nbc(x, y, t1, t2);
		case ORC_KMA_BC: return m_bc(x, y, t1, t2);
		case ORC_KMA_NL1: return m_nl1(x, y, t1, t2);
		case ORC_KMA_NL2: return m_nl2(x, y, t1, t2);
		case ORC_KMA_NLINF: return m_nlinf(x, y, t1, t2);
		case ORC_KMA_L1: return m_l1(x, y);
		case ORC_KMA_L2: return m_l2(x, y);
		case ORC_KMA_LINF: return m_linf(x, y);
		case ORC_KMA_LN: return m_ln(x, y, lnorm);
		case ORC_KMA_NLN: return m_nln(x, y, t1, t2, lnorm);
		default: return -1;
	}
}

/* ------------------------------------------------------------------ */
/* row sample (mat1): 8 shorts per row, total in shorts 6-7            */
/* ------------------------------------------------------------------ */
typedef struct {
	uint16_t *buf;     /* 8 * rows shorts */
	unsigned char *refs;
	int rows;          /* rows loaded (FileBuffLoadMat len) */
	int len;           /* after stripMat */
	unsigned nnucs;    /* FileBuffLoadMat nNucs: rows (any ref) with minDepth <= total */
} Mat1;

static int load_mat1(const Blob *b, size_t pos, unsigned minDepth, Mat1 *m) {
	int cap = 1024;
	Row r;
	m->buf = malloc((size_t) cap * 16);
	m->refs = malloc((size_t) cap + 1);
	m->rows = 0;
	m->nnucs = 0;
	while(next_row(b, &pos, &r)) {
		if(m->rows == cap) {
			cap *= 2;
			m->buf = realloc(m->buf, (size_t) cap * 16);
			m->refs = realloc(m->refs, (size_t) cap + 1);
		}
		uint16_t *o = m->buf + 8 * (size_t) m->rows;
		memcpy(o, r.c, 12);
		memcpy(o + 6, &r.tot, 4);
		m->refs[m->rows++] = r.ref;
		if(minDepth <= r.tot) ++m->nnucs;
	}
	m->refs[m->rows] = 0;
	return 0;
}

/* matcmp.c:27 stripMat, with its 7-short stride */
static void strip_mat1(Mat1 *m) {
	const unsigned char *ref = m->refs;
	int left = m->rows + 1, len = 0;
	while(left && *ref != '-') {
		--left;
		++ref;
		++len;
	}
	if(left) {
		uint16_t *dst = m->buf + 7 * (size_t) len - 1, *src = dst;
		unsigned char *vref = (unsigned char *) ref;
		while(--left) {
			if(*ref != '-') {
				*vref++ = *ref++;
				for(int t = 0; t < 7; ++t) *++dst = *++src;
				++len;
			} else {
				++ref;
				src += 7;
			}
		}
	}
	m->len = len;
}

/* ------------------------------------------------------------------ */
/* B1: matcmp.c:448 cmpMats over sample j's rows                       */
/* ------------------------------------------------------------------ */
static double cmp_mats(const Mat1 *m1, const Blob *b, size_t pos, int metric_id, unsigned lnorm, unsigned norm,
                       unsigned minDepth, unsigned minLength, double minCov, uint32_t *ntot) {
	double dist = 0;
	unsigned rowNum = 0, rowsInc = 0, nNucs = 0;
	const uint16_t *c1 = m1->buf;
	Row r;
	while(next_row(b, &pos, &r)) {
		if(r.ref == '-') continue;
		if((unsigned) m1->len < ++rowNum) {
			*ntot = r.tot;   /* mat2->total keeps the current row's */
			return -1;
		}
		if(minDepth <= r.tot) {
			++nNucs;
			uint32_t t1;
			/* rows past the loaded ones (len = rows + 1 without insertions) are zero here */
			if(c1 + 8 <= m1->buf + 8 * (size_t) m1->rows) {
				memcpy(&t1, c1 + 6, 4);
			} else {
				t1 = 0;
			}
			static const uint16_t zero[6] = {0};
			const uint16_t *x = (c1 + 8 <= m1->buf + 8 * (size_t) m1->rows) ? c1 : zero;
			double d;
			if(minDepth <= t1 && 0 <= (d = metric(metric_id, lnorm, x, r.c, (int) t1, (int) r.tot))) {
				dist += d;
				++rowsInc;
			}
		}
		c1 += 8;
	}
	if(nNucs < minLength || nNucs < minCov * rowNum) return -2.0;
	if(rowsInc < minLength || rowsInc < minCov * rowNum) {
		*ntot = 0;
		return -1.0;
	}
	*ntot = rowsInc;
	return norm ? dist / rowsInc * norm : dist;
}

static inline int32_t cvt32(double x) {
	if(!(x > -2147483649.0 && x < 2147483648.0)) return INT32_MIN;
	return (int32_t) x;
}

static void store(int et, double bs, void *M, int64_t f, double v) {
	switch(et) {
		case 8: ((double *) M)[f] = v; break;
		case 4: ((float *) M)[f] = (float) v; break;
		case 2: ((uint16_t *) M)[f] = (uint16_t) cvt32(v * bs + 0.5); break;
		default: ((uint8_t *) M)[f] = (uint8_t) cvt32(v * bs + 0.5); break;
	}
}

/* ------------------------------------------------------------------ */
/* B2: ltdmatrixthrd.c:376 ltdMatrixThrd (t = 1 order)                  */
/* ------------------------------------------------------------------ */
int orc_kma_dist(int nfiles, const char **files, const char *tmpl, int metric_id, unsigned lnorm, unsigned norm,
                 unsigned minDepth, unsigned minLength, double minCov, int etype, double bs, void *D, void *N,
                 unsigned char *include, int *n_out) {
	Blob *blobs = calloc((size_t) nfiles, sizeof(Blob));
	long *start = malloc((size_t) nfiles * sizeof(long));
	int rc = 0, n = 0, i = 0;
	*n_out = 0;
	for(int k = 0; k < nfiles; ++k) {
		include[k] = 1;
		start[k] = -1;
	}
	/* the first sample that holds the template and passes, over its rows with ref != '-' */
	for(; i < nfiles; ++i) {
		if(blob_load(files[i], &blobs[i])) {
			rc = -3;
			goto done;
		}
		start[i] = find_template(&blobs[i], tmpl);
		if(start[i] < 0) {
			include[i] = 0;
			continue;
		}
		size_t pos = (size_t) start[i];
		Row r;
		unsigned cnt = 0, len = 0;
		while(next_row(&blobs[i], &pos, &r)) {
			if(r.ref != '-') {
				++len;
				if(minDepth <= r.tot) ++cnt;
			}
		}
		if(cnt < minLength || cnt < minCov * len) {
			include[i] = 0;
			continue;
		}
		break;
	}
	if(i >= nfiles) goto done;   /* nothing included */
	n = 1;
	/* later samples: loaded whole, checked over all rows, stripped, compared */
	for(++i; i < nfiles; ++i) {
		if(blob_load(files[i], &blobs[i])) {
			rc = -3;
			goto done;
		}
		start[i] = find_template(&blobs[i], tmpl);
		if(start[i] < 0) {
			include[i] = 0;
			continue;
		}
		Mat1 m1;
		load_mat1(&blobs[i], (size_t) start[i], minDepth, &m1);
		if(m1.nnucs < minLength || m1.nnucs < minCov * m1.rows) {
			include[i] = 0;
			free(m1.buf);
			free(m1.refs);
			continue;
		}
		strip_mat1(&m1);
		const int row = n;
		int col = 0;
		for(int s = 0; s < i; ++s) {
			if(!include[s]) continue;
			uint32_t nt = 0;
			const double d = cmp_mats(&m1, &blobs[s], (size_t) start[s], metric_id, lnorm, norm, minDepth,
			                          minLength, minCov, &nt);
			if(d == -2.0) {
				rc = -2;   /* the reference exits(1) here (ltdmatrixthrd.c:337) */
				free(m1.buf);
				free(m1.refs);
				goto done;
			}
			const int64_t f = (int64_t) row * (row - 1) / 2 + col;
			store(etype, bs, D, f, d);
			if(N) store(etype, bs, N, f, (double) nt);
			++col;
		}
		free(m1.buf);
		free(m1.refs);
		++n;
	}
	*n_out = n;
done:
	for(int k = 0; k < nfiles; ++k) free(blobs[k].p);
	free(blobs);
	free(start);
	return rc;
}
