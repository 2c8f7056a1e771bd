/*
 * kma.c -- KMA count-matrix (*.mat[.gz]) loader for `ccphylo dist`, the host
 * side of SURVEY rows B1/B2.
 *
 * The reference re-opens and re-parses a sample's file for every pair it is
 * in (ltdmatrixthrd.c:297-317, O(N^2) parses).  Here every file is read once,
 * in parallel (one pthread per file, up to `threads`), and turned into the two
 * views the GPU kernel compares (include/ccphylo_amd.h, ccg_kma_args):
 *   rec1: the sample as cmpMats' mat1 -- all rows as FileBuffLoadMat stores
 *         them (matparse.c:213), then stripMat (matcmp.c:27) applied to that
 *         buffer exactly, 7-short stride included;
 *   rec2: the sample as mat2 -- its rows with ref != '-' (matcmp.c:468).
 * Which samples are included follows ltdMatrixThrd (ltdmatrixthrd.c:376-562):
 * the first sample holding the template is checked over its rows with
 * ref != '-', every later one over all its rows (FileBuffLoadMat's nNucs).
 */
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>
#include "ccphylo_host.h"
#include "hostint.h"

typedef struct {
	const char *path, *tmpl;
	unsigned minDepth;
	int ok;              /* file readable */
	int found;           /* template present */
	int rows;            /* all rows of the template */
	unsigned char *refs; /* rows + 1 (0-terminated like FileBuffLoadMat's) */
	uint16_t *buf;       /* rows x 8: A C G T - N, u32 total */
	unsigned nn_all;     /* rows with minDepth <= total */
	unsigned nn_ins;     /* the same over rows with ref != '-' */
	int len_ins;         /* rows with ref != '-' */
} Sample;

/* whole file through zlib (plain files pass through gzread unchanged) */
static unsigned char *slurp(const char *path, size_t *n) {
	gzFile g = gzopen(path, "rb");
	if(!g) return NULL;
	size_t cap = 1 << 22, len = 0;
	unsigned char *p = ccq_xmalloc(cap + 1);
	for(;;) {
		if(len == cap) {
			cap <<= 1;
			p = ccq_xrealloc(p, cap + 1);
		}
		int got = gzread(g, p + len, (unsigned) (cap - len > (1u << 30) ? (1u << 30) : cap - len));
		if(got <= 0) break;
		len += (size_t) got;
	}
	gzclose(g);
	p[len] = 0;
	*n = len;
	return p;
}

/* matparse.c:45 FileBuffGetRow field order: after the ref byte the fields are
 * A C G T N -; counts keep A C G T - N (u16), the total is the full sum */
static void parse_sample(Sample *s) {
	size_t n = 0;
	unsigned char *p = slurp(s->path, &n);
	s->ok = p != NULL;
	s->found = 0;
	s->rows = 0;
	if(!p) return;
	const size_t tl = strlen(s->tmpl);
	size_t k = 0;
	/* FileBuffSkipTemplate (matparse.c:142): next '#', then the name line */
	while(k < n) {
		const unsigned char *h = memchr(p + k, '#', n - k);
		if(!h) break;
		size_t a = (size_t) (h - p) + 1;
		const unsigned char *e = memchr(p + a, '\n', n - a);
		if(!e) break;
		size_t b = (size_t) (e - p);
		k = b + 1;
		if(b - a == tl && !memcmp(p + a, s->tmpl, tl)) {
			s->found = 1;
			break;
		}
	}
	if(!s->found) {
		free(p);
		return;
	}
	int cap = 4096;
	s->buf = ccq_xmalloc((size_t) cap * 16);
	s->refs = ccq_xmalloc((size_t) cap + 1);
	s->nn_all = s->nn_ins = 0;
	s->len_ins = 0;
	/* rows until a blank line, a '#' line or EOF */
	while(k < n && p[k] != '\n' && p[k] != '#') {
		if(s->rows == cap) {
			cap <<= 1;
			s->buf = ccq_xrealloc(s->buf, (size_t) cap * 16);
			s->refs = ccq_xrealloc(s->refs, (size_t) cap + 1);
		}
		const unsigned char ref = p[k++];
		uint32_t f[6] = {0, 0, 0, 0, 0, 0};
		int fi = -1, num = 0;
		for(; k < n && p[k] != '\n'; ++k) {
			if(p[k] == '\t') {
				if(fi >= 0 && fi < 6) f[fi] = (uint32_t) num;
				++fi;
				num = 0;
			} else {
				num = 10 * num + (p[k] - '0');
			}
		}
		if(fi >= 0 && fi < 6) f[fi] = (uint32_t) num;
		++k;
		uint16_t *o = s->buf + 8 * (size_t) s->rows;
		const uint32_t tot = f[0] + f[1] + f[2] + f[3] + f[4] + f[5];
		o[0] = (uint16_t) f[0];
		o[1] = (uint16_t) f[1];
		o[2] = (uint16_t) f[2];
		o[3] = (uint16_t) f[3];
		o[4] = (uint16_t) f[5];
		o[5] = (uint16_t) f[4];
		memcpy(o + 6, &tot, 4);
		s->refs[s->rows++] = ref;
		const int deep = s->minDepth <= tot;
		s->nn_all += deep;
		if(ref != '-') {
			s->nn_ins += deep;
			++s->len_ins;
		}
	}
	s->refs[s->rows] = 0;
	free(p);
}

/* matcmp.c:27 stripMat on a copy of the loaded buffer: rows with ref '-' are
 * squeezed out with a 7-short stride (the reference's rows are 8 shorts), and
 * without any such row the length comes out one larger.  Returns the length. */
static int strip_rows(const Sample *s, uint16_t *out) {
	memcpy(out, s->buf, (size_t) s->rows * 16);
	int left = s->rows + 1, len = 0;
	const unsigned char *ref = s->refs;
	while(left && *ref != '-') {
		--left;
		++ref;
		++len;
	}
	if(left) {
		uint16_t *dst = out + 7 * (size_t) len - 1;
		const uint16_t *src = dst;
		while(--left) {
			if(*ref++ != '-') {
				for(int t = 1; t <= 7; ++t) dst[t] = src[t];
				dst += 7;
				src += 7;
				++len;
			} else {
				src += 7;
			}
		}
	}
	return len;
}

typedef struct {
	Sample *s;
	int n, next;
	pthread_mutex_t mu;
} Pool;

static void *pool_run(void *arg) {
	Pool *P = arg;
	for(;;) {
		pthread_mutex_lock(&P->mu);
		const int k = P->next++;
		pthread_mutex_unlock(&P->mu);
		if(k >= P->n) return NULL;
		parse_sample(&P->s[k]);
	}
}

ccq_kma *ccq_load_kma(char **files, int nfiles, const char *tmpl, unsigned minDepth, unsigned minLength,
                      double minCov, int threads, FILE *log) {
	Sample *S = calloc((size_t) (nfiles > 0 ? nfiles : 1), sizeof(Sample));
	ccq_kma *K = calloc(1, sizeof(ccq_kma));
	if(!S || !K) abort();
	for(int k = 0; k < nfiles; ++k) {
		S[k].path = files[k];
		S[k].tmpl = tmpl;
		S[k].minDepth = minDepth;
	}
	Pool P = {S, nfiles, 0, PTHREAD_MUTEX_INITIALIZER};
	if(threads < 1) threads = 1;
	if(threads > nfiles) threads = nfiles;
	pthread_t th[64];
	if(threads > 64) threads = 64;
	int started = 0;
	for(int t = 1; t < threads; ++t) started += pthread_create(&th[started], NULL, pool_run, &P) == 0;
	pool_run(&P);
	for(int t = 0; t < started; ++t) pthread_join(th[t], NULL);

	K->nfiles = nfiles;
	K->include = calloc((size_t) (nfiles > 0 ? nfiles : 1), 1);
	K->status = 0;
	/* ltdmatrixthrd.c:405-455: the first sample that holds the template and
	 * passes over its rows with ref != '-' */
	int first = -1;
	for(int k = 0; k < nfiles && first < 0; ++k) {
		if(!S[k].ok) {
			fprintf(log, "Cannot open file:\t%s\n", files[k]);
			K->status = -3;
			goto done;
		}
		if(!S[k].found) {
			fprintf(log, "Template (\"%s\") is not included in:\t%s\n", tmpl, files[k]);
			continue;
		}
		if(S[k].nn_ins < minLength || S[k].nn_ins < minCov * S[k].len_ins) {
			fprintf(log, "Template (\"%s\") did not exceed threshold for inclusion:\t%s\n", tmpl, files[k]);
			continue;
		}
		first = k;
		K->include[k] = 1;
	}
	/* :458-534: later samples over all their rows */
	for(int k = first < 0 ? nfiles : first + 1; k < nfiles; ++k) {
		if(!S[k].ok) {
			fprintf(log, "Cannot open file:\t%s\n", files[k]);
			K->status = -3;
			goto done;
		}
		if(!S[k].found) {
			fprintf(log, "Template (\"%s\") is not included in:\t%s\n", tmpl, files[k]);
			continue;
		}
		if(S[k].nn_all < minLength || S[k].nn_all < minCov * S[k].rows) {
			fprintf(log, "Template (\"%s\") did not exceed threshold for inclusion:\t%s\n", tmpl, files[k]);
			continue;
		}
		K->include[k] = 1;
	}
	/* the two views of the included samples */
	int n = 0;
	int64_t st1 = 1, st2 = 1;
	for(int k = 0; k < nfiles; ++k) {
		if(!K->include[k]) continue;
		++n;
		if(S[k].rows + 1 > st1) st1 = S[k].rows + 1;
		if(S[k].len_ins > st2) st2 = S[k].len_ins;
	}
	K->n = n;
	K->stride1 = st1;
	K->stride2 = st2;
	K->rec1 = calloc((size_t) (n ? n : 1) * (size_t) st1, 16);
	K->rec2 = calloc((size_t) (n ? n : 1) * (size_t) st2, 16);
	K->len1 = calloc((size_t) (n ? n : 1), 4);
	K->len2 = calloc((size_t) (n ? n : 1), 4);
	K->file_of = calloc((size_t) (n ? n : 1), 4);
	if(!K->rec1 || !K->rec2 || !K->len1 || !K->len2 || !K->file_of) abort();
	for(int k = 0, r = 0; k < nfiles; ++k) {
		if(!K->include[k]) continue;
		K->file_of[r] = k;
		K->len1[r] = strip_rows(&S[k], K->rec1 + (size_t) r * st1 * 8);
		uint16_t *o = K->rec2 + (size_t) r * st2 * 8;
		int m = 0;
		for(int q = 0; q < S[k].rows; ++q) {
			if(S[k].refs[q] != '-') memcpy(o + 8 * (size_t) m++, S[k].buf + 8 * (size_t) q, 16);
		}
		K->len2[r] = m;
		++r;
	}
done:
	for(int k = 0; k < nfiles; ++k) {
		free(S[k].buf);
		free(S[k].refs);
	}
	free(S);
	return K;
}

void ccq_kma_free(ccq_kma *K) {
	if(!K) return;
	free(K->include);
	free(K->rec1);
	free(K->rec2);
	free(K->len1);
	free(K->len2);
	free(K->file_of);
	free(K);
}
