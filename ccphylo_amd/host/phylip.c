/*
 * phylip.c -- Phylip distance-matrix reader/writer of the host layer.
 *
 * Reader follows the observable behaviour of ref phy.c:251-507 (loadPhy):
 * optional '#' comment line, a size line whose digits are accumulated, then
 * one row per taxon: name up to the separator, i lower-triangular distances
 * (empty tokens skipped, strtod, anything after the i-th value ignored so
 * full matrices load too, phy.c:489-500).  Name buffers keep the reference's
 * capacity arithmetic (start size, doubling on fill, phy.c:404-437) because
 * Newick child order depends on it (nwck.c:45).
 * Writer follows ref phy.c:59-123 (printphy).
 */
#include <ctype.h>
#include <errno.h>
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>
#include "ccphylo_host.h"
#include "hostint.h"

ccq_names *ccq_names_new(int n, uint32_t init_size) {
	ccq_names *T = ccq_xmalloc(sizeof(ccq_names));
	T->cap = n;
	T->names = ccq_xmalloc((size_t) n * sizeof(ccq_str *));
	for(int i = 0; i < n; ++i) {
		T->names[i] = ccq_new(init_size);
	}
	T->header = ccq_new(64);
	return T;
}

void ccq_names_free(ccq_names *T) {
	if(T) {
		for(int i = 0; i < T->cap; ++i) {
			ccq_free(T->names[i]);
		}
		free(T->names);
		ccq_free(T->header);
		free(T);
	}
}

static void grow_names(ccq_names *T, int n) {
	if(T->cap < n) {
		T->names = ccq_xrealloc(T->names, (size_t) n * sizeof(ccq_str *));
		for(int i = T->cap; i < n; ++i) {
			T->names[i] = ccq_new(32);   /* phy.c:377 */
		}
		T->cap = n;
	}
}

/* store one byte of a growing buffer; doubles the capacity when it fills */
static inline void put_grow(ccq_str *s, uint32_t *w, unsigned char c) {
	s->seq[(*w)++] = c;
	if(*w == s->size) {
		s->size <<= 1;
		s->seq = ccq_xrealloc(s->seq, s->size);
	}
}


static int store_dist(ccq_ltd *D, int64_t f, const char *tok) {
	char *end;
	double v = strtod(tok, &end);
	if(*end != 0) {
		return 0;
	}
	ccq_ltd_set(D, f, v, 0.5);
	return 1;
}

/* ---------------- parallel row parsing ----------------
 * loadPhy (phy.c:251) converts every cell with strtod and is single-threaded;
 * it is most of `ccphylo tree`'s wall time at N = 10k.  Here the rows of a
 * matrix are first located in memory (one newline per row), then parsed by
 * several threads, each cell with the same result as strtod: tokens of the
 * form [-]digits[.digits] with at most 19 significant digits, a mantissa below
 * 2^53 and at most 22 fraction digits are one correctly rounded division
 * m / 10^k (exact operands, so the quotient is the correctly rounded decimal
 * value, which is what glibc's strtod returns); anything else goes to strtod. */
static const double POW10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                                 1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};

static int parse_cell(const char *s, size_t len, double *out) {
	size_t k = 0;
	int neg = 0;
	if(k < len && (s[k] == '-' || s[k] == '+')) {
		neg = s[k] == '-';
		++k;
	}
	uint64_t m = 0;
	int digits = 0, frac = 0, dot = 0, any = 0;
	for(; k < len; ++k) {
		const char c = s[k];
		if(c >= '0' && c <= '9') {
			any = 1;
			if(m || c != '0') ++digits;
			if(digits > 19) goto slow;
			m = m * 10 + (uint64_t) (c - '0');
			frac += dot;
		} else if(c == '.' && !dot) {
			dot = 1;
		} else {
			goto slow;
		}
	}
	if(!any || m >= (1ull << 53) || frac > 22) goto slow;
	{
		double v = (double) m / POW10[frac];
		*out = neg ? -v : v;
		return 1;
	}
slow: {
		char buf[256];
		if(len >= sizeof(buf)) return 0;
		memcpy(buf, s, len);
		buf[len] = 0;
		char *end;
		*out = strtod(buf, &end);
		return *end == 0;
	}
}

typedef struct {
	const char *base;
	const size_t *start;      /* row i spans [start[i], start[i + 1]) (newline excluded) */
	ccq_ltd *D;
	ccq_names *T;
	char sep, quotes;
	int r0, r1;               /* rows of this worker */
	int n;                    /* rows of the matrix */
	int last_eof;             /* the matrix's last row ends at EOF without a newline */
	int bad_row, bad_col;     /* first malformed cell (row -1: none) */
	int bad_eof;              /* ... a token cut by EOF (phy.c's unexpected end of file) */
	char bad_tok[256];
} RowJob;

/* one row exactly as the sequential reader below consumes it */
static void *parse_rows(void *arg) {
	RowJob *J = arg;
	J->bad_row = -1;
	J->bad_eof = 0;
	for(int i = J->r0; i < J->r1; ++i) {
		const char *p = J->base + J->start[i], *e = J->base + J->start[i + 1];
		if(e > p && e[-1] == '\n') --e;
		ccq_str *nm = J->T->names[i];
		uint32_t w = 0;
		if(J->quotes) put_grow(nm, &w, (unsigned char) J->quotes);
		/* the name, terminator included, then trailing blanks dropped */
		for(;;) {
			const unsigned char c = p < e ? (unsigned char) *p : '\n';
			++p;
			put_grow(nm, &w, c);
			if(c == (unsigned char) J->sep || c == '\n') break;
		}
		while(w > 0 && isspace(nm->seq[w - 1])) --w;
		nm->len = w;
		if(J->quotes) {
			nm->seq[w++] = (unsigned char) J->quotes;
			nm->len++;
		}
		nm->seq[w] = 0;
		int64_t f = (int64_t) i * (i - 1) / 2;
		for(int j = 0; j < i; ++j, ++f) {
			const char *t;
			size_t tl;
			int cut = 0;
			do {   /* empty tokens are skipped */
				t = p;
				while(p < e && *p != J->sep) ++p;
				tl = (size_t) (p - t);
				if(p < e) {
					++p;
				} else {
					/* ended by the row end: a newline, or EOF on the last row */
					cut = J->last_eof && i == J->n - 1;
					if(tl == 0) break;
				}
			} while(tl == 0);
			if(cut) {
				J->bad_row = i;
				J->bad_col = j;
				J->bad_eof = 1;
				return NULL;
			}
			double v;
			if(tl == 0 || !parse_cell(t, tl, &v)) {
				J->bad_row = i;
				J->bad_col = j;
				if(tl >= sizeof(J->bad_tok)) tl = sizeof(J->bad_tok) - 1;
				memcpy(J->bad_tok, t, tl);
				J->bad_tok[tl] = 0;
				return NULL;
			}
			ccq_ltd_set(J->D, f, v, 0.5);
		}
	}
	return NULL;
}

static int host_threads(void) {
	const char *e = getenv("OMP_NUM_THREADS");
	long t = e ? atol(e) : sysconf(_SC_NPROCESSORS_ONLN);
	if(t < 1) t = 1;
	return t > 32 ? 32 : (int) t;
}

/* rows of an n-taxon matrix from the reader: slurp up to the n-th newline,
 * parse in parallel; bytes past the matrix go back into the reader */
static double now_s(void) {
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

static int load_rows_parallel(ccq_reader *r, ccq_ltd *D, ccq_names *T, int n, char sep, char quotes, int *err) {
	const int timing = getenv("CCQ_PHY_TIMING") != NULL;
	const double t0 = timing ? now_s() : 0;
	size_t cap = 1 << 24, len = 0;
	char *buf = ccq_xmalloc(cap);
	size_t *start = ccq_xmalloc(((size_t) n + 1) * sizeof(size_t));
	int rows = 0;
	start[0] = 0;
	size_t scan = 0;
	for(;;) {
		/* move the reader's pending bytes into buf */
		size_t avail = r->len - r->pos;
		if(avail) {
			if(len + avail > cap) {
				while(len + avail > cap) cap <<= 1;
				buf = ccq_xrealloc(buf, cap);
			}
			memcpy(buf + len, r->buf + r->pos, avail);
			len += avail;
			r->pos = r->len;
		}
		while(rows < n && scan < len) {
			const char *nl = memchr(buf + scan, '\n', len - scan);
			if(!nl) {
				scan = len;
				break;
			}
			scan = (size_t) (nl - buf) + 1;
			start[++rows] = scan;
		}
		if(rows == n) break;
		if(!ccq_fill(r)) {
			/* EOF: the last row may lack its newline (phy.c:500) */
			if(rows == n - 1 && len > start[rows]) {
				start[++rows] = len;
			}
			break;
		}
	}
	const int last_eof = rows == n && (start[n] == 0 || buf[start[n] - 1] != '\n');
	if(rows < n) {
		fprintf(stderr, "Malformatted phylip file, unexpected end of file, distance pos:\t(%d,%d)\n", rows, 0);
		*err = 1;
		free(buf);
		free(start);
		return 0;
	}
	/* bytes after the matrix stay in the reader for the next one */
	const size_t rest = len - start[n];
	if(rest) {
		if(rest > r->cap) {
			r->cap = rest;
			r->buf = ccq_xrealloc(r->buf, r->cap);
		}
		memcpy(r->buf, buf + start[n], rest);
		r->len = rest;
		r->pos = 0;
	}
	const double t1 = timing ? now_s() : 0;
	int nt = host_threads();
	if(nt > n / 64 + 1) nt = n / 64 + 1;
	RowJob *jobs = ccq_xmalloc((size_t) nt * sizeof(RowJob));
	pthread_t *th = ccq_xmalloc((size_t) nt * sizeof(pthread_t));
	/* equal bytes per worker */
	const size_t total = start[n];
	int row = 0;
	for(int t = 0; t < nt; ++t) {
		jobs[t].base = buf;
		jobs[t].start = start;
		jobs[t].D = D;
		jobs[t].T = T;
		jobs[t].sep = sep;
		jobs[t].quotes = quotes;
		jobs[t].r0 = row;
		jobs[t].n = n;
		jobs[t].last_eof = last_eof;
		const size_t goal = total / nt * (size_t) (t + 1);
		while(row < n && (t == nt - 1 || start[row + 1] <= goal)) ++row;
		jobs[t].r1 = row;
	}
	int started = 0;
	for(int t = 1; t < nt; ++t) {
		if(pthread_create(&th[t], NULL, parse_rows, &jobs[t]) == 0) {
			++started;
		} else {
			parse_rows(&jobs[t]);
			th[t] = 0;
		}
	}
	parse_rows(&jobs[0]);
	for(int t = 1; t < nt; ++t) {
		if(th[t]) pthread_join(th[t], NULL);
	}
	(void) started;
	for(int t = 0; t < nt; ++t) {
		if(jobs[t].bad_row >= 0 && jobs[t].bad_eof) {
			/* the serial reader's EOF inside a distance (returns, no exit) */
			fprintf(stderr, "Malformatted phylip file, unexpected end of file, distance pos:\t(%d,%d)\n",
			        jobs[t].bad_row, jobs[t].bad_col);
			*err = 1;
			free(jobs);
			free(th);
			free(buf);
			free(start);
			return 0;
		}
		if(jobs[t].bad_row >= 0) {
			fprintf(stderr, "Malformatted distance at pos:\t(%d,%d)\n\"%s\"\n", jobs[t].bad_row, jobs[t].bad_col,
			        jobs[t].bad_tok);
			exit(errno | 1);
		}
	}
	if(timing) fprintf(stderr, "# phylip rows: slurp %.3f s, parse %.3f s (%d threads)\n", t1 - t0, now_s() - t1, nt);
	free(jobs);
	free(th);
	free(buf);
	free(start);
	D->n = n;
	return n;
}

int ccq_load_phy(ccq_reader *r, ccq_ltd *D, ccq_names *T, char sep, char quotes, int *err) {
	int c;
	ccq_str *h = T->header;
	*err = 0;
	D->n = 0;
	if((c = ccq_getc(r)) == EOF) {
		return 0;
	}
	if(c == '#') {
		uint32_t w = 0;
		for(;;) {
			if((c = ccq_getc(r)) == EOF) {
				return 0;
			}
			if(c == '\n') {
				break;
			}
			put_grow(h, &w, (unsigned char) c);
		}
		h->seq[w] = 0;
		h->len = w;
		if(ccq_peek(r) == EOF) {
			return 0;
		}
		c = ccq_getc(r);
	} else {
		h->len = 0;
		h->seq[0] = 0;
	}

	/* size line: every digit counts (phy.c:339-351) */
	int n = 0;
	while(c != '\n') {
		if('0' <= c && c <= '9') {
			n = 10 * n + (c - '0');
		}
		if((c = ccq_getc(r)) == EOF) {
			return 0;
		}
	}
	if(ccq_peek(r) == EOF) {
		return 0;
	}
	ccq_ltd_reserve(D, n);
	grow_names(T, n);
	if(n == 0) {
		return 0;
	}
	if(n >= 512 && !getenv("CCQ_SERIAL_PHY")) {
		return load_rows_parallel(r, D, T, n, sep, quotes, err);
	}

	char tok[256];
	for(int i = 0; i < n; ++i) {
		ccq_str *nm = T->names[i];
		uint32_t w = 0;
		if(quotes) {
			put_grow(nm, &w, (unsigned char) quotes);
		}
		do {
			if((c = ccq_getc(r)) == EOF) {
				fprintf(stderr, "Malformatted phylip file, name on row: %d\n", i + 1);
				*err = 1;
				return 0;
			}
			put_grow(nm, &w, (unsigned char) c);
		} while(c != sep && c != '\n');
		while(w > 0 && isspace(nm->seq[w - 1])) {
			--w;
		}
		nm->len = w;
		if(quotes) {
			nm->seq[w++] = (unsigned char) quotes;
			nm->len++;
		}
		nm->seq[w] = 0;

		int64_t f = (int64_t) i * (i - 1) / 2;
		for(int j = i; j--; ++f) {
			int stop = j != 0 ? sep : '\n';
			size_t t = 0;
			while(t == 0) {
				while((c = ccq_getc(r)) != stop && c != sep) {
					if(c == EOF) {
						fprintf(stderr, "Malformatted phylip file, unexpected end of file, distance pos:\t(%d,%d)\n", i, i - j - 1);
						*err = 1;
						return 0;
					}
					if(t < sizeof(tok) - 1) {
						tok[t++] = (char) c;
					}
				}
				tok[t] = 0;
				if(t == 0) {
					/* an empty token is skipped and the next one read instead */
					t = 0;
				}
			}
			if(!store_dist(D, f, tok)) {
				fprintf(stderr, "Malformatted distance at pos:\t(%d,%d)\n\"%s\"\n", i, i - j - 1, tok);
				exit(errno | 1);
			}
		}
		while(c != '\n') {
			if((c = ccq_getc(r)) == EOF) {
				if(i != n - 1) {
					fprintf(stderr, "Malformatted phylip file, missing newline at row:\t%d\n", i);
					*err = 1;
					return 0;
				}
				break;
			}
		}
	}
	D->n = n;
	return n;
}

/* phy.c:33 stripDir */
static char *strip_dir(char *s) {
	char *p = s;
	for(; *p; ++p) {
		if(*p == '/') {
			s = p + 1;
		}
	}
	return s;
}

/* growable text buffer of a writer thread */
typedef struct {
	char *p;
	size_t len, cap;
} Text;

static inline void text_need(Text *t, size_t k) {
	if(t->len + k > t->cap) {
		while(t->len + k > t->cap) t->cap = t->cap ? 2 * t->cap : 1 << 16;
		t->p = ccq_xrealloc(t->p, t->cap);
	}
}

/* "\t%d" without printf (the common integer cells of SNP matrices) */
static inline void text_int(Text *t, int32_t v) {
	char tmp[16];
	int k = 0;
	uint32_t u = v < 0 ? 0u - (uint32_t) v : (uint32_t) v;
	do {
		tmp[k++] = (char) ('0' + u % 10);
		u /= 10;
	} while(u);
	text_need(t, (size_t) k + 2);
	t->p[t->len++] = '\t';
	if(v < 0) t->p[t->len++] = '-';
	while(k) t->p[t->len++] = tmp[--k];
}

typedef struct {
	const ccq_ltd *D;
	char **names;
	const unsigned char *include;
	unsigned format;
	int precision;
	int i0, i1;          /* file indices [i0, i1) */
	int row0;            /* LT row of the first included index */
	Text out;
} PrintJob;

/* phy.c:59-123 printphy for a range of rows, into the job's buffer */
static void *print_rows(void *arg) {
	PrintJob *J = arg;
	int row = J->row0;
	int64_t f = (int64_t) row * (row - 1) / 2;
	char cell[512];
	for(int i = J->i0; i < J->i1; ++i) {
		if(J->include && !J->include[i]) continue;
		char *name = J->names[i];
		size_t L = strlen(name);
		if(L && ((name[0] == '"' && name[L - 1] == '"') || (name[0] == '\'' && name[L - 1] == '\''))) {
			name[L - 1] = 0;
			++name;
		}
		name = strip_dir(name);
		int k = (J->format & 1) ? snprintf(cell, sizeof(cell), "%s", name) : snprintf(cell, sizeof(cell), "%-10.10s", name);
		if(k >= (int) sizeof(cell)) {
			const size_t nl = strlen(name);
			text_need(&J->out, nl);
			memcpy(J->out.p + J->out.len, name, nl);
			J->out.len += nl;
		} else {
			text_need(&J->out, (size_t) k);
			memcpy(J->out.p + J->out.len, cell, (size_t) k);
			J->out.len += (size_t) k;
		}
		for(int j = 0; j < row; ++j, ++f) {
			const double d = ccq_ltd_get(J->D, f);
			if(d == (double) ccq_cvt_i32(d)) {
				text_int(&J->out, ccq_cvt_i32(d));
			} else {
				k = snprintf(cell, sizeof(cell), "\t%.*f", J->precision, d);
				if(k >= (int) sizeof(cell)) {
					/* huge values at high precision: format into a right-sized buffer */
					char *big = ccq_xmalloc((size_t) k + 1);
					snprintf(big, (size_t) k + 1, "\t%.*f", J->precision, d);
					text_need(&J->out, (size_t) k);
					memcpy(J->out.p + J->out.len, big, (size_t) k);
					free(big);
				} else {
					text_need(&J->out, (size_t) k);
					memcpy(J->out.p + J->out.len, cell, (size_t) k);
				}
				J->out.len += (size_t) k;
			}
		}
		text_need(&J->out, 1);
		J->out.p[J->out.len++] = '\n';
		++row;
	}
	return NULL;
}

/* phy.c:59 printphy: rows formatted by several threads (equal cells each),
 * written in order -- the same bytes as one fprintf loop */
void ccq_print_phy(FILE *out, const ccq_ltd *D, char **names, const unsigned char *include,
                   const char *comment, unsigned format, int precision) {
	if(format & 4) {
		fprintf(out, "#%s\n", comment ? comment : "(null)");
	}
	fprintf(out, "%10d\n", D->n);
	const int n = D->n;
	/* file indices of the included rows */
	int *idx = ccq_xmalloc(((size_t) n + 1) * sizeof(int));
	for(int i = 0, r = 0; r < n; ++i) {
		if(include && !include[i]) continue;
		idx[r++] = i;
	}
	int nt = n >= 256 ? host_threads() : 1;
	if(nt > n / 32 + 1) nt = n / 32 + 1;
	PrintJob *jobs = calloc((size_t) nt, sizeof(PrintJob));
	pthread_t *th = calloc((size_t) nt, sizeof(pthread_t));
	const double cells = (double) n * (n - 1) / 2;
	int r = 0;
	for(int t = 0; t < nt; ++t) {
		PrintJob *J = &jobs[t];
		J->D = D;
		J->names = names;
		J->include = include;
		J->format = format;
		J->precision = precision;
		J->row0 = r;
		/* rows [r, r1) with about cells * (t + 1) / nt cells below r1 */
		int r1 = t == nt - 1 ? n : (int) (0.5 + sqrt(2.0 * cells * (t + 1) / nt));
		if(r1 < r) r1 = r;
		if(r1 > n) r1 = n;
		J->i0 = r < n ? idx[r] : (n ? idx[n - 1] + 1 : 0);
		J->i1 = r1 < n ? idx[r1] : (n ? idx[n - 1] + 1 : 0);
		r = r1;
	}
	for(int t = 1; t < nt; ++t) {
		if(pthread_create(&th[t], NULL, print_rows, &jobs[t]) != 0) {
			print_rows(&jobs[t]);
			th[t] = 0;
		}
	}
	if(nt) print_rows(&jobs[0]);
	for(int t = 0; t < nt; ++t) {
		if(t && th[t]) pthread_join(th[t], NULL);
	}
	for(int t = 0; t < nt; ++t) {
		if(jobs[t].out.len) fwrite(jobs[t].out.p, 1, jobs[t].out.len, out);
		free(jobs[t].out.p);
	}
	free(jobs);
	free(th);
	free(idx);
}

/* the name field ccq_print_phy writes (quotes stripped, directories dropped,
 * padded / cut to 10 unless format bit 1), stored as ccq_load_phy reads it */
void ccq_names_set(ccq_names *T, char **names, int n, unsigned format, char sep) {
	grow_names(T, n);
	char cell[512];
	for(int i = 0; i < n; ++i) {
		const size_t L0 = strlen(names[i]);
		char *tmp = ccq_xmalloc(L0 + 1), *name = tmp;
		memcpy(tmp, names[i], L0 + 1);
		if(L0 && ((name[0] == '"' && name[L0 - 1] == '"') || (name[0] == '\'' && name[L0 - 1] == '\''))) {
			name[L0 - 1] = 0;
			++name;
		}
		name = strip_dir(name);
		const char *field = name;
		if(!(format & 1)) {
			snprintf(cell, sizeof(cell), "%-10.10s", name);
			field = cell;
		}
		ccq_str *nm = T->names[i];
		uint32_t w = 0;
		for(const char *p = field; *p; ++p) put_grow(nm, &w, (unsigned char) *p);
		put_grow(nm, &w, (unsigned char) (i ? sep : '\n'));   /* row 0 has no cells: its name ends the line */
		while(w > 0 && isspace(nm->seq[w - 1])) --w;
		nm->len = w;
		nm->seq[w] = 0;
		free(tmp);
	}
	T->header->len = 0;
	T->header->seq[0] = 0;
}
