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
#include <stdlib.h>
#include <string.h>
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

void ccq_print_phy(FILE *out, const ccq_ltd *D, char **names, const unsigned char *include,
                   const char *comment, unsigned format, int precision) {
	if(format & 4) {
		fprintf(out, "#%s\n", comment ? comment : "(null)");
	}
	fprintf(out, "%10d\n", D->n);
	int64_t f = 0;
	int row = 0;
	for(int i = 0; row != D->n; ++i) {
		if(include && !include[i]) {
			continue;
		}
		char *name = names[i];
		size_t L = strlen(name);
		if(L && ((name[0] == '"' && name[L - 1] == '"') || (name[0] == '\'' && name[L - 1] == '\''))) {
			name[L - 1] = 0;
			++name;
		}
		name = strip_dir(name);
		if(format & 1) {
			fputs(name, out);
		} else {
			fprintf(out, "%-10.10s", name);
		}
		for(int j = 0; j < row; ++j, ++f) {
			double d = ccq_ltd_get(D, f);
			if(d == (double) ccq_cvt_i32(d)) {
				fprintf(out, "\t%d", ccq_cvt_i32(d));
			} else {
				fprintf(out, "\t%.*f", precision, d);
			}
		}
		fputc('\n', out);
		++row;
	}
}
