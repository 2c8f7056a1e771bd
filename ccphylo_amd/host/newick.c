/*
 * newick.c -- rebuilds the Newick string from the GPU engine's join list.
 *
 * The engine returns, per join, the rows (i, j) and limb lengths; this file
 * replays what the reference does to the name table around each join
 * (dnj.c:1014-1024, nj.c:1578-1590): formNode(names[j], names[i], Lj, Li),
 * then the row-i <-> last-row name exchange, and finally formLastNode /
 * formLastBiNode plus the leading '(' fix (dnj.c:1036-1049).
 * formNode keeps the buffer with the larger CAPACITY first (nwck.c:45-50),
 * so capacities are modelled exactly (ccq_str.size).
 */
#include <stdlib.h>
#include <string.h>
#include "ccphylo_host.h"
#include "hostint.h"

static void swap_str(ccq_str *a, ccq_str *b) {
	unsigned char *s = a->seq;
	uint32_t z = a->size, l = a->len;
	a->seq = b->seq;
	a->size = b->size;
	a->len = b->len;
	b->seq = s;
	b->size = z;
	b->len = l;
}

static void ensure(ccq_str *a, const ccq_str *b) {
	uint32_t want = a->len + b->len + 32;
	if(a->size < want) {
		a->seq = ccq_xrealloc(a->seq, want);
		a->size = want;
	}
}

/* str.c:51 byteshift: prepend one byte */
static void prepend(ccq_str *a, unsigned char c) {
	memmove(a->seq + 1, a->seq, a->len);
	a->seq[0] = c;
	a->seq[++a->len] = 0;
}

/* the buffer was sized len1 + len2 + 32, enough for two %.*f at the
 * precisions the CLI accepts; snprintf keeps it safe otherwise */
static void append(ccq_str *a, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
#include <stdarg.h>
static void append(ccq_str *a, const char *fmt, ...) {
	va_list ap;
	va_start(ap, fmt);
	int need = vsnprintf(NULL, 0, fmt, ap);
	va_end(ap);
	if(a->len + (uint32_t) need + 1 > a->size) {
		/* the reference would overrun here; grow without touching `size`
		 * semantics beyond what it already reports */
		a->seq = ccq_xrealloc(a->seq, a->len + need + 1);
	}
	va_start(ap, fmt);
	vsprintf((char *) a->seq + a->len, fmt, ap);
	va_end(ap);
	a->len += need;
}

/* nwck.c:35-77 formNode */
static void form_node(ccq_str *a, ccq_str *b, double La, double Lb, int prec) {
	if(a->size < b->size) {
		swap_str(a, b);
		double t = La;
		La = Lb;
		Lb = t;
	}
	ensure(a, b);
	prepend(a, '(');
	if(La < 0 && Lb < 0) {
		append(a, ",%s)", (char *) b->seq);
	} else {
		append(a, ":%.*f,%s:%.*f)", prec, La, (char *) b->seq, prec, Lb);
	}
}

/* nwck.c:79-112 formLastNode */
static void form_last_node(ccq_str *a, ccq_str *b, double L, int prec) {
	if(a->size < b->size) {
		swap_str(a, b);
	}
	ensure(a, b);
	a->seq[--a->len] = 0;
	if(L < 0) {
		append(a, ",%s)", (char *) b->seq);
	} else {
		append(a, ",%s:%.*f)", (char *) b->seq, prec, L);
	}
}

/* nwck.c:114-153 formLastBiNode */
static void form_last_bi_node(ccq_str *a, ccq_str *b, double L, int prec) {
	if(a->size < b->size) {
		swap_str(a, b);
	}
	ensure(a, b);
	prepend(a, '(');
	if(L < 0) {
		append(a, ",%s)", (char *) b->seq);
	} else {
		L /= 2;
		append(a, ":%.*f,%s:%.*f)", prec, L, (char *) b->seq, prec, L);
	}
}

void ccq_newick_pair(ccq_names *T, double d, int precision) {
	form_last_bi_node(T->names[0], T->names[1], d, precision);
}

void ccq_replay_newick(ccq_names *T, int n0, const ccq_join *joins, int njoins,
                       int final_n, double final_d, int flags, int precision) {
	ccq_str **names = T->names;
	int n = n0;
	for(int k = 0; k < njoins; ++k) {
		int i = joins[k].i, j = joins[k].j;
		form_node(names[j], names[i], joins[k].Lj, joins[k].Li, precision);
		--n;
		ccq_str *t = names[i];
		names[i] = names[n];
		names[n] = t;
	}
	(void) final_n;
	if(n == 2) {
		if(flags & 1) {
			form_last_bi_node(names[0], names[1], final_d, precision);
		} else {
			form_last_node(names[0], names[1], final_d, precision);
		}
	} else {
		while(n != 1) {
			--n;
			if(flags & 1) {
				form_last_bi_node(names[0], names[n], -1.0, precision);
			} else {
				form_last_node(names[0], names[n], -1.0, precision);
			}
		}
	}
	if(names[0]->seq[0] != '(') {
		prepend(names[0], '(');
	}
}
