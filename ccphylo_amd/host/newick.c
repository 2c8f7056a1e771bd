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
 *
 * Two replays give the same bytes:
 *   - ccq_replay_newick_strings edits the strings as the reference does: a
 *     one-byte shift of the left string and an append per join, O(length of
 *     the growing strings) per join, O(N^2) bytes for caterpillar trees;
 *   - ccq_replay_newick first replays only (capacity,
 *     length) per name slot to decide every child order, recording the joins
 *     as a tree, then writes the final string once by an explicit-stack walk:
 *     O(N + output) for any shape.
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

void ccq_replay_newick_strings(ccq_names *T, int n0, const ccq_join *joins, int njoins,
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

/* ------------------------------------------------------------------ */
/* O(N + output) replay: symbolic (size, len) pass + one serialization  */
/* ------------------------------------------------------------------ */
enum { NW_LEAF = 0, NW_NODE = 1, NW_LAST = 2, NW_BI = 3 };

typedef struct {
	int kind;
	int a, b;                 /* child node ids (leaves are 0 .. n0-1) */
	int64_t ta, tb;           /* pool offsets of the ":<length>" texts, -1 = none */
	uint32_t la, lb;          /* their lengths */
} nw_node;

typedef struct {
	char *p;
	size_t len, cap;
} nw_pool;

static int64_t pool_text(nw_pool *P, int prec, double L, uint32_t *tlen) {
	int need = snprintf(NULL, 0, ":%.*f", prec, L);
	if(P->len + (size_t) need + 1 > P->cap) {
		P->cap = (P->len + (size_t) need + 1) * 2;
		P->p = ccq_xrealloc(P->p, P->cap);
	}
	snprintf(P->p + P->len, (size_t) need + 1, ":%.*f", prec, L);
	int64_t off = (int64_t) P->len;
	P->len += (size_t) need;
	*tlen = (uint32_t) need;
	return off;
}

typedef struct {
	uint32_t size, len;       /* the slot's Qseqs capacity and length, as the reference has them */
	int node;
} nw_slot;

/* serialization stack entry: a node, one byte, a pool text, or a backspace */
enum { NW_E_NODE = 0, NW_E_CHAR = 1, NW_E_TEXT = 2, NW_E_BACK = 3 };
typedef struct {
	int kind;
	uint32_t len;
	int64_t v;
} nw_ent;

static void two_children(nw_node *z, nw_slot *x, nw_slot *y, nw_pool *P, int prec, double L1, double L2) {
	z->a = x->node;
	z->b = y->node;
	z->ta = z->tb = -1;
	z->la = z->lb = 0;
	if(!(L1 < 0 && L2 < 0)) {
		z->ta = pool_text(P, prec, L1, &z->la);
		z->tb = pool_text(P, prec, L2, &z->lb);
	}
	x->len += 1 + 1 + y->len + 1 + z->la + z->lb;     /* '(' A ta ',' B tb ')' */
}

void ccq_replay_newick(ccq_names *T, int n0, const ccq_join *joins, int njoins,
                       int final_n, double final_d, int flags, int precision) {
	(void) final_n;
	ccq_str **names = T->names;
	const int max_nodes = n0 + njoins + n0 + 2;
	nw_node *nd = ccq_xmalloc((size_t) max_nodes * sizeof(nw_node));
	nw_slot *sl = ccq_xmalloc((size_t) (n0 > 0 ? n0 : 1) * sizeof(nw_slot));
	ccq_str **leaf = ccq_xmalloc((size_t) (n0 > 0 ? n0 : 1) * sizeof(ccq_str *));
	nw_pool P = {NULL, 0, 0};
	int nn = n0;
	for(int k = 0; k < n0; ++k) {
		nd[k].kind = NW_LEAF;
		leaf[k] = names[k];
		sl[k].size = names[k]->size;
		sl[k].len = names[k]->len;
		sl[k].node = k;
	}
	/* formNode(node1 = slot j, node2 = slot i, L1 = Lj, L2 = Li), nwck.c:35 */
	int n = n0;
	for(int k = 0; k < njoins; ++k) {
		nw_slot *x = &sl[joins[k].j], *y = &sl[joins[k].i];
		double L1 = joins[k].Lj, L2 = joins[k].Li;
		if(x->size < y->size) {          /* nwck.c:45-50: the contents trade places */
			nw_slot t = *x;
			*x = *y;
			*y = t;
			double tl = L1;
			L1 = L2;
			L2 = tl;
		}
		uint32_t want = x->len + y->len + 32;
		if(x->size < want) x->size = want;
		nd[nn].kind = NW_NODE;
		two_children(&nd[nn], x, y, &P, precision, L1, L2);
		x->node = nn++;
		/* the row exchange (dnj.c:1021-1024) */
		--n;
		nw_slot t = sl[joins[k].i];
		sl[joins[k].i] = sl[n];
		sl[n] = t;
		ccq_str *ts = names[joins[k].i];
		names[joins[k].i] = names[n];
		names[n] = ts;
	}
	/* closing nodes: formLastNode / formLastBiNode (nwck.c:79 / :114) */
	const int m = n == 2 ? 1 : n - 1;
	for(int c = 0; c < m; ++c) {
		const int bslot = n == 2 ? 1 : n - 1 - c;
		const double L = n == 2 ? final_d : -1.0;
		nw_slot *x = &sl[0], *y = &sl[bslot];
		if(x->size < y->size) {
			nw_slot t = *x;
			*x = *y;
			*y = t;
		}
		uint32_t want = x->len + y->len + 32;
		if(x->size < want) x->size = want;
		nw_node *z = &nd[nn];
		if(flags & 1) {
			z->kind = NW_BI;
			two_children(z, x, y, &P, precision, L < 0 ? -1.0 : L / 2, L < 0 ? -1.0 : L / 2);
		} else {
			z->kind = NW_LAST;
			z->a = x->node;
			z->b = y->node;
			z->ta = -1;
			z->la = 0;
			z->tb = -1;
			z->lb = 0;
			if(L >= 0) z->tb = pool_text(&P, precision, L, &z->lb);
			x->len += 1 + y->len + z->lb + 1 - 1;     /* drop one byte, then ',' B tb ')' */
		}
		x->node = nn++;
	}
	/* one pass over the join tree, explicit stack (depth up to N for caterpillars) */
	const size_t out_len = sl[0].len;
	size_t cap = (size_t) sl[0].size > out_len + 2 ? (size_t) sl[0].size : out_len + 2;
	unsigned char *out = ccq_xmalloc(cap);
	size_t o = 0;
	nw_ent *st = ccq_xmalloc((size_t) (6 * (size_t) (nn - n0) + 8) * sizeof(nw_ent));
	size_t sp = 0;
	st[sp++] = (nw_ent) {NW_E_NODE, 0, sl[0].node};
	while(sp) {
		nw_ent e = st[--sp];
		if(e.kind == NW_E_CHAR) {
			out[o++] = (unsigned char) e.v;
		} else if(e.kind == NW_E_TEXT) {
			memcpy(out + o, P.p + e.v, e.len);
			o += e.len;
		} else if(e.kind == NW_E_BACK) {
			if(o) --o;
		} else {
			const nw_node *z = &nd[e.v];
			if(z->kind == NW_LEAF) {
				memcpy(out + o, leaf[e.v]->seq, leaf[e.v]->len);
				o += leaf[e.v]->len;
				continue;
			}
			st[sp++] = (nw_ent) {NW_E_CHAR, 0, ')'};
			if(z->tb >= 0) st[sp++] = (nw_ent) {NW_E_TEXT, z->lb, z->tb};
			st[sp++] = (nw_ent) {NW_E_NODE, 0, z->b};
			st[sp++] = (nw_ent) {NW_E_CHAR, 0, ','};
			if(z->kind == NW_LAST) {
				st[sp++] = (nw_ent) {NW_E_BACK, 0, 0};
			} else {
				if(z->ta >= 0) st[sp++] = (nw_ent) {NW_E_TEXT, z->la, z->ta};
				out[o++] = '(';
			}
			st[sp++] = (nw_ent) {NW_E_NODE, 0, z->a};
		}
	}
	out[o] = 0;
	/* The name table outlives the tree (tree.c:61-66): the next matrix's names
	 * are read into these buffers, and their capacities decide its child
	 * orders, so every slot leaves with the capacity the reference's buffer
	 * would have. */
	for(int k = 1; k < n0; ++k) {
		ccq_str *q = names[k];
		if(q->size < sl[k].size) q->seq = ccq_xrealloc(q->seq, sl[k].size);
		q->size = sl[k].size;
		q->len = 0;
		q->seq[0] = 0;
	}
	ccq_str *r = names[0];
	free(r->seq);
	r->seq = out;
	r->len = (uint32_t) o;
	r->size = sl[0].size;
	if(r->seq[0] != '(') prepend(r, '(');     /* dnj.c:1047-1049 */
	free(st);
	free(P.p);
	free(sl);
	free(leaf);
	free(nd);
}
