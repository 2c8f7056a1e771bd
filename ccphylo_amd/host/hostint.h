/* hostint.h -- internals shared by the host-layer translation units */
#ifndef CCPHYLO_HOSTINT_H
#define CCPHYLO_HOSTINT_H
#include <stdint.h>
#include <stdio.h>
#include <zlib.h>

struct ccq_reader {
	gzFile gz;
	unsigned char *buf;
	size_t cap, len, pos;
	int eof;
	char *path;      /* NULL for stdin; bulk readers re-open a plain file (fasta_par.c) */
};

void *ccq_xmalloc(size_t n);
void *ccq_xrealloc(void *p, size_t n);
int ccq_fill(struct ccq_reader *r);

/* next byte or EOF */
static inline int ccq_getc(struct ccq_reader *r) {
	if(r->pos == r->len && !ccq_fill(r)) {
		return EOF;
	}
	return r->buf[r->pos++];
}

/* x86-64 lowering of (unsigned short/char) = double in the reference build:
 * cvttsd2si to a 32-bit int (INT_MIN when out of range), then a narrowing
 * store.  The GPU kernels implement the same function (dtouc in bytescale.h). */
static inline int32_t ccq_cvt_i32(double x) {
	if(!(x > -2147483649.0 && x < 2147483648.0)) {
		return INT32_MIN;
	}
	return (int32_t) x;
}

#endif
