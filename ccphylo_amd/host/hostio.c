/*
 * hostio.c -- strings, readers and the packed LT container of the host layer.
 *
 * ref: qseqs.c:24 setQseqs (capacity field), filebuff.c:52 openAndDetermine
 * (gzip autodetect; here zlib's transparent gzread), matrix.c:32 ltdMatrixInit
 * (row i of the strictly-lower-triangular matrix starts at i(i-1)/2).
 */
#include <stdlib.h>
#include <string.h>
#include <zlib.h>
#include "ccphylo_host.h"
#include "hostint.h"

void *ccq_xmalloc(size_t n) {
	void *p = malloc(n ? n : 1);
	if(!p) {
		fprintf(stderr, "Error: out of host memory (%zu bytes)\n", n);
		exit(12);
	}
	return p;
}

void *ccq_xrealloc(void *p, size_t n) {
	p = realloc(p, n ? n : 1);
	if(!p) {
		fprintf(stderr, "Error: out of host memory (%zu bytes)\n", n);
		exit(12);
	}
	return p;
}

ccq_str *ccq_new(uint32_t size) {
	ccq_str *s = ccq_xmalloc(sizeof(ccq_str));
	s->size = size;
	s->len = 0;
	s->seq = ccq_xmalloc(size);
	s->seq[0] = 0;
	return s;
}

void ccq_free(ccq_str *s) {
	if(s) {
		free(s->seq);
		free(s);
	}
}

/* ---------------- reader ---------------- */
ccq_reader *ccq_open(const char *path) {
	ccq_reader *r = ccq_xmalloc(sizeof(ccq_reader));
	r->path = NULL;
	if(path[0] == '-' && path[1] == 0) {
		r->gz = gzdopen(0, "rb");
	} else {
		r->gz = gzopen(path, "rb");
		r->path = strdup(path);
	}
	if(!r->gz) {
		free(r->path);
		free(r);
		return NULL;
	}
	gzbuffer(r->gz, 1 << 20);
	r->cap = 1 << 20;
	r->buf = ccq_xmalloc(r->cap);
	r->len = 0;
	r->pos = 0;
	r->eof = 0;
	return r;
}

int ccq_fill(ccq_reader *r) {
	if(r->eof) {
		return 0;
	}
	int got = gzread(r->gz, r->buf, (unsigned) r->cap);
	if(got <= 0) {
		r->eof = 1;
		r->len = r->pos = 0;
		return 0;
	}
	r->len = (size_t) got;
	r->pos = 0;
	return 1;
}

void ccq_close(ccq_reader *r) {
	if(r) {
		gzclose(r->gz);
		free(r->buf);
		free(r->path);
		free(r);
	}
}

int ccq_peek(ccq_reader *r) {
	if(r->pos == r->len && !ccq_fill(r)) {
		return EOF;
	}
	return r->buf[r->pos];
}

/* ---------------- packed LT container ---------------- */
static size_t lt_bytes(int size, int et) {
	return size > 1 ? (size_t) size * (size_t) (size - 1) / 2 * (size_t) et : (size_t) et;
}

ccq_ltd *ccq_ltd_new(int size, int et, double bs) {
	ccq_ltd *D = ccq_xmalloc(sizeof(ccq_ltd));
	D->n = 0;
	D->size = size;
	D->et = et;
	D->bs = bs;
	D->mat = ccq_xmalloc(lt_bytes(size, et));
	return D;
}

void ccq_ltd_free(ccq_ltd *D) {
	if(D) {
		free(D->mat);
		free(D);
	}
}

void ccq_ltd_reserve(ccq_ltd *D, int size) {
	if(D->size < size) {
		D->mat = ccq_xrealloc(D->mat, lt_bytes(size, D->et));
		D->size = size;
	}
}

double ccq_ltd_get(const ccq_ltd *D, int64_t f) {
	switch(D->et) {
		case 8: return ((double *) D->mat)[f];
		case 4: return ((float *) D->mat)[f];
		case 2: return ((uint16_t *) D->mat)[f] / D->bs;
		default: return ((uint8_t *) D->mat)[f] / D->bs;
	}
}

void ccq_ltd_set(ccq_ltd *D, int64_t f, double v, double round) {
	switch(D->et) {
		case 8: ((double *) D->mat)[f] = v; break;
		case 4: ((float *) D->mat)[f] = (float) v; break;
		case 2: ((uint16_t *) D->mat)[f] = (uint16_t) ccq_cvt_i32(v * D->bs + round); break;
		default: ((uint8_t *) D->mat)[f] = (uint8_t) ccq_cvt_i32(v * D->bs + round); break;
	}
}
