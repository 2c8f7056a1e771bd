/*
 * fasta_par.c -- the MSA loader of `ccphylo dist` in parallel: the same
 * ccq_msa as ccq_load_msa (fasta.c), byte for byte, with the per-sequence
 * work on `threads` host threads.
 *
 * ref: seqparse.c:28 FileBuffgetFsa (record boundaries), cdist.c:196-333
 * ltdMsaMatrix_get (inclusion rules), qseqs.c:60 qseq2nibble, fsacmp.c:164 /
 * :181 initIncPos / getIncPos.
 *
 * The input is read in windows of decompressed bytes.  In each window the
 * records are located first:
 *   - a record starts at a '>' (the window's first record at its first byte)
 *     and its header runs to the next '\n';
 *   - its residues run to the next '>' (any '>' after the header: seqparse.c
 *     stops at every '>');
 *   - a header with no '\n', or a '\n' that is the last byte of the input,
 *     ends the input without a record (FileBuffgetFsa returns 0 there).
 * A record cut by the window's end moves to the next window.
 *
 * The first usable sequence is found serially, because it fixes the length,
 * the reference and minLength (cdist.c:287-321, minLength ratchets over the
 * excluded candidates).  Every later record is independent:
 *   - codes through the table, keeping those < 8 (the `(*seq >> 3) == 0` rule);
 *   - 2-bit packing into a provisional row;
 *   - pair mode: its own include mask (getIncPos of the sequence with itself);
 *   - non-pair mode: getIncPos against the reference, ANDed into a per-thread
 *     mask.  A position is cleared from (seq, ref) alone (the proximity walk
 *     of fsacmp.c:206-229 clears [lastSNP, i] whatever bits are already
 *     clear), so the AND over threads equals the reference's in-order updates.
 *     The reference also rewrites codes with bit 16 there; the 2-bit table
 *     (fsacmp.c:32) has no such code, so the reference stays read-only.
 * A serial pass in record order then prints the Included / Excluded lines,
 * stops at the first length mismatch as the reference does (exit 1), and
 * closes the gaps of excluded rows.
 */
#include <ctype.h>
#include <fcntl.h>
#include <pthread.h>
#include <sys/stat.h>
#include <unistd.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include "ccphylo_host.h"
#include "hostint.h"

static double now_s(void) {
	struct timespec t;
	clock_gettime(CLOCK_MONOTONIC, &t);
	return t.tv_sec + 1e-9 * t.tv_nsec;
}

#define WIN0 ((size_t) 256 << 20)   /* initial window; doubled while one record does not fit */

/* CCQ_FASTA_WINDOW=<bytes>: a small first window (tests of the carry-over) */
static int const_env_window(size_t *cap) {
	const char *e = getenv("CCQ_FASTA_WINDOW");
	if(!e) return 0;
	long v = atol(e);
	*cap = v < 16 ? 16 : (size_t) v;
	return 1;
}

typedef struct {
	size_t start, hend, end;        /* record start, its header '\n', next record */
	int len, inc, keep, mism;
	char *name;
} frec;

typedef struct {
	const unsigned char *buf;
	frec *recs;
	int nrec, next;                 /* work counter (atomic) */
	const unsigned char *table;
	int pair, variant, len, W;
	unsigned proxi, minLength;
	uint64_t *seqs;                 /* provisional rows: slot0 + record index */
	uint32_t *incs;                 /* pair: per row; else unused */
	int slot0;
	const unsigned char *ref;       /* codes of the first usable sequence */
	uint32_t **tmask;               /* non-pair: per-thread AND of the kept records' masks */
} fwork;

typedef struct {
	fwork *w;
	int t;
	unsigned char *codes;
	size_t cap;
} farg;

/* header [start, hend) without trailing white space, '>' dropped */
static char *rec_name(const unsigned char *buf, const frec *f) {
	size_t a = f->start, z = f->hend + 1;   /* the reference trims from the '\n' on (seqparse.c:71) */
	while(z > a && isspace(buf[z - 1])) --z;
	size_t n = z > a ? z - a - 1 : 0;
	char *s = ccq_xmalloc(n + 1);
	if(n) memcpy(s, buf + a + 1, n);
	s[n] = 0;
	return s;
}

/* residues -> codes < 8, returns the length */
static int rec_codes(const unsigned char *buf, const frec *f, const unsigned char *table, unsigned char *o) {
	const unsigned char *s = buf + f->hend + 1, *e = buf + f->end;
	unsigned char *o0 = o;
	for(; s < e; ++s) {
		const unsigned char c = table[*s];
		*o = c;
		o += c < 8;
	}
	return (int) (o - o0);
}

/* proxi == 0 (the default): one pass from the text to the packed row and
 * the row's N bits (code 4), MSB-first like qseq2nibble.  Without a
 * proximity window getIncPos only clears the positions where the sequence or
 * the reference has code 4 (fsacmp.c:196-205; no code has bit 16), so these
 * bits are the whole mask update.  Returns the length. */
static int rec_pack_n(const unsigned char *buf, const frec *f, const unsigned char *table, uint64_t *row,
                      uint32_t *nbits, int W) {
	const unsigned char *s = buf + f->hend + 1, *e = buf + f->end;
	uint64_t x = 0;
	uint32_t nb = 0;
	int k = 0, w = 0;
	for(; s < e; ++s) {
		const unsigned char c = table[*s];
		if(c >= 8) continue;
		x = (x << 2) | (c == 4 ? 0u : c);
		nb = (nb << 1) | (c == 4);
		if(((++k) & 31) == 0) {
			if(w < W) {
				row[w] = x;
				nbits[w] = nb;
			}
			++w;
			x = 0;
			nb = 0;
		}
	}
	if(k & 31) {   /* left-aligned tail (qseqs.c:83) */
		const int r = 32 - (k & 31);
		if(w < W) {
			row[w] = x << (2 * r);
			nbits[w] = nb << r;
		}
		++w;
	}
	for(; w < W; ++w) {
		row[w] = 0;
		nbits[w] = 0;
	}
	return k;
}

/* a plain (not gzip) regular file is read with pread on several threads:
 * the window fills at page-cache speed instead of one gzread copy */
typedef struct {
	int fd;
	unsigned char *dst;
	size_t len;
	off_t off;
	ssize_t got;
} pslice;

static void *pread_slice(void *p) {
	pslice *s = p;
	size_t done = 0;
	while(done < s->len) {
		const ssize_t g = pread(s->fd, s->dst + done, s->len - done, s->off + (off_t) done);
		if(g <= 0) break;
		done += (size_t) g;
	}
	s->got = (ssize_t) done;
	return NULL;
}

/* reads up to len bytes at off into dst with `threads` slices; returns the bytes read */
static size_t pread_par(int fd, unsigned char *dst, size_t len, off_t off, int threads) {
	enum { MAXS = 64 };
	pslice sl[MAXS];
	pthread_t th[MAXS];
	int ns = threads < MAXS ? threads : MAXS;
	const size_t chunk = ((len + ns - 1) / ns + 4095) & ~(size_t) 4095;
	int k = 0;
	for(size_t a = 0; a < len && k < ns; a += chunk, ++k) {
		sl[k].fd = fd;
		sl[k].dst = dst + a;
		sl[k].len = len - a < chunk ? len - a : chunk;
		sl[k].off = off + (off_t) a;
		sl[k].got = 0;
		if(pthread_create(th + k, NULL, pread_slice, sl + k)) pread_slice(sl + k), th[k] = 0;
	}
	size_t total = 0;
	int short_read = 0;
	for(int q = 0; q < k; ++q) {
		if(th[q]) pthread_join(th[q], NULL);
		if(!short_read) total += (size_t) sl[q].got;
		short_read |= (size_t) sl[q].got < sl[q].len;   /* EOF inside slice q: later slices read nothing */
	}
	return total;
}

static void *worker(void *p) {
	farg *a = p;
	fwork *w = a->w;
	for(;;) {
		const int e = __atomic_fetch_add(&w->next, 1, __ATOMIC_RELAXED);
		if(e >= w->nrec) break;
		frec *f = w->recs + e;
		size_t need = f->end - f->hend + 1;
		if(need < (size_t) w->W * 4 + 4) need = (size_t) w->W * 4 + 4;
		if(need > a->cap) {
			free(a->codes);
			a->cap = need + (need >> 2);
			a->codes = ccq_xmalloc(a->cap);
		}
		f->name = rec_name(w->buf, f);
		const size_t slot = (size_t) w->slot0 + e;
		if(w->proxi == 0) {
			/* one pass: packed row and N bits (the mask update without proximity) */
			uint32_t *nbits = (uint32_t *) a->codes;   /* W words fit: need >= 4 W bytes (below) */
			uint64_t *dst = w->seqs + slot * w->W;
			f->len = rec_pack_n(w->buf, f, w->table, dst, nbits, w->W);
			if(f->len != w->len) {
				f->mism = 1;
				continue;
			}
			int ns = 0;
			for(int k = 0; k < w->W; ++k) ns += __builtin_popcount(nbits[k]);
			if(w->pair) {
				uint32_t *m = w->incs + slot * w->W;
				memset(m, 0, (size_t) w->W * sizeof(uint32_t));   /* the word past the length stays 0 */
				ccq_init_inc(m, w->len);
				for(int k = 0; k < w->W; ++k) m[k] &= ~nbits[k];
				f->inc = ccq_npos(m, w->len);
				f->keep = (unsigned) f->inc >= w->minLength;
			} else {
				f->inc = w->len - ns;
				f->keep = w->minLength < (unsigned) f->inc;
				if(f->keep) {
					uint32_t *tm = w->tmask[a->t];
					for(int k = 0; k < w->W; ++k) tm[k] &= ~nbits[k];
				}
			}
			continue;
		}
		f->len = rec_codes(w->buf, f, w->table, a->codes);
		if(f->len != w->len) {
			f->mism = 1;
			continue;
		}
		uint64_t *dst = w->seqs + slot * w->W;
		memset(dst, 0, (size_t) w->W * sizeof(uint64_t));
		const int ns = ccq_pack(a->codes, w->len, dst);
		if(w->pair) {
			uint32_t *m = w->incs + slot * w->W;
			memset(m, 0, (size_t) w->W * sizeof(uint32_t));
			ccq_init_inc(m, w->len);
			ccq_inc_update(m, a->codes, a->codes, w->len, w->proxi, w->variant);
			f->inc = ccq_npos(m, w->len);
			f->keep = (unsigned) f->inc >= w->minLength;
		} else {
			f->inc = w->len - ns;
			f->keep = w->minLength < (unsigned) f->inc;
			if(f->keep) {
				ccq_inc_update(w->tmask[a->t], a->codes, (unsigned char *) w->ref, w->len, w->proxi, w->variant);
			}
		}
	}
	return NULL;
}

/* records of buf[0, blen); *used = where the next window starts; *stop = the
 * input ends in this window (no further record, the rest dropped) */
static int locate(const unsigned char *buf, size_t blen, int eof, frec **recs, int *cap, size_t *used, int *stop) {
	int n = 0;
	size_t p = 0;
	*stop = 0;
	while(p < blen) {
		const unsigned char *nl = memchr(buf + p, '\n', blen - p);
		if(!nl || (size_t) (nl - buf) + 1 >= blen) {
			if(eof) *stop = 1;   /* FileBuffgetFsa returns 0: the input ends here */
			break;
		}
		const size_t hend = (size_t) (nl - buf);
		const unsigned char *nx = memchr(buf + hend + 1, '>', blen - hend - 1);
		if(!nx && !eof) break;   /* cut by the window */
		if(n == *cap) {
			*cap = *cap ? 2 * *cap : 1024;
			*recs = ccq_xrealloc(*recs, (size_t) *cap * sizeof(frec));
		}
		frec *f = *recs + n++;
		memset(f, 0, sizeof(*f));
		f->start = p;
		f->hend = hend;
		f->end = nx ? (size_t) (nx - buf) : blen;
		p = f->end;
	}
	if(p >= blen && eof) *stop = 1;
	*used = p;
	return n;
}

ccq_msa *ccq_load_msa_par(ccq_reader *r, unsigned flag, unsigned minLength, double minCov, unsigned proxi, int threads,
                          FILE *log) {
	unsigned char table[256];
	const int variant = (flag & 32) ? 32 : (flag & 8) ? 8 : 0;
	ccq_code_table(flag, table);
	if(threads < 1) threads = 1;
	ccq_msa *M = ccq_xmalloc(sizeof(ccq_msa));
	memset(M, 0, sizeof(*M));
	M->pair = (flag & 2) != 0;
	int hcap = 16, rows_cap = 0, len = 0, W = 0, have_ref = 0;
	M->headers = ccq_xmalloc(hcap * sizeof(char *));
	uint32_t *gmask = NULL;
	unsigned char *ref = NULL, *scodes = NULL;
	size_t scap = 0;
	uint32_t **tmask = ccq_xmalloc(threads * sizeof(uint32_t *));
	memset(tmask, 0, threads * sizeof(uint32_t *));
	farg *args = ccq_xmalloc(threads * sizeof(farg));
	memset(args, 0, threads * sizeof(farg));
	pthread_t *tid = ccq_xmalloc(threads * sizeof(pthread_t));
	/* the window starts with the reader's buffered bytes */
	size_t cap = WIN0, blen = 0;
	const_env_window(&cap);
	unsigned char *buf = ccq_xmalloc(cap);
	if(r->pos < r->len) {
		blen = r->len - r->pos;
		if(blen > cap) {
			cap = blen;
			buf = ccq_xrealloc(buf, cap);
		}
		memcpy(buf, r->buf + r->pos, blen);
		r->pos = r->len;
	}
	int eof = r->eof;
	/* plain regular file: re-open it and continue at the reader's offset
	 * (gzdirect: transparent reads, so the uncompressed offset is the file's) */
	int fd = -1;
	off_t foff = 0;
	if(!eof && r->path && gzdirect(r->gz)) {
		struct stat st;
		fd = open(r->path, O_RDONLY);
		if(fd >= 0 && (fstat(fd, &st) || !S_ISREG(st.st_mode))) {
			close(fd);
			fd = -1;
		}
		foff = (off_t) gztell(r->gz);
		if(foff < 0 && fd >= 0) {
			close(fd);
			fd = -1;
		}
	}
	frec *recs = NULL;
	int rcap = 0;
	const int timing = getenv("CCQ_FASTA_TIMING") != NULL;   /* development aid: phase times on stderr */
	double t_read = 0, t_loc = 0, t_par = 0, t_ser = 0, t0 = now_s();
	for(;;) {
		if(fd >= 0) {
			if(blen < cap && !eof) {
				const size_t got = pread_par(fd, buf + blen, cap - blen, foff, threads);
				foff += (off_t) got;
				if(got < cap - blen) eof = 1;
				blen += got;
			}
		} else {
			while(blen < cap && !eof) {
				const size_t want = cap - blen > ((size_t) 1 << 30) ? ((size_t) 1 << 30) : cap - blen;
				const int got = gzread(r->gz, buf + blen, (unsigned) want);
				if(got <= 0) eof = 1;
				else blen += (size_t) got;
			}
		}
		size_t used;
		int stop;
		double t1 = now_s();
		t_read += t1 - t0;
		const int nrec = locate(buf, blen, eof, &recs, &rcap, &used, &stop);
		t0 = now_s();
		t_loc += t0 - t1;
		int e0 = 0;
		/* ---- the first usable sequence, serially (cdist.c:287-321) */
		for(; e0 < nrec && !have_ref; ++e0) {
			frec *f = recs + e0;
			const size_t need = f->end - f->hend + 1;
			if(need > scap) {
				free(scodes);
				scap = need;
				scodes = ccq_xmalloc(scap);
			}
			f->name = rec_name(buf, f);
			len = rec_codes(buf, f, table, scodes);
			if(minLength < minCov * len) minLength = (unsigned) (minCov * len);
			W = len / 32 + 1;
			if(rows_cap < hcap) rows_cap = hcap;
			M->seqs = ccq_xrealloc(M->seqs, (size_t) rows_cap * W * sizeof(uint64_t));
			uint32_t *m;
			if(M->pair) {
				M->incs = ccq_xrealloc(M->incs, (size_t) rows_cap * W * sizeof(uint32_t));
				m = M->incs + (size_t) M->n * W;
			} else {
				gmask = ccq_xrealloc(gmask, W * sizeof(uint32_t));
				m = gmask;
			}
			memset(m, 0, W * sizeof(uint32_t));
			ccq_init_inc(m, len);
			uint64_t *dst = M->seqs + (size_t) M->n * W;
			memset(dst, 0, W * sizeof(uint64_t));
			ccq_pack(scodes, len, dst);
			ccq_inc_update(m, scodes, scodes, len, proxi, variant);
			const int inc = ccq_npos(m, len);
			if((unsigned) inc < minLength) {
				fprintf(log, "# Excluded:\t%s\t( %d / %d )\n", f->name, inc, len);
				free(f->name);
			} else {
				fprintf(log, "# Included:\t%s\t( %d / %d )\n", f->name, inc, len);
				M->headers[M->n++] = f->name;
				ref = ccq_xmalloc((size_t) len + 1);
				memcpy(ref, scodes, len);
				have_ref = 1;
				for(int t = 0; t < threads && !M->pair; ++t) {
					tmask[t] = ccq_xmalloc(W * sizeof(uint32_t));
					memset(tmask[t], 0xFF, W * sizeof(uint32_t));
				}
			}
			f->name = NULL;
		}
		/* ---- every later record in parallel, in provisional rows M->n + e */
		const int nb = nrec - e0;
		if(nb > 0) {
			const int need = M->n + nb;
			if(need > rows_cap) {
				while(rows_cap < need) rows_cap *= 2;
				M->seqs = ccq_xrealloc(M->seqs, (size_t) rows_cap * W * sizeof(uint64_t));
				if(M->pair) M->incs = ccq_xrealloc(M->incs, (size_t) rows_cap * W * sizeof(uint32_t));
			}
			fwork w;
			memset(&w, 0, sizeof(w));
			w.buf = buf;
			w.recs = recs + e0;
			w.nrec = nb;
			w.table = table;
			w.pair = M->pair;
			w.variant = variant;
			w.len = len;
			w.W = W;
			w.proxi = proxi;
			w.minLength = minLength;
			w.seqs = M->seqs;
			w.incs = M->incs;
			w.slot0 = M->n;
			w.ref = ref;
			w.tmask = tmask;
			const int nt = threads < nb ? threads : nb;
			for(int t = 0; t < nt; ++t) {
				args[t].w = &w;
				args[t].t = t;
				if(pthread_create(tid + t, NULL, worker, args + t)) {
					fprintf(stderr, "Error: could not start a loader thread\n");
					exit(1);
				}
			}
			for(int t = 0; t < nt; ++t) pthread_join(tid[t], NULL);
			t1 = now_s();
			t_par += t1 - t0;
			t0 = t1;
			/* ---- in record order: logs, the reference's exit on a length
			 * mismatch, headers, and rows moved over the excluded ones */
			for(int e = 0; e < nb; ++e) {
				frec *f = recs + e0 + e;
				if(f->mism) {
					fprintf(stderr, "Sequences does not match: >%s\n", f->name);
					exit(1);
				}
				fprintf(log, f->keep ? "# Included:\t%s\t( %d / %d )\n" : "# Excluded:\t%s\t( %d / %d )\n", f->name, f->inc,
				        len);
				if(!f->keep) {
					free(f->name);
					continue;
				}
				if(M->n == hcap) {
					hcap <<= 1;
					M->headers = ccq_xrealloc(M->headers, hcap * sizeof(char *));
				}
				const int from = w.slot0 + e;
				if(from != M->n) {
					memmove(M->seqs + (size_t) M->n * W, M->seqs + (size_t) from * W, (size_t) W * sizeof(uint64_t));
					if(M->pair) {
						memmove(M->incs + (size_t) M->n * W, M->incs + (size_t) from * W, (size_t) W * sizeof(uint32_t));
					}
				}
				M->headers[M->n++] = f->name;
			}
		}
		t1 = now_s();
		t_ser += t1 - t0;
		t0 = t1;
		if(stop) break;
		/* the cut record moves to the front; a window without a whole record grows */
		if(used == 0 && blen == cap) {
			cap *= 2;
			buf = ccq_xrealloc(buf, cap);
		}
		memmove(buf, buf + used, blen - used);
		blen -= used;
		if(eof && blen == 0) break;
	}
	if(timing) {
		fprintf(stderr, "ccq_load_msa_par: read %.3f s, locate %.3f s, parallel %.3f s, serial %.3f s (%d threads)\n",
		        t_read, t_loc, t_par, t_ser, threads);
	}
	if(fd >= 0) close(fd);
	if(!M->pair && have_ref) {
		for(int t = 0; t < threads; ++t) {
			if(!tmask[t]) continue;
			for(int k = 0; k < W; ++k) gmask[k] &= tmask[t][k];
			free(tmask[t]);
		}
	}
	M->len = len;
	M->W = W;
	M->minLength = minLength;
	if(!M->pair) M->incs = gmask;
	for(int t = 0; t < threads; ++t) free(args[t].codes);
	free(args);
	free(tid);
	free(tmask);
	free(recs);
	free(buf);
	free(ref);
	free(scodes);
	return M;
}
