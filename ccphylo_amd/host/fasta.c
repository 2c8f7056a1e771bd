/*
 * fasta.c -- FASTA/MSA loading, 2-bit packing and include masks (host side,
 * O(N*L) once per run; the O(N^2*L) comparison is on the GPU).
 *
 * ref: fsacmp.c:32 get2BitTable, seqparse.c:28 FileBuffgetFsa,
 * qseqs.c:60 qseq2nibble, fsacmp.c:164 initIncPos, :181/:240/:296 getIncPos*,
 * :487 getNpos, cdist.c:196-333 ltdMsaMatrix_get (inclusion rules).
 */
#include <ctype.h>
#include <stdlib.h>
#include <string.h>
#include "ccphylo_host.h"
#include "hostint.h"

void ccq_code_table(unsigned flag, unsigned char table[256]) {
	static const char amb[] = "RYSWKMBDHVXryswkmbdhvx";
	memset(table, 32, 256);
	const char *up = "ACGTU";
	const unsigned char val[5] = {0, 1, 2, 3, 3};
	for(int k = 0; k < 5; ++k) {
		table[(unsigned char) up[k]] = val[k];
		table[(unsigned char) tolower(up[k])] = (flag & 8) ? val[k] : 4;
	}
	table['N'] = table['n'] = table['-'] = 4;
	for(const char *p = amb; *p; ++p) {
		table[(unsigned char) *p] = 4;
	}
}

int ccq_read_fasta(ccq_reader *r, ccq_str *header, ccq_str *seq, const unsigned char *table) {
	int c;
	uint32_t w = 0;
	header->len = 0;
	header->seq[0] = 0;
	seq->len = 0;
	seq->seq[0] = 0;
	if(ccq_peek(r) == EOF) {
		return 0;
	}
	/* header line, '>' included (seqparse.c:49-80) */
	for(;;) {
		if((c = ccq_getc(r)) == EOF) {
			return 0;
		}
		if(w + 1 >= header->size) {
			header->size <<= 1;
			header->seq = ccq_xrealloc(header->seq, header->size);
		}
		header->seq[w++] = (unsigned char) c;
		if(c == '\n') {
			break;
		}
	}
	if(ccq_peek(r) == EOF) {
		return 0;
	}
	while(w > 0 && isspace(header->seq[w - 1])) {
		--w;
	}
	header->seq[w] = 0;
	header->len = w;
	/* residues up to the next '>', codes >= 8 dropped (seqparse.c:84-98) */
	w = 0;
	while((c = ccq_peek(r)) != EOF && c != '>') {
		unsigned char code = table[(unsigned char) c];
		++r->pos;
		if(code < 8) {
			if(w + 1 >= seq->size) {
				seq->size <<= 1;
				seq->seq = ccq_xrealloc(seq->seq, seq->size);
			}
			seq->seq[w++] = code;
		}
	}
	seq->seq[w] = 0;
	seq->len = w;
	return 1;
}

int ccq_pack(const unsigned char *codes, int len, uint64_t *out) {
	int ns = 0, W = (len + 31) / 32;
	for(int w = 0; w < W; ++w) {
		uint64_t x = 0;
		int p0 = w * 32, cnt = len - p0 < 32 ? len - p0 : 32;
		for(int t = 0; t < cnt; ++t) {
			unsigned char c = codes[p0 + t];
			ns += c == 4;
			x = (x << 2) | (c == 4 ? 0 : c);
		}
		out[w] = x << (2 * (32 - cnt));   /* left-aligned tail (qseqs.c:83) */
	}
	return ns;
}

void ccq_init_inc(uint32_t *inc, int len) {
	int W = (len + 31) / 32;
	for(int w = 0; w < W; ++w) {
		inc[w] = ~0u;
	}
	if(len & 31) {
		inc[W - 1] <<= 32 - (len & 31);
	}
}

static inline void drop(uint32_t *inc, unsigned p) {
	inc[p >> 5] &= ~(0x80000000u >> (p & 31));
}

void ccq_inc_update(uint32_t *inc, unsigned char *seq, unsigned char *ref, int len, unsigned proxi, int variant) {
	long prev = -1;   /* last "SNP" position; -1 never opens a window */
	for(unsigned p = 0; p < (unsigned) len; ++p) {
		unsigned char c = seq[p], r = ref[p];
		int event;
		if(variant == 0) {
			event = c != r || c == 4 || (c & 16);
			if(c == 4 || r == 4) {
				drop(inc, p);
			} else if(event && ((c & 16) || (r & 16))) {
				drop(inc, p);
				seq[p] &= 15;
				ref[p] &= 15;
			}
		} else if(c == 4 || r == 4) {
			drop(inc, p);
			event = 0;
		} else if(variant == 32 && ((c & 16) || (r & 16))) {
			drop(inc, p);
			seq[p] &= 15;
			ref[p] &= 15;
			event = 0;
		} else {
			event = c != r;
		}
		if(event) {
			if(prev >= 0 && p - (unsigned) prev <= proxi) {
				for(unsigned q = (unsigned) prev; q <= p; ++q) {
					drop(inc, q);
				}
			}
			prev = p;
		}
	}
}

int ccq_npos(const uint32_t *inc, int len) {
	int n = 0;
	for(int w = 0; w < (len + 31) / 32; ++w) {
		n += __builtin_popcount(inc[w]);
	}
	return n;
}

ccq_msa *ccq_load_msa(ccq_reader *r, unsigned flag, unsigned minLength, double minCov,
                      unsigned proxi, FILE *log) {
	unsigned char table[256];
	int variant = (flag & 32) ? 32 : (flag & 8) ? 8 : 0;
	ccq_code_table(flag, table);
	ccq_msa *M = ccq_xmalloc(sizeof(ccq_msa));
	memset(M, 0, sizeof(*M));
	M->pair = (flag & 2) != 0;
	int cap = 16;
	ccq_str *hdr = ccq_new(64), *seq = ccq_new(1 << 20), *ref = ccq_new(1 << 20);
	int have_ref = 0, len = 0, W = 0;
	M->headers = ccq_xmalloc(cap * sizeof(char *));
	uint32_t *gmask = NULL;

	while(ccq_read_fasta(r, hdr, seq, table)) {
		if(M->n == cap) {
			cap <<= 1;
			M->headers = ccq_xrealloc(M->headers, cap * sizeof(char *));
			if(W) {
				M->seqs = ccq_xrealloc(M->seqs, (size_t) cap * W * sizeof(uint64_t));
				if(M->pair) {
					M->incs = ccq_xrealloc(M->incs, (size_t) cap * W * sizeof(uint32_t));
				}
			}
		}
		const char *name = (const char *) hdr->seq + 1;
		if(have_ref) {
			if((int) seq->len != len) {
				fprintf(stderr, "Sequences does not match: %s\n", (char *) hdr->seq);
				exit(1);
			}
			uint64_t *dst = M->seqs + (size_t) M->n * W;
			int inc;
			int keep;
			if(M->pair) {
				uint32_t *m = M->incs + (size_t) M->n * W;
				memset(m, 0, W * sizeof(uint32_t));
				ccq_init_inc(m, len);
				memset(dst, 0, W * sizeof(uint64_t));
				ccq_pack(seq->seq, len, dst);
				ccq_inc_update(m, seq->seq, seq->seq, len, proxi, variant);
				inc = ccq_npos(m, len);
				keep = (unsigned) inc >= minLength;
			} else {
				memset(dst, 0, W * sizeof(uint64_t));
				inc = len - ccq_pack(seq->seq, len, dst);
				keep = minLength < (unsigned) inc;
				if(keep) {
					ccq_inc_update(gmask, seq->seq, ref->seq, len, proxi, variant);
				}
			}
			fprintf(log, keep ? "# Included:\t%s\t( %d / %d )\n" : "# Excluded:\t%s\t( %d / %d )\n", name, inc, len);
			if(keep) {
				M->headers[M->n++] = strdup(name);
			}
		} else {
			/* first usable sequence: sets the length and the reference (cdist.c:287-321) */
			len = (int) seq->len;
			if(minLength < minCov * len) {
				minLength = (unsigned) (minCov * len);
			}
			W = len / 32 + 1;
			M->seqs = ccq_xrealloc(M->seqs, (size_t) cap * W * sizeof(uint64_t));
			uint32_t *m;
			if(M->pair) {
				M->incs = ccq_xrealloc(M->incs, (size_t) cap * W * sizeof(uint32_t));
				m = M->incs + (size_t) M->n * W;
			} else {
				gmask = ccq_xrealloc(gmask, W * sizeof(uint32_t));
				m = gmask;
			}
			memset(m, 0, W * sizeof(uint32_t));
			ccq_init_inc(m, len);
			uint64_t *dst = M->seqs + (size_t) M->n * W;
			memset(dst, 0, W * sizeof(uint64_t));
			ccq_pack(seq->seq, len, dst);
			ccq_inc_update(m, seq->seq, seq->seq, len, proxi, variant);
			int inc = ccq_npos(m, len);
			if((unsigned) inc < minLength) {
				fprintf(log, "# Excluded:\t%s\t( %d / %d )\n", name, inc, len);
			} else {
				fprintf(log, "# Included:\t%s\t( %d / %d )\n", name, inc, len);
				M->headers[M->n++] = strdup(name);
				ccq_str *t = ref;
				ref = seq;
				seq = t;
				have_ref = 1;
			}
		}
	}
	M->len = len;
	M->W = W;
	M->minLength = minLength;
	if(!M->pair) {
		M->incs = gmask;
	}
	ccq_free(hdr);
	ccq_free(seq);
	ccq_free(ref);
	return M;
}

void ccq_msa_free(ccq_msa *M) {
	if(M) {
		for(int i = 0; i < M->n; ++i) {
			free(M->headers[i]);
		}
		free(M->headers);
		free(M->seqs);
		free(M->incs);
		free(M);
	}
}

/* cdist.c:36-194 ltdFsaMatrix_get: the entry `tmpl` of every file.  All files
 * keep their slot (n = nfiles, stride W): cmpFsaThrd enumerates pairs over the
 * file indices (fsacmpthrd.c:192-218).  Files without the entry keep zero
 * sequences (the reference leaves them uninitialised).  Returns NULL where
 * the reference exits(1) (not FASTA, lengths differ), after its message. */
ccq_msa *ccq_load_fsa_files(char **files, int nfiles, const char *tmpl, unsigned flag, unsigned minLength,
                            double minCov, unsigned proxi, unsigned char *include, FILE *log) {
	unsigned char table[256];
	const int variant = (flag & 32) ? 32 : (flag & 8) ? 8 : 0;
	ccq_code_table(flag, table);
	ccq_msa *M = ccq_xmalloc(sizeof(ccq_msa));
	memset(M, 0, sizeof(*M));
	M->pair = (flag & 2) != 0;
	M->n = nfiles;
	M->headers = ccq_xmalloc((nfiles > 0 ? nfiles : 1) * sizeof(char *));
	ccq_str *hdr = ccq_new(64), *seq = ccq_new(1 << 20), *ref = ccq_new(1 << 20);
	int len = 0, W = 0, have_ref = 0;
	for(int f = 0; f < nfiles; ++f) {
		M->headers[f] = strdup(files[f]);
		include[f] = 1;
	}
	for(int f = 0; f < nfiles; ++f) {
		ccq_reader *r = ccq_open(files[f]);
		if(!r || ccq_peek(r) != '>') {
			fprintf(stderr, "\"%s\" is not fasta.\n", files[f]);
			if(r) ccq_close(r);
			goto fail;
		}
		int found = 0;
		while(ccq_read_fasta(r, hdr, seq, table)) {
			if(!strcmp((const char *) hdr->seq + 1, tmpl)) {
				found = 1;
				break;
			}
		}
		ccq_close(r);
		if(!found) {
			fprintf(log, "Missing template entry (\"%s\") in file:\t%s\n", tmpl, files[f]);
			include[f] = 0;
			continue;
		}
		if(!have_ref) {
			/* the first usable file: length, minCov, reference (cdist.c:116-163);
			 * rows packed for earlier (excluded) files are kept */
			len = (int) seq->len;
			if(minLength < minCov * len) minLength = (unsigned) (minCov * len);
			const int W2 = len / 32 + 1;
			if(W2 != W) {
				uint64_t *s2 = calloc((size_t) nfiles * W2, sizeof(uint64_t));
				uint32_t *i2 = calloc((size_t) (M->pair ? nfiles : 1) * W2, sizeof(uint32_t));
				if(!s2 || !i2) abort();
				for(int q = 0; W && q < nfiles; ++q) {
					memcpy(s2 + (size_t) q * W2, M->seqs + (size_t) q * W, (size_t) (W < W2 ? W : W2) * 8);
				}
				free(M->seqs);
				free(M->incs);
				M->seqs = s2;
				M->incs = i2;
				W = W2;
			}
		} else if((int) seq->len != len) {
			fprintf(stderr, "Sequences does not match: %s\n", files[f]);
			goto fail;
		}
		uint64_t *dst = M->seqs + (size_t) f * W;
		uint32_t *m = M->incs + (M->pair ? (size_t) f * W : 0);
		int inc;
		if(!have_ref || M->pair) {
			ccq_init_inc(m, len);
			ccq_pack(seq->seq, len, dst);
			ccq_inc_update(m, seq->seq, seq->seq, len, proxi, variant);
			inc = ccq_npos(m, len);
		} else {
			inc = len - ccq_pack(seq->seq, len, dst);
		}
		if((unsigned) inc < minLength) {
			fprintf(log, "# Excluded:\t%s\t( %d / %d )\n", files[f], inc, len);
			include[f] = 0;
			continue;
		}
		fprintf(log, "# Included:\t%s\t( %d / %d )\n", files[f], inc, len);
		if(!have_ref) {
			ccq_str *t = ref;
			ref = seq;
			seq = t;
			have_ref = 1;
		} else if(!M->pair) {
			ccq_inc_update(M->incs, seq->seq, ref->seq, len, proxi, variant);
		}
	}
	M->len = len;
	M->W = W > 0 ? W : 1;
	M->minLength = minLength;
	if(!M->seqs) {
		M->seqs = ccq_xmalloc(8);
		M->incs = ccq_xmalloc(4);
		M->seqs[0] = 0;
		M->incs[0] = 0;
	}
	ccq_free(hdr);
	ccq_free(seq);
	ccq_free(ref);
	return M;
fail:
	ccq_free(hdr);
	ccq_free(seq);
	ccq_free(ref);
	ccq_msa_free(M);
	return NULL;
}
