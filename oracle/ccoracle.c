/*
 * ccoracle.c -- plain-C restatement of ccphylo 0.8.5's dist/tree hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see ccoracle.h).  Every function cites the
 * reference file:line whose observable behaviour it restates, including the
 * reference's quirks (they are part of "identical output"):
 *   - updateD (nj.c:836) does not advance its sD/N cursor when both D_ik and
 *     D_kj are missing, so later sD/N updates land `lag` slots early;
 *   - updateD's D_kj-only column branch subtracts D_j[k], i.e. the flat LT
 *     element j(j-1)/2 + k (nj.c:1022);
 *   - maskProxi (fsacmp.c:355) works on position p+1 instead of p;
 *   - double -> u16/u8 stores truncate through a 32-bit int (x86 cvttsd2si).
 * Parity of this file is pinned by tests/test_oracle.py against golden
 * vectors produced by the reference binary (oracle/Makefile).
 */
#include <float.h>
#include <limits.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>
#include "ccoracle.h"

/* ------------------------------------------------------------------ */
/* element access for the packed LT matrix (matrix.c:32, bytescale.h)  */
/* ------------------------------------------------------------------ */
typedef struct {
	int et;          /* 8, 4, 2, 1 */
	double bs;       /* ByteScale */
	void *base;
} Ltd;

static inline int64_t tri(int64_t i) { return i * (i - 1) / 2; }

/* x86-64 gcc lowers (unsigned short/char) = double as cvttsd2si (32-bit)
 * followed by a narrowing store; out of range gives INT_MIN. */
static inline int32_t cvt_i32(double x) {
	if(!(x > -2147483649.0 && x < 2147483648.0)) {
		return INT32_MIN;
	}
	return (int32_t) x;
}

static inline double ld(const Ltd *D, int64_t f) {
	switch(D->et) {
		case 8: return ((double *) D->base)[f];
		case 4: return ((float *) D->base)[f];
		case 2: return ((uint16_t *) D->base)[f] / D->bs;
		default: return ((uint8_t *) D->base)[f] / D->bs;
	}
}

/* store v with the reference's rounding constant (dtouc(v, r)) */
static inline void st(Ltd *D, int64_t f, double v, double r) {
	switch(D->et) {
		case 8: ((double *) D->base)[f] = v; break;
		case 4: ((float *) D->base)[f] = (float) v; break;
		case 2: ((uint16_t *) D->base)[f] = (uint16_t) cvt_i32(v * D->bs + r); break;
		default: ((uint8_t *) D->base)[f] = (uint8_t) cvt_i32(v * D->bs + r); break;
	}
}

static inline double at(const Ltd *D, int64_t i, int64_t j) {
	return i > j ? ld(D, tri(i) + j) : ld(D, tri(j) + i);
}

/* ------------------------------------------------------------------ */
/* A1-A5: sequences and SNP counts                                     */
/* ------------------------------------------------------------------ */

/* fsacmp.c:32-91 get2BitTable */
void orc_code_table(unsigned flag, uint8_t table[256]) {
	const char *iupac = "RYSWKMBDHVXryswkmbdhvx";
	memset(table, 32, 256);
	table['A'] = 0; table['C'] = 1; table['G'] = 2; table['T'] = 3; table['U'] = 3;
	table['N'] = 4; table['-'] = 4;
	if(flag & 8) {
		table['a'] = 0; table['c'] = 1; table['g'] = 2; table['t'] = 3; table['u'] = 3;
	} else {
		table['a'] = 4; table['c'] = 4; table['g'] = 4; table['t'] = 4; table['u'] = 4;
	}
	table['n'] = 4;
	for(; *iupac; ++iupac) {
		table[(uint8_t) *iupac] = 4;
	}
}

/* qseqs.c:60-88 qseq2nibble: position p -> bits 63-2(p%32), code 4 -> 00 */
int orc_pack(const uint8_t *codes, int len, uint64_t *out) {
	int ns = 0;
	for(int w = 0; w * 32 < len; ++w) {
		uint64_t word = 0;
		int end = len < (w + 1) * 32 ? len : (w + 1) * 32;
		for(int p = w * 32; p < end; ++p) {
			word <<= 2;
			if(codes[p] == 4) {
				++ns;
			} else {
				word |= codes[p];
			}
		}
		if(end - w * 32 < 32) {
			word <<= 2 * (32 - (end - w * 32));
		}
		out[w] = word;
	}
	return ns;
}

/* fsacmp.c:164-179 initIncPos: ceil(len/32) words of ones, tail cleared */
void orc_init_inc(uint32_t *inc, int len) {
	int W = (len + 31) / 32;
	for(int w = 0; w < W; ++w) {
		inc[w] = 0xFFFFFFFFu;
	}
	if(len & 31) {
		inc[W - 1] <<= (32 - (len & 31));
	}
}

static inline void clear_bit(uint32_t *inc, unsigned p) {
	inc[p >> 5] &= ~(1u << (31 - (p & 31)));
}

/* the proximity run of fsacmp.c:209-231: clears [from, to] (from >= 0) */
static void clear_run(uint32_t *inc, unsigned from, unsigned to) {
	for(unsigned p = from; p <= to; ++p) {
		clear_bit(inc, p);
	}
}

/* fsacmp.c:181 getIncPos (variant 0), :296 getIncPosInsig (8),
 * :240 getIncPosInsigPrune (32).  seq/ref codes may be stripped (&= 15). */
void orc_inc_update(uint32_t *inc, uint8_t *seq, uint8_t *ref, int len, unsigned proxi, int variant) {
	long last = -1;
	for(unsigned i = 0; i < (unsigned) len; ++i) {
		uint8_t c = seq[i], r = ref[i];
		int snp = 0;
		if(variant == 0) {
			if(c != r || c == 4 || (c & 16)) {
				if(c == 4 || r == 4) {
					clear_bit(inc, i);
				} else if((c & 16) || (r & 16)) {
					clear_bit(inc, i);
					seq[i] &= 15;
					ref[i] &= 15;
				}
				snp = 1;
			}
		} else if(c == 4 || r == 4) {
			clear_bit(inc, i);
		} else if(variant == 32 && ((c & 16) || (r & 16))) {
			clear_bit(inc, i);
			seq[i] &= 15;
			ref[i] &= 15;
		} else if(c != r) {
			snp = 1;
		}
		if(snp) {
			/* unsigned compare (i - lastSNP <= proxi); a first SNP (last = -1)
			 * never clears because (unsigned)-1 < end is false (fsacmp.c:217) */
			if(last >= 0 && (unsigned)(i - (unsigned) last) <= proxi) {
				clear_run(inc, (unsigned) last, i);
			}
			last = i;
		}
	}
}

/* fsacmp.c:487-503 getNpos */
int orc_npos(const uint32_t *inc, int len) {
	int n = 0, W = (len + 31) / 32;
	for(int w = 0; w < W; ++w) {
		n += __builtin_popcount(inc[w]);
	}
	return n;
}

/* include bit k (LSB = 0) <-> 2-bit slot k of the u64 word */
static inline uint64_t spread32(uint32_t m) {
	uint64_t x = m;
	x = (x | (x << 16)) & 0x0000FFFF0000FFFFull;
	x = (x | (x << 8)) & 0x00FF00FF00FF00FFull;
	x = (x | (x << 4)) & 0x0F0F0F0F0F0F0F0Full;
	x = (x | (x << 2)) & 0x3333333333333333ull;
	x = (x | (x << 1)) & 0x5555555555555555ull;
	return x;
}

static inline int diff_count(uint64_t a, uint64_t b, uint32_t m) {
	uint64_t x = a ^ b;
	x = (x | (x >> 1)) & 0x5555555555555555ull;
	return __builtin_popcountll(x & spread32(m));
}

/* fsacmp.c:552-585 fsacmp */
uint32_t orc_fsacmp(const uint64_t *a, const uint64_t *b, const uint32_t *inc, int len) {
	uint32_t d = 0;
	int W = (len + 31) / 32;
	for(int w = 0; w < W; ++w) {
		d += diff_count(a[w], b[w], inc[w]);
	}
	return d;
}

/* fsacmp.c:587-633 fsacmpair: (dist << 32) | n */
uint64_t orc_fsacmpair(const uint64_t *a, const uint64_t *b, const uint32_t *inc, int len) {
	uint32_t d = 0, n = 0;
	int W = (len + 31) / 32;
	for(int w = 0; w < W; ++w) {
		d += diff_count(a[w], b[w], inc[w]);
		n += __builtin_popcount(inc[w]);
	}
	return ((uint64_t) d << 32) | n;
}

/* fsacmp.c:355-485 maskProxi.  Scans words from the end, bits from the LSB;
 * `i` runs one ahead of the position it stands for (p + 1), and the run
 * cleared is [p + 1, lastSNP] in that shifted numbering.  `out` must have
 * room for ceil(len/32) + 1 + proxi/32 + 1 words (the reference can run off
 * the end when the last position is a SNP; only zero tail bits are hit). */
void orc_mask_proxi(uint32_t *out, const uint32_t *inc1, const uint32_t *inc2,
                    const uint64_t *s1, const uint64_t *s2, unsigned len, unsigned proxi) {
	unsigned W = (len + 31) / 32;
	long last = (long) len + proxi;
	unsigned i = ((len + 31) / 32) * 32;
	for(unsigned w = W; w-- > 0;) {
		uint64_t k1 = s1[w], k2 = s2[w];
		uint32_t m = inc1[w] & inc2[w];
		out[w] = m;
		if(proxi && m && k1 != k2) {
			while(m) {
				if((m & 1) && (k1 & 3) != (k2 & 3)) {
					if((unsigned)((unsigned) last - i) <= proxi) {
						/* clear from i up to and including last, skipping words that
						 * become empty (fsacmp.c:403-419) */
						unsigned j = i, end = (unsigned) last + 1;
						while(j < end) {
							out[j >> 5] &= ~(1u << (31 - (j & 31)));
							if(out[j >> 5]) {
								++j;
							} else {
								j = ((j >> 5) + 1) << 5;
							}
						}
					}
					last = i;
				}
				k1 >>= 2;
				k2 >>= 2;
				m >>= 1;
				--i;
			}
			i = (i >> 5) << 5;
		} else {
			i -= 32;
		}
	}
}

/* x86 store of a double into u16/u8 LT cells */
static void st_raw(int et, double bs, void *M, int64_t f, double v_scaled_plus_round) {
	(void) bs;
	if(et == 2) {
		((uint16_t *) M)[f] = (uint16_t) cvt_i32(v_scaled_plus_round);
	} else {
		((uint8_t *) M)[f] = (uint8_t) cvt_i32(v_scaled_plus_round);
	}
}

/* fsacmpthrd.c:108-259 cmpFsaThrd and :261-480 cmpairFsaThrd, for the MSA
 * driver (cdist.c:196) where every loaded taxon is included, so LT cell
 * (pi, pj) holds pair (pi, pj). */
typedef struct {
	int n, len, pair, etype;
	const uint64_t *seqs;
	const uint32_t *incs;
	unsigned norm, minLength, proxi;
	double nFactor, byteScale;
	void *D, *N;
	int64_t W;
	int r0, stride;   /* rows r0, r0 + stride, ... (threads) */
	const uint64_t *spread;   /* non-pair: spread32 of each mask word, computed once */
} SnpArg;

/* orc_fsacmp with the mask words already spread (the same sum) */
static inline uint32_t fsacmp_spread(const uint64_t *a, const uint64_t *b, const uint64_t *sp, int W32) {
	uint32_t d = 0;
	for(int w = 0; w < W32; ++w) {
		uint64_t x = a[w] ^ b[w];
		d += __builtin_popcountll((x | (x >> 1)) & 0x5555555555555555ull & sp[w]);
	}
	return d;
}

/* one LT row i: cells (i, 0..i-1) */
static void snp_row(const SnpArg *a, int64_t i, uint32_t *pm) {
	const int64_t W = a->W;
	const uint64_t *seqs = a->seqs;
	const uint32_t *incs = a->incs;
	const int etype = a->etype;
	const double byteScale = a->byteScale;
	void *D = a->D, *N = a->N;
	for(int64_t j = 0; j < i; ++j) {
		const int64_t f = tri(i) + j;
		if(!a->pair) {
			uint64_t dist = fsacmp_spread(seqs + i * W, seqs + j * W, a->spread, (a->len + 31) / 32);
			double v = a->nFactor * dist;
			if(etype == 8) {
				((double *) D)[f] = v;
			} else if(etype == 4) {
				((float *) D)[f] = v;
			} else {
				st_raw(etype, byteScale, D, f, v * byteScale + 0.5);
			}
			continue;
		}
		memset(pm, 0, (W + 4 + a->proxi / 32) * sizeof(uint32_t));
		orc_mask_proxi(pm, incs + i * W, incs + j * W, seqs + i * W, seqs + j * W, a->len, a->proxi);
		uint64_t dn = orc_fsacmpair(seqs + i * W, seqs + j * W, pm, a->len);
		uint32_t inc = (uint32_t) dn;
		uint64_t dist = dn >> 32;
		const unsigned norm = a->norm;
		if(etype == 8) {
			double *Dp = D;
			if(a->minLength <= inc) {
				if(norm) {
					Dp[f] = (double) (dist * norm);
					Dp[f] /= inc;
				} else {
					Dp[f] = (double) dist;
				}
			} else {
				Dp[f] = -1.0;
			}
			if(N) ((double *) N)[f] = inc;
		} else if(etype == 4) {
			float *Dp = D;
			if(a->minLength <= inc) {
				if(norm) {
					Dp[f] = (float) (dist * norm);
					Dp[f] /= (float) inc;
				} else {
					Dp[f] = (float) dist;
				}
			} else {
				Dp[f] = -1.0f;
			}
			if(N) ((float *) N)[f] = (float) inc;
		} else {
			double v;
			if(a->minLength <= inc) {
				if(norm) {
					v = ((double) (dist * norm) * byteScale + 0.5) / inc;
				} else {
					v = (double) dist * byteScale + 0.5;
				}
			} else {
				v = -1.0 * byteScale + 0;
			}
			st_raw(etype, byteScale, D, f, v);
			if(N) st_raw(etype, byteScale, N, f, inc * byteScale + 0.5);
		}
	}
}

static void *snp_worker(void *p) {
	SnpArg *a = p;
	uint32_t *pm = a->pair ? malloc((a->W + 4 + a->proxi / 32) * sizeof(uint32_t)) : NULL;
	for(int64_t i = 1 + a->r0; i < a->n; i += a->stride) snp_row(a, i, pm);
	free(pm);
	return NULL;
}

int orc_snp_ltd_ex(int n, int len, const uint64_t *seqs, const uint32_t *incs, int pair,
                   unsigned norm, unsigned minLength, double minCov, unsigned proxi,
                   int etype, double byteScale, void *D, void *N, int threads) {
	SnpArg a = {n, len, pair, etype, seqs, incs, norm, minLength, proxi, 1.0, byteScale, D, N,
	            len / 32 + 1 /* stride used by the reference (cdist.c:290) */, 0, 1, NULL};
	int inc_total = 0;
	uint64_t *spread = NULL;
	if(!pair) {
		spread = malloc(((len + 31) / 32 + 1) * sizeof(uint64_t));
		for(int w = 0; w < (len + 31) / 32; ++w) spread[w] = spread32(incs[w]);
		a.spread = spread;
		inc_total = orc_npos(incs, len);
		if(norm) {
			a.nFactor = norm;
			a.nFactor /= inc_total;
		}
	} else if(minLength < minCov * len) {
		a.minLength = minCov * len;
	}
	if(threads > 256) threads = 256;
	if(threads <= 1 || n < 256) {
		snp_worker(&a);
		free(spread);
		return inc_total;
	}
	pthread_t th[256];
	SnpArg args[256];
	for(int t = 0; t < threads; ++t) {
		args[t] = a;
		args[t].r0 = t;
		args[t].stride = threads;
		pthread_create(&th[t], NULL, snp_worker, &args[t]);
	}
	for(int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
	free(spread);
	return inc_total;
}

int orc_snp_ltd(int n, int len, const uint64_t *seqs, const uint32_t *incs, int pair,
                unsigned norm, unsigned minLength, double minCov, unsigned proxi,
                int etype, double byteScale, void *D, void *N) {
	return orc_snp_ltd_ex(n, len, seqs, incs, pair, norm, minLength, minCov, proxi, etype, byteScale, D, N, 1);
}

/* ------------------------------------------------------------------ */
/* C/D: neighbor joining                                               */
/* ------------------------------------------------------------------ */

/* nj.c:111-180 initSummaD: sD[k] summed sequentially in increasing m */
static void init_sums(const Ltd *D, int n, double *sD, int32_t *N) {
	for(int k = 0; k < n; ++k) {
		sD[k] = 0;
		N[k] = 1;
	}
	for(int64_t i = 1; i < n; ++i) {
		for(int64_t j = 0; j < i; ++j) {
			double d = ld(D, tri(i) + j);
			if(0 <= d) {
				sD[i] += d;
				sD[j] += d;
				++N[i];
				++N[j];
			}
		}
	}
}

/* the same sums with `threads` pthreads: thread t owns a range of k and
 * keeps each sD[k]'s order (its row part d(k, 0..k-1), then its column part
 * d(k+1, k), d(k+2, k), ...), so the result equals init_sums bit for bit.
 * Test infrastructure for large n (tests/test_gpu_large.py). */
typedef struct {
	const Ltd *D;
	int n, k0, k1;
	double *sD, *Q;
	int32_t *N, *P;
	int stride;   /* init_hnj_par: rows k0, k0 + stride, ... */
} ParArg;

static void *init_sums_worker(void *p) {
	ParArg *a = p;
	const Ltd *D = a->D;
	for(int64_t k = a->k0; k < a->k1; ++k) {
		double s = 0;
		int32_t c = 1;
		int64_t base = tri(k);
		for(int64_t m = 0; m < k; ++m) {
			double d = ld(D, base + m);
			if(0 <= d) {
				s += d;
				++c;
			}
		}
		a->sD[k] = s;
		a->N[k] = c;
	}
	for(int64_t i = a->k0 + 1; i < a->n; ++i) {
		int64_t base = tri(i), lim = i < a->k1 ? i : a->k1;
		for(int64_t k = a->k0; k < lim; ++k) {
			double d = ld(D, base + k);
			if(0 <= d) {
				a->sD[k] += d;
				++a->N[k];
			}
		}
	}
	return NULL;
}

static void *init_hnj_worker(void *p);

static void run_par(void *(*fn)(void *), ParArg *proto, int threads, int by_rows) {
	pthread_t th[256];
	ParArg args[256];
	if(threads > 256) threads = 256;
	for(int t = 0; t < threads; ++t) {
		args[t] = *proto;
		if(by_rows) {
			args[t].k0 = t;
			args[t].stride = threads;
		} else {
			args[t].k0 = (int) ((int64_t) proto->n * t / threads);
			args[t].k1 = (int) ((int64_t) proto->n * (t + 1) / threads);
		}
		pthread_create(&th[t], NULL, fn, &args[t]);
	}
	for(int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
}

static void init_sums_par(const Ltd *D, int n, double *sD, int32_t *N, int threads) {
	if(threads <= 1 || n < 1024) {
		init_sums(D, n, sD, N);
		return;
	}
	ParArg a = {D, n, 0, 0, sD, NULL, N, NULL, 1};
	run_par(init_sums_worker, &a, threads, 0);
}

void orc_init_sums(int n, int etype, double byteScale, const void *D, double *sD, int32_t *N) {
	Ltd L = {etype, byteScale, (void *) D};
	init_sums(&L, n, sD, N);
}

/* the Q criterion exactly as written in nj.c:227 / dnj.c:103 */
static inline double qval(int Ni, int Nj, double d, double sDi, double sDj) {
	return ((Ni + Nj - 4) >> 1) * d - sDi - sDj;
}

/* nj.c:42 limbLength / :81 limbLengthNeg */
static void limb_length(double *Li, double *Lj, int i, int j, const double *sD, const int32_t *N,
                        double Dij, int neg) {
	int Ni = N[i] - 2, Nj = N[j] - 2;
	if(0 < Ni && 0 < Nj) {
		double delta = ((sD[i] - Dij) / Ni) - ((sD[j] - Dij) / Nj);
		*Li = (Dij + delta) / 2;
		*Lj = (Dij - delta) / 2;
		if(!neg) {
			if(*Li < 0) {
				*Lj = Dij;
				*Li = 0;
			} else if(*Lj < 0) {
				*Li = Dij;
				*Lj = 0;
			}
		}
	} else if(0 < Ni) {
		*Li = 0;
		*Lj = Dij;
	} else if(0 < Nj) {
		*Li = Dij;
		*Lj = 0;
	} else {
		*Li = (*Lj = Dij / 2);
	}
}

/* nj.c:182-247 initQ: min starts at 1, last minimal cell in row-major order */
static uint64_t init_q(const Ltd *D, int n, const double *sD, const int32_t *N) {
	double min = 1;
	int mi = 0, mj = 0;
	for(int64_t i = 1; i < n; ++i) {
		int64_t base = tri(i);
		for(int64_t j = 0; j < i; ++j) {
			double q = ld(D, base + j);
			if(0 <= q) {
				q = qval(N[i], N[j], q, sD[i], sD[j]);
				if(q <= min) {
					min = q;
					mi = i;
					mj = j;
				}
			}
		}
	}
	return ((uint64_t) mi << 32) | (uint32_t) mj;
}

/* typed "D -= Lj" of the D_kj-only branch (nj.c:930-941 / :1020-1031);
 * returns the stored value as the reference sees it (before uctod) */
static double sub_store(Ltd *D, int64_t f, double Lj) {
	switch(D->et) {
		case 8: {
			double *p = (double *) D->base + f;
			*p -= Lj;
			return *p;
		}
		case 4: {
			float *p = (float *) D->base + f;
			*p -= Lj;
			return *p;
		}
		case 2: {
			uint16_t *p = (uint16_t *) D->base + f;
			*p = (uint16_t) cvt_i32(*p - (Lj * D->bs + 0));
			return *p;
		}
		default: {
			uint8_t *p = (uint8_t *) D->base + f;
			*p = (uint8_t) cvt_i32(*p - (Lj * D->bs + 0));
			return *p;
		}
	}
}

/* nj.c:1022 `dist = (D[k][j] -= Lj) - D_j[k]` in the element type, where
 * D_j[k] is flat element j(j-1)/2 + k (read after the store). */
static double sub_garbage(Ltd *D, int64_t f, int64_t g, double Lj) {
	switch(D->et) {
		case 8: {
			double *b = D->base;
			b[f] -= Lj;
			return b[f] - b[g];
		}
		case 4: {
			float *b = D->base;
			b[f] -= Lj;
			return (float) (b[f] - b[g]);
		}
		case 2: {
			uint16_t *b = D->base;
			b[f] = (uint16_t) cvt_i32(b[f] - (Lj * D->bs + 0));
			return ((int) b[f] - (int) b[g]) / D->bs;
		}
		default: {
			uint8_t *b = D->base;
			b[f] = (uint8_t) cvt_i32(b[f] - (Lj * D->bs + 0));
			return ((int) b[f] - (int) b[g]) / D->bs;
		}
	}
}

/* nj.c:836-1044 updateD.  `c` is the reference's sDvec/Nptr cursor: it
 * advances once per k that takes a branch, and once for j and for i. */
static void update_d(Ltd *D, int n, double *sD, int32_t *N, int i, int j, double Li, double Lj) {
	double Dij = ld(D, tri(i) + j), sd = 0;
	int nn = 1;
	int64_t c = 0;
	int64_t ri = tri(i), rj = tri(j);
	for(int64_t k = 0; k < j; ++k) {
		double Dik = ld(D, ri + k), Dkj = ld(D, rj + k);
		if(0 <= Dik && 0 <= Dkj) {
			double d = (Dik + Dkj - Dij) / 2;
			d = d < 0 ? 0 : d;
			st(D, rj + k, d, 0.25);
			sD[c] -= (Dik + Dkj - d);
			--N[c];
			++c;
			sd += d;
			++nn;
		} else if(0 <= Dik) {
			double d = Dik - Li;
			st(D, rj + k, d, 0);
			sD[c] -= Li;
			++c;
			sd += d;
			++nn;
		} else if(0 <= Dkj) {
			double d = sub_store(D, rj + k, Lj);
			if(D->et <= 2) d /= D->bs;
			sD[c] += (d - Dkj);
			--N[c];
			++c;
			sd += d;
			++nn;
		}
	}
	++c;   /* skip j */
	for(int64_t k = j + 1; k < n; ++k) {
		if(k == i) {
			++c;
			continue;
		}
		int64_t fk = tri(k) + j;
		double Dik = k < i ? ld(D, ri + k) : ld(D, tri(k) + i);
		double Dkj = ld(D, fk);
		if(0 <= Dik && 0 <= Dkj) {
			double d = (Dkj + Dik - Dij) / 2;
			d = d < 0 ? 0 : d;
			st(D, fk, d, 0.25);
			sD[c] -= (Dik + Dkj - d);
			--N[c];
			++c;
			sd += d;
			++nn;
		} else if(0 <= Dik) {
			double d = Dik - Li;
			st(D, fk, d, 0);
			sD[c] -= Li;
			++c;
			sd += d;
			++nn;
		} else if(0 <= Dkj) {
			double d = sub_garbage(D, fk, rj + k, Lj);
			sD[c] += d;
			--N[c];
			++c;
			sd += d;
			++nn;
		}
	}
	N[j] = nn;
	sD[j] = sd;
}

/* matrix.c:518-602 ltdMatrix_popArrange (+ nj.c:1588-1589 vectors) */
static void pop_arrange(Ltd *D, int n_new, int pos) {
	if(pos == n_new) {
		return;
	}
	int64_t src = tri(n_new), dst = tri(pos);
	size_t es = D->et;
	char *b = D->base;
	memmove(b + dst * es, b + src * es, (size_t) pos * es);
	for(int64_t k = pos + 1; k < n_new; ++k) {
		memcpy(b + (tri(k) + pos) * es, b + (src + k) * es, es);
	}
}

/* hclust.c:56-130 initHNJ: per-row min Q (ties: smaller D, then later j) */
static void init_hnj(const Ltd *D, int n, const double *sD, const int32_t *N, double *Q, int32_t *P) {
	for(int64_t i = 0; i < n; ++i) {
		double min = DBL_MAX, minD = DBL_MAX;
		int pos = 0;
		int64_t base = tri(i);
		for(int64_t j = 0; j < i; ++j) {
			double d = ld(D, base + j);
			if(0 <= d) {
				double q = qval(N[i], N[j], d, sD[i], sD[j]);
				if(q <= min && (q < min || d <= minD)) {
					min = q;
					minD = d;
					pos = j;
				}
			}
		}
		Q[i] = min;
		P[i] = pos;
	}
}

/* init_hnj over interleaved rows with `threads` pthreads (rows are independent) */
static void init_hnj_rows(const Ltd *D, int64_t i, const double *sD, const int32_t *N, double *Q, int32_t *P) {
	double min = DBL_MAX, minD = DBL_MAX;
	int pos = 0;
	int64_t base = tri(i);
	for(int64_t j = 0; j < i; ++j) {
		double d = ld(D, base + j);
		if(0 <= d) {
			double q = qval(N[i], N[j], d, sD[i], sD[j]);
			if(q <= min && (q < min || d <= minD)) {
				min = q;
				minD = d;
				pos = j;
			}
		}
	}
	Q[i] = min;
	P[i] = pos;
}

static void *init_hnj_worker(void *p) {
	ParArg *a = p;
	for(int64_t i = a->k0; i < a->n; i += a->stride) init_hnj_rows(a->D, i, a->sD, a->N, a->Q, a->P);
	return NULL;
}

static void init_hnj_par(const Ltd *D, int n, const double *sD, const int32_t *N, double *Q, int32_t *P, int threads) {
	if(threads <= 1 || n < 1024) {
		init_hnj(D, n, sD, N, Q, P);
		return;
	}
	ParArg a = {D, n, 0, n, (double *) sD, Q, (int32_t *) N, P, 1};
	run_par(init_hnj_worker, &a, threads, 1);
}

/* fresh min over LT row i with `<=` (dnj.c:99-112) */
static double row_min(const Ltd *D, int i, const double *sD, const int32_t *N, int *pj, int64_t *cells) {
	double best = DBL_MAX;
	int mj = 0;
	int64_t base = tri(i);
	for(int64_t j = 0; j < i; ++j) {
		double q = ld(D, base + j);
		if(0 <= q) {
			q = qval(N[i], N[j], q, sD[i], sD[j]);
			if(q <= best) {
				best = q;
				mj = j;
			}
		}
	}
	if(cells) *cells += i;
	*pj = mj;
	return best;
}

/* dnj.c:43-128 minQpair */
static uint64_t min_q_pair(const Ltd *D, int n, const double *sD, const int32_t *N, double *Q, int32_t *P,
                           int cand, int64_t *stats) {
	double min = DBL_MAX;
	uint64_t pos = 0;
	if(cand && min != Q[cand]) {
		min = Q[cand];
		pos = ((uint64_t) cand << 32) | (uint32_t) P[cand];
	}
	for(int i = n - 1; i > 0; --i) {
		if(Q[i] < min) {
			int mj;
			double q = row_min(D, i, sD, N, &mj, stats ? stats + 1 : 0);
			if(stats) ++stats[0];
			P[i] = mj;
			Q[i] = q;
			if(q < min) {
				min = q;
				pos = ((uint64_t) i << 32) | (uint32_t) mj;
			}
		}
	}
	return pos;
}

/* min_q_pair with `threads` pthreads (test infrastructure for large n, where
 * one join rescans ~1e9 cells).  The serial loop's decisions are replayed in
 * its own order: rows are collected in descending order while Q[r] < min (the
 * running min only decreases, so a row with Q[r] >= min at collection time is
 * skipped by the serial loop too), their fresh row minima are computed in
 * parallel into scratch (row_min is a function of row r alone), then the batch
 * is walked in order with dnj.c:78's test against the now-current min: an
 * accepted row stores P/Q and may lower min, a rejected one keeps its stale
 * Q/P and its fresh value is discarded.  So Q, P, the returned pos and the
 * reference-rule counters equal min_q_pair's bit for bit (pinned by
 * tests/test_oracle_golden.py::test_oracle_parallel_min_q_pair). */
typedef struct {
	const Ltd *D;
	const double *sD;
	const int32_t *N;
	const int *rows;
	double *fq;
	int *fj;
	int cnt;
	int next;     /* atomic row cursor */
} RescanArg;

static void *rescan_worker(void *p) {
	RescanArg *a = p;
	for(;;) {
		int k = __atomic_fetch_add(&a->next, 1, __ATOMIC_RELAXED);
		if(k >= a->cnt) break;
		a->fq[k] = row_min(a->D, a->rows[k], a->sD, a->N, &a->fj[k], 0);
	}
	return NULL;
}

#define RESCAN_BATCH_ROWS 8192
/* below this many cells a batch is rescanned on the calling thread
 * (ORC_PAR_CELLS overrides it: the tests force the threaded path at small n) */
static int64_t rescan_par_cells(void) {
	const char *e = getenv("ORC_PAR_CELLS");
	return e ? atoll(e) : (1 << 22);
}

static uint64_t min_q_pair_par(const Ltd *D, int n, const double *sD, const int32_t *N, double *Q, int32_t *P,
                               int cand, int64_t *stats, int threads, int *rows, double *fq, int *fj) {
	double min = DBL_MAX;
	uint64_t pos = 0;
	if(cand && min != Q[cand]) {
		min = Q[cand];
		pos = ((uint64_t) cand << 32) | (uint32_t) P[cand];
	}
	int lim = 64;   /* batches grow, so an early steep drop of min wastes little */
	const int64_t par_cells = rescan_par_cells();
	for(int i = n - 1; i > 0;) {
		int cnt = 0, r = i;
		int64_t cells = 0;
		for(; r > 0 && cnt < lim; --r) {
			if(Q[r] < min) {
				rows[cnt++] = r;
				cells += r;
			}
		}
		if(cells >= par_cells && threads > 1) {
			RescanArg a = {D, sD, N, rows, fq, fj, cnt, 0};
			pthread_t th[256];
			int nt = threads > 256 ? 256 : threads;
			for(int t = 0; t < nt; ++t) pthread_create(&th[t], NULL, rescan_worker, &a);
			for(int t = 0; t < nt; ++t) pthread_join(th[t], NULL);
		} else {
			for(int k = 0; k < cnt; ++k) fq[k] = row_min(D, rows[k], sD, N, &fj[k], 0);
		}
		for(int k = 0; k < cnt; ++k) {
			const int row = rows[k];
			if(Q[row] < min) {
				if(stats) {
					++stats[0];
					stats[1] += row;
				}
				P[row] = fj[k];
				Q[row] = fq[k];
				if(fq[k] < min) {
					min = fq[k];
					pos = ((uint64_t) row << 32) | (uint32_t) fj[k];
				}
			}
		}
		i = r;
		if(lim < RESCAN_BATCH_ROWS) lim *= 2;
	}
	return pos;
}

/* dnj.c:607-710 updateDNJ (after updateD): returns p */
static int update_dnj_q(const Ltd *D, int n, const double *sD, const int32_t *N, double *Q, int32_t *P,
                        int i, int j) {
	int mj;
	Q[j] = row_min(D, j, sD, N, &mj, 0);
	P[j] = mj;
	double min = Q[j];
	int p = j;
	for(int k = j + 1; k < n; ++k) {
		if(k == i) {
			continue;
		}
		double d = ld(D, tri(k) + j);
		if(0 <= d) {
			double q = qval(N[j], N[k], d, sD[j], sD[k]);
			if(q <= Q[k]) {
				Q[k] = q;
				P[k] = j;
				if(q <= min) {
					min = q;
					p = k;
				}
			}
		}
	}
	return p;
}

/* dnj.c:817-975 DNJ_popArrange; *n is decremented.  Returns p (0 when the
 * removed row was the last one). */
static int dnj_pop_arrange(Ltd *D, int *n, double *sD, int32_t *N, double *Q, int32_t *P, int pos) {
	int nn = --*n;
	if(pos == nn) {
		return 0;
	}
	sD[pos] = sD[nn];
	N[pos] = N[nn];
	pop_arrange(D, nn, pos);
	int mj;
	Q[pos] = row_min(D, pos, sD, N, &mj, 0);
	P[pos] = mj;
	double min = Q[pos];
	int p = pos;
	for(int k = pos + 1; k < nn; ++k) {
		double d = ld(D, tri(k) + pos);
		if(0 <= d) {
			double q = d * ((N[pos] + N[k] - 4) >> 1) - sD[pos] - sD[k];
			if(q <= Q[k]) {
				Q[k] = q;
				P[k] = pos;
				if(q <= min) {
					min = q;
					p = k;
				}
			}
		}
	}
	return p;
}

/* dnj.c:977 minPos */
static int min_pos(const double *Q, int i, int j) {
	return (Q[j] < Q[i] || (i < j && Q[j] == Q[i])) ? j : i;
}

/* hclust.c:353-381 minQ: returns the row of the (last) minimal bound */
static int min_q_row(const double *Q, int n) {
	double min = DBL_MAX;
	int mi = 0;
	for(int i = 1; i < n; ++i) {
		if(Q[i] <= min) {
			min = Q[i];
			mi = i;
		}
	}
	return mi;
}

/* hclust.c:413-450 updatePrevQ: Q[k] from the row's remembered partner P[k]
 * for k = 0 .. n-2 (the last row is not revisited).  Row 0 reads element
 * P[0] = 0 of the flat buffer, i.e. D(1, 0) (mat[0] is the buffer base). */
static void update_prev_q(const Ltd *D, int n, const double *sD, const int32_t *N, double *Q, const int32_t *P) {
	for(int64_t k = 0; k < n - 1; ++k) {
		double d = ld(D, tri(k) + P[k]);
		if(0 <= d) {
			Q[k] = ((N[k] + N[P[k]] - 4) >> 1) * d - sD[k] - sD[P[k]];
		}
	}
}

/* hclust.c:452-561 updateHNJ after updateD: updatePrevQ, row j, then column
 * j over k > j, k != i (the min/p it tracks is never used by hclust) */
static void update_hnj_q(const Ltd *D, int n, const double *sD, const int32_t *N, double *Q, int32_t *P, int i, int j) {
	update_prev_q(D, n, sD, N, Q, P);
	double qj = DBL_MAX;
	int pj = 0;
	int64_t base = tri(j);
	for(int64_t k = 0; k < j; ++k) {
		double d = ld(D, base + k);
		if(0 <= d) {
			double q = ((N[j] + N[k] - 4) >> 1) * d - sD[j] - sD[k];
			if(q <= qj) {
				qj = q;
				pj = (int) k;
			}
		}
	}
	Q[j] = qj;
	P[j] = pj;
	for(int64_t k = j + 1; k < n; ++k) {
		if(k == i) {
			continue;
		}
		double d = ld(D, tri(k) + j);
		if(0 <= d) {
			double q = ((N[j] + N[k] - 4) >> 1) * d - sD[j] - sD[k];
			if(P[k] == i || P[k] == j) {
				Q[k] = q;
				P[k] = j;
			} else if(q <= Q[k]) {
				Q[k] = q;
				if(P[k] < j) {
					P[k] = j;
				}
			}
		}
	}
}

/* hclust.c:1308-1432 HNJ_popArrange; *n is decremented */
static void hnj_pop_arrange(Ltd *D, int *n, double *sD, int32_t *N, double *Q, int32_t *P, int pos) {
	int nn = --*n;
	if(pos == nn) {
		return;
	}
	sD[pos] = sD[nn];
	N[pos] = N[nn];
	pop_arrange(D, nn, pos);
	double qp = DBL_MAX;
	int pp = 0;
	int64_t base = tri(pos);
	for(int64_t k = 0; k < pos; ++k) {
		double d = ld(D, base + k);
		if(0 <= d) {
			double q = d * ((N[pos] + N[k] - 4) >> 1) - sD[pos] - sD[k];
			if(q <= qp) {
				qp = q;
				pp = (int) k;
			}
		}
	}
	Q[pos] = qp;
	P[pos] = pp;
	for(int64_t k = pos + 1; k < nn; ++k) {
		double d = ld(D, tri(k) + pos);
		if(0 <= d) {
			double q = d * ((N[pos] + N[k] - 4) >> 1) - sD[pos] - sD[k];
			if(q <= Q[k] && (P[k] < pos || q < Q[k])) {
				Q[k] = q;
				P[k] = pos;
			}
		}
	}
}

/* dnj.c:1020-1052, the DNJ loop from candidate row j: minQpair, limbLength,
 * updateD, updateDNJ, DNJ_popArrange, minPos.  *np is the matrix size (updated);
 * returns the joins made.  next_cand (may be NULL) receives the candidate the
 * loop would start its next minQpair from (the state a resume continues). */
static int dnj_loop(Ltd *D, int *np, double *sD, int32_t *N, double *Q, int32_t *P, int j, int neg,
                    orc_join *joins, int lim, int64_t *stats, int threads, int *next_cand) {
	int n = *np, nj = 0;
	int *rows = NULL, *fj = NULL;
	double *fq = NULL;
	if(threads > 1) {
		rows = malloc(RESCAN_BATCH_ROWS * sizeof(int));
		fj = malloc(RESCAN_BATCH_ROWS * sizeof(int));
		fq = malloc(RESCAN_BATCH_ROWS * sizeof(double));
	}
	uint64_t pos;
	while(n != 2 && nj < lim &&
	      (pos = threads > 1 ? min_q_pair_par(D, n, sD, N, Q, P, j, stats, threads, rows, fq, fj)
	                         : min_q_pair(D, n, sD, N, Q, P, j, stats))) {
		j = (int) (pos & 0xFFFFFFFFu);
		int i = (int) (pos >> 32);
		double Li, Lj;
		limb_length(&Li, &Lj, i, j, sD, N, ld(D, tri(i) + j), neg);
		joins[nj].i = i; joins[nj].j = j; joins[nj].Li = Li; joins[nj].Lj = Lj; ++nj;
		update_d(D, n, sD, N, i, j, Li, Lj);
		int mi = update_dnj_q(D, n, sD, N, Q, P, i, j);
		int mj = dnj_pop_arrange(D, &n, sD, N, Q, P, i);
		if(mj == n) {
			j = mi;
		} else if(mi == n) {
			j = mj;
		} else {
			j = min_pos(Q, mi, mj);
		}
	}
	free(rows);
	free(fj);
	free(fq);
	*np = n;
	if(next_cand) *next_cand = j;
	return nj;
}

int orc_tree(int n, int etype, double byteScale, void *Dbase, int method, int flags,
             orc_join *joins, int *final_n, double *final_d, int64_t *stats) {
	return orc_tree_ex(n, etype, byteScale, Dbase, method, flags, joins, final_n, final_d, stats, 0, 1);
}

int orc_tree_ex(int n, int etype, double byteScale, void *Dbase, int method, int flags,
                orc_join *joins, int *final_n, double *final_d, int64_t *stats, int max_joins, int threads) {
	/* max_joins > 0: stop after that many joins (a prefix of the same run) */
	const int lim = max_joins > 0 ? max_joins : INT_MAX;
	Ltd D = {etype, byteScale, Dbase};
	int neg = (flags & 2) != 0;
	int nj = 0;
	double *sD = malloc((size_t) (n > 0 ? n : 1) * sizeof(double));
	double *Q = malloc((size_t) (n > 0 ? n : 1) * sizeof(double));
	int32_t *N = malloc((size_t) (n > 0 ? n : 1) * sizeof(int32_t));
	int32_t *P = malloc((size_t) (n > 0 ? n : 1) * sizeof(int32_t));
	if(stats) {
		stats[0] = stats[1] = 0;
	}
	init_sums_par(&D, n, sD, N, threads);
	if(method == 0) {
		/* nj.c:1560-1610 */
		uint64_t pair;
		while(n != 2 && nj < lim && (pair = init_q(&D, n, sD, N))) {
			int j = (int) (pair & 0xFFFFFFFFu), i = (int) (pair >> 32);
			double Li, Lj;
			limb_length(&Li, &Lj, i, j, sD, N, ld(&D, tri(i) + j), neg);
			joins[nj].i = i; joins[nj].j = j; joins[nj].Li = Li; joins[nj].Lj = Lj; ++nj;
			update_d(&D, n, sD, N, i, j, Li, Lj);
			--n;
			pop_arrange(&D, n, i);
			sD[i] = sD[n];
			N[i] = N[n];
		}
	} else if(method == 2) {
		/* hclust.c:1671-1718 hclust with initHNJ / minQ / updateHNJ / HNJ_popArrange */
		init_hnj_par(&D, n, sD, N, Q, P, threads);
		while(n != 2 && nj < lim) {
			int i = min_q_row(Q, n);
			int j = P[i];
			if(i == 0 && j == 0) {
				break;
			}
			double Li, Lj;
			limb_length(&Li, &Lj, i, j, sD, N, ld(&D, tri(i) + j), neg);
			joins[nj].i = i; joins[nj].j = j; joins[nj].Li = Li; joins[nj].Lj = Lj; ++nj;
			update_d(&D, n, sD, N, i, j, Li, Lj);
			update_hnj_q(&D, n, sD, N, Q, P, i, j);
			hnj_pop_arrange(&D, &n, sD, N, Q, P, i);
		}
	} else {
		/* dnj.c:985-1052 */
		init_hnj_par(&D, n, sD, N, Q, P, threads);
		nj = dnj_loop(&D, &n, sD, N, Q, P, min_q_row(Q, n), neg, joins, lim, stats, threads, NULL);
	}
	*final_n = n;
	*final_d = n == 2 ? ld(&D, 0) : -1.0;
	free(sD);
	free(Q);
	free(N);
	free(P);
	return nj;
}

int orc_dnj_init(int n, int etype, double byteScale, const void *Dbase, double *sD, double *Q, int32_t *N, int32_t *P,
                 int threads) {
	Ltd D = {etype, byteScale, (void *) Dbase};
	init_sums_par(&D, n, sD, N, threads);
	init_hnj_par(&D, n, sD, N, Q, P, threads);
	return min_q_row(Q, n);
}

int orc_dnj_resume(int n, int etype, double byteScale, void *Dbase, double *sD, double *Q, int32_t *N, int32_t *P,
                   int cand, int flags, orc_join *joins, int *final_n, double *final_d, int64_t *stats,
                   int max_joins, int threads, int *next_cand) {
	Ltd D = {etype, byteScale, Dbase};
	if(stats) {
		stats[0] = stats[1] = 0;
	}
	int nj = dnj_loop(&D, &n, sD, N, Q, P, cand, (flags & 2) != 0, joins, max_joins > 0 ? max_joins : INT_MAX, stats,
	                  threads, next_cand);
	*final_n = n;
	*final_d = n == 2 ? ld(&D, 0) : -1.0;
	return nj;
}
