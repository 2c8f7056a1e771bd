/*
 * ccoracle.h -- CPU restatement of ccphylo's dist/tree hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in ccphylo_amd/ links, loads or calls
 * this code: it is the checker used by tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg.  Parity of this restatement is pinned against
 * the reference binary built by oracle/Makefile (golden vectors committed in
 * tests/golden/, see tests/golden/gen_golden.py).
 *
 * Element types of the lower-triangular matrix follow the reference
 * (matrix.c:59-71): 8 = double, 4 = float, 2 = u16, 1 = u8 (ByteScale-scaled).
 */
#ifndef CCORACLE_H
#define CCORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
	int32_t i, j;      /* rows joined (j < i), numbering at the time of the join */
	double Li, Lj;     /* limb lengths (nj.c:42 limbLength) */
} orc_join;

/* A1: byte -> code table (fsacmp.c:32 get2BitTable) */
void orc_code_table(unsigned flag, uint8_t table[256]);
/* A2: MSB-first 2-bit packing, 32 nt / u64 (qseqs.c:60 qseq2nibble); returns #code-4 */
int orc_pack(const uint8_t *codes, int len, uint64_t *out);
/* A3: include masks (fsacmp.c:164 initIncPos, :181/:240/:296 getIncPos*, :487 getNpos)
 * variant: 0 = getIncPos, 8 = getIncPosInsig, 32 = getIncPosInsigPrune */
void orc_init_inc(uint32_t *inc, int len);
void orc_inc_update(uint32_t *inc, uint8_t *seq, uint8_t *ref, int len, unsigned proxi, int variant);
int orc_npos(const uint32_t *inc, int len);
/* A4/A5 (fsacmp.c:552 fsacmp, :587 fsacmpair) */
uint32_t orc_fsacmp(const uint64_t *a, const uint64_t *b, const uint32_t *inc, int len);
uint64_t orc_fsacmpair(const uint64_t *a, const uint64_t *b, const uint32_t *inc, int len);
/* A5 pairwise mask with proximity (fsacmp.c:355 maskProxi) */
void orc_mask_proxi(uint32_t *out, const uint32_t *inc1, const uint32_t *inc2,
                    const uint64_t *s1, const uint64_t *s2, unsigned len, unsigned proxi);

/* A6/A7: fill the LT matrix of n included taxa in reference order
 * (fsacmpthrd.c:108 cmpFsaThrd, :261 cmpairFsaThrd).  seqs: n x W u64
 * (W = len/32 + 1 words per taxon, stride W), incs: 1 x W (non-pair) or
 * n x W (pair).  N may be NULL.  Returns the non-pair "inc" (getNpos). */
int orc_snp_ltd(int n, int len, const uint64_t *seqs, const uint32_t *incs, int pair,
                unsigned norm, unsigned minLength, double minCov, unsigned proxi,
                int etype, double byteScale, void *D, void *N);

/* C/D: tree construction.  D is the packed LT matrix (destroyed).
 * method: 0 = nj (nj.c:1560), 1 = dnj (dnj.c:985), 2 = hnj (hclust.c:1671).  flags: tree -f
 * (2 = limbLengthNeg).  Writes up to n-2 joins, returns the number of joins;
 * *final_n receives D->n at exit and *final_d the last pair's distance
 * (valid when *final_n == 2).  stats (may be NULL): [0] rows rescanned,
 * [1] cells rescanned (dnj only). */
int orc_tree(int n, int etype, double byteScale, void *D, int method, int flags,
             orc_join *joins, int *final_n, double *final_d, int64_t *stats);

/* orc_tree with a join limit (max_joins > 0: the first max_joins joins of the
 * same run) and `threads` pthreads for the O(n^2) initSummaD / initHNJ passes
 * (same per-row operation order) and DNJ's minQpair rescans (same decisions,
 * see min_q_pair_par), so bit-identical to threads = 1. */
int orc_tree_ex(int n, int etype, double byteScale, void *D, int method, int flags,
                orc_join *joins, int *final_n, double *final_d, int64_t *stats, int max_joins, int threads);

/* Resume the DNJ loop (dnj.c:1020-1052) from a saved state: D holds the LT of
 * the current n rows, sD/Q/N/P the per-row vectors after the last join (as
 * the next minQpair reads them) and cand the candidate row minPos chose
 * (dnj.c:1026-1032).  The arrays are updated in place; *next_cand (may be
 * NULL) receives the candidate for a further resume.  threads > 1 rescans
 * minQpair's rows with pthreads (same decisions, see min_q_pair_par). */
int orc_dnj_resume(int n, int etype, double byteScale, void *D, double *sD, double *Q, int32_t *N, int32_t *P,
                   int cand, int flags, orc_join *joins, int *final_n, double *final_d, int64_t *stats,
                   int max_joins, int threads, int *next_cand);

/* The state orc_dnj_resume starts a whole DNJ run from: initSummaD
 * (nj.c:111), initHNJ (hclust.c:56) and the first candidate (minQ,
 * hclust.c:353, as dnj.c:1015).  Returns the candidate row. */
int orc_dnj_init(int n, int etype, double byteScale, const void *D, double *sD, double *Q, int32_t *N, int32_t *P,
                 int threads);

/* orc_snp_ltd with `threads` pthreads over the LT rows (same cells). */
int orc_snp_ltd_ex(int n, int len, const uint64_t *seqs, const uint32_t *incs, int pair,
                   unsigned norm, unsigned minLength, double minCov, unsigned proxi,
                   int etype, double byteScale, void *D, void *N, int threads);

/* B1/B2: distances between KMA count matrices (*.mat[.gz]) of template
 * `tmpl` (ltdmatrixthrd.c:376 ltdMatrixThrd, matcmp.c:448 cmpMats, metrics
 * matcmp.c:63-446; kma_oracle.c).  D/N receive the packed LT of the *n_out
 * included samples (room for nfiles(nfiles-1)/2 elements; N may be NULL);
 * include[nfiles] the inclusion flags.  Returns 0; -2 where the reference
 * exits(1) ("did not exceed threshold", ltdmatrixthrd.c:337); -3 when a file
 * cannot be read. */
#define ORC_KMA_COS    0
#define ORC_KMA_CHI2   2
#define ORC_KMA_NCHI2  3
#define ORC_KMA_NC     4
#define ORC_KMA_C      5
#define ORC_KMA_NBC    8
#define ORC_KMA_BC     9
#define ORC_KMA_NL1   10
#define ORC_KMA_NL2   11
#define ORC_KMA_NLINF 12
#define ORC_KMA_L1    13
#define ORC_KMA_L2    14
#define ORC_KMA_LINF  15
#define ORC_KMA_LN    16
#define ORC_KMA_NLN   17
int orc_kma_dist(int nfiles, const char **files, const char *tmpl, int metric, unsigned lnorm, unsigned norm,
                 unsigned minDepth, unsigned minLength, double minCov, int etype, double bs, void *D, void *N,
                 unsigned char *include, int *n_out);

/* initSummaD (nj.c:111) on its own, for unit tests */
void orc_init_sums(int n, int etype, double byteScale, const void *D, double *sD, int32_t *N);

#ifdef __cplusplus
}
#endif
#endif
