/*
 * ccphylo_host.h -- host-side stable API surface of ccphylo_amd (plain C).
 *
 * These are the reference's I/O boundaries re-implemented (not copied) so
 * that `ccphylo dist` / `ccphylo tree` stay byte-compatible:
 *   - Phylip reader / writer            (ref phy.c:251 loadPhy, phy.c:59 printphy)
 *   - Newick builder, replayed from the join list produced on the GPU
 *                                       (ref nwck.c:35 formNode, :79 formLastNode,
 *                                        :114 formLastBiNode, str.c:51 byteshift)
 *   - FASTA / MSA loading, 2-bit packing and include masks
 *                                       (ref seqparse.c:28, qseqs.c:60, fsacmp.c:32-503,
 *                                        cdist.c:196 ltdMsaMatrix_get)
 * All compute on the hot path goes through include/ccphylo_amd.h.
 */
#ifndef CCPHYLO_HOST_H
#define CCPHYLO_HOST_H
#include <stdint.h>
#include <stdio.h>

#ifdef __cplusplus
extern "C" {
#endif

/* growable byte string with the reference's capacity semantics (qseqs.h) */
typedef struct {
	uint32_t size;   /* capacity in bytes; drives Newick child order (nwck.c:45) */
	uint32_t len;
	unsigned char *seq;
} ccq_str;

ccq_str *ccq_new(uint32_t size);
void ccq_free(ccq_str *s);

/* ---- buffered, gzip-transparent reader (ref filebuff.c:52) ---- */
typedef struct ccq_reader ccq_reader;
ccq_reader *ccq_open(const char *path);          /* "-" = stdin; NULL on failure */
void ccq_close(ccq_reader *r);
int ccq_peek(ccq_reader *r);                      /* EOF at end */

/* ---- Phylip ---- */
/* A loaded matrix: packed LT, element type et (8/4/2/1), ByteScale bs. */
typedef struct {
	int n;
	int size;              /* allocated rows (matrix.h `size`) */
	int et;
	double bs;
	void *mat;             /* n(n-1)/2 elements of et bytes */
} ccq_ltd;

ccq_ltd *ccq_ltd_new(int size, int et, double bs);
void ccq_ltd_free(ccq_ltd *D);
void ccq_ltd_reserve(ccq_ltd *D, int size);
double ccq_ltd_get(const ccq_ltd *D, int64_t flat);
void ccq_ltd_set(ccq_ltd *D, int64_t flat, double v, double round);

/* Name table reused across matrices, as in tree.c:61-66 + phy.c:360-379. */
typedef struct {
	int cap;               /* entries allocated */
	ccq_str **names;
	ccq_str *header;       /* '#' comment line of the current matrix */
} ccq_names;

ccq_names *ccq_names_new(int n, uint32_t init_size);
void ccq_names_free(ccq_names *T);

/* Names 0..n-1 as `ccphylo dist | ccphylo tree` would hold them: the field
 * ccq_print_phy writes for names[i] under `format` (phy.c:59), stored the
 * way ccq_load_phy reads a row "field<sep>" (phy.c:360-379: byte by byte
 * with capacity doubling, trailing white space trimmed), so a Newick
 * replayed over them has that pipeline's child order (nwck.c:45 compares
 * capacities).  Used by the fused `dist --tree` path. */
void ccq_names_set(ccq_names *T, char **names, int n, unsigned format, char sep);

/* Loads the next matrix (phy.c:251 semantics).  Returns n (0 at EOF / on a
 * malformed file, with *err set), grows D and T as needed. */
int ccq_load_phy(ccq_reader *r, ccq_ltd *D, ccq_names *T, char sep, char quotes, int *err);

/* phy.c:59 printphy.  names[i] are C strings (may be modified by the quote
 * strip, as in the reference).  include may be NULL.  format bit 1 =
 * relaxed names, bit 4 = comment line. */
void ccq_print_phy(FILE *out, const ccq_ltd *D, char **names, const unsigned char *include,
                   const char *comment, unsigned format, int precision);

/* ---- Newick replay (GPU join list -> tree string) ---- */
typedef struct {
	int32_t i, j;          /* rows joined (j < i) at the time of the join */
	double Li, Lj;
} ccq_join;

/* Applies formNode(names[j], names[i], Lj, Li) and the row exchange for
 * every join, then the closing node(s) (dnj.c:1024-1049 / nj.c:1581-1607).
 * n0 = taxa at start, final_n / final_d as returned by the engine.
 * flags: tree -f (1 = bifurcating root).  Result in T->names[0]. */
void ccq_replay_newick(ccq_names *T, int n0, const ccq_join *joins, int njoins,
                       int final_n, double final_d, int flags, int precision);
/* The same bytes by editing the strings join by join as nwck.c does (O(N^2)
 * bytes for caterpillar trees); ccq_replay_newick replays only capacities and
 * lengths, then writes the string once.  Kept for tests and comparison. */
void ccq_replay_newick_strings(ccq_names *T, int n0, const ccq_join *joins, int njoins,
                               int final_n, double final_d, int flags, int precision);
/* tree.c:95-97: a two-taxon matrix */
void ccq_newick_pair(ccq_names *T, double d, int precision);

/* ---- FASTA / MSA ---- */
void ccq_code_table(unsigned flag, unsigned char table[256]);
/* seqparse.c:28 FileBuffgetFsa: header (with '>') and codes (< 8 kept) */
int ccq_read_fasta(ccq_reader *r, ccq_str *header, ccq_str *seq, const unsigned char *table);
int ccq_pack(const unsigned char *codes, int len, uint64_t *out);
void ccq_init_inc(uint32_t *inc, int len);
void ccq_inc_update(uint32_t *inc, unsigned char *seq, unsigned char *ref, int len, unsigned proxi, int variant);
int ccq_npos(const uint32_t *inc, int len);

/* An MSA loaded per ltdMsaMatrix_get (cdist.c:196-333): included taxa only,
 * packed seqs (stride W = len/32 + 1 words) and mask(s). */
typedef struct {
	int n, len, W, pair;
	char **headers;
	uint64_t *seqs;        /* n * W */
	uint32_t *incs;        /* W (non-pair) or n * W (pair) */
	unsigned minLength;    /* after the minCov adjustment (cdist.c:289) */
} ccq_msa;

/* Reads every record; logs "# Included/# Excluded" to `log` like the
 * reference.  variant: 0, 8 or 32 (dist.c:802-806). */
ccq_msa *ccq_load_msa(ccq_reader *r, unsigned flag, unsigned minLength, double minCov,
                      unsigned proxi, FILE *log);
void ccq_msa_free(ccq_msa *M);
/* The same result as ccq_load_msa, the per-sequence work (codes, packing,
 * include masks) on `threads` host threads over windows of the input
 * (fasta_par.c); the Included/Excluded lines and the length-mismatch exit
 * come in record order as the reference prints them. */
ccq_msa *ccq_load_msa_par(ccq_reader *r, unsigned flag, unsigned minLength, double minCov, unsigned proxi, int threads,
                          FILE *log);

/* Multi-file FASTA with -r (cdist.c:36 ltdFsaMatrix_get): entry `tmpl` of
 * every file; n = nfiles (every file keeps its slot), include[nfiles] the
 * inclusion flags.  NULL where the reference exits(1). */
ccq_msa *ccq_load_fsa_files(char **files, int nfiles, const char *tmpl, unsigned flag, unsigned minLength,
                            double minCov, unsigned proxi, unsigned char *include, FILE *log);

/* KMA count matrices (*.mat[.gz]) of template `tmpl` for ccg_kma_ltd
 * (ltdmatrixthrd.c:376 ltdMatrixThrd's inclusion rules; every file read once,
 * `threads` at a time).  Exclusions are logged like the reference. */
typedef struct {
	int nfiles, n;             /* files given, samples included */
	int status;                /* 0, or -3 when a file cannot be read */
	unsigned char *include;    /* per file */
	int *file_of;              /* included sample -> file index */
	int64_t stride1, stride2;  /* rows per sample in rec1 / rec2 */
	uint16_t *rec1, *rec2;     /* n x stride x 8 (see ccg_kma_args) */
	int32_t *len1, *len2;
} ccq_kma;
ccq_kma *ccq_load_kma(char **files, int nfiles, const char *tmpl, unsigned minDepth, unsigned minLength,
                      double minCov, int threads, FILE *log);
void ccq_kma_free(ccq_kma *K);

#ifdef __cplusplus
}
#endif
#endif
