/*
 * ccphylo_amd.h -- C-ABI of the MI355X (gfx950) hot-path engine.
 *
 * Plain pointers and sizes only.  Every entry point is synchronous to the
 * caller; the *_dev ones first wait for all prior work on the device, so
 * their inputs may be produced on any stream (e.g. PyTorch's).  Each returns
 * 0 or a negative CCG_E* code (never exit()s, unlike the
 * reference's ERROR(), pherror.h:28).  There is no CPU fallback: if the HIP
 * runtime or a gfx950 device is missing, ccg_init fails with CCG_ENODEV.
 *
 * Drop-in mapping (reference ccphylo 0.8.5):
 *   ccg_snp_ltd   replaces fsaCmpThreadOut(tnum, &cmpFsaThrd | &cmpairFsaThrd, D, N, ...)
 *                 declared fsacmpthrd.h:49, impl fsacmpthrd.c:76-106,
 *                 called from cdist.c:351/:354 (MSA) and cdist.c:181/:184.
 *   ccg_kma_ltd   replaces the per-pair cmpMats (matcmp.c:448) calls of
 *                 ltdMatrixThrd (ltdmatrixthrd.h:52, called dist.c:168):
 *                 distances between KMA count matrices (*.mat); the host
 *                 loader (ccq_load_kma) reads every sample once.
 *   ccg_tree_shard  the same loop with the LT rows split over ranks
 *                 (SURVEY.md 8(e)), one process per GPU, collectives over
 *                 RCCL (ccg_rccl_open) or a caller-supplied transport.
 *   ccg_tree      replaces dnj_thread(D, sD, Q, N, names, t) (dnj.c:1054,
 *                 called tree.c:89) and nj_thread(D, sD, N, names, t)
 *                 (nj.c:1612, called tree.c:91).  It returns the join list;
 *                 the Newick string is rebuilt on the host by replaying
 *                 formNode (nwck.c:35) over it -- see include/ccphylo_host.h.
 */
#ifndef CCPHYLO_AMD_H
#define CCPHYLO_AMD_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CCG_OK        0
#define CCG_EINVAL   -1   /* bad argument */
#define CCG_ENODEV   -2   /* no HIP device / not gfx950 */
#define CCG_ENOMEM   -3   /* device allocation failed */
#define CCG_EHIP     -4   /* other HIP runtime error */
#define CCG_EUNSUP   -5   /* valid request the GPU engine does not implement */

typedef struct ccg_ctx ccg_ctx;

/* Opens `device` (ordinal in HIP_VISIBLE_DEVICES numbering) and creates the
 * engine stream.  Fails with CCG_ENODEV when no gfx950 device is present. */
int ccg_init(int device, ccg_ctx **ctx);

/* Optional, after ccg_init: cu_mask (mask_words 32-bit words, bit k = CU k;
 * 0 words: the whole chip again) limits the context's stream to those compute
 * units (hipExtStreamCreateWithCUMask), so that two contexts of one device can
 * run side by side -- e.g. one matrix's dist beside the previous matrix's tree.
 * On gfx950 bit k is a CU of XCD k % 8 (the first 64 bits: 8 CUs per XCD);
 * a mask that leaves an XCD without a CU is CCG_EINVAL (that XCD would run
 * unmasked).  Within an XCD, bit k sits on shader engine (k / 8) % 4, and
 * blocks are dealt round-robin over engines as over XCDs: a context runs like
 * 32 x its fewest CUs on one engine, so masks of 32 j bits (j per engine) are
 * the ones that pay (bits 0..55 run like 32 CUs).  May be called again; the
 * previous stream is drained first.
 * A CU-masked stream is never destroyed (a ROCm 7.2 runtime defect: a later
 * stream's kernels hang after one is destroyed; tools/micro/cu_mask.hip), so
 * each masked configuration keeps one HIP stream until the process exits.
 * flags CCG_CTX_NOSYNC: the device-pointer entry points do not wait for the
 * whole device first (the caller orders its inputs; a device-wide wait would
 * wait for the other context's work), and the context keeps its workspaces
 * -- the tree's, and the dist's bit planes (about n x L / 4 bytes) -- until
 * ccg_destroy, so that no call frees device memory (hipFree waits for every
 * stream of the device). */
#define CCG_CTX_NOSYNC 1
int ccg_ctx_configure(ccg_ctx *ctx, const uint32_t *cu_mask, int mask_words, int flags);
/* Process end, after the last HIP work of the process: destroys the CU-masked
 * streams ccg_ctx_configure kept (no HIP stream may be created afterwards;
 * contexts configured with a mask are unusable).  Optional: without it they
 * go with the process (ccphylo_amd's Python layer calls it at exit; under
 * rocprofv3 a Python + torch process that still held masked streams at
 * teardown segfaulted in __cxa_finalize, profiles/r06_exit_rocprof.txt). */
int ccg_shutdown(void);
/* HIP devices visible to this process (the multi-GPU CLI deals ranks over them) */
int ccg_device_count(int *count);
void ccg_destroy(ccg_ctx *ctx);
const char *ccg_strerror(int code);
/* device name + arch, for logs */
int ccg_device_info(ccg_ctx *ctx, char *buf, size_t len);

/* ------------------------------------------------------------------ */
/* dist: all-pairs SNP distances (fsacmp.c:552 / :587 per pair)        */
/* ------------------------------------------------------------------ */
typedef struct {
	int n;                 /* taxa, all included (cdist.c:331 include[] == 1) */
	int len;               /* alignment length */
	int stride;            /* u64 words per taxon in seqs/incs rows (>= ceil(len/32)) */
	const uint64_t *seqs;  /* n*stride words, qseq2nibble layout (qseqs.c:60) */
	const uint32_t *incs;  /* stride words (pair = 0) or n*stride (pair = 1), fsacmp.c:164 layout */
	int pair;              /* 0: cmpFsaThrd semantics, 1: cmpairFsaThrd semantics */
	unsigned norm;         /* -W */
	unsigned minLength;    /* already max(minLength, minCov*len) (cdist.c:289) */
	unsigned proxi;        /* -P; pair mode: maskProxi (fsacmp.c:355) per pair */
	int etype;             /* 8 double, 4 float, 2 u16, 1 u8 (matrix.c:59-71) */
	double byteScale;      /* ByteScale for etype 2/1 (bytescale.c:45) */
	int64_t row_begin;     /* LT rows [row_begin, row_end) to compute; 0,0 = all */
	int64_t row_end;
} ccg_snp_args;

/* Host buffers: D (and N when pair && N != NULL) receive the packed LT of
 * n(n-1)/2 elements of `etype` bytes in reference cell order (pi, pj).  With
 * a row range, only cells of those rows are written (offsets still global).
 * *inc_out (may be NULL) receives getNpos(mask) for pair == 0. */
int ccg_snp_ltd(ccg_ctx *ctx, const ccg_snp_args *a, void *D, void *N, int *inc_out);

/* Same, with a->seqs / a->incs and D / N all DEVICE pointers (HBM-resident
 * pipeline: dist writes the LT that ccg_tree_dev consumes in place). */
int ccg_snp_ltd_dev(ccg_ctx *ctx, const ccg_snp_args *a, void *D_dev, void *N_dev, int *inc_out);

/* Duration of the last dist call's pair kernels on this context (the
 * compare and epilogue launches, without the bit-plane build), from HIP
 * events on the engine stream; benchmarks use it for the roofline. */
int ccg_last_dist_ms(ccg_ctx *ctx, double *ms);

/* ------------------------------------------------------------------ */
/* dist on KMA count matrices (matcmp.c:448 cmpMats per pair)          */
/* ------------------------------------------------------------------ */
/* -d metrics (dist.c:736-790 names -> these ids) */
#define CCG_KMA_COS    0   /* cos (default)  matcmp.c:420 */
#define CCG_KMA_CHI2   2   /* chi2   :381 */
#define CCG_KMA_NCHI2  3   /* nchi2  :396 */
#define CCG_KMA_NC     4   /* nc     :243 */
#define CCG_KMA_C      5   /* c      :278 */
#define CCG_KMA_NBC    8   /* nbc    :206 */
#define CCG_KMA_BC     9   /* bc     :227 */
#define CCG_KMA_NL1   10   /* nl1    :63 */
#define CCG_KMA_NL2   11   /* nl2    :81 */
#define CCG_KMA_NLINF 12   /* nlinf  :122 */
#define CCG_KMA_L1    13   /* l1     :143 */
#define CCG_KMA_L2    14   /* l2     :158 */
#define CCG_KMA_LINF  15   /* linf   :193 */
#define CCG_KMA_LN    16   /* l<n>   :173 (pow: parity within 1e-12 relative) */
#define CCG_KMA_NLN   17   /* nl<n>  :98  (pow: parity within 1e-12 relative) */

/* One position of a sample: 8 u16 = counts A C G T - N, then the u32 depth
 * total (little endian), the row layout of FileBuffLoadMat (matparse.c:213). */
typedef struct {
	int n;                  /* included samples, in LT row order */
	int metric;             /* CCG_KMA_* */
	unsigned lnorm;         /* n of l<n> / nl<n> */
	unsigned norm;          /* -W */
	unsigned minDepth;      /* -E */
	unsigned minLength;     /* -L */
	double minCov;          /* -C / 100 */
	int etype;              /* 8, 4, 2, 1 */
	double byteScale;
	int64_t stride1;        /* rows per sample in rec1 */
	const uint16_t *rec1;   /* n x stride1 x 8: a sample as the row sample (mat1,
	                           after stripMat matcmp.c:27), zero past len1 */
	const int32_t *len1;    /* mat1->len after stripMat */
	int64_t stride2;        /* rows per sample in rec2 */
	const uint16_t *rec2;   /* n x stride2 x 8: a sample as the column sample
	                           (its rows with ref != '-', in order) */
	const int32_t *len2;    /* rows in rec2 */
} ccg_kma_args;

/* Host buffers.  D / N (N may be NULL) receive the packed LT of n elements
 * of `etype` in reference cell order: cell (i, j) = cmpMats(sample i as mat1,
 * sample j as mat2).  *fatal (may be NULL) receives the flat index of the
 * first cell where cmpMats returns -2 -- the reference then exits(1)
 * ("did not exceed threshold", ltdmatrixthrd.c:337) -- or -1. */
int ccg_kma_ltd(ccg_ctx *ctx, const ccg_kma_args *a, void *D, void *N, int64_t *fatal);
/* Same with rec1/len1/rec2/len2 and D/N all device pointers. */
int ccg_kma_ltd_dev(ccg_ctx *ctx, const ccg_kma_args *a, void *D_dev, void *N_dev, int64_t *fatal);

/* ------------------------------------------------------------------ */
/* tree: NJ / DNJ on an HBM-resident packed LT matrix                  */
/* ------------------------------------------------------------------ */
typedef struct {
	int32_t i, j;          /* rows joined (j < i) at the time of the join */
	double Li, Lj;         /* limb lengths (nj.c:42 / :81) */
} ccg_join;

#define CCG_TREE_NJ   0    /* -m nj  (nj.c:1560, the -t 1 semantics) */
#define CCG_TREE_DNJ  1    /* -m dnj (dnj.c:985, default) */
#define CCG_TREE_HNJ  2    /* -m hnj (hclust.c:1671: initHNJ, minQ, updateHNJ, HNJ_popArrange) */

typedef struct {
	int n;                 /* taxa (> 2) */
	int etype;             /* 8, 4, 2, 1 */
	double byteScale;
	int method;            /* CCG_TREE_NJ / CCG_TREE_DNJ / CCG_TREE_HNJ */
	int flags;             /* tree -f: bit 2 = limbLengthNeg (nj.c:81) */
	int exact;             /* 1: row sums of a join accumulated serially in the
	                          reference order (bit-identical to the reference);
	                          0: fixed-order parallel tree sum (deterministic,
	                          may differ from the reference in the last ulp) */
	int profile;           /* 1: time every kernel with HIP events on the engine
	                          stream; per-kernel totals go to stats[4..] */
	int max_joins;         /* > 0: stop after this many joins (benchmarks time a
	                          prefix of a large tree); 0: run to n = 2 */
} ccg_tree_args;

/* stats layout (ccg_tree / ccg_tree_dev / ccg_tree_shard*, 12 + 2*CCG_NKSTAT
 * entries when profile = 1, else 4): [0] rows listed for rescans, [1] cells
 * rescanned (loaded; the single engine's scan may prune listed rows), [2] kernel launches, [3] device time (us); then for kernel class
 * c: [4+2c] launches, [5+2c] summed duration in ns; then [4+2*CCG_NKSTAT]
 * cells rescanned by CCG_K_TOP and [5+2*CCG_NKSTAT] by CCG_K_REST;
 * [6+2*CCG_NKSTAT] exact row sums that needed the serial order,
 * [7+2*CCG_NKSTAT] of those computed by the serial chain (the parallel form
 * declined); [8+2*CCG_NKSTAT]: single engine, the cells of S (part of [1])
 * that k_dnj_plan's helper blocks rescanned (pruning, CCG_K_FIND's bytes);
 * sharded engines, the bytes this rank put into the initSummaD collectives;
 * sharded engines only: [9+2*CCG_NKSTAT] columns whose column part
 * went through the serial gather (the rest are exact sums of per-rank
 * statistics); DNJ: [10+2*CCG_NKSTAT] rows and [11+2*CCG_NKSTAT] cells that
 * the reference's own minQpair rule rescans (dnj.c:78, a row whose stored Q is
 * below the running min), counted from the replay's accept decisions: the
 * SURVEY 8(d) unit beside the engine's speculative [0] / [1].  Classes: */
#define CCG_K_INIT     0   /* initSummaD / initHNJ / first candidate */
#define CCG_K_TOP      1   /* sharded DNJ k_dnj_select: requeue fold, top rows S, their rescans */
#define CCG_K_REST     2   /* DNJ k_dnj_scan: rescans of the listed rows (one GPU: S and the rows below it) */
#define CCG_K_ARGMIN   3   /* NJ: full Q argmin (initQ) */
#define CCG_K_UPDATE   4   /* updateD (DNJ: after minQpair's replay; NJ: after the argmin fold) */
#define CCG_K_REQUEUE  5   /* DNJ: updateDNJ Q/P + DNJ_popArrange */
#define CCG_K_POP      6   /* NJ: ltdMatrix_popArrange */
#define CCG_K_FIND     7   /* DNJ k_dnj_plan (one GPU: requeue fold, S, partner-cell bound, entry
                              list) / k_dnj_find (sharded: bound U and the rows below S) */
#define CCG_K_COLL     8   /* sharded engine: collectives (enqueue time, or the
                              host round trip of a host-staged transport) */
#define CCG_K_XSUM     9   /* exact mode: k_exact_sum, the serial-order row sum of j */
#define CCG_NKSTAT     10

/* D: host LT (n(n-1)/2 elements), left unmodified.  joins: room for n-2.
 * On return *njoins joins were made; *final_n is the matrix size at exit
 * (2 normally; > 2 when the reference loop would stop early with pos == 0)
 * and *final_d the remaining pair's distance (D(1,0)) when *final_n == 2.
 * stats (may be NULL, 4 entries): [0] rows rescanned, [1] cells rescanned,
 * [2] kernel launches, [3] device time in microseconds. */
int ccg_tree(ccg_ctx *ctx, const ccg_tree_args *a, const void *D,
             ccg_join *joins, int *njoins, int *final_n, double *final_d, int64_t *stats);

/* Same on a DEVICE LT buffer, which is consumed (overwritten). */
int ccg_tree_dev(ccg_ctx *ctx, const ccg_tree_args *a, void *D_dev,
                 ccg_join *joins, int *njoins, int *final_n, double *final_d, int64_t *stats);

/* A DNJ loop state between two joins (dnj.c:985-1052): what the next
 * minQpair (dnj.c:43) reads.  Host arrays of at least n entries. */
typedef struct {
	int n;                 /* matrix size (D holds its n(n-1)/2 cells) */
	int cand;              /* minQpair's candidate row (minPos, dnj.c:1026-1032) */
	double *sD, *Q;        /* row sums (initSummaD / updateD) and stale row minima */
	int32_t *N, *P;        /* taxa counts and the rows' partners */
} ccg_dnj_state;

/* ccg_tree_dev with CCG_TREE_DNJ, checkpointed: `in` (may be NULL) starts the
 * loop from that state instead of initSummaD / initHNJ (D_dev holds its LT,
 * a->n == in->n); `out` (may be NULL) receives the state at exit, after
 * a->max_joins joins, D_dev then holding its LT.  A run from `in` makes the
 * joins the uninterrupted run makes after the same state (bit-identical; the
 * reference has no checkpoint, so this is its loop split in two).  The single
 * GPU engine only (no sharding); out->n = 0 if the loop stopped (pos == 0)
 * or finished (n == 2: no join is left to resume). */
int ccg_tree_dev_state(ccg_ctx *ctx, const ccg_tree_args *a, void *D_dev, const ccg_dnj_state *in,
                       ccg_dnj_state *out, ccg_join *joins, int *njoins, int *final_n, double *final_d,
                       int64_t *stats);

/* ------------------------------------------------------------------ */
/* sharded tree: one LT matrix split over `world` ranks  */
/* ------------------------------------------------------------------ */
/* Row ownership: bands of CCG_SHARD_BAND consecutive LT rows are dealt
 * round-robin, band b = rows [8b, 8b+8) to rank b % world, so the rows the
 * join loop drops from the end (ltdMatrix_popArrange, matrix.c:518) drain
 * every rank evenly.  A rank stores its rows in increasing order, back to
 * back, row r holding its r elements (columns 0..r-1) as in the reference's
 * LT buffer (matrix.c:74-83). */
#define CCG_SHARD_BAND 8
int ccg_shard_owner(int64_t row, int world);
/* element offset of an owned row in its rank's buffer */
int64_t ccg_shard_row_offset(int64_t row, int rank, int world);
/* elements of a rank's rows below n (the size of its buffer for n taxa) */
int64_t ccg_shard_elems(int64_t n, int rank, int world);

/* The collectives of the sharded loop; every rank makes the same calls in the
 * same order.  host_staged = 0: buffers are device pointers and each call is
 * enqueued on `stream` (a hipStream_t), as RCCL does; host_staged = 1: they
 * are host memory and the engine has synchronised its stream first (test
 * transports, e.g. torch.distributed gloo).
 *   allreduce_sum_u8: bytewise sum in place.  The engine only reduces arrays
 *     in which at most one rank holds a non-zero byte, so the sum is a gather
 *     of owned pieces, exact for every element type.
 *   broadcast: `bytes` from `send` on rank `root` into `recv` on every rank
 *     (root included); `send` is ignored elsewhere.
 *   allgather (may be NULL): `bytes` from `send` on every rank r land at
 *     recv + r * bytes on every rank (`send` may alias that slot).  NULL: the
 *     engine emulates it with allreduce_sum_u8 over a zeroed world x bytes
 *     buffer (twice the ring bytes). */
typedef struct {
	void *user;
	int rank, world;
	int host_staged;
	int (*allreduce_sum_u8)(void *user, void *buf, size_t bytes, void *stream);
	int (*broadcast)(void *user, const void *send, void *recv, size_t bytes, int root, void *stream);
	int (*allgather)(void *user, const void *send, void *recv, size_t bytes, void *stream);
} ccg_coll;

/* RCCL transport (librccl.so.1 is loaded on first use).  Rank 0 makes the
 * 128-byte id and the caller ships it to the other ranks (e.g. through the
 * torch.distributed TCP store); ccg_rccl_open blocks until all ranks joined. */
#define CCG_RCCL_ID_BYTES 128
int ccg_rccl_unique_id(void *id);
int ccg_rccl_open(ccg_ctx *ctx, const void *id, int rank, int world, ccg_coll *out);
int ccg_rccl_close(ccg_coll *coll);
/* ncclCommAbort: unblocks this rank's pending collectives after a peer failed
 * (the multi-GPU CLI calls it on every rank's communicator when one fails). */
int ccg_rccl_abort(ccg_coll *coll);

/* NJ (a->method = CCG_TREE_NJ, nj_thread nj.c:1612), DNJ (CCG_TREE_DNJ,
 * dnj_thread dnj.c:1054) or HNJ (CCG_TREE_HNJ, hclust.c:1671) on the rank's
 * rows.  Every rank returns the full
 * join list, identical on all ranks and bit-identical to ccg_tree with the
 * same method and `exact` flag for any world size.  Dloc_dev holds the
 * rank's ccg_shard_elems(n, rank, world) elements and is consumed.
 * CCG_EUNSUP for matrices with missing (negative) entries. */
int ccg_tree_shard_dev(ccg_ctx *ctx, const ccg_tree_args *a, const ccg_coll *coll, void *Dloc_dev,
                       ccg_join *joins, int *njoins, int *final_n, double *final_d, int64_t *stats);
/* Same from the full host LT (every rank passes the whole matrix; only the
 * rank's own rows are uploaded). */
int ccg_tree_shard(ccg_ctx *ctx, const ccg_tree_args *a, const ccg_coll *coll, const void *D,
                   ccg_join *joins, int *njoins, int *final_n, double *final_d, int64_t *stats);

/* Device bytes ccg_tree_shard_dev allocates beside the rank's shard for a run
 * of n taxa over `world` ranks (the replicated per-taxon vectors, the per-join
 * buffers, the initSummaD exchange), for planning a large run's memory
 * (configs[4]: n = 1e6, a 250 GB float shard per rank).  *gather_bytes (may
 * be NULL) bounds the extra buffer the exact initSummaD allocates, during the
 * init only, when some column sums need the serial gather (non-integral cells,
 * DESIGN.md 6; integer SNP counts need none). */
int ccg_tree_shard_bytes(int64_t n, int etype, int method, int world, int64_t *device_bytes, int64_t *gather_bytes);

/* dist straight into one rank's shard ("dist writes the
 * shards that DNJ consumes in place"): ccg_snp_ltd_dev semantics
 * (a->row_begin = a->row_end = 0), but only the rank's owned rows are
 * computed, stored as ccg_tree_shard_dev reads them (ccg_shard_row_offset);
 * Dloc_dev holds ccg_shard_elems(n, rank, world) elements.  seqs / incs are
 * device pointers holding every taxon.  Pair mode (a->pair, incs = one mask
 * per taxon, -P via a->proxi) stores D only (cmpairFsaThrd semantics). */
int ccg_snp_ltd_shard_dev(ccg_ctx *ctx, const ccg_snp_args *a, int rank, int world, void *Dloc_dev, int *inc_out);
/* Same with a->seqs / a->incs in HOST memory (Dloc_dev still a device
 * buffer): the packed rows stream through a 256 MB staging buffer into the
 * bit planes, so the rank's HBM holds the planes and its shard only (at
 * configs[4], n = 1e6 x 100 kbp: 25 GB + 250 GB, where a device copy of the
 * packed MSA would add 25 GB).  ccg_snp_ltd streams the same way. */
int ccg_snp_ltd_shard(ccg_ctx *ctx, const ccg_snp_args *a, int rank, int world, void *Dloc_dev, int *inc_out);

/* The text round trip of `ccphylo dist | ccphylo tree` applied in place to
 * `elems` cells of a device LT (etype 8 or 4): an integral cell is kept
 * (printphy's "%d", phy.c:115), any other becomes strtod("%.*f" of it) with
 * `precision` digits (phy.c:117, loadPhy's strtod phy.c:469), computed exactly
 * (round-half-even of d * 10^p, then one correctly rounded division).  Used by
 * the fused `dist -W ... --tree`, whose normalised distances the pipeline
 * would round.  CCG_EUNSUP for etype 2/1, or for a cell with more significant
 * digits than a double holds at that precision. */
int ccg_round_decimal_dev(ccg_ctx *ctx, void *D_dev, int64_t elems, int etype, int precision);

/* ------------------------------------------------------------------ */
/* device memory helpers (for callers that keep the pipeline in HBM)   */
/* ------------------------------------------------------------------ */
int ccg_malloc(ccg_ctx *ctx, void **ptr, size_t bytes);
int ccg_free(ccg_ctx *ctx, void *ptr);
int ccg_memcpy_h2d(ccg_ctx *ctx, void *dst, const void *src, size_t bytes);
int ccg_memcpy_d2h(ccg_ctx *ctx, void *dst, const void *src, size_t bytes);
int ccg_synchronize(ccg_ctx *ctx);

/* ------------------------------------------------------------------ */
/* self-test hook (tests/test_gpu_exact_sum.py)                        */
/* ------------------------------------------------------------------ */
/* The serial sum s = ((0 + c[0]) + c[1]) + ... of n doubles c[k] >= 0 as the
 * tree engine's exact mode computes the new row sum of j (nj.c:911 / :1002):
 * the parallel binade-segmented form, or the chain where it declines.
 * *parallel = 1 when the parallel form produced it. */
int ccg_selftest_row_sum(ccg_ctx *ctx, const double *c, int n, double *out, int *parallel);

#ifdef __cplusplus
}
#endif
#endif
