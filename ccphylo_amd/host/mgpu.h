/* mgpu.h -- multi-GPU drivers of the CLI (mgpu.c): one matrix sharded over
 * G ranks, one host thread per rank. */
#ifndef CCPHYLO_MGPU_H
#define CCPHYLO_MGPU_H
#include <stddef.h>
#include "ccphylo_amd.h"

#define CCQ_TRANSPORT_RCCL 0   /* RCCL over xGMI, one device per rank */
#define CCQ_TRANSPORT_HOST 1   /* host-memory collectives between the rank threads */

typedef struct {
	int gpus;        /* ranks */
	int device0;     /* rank g runs on device (device0 + g) mod the device count */
	int transport;   /* CCQ_TRANSPORT_* */
	int round_precision;   /* dist --tree: >= 0 rounds each shard cell as the Phylip text would
	                          (ccg_round_decimal_dev, -W with -x digits); < 0: none */
} ccq_mgpu;

/* ccg_tree_shard on every rank from the full host LT D (ta->n taxa); the
 * join list (identical on all ranks, checked) in joins[0..n-3].  0 or a
 * CCG_E* code with a message in err. */
int ccq_mgpu_tree(const ccq_mgpu *c, const void *D, const ccg_tree_args *ta, ccg_join *joins, int *nj, int *fn,
                  double *fd, char *err, size_t errlen);

/* the fused pipeline: ccg_snp_ltd_shard_dev of the packed MSA (sa: host
 * seqs / incs, non-pair) into each rank's bands, then ccg_tree_shard_dev on
 * them, all in HBM; *inc = the included positions. */
int ccq_mgpu_dist_tree(const ccq_mgpu *c, const ccg_snp_args *sa, const ccg_tree_args *ta, ccg_join *joins, int *nj,
                       int *fn, double *fd, int *inc, char *err, size_t errlen);

#endif
