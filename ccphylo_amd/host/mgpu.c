/*
 * mgpu.c -- the multi-GPU drivers of the CLI: one LT matrix sharded over G
 * ranks, one host thread per rank, each on its own device (rank g on device
 * (dev0 + g) mod the device count), for `ccphylo tree --gpus G` and the fused
 * `ccphylo dist --tree` (configs[3] / [4] of BASELINE.json).
 *
 * ref: tree.c:146 main_tree / tree.c:89-93 (the dnj_thread / nj_thread call
 * sites the sharded engine replaces), dist.c:473 main_dist.
 *
 * Transports (ccg_coll, include/ccphylo_amd.h):
 *   rccl:  RCCL over xGMI; the main thread makes the unique id and every
 *          rank thread joins it with ccg_rccl_open (ncclCommInitRank), one
 *          communicator per device;
 *   host:  the ranks are threads of this process and the collectives go
 *          through host memory (host_staged = 1): a barrier, then each rank
 *          sums / copies its own slice of the byte range.  For G ranks on
 *          fewer devices (tests on a one-GPU box) and as a reference for the
 *          RCCL path.
 * Every rank returns the whole join list; the drivers check that all ranks
 * agree (the replicated state is computed identically by construction).
 */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>
#include "ccphylo_amd.h"
#include "ccphylo_host.h"
#include "mgpu.h"

/* ------------------------------------------------------------------ host transport */
/* An abortable barrier: a rank that fails (setup, an engine error, a
 * collective it cannot serve) calls tg_abort, and every rank waiting in the
 * group -- or arriving later -- leaves its collective with an error instead
 * of waiting for a peer that will never come. */
typedef struct {
	int world;
	pthread_mutex_t mu;
	pthread_cond_t cv;
	int count, aborted, fail;
	unsigned gen;
	void **bufs;          /* each rank's buffer of the current call */
	const void *root_buf;
	unsigned char *acc;   /* the allreduce result */
	size_t acap;
	int acc_fail;         /* rank 0 could not grow acc: every rank fails the call */
	int first_fail;       /* the rank that aborted the group first (its error is the one reported) */
	ccg_coll **rccl;      /* each rank's open RCCL communicator (NULL once closed or aborted) */
} tgroup;

typedef struct {
	tgroup *g;
	int rank;
} tuser;

/* 0, or -1 when the group was aborted before every rank arrived */
static int tg_wait(tgroup *g) {
	pthread_mutex_lock(&g->mu);
	if(g->aborted) {
		pthread_mutex_unlock(&g->mu);
		return -1;
	}
	const unsigned gen = g->gen;
	if(++g->count == g->world) {
		g->count = 0;
		++g->gen;
		pthread_cond_broadcast(&g->cv);
		pthread_mutex_unlock(&g->mu);
		return 0;
	}
	while(gen == g->gen && !g->aborted) pthread_cond_wait(&g->cv, &g->mu);
	const int rc = gen == g->gen ? -1 : 0;
	pthread_mutex_unlock(&g->mu);
	return rc;
}

static void tg_abort(tgroup *g, int rank) {
	pthread_mutex_lock(&g->mu);
	if(!g->aborted) g->first_fail = rank;
	g->aborted = 1;
	pthread_cond_broadcast(&g->cv);
	/* RCCL: the peers wait inside their collectives on the device; aborting
	 * every open communicator makes those calls return */
	for(int r = 0; g->rccl && r < g->world; ++r) {
		if(g->rccl[r]) {
			ccg_rccl_abort(g->rccl[r]);
			g->rccl[r] = NULL;
		}
	}
	pthread_mutex_unlock(&g->mu);
}

/* RCCL communicator registry (tg_abort's targets) */
static void tg_rccl_set(tgroup *g, int rank, ccg_coll *c) {
	pthread_mutex_lock(&g->mu);
	g->rccl[rank] = c;
	pthread_mutex_unlock(&g->mu);
}

/* the rank leaves the registry before closing its communicator itself
 * (ccg_rccl_close destroys it, or frees what an abort left of it) */
static void tg_rccl_take(tgroup *g, int rank) {
	pthread_mutex_lock(&g->mu);
	g->rccl[rank] = NULL;
	pthread_mutex_unlock(&g->mu);
}

/* every rank states whether its setup succeeded; 1 when all did (the same
 * answer on every rank), 0 otherwise */
static int tg_agree(tgroup *g, int rank, int ok) {
	pthread_mutex_lock(&g->mu);
	if(!ok && !g->fail) {
		g->fail = 1;
		g->first_fail = rank;
	}
	pthread_mutex_unlock(&g->mu);
	if(tg_wait(g)) return 0;
	pthread_mutex_lock(&g->mu);
	const int all = !g->fail;
	pthread_mutex_unlock(&g->mu);
	/* nobody may change fail again before every rank has read it */
	if(tg_wait(g)) return 0;
	return all;
}

static int tg_allreduce(void *user, void *buf, size_t bytes, void *stream) {
	(void) stream;
	tuser *u = user;
	tgroup *g = u->g;
	g->bufs[u->rank] = buf;
	if(u->rank == 0) {
		g->acc_fail = 0;
		if(g->acap < bytes) {
			free(g->acc);
			g->acc = malloc(bytes ? bytes : 1);
			g->acap = g->acc ? bytes : 0;
			g->acc_fail = !g->acc;
		}
	}
	if(tg_wait(g)) return -1;
	if(g->acc_fail) return -1;   /* the same on every rank: they all leave here */
	/* rank r sums slice r of every rank's buffer (one non-zero contributor
	 * per byte: 64-bit adds never carry between bytes) */
	const size_t words = bytes / 8, per = (words + g->world - 1) / g->world;
	const size_t w0 = (size_t) u->rank * per, w1 = w0 + per < words ? w0 + per : words;
	for(size_t w = w0; w < w1; ++w) {
		uint64_t s = 0;
		for(int q = 0; q < g->world; ++q) {
			uint64_t x;
			memcpy(&x, (const unsigned char *) g->bufs[q] + 8 * w, 8);
			s += x;
		}
		memcpy(g->acc + 8 * w, &s, 8);
	}
	if(u->rank == 0) {
		for(size_t b = 8 * words; b < bytes; ++b) {
			unsigned char s = 0;
			for(int q = 0; q < g->world; ++q) s += ((const unsigned char *) g->bufs[q])[b];
			g->acc[b] = s;
		}
	}
	if(tg_wait(g)) return -1;
	memcpy(buf, g->acc, bytes);
	return tg_wait(g);   /* acc is reused by the next call */
}

static int tg_allgather(void *user, const void *send, void *recv, size_t bytes, void *stream) {
	(void) stream;
	tuser *u = user;
	tgroup *g = u->g;
	g->bufs[u->rank] = (void *) send;
	if(tg_wait(g)) return -1;
	/* every rank copies the others' slots (its own may alias recv's) */
	for(int q = 0; q < g->world; ++q) {
		unsigned char *dst = (unsigned char *) recv + (size_t) q * bytes;
		if(dst != g->bufs[q]) memcpy(dst, g->bufs[q], bytes);
	}
	return tg_wait(g);
}

static int tg_bcast(void *user, const void *send, void *recv, size_t bytes, int root, void *stream) {
	(void) stream;
	tuser *u = user;
	tgroup *g = u->g;
	if(u->rank == root) g->root_buf = send;
	if(tg_wait(g)) return -1;
	if(u->rank != root || recv != send) memcpy(recv, g->root_buf, bytes);
	return tg_wait(g);
}

/* ------------------------------------------------------------------ rank threads */
typedef struct {
	/* shared */
	const ccq_mgpu *cfg;
	tgroup *tg;
	unsigned char id[CCG_RCCL_ID_BYTES];
	int ndev;
	/* the work: tree of a host LT, or dist of an MSA then tree */
	const void *D;
	const ccg_tree_args *ta;
	const ccg_snp_args *sa;
	/* per rank */
	int rank, rc, inc;
	ccg_join *joins;
	int nj, fn;
	double fd;
	int64_t st[4];
	char err[256];
} rank_job;

static void set_err(rank_job *j, const char *what, int rc) {
	snprintf(j->err, sizeof(j->err), "rank %d: %s: %s", j->rank, what, ccg_strerror(rc));
	j->rc = rc ? rc : CCG_EHIP;
}

static void *rank_main(void *p) {
	rank_job *j = p;
	const ccq_mgpu *c = j->cfg;
	ccg_ctx *ctx = NULL;
	ccg_coll coll;
	int have_coll = 0;
	void *dloc = NULL;
	tuser tu = {j->tg, j->rank};
	/* local setup first (device, shard buffer); the ranks agree on it before
	 * any of them enters a collective, so one rank's failure ends them all */
	int rc = ccg_init((c->device0 + j->rank) % j->ndev, &ctx);
	if(rc) set_err(j, "ccg_init", rc);
	/* test hook: CCQ_MGPU_FAIL=setup:<rank> or run:<rank> makes that rank fail
	 * its setup, or leave instead of running the tree (its peers are then in
	 * their collectives), so the tests can check that the CLI exits */
	const char *inj = getenv("CCQ_MGPU_FAIL");
	const int inj_setup = inj && !strncmp(inj, "setup:", 6) && atoi(inj + 6) == j->rank;
	const int inj_run = inj && !strncmp(inj, "run:", 4) && atoi(inj + 4) == j->rank;
	if(!rc && inj_setup) {
		rc = CCG_EHIP;
		snprintf(j->err, sizeof(j->err), "rank %d: injected setup failure (CCQ_MGPU_FAIL)", j->rank);
		j->rc = rc;
	}
	if(!rc && j->sa) {
		const int64_t elems = ccg_shard_elems(j->sa->n, j->rank, c->gpus);
		if((rc = ccg_malloc(ctx, &dloc, (size_t) (elems > 0 ? elems : 1) * j->ta->etype))) set_err(j, "shard buffer", rc);
	}
	if(!tg_agree(j->tg, j->rank, !rc)) {
		if(!rc) snprintf(j->err, sizeof(j->err), "rank %d: stopped: another rank failed its setup", j->rank);
		if(!j->rc) j->rc = CCG_EHIP;
		goto out;
	}
	if(c->transport == CCQ_TRANSPORT_RCCL) {
		/* a rank whose ncclCommInitRank fails leaves the others waiting in
		 * theirs (RCCL has no cancellable init here); every earlier failure is
		 * caught by the agreement above */
		if((rc = ccg_rccl_open(ctx, j->id, j->rank, c->gpus, &coll))) set_err(j, "ccg_rccl_open", rc);
		else {
			have_coll = 1;
			tg_rccl_set(j->tg, j->rank, &coll);
		}
		if(!tg_agree(j->tg, j->rank, !rc)) {
			if(!j->rc) j->rc = CCG_EHIP;
			goto out;
		}
	} else {
		memset(&coll, 0, sizeof(coll));
		coll.user = &tu;
		coll.rank = j->rank;
		coll.world = c->gpus;
		coll.host_staged = 1;
		coll.allreduce_sum_u8 = tg_allreduce;
		coll.broadcast = tg_bcast;
		coll.allgather = tg_allgather;
	}
	if(inj_run) {
		rc = CCG_EHIP;
		snprintf(j->err, sizeof(j->err), "rank %d: injected failure before the tree (CCQ_MGPU_FAIL)", j->rank);
		j->rc = rc;
	} else if(!j->sa) {
		/* tree of a host LT: the rank uploads its own row bands */
		rc = ccg_tree_shard(ctx, j->ta, &coll, j->D, j->joins, &j->nj, &j->fn, &j->fd, j->st);
		if(rc) set_err(j, "ccg_tree_shard", rc);
	} else if((rc = ccg_snp_ltd_shard(ctx, j->sa, j->rank, c->gpus, dloc, &j->inc))) {
		/* dist into the rank's bands (the packed MSA streams from host memory
		 * into the bit planes: HBM holds the planes and the shard only), then
		 * the tree on them, all in HBM */
		set_err(j, "ccg_snp_ltd_shard", rc);
	} else if(c->round_precision >= 0 &&
	          (rc = ccg_round_decimal_dev(ctx, dloc, ccg_shard_elems(j->sa->n, j->rank, c->gpus), j->ta->etype,
	                                      c->round_precision))) {
		set_err(j, "ccg_round_decimal_dev", rc);
	} else {
		rc = ccg_tree_shard_dev(ctx, j->ta, &coll, dloc, j->joins, &j->nj, &j->fn, &j->fd, j->st);
		if(rc) set_err(j, "ccg_tree_shard_dev", rc);
	}
	/* the others leave their next (or current) collective */
	if(rc) tg_abort(j->tg, j->rank);
out:
	if(have_coll) {
		tg_rccl_take(j->tg, j->rank);   /* no tg_abort reaches it after this */
		ccg_rccl_close(&coll);
	}
	if(dloc) ccg_free(ctx, dloc);
	if(ctx) ccg_destroy(ctx);
	return NULL;
}

static int run_ranks(const ccq_mgpu *c, const void *D, const ccg_tree_args *ta, const ccg_snp_args *sa, int n,
                     ccg_join *joins, int *nj, int *fn, double *fd, int *inc, char *err, size_t errlen) {
	const int G = c->gpus;
	int ndev = 0, rc = ccg_device_count(&ndev);
	if(rc) {
		snprintf(err, errlen, "no HIP device: %s", ccg_strerror(rc));
		return rc;
	}
	if(c->transport == CCQ_TRANSPORT_RCCL && G > ndev) {
		snprintf(err, errlen, "--gpus %d with RCCL needs %d devices (%d visible); --transport host runs several ranks "
		         "per device", G, G, ndev);
		return CCG_EINVAL;
	}
	tgroup tg;
	memset(&tg, 0, sizeof(tg));
	tg.world = G;
	tg.bufs = calloc((size_t) G, sizeof(void *));
	tg.rccl = calloc((size_t) G, sizeof(ccg_coll *));
	pthread_mutex_init(&tg.mu, NULL);
	pthread_cond_init(&tg.cv, NULL);
	rank_job *jobs = calloc((size_t) G, sizeof(rank_job));
	pthread_t *th = calloc((size_t) G, sizeof(pthread_t));
	unsigned char id[CCG_RCCL_ID_BYTES];
	/* RCCL prints its banner / debug lines on stdout, where the CLI writes
	 * the Newick: stdout points at stderr while the ranks run */
	int saved_out = -1;
	if(c->transport == CCQ_TRANSPORT_RCCL) {
		fflush(stdout);
		saved_out = dup(1);
		if(saved_out >= 0) dup2(2, 1);
	}
	if(c->transport == CCQ_TRANSPORT_RCCL && (rc = ccg_rccl_unique_id(id))) {
		snprintf(err, errlen, "ccg_rccl_unique_id: %s", ccg_strerror(rc));
		goto out;
	}
	for(int g = 0; g < G; ++g) {
		rank_job *j = jobs + g;
		j->cfg = c;
		j->tg = &tg;
		memcpy(j->id, id, sizeof(id));
		j->ndev = ndev;
		j->D = D;
		j->ta = ta;
		j->sa = sa;
		j->rank = g;
		j->joins = g == 0 ? joins : malloc((size_t) (n > 2 ? n : 2) * sizeof(ccg_join));
		if(!j->joins || pthread_create(th + g, NULL, rank_main, j)) {
			snprintf(err, errlen, "cannot start rank %d", g);
			rc = CCG_ENOMEM;
			tg_abort(&tg, g);   /* the started ranks leave their setup agreement */
			for(int q = 0; q < g; ++q) pthread_join(th[q], NULL);
			goto out;
		}
	}
	for(int g = 0; g < G; ++g) pthread_join(th[g], NULL);
	rc = CCG_OK;
	/* the error of the rank that failed first (the others only stopped) */
	if(tg.aborted || tg.fail) {
		rc = jobs[tg.first_fail].rc ? jobs[tg.first_fail].rc : CCG_EHIP;
		snprintf(err, errlen, "%s", jobs[tg.first_fail].err);
	}
	for(int g = 0; g < G && !rc; ++g) {
		if(jobs[g].rc) {
			rc = jobs[g].rc;
			snprintf(err, errlen, "%s", jobs[g].err);
		}
	}
	for(int g = 1; g < G && !rc; ++g) {   /* every rank holds the same replicated state */
		if(jobs[g].nj != jobs[0].nj || jobs[g].fn != jobs[0].fn ||
		   memcmp(jobs[g].joins, joins, (size_t) jobs[0].nj * sizeof(ccg_join))) {
			snprintf(err, errlen, "rank %d's join list differs from rank 0's", g);
			rc = CCG_EHIP;
		}
	}
	if(!rc) {
		*nj = jobs[0].nj;
		*fn = jobs[0].fn;
		*fd = jobs[0].fd;
		if(inc) *inc = jobs[0].inc;
	}
out:
	if(saved_out >= 0) {
		fflush(stdout);
		dup2(saved_out, 1);
		close(saved_out);
	}
	for(int g = 1; g < G; ++g) free(jobs[g].joins);
	free(jobs);
	free(th);
	pthread_mutex_destroy(&tg.mu);
	pthread_cond_destroy(&tg.cv);
	free(tg.bufs);
	free(tg.rccl);
	free(tg.acc);
	return rc;
}

int ccq_mgpu_tree(const ccq_mgpu *c, const void *D, const ccg_tree_args *ta, ccg_join *joins, int *nj, int *fn,
                  double *fd, char *err, size_t errlen) {
	return run_ranks(c, D, ta, NULL, ta->n, joins, nj, fn, fd, NULL, err, errlen);
}

int ccq_mgpu_dist_tree(const ccq_mgpu *c, const ccg_snp_args *sa, const ccg_tree_args *ta, ccg_join *joins, int *nj,
                       int *fn, double *fd, int *inc, char *err, size_t errlen) {
	return run_ranks(c, NULL, ta, sa, ta->n, joins, nj, fn, fd, inc, err, errlen);
}
