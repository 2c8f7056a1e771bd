/*
 * main.c -- `ccphylo dist` and `ccphylo tree`, the stable CLI surface, with
 * the hot path on the GPU engine (include/ccphylo_amd.h).
 *
 * Mirrors ref main.c:99 (dispatch), dist.c:473 main_dist / :42 makeMatrix /
 * cdist.c:196 ltdMsaMatrix_get, and tree.c:146 main_tree / :37 formTree:
 * same options, same stdout bytes, same stderr progress lines.  Option forms
 * the GPU engine does not implement (-V, -y, -a, union inputs, the z / p /
 * np count-matrix metrics, tree methods other than nj / dnj / hnj) are
 * refused with an error instead of being silently approximated.
 *
 * Extra (not in the reference): `tree --fast_sums` uses a fixed-order
 * parallel row sum instead of the reference's serial one;
 * `--device N` selects the GPU; `tree --gpus G [--transport rccl|host]`
 * shards the matrix over G ranks (host/mgpu.c); `dist --tree FILE` runs
 * dist and the tree in HBM without the Phylip text (`-m`, `--gpus`,
 * `--transport`, `--fast_sums` as for tree).
 */
#include <ctype.h>
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include "ccphylo_amd.h"
#include "ccphylo_host.h"
#include "mgpu.h"

static void die_opt(const char *kind, const char *opt) {
	fprintf(stderr, "%s argument:\t\"%s\"\n", kind, opt);
	exit(1);
}

static int is_num(const char *s) {
	char *e;
	if(!s || !*s) return 0;
	strtod(s, &e);
	return *e == 0;
}

typedef struct {
	int argc, k;
	char **argv;
} Args;

/* value of an option: attached ("-x5", "--opt=5") or the next argv word */
static char *opt_value(Args *A, const char *attached, const char *opt) {
	if(attached && *attached) return (char *) attached;
	if(A->k + 1 < A->argc) return A->argv[++A->k];
	die_opt("Missing", opt);
	return NULL;
}

/* optional numeric value (cmdline.c getdDefArg): only if it does not start with '-' */
static double opt_dvalue_def(Args *A, const char *attached, double def, const char *opt) {
	const char *v = NULL;
	if(attached && *attached) {
		v = attached;
	} else if(A->k + 1 < A->argc && A->argv[A->k + 1][0] != '-') {
		v = A->argv[++A->k];
	}
	if(!v) return def;
	if(!is_num(v)) die_opt("Invalid", opt);
	return strtod(v, NULL);
}

static long opt_num(Args *A, const char *attached, const char *opt) {
	char *v = opt_value(A, attached, opt), *e;
	long x = strtol(v, &e, 10);
	if(*e) die_opt("Invalid", opt);
	return x;
}

static ccg_ctx *open_gpu(int device) {
	ccg_ctx *ctx = NULL;
	int rc = ccg_init(device, &ctx);
	if(rc) {
		fprintf(stderr, "ccphylo_amd: cannot open GPU %d: %s\n", device, ccg_strerror(rc));
		exit(1);
	}
	return ctx;
}

/* ================================================================ tree */
static int tree_help(FILE *out) {
	fprintf(out, "#CCPhylo forms tree(s) in newick format given a set of phylip distance matrices.\n");
	fprintf(out, "#   %-24s\t%-32s\t%s\n", "Options are:", "Desc:", "Default:");
	fprintf(out, "#    -%c, --%-16s\t%-32s\t%s\n", 'i', "input", "Input file", "stdin");
	fprintf(out, "#    -%c, --%-16s\t%-32s\t%s\n", 'o', "output", "Output file", "stdout");
	fprintf(out, "#    -%c, --%-16s\t%-32s\t%s\n", 'S', "separator", "Separator", "\\t");
	fprintf(out, "#    -%c, --%-16s\t%-32s\t%s\n", 'q', "quotes", "Quote taxa", "\\0");
	fprintf(out, "#    -%c, --%-16s\t%-32s\t%s\n", 'x', "print_precision", "Floating point print precision", "9");
	fprintf(out, "#    -%c, --%-16s\t%-32s\t%s\n", 'm', "method", "Tree construction method.", "dnj");
	fprintf(out, "#    -%c, --%-16s\t%-32s\t%s\n", 'M', "method_help", "Help on option \"-m\"", "");
	fprintf(out, "#    -%c, --%-16s\t%-32s\t%s\n", 'f', "flag", "Output flags", "0");
	fprintf(out, "#    -%c, --%-16s\t%-32s\t%s\n", 'F', "flag_help", "Help on option \"-f\"", "");
	fprintf(out, "#    -%c, --%-16s\t%-32s\t%s\n", 'p', "float_precision", "Float precision on distance matrix", "False / double");
	fprintf(out, "#    -%c, --%-16s\t%-32s\t%s\n", 's', "short_precision", "Short precision on distance matrix", "False / double / 1e0");
	fprintf(out, "#    -%c, --%-16s\t%-32s\t%s\n", 'b', "byte_precision", "Byte precision on distance matrix", "False / double / 1e0");
	fprintf(out, "#    -%c, --%-16s\t%-32s\t%s\n", 'g', "free", "Gradually free up D", "False");
	fprintf(out, "#    -%c, --%-16s\t%-32s\t%s\n", 'H', "mmap", "Allocate matrix on the disk", "False");
	fprintf(out, "#    -%c, --%-16s\t%-32s\t%s\n", 'T', "tmp", "Set directory for temporary files", "");
	fprintf(out, "#    -%c, --%-16s\t%-32s\t%s\n", 't', "threads", "Number of threads", "1");
	fprintf(out, "#    -%c, --%-16s\t%-32s\t%s\n", 'h', "help", "Shows this helpmessage", "");
	fprintf(out, "#        --%-16s\t%-32s\t%s\n", "gpus", "Shard the matrix over G GPUs (nj, dnj)", "off");
	fprintf(out, "#        --%-16s\t%-32s\t%s\n", "transport", "rccl / host collectives for --gpus", "rccl");
	fprintf(out, "#        --%-16s\t%-32s\t%s\n", "fast_sums", "Parallel row sums (not the reference's)", "False");
	fprintf(out, "#        --%-16s\t%-32s\t%s\n", "device", "First GPU", "0");
	return out == stderr;
}

/* --transport value */
static int transport_id(const char *v) {
	if(!strcmp(v, "rccl")) return CCQ_TRANSPORT_RCCL;
	if(!strcmp(v, "host")) return CCQ_TRANSPORT_HOST;
	die_opt("Invalid", "\"--transport\"");
	return -1;
}

static int main_tree(int argc, char **argv) {
	const char *in = "-", *outname = "-", *method = "dnj";
	int flag = 0, precision = 9, et = 8, fast = 0, device = 0, stats = 0, gpus = 0, transport = CCQ_TRANSPORT_RCCL;
	char sep = '\t', quotes = 0;
	double bs = 1.0;
	Args A = {argc, 0, argv};
	for(A.k = 1; A.k < argc; ++A.k) {
		char *a = argv[A.k];
		if(a[0] != '-' || a[1] == 0) {
			in = a;
			if(A.k + 1 < argc) {
				fprintf(stderr, "Unexpected non-option argument(s).\n");
				return 1;
			}
			break;
		}
		if(a[1] == '-') {
			char *name = a + 2, *eq = strchr(name, '=');
			char *att = NULL;
			if(eq) {
				*eq = 0;
				att = eq + 1;
			}
			if(*name == 0) { continue; }
			else if(!strcmp(name, "input")) in = opt_value(&A, att, "input");
			else if(!strcmp(name, "output")) outname = opt_value(&A, att, "output");
			else if(!strcmp(name, "separator")) sep = opt_value(&A, att, "separator")[0];
			else if(!strcmp(name, "quotes")) quotes = opt_value(&A, att, "quotes")[0];
			else if(!strcmp(name, "print_precision")) precision = (int) opt_num(&A, att, "print_precision");
			else if(!strcmp(name, "method")) method = opt_value(&A, att, "method");
			else if(!strcmp(name, "method_help")) method = "mh";
			else if(!strcmp(name, "flag")) flag = (int) opt_num(&A, att, "flag");
			else if(!strcmp(name, "flag_help")) flag = -1;
			else if(!strcmp(name, "threads")) (void) opt_num(&A, att, "threads");
			else if(!strcmp(name, "float_precision")) et = 4;
			else if(!strcmp(name, "short_precision")) { et = 2; bs = opt_dvalue_def(&A, att, bs, "short_precision"); }
			else if(!strcmp(name, "byte_precision")) { et = 1; bs = opt_dvalue_def(&A, att, bs, "byte_precision"); }
			else if(!strcmp(name, "free") || !strcmp(name, "mmap")) { /* host memory knobs: no effect on HBM */ }
			else if(!strcmp(name, "tmp")) (void) opt_value(&A, att, "tmp");
			else if(!strcmp(name, "fast_sums")) fast = 1;
			else if(!strcmp(name, "device")) device = (int) opt_num(&A, att, "device");
			else if(!strcmp(name, "gpus")) gpus = (int) opt_num(&A, att, "gpus");
			else if(!strcmp(name, "transport")) transport = transport_id(opt_value(&A, att, "transport"));
			else if(!strcmp(name, "stats")) stats = 1;
			else if(!strcmp(name, "help")) return tree_help(stdout);
			else die_opt("Unknown", a);
			continue;
		}
		for(char *p = a + 1; *p; ++p) {
			char o = *p, *att = p + 1;
			int took = 1;
			switch(o) {
				case 'i': in = opt_value(&A, att, "i"); break;
				case 'o': outname = opt_value(&A, att, "o"); break;
				case 'S': sep = opt_value(&A, att, "S")[0]; break;
				case 'q': quotes = opt_value(&A, att, "q")[0]; break;
				case 'x': precision = (int) opt_num(&A, att, "x"); break;
				case 'm': method = opt_value(&A, att, "m"); break;
				case 'f': flag = (int) opt_num(&A, att, "f"); break;
				case 't': (void) opt_num(&A, att, "t"); break;
				case 'T': (void) opt_value(&A, att, "T"); break;
				case 's': et = 2; bs = opt_dvalue_def(&A, att, bs, "s"); break;
				case 'b': et = 1; bs = opt_dvalue_def(&A, att, bs, "b"); break;
				case 'M': method = "mh"; took = 0; break;
				case 'F': flag = -1; took = 0; break;
				case 'p': et = 4; took = 0; break;
				case 'g': case 'H': took = 0; break;
				case 'h': return tree_help(stdout);
				default: {
					char bad[3] = {'-', o, 0};
					die_opt("Unknown", bad);
				}
			}
			if(took) break;
		}
	}
	if(flag == -1) {
		fprintf(stdout, "# Format flags output, add them to combine them.\n");
		fprintf(stdout, "#\n");
		fprintf(stdout, "#   1:\tStrictly bifurcate the root\n");
		fprintf(stdout, "#   2:\tAllow negative branchlengths\n");
		fprintf(stdout, "#\n");
		return 0;
	}
	int m;
	if(!strcmp(method, "dnj")) {
		m = CCG_TREE_DNJ;
	} else if(!strcmp(method, "nj")) {
		m = CCG_TREE_NJ;
	} else if(!strcmp(method, "hnj")) {
		m = CCG_TREE_HNJ;
	} else if(!strcmp(method, "mh")) {
		fprintf(stdout, "# Tree construction methods:\n#\n");
		fprintf(stdout, "# %-8s\t%s\n", "nj", "Neighbor-Joining");
		fprintf(stdout, "# %-8s\t%s\n", "hnj", "Heuristic Neighbor-Joining");
		fprintf(stdout, "# %-8s\t%s\n", "dnj", "Dynamic Neighbor-Joining");
		fprintf(stdout, "#\n");
		return 0;
	} else if(!strcmp(method, "upgma") || !strcmp(method, "cf") || !strcmp(method, "ff") || !strcmp(method, "mn") ||
	          !strcmp(method, "frank")) {
		fprintf(stderr, "ccphylo_amd: tree method \"%s\" is not implemented by the GPU engine (nj, dnj, hnj are).\n", method);
		return 1;
	} else {
		die_opt("Invalid", "\"-m\"");
		return 1;
	}
	if((et == 2 || et == 1) && bs == 0) die_opt("Invalid", et == 2 ? "\"--short_precision\"" : "\"--byte_precision\"");
	if(gpus < 0) die_opt("Invalid", "\"--gpus\"");

	FILE *out = (outname[0] == '-' && outname[1] == 0) ? stdout : fopen(outname, "wb");
	if(!out) {
		fprintf(stderr, "Error: %d (%s)\n", errno, strerror(errno));
		return errno ? errno : 1;
	}
	ccq_reader *r = ccq_open(in);
	if(!r) {
		fprintf(stderr, "Error: %d (%s)\n", errno, strerror(errno));
		return errno ? errno : 1;
	}
	ccg_ctx *ctx = NULL;
	ccq_ltd *D = ccq_ltd_new(32, et, bs);        /* tree.c:52 */
	ccq_names *T = ccq_names_new(32, 4);         /* tree.c:61-66 */
	int err = 0, n;
	ccg_join *joins = NULL;
	size_t jcap = 0;
	clock_t t0 = clock(), t1;
	while((n = ccq_load_phy(r, D, T, sep, quotes, &err)) > 0) {
		t1 = clock();
		fprintf(stderr, "# Total time used loading matrix: %.2f s.\n", (double) (t1 - t0) / 1000000);
		t0 = t1;
		if(n > 2) {
			if(jcap < (size_t) n) {
				jcap = n;
				joins = realloc(joins, jcap * sizeof(ccg_join));
			}
			ccg_tree_args ta = {n, et, bs, m, flag, !fast, 0, 0};
			int nj = 0, fn = 0;
			double fd = 0;
			int64_t st[12 + 2 * CCG_NKSTAT];
			memset(st, 0, sizeof(st));
			int rc;
			if(gpus) {
				/* one matrix over G ranks, one thread per rank (host/mgpu.c) */
				ccq_mgpu mc = {gpus, device, transport, -1};
				char emsg[320] = "";
				rc = ccq_mgpu_tree(&mc, D->mat, &ta, joins, &nj, &fn, &fd, emsg, sizeof(emsg));
				if(rc) {
					fprintf(stderr, "ccphylo_amd: sharded tree construction failed: %s\n", emsg);
					return 1;
				}
			} else {
				if(!ctx) ctx = open_gpu(device);
				rc = ccg_tree(ctx, &ta, D->mat, joins, &nj, &fn, &fd, st);
			}
			if(rc) {
				fprintf(stderr, "ccphylo_amd: tree construction failed: %s\n", ccg_strerror(rc));
				return 1;
			}
			if(stats && !gpus) {
				fprintf(stderr, "# gpu: %d joins, %lld rows / %lld cells rescanned, %lld launches, %.3f ms\n", nj,
				        (long long) st[0], (long long) st[1], (long long) st[2], st[3] / 1000.0);
			}
			ccq_replay_newick(T, n, (const ccq_join *) joins, nj, fn, fd, flag, precision);
		} else if(n == 2) {
			ccq_newick_pair(T, ccq_ltd_get(D, 0), precision);
		}
		if(T->header->len) {
			fprintf(out, ">%s%s;\n", (char *) T->header->seq, (char *) T->names[0]->seq);
		} else {
			fprintf(out, "%s;\n", (char *) T->names[0]->seq);
		}
		t1 = clock();
		fprintf(stderr, "# Total time used Constructing tree: %.2f s.\n", (double) (t1 - t0) / 1000000);
		t0 = t1;
	}
	if(out != stdout) fclose(out);
	else fflush(stdout);
	ccq_close(r);
	ccq_ltd_free(D);
	ccq_names_free(T);
	free(joins);
	if(ctx) ccg_destroy(ctx);
	return err ? 1 : 0;
}

/* ================================================================ dist */
static int dist_help(FILE *out) {
	fprintf(out, "#CCPhylo dist calculates distances between samples based on overlaps between nucleotide count matrices created by e.g. KMA.\n");
	fprintf(out, "#   %-24s\t%-32s\t%s\n", "Options are:", "Desc:", "Default:");
	fprintf(out, "#    -%c, --%-16s\t%-32s\t%s\n", 'i', "input", "Input file(s)", "stdin");
	fprintf(out, "#    -%c, --%-16s\t%-32s\t%s\n", 'o', "output", "Output file", "stdout");
	fprintf(out, "#    -%c, --%-16s\t%-32s\t%s\n", 'n', "nucleotide_numbers", "Output number of nucleotides included", "False/None");
	fprintf(out, "#    -%c, --%-16s\t%-32s\t%s\n", 'x', "print_precision", "Floating point print precision", "9");
	fprintf(out, "#    -%c, --%-16s\t%-32s\t%s\n", 'L', "min_len", "Minimum overlapping length", "1");
	fprintf(out, "#    -%c, --%-16s\t%-32s\t%s\n", 'C', "min_cov", "Minimum coverage", "50.0%");
	fprintf(out, "#    -%c, --%-16s\t%-32s\t%s\n", 'W', "normalization_weight", "Normalization weight", "0 / None");
	fprintf(out, "#    -%c, --%-16s\t%-32s\t%s\n", 'P', "proximity", "Minimum proximity between SNPs", "0");
	fprintf(out, "#    -%c, --%-16s\t%-32s\t%s\n", 'f', "flag", "Output flags", "1");
	fprintf(out, "#    -%c, --%-16s\t%-32s\t%s\n", 'F', "flag_help", "Help on option \"-f\"", "");
	fprintf(out, "#    -%c, --%-16s\t%-32s\t%s\n", 'p', "float_precision", "Float precision on distance matrix", "double");
	fprintf(out, "#    -%c, --%-16s\t%-32s\t%s\n", 's', "short_precision", "Short precision on distance matrix", "double / 1e0");
	fprintf(out, "#    -%c, --%-16s\t%-32s\t%s\n", 'b', "byte_precision", "Byte precision on distance matrix", "double / 1e0");
	fprintf(out, "#    -%c, --%-16s\t%-32s\t%s\n", 't', "threads", "Number of threads", "1");
	fprintf(out, "#    -%c, --%-16s\t%-32s\t%s\n", 'h', "help", "Shows this helpmessage", "");
	fprintf(out, "#        --%-16s\t%-32s\t%s\n", "tree", "Also build the tree in HBM, Newick to FILE", "off");
	fprintf(out, "#        --%-16s\t%-32s\t%s\n", "tree_method", "nj / dnj / hnj for --tree", "dnj");
	fprintf(out, "#        --%-16s\t%-32s\t%s\n", "tree_flag", "tree -f flags for --tree", "0");
	fprintf(out, "#        --%-16s\t%-32s\t%s\n", "gpus", "Shard --tree over G GPUs", "1");
	fprintf(out, "#        --%-16s\t%-32s\t%s\n", "transport", "rccl / host collectives for --gpus", "rccl");
	return out == stderr;
}

/* dist.c:736-790: -d name -> metric; z, p, np -> -1 (not on the GPU engine) */
static int kma_metric_id(const char *m, int *id, unsigned *lnorm) {
	static const struct {
		const char *name;
		int id;
	} tab[] = {{"cos", CCG_KMA_COS}, {"z", -1}, {"chi2", CCG_KMA_CHI2}, {"nchi2", CCG_KMA_NCHI2},
	           {"nc", CCG_KMA_NC}, {"c", CCG_KMA_C}, {"np", -1}, {"p", -1}, {"nbc", CCG_KMA_NBC},
	           {"bc", CCG_KMA_BC}, {"nl1", CCG_KMA_NL1}, {"nl2", CCG_KMA_NL2}, {"nlinf", CCG_KMA_NLINF},
	           {"l1", CCG_KMA_L1}, {"l2", CCG_KMA_L2}, {"linf", CCG_KMA_LINF}};
	for(size_t k = 0; k < sizeof(tab) / sizeof(tab[0]); ++k) {
		if(!strcmp(m, tab[k].name)) {
			*id = tab[k].id;
			return 0;
		}
	}
	char *e;
	if(m[0] == 'l') {
		*lnorm = (unsigned) strtoul(m + 1, &e, 10);
		*id = CCG_KMA_LN;
		return *e != 0;
	}
	if(!strncmp(m, "nl", 2)) {
		*lnorm = (unsigned) strtoul(m + 2, &e, 10);
		*id = CCG_KMA_NLN;
		return *e != 0;
	}
	return 1;
}

/* filebuff.c:26 fileExist: the format is the file's first raw byte */
static int first_byte(const char *path) {
	FILE *f = fopen(path, "rb");
	if(!f) return EOF;
	int c = fgetc(f);
	fclose(f);
	return c;
}

/* dist.c:138-180 with count matrices: ltdMatrixThrd's samples, cmpMats per
 * pair on the GPU (ccg_kma_ltd), printphy of D (and N) */
static int dist_kma(char **files, int nfiles, const char *tmpl, const char *outname, const char *noutname,
                    int metric, unsigned lnorm, unsigned norm, unsigned minDepth, unsigned minLength, double minCov,
                    unsigned flag, int precision, int et, double bs, unsigned threads, int device) {
	if(metric < 0) {
		fprintf(stderr, "ccphylo_amd: distance method is not implemented by the GPU engine (z, p, np).\n");
		return 1;
	}
	FILE *out = (outname[0] == '-' && outname[1] == 0) ? stdout : fopen(outname, "wb");
	if(!out) {
		fprintf(stderr, "Error: %d (%s)\n", errno, strerror(errno));
		return 1;
	}
	FILE *nout = NULL;
	if(noutname) {
		if(!strcmp(noutname, outname)) nout = out;
		else if(noutname[0] == '-' && noutname[1] == 0) nout = stdout;
		else nout = fopen(noutname, "wb");
		if(!nout) {
			fprintf(stderr, "Error: %d (%s)\n", errno, strerror(errno));
			return 1;
		}
	}
	ccq_kma *K = ccq_load_kma(files, nfiles, tmpl, minDepth, minLength, minCov, threads > 16 ? (int) threads : 16,
	                          stderr);
	if(K->status) return 1;
	const int n = K->n;
	ccq_ltd *D = ccq_ltd_new(n > 1 ? n : 2, et, bs), *N = ccq_ltd_new(n > 1 ? n : 2, et, bs);
	D->n = N->n = 0;
	if(n > 1) {
		ccg_ctx *ctx = open_gpu(device);
		ccg_kma_args a;
		memset(&a, 0, sizeof(a));
		a.n = n;
		a.metric = metric;
		a.lnorm = lnorm;
		a.norm = norm;
		a.minDepth = minDepth;
		a.minLength = minLength;
		a.minCov = minCov;
		a.etype = et;
		a.byteScale = bs;
		a.stride1 = K->stride1;
		a.rec1 = K->rec1;
		a.len1 = K->len1;
		a.stride2 = K->stride2;
		a.rec2 = K->rec2;
		a.len2 = K->len2;
		int64_t fatal = -1;
		int rc = ccg_kma_ltd(ctx, &a, D->mat, N->mat, &fatal);
		ccg_destroy(ctx);
		if(rc) {
			fprintf(stderr, "ccphylo_amd: distance computation failed: %s\n", ccg_strerror(rc));
			return 1;
		}
		if(fatal >= 0) {
			int64_t i = 1;
			while((i + 1) * i / 2 <= fatal) ++i;
			const int64_t j = fatal - i * (i - 1) / 2;
			fprintf(stderr, "Template (\"%s\") did not exceed threshold for inclusion:\t%s\n", tmpl,
			        files[K->file_of[j]]);
			return 1;
		}
		if(et >= 4) {   /* cmpMatThrd's warning (it names files[row]) */
			for(int64_t i = 1, f = 0; i < n; ++i) {
				for(int64_t j = 0; j < i; ++j, ++f) {
					if(ccq_ltd_get(D, f) == -1.0) {
						fprintf(stderr, "No sufficient overlap between samples:\t%s\t%s\n", files[i],
						        files[K->file_of[j]]);
					}
				}
			}
		}
		D->n = N->n = n;
	}
	if(1 < D->n) {
		ccq_print_phy(out, D, files, K->include, tmpl, flag, precision);
		if(nout && 1 < N->n) ccq_print_phy(nout, N, files, K->include, tmpl, flag, precision);
	}
	if(out != stdout) fclose(out);
	else fflush(stdout);
	if(nout && nout != out && nout != stdout) fclose(nout);
	ccq_ltd_free(D);
	ccq_ltd_free(N);
	ccq_kma_free(K);
	return 0;
}

/* cmpFsaThrd's pair order over file indices (fsacmpthrd.c:192-218): the
 * skip condition is `&&`, so a pair with one excluded file is not skipped;
 * cells (pi, pj) get these pairs in turn */
static void fsa_cell_pairs(const unsigned char *include, int n, int64_t cells, int *pi_, int *pj_) {
	int first = 0;
	while(first < n && !include[first]) ++first;
	int si = first + 1, sj = 0;
	for(int64_t c = 0; c < cells; ++c) {
		int i = si, j = sj;
		while(!include[i] && !include[j]) {
			while(i < n && !include[i]) ++i;
			while(j < i && !include[j]) ++j;
			if(i == j) {
				++i;
				j = 0;
			}
		}
		pi_[c] = i;
		pj_[c] = j;
		si = i;
		sj = j + 1;
		if(si == sj) {
			++si;
			sj = 0;
		}
	}
}

/* dist.c:138-180 with FASTA files and -r: ltdFsaMatrix_get (cdist.c:36) */
static int dist_fsa_files(char **files, int nfiles, const char *tmpl, const char *outname, const char *noutname,
                          unsigned flag, unsigned norm, unsigned minLength, double minCov, unsigned proxi,
                          int precision, int et, double bs, int device) {
	FILE *out = (outname[0] == '-' && outname[1] == 0) ? stdout : fopen(outname, "wb");
	if(!out) {
		fprintf(stderr, "Error: %d (%s)\n", errno, strerror(errno));
		return 1;
	}
	FILE *nout = NULL;
	if(noutname) {
		if(!strcmp(noutname, outname)) nout = out;
		else if(noutname[0] == '-' && noutname[1] == 0) nout = stdout;
		else nout = fopen(noutname, "wb");
	}
	unsigned char *include = calloc((size_t) nfiles, 1);
	ccq_msa *M = ccq_load_fsa_files(files, nfiles, tmpl, flag, minLength, minCov, proxi, include, stderr);
	if(!M) return 1;
	int Dn = 0;
	for(int f = 0; f < nfiles; ++f) Dn += include[f] != 0;
	ccq_ltd *D = ccq_ltd_new(Dn > 1 ? Dn : 2, et, bs), *N = ccq_ltd_new(Dn > 1 ? Dn : 2, et, bs);
	D->n = N->n = 0;
	const int W = M->W;
	if(!Dn) {
		fprintf(stderr, "All sequences were trimmed away.\n");
	} else {
		ccg_ctx *ctx = open_gpu(device);
		ccg_snp_args sa;
		memset(&sa, 0, sizeof(sa));
		sa.len = M->len;
		sa.stride = W;
		sa.pair = M->pair;
		sa.norm = norm;
		sa.minLength = M->minLength;
		sa.proxi = M->pair ? proxi : 0;
		sa.etype = et;
		sa.byteScale = bs;
		int rc = CCG_OK;
		if(!M->pair) {
			fprintf(stderr, "# %d / %d bases included in distance matrix.\n", ccq_npos(M->incs, M->len), M->len);
		}
		if(M->pair || Dn == nfiles) {
			/* pairs of included files in order (cmpairFsaThrd skips with `||`) */
			uint64_t *sq = malloc((size_t) Dn * W * 8);
			uint32_t *ic = malloc((size_t) (M->pair ? Dn : 1) * W * 4);
			for(int f = 0, r = 0; f < nfiles; ++f) {
				if(!include[f]) continue;
				memcpy(sq + (size_t) r * W, M->seqs + (size_t) f * W, (size_t) W * 8);
				if(M->pair) memcpy(ic + (size_t) r * W, M->incs + (size_t) f * W, (size_t) W * 4);
				++r;
			}
			if(!M->pair) memcpy(ic, M->incs, (size_t) W * 4);
			sa.n = Dn;
			sa.seqs = sq;
			sa.incs = ic;
			if(Dn > 1) rc = ccg_snp_ltd(ctx, &sa, D->mat, (M->pair && nout) ? N->mat : NULL, NULL);
			free(sq);
			free(ic);
		} else if(Dn > 1) {
			/* all files, then the cells in cmpFsaThrd's quirky pair order */
			ccq_ltd *F = ccq_ltd_new(nfiles, et, bs);
			sa.n = nfiles;
			sa.seqs = M->seqs;
			sa.incs = M->incs;
			rc = ccg_snp_ltd(ctx, &sa, F->mat, NULL, NULL);
			const int64_t cells = (int64_t) Dn * (Dn - 1) / 2;
			int *pi_ = malloc((size_t) cells * sizeof(int)), *pj_ = malloc((size_t) cells * sizeof(int));
			fsa_cell_pairs(include, nfiles, cells, pi_, pj_);
			for(int64_t c = 0; c < cells; ++c) {
				const int64_t src = (int64_t) pi_[c] * (pi_[c] - 1) / 2 + pj_[c];
				memcpy((char *) D->mat + c * et, (char *) F->mat + src * et, (size_t) et);
			}
			free(pi_);
			free(pj_);
			ccq_ltd_free(F);
		}
		ccg_destroy(ctx);
		if(rc) {
			fprintf(stderr, "ccphylo_amd: distance computation failed: %s\n", ccg_strerror(rc));
			return 1;
		}
		D->n = Dn;
		if(M->pair) N->n = Dn;
	}
	if(1 < D->n) {
		ccq_print_phy(out, D, files, include, tmpl, flag, precision);
		if(nout && 1 < N->n) ccq_print_phy(nout, N, files, include, tmpl, flag, precision);
	}
	if(out != stdout) fclose(out);
	else fflush(stdout);
	if(nout && nout != out && nout != stdout) fclose(nout);
	ccq_ltd_free(D);
	ccq_ltd_free(N);
	ccq_msa_free(M);
	free(include);
	return 0;
}

/* `dist --tree FILE`: the MSA's distances and the tree in HBM, without the
 * Phylip text (configs[4]: a 1e6-taxon matrix has no text form).  With
 * --gpus G > 1 the LT is written straight into the ranks' row bands
 * (ccg_snp_ltd_shard) and the sharded tree consumes it there; with one GPU
 * the single-GPU engine runs on the full LT.  The Newick equals `ccphylo
 * dist | ccphylo tree` for the same MSA: integer SNP counts print exactly,
 * -W normalised distances are rounded to -x digits as the text would round
 * them (ccg_round_decimal_dev), taxon names as that pipeline's reader holds
 * them (ccq_names_set). */
static int dist_tree(const char *in, const char *treename, const char *tmethod, int tflag, unsigned flag,
                     unsigned norm, unsigned minLength, double minCov, unsigned proxi, int precision, int et,
                     double bs, unsigned threads, int device, int gpus, int transport, int fast) {
	int m;
	if(!strcmp(tmethod, "dnj")) m = CCG_TREE_DNJ;
	else if(!strcmp(tmethod, "nj")) m = CCG_TREE_NJ;
	else if(!strcmp(tmethod, "hnj")) m = CCG_TREE_HNJ;
	else {
		fprintf(stderr, "ccphylo_amd: --tree_method %s: the fused pipeline runs nj, dnj and hnj.\n", tmethod);
		return 1;
	}
	if(norm && (et == 2 || et == 1)) {
		/* the pipeline's text round trip of -W cells through dtouc is not restated */
		fprintf(stderr, "ccphylo_amd: -W with -s / -b and --tree: use `ccphylo dist ... | ccphylo tree`.\n");
		return 1;
	}
	FILE *tout = (treename[0] == '-' && treename[1] == 0) ? stdout : fopen(treename, "wb");
	if(!tout) {
		fprintf(stderr, "Error: %d (%s)\n", errno, strerror(errno));
		return 1;
	}
	ccq_reader *r = ccq_open(in);
	if(!r) {
		fprintf(stderr, "Error: %d (%s)\n", errno, strerror(errno));
		return 1;
	}
	if(ccq_peek(r) != '>') {
		fprintf(stderr, "ccphylo_amd: --tree needs an MSA (FASTA) input.\n");
		return 1;
	}
	ccq_msa *M = ccq_load_msa_par(r, flag, minLength, minCov, proxi, threads > 16 ? (int) threads : 16, stderr);
	ccq_close(r);
	const int n = M->n;
	if(n < 3) {
		fprintf(stderr, "ccphylo_amd: --tree needs at least 3 included sequences (%d).\n", n);
		return 1;
	}
	if(!M->pair) fprintf(stderr, "# %d / %d bases included in distance matrix.\n", ccq_npos(M->incs, M->len), M->len);
	ccg_snp_args sa;
	memset(&sa, 0, sizeof(sa));
	sa.n = n;
	sa.len = M->len;
	sa.stride = M->W;
	sa.seqs = M->seqs;
	sa.incs = M->incs;
	sa.pair = M->pair;   /* -f 2: per-taxon masks, fsacmpair per cell (and -P maskProxi) */
	sa.proxi = M->pair ? proxi : 0;
	sa.norm = norm;
	sa.minLength = M->minLength;
	sa.etype = et;
	sa.byteScale = bs;
	ccg_tree_args ta = {n, et, bs, m, tflag, !fast, 0, 0};
	ccg_join *joins = malloc((size_t) n * sizeof(ccg_join));
	int nj = 0, fn = 0, inc = 0;
	double fd = 0;
	/* -W distances are not integral: the Phylip text of `dist | tree` rounds
	 * them to -x digits, and so does this path (ccg_round_decimal_dev) */
	const int rp = norm ? precision : -1;
	char emsg[320] = "";
	clock_t t0 = clock();
	int rc;
	if(gpus <= 1) {
		/* one GPU: the full LT (the world-1 band layout) and the single-GPU
		 * engine, which also runs the missing-entry rules of updateD
		 * (nj.c:1021-1030) and -m hnj, exactly as `dist | tree` would */
		ccg_ctx *ctx = open_gpu(device);
		void *dD = NULL;
		const size_t lt = (size_t) n * (size_t) (n - 1) / 2 * (size_t) et;
		if((rc = ccg_malloc(ctx, &dD, lt))) snprintf(emsg, sizeof(emsg), "LT buffer: %s", ccg_strerror(rc));
		else if((rc = ccg_snp_ltd_shard(ctx, &sa, 0, 1, dD, &inc)))
			snprintf(emsg, sizeof(emsg), "ccg_snp_ltd_shard: %s", ccg_strerror(rc));
		else if(rp >= 0 && (rc = ccg_round_decimal_dev(ctx, dD, (int64_t) n * (n - 1) / 2, et, rp)))
			snprintf(emsg, sizeof(emsg), "ccg_round_decimal_dev: %s", ccg_strerror(rc));
		else if((rc = ccg_tree_dev(ctx, &ta, dD, joins, &nj, &fn, &fd, NULL)))
			snprintf(emsg, sizeof(emsg), "ccg_tree_dev: %s", ccg_strerror(rc));
		if(dD) ccg_free(ctx, dD);
		ccg_destroy(ctx);
	} else {
		ccq_mgpu mc = {gpus, device, transport, rp};
		rc = ccq_mgpu_dist_tree(&mc, &sa, &ta, joins, &nj, &fn, &fd, &inc, emsg, sizeof(emsg));
		if(rc == CCG_EUNSUP)
			fprintf(stderr, "ccphylo_amd: the matrix has missing entries (pairs below the minimum length); "
			                "their updateD rules run on one GPU: use --gpus 1.\n");
	}
	if(rc) {
		fprintf(stderr, "ccphylo_amd: dist --tree failed: %s\n", emsg);
		return 1;
	}
	fprintf(stderr, "# Total time used computing distances and tree: %.2f s.\n", (double) (clock() - t0) / 1000000);
	ccq_names *T = ccq_names_new(32, 4);   /* as tree.c:61-66 */
	ccq_names_set(T, M->headers, n, flag, '\t');
	ccq_replay_newick(T, n, (const ccq_join *) joins, nj, fn, fd, tflag, precision);
	fprintf(tout, "%s;\n", (char *) T->names[0]->seq);
	if(tout != stdout) fclose(tout);
	else fflush(stdout);
	ccq_names_free(T);
	free(joins);
	ccq_msa_free(M);
	return 0;
}

static int main_dist(int argc, char **argv) {
	const char *outname = "-", *noutname = NULL, *treename = NULL, *tmethod = "dnj";
	char **files = NULL;
	int nfiles = 0, precision = 9, et = 8, device = 0, gpus = 0, transport = CCQ_TRANSPORT_RCCL, fast = 0, tflag = 0;
	unsigned flag = 1, norm = 0, minLength = 1, proxi = 0, minDepth = 15, threads = 1;
	double minCov = 0.5, bs = 1.0;
	const char *unsup = NULL, *tmpl = NULL, *method = "cos";
	Args A = {argc, 0, argv};
	for(A.k = 1; A.k < argc; ++A.k) {
		char *a = argv[A.k];
		if(a[0] != '-' || a[1] == 0) {
			files = argv + A.k;
			nfiles = argc - A.k;
			break;
		}
		if(a[1] == '-') {
			char *name = a + 2, *eq = strchr(name, '=');
			char *att = NULL;
			if(eq) {
				*eq = 0;
				att = eq + 1;
			}
			if(!strcmp(name, "input")) {
				if(att) {
					files = &argv[A.k];
					argv[A.k] = att;
					nfiles = 1;
				} else {
					files = argv + A.k + 1;
					nfiles = 0;
				}
				while(A.k + 1 < argc && (argv[A.k + 1][0] != '-' || argv[A.k + 1][1] == 0)) {
					++A.k;
					++nfiles;
				}
			}
			else if(!strcmp(name, "output")) outname = opt_value(&A, att, "output");
			else if(!strcmp(name, "nucleotide_numbers")) noutname = opt_value(&A, att, "nucleotide_numbers");
			else if(!strcmp(name, "separator")) (void) opt_value(&A, att, "separator");
			else if(!strcmp(name, "print_precision")) precision = (int) opt_num(&A, att, "print_precision");
			else if(!strcmp(name, "min_len")) minLength = (unsigned) opt_num(&A, att, "min_len");
			else if(!strcmp(name, "min_cov")) minCov = strtod(opt_value(&A, att, "min_cov"), NULL) / 100;
			else if(!strcmp(name, "normalization_weight")) norm = (unsigned) opt_num(&A, att, "normalization_weight");
			else if(!strcmp(name, "proximity")) proxi = (unsigned) opt_num(&A, att, "proximity");
			else if(!strcmp(name, "flag")) flag = (unsigned) opt_num(&A, att, "flag");
			else if(!strcmp(name, "flag_help")) flag = (unsigned) -1;
			else if(!strcmp(name, "threads")) threads = (unsigned) opt_num(&A, att, "threads");
			else if(!strcmp(name, "float_precision")) et = 4;
			else if(!strcmp(name, "short_precision")) { et = 2; bs = opt_dvalue_def(&A, att, bs, "short_precision"); }
			else if(!strcmp(name, "byte_precision")) { et = 1; bs = opt_dvalue_def(&A, att, bs, "byte_precision"); }
			else if(!strcmp(name, "mmap")) { }
			else if(!strcmp(name, "tmp")) (void) opt_value(&A, att, "tmp");
			else if(!strcmp(name, "device")) device = (int) opt_num(&A, att, "device");
			else if(!strcmp(name, "tree")) treename = opt_value(&A, att, "tree");
			else if(!strcmp(name, "tree_method")) tmethod = opt_value(&A, att, "tree_method");
			else if(!strcmp(name, "tree_flag")) tflag = (int) opt_num(&A, att, "tree_flag");
			else if(!strcmp(name, "gpus")) gpus = (int) opt_num(&A, att, "gpus");
			else if(!strcmp(name, "transport")) transport = transport_id(opt_value(&A, att, "transport"));
			else if(!strcmp(name, "fast_sums")) fast = 1;
			else if(!strcmp(name, "distance")) method = opt_value(&A, att, name);
			else if(!strcmp(name, "distance_help")) method = NULL;
			else if(!strcmp(name, "min_depth")) minDepth = (unsigned) strtod(opt_value(&A, att, name), NULL);
			else if(!strcmp(name, "significance_lvl")) (void) opt_value(&A, att, name);
			else if(!strcmp(name, "reference")) tmpl = opt_value(&A, att, name);
			else if(!strcmp(name, "add") || !strcmp(name, "methylation_motifs") ||
			        !strcmp(name, "nucleotide_variations")) { (void) opt_value(&A, att, name); unsup = name; }
			else if(!strcmp(name, "help")) return dist_help(stdout);
			else die_opt("Unknown", a);
			continue;
		}
		for(char *p = a + 1; *p; ++p) {
			char o = *p, *att = p + 1;
			int took = 1;
			switch(o) {
				case 'i':
					if(*att) {
						argv[A.k] = att;
						files = argv + A.k;
						nfiles = 1;
					} else {
						files = argv + A.k + 1;
						nfiles = 0;
					}
					while(A.k + 1 < argc && (argv[A.k + 1][0] != '-' || argv[A.k + 1][1] == 0)) {
						++A.k;
						++nfiles;
					}
					break;
				case 'o': outname = opt_value(&A, att, "o"); break;
				case 'n': noutname = opt_value(&A, att, "n"); break;
				case 'S': (void) opt_value(&A, att, "S"); break;
				case 'x': precision = (int) opt_num(&A, att, "x"); break;
				case 'L': minLength = (unsigned) opt_num(&A, att, "L"); break;
				case 'C': minCov = strtod(opt_value(&A, att, "C"), NULL) / 100; break;
				case 'W': norm = (unsigned) opt_num(&A, att, "W"); break;
				case 'P': proxi = (unsigned) opt_num(&A, att, "P"); break;
				case 'f': flag = (unsigned) opt_num(&A, att, "f"); break;
				case 't': threads = (unsigned) opt_num(&A, att, "t"); break;
				case 'T': (void) opt_value(&A, att, "T"); break;
				case 'd': method = opt_value(&A, att, "d"); break;
				case 'E': minDepth = (unsigned) strtod(opt_value(&A, att, "E"), NULL); break;
				case 'l': (void) opt_value(&A, att, "l"); break;
				case 'r': tmpl = opt_value(&A, att, "r"); break;
				case 'a': case 'y': case 'V': {
					static char nm[2];
					nm[0] = o;
					(void) opt_value(&A, att, nm);
					unsup = nm;
					break;
				}
				case 's': et = 2; bs = opt_dvalue_def(&A, att, bs, "s"); break;
				case 'b': et = 1; bs = opt_dvalue_def(&A, att, bs, "b"); break;
				case 'p': et = 4; took = 0; break;
				case 'F': flag = (unsigned) -1; took = 0; break;
				case 'D': method = NULL; took = 0; break;
				case 'H': took = 0; break;
				case 'h': return dist_help(stdout);
				default: {
					char bad[3] = {'-', o, 0};
					die_opt("Unknown", bad);
				}
			}
			if(took) break;
		}
	}
	if(minCov < 0 || 1 < minCov) die_opt("Invalid", "\"--min_cov\"");
	if(bs == 0) die_opt("Invalid", et == 2 ? "\"--short_precision\"" : "\"--byte_precision\"");
	if(flag == (unsigned) -1) {
		fprintf(stdout, "# Format flags output, add them to combine them.\n");
		fprintf(stdout, "#\n");
		fprintf(stdout, "#   1:\tRelaxed Phylip\n");
		fprintf(stdout, "#   2:\tDistances are pairwise, always true on *.mat files\n");
		fprintf(stdout, "#   4:\tInclude template name in phylip file\n");
		fprintf(stdout, "#   8:\tInclude insignificant bases in distance calculation, only affects fasta input\n");
		fprintf(stdout, "#  16:\tDistances based on fasta input\n");
		fprintf(stdout, "#  32:\tDo not include insignificant bases in pruning\n");
		fprintf(stdout, "#\n");
		return 0;
	}
	if(!method) {
		fprintf(stdout, "# Distance calculation methods:\n");
		fprintf(stdout, "#\n");
		fprintf(stdout, "# cos:\tCalculate distance between positions as the angle between the count vectors.\n");
		fprintf(stdout, "# z:\tMake consensus comparison if vectors passes a McNemar test\n");
		fprintf(stdout, "# chi2:\tCalculate the chi square distance\n");
		fprintf(stdout, "# nchi2:\tCalculate the normalized chi square distance\n");
		fprintf(stdout, "# c:\tCalculate the Clausen distance between the count vectors. d(A,B) = (||A-B||_1 / sum(max{Ai, Bi}))\n");
		fprintf(stdout, "# nc:\tCalculate the normalized Clausen distance between the count vectors.\n");
		fprintf(stdout, "# bc:\tCalculate the Bray-Curtis dissimilarity between the count vectors.\n");
		fprintf(stdout, "# nbc:\tCalculate the normalized Bray-Curtis dissimilarity between the count vectors.\n");
		fprintf(stdout, "# ln:\tCalculate distance between positions as the n-norm distance between the count vectors. Replace \"n\" with the waned norm\n");
		fprintf(stdout, "# linf:\tCalculate distance between positions as the l_infinity distance between the count vectors.\n");
		fprintf(stdout, "# nln:\tCalculate distance between positions as the normalized n-norm distance between the count vectors. Replace last \"n\" with the waned norm\n");
		fprintf(stdout, "# nlinf:\tCalculate distance between positions as the normalized l_infinity distance between the count vectors.\n");
		fprintf(stdout, "#\n");
		return 0;
	}
	int metric;
	unsigned lnorm = 0;
	if(kma_metric_id(method, &metric, &lnorm)) die_opt("Invalid", "\"-d\"");
	if(unsup) {
		fprintf(stderr, "ccphylo_amd: dist option \"%s\" is not implemented by the GPU engine.\n", unsup);
		return 1;
	}
	if(tmpl && nfiles > 1 && !(flag & 16) && first_byte(files[0]) != '>') {   /* dist.c:99-108 */
		return dist_kma(files, nfiles, tmpl, outname, noutname, metric, lnorm, norm, minDepth, minLength, minCov,
		                flag, precision, et, bs, threads, device);
	}
	if(tmpl && nfiles > 1) {
		return dist_fsa_files(files, nfiles, tmpl, outname, noutname, flag, norm, minLength, minCov, proxi,
		                      precision, et, bs, device);
	}
	if(nfiles > 1) {
		fprintf(stderr, "ccphylo_amd: multi-file dist input is not implemented by the GPU engine (use one MSA).\n");
		return 1;
	}
	if(treename) {
		return dist_tree(nfiles ? files[0] : "-", treename, tmethod, tflag, flag, norm, minLength, minCov, proxi,
		                 precision, et, bs, threads, device, gpus, transport, fast);
	}
	FILE *out = (outname[0] == '-' && outname[1] == 0) ? stdout : fopen(outname, "wb");
	if(!out) {
		fprintf(stderr, "Error: %d (%s)\n", errno, strerror(errno));
		return 1;
	}
	FILE *nout = NULL;
	if(noutname) {
		/* dist.c:74-84 opens (truncates) it; cdist.c:367 then prints N to outfile */
		if(!strcmp(noutname, outname)) nout = out;
		else if(noutname[0] == '-' && noutname[1] == 0) nout = stdout;
		else nout = fopen(noutname, "wb");
	}
	const char *in = nfiles ? files[0] : "-";
	ccq_reader *r = ccq_open(in);
	if(!r) {
		fprintf(stderr, "Error: %d (%s)\n", errno, strerror(errno));
		return 1;
	}
	if(!(flag & 16) && ccq_peek(r) != '>') {
		fprintf(stderr, "ccphylo_amd: count-matrix (.mat) / union input is not implemented by the GPU engine.\n");
		return 1;
	}
	/* the per-sequence work on host threads (fasta_par.c; the same result as
	 * the serial ccq_load_msa) */
	ccq_msa *M = ccq_load_msa_par(r, flag, minLength, minCov, proxi, threads > 16 ? (int) threads : 16, stderr);
	ccq_close(r);
	int n = M->n;
	if(n * (n - 1) / 2 < 1) {
		fprintf(stderr, "Adjustning number of nodes to %d, to conform with the matrix size.\n", n * (n - 1) / 2);
	}
	ccq_ltd *D = ccq_ltd_new(n > 1 ? n : 2, et, bs), *N = NULL;
	if(!n) {
		fprintf(stderr, "All sequences were trimmed away.\n");
		D->n = 0;
	} else {
		if(noutname) N = ccq_ltd_new(n > 1 ? n : 2, et, bs);
		ccg_ctx *ctx = open_gpu(device);
		ccg_snp_args sa;
		memset(&sa, 0, sizeof(sa));
		sa.n = n;
		sa.len = M->len;
		sa.stride = M->W;
		sa.seqs = M->seqs;
		sa.incs = M->incs;
		sa.pair = M->pair;
		sa.norm = norm;
		sa.minLength = M->minLength;
		sa.proxi = M->pair ? proxi : 0;
		sa.etype = et;
		sa.byteScale = bs;
		int inc = 0;
		if(!M->pair) {
			inc = ccq_npos(M->incs, M->len);
			fprintf(stderr, "# %d / %d bases included in distance matrix.\n", inc, M->len);
		}
		int rc = ccg_snp_ltd(ctx, &sa, D->mat, N ? N->mat : NULL, NULL);
		if(rc) {
			fprintf(stderr, "ccphylo_amd: distance computation failed: %s\n", ccg_strerror(rc));
			return 1;
		}
		ccg_destroy(ctx);
		D->n = n;
		if(N) N->n = M->pair ? n : 0;
	}
	if(1 < D->n) {
		ccq_print_phy(out, D, M->headers, NULL, NULL, flag, precision);
		if(N && 1 < N->n) ccq_print_phy(out, N, M->headers, NULL, NULL, flag, precision);
	}
	if(out != stdout) fclose(out);
	else fflush(stdout);
	if(nout && nout != out && nout != stdout) fclose(nout);
	ccq_ltd_free(D);
	ccq_ltd_free(N);
	ccq_msa_free(M);
	return 0;
}

static int main_help(FILE *out) {
	fprintf(out, "# CCPhylo (ccphylo_amd: MI355X engine for dist and tree)\n");
	fprintf(out, "# Usage: ccphylo <command> [options]\n");
	fprintf(out, "#    %-16s\t%s\n", "dist", "all-pairs SNP distances of an MSA (GPU)");
	fprintf(out, "#    %-16s\t%s\n", "tree", "NJ / DNJ trees from Phylip matrices (GPU)");
	return out == stderr;
}

int main(int argc, char **argv) {
	if(argc < 2) {
		fprintf(stderr, "Too few arguments handed.\n");
		return main_help(stderr);
	}
	if(!strcmp(argv[1], "dist")) return main_dist(argc - 1, argv + 1);
	if(!strcmp(argv[1], "tree")) return main_tree(argc - 1, argv + 1);
	if(!strcmp(argv[1], "-h") || !strcmp(argv[1], "--help")) return main_help(stdout);
	fprintf(stderr, "ccphylo_amd: command \"%s\" is outside the GPU engine's scope (dist, tree).\n", argv[1]);
	return 1;
}
