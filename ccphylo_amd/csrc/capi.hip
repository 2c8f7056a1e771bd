// capi.hip -- the extern "C" boundary of libccphylo_amd.so (include/ccphylo_amd.h).
#include <stdio.h>
#include <string.h>
#include <stdlib.h>
#include <mutex>
#include <vector>
#include "ccg_internal.h"

int ccg_snp_dev_impl(ccg_ctx *ctx, const ccg_snp_args *a, void *D, void *N, int *inc_out, bool host_in);
int ccg_snp_shard_dev_impl(ccg_ctx *ctx, const ccg_snp_args *a, int rank, int world, void *Dloc, int *inc_out,
                           bool host_in);
int ccg_tree_impl(ccg_ctx *ctx, const ccg_tree_args *a, void *Dd, ccg_join *joins, int *njoins, int *final_n,
                  double *final_d, int64_t *stats, const ccg_dnj_state *sin, ccg_dnj_state *sout);
int ccg_selftest_row_sum_impl(ccg_ctx *ctx, const double *c, int n, double *out, int *parallel);

// per host thread, like the tree's grid state: two contexts driven from two
// threads (the pipelined bench) keep their own messages
static thread_local char g_last_error[512];

void ccg_set_last_error(hipError_t e, const char *what, const char *file, int line) {
	snprintf(g_last_error, sizeof(g_last_error), "%s (%d) in %s at %s:%d", hipGetErrorString(e), (int) e, what, file,
	         line);
	fprintf(stderr, "ccphylo_amd: HIP error: %s\n", g_last_error);
}

void ccg_set_last_msg(const char *msg) {
	snprintf(g_last_error, sizeof(g_last_error), "%s", msg);
	fprintf(stderr, "ccphylo_amd: %s\n", g_last_error);
}

int ccg_ctx_workspace(ccg_ctx *c, int k, size_t bytes, void **p) {
	if(c->ws[k] && c->ws_bytes[k] >= bytes) {
		*p = c->ws[k];
		return CCG_OK;
	}
	if(c->ws[k]) {   // grow: the only hipFree of a tree run, at a context's first run of a larger tree
		CCG_CHECK(hipStreamSynchronize(c->stream));
		CCG_CHECK(hipFree(c->ws[k]));
		c->ws[k] = NULL;
		c->ws_bytes[k] = 0;
	}
	if(hipMalloc(&c->ws[k], bytes) != hipSuccess) {   // quietly: the block bounds' slot is optional
		(void) hipGetLastError();
		c->ws[k] = NULL;
		return CCG_ENOMEM;
	}
	c->ws_bytes[k] = bytes;
	*p = c->ws[k];
	return CCG_OK;
}

extern "C" {

const char *ccg_strerror(int code) {
	switch(code) {
		case CCG_OK: return "success";
		case CCG_EINVAL: return "invalid argument";
		case CCG_ENODEV: return "no gfx950 (MI355X) HIP device available";
		case CCG_ENOMEM: return "device out of memory";
		case CCG_EHIP: return g_last_error[0] ? g_last_error : "HIP runtime error";
		case CCG_EUNSUP: return "not supported by the GPU engine";
		default: return "unknown error";
	}
}

int ccg_device_count(int *count) {
	if(!count) return CCG_EINVAL;
	*count = 0;
	int c = 0;
	if(hipGetDeviceCount(&c) != hipSuccess || c <= 0) return CCG_ENODEV;
	*count = c;
	return CCG_OK;
}

int ccg_init(int device, ccg_ctx **out) {
	if(!out) return CCG_EINVAL;
	*out = NULL;
	int count = 0;
	if(hipGetDeviceCount(&count) != hipSuccess || count <= 0 || device < 0 || device >= count) {
		return CCG_ENODEV;
	}
	hipDeviceProp_t prop;
	if(hipGetDeviceProperties(&prop, device) != hipSuccess) return CCG_ENODEV;
	if(strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
		snprintf(g_last_error, sizeof(g_last_error), "device %d is %s, this build targets gfx950", device,
		         prop.gcnArchName);
		return CCG_ENODEV;
	}
	CCG_CHECK(hipSetDevice(device));
	ccg_ctx *c = (ccg_ctx *) calloc(1, sizeof(ccg_ctx));
	if(!c) return CCG_ENOMEM;
	c->device = device;
	c->ncu = prop.multiProcessorCount;
	snprintf(c->name, sizeof(c->name), "%s (%s, %d CUs)", prop.name, prop.gcnArchName, prop.multiProcessorCount);
	if(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
	   hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess) {
		free(c);
		return CCG_EHIP;
	}
	*out = c;
	return CCG_OK;
}

// every CU-masked stream the process made (never destroyed before ccg_shutdown)
static std::mutex g_masked_mu;
static std::vector<hipStream_t> g_masked;
static bool g_shut = false;   // ccg_shutdown ran: a masked context's stream is gone

int ccg_ctx_configure(ccg_ctx *c, const uint32_t *cu_mask, int mask_words, int flags) {
	if(!c || mask_words < 0 || (mask_words && !cu_mask)) return CCG_EINVAL;
	CCG_CHECK(hipSetDevice(c->device));
	hipStream_t s = NULL;
	if(mask_words) {   // the engine stream again, limited to the CUs of the mask
		// mask bit k runs on XCD k % nx (slot k / nx within it), and an XCD
		// whose share of the mask is empty runs on ALL of its CUs
		// (profiles/r06_cu_mask_map.txt): such a mask does not limit the stream
		hipDeviceProp_t p;
		CCG_CHECK(hipGetDeviceProperties(&p, c->device));
		const int ncu = p.multiProcessorCount, nx = ncu >= 32 ? ncu / 32 : 1;
		for(int x = 0; x < nx; ++x) {
			bool any = false;
			for(int k = x; k < ncu && k < 32 * mask_words && !any; k += nx) any = (cu_mask[k / 32] >> (k % 32)) & 1u;
			if(!any) {
				snprintf(g_last_error, sizeof(g_last_error),
				         "ccg_ctx_configure: the CU mask leaves XCD %d (mask bits k with k %% %d == %d) without a CU; "
				         "that XCD would run on all of its CUs",
				         x, nx, x);
				return CCG_EINVAL;
			}
		}
		CCG_CHECK(hipExtStreamCreateWithCUMask(&s, (uint32_t) mask_words, cu_mask));
	} else if(c->masked) {   // back to the whole chip
		CCG_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
	}
	if(s) {
		CCG_CHECK(hipStreamSynchronize(c->stream));
		// a CU-masked stream is drained but never destroyed: on this ROCm
		// (7.2, gfx950) destroying one leaves the runtime to hand a dead
		// hardware queue to a later stream, whose kernels then never complete
		// (the pure-HIP reproducer `tools/micro/cu_mask engine 2 8 1 1 0 0`:
		// the second stream created after the destroy hangs; a plain stream
		// destroyed the same way, or the masked one kept, run clean:
		// profiles/r06_cu_mask_destroy.txt).  It is released with the process.
		if(!c->masked) CCG_CHECK(hipStreamDestroy(c->stream));
		if(mask_words) {   // parked for ccg_shutdown
			std::lock_guard<std::mutex> g(g_masked_mu);
			g_masked.push_back(s);
		}
		c->stream = s;
		c->masked = mask_words != 0;
		c->cus = 0;
		for(int k = 0; mask_words && k < c->ncu && k < 32 * mask_words; ++k) c->cus += (cu_mask[k / 32] >> (k % 32)) & 1u;
	}
	c->flags = flags;
	return CCG_OK;
}

void ccg_destroy(ccg_ctx *c) {
	if(!c) return;
	hipSetDevice(c->device);
	if(!(c->masked && g_shut)) hipStreamSynchronize(c->stream);
	for(int k = 0; k < 3; ++k)
		if(c->ws[k]) hipFree(c->ws[k]);
	hipEventDestroy(c->ev0);
	hipEventDestroy(c->ev1);
	if(!c->masked) hipStreamDestroy(c->stream);   // (a CU-masked one stays: ccg_ctx_configure)
	free(c);
}

int ccg_shutdown(void) {
	std::lock_guard<std::mutex> g(g_masked_mu);
	int rc = CCG_OK;
	for(hipStream_t s : g_masked) {
		if(hipStreamSynchronize(s) != hipSuccess || hipStreamDestroy(s) != hipSuccess) rc = CCG_EHIP;
	}
	g_masked.clear();
	g_shut = true;
	return rc;
}

int ccg_device_info(ccg_ctx *c, char *buf, size_t len) {
	if(!c || !buf || !len) return CCG_EINVAL;
	snprintf(buf, len, "%s", c->name);
	return CCG_OK;
}

int ccg_snp_ltd_dev(ccg_ctx *c, const ccg_snp_args *a, void *D, void *N, int *inc_out) {
	if(!c || !a || !D) return CCG_EINVAL;
	CCG_CHECK(hipSetDevice(c->device));
	CCG_DEVICE_SYNC(c);   // inputs may come from other streams (e.g. torch's)
	return ccg_snp_dev_impl(c, a, D, N, inc_out, false);
}

int ccg_snp_ltd_shard_dev(ccg_ctx *c, const ccg_snp_args *a, int rank, int world, void *Dloc, int *inc_out) {
	if(!c || !a || !Dloc) return CCG_EINVAL;
	CCG_CHECK(hipSetDevice(c->device));
	CCG_DEVICE_SYNC(c);
	return ccg_snp_shard_dev_impl(c, a, rank, world, Dloc, inc_out, false);
}

int ccg_snp_ltd_shard(ccg_ctx *c, const ccg_snp_args *a, int rank, int world, void *Dloc, int *inc_out) {
	if(!c || !a || !Dloc || !a->seqs || !a->incs) return CCG_EINVAL;
	CCG_CHECK(hipSetDevice(c->device));
	CCG_DEVICE_SYNC(c);
	return ccg_snp_shard_dev_impl(c, a, rank, world, Dloc, inc_out, true);
}

int ccg_snp_ltd(ccg_ctx *c, const ccg_snp_args *a, void *D, void *N, int *inc_out) {
	if(!c || !a || !D || !a->seqs || !a->incs) return CCG_EINVAL;
	if(a->n < 0 || a->len <= 0 || a->stride < (a->len + 31) / 32) return CCG_EINVAL;
	CCG_CHECK(hipSetDevice(c->device));
	size_t n = (size_t) a->n;
	size_t lt = n > 1 ? n * (n - 1) / 2 * (size_t) a->etype : 0;
	void *d_D = NULL, *d_N = NULL;
	int rc = CCG_OK;
	if(hipMalloc(&d_D, lt ? lt : 8) != hipSuccess || (N && a->pair && hipMalloc(&d_N, lt ? lt : 8) != hipSuccess)) {
		rc = CCG_ENOMEM;
		goto done;
	}
	// untouched cells (outside a row range) keep the caller's contents
	if(lt && (a->row_begin || a->row_end)) {
		if(hipMemcpyAsync(d_D, D, lt, hipMemcpyHostToDevice, c->stream) != hipSuccess ||
		   (d_N && hipMemcpyAsync(d_N, N, lt, hipMemcpyHostToDevice, c->stream) != hipSuccess)) {
			rc = CCG_EHIP;
			goto done;
		}
	}
	// the packed sequences stream from host memory into the bit planes
	rc = ccg_snp_dev_impl(c, a, d_D, d_N, inc_out, true);
	if(rc == CCG_OK && lt) {
		if(hipMemcpyAsync(D, d_D, lt, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
		   (d_N && hipMemcpyAsync(N, d_N, lt, hipMemcpyDeviceToHost, c->stream) != hipSuccess) ||
		   hipStreamSynchronize(c->stream) != hipSuccess) {
			rc = CCG_EHIP;
		}
	}
done:
	hipStreamSynchronize(c->stream);
	if(d_D) hipFree(d_D);
	if(d_N) hipFree(d_N);
	return rc;
}

int ccg_tree_dev(ccg_ctx *c, const ccg_tree_args *a, void *D, ccg_join *joins, int *njoins, int *final_n,
                 double *final_d, int64_t *stats) {
	if(!c || !a || !D || !joins || !njoins || !final_n || !final_d) return CCG_EINVAL;
	if(a->n < 3 || (a->method != CCG_TREE_NJ && a->method != CCG_TREE_DNJ && a->method != CCG_TREE_HNJ))
		return CCG_EINVAL;
	if(a->etype != 8 && a->etype != 4 && a->etype != 2 && a->etype != 1) return CCG_EINVAL;
	if((a->etype == 2 || a->etype == 1) && !(a->byteScale != 0)) return CCG_EINVAL;
	CCG_CHECK(hipSetDevice(c->device));
	CCG_DEVICE_SYNC(c);   // inputs may come from other streams (e.g. torch's)
	return ccg_tree_impl(c, a, D, joins, njoins, final_n, final_d, stats, NULL, NULL);
}

int ccg_tree_dev_state(ccg_ctx *c, const ccg_tree_args *a, void *D, const ccg_dnj_state *in, ccg_dnj_state *out,
                       ccg_join *joins, int *njoins, int *final_n, double *final_d, int64_t *stats) {
	if(!c || !a || !D || !joins || !njoins || !final_n || !final_d) return CCG_EINVAL;
	if(a->n < 3 || a->method != CCG_TREE_DNJ) return CCG_EINVAL;
	if(a->etype != 8 && a->etype != 4 && a->etype != 2 && a->etype != 1) return CCG_EINVAL;
	if((a->etype == 2 || a->etype == 1) && !(a->byteScale != 0)) return CCG_EINVAL;
	if(in && (in->n != a->n || !in->sD || !in->Q || !in->N || !in->P || in->cand < 0 || in->cand >= in->n))
		return CCG_EINVAL;
	if(out && (!out->sD || !out->Q || !out->N || !out->P)) return CCG_EINVAL;
	CCG_CHECK(hipSetDevice(c->device));
	CCG_DEVICE_SYNC(c);
	return ccg_tree_impl(c, a, D, joins, njoins, final_n, final_d, stats, in, out);
}

int ccg_tree(ccg_ctx *c, const ccg_tree_args *a, const void *D, ccg_join *joins, int *njoins, int *final_n,
             double *final_d, int64_t *stats) {
	if(!c || !a || !D) return CCG_EINVAL;
	if(a->n < 3) return CCG_EINVAL;
	CCG_CHECK(hipSetDevice(c->device));
	size_t bytes = (size_t) a->n * (size_t) (a->n - 1) / 2 * (size_t) a->etype;
	void *d = NULL;
	if(hipMalloc(&d, bytes) != hipSuccess) return CCG_ENOMEM;
	int rc = CCG_OK;
	if(hipMemcpyAsync(d, D, bytes, hipMemcpyHostToDevice, c->stream) != hipSuccess) {
		rc = CCG_EHIP;
	} else {
		rc = ccg_tree_dev(c, a, d, joins, njoins, final_n, final_d, stats);
	}
	hipStreamSynchronize(c->stream);
	hipFree(d);
	return rc;
}

int ccg_malloc(ccg_ctx *c, void **p, size_t bytes) {
	if(!c || !p) return CCG_EINVAL;
	CCG_CHECK(hipSetDevice(c->device));
	CCG_CHECK(hipMalloc(p, bytes ? bytes : 1));
	return CCG_OK;
}

int ccg_free(ccg_ctx *c, void *p) {
	if(!c) return CCG_EINVAL;
	CCG_CHECK(hipFree(p));
	return CCG_OK;
}

int ccg_memcpy_h2d(ccg_ctx *c, void *dst, const void *src, size_t bytes) {
	if(!c) return CCG_EINVAL;
	CCG_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, c->stream));
	CCG_CHECK(hipStreamSynchronize(c->stream));
	return CCG_OK;
}

int ccg_memcpy_d2h(ccg_ctx *c, void *dst, const void *src, size_t bytes) {
	if(!c) return CCG_EINVAL;
	CCG_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, c->stream));
	CCG_CHECK(hipStreamSynchronize(c->stream));
	return CCG_OK;
}

int ccg_synchronize(ccg_ctx *c) {
	if(!c) return CCG_EINVAL;
	CCG_CHECK(hipStreamSynchronize(c->stream));
	return CCG_OK;
}

int ccg_selftest_row_sum(ccg_ctx *c, const double *v, int n, double *out, int *parallel) {
	if(!c || !v || n < 1 || !out || !parallel) return CCG_EINVAL;
	hipSetDevice(c->device);
	return ccg_selftest_row_sum_impl(c, v, n, out, parallel);
}

}   // extern "C"
