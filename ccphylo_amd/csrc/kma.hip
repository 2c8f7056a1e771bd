// kma.hip -- distances between KMA count matrices (ccphylo dist on *.mat),
// cmpMats (matcmp.c:448) for every pair of included
// samples, as ltdMatrixThrd (ltdmatrixthrd.c:376) fills the LT.
//
// A pair's distance is a SEQUENTIAL double sum over positions (the
// reference's order), so a pair never splits across threads: parallelism is
// over pairs.  Blocks own 32 x 32 sample tiles of the LT; each thread keeps
// 2 x 2 pairs in registers and the block stages 32-position chunks of the 64
// samples' rows through LDS (every row read from HBM once per tile instead of
// once per pair).  Per position the metric is a handful of integer and f64
// ops -- VALU-bound; the norms sqrt(sum c^2) of `cos` depend on one sample
// only and are precomputed per row (k_kma_norms).
//
// Exactness: every metric runs the reference's operation order under
// -ffp-contract=off; int products wrap like the reference's 32-bit imul.
#include <stdio.h>
#include <string.h>
#include "ccg_internal.h"

#define KT 32        // samples per tile side
#define KP 32        // positions per LDS chunk
#define KTB 256      // threads per block (16 x 16, 2 x 2 pairs each)

__device__ __forceinline__ int imul32(int a, int b) { return (int) ((unsigned) a * (unsigned) b); }

struct Cnt {
	int c[6];
	int tot;   // the u32 total passed as int (veccmp's int parameters)
};

__device__ __forceinline__ Cnt unpack(uint4 w) {
	Cnt r;
	r.c[0] = (int) (w.x & 0xFFFFu);
	r.c[1] = (int) (w.x >> 16);
	r.c[2] = (int) (w.y & 0xFFFFu);
	r.c[3] = (int) (w.y >> 16);
	r.c[4] = (int) (w.z & 0xFFFFu);
	r.c[5] = (int) (w.z >> 16);
	r.tot = (int) w.w;
	return r;
}

// ------------------------------------------------------------------ metrics
template <int M>
__device__ __forceinline__ double kma_metric(const Cnt &x, const Cnt &y, double s1, double s2, unsigned ln) {
	if constexpr(M == CCG_KMA_COS) {   // matcmp.c:420; s = sqrt(sum c^2), 0 iff the sum is 0
		long long dot = 0;
#pragma unroll
		for(int k = 0; k < 5; ++k) dot += imul32(x.c[k], y.c[k]);
		if(s1 == 0 || s2 == 0) return -1;
		double d = 1 - (double) dot / (s1 * s2);
		return d < 0 ? 0 : d;
	} else if constexpr(M == CCG_KMA_L1) {   // :143
		int s = 0;
#pragma unroll
		for(int k = 0; k < 5; ++k) s += abs(x.c[k] - y.c[k]);
		return s;
	} else if constexpr(M == CCG_KMA_L2) {   // :158
		int s = 0;
#pragma unroll
		for(int k = 0; k < 5; ++k) {
			const int t = x.c[k] - y.c[k];
			s += imul32(t, t);
		}
		return sqrt((double) s);
	} else if constexpr(M == CCG_KMA_LINF) {   // :193
		int m = abs(x.c[0] - y.c[0]);
#pragma unroll
		for(int k = 1; k < 5; ++k) {
			const int t = abs(x.c[k] - y.c[k]);
			m = m < t ? t : m;
		}
		return m;
	} else if constexpr(M == CCG_KMA_LN) {   // :173
		double d = pow((double) abs(x.c[0] - y.c[0]), (double) ln);
#pragma unroll
		for(int k = 1; k < 5; ++k) d += pow((double) abs(x.c[k] - y.c[k]), (double) ln);
		d = pow(d, 1.0 / ln);
		return d < 0 ? 0 : d;
	} else if constexpr(M == CCG_KMA_C) {   // :278
		double d;
		int T;
		if(x.c[0] < y.c[0]) {
			d = x.c[0];
			T = y.c[0];
		} else {
			d = y.c[0];
			T = x.c[0];
		}
#pragma unroll
		for(int k = 1; k < 5; ++k) {
			const bool lt = x.c[k] < y.c[k];
			d += lt ? x.c[k] : y.c[k];
			T += lt ? y.c[k] : x.c[k];
		}
		if(!T) return -1;
		d = 1 - d / T;
		return d < 0 ? 0 : d;
	} else if constexpr(M == CCG_KMA_BC) {   // :227
		double d = x.c[0] < y.c[0] ? x.c[0] : y.c[0];
#pragma unroll
		for(int k = 1; k < 5; ++k) d += x.c[k] < y.c[k] ? x.c[k] : y.c[k];
		d /= (x.tot - x.c[5] + y.tot - y.c[5]);
		d = 1 - 2 * d;
		return d < 0 ? 0 : d;
	} else if constexpr(M == CCG_KMA_CHI2) {   // :381
		double d = 0;
#pragma unroll
		for(int k = 0; k < 5; ++k) {
			const double T = x.c[k] - y.c[k];
			if(T != 0) {
				const double q = T * T / (x.c[k] + y.c[k]);
				d = k ? d + q : q;
			}
		}
		return sqrt(d);
	} else {
		// the normalized metrics: fractions of the total without N (slot 5)
		const int t1 = x.tot - x.c[5], t2 = y.tot - y.c[5];
		if constexpr(M == CCG_KMA_NL1) {   // :63
			double d = 0;
#pragma unroll
			for(int k = 0; k < 5; ++k) {
				double t = (double) x.c[k] / t1 - (double) y.c[k] / t2;
				t = t < 0 ? -t : t;
				d = k ? d + t : t;
			}
			return d;
		} else if constexpr(M == CCG_KMA_NL2) {   // :81
			double d = 0;
#pragma unroll
			for(int k = 0; k < 5; ++k) {
				const double t = (double) x.c[k] / t1 - (double) y.c[k] / t2;
				d = k ? d + t * t : t * t;
			}
			return sqrt(d);
		} else if constexpr(M == CCG_KMA_NLN) {   // :98 (first term without |.|)
			double d = pow((double) x.c[0] / t1 - (double) y.c[0] / t2, (double) ln);
#pragma unroll
			for(int k = 1; k < 5; ++k) {
				double t = (double) x.c[k] / t1 - (double) y.c[k] / t2;
				t = t < 0 ? -t : t;
				d += pow(t, (double) ln);
			}
			d = pow(d, 1.0 / ln);
			return d < 0 ? 0 : d;
		} else if constexpr(M == CCG_KMA_NLINF) {   // :122 (compares component 0 only)
			const double t = (double) x.c[0] / t1 - (double) y.c[0] / t2;
			return t < 0 ? -t : t;
		} else if constexpr(M == CCG_KMA_NBC) {   // :206
			double d = 0;
#pragma unroll
			for(int k = 0; k < 5; ++k) {
				const double a = (double) x.c[k] / t1, b = (double) y.c[k] / t2, m = a < b ? a : b;
				d = k ? d + m : m;
			}
			d = 1 - d;
			return d < 0 ? 0 : d;
		} else if constexpr(M == CCG_KMA_NC) {   // :243 (denominator reset each step)
			double a = (double) x.c[0] / t1, b = (double) y.c[0] / t2, d, T;
			if(a < b) {
				d = a;
				T = b;
			} else {
				d = b;
				T = a;
			}
#pragma unroll
			for(int k = 1; k < 5; ++k) {
				a = (double) x.c[k] / t1;
				b = (double) y.c[k] / t2;
				T = 1;
				if(a < b) {
					d += a;
					T += b;
				} else {
					d += b;
					T += a;
				}
			}
			d = 1 - d / T;
			return d < 0 ? 0 : d;
		} else {   // CCG_KMA_NCHI2 :396
			double d = 0;
#pragma unroll
			for(int k = 0; k < 5; ++k) {
				const double a = (double) x.c[k] / t1, b = (double) y.c[k] / t2, df = a - b;
				if(df != 0) {
					const double q = df * df / (a + b);
					d = k ? d + q : q;
				}
			}
			return sqrt(d);
		}
	}
}

// cos: sqrt of the sum of squares of components 0..4 per row (an unsigned
// long of wrapped int products in the reference), 0 iff that sum is 0
__global__ void k_kma_norms(const uint4 *__restrict__ rec, long long rows, double *__restrict__ s) {
	for(long long k = (long long) blockIdx.x * blockDim.x + threadIdx.x; k < rows;
	    k += (long long) gridDim.x * blockDim.x) {
		const Cnt x = unpack(rec[k]);
		unsigned long long c = 0;
#pragma unroll
		for(int t = 0; t < 5; ++t) c += (unsigned long long) (long long) imul32(x.c[t], x.c[t]);
		s[k] = sqrt((double) c);
	}
}

// nNucs of cmpMats (matcmp.c:470): rows of the column sample with
// minDepth <= total; it depends on the column sample only
__global__ __launch_bounds__(256) void k_kma_nnucs(const uint4 *__restrict__ rec2, const int *__restrict__ len2,
                                                   long long stride2, unsigned minDepth, unsigned *__restrict__ out) {
	__shared__ unsigned s;
	if(threadIdx.x == 0) s = 0;
	__syncthreads();
	const int j = blockIdx.x, l = len2[j];
	unsigned c = 0;
	for(int r = threadIdx.x; r < l; r += blockDim.x) c += minDepth <= rec2[(long long) j * stride2 + r].w;
	atomicAdd(&s, c);
	__syncthreads();
	if(threadIdx.x == 0) out[j] = s;
}

struct KmaDev {
	const uint4 *rec1, *rec2;
	const double *s1, *s2;
	const int *len1, *len2;
	const unsigned *nnucs;
	long long stride1, stride2;
	int n;
	unsigned minDepth, minLength, norm, ln;
	double minCov, bs;
	unsigned long long *fatal;
};

// ------------------------------------------------------------------ pairs
template <int M, int ET>
__global__ __launch_bounds__(KTB) void k_kma_pairs(KmaDev a, typename Elem<ET>::T *__restrict__ D,
                                                   typename Elem<ET>::T *__restrict__ N) {
	__shared__ uint4 r1[KT][KP + 1], r2[KT][KP + 1];
	__shared__ double q1[M == CCG_KMA_COS ? KT : 1][KP + 1], q2[M == CCG_KMA_COS ? KT : 1][KP + 1];
	__shared__ int sb[KT][KT];   // per-pair position bound (0: no accumulation)
	// tile (bi, bj), bj <= bi, from the triangular block index
	const long long t = blockIdx.x;
	long long bi = (long long) ((sqrt(8.0 * (double) t + 1.0) - 1.0) * 0.5);
	while(bi * (bi + 1) / 2 > t) --bi;
	while((bi + 1) * (bi + 2) / 2 <= t) ++bi;
	const int bj = (int) (t - bi * (bi + 1) / 2);
	const int i0 = (int) bi * KT, j0 = bj * KT;
	const int tid = threadIdx.x, ti = tid >> 4, tj = tid & 15;
	// pair bounds: cmpMats stops early (-1) when sample j has more rows than
	// sample i's stripped length; otherwise it runs over all rows of j
	__shared__ int s_max;
	if(tid == 0) s_max = 0;
	__syncthreads();
	int tmax = 0;
	for(int e = tid; e < KT * KT; e += KTB) {
		const int i = i0 + e / KT, j = j0 + e % KT;
		int b = 0;
		if(i < a.n && j < i) {
			const int l1 = a.len1[i], l2 = a.len2[j];
			b = l2 > l1 ? 0 : l2;
		}
		sb[e / KT][e % KT] = b;
		tmax = b > tmax ? b : tmax;
	}
	atomicMax(&s_max, tmax);
	__syncthreads();
	const int rmax = s_max;
	int bnd[2][2];
	double acc[2][2];
	int inc[2][2];
#pragma unroll
	for(int u = 0; u < 2; ++u)
#pragma unroll
		for(int v = 0; v < 2; ++v) {
			bnd[u][v] = sb[ti + 16 * u][tj + 16 * v];
			acc[u][v] = 0;
			inc[u][v] = 0;
		}
	for(int c0 = 0; c0 < rmax; c0 += KP) {
		// stage rows [c0, c0 + KP) of the tile's 32 row samples and 32 column samples
		for(int e = tid; e < KT * KP; e += KTB) {
			const int s = e / KP, p = e % KP, r = c0 + p;
			const int i = i0 + s, j = j0 + s;
			uint4 z = make_uint4(0, 0, 0, 0), w1 = z, w2 = z;
			double n1 = 0, n2 = 0;
			if(i < a.n && r < a.stride1) {
				w1 = a.rec1[(long long) i * a.stride1 + r];
				if(M == CCG_KMA_COS) n1 = a.s1[(long long) i * a.stride1 + r];
			}
			if(j < a.n && r < a.stride2) {
				w2 = a.rec2[(long long) j * a.stride2 + r];
				if(M == CCG_KMA_COS) n2 = a.s2[(long long) j * a.stride2 + r];
			}
			r1[s][p] = w1;
			r2[s][p] = w2;
			if(M == CCG_KMA_COS) {
				q1[s][p] = n1;
				q2[s][p] = n2;
			}
		}
		__syncthreads();
		const int pend = rmax - c0 < KP ? rmax - c0 : KP;
		for(int p = 0; p < pend; ++p) {
			const int r = c0 + p;
			Cnt x[2], y[2];
			double nx[2] = {0, 0}, ny[2] = {0, 0};
#pragma unroll
			for(int u = 0; u < 2; ++u) {
				x[u] = unpack(r1[ti + 16 * u][p]);
				y[u] = unpack(r2[tj + 16 * u][p]);
				if(M == CCG_KMA_COS) {
					nx[u] = q1[ti + 16 * u][p];
					ny[u] = q2[tj + 16 * u][p];
				}
			}
#pragma unroll
			for(int u = 0; u < 2; ++u)
#pragma unroll
				for(int v = 0; v < 2; ++v) {
					if(r < bnd[u][v] && a.minDepth <= (unsigned) y[v].tot && a.minDepth <= (unsigned) x[u].tot) {
						const double d = kma_metric<M>(x[u], y[v], nx[u], ny[v], a.ln);
						if(0 <= d) {
							acc[u][v] += d;
							++inc[u][v];
						}
					}
				}
		}
		__syncthreads();
	}
	// epilogue: cmpMats' returns (matcmp.c:478-493) and cmpMatThrd's stores
#pragma unroll
	for(int u = 0; u < 2; ++u)
#pragma unroll
		for(int v = 0; v < 2; ++v) {
			const int i = i0 + ti + 16 * u, j = j0 + tj + 16 * v;
			if(i >= a.n || j >= i) continue;
			const long long f = (long long) i * (i - 1) / 2 + j;
			const int l1 = a.len1[i], l2 = a.len2[j];
			double dist, nt;
			if(l2 > l1) {
				// early -1: the total of sample j's row number l1 + 1
				dist = -1;
				nt = (double) (unsigned) a.rec2[(long long) j * a.stride2 + l1].w;
			} else {
				const unsigned nn = a.nnucs[j];   // nNucs of sample j (k_kma_nnucs)
				const unsigned ri = (unsigned) inc[u][v];
				if(nn < a.minLength || nn < a.minCov * (unsigned) l2) {
					atomicMin(a.fatal, (unsigned long long) f);
					dist = -2;
					nt = 0;
				} else if(ri < a.minLength || ri < a.minCov * (unsigned) l2) {
					dist = -1;
					nt = 0;
				} else {
					dist = a.norm ? acc[u][v] / ri * a.norm : acc[u][v];
					nt = ri;
				}
			}
			D[f] = Elem<ET>::put(dist, 0.5, a.bs);
			if(N) N[f] = Elem<ET>::put(nt, 0.5, a.bs);
		}
}

// ------------------------------------------------------------------ host
template <int M>
static void launch_et(int et, unsigned grid, hipStream_t st, const KmaDev &k, void *D, void *N) {
	switch(et) {
		case 8: k_kma_pairs<M, 8><<<grid, KTB, 0, st>>>(k, (double *) D, (double *) N); break;
		case 4: k_kma_pairs<M, 4><<<grid, KTB, 0, st>>>(k, (float *) D, (float *) N); break;
		case 2: k_kma_pairs<M, 2><<<grid, KTB, 0, st>>>(k, (uint16_t *) D, (uint16_t *) N); break;
		default: k_kma_pairs<M, 1><<<grid, KTB, 0, st>>>(k, (uint8_t *) D, (uint8_t *) N); break;
	}
}

static int kma_launch(int metric, int et, unsigned grid, hipStream_t st, const KmaDev &k, void *D, void *N) {
	switch(metric) {
		case CCG_KMA_COS: launch_et<CCG_KMA_COS>(et, grid, st, k, D, N); break;
		case CCG_KMA_CHI2: launch_et<CCG_KMA_CHI2>(et, grid, st, k, D, N); break;
		case CCG_KMA_NCHI2: launch_et<CCG_KMA_NCHI2>(et, grid, st, k, D, N); break;
		case CCG_KMA_NC: launch_et<CCG_KMA_NC>(et, grid, st, k, D, N); break;
		case CCG_KMA_C: launch_et<CCG_KMA_C>(et, grid, st, k, D, N); break;
		case CCG_KMA_NBC: launch_et<CCG_KMA_NBC>(et, grid, st, k, D, N); break;
		case CCG_KMA_BC: launch_et<CCG_KMA_BC>(et, grid, st, k, D, N); break;
		case CCG_KMA_NL1: launch_et<CCG_KMA_NL1>(et, grid, st, k, D, N); break;
		case CCG_KMA_NL2: launch_et<CCG_KMA_NL2>(et, grid, st, k, D, N); break;
		case CCG_KMA_NLINF: launch_et<CCG_KMA_NLINF>(et, grid, st, k, D, N); break;
		case CCG_KMA_L1: launch_et<CCG_KMA_L1>(et, grid, st, k, D, N); break;
		case CCG_KMA_L2: launch_et<CCG_KMA_L2>(et, grid, st, k, D, N); break;
		case CCG_KMA_LINF: launch_et<CCG_KMA_LINF>(et, grid, st, k, D, N); break;
		case CCG_KMA_LN: launch_et<CCG_KMA_LN>(et, grid, st, k, D, N); break;
		case CCG_KMA_NLN: launch_et<CCG_KMA_NLN>(et, grid, st, k, D, N); break;
		default: return CCG_EUNSUP;
	}
	return CCG_OK;
}

static bool kma_metric_ok(int m) {
	return m == CCG_KMA_COS || m == CCG_KMA_CHI2 || m == CCG_KMA_NCHI2 || m == CCG_KMA_NC || m == CCG_KMA_C ||
	       m == CCG_KMA_NBC || m == CCG_KMA_BC || (m >= CCG_KMA_NL1 && m <= CCG_KMA_NLN);
}

static int kma_check(const ccg_kma_args *a) {
	if(!a || a->n < 0 || a->stride1 < 0 || a->stride2 < 0) return CCG_EINVAL;
	if(a->etype != 8 && a->etype != 4 && a->etype != 2 && a->etype != 1) return CCG_EINVAL;
	if((a->etype == 2 || a->etype == 1) && !(a->byteScale != 0)) return CCG_EINVAL;
	if(!kma_metric_ok(a->metric)) return CCG_EUNSUP;
	if((a->metric == CCG_KMA_LN || a->metric == CCG_KMA_NLN) && a->lnorm == 0) return CCG_EINVAL;
	return CCG_OK;
}

// device pointers throughout
static int kma_run(ccg_ctx *c, const ccg_kma_args *a, void *D, void *N, int64_t *fatal) {
	hipStream_t st = c->stream;
	const int n = a->n;
	if(fatal) *fatal = -1;
	if(n < 2) return CCG_OK;
	const long long rows1 = (long long) n * a->stride1, rows2 = (long long) n * a->stride2;
	double *s = NULL;
	unsigned long long *fat = NULL;
	int rc = CCG_OK;
	const bool cos = a->metric == CCG_KMA_COS;
	if(hipMalloc((void **) &fat, 8 + (size_t) n * 4) != hipSuccess ||
	   (cos && hipMalloc((void **) &s, (size_t) (rows1 + rows2 + 1) * 8) != hipSuccess)) {
		rc = CCG_ENOMEM;
	} else {
		KmaDev k;
		k.rec1 = (const uint4 *) a->rec1;
		k.rec2 = (const uint4 *) a->rec2;
		k.s1 = s;
		k.s2 = s ? s + rows1 : NULL;
		k.len1 = a->len1;
		k.len2 = a->len2;
		k.stride1 = a->stride1;
		k.stride2 = a->stride2;
		k.n = n;
		k.minDepth = a->minDepth;
		k.minLength = a->minLength;
		k.norm = a->norm;
		k.ln = a->lnorm;
		k.minCov = a->minCov;
		k.bs = a->byteScale;
		k.fatal = fat;
		k.nnucs = (const unsigned *) (fat + 1);
		unsigned long long none = ~0ull;
		if(hipMemcpyAsync(fat, &none, 8, hipMemcpyHostToDevice, st) != hipSuccess) rc = CCG_EHIP;
		if(!rc) k_kma_nnucs<<<n, 256, 0, st>>>(k.rec2, a->len2, a->stride2, a->minDepth, (unsigned *) (fat + 1));
		if(!rc && cos) {
			k_kma_norms<<<2048, 256, 0, st>>>(k.rec1, rows1, s);
			k_kma_norms<<<2048, 256, 0, st>>>(k.rec2, rows2, s + rows1);
		}
		const long long nb = (n + KT - 1) / KT, tiles = nb * (nb + 1) / 2;
		if(!rc) rc = kma_launch(a->metric, a->etype, (unsigned) tiles, st, k, D, N);
		if(!rc && hipGetLastError() != hipSuccess) rc = CCG_EHIP;
		if(!rc) {
			unsigned long long h = 0;
			if(hipMemcpyAsync(&h, fat, 8, hipMemcpyDeviceToHost, st) != hipSuccess ||
			   hipStreamSynchronize(st) != hipSuccess) {
				rc = CCG_EHIP;
			} else if(fatal) {
				*fatal = h == ~0ull ? -1 : (int64_t) h;
			}
		}
	}
	hipStreamSynchronize(st);
	if(s) hipFree(s);
	if(fat) hipFree(fat);
	return rc;
}

extern "C" {

int ccg_kma_ltd_dev(ccg_ctx *c, const ccg_kma_args *a, void *D, void *N, int64_t *fatal) {
	int rc = kma_check(a);
	if(rc) return rc;
	if(!c || (a->n > 1 && (!D || !a->rec1 || !a->rec2 || !a->len1 || !a->len2))) return CCG_EINVAL;
	CCG_CHECK(hipSetDevice(c->device));
	CCG_DEVICE_SYNC(c);   // inputs may come from other streams (e.g. torch's)
	return kma_run(c, a, D, N, fatal);
}

int ccg_kma_ltd(ccg_ctx *c, const ccg_kma_args *a, void *D, void *N, int64_t *fatal) {
	int rc = kma_check(a);
	if(rc) return rc;
	if(!c || (a->n > 1 && (!D || !a->rec1 || !a->rec2 || !a->len1 || !a->len2))) return CCG_EINVAL;
	if(fatal) *fatal = -1;
	if(a->n < 2) return CCG_OK;
	CCG_CHECK(hipSetDevice(c->device));
	const size_t n = (size_t) a->n, b1 = n * (size_t) a->stride1 * 16, b2 = n * (size_t) a->stride2 * 16;
	const size_t lt = n * (n - 1) / 2 * (size_t) a->etype;
	char *m = NULL;
	const size_t sz = b1 + b2 + 2 * n * 4 + 2 * lt + 64;
	if(hipMalloc((void **) &m, sz) != hipSuccess) return CCG_ENOMEM;
	ccg_kma_args d = *a;
	char *p = m;
	d.rec1 = (const uint16_t *) p;
	p += (b1 + 15) & ~(size_t) 15;
	d.rec2 = (const uint16_t *) p;
	p += (b2 + 15) & ~(size_t) 15;
	d.len1 = (const int32_t *) p;
	p += n * 4;
	d.len2 = (const int32_t *) p;
	p += n * 4;
	p = (char *) (((uintptr_t) p + 15) & ~(uintptr_t) 15);
	void *dD = p, *dN = N ? p + lt : NULL;
	hipStream_t st = c->stream;
	if(hipMemcpyAsync((void *) d.rec1, a->rec1, b1, hipMemcpyHostToDevice, st) != hipSuccess ||
	   hipMemcpyAsync((void *) d.rec2, a->rec2, b2, hipMemcpyHostToDevice, st) != hipSuccess ||
	   hipMemcpyAsync((void *) d.len1, a->len1, n * 4, hipMemcpyHostToDevice, st) != hipSuccess ||
	   hipMemcpyAsync((void *) d.len2, a->len2, n * 4, hipMemcpyHostToDevice, st) != hipSuccess) {
		rc = CCG_EHIP;
	} else {
		rc = kma_run(c, &d, dD, dN, fatal);
	}
	if(!rc && (hipMemcpyAsync(D, dD, lt, hipMemcpyDeviceToHost, st) != hipSuccess ||
	           (N && hipMemcpyAsync(N, dN, lt, hipMemcpyDeviceToHost, st) != hipSuccess) ||
	           hipStreamSynchronize(st) != hipSuccess)) {
		rc = CCG_EHIP;
	}
	hipStreamSynchronize(st);
	hipFree(m);
	return rc;
}

}   // extern "C"
