// ccg_internal.h -- shared device helpers of the gfx950 engine.
//
// Element types follow the reference LT container (matrix.c:59-71) and its
// ByteScale conversions (bytescale.h:22-23): dtouc(v, r) = v*BS + r stored
// through x86's 32-bit truncating conversion, uctod(u) = u / BS.
// Everything is compiled with -ffp-contract=off so that expressions like
// ((Ni + Nj - 4) >> 1) * d - sDi - sDj round exactly as the reference's.
#pragma once
#pragma clang diagnostic ignored "-Wunused-result"
#pragma clang diagnostic ignored "-Wunused-value"
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <float.h>
#include "ccphylo_amd.h"

#define CCG_CHECK(expr)                                                        \
	do {                                                                       \
		hipError_t e_ = (expr);                                                \
		if(e_ != hipSuccess) {                                                 \
			ccg_set_last_error(e_, #expr, __FILE__, __LINE__);                 \
			return e_ == hipErrorOutOfMemory ? CCG_ENOMEM : CCG_EHIP;          \
		}                                                                      \
	} while(0)

void ccg_set_last_error(hipError_t e, const char *what, const char *file, int line);
// free-form text for ccg_strerror(CCG_EHIP) (collective transports)
void ccg_set_last_msg(const char *msg);

struct ccg_ctx {
	int device;
	hipStream_t stream;
	hipEvent_t ev0, ev1;
	char name[256];
	float dist_ms;   // the last dist call's pair kernels (HIP events on the engine stream)
	int flags;       // CCG_CTX_* (ccg_ctx_configure)
	int masked;      // the stream was created with a CU mask (ccg_ctx_configure)
	int ncu, cus;    // the device's CUs; the CUs the stream may use (0: all)
	// device workspaces kept across runs (grown on demand, freed by
	// ccg_destroy): slots 0 / 1 the tree's, slot 2 the dist's bit planes in a
	// CCG_CTX_NOSYNC context.  A run then makes no hipFree, which waits for
	// every stream of the device, so such a context never waits for another
	void *ws[3];
	size_t ws_bytes[3];
};
// slot k of the context's workspace cache, at least `bytes` long
int ccg_ctx_workspace(ccg_ctx *c, int k, size_t bytes, void **p);
// every device-pointer entry point first waits for the whole device (inputs
// may come from other streams) unless the caller orders them itself
#define CCG_DEVICE_SYNC(c) \
	do { \
		if(!((c)->flags & CCG_CTX_NOSYNC)) CCG_CHECK(hipDeviceSynchronize()); \
	} while(0)

// ---------------------------------------------------------------- numerics
__device__ __forceinline__ int32_t cvt_i32_x86(double x) {
	// cvttsd2si: INT_MIN on overflow / NaN (the GPU instruction saturates)
	if(!(x > -2147483649.0 && x < 2147483648.0)) {
		return INT32_MIN;
	}
	return (int32_t) x;
}

template <int ET> struct Elem;
template <> struct Elem<8> {
	typedef double T;
	static __device__ __forceinline__ double get(T v, double) { return v; }
	static __device__ __forceinline__ T put(double v, double, double) { return v; }
};
template <> struct Elem<4> {
	typedef float T;
	static __device__ __forceinline__ double get(T v, double) { return (double) v; }
	static __device__ __forceinline__ T put(double v, double, double) { return (float) v; }
};
template <> struct Elem<2> {
	typedef uint16_t T;
	static __device__ __forceinline__ double get(T v, double bs) { return v / bs; }
	static __device__ __forceinline__ T put(double v, double r, double bs) {
		return (uint16_t) cvt_i32_x86(v * bs + r);
	}
};
template <> struct Elem<1> {
	typedef uint8_t T;
	static __device__ __forceinline__ double get(T v, double bs) { return v / bs; }
	static __device__ __forceinline__ T put(double v, double r, double bs) {
		return (uint8_t) cvt_i32_x86(v * bs + r);
	}
};

__host__ __device__ __forceinline__ int64_t tri(int64_t i) { return i * (i - 1) / 2; }

// Q criterion exactly as nj.c:227 / dnj.c:103 write it
__device__ __forceinline__ double qcrit(int Ni, int Nj, double d, double sDi, double sDj) {
	double q = (double) ((Ni + Nj - 4) >> 1) * d;
	q = q - sDi;
	return q - sDj;
}

// ------------------------------------------------------------ reductions
// ------------------------------------------------------------ DPP wave ops
// Wave64 scans/reductions with DPP row shifts and row broadcasts (GFX9
// family): a few cycles per step instead of an LDS-crossbar ds_bpermute per
// __shfl.  Steps: row_shr 1,2,4,8 (inclusive within each 16-lane row), then
// row_bcast:15 into rows 1,3 and row_bcast:31 into rows 2,3; lanes without a
// source keep `old` (the identity).  Lane 63 ends with the whole wave.
#define DPP_ROW_SHR1 0x111
#define DPP_ROW_SHR2 0x112
#define DPP_ROW_SHR4 0x114
#define DPP_ROW_SHR8 0x118
#define DPP_WAVE_SHR1 0x138
#define DPP_ROW_BCAST15 0x142
#define DPP_ROW_BCAST31 0x143

template <int CTRL, int RM>
__device__ __forceinline__ int dpp_i(int old, int src) {
	return __builtin_amdgcn_update_dpp(old, src, CTRL, RM, 0xF, false);
}
template <int CTRL, int RM>
__device__ __forceinline__ double dpp_d(double old, double src) {
	const long long o = __double_as_longlong(old), v = __double_as_longlong(src);
	const int lo = __builtin_amdgcn_update_dpp((int) o, (int) v, CTRL, RM, 0xF, false);
	const int hi = __builtin_amdgcn_update_dpp((int) (o >> 32), (int) (v >> 32), CTRL, RM, 0xF, false);
	return __longlong_as_double(((long long) hi << 32) | (unsigned) lo);
}
template <int CTRL, int RM>
__device__ __forceinline__ long long dpp_l(long long old, long long src) {
	const int lo = __builtin_amdgcn_update_dpp((int) old, (int) src, CTRL, RM, 0xF, false);
	const int hi = __builtin_amdgcn_update_dpp((int) (old >> 32), (int) (src >> 32), CTRL, RM, 0xF, false);
	return ((long long) hi << 32) | (unsigned) lo;
}
__device__ __forceinline__ double readlane_d(double v, int lane) {
	const long long x = __double_as_longlong(v);
	const int lo = __builtin_amdgcn_readlane((int) x, lane), hi = __builtin_amdgcn_readlane((int) (x >> 32), lane);
	return __longlong_as_double(((long long) hi << 32) | (unsigned) lo);
}
__device__ __forceinline__ long long readlane_l(long long x, int lane) {
	const int lo = __builtin_amdgcn_readlane((int) x, lane), hi = __builtin_amdgcn_readlane((int) (x >> 32), lane);
	return ((long long) hi << 32) | (unsigned) lo;
}

#define CCG_DPP_STEPS(STEP)         \
	STEP(DPP_ROW_SHR1, 0xF)         \
	STEP(DPP_ROW_SHR2, 0xF)         \
	STEP(DPP_ROW_SHR4, 0xF)         \
	STEP(DPP_ROW_SHR8, 0xF)         \
	STEP(DPP_ROW_BCAST15, 0xA)      \
	STEP(DPP_ROW_BCAST31, 0xC)

// inclusive prefix sum over the wave
__device__ __forceinline__ int wave_incl_sum(int x) {
#define S_(C, R) x += dpp_i<C, R>(0, x);
	CCG_DPP_STEPS(S_)
#undef S_
	return x;
}
__device__ __forceinline__ long long wave_incl_sum_l(long long x) {
#define S_(C, R) x += dpp_l<C, R>(0, x);
	CCG_DPP_STEPS(S_)
#undef S_
	return x;
}
// inclusive prefix min over the wave
__device__ __forceinline__ double wave_incl_min(double x) {
#define S_(C, R)                               \
	{                                          \
		const double t_ = dpp_d<C, R>(DBL_MAX, x); \
		x = t_ < x ? t_ : x;                   \
	}
	CCG_DPP_STEPS(S_)
#undef S_
	return x;
}
__device__ __forceinline__ int wave_incl_min_i(int x) {
#define S_(C, R)                                 \
	{                                            \
		const int t_ = dpp_i<C, R>(INT32_MAX, x);  \
		x = t_ < x ? t_ : x;                     \
	}
	CCG_DPP_STEPS(S_)
#undef S_
	return x;
}
// exclusive prefix min: lane l gets min(carry, x[0..l-1])
__device__ __forceinline__ double wave_excl_min(double x, double carry) {
	const double inc = wave_incl_min(x);
	const double ex = dpp_d<DPP_WAVE_SHR1, 0xF>(DBL_MAX, inc);
	return ex < carry ? ex : carry;
}

// (q, idx) candidates: smaller q wins, equal q -> larger idx wins.  This is
// the closed form of the reference's sequential `q <= min` last-wins scans;
// being a total order, any association of the fold gives the same winner.
struct QArg {
	double q;
	int idx;
};

__device__ __forceinline__ bool qarg_better(double q, int idx, double bq, int bidx) {
	return q < bq || (q == bq && idx > bidx);
}

// wave-wide (q, idx) reduce; the result in every lane
__device__ __forceinline__ void qarg_wave_reduce(double &q, int &idx) {
#define S_(C, R)                                          \
	{                                                     \
		const double oq_ = dpp_d<C, R>(DBL_MAX, q);       \
		const int oi_ = dpp_i<C, R>(INT32_MIN, idx);      \
		if(qarg_better(oq_, oi_, q, idx)) {               \
			q = oq_;                                      \
			idx = oi_;                                    \
		}                                                 \
	}
	CCG_DPP_STEPS(S_)
#undef S_
	q = readlane_d(q, 63);
	idx = __builtin_amdgcn_readlane(idx, 63);
}

// the same, carrying a payload (cq, cp) of the winning element
__device__ __forceinline__ void qarg_wave_reduce_carry(double &q, int &idx, double &cq, int &cp) {
#define S_(C, R)                                          \
	{                                                     \
		const double oq_ = dpp_d<C, R>(DBL_MAX, q);       \
		const int oi_ = dpp_i<C, R>(INT32_MIN, idx);      \
		const double ocq_ = dpp_d<C, R>(DBL_MAX, cq);     \
		const int ocp_ = dpp_i<C, R>(0, cp);              \
		if(qarg_better(oq_, oi_, q, idx)) {               \
			q = oq_;                                      \
			idx = oi_;                                    \
			cq = ocq_;                                    \
			cp = ocp_;                                    \
		}                                                 \
	}
	CCG_DPP_STEPS(S_)
#undef S_
	q = readlane_d(q, 63);
	idx = __builtin_amdgcn_readlane(idx, 63);
	cq = readlane_d(cq, 63);
	cp = __builtin_amdgcn_readlane(cp, 63);
}

// four independent wave-wide (q, idx) reduces in lockstep (four dependency
// chains interleaved step by step), the second carrying a payload (cq, cp)
__device__ __forceinline__ void qarg_wave_reduce4(double (&q)[4], int (&idx)[4], double &cq, int &cp) {
#define S_(C, R)                                              \
	{                                                         \
		double oq_[4];                                        \
		int oi_[4];                                           \
		_Pragma("unroll") for(int t = 0; t < 4; ++t) {        \
			oq_[t] = dpp_d<C, R>(DBL_MAX, q[t]);              \
			oi_[t] = dpp_i<C, R>(INT32_MIN, idx[t]);          \
		}                                                     \
		const double ocq_ = dpp_d<C, R>(DBL_MAX, cq);         \
		const int ocp_ = dpp_i<C, R>(0, cp);                  \
		_Pragma("unroll") for(int t = 0; t < 4; ++t) {        \
			const bool b_ = qarg_better(oq_[t], oi_[t], q[t], idx[t]); \
			q[t] = b_ ? oq_[t] : q[t];                        \
			idx[t] = b_ ? oi_[t] : idx[t];                    \
			if(t == 1) {                                      \
				cq = b_ ? ocq_ : cq;                          \
				cp = b_ ? ocp_ : cp;                          \
			}                                                 \
		}                                                     \
	}
	CCG_DPP_STEPS(S_)
#undef S_
#pragma unroll
	for(int t = 0; t < 4; ++t) {
		q[t] = readlane_d(q[t], 63);
		idx[t] = __builtin_amdgcn_readlane(idx[t], 63);
	}
	cq = readlane_d(cq, 63);
	cp = __builtin_amdgcn_readlane(cp, 63);
}

// block-wide (q, idx) reduce; result valid in every thread.  `sq`/`si` are
// LDS scratch of blockDim/64 entries.
__device__ __forceinline__ void qarg_block_reduce(double &q, int &idx, double *sq, int *si) {
	qarg_wave_reduce(q, idx);
	const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
	__syncthreads();
	if(lane == 0) {
		sq[wid] = q;
		si[wid] = idx;
	}
	__syncthreads();
	q = sq[0];
	idx = si[0];
	for(int w = 1; w < nw; ++w) {
		if(qarg_better(sq[w], si[w], q, idx)) {
			q = sq[w];
			idx = si[w];
		}
	}
	__syncthreads();
}

// ---------------------------------------------------- in-kernel hand-offs
// Guideline 16 form R1: every handed-off byte is stored write-through (sc1)
// and loaded with sc1 loads by the consumer; each storing wave drains its
// stores (vmcnt(0)) before the workgroup barrier, then ONE lane takes an
// agent-scope ticket.  No release/acquire fences (an L2 write-back per block).
template <typename T>
__device__ __forceinline__ void st_wt(T *p, T v) {
	__hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T>
__device__ __forceinline__ T ld_wt(const T *p) {
	return __hip_atomic_load(const_cast<T *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// true in every thread of the last block to arrive
__device__ __forceinline__ bool last_block_arrive(unsigned *counter) {
	__shared__ int s_last;
	asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
	__syncthreads();
	if(threadIdx.x == 0) {
		unsigned t = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		s_last = (t == gridDim.x * gridDim.y - 1);
	}
	__syncthreads();
	return s_last;
}
