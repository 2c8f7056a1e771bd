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

struct ccg_ctx {
	int device;
	hipStream_t stream;
	hipEvent_t ev0, ev1;
	char name[256];
};

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
// (q, idx) candidates: smaller q wins, equal q -> larger idx wins.  This is
// the closed form of the reference's sequential `q <= min` last-wins scans.
struct QArg {
	double q;
	int idx;
};

__device__ __forceinline__ bool qarg_better(double q, int idx, double bq, int bidx) {
	return q < bq || (q == bq && idx > bidx);
}

__device__ __forceinline__ void qarg_wave_reduce(double &q, int &idx) {
#pragma unroll
	for(int off = 32; off > 0; off >>= 1) {
		double oq = __shfl_xor(q, off, 64);
		int oi = __shfl_xor(idx, off, 64);
		if(qarg_better(oq, oi, q, idx)) {
			q = oq;
			idx = oi;
		}
	}
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
