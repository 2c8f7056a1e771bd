// The fp4 MFMA issue ceiling with the dist kernel's shape (DESIGN.md "dist"):
// 16 independent 32x32 accumulators per wave (a wave's 128x128 quadrant), one
// wave per SIMD, operands in registers, and NV independent 32-bit VALU ops
// placed after every MFMA (sched_group_barrier), as k_snp_mfma3 places its
// plane-to-fp4 spreads.  Prints, per NV, the shader cycles per MFMA
// (s_memtime on one wave) and the chip's MAC rate, so the VALU a wave can
// hide under its own MFMAs is measured rather than assumed.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/micro/mfma_valu tools/micro/mfma_valu.hip
//   tools/micro/mfma_valu
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));

#define FMT_FP4 4
#define SCALE_ONE 127

#define CK(x)                                                                   \
	do {                                                                        \
		hipError_t e_ = (x);                                                    \
		if(e_ != hipSuccess) {                                                  \
			fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));             \
			exit(1);                                                            \
		}                                                                       \
	} while(0)

template <int NV>
__global__ __launch_bounds__(256, 1) void k_mix(int iters, float *sink, unsigned *vsink, unsigned long long *cyc) {
	v8i A[4], B[4];
	for(int t = 0; t < 4; ++t)
		for(int r = 0; r < 8; ++r) {
			A[t][r] = 0x22222222 ^ (threadIdx.x * 0x01010101 * (r + t));
			B[t][r] = 0x2a2a2a2a ^ (threadIdx.x * 0x10101010 * (r + 3 * t));
		}
	unsigned x[8];
	for(int k = 0; k < 8; ++k) x[k] = threadIdx.x * (k + 1);
	const unsigned c = 0x88888888u ^ blockIdx.x;
	v16f acc[16];
	for(int t = 0; t < 16; ++t) acc[t] = v16f{};
	const unsigned long long t0 = __builtin_readcyclecounter();
	for(int i = 0; i < iters; ++i) {
#pragma unroll
		for(int t = 0; t < 16; ++t) {
			acc[t] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(A[t & 3], B[t >> 2], acc[t], FMT_FP4, FMT_FP4, 0,
			                                                         SCALE_ONE, 0, SCALE_ONE);
#pragma unroll
			for(int v = 0; v < NV; ++v) {
				const int k = (t * NV + v) & 7;
				x[k] = __builtin_amdgcn_bitop3_b32(x[k], x[(k + 3) & 7], c, 0xBE);
			}
		}
#pragma unroll
		for(int t = 0; t < 16; ++t) {
			__builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
			if(NV) __builtin_amdgcn_sched_group_barrier(0x002, NV, 0);
		}
	}
	const unsigned long long t1 = __builtin_readcyclecounter();
	float s = 0;
	for(int t = 0; t < 16; ++t)
		for(int r = 0; r < 16; ++r) s += acc[t][r];
	unsigned xs = 0;
	for(int k = 0; k < 8; ++k) xs ^= x[k];
	if(s == 1234.5f) sink[threadIdx.x] = s;
	if(xs == 0x12345u) vsink[threadIdx.x] = xs;
	if(blockIdx.x == 0 && threadIdx.x == 0) *cyc = t1 - t0;
}

template <int NV>
static void run(int cus, float *sink, unsigned *vsink, unsigned long long *dcyc) {
	const int iters = 200000;   // ~60-160 ms per launch: the clock the chip sustains, not its first millisecond
	k_mix<NV><<<cus, 256>>>(50, sink, vsink, dcyc);
	CK(hipDeviceSynchronize());
	hipEvent_t e0, e1;
	CK(hipEventCreate(&e0));
	CK(hipEventCreate(&e1));
	CK(hipEventRecord(e0));
	k_mix<NV><<<cus, 256>>>(iters, sink, vsink, dcyc);
	CK(hipEventRecord(e1));
	CK(hipEventSynchronize(e1));
	float ms;
	CK(hipEventElapsedTime(&ms, e0, e1));
	unsigned long long cyc;
	CK(hipMemcpy(&cyc, dcyc, sizeof cyc, hipMemcpyDeviceToHost));
	const double mfmas = (double) iters * 16;
	const double macs = (double) cus * 4 * mfmas * 32.0 * 32 * 64;
	printf("NV %2d: %.3f ms, %.1f cycles per MFMA (s_memtime, wave 0), %.3e MAC/s = %.3f of the 5e15 dense peak, "
	       "clock %.2f GHz\n",
	       NV, ms, cyc / mfmas, macs / (ms * 1e-3), macs / (ms * 1e-3) / 5e15, cyc / (ms * 1e-3) / 1e9);
	CK(hipEventDestroy(e0));
	CK(hipEventDestroy(e1));
}

int main() {
	hipDeviceProp_t p;
	CK(hipGetDeviceProperties(&p, 0));
	const int cus = p.multiProcessorCount;
	float *sink;
	unsigned *vsink;
	unsigned long long *dcyc;
	CK(hipMalloc(&sink, 4096));
	CK(hipMalloc(&vsink, 4096));
	CK(hipMalloc(&dcyc, 8));
	printf("%d CUs, 1 block of 4 waves per CU, 16 accumulators per wave\n", cus);
	run<0>(cus, sink, vsink, dcyc);
	run<2>(cus, sink, vsink, dcyc);
	run<3>(cus, sink, vsink, dcyc);
	run<4>(cus, sink, vsink, dcyc);
	run<5>(cus, sink, vsink, dcyc);
	run<6>(cus, sink, vsink, dcyc);
	run<7>(cus, sink, vsink, dcyc);
	run<8>(cus, sink, vsink, dcyc);
	run<10>(cus, sink, vsink, dcyc);
	run<12>(cus, sink, vsink, dcyc);
	run<16>(cus, sink, vsink, dcyc);
	return 0;
}
