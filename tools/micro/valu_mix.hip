// Calibration: issue rate of each instruction of the SNP dist inner loop on
// gfx950, from registers (development aid; DESIGN.md 5 "dist roofline").
// One word pair of k_snp_tile costs v_xor_b32, v_bitop3_b32 (table 0xBE,
// (a^b)|c) and v_bcnt_u32_b32 with accumulate.  Each kernel runs CH
// independent chains per lane of ONE instruction kind (or of the 3-op mix),
// with inline asm so that nothing is hoisted or fused, and reports
// instruction-lanes/s against the nominal 256 CU x 4 SIMD x 32 lanes x
// 2.4 GHz = 7.86e13 (a wave64 instruction every 2 cycles per SIMD).
#include <hip/hip_runtime.h>
#include <stdio.h>

#define CH 16

template <int OP>
__global__ __launch_bounds__(256) void k_rate(const unsigned *seed, int iters, unsigned *out) {
	unsigned x[CH], y[CH], z[CH];
#pragma unroll
	for(int c = 0; c < CH; ++c) {
		x[c] = seed[(threadIdx.x + c) & 255];
		y[c] = seed[(threadIdx.x * 3 + c + 1) & 255];
		z[c] = seed[(threadIdx.x * 5 + c + 2) & 255];
	}
	for(int it = 0; it < iters; ++it) {
#pragma unroll
		for(int c = 0; c < CH; ++c) {
			if(OP == 0) {   // v_xor_b32
				asm volatile("v_xor_b32 %0, %1, %0" : "+v"(x[c]) : "v"(y[c]));
			} else if(OP == 1) {   // v_bitop3_b32 (a^b)|c
				asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0xbe" : "+v"(x[c]) : "v"(y[c]), "v"(z[c]));
			} else if(OP == 2) {   // v_bcnt_u32_b32 with accumulate
				asm volatile("v_bcnt_u32_b32 %0, %1, %0" : "+v"(x[c]) : "v"(y[c]));
			} else if(OP == 3) {   // v_or_b32 (VOP2, for comparison with bitop3)
				asm volatile("v_or_b32 %0, %1, %0" : "+v"(x[c]) : "v"(y[c]));
			} else {   // the word-pair mix: t = a ^ b; t = (c ^ d) | t; acc += bcnt(t)
				unsigned t;
				asm volatile("v_xor_b32 %0, %1, %2" : "=v"(t) : "v"(y[c]), "v"(z[c]));
				asm volatile("v_bitop3_b32 %0, %1, %2, %0 bitop3:0xbe" : "+v"(t) : "v"(z[c]), "v"(y[c]));
				asm volatile("v_bcnt_u32_b32 %0, %1, %0" : "+v"(x[c]) : "v"(t));
			}
		}
	}
	unsigned s = 0;
#pragma unroll
	for(int c = 0; c < CH; ++c) s += x[c];
	out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int OP>
static void run(const char *name, const unsigned *seed, unsigned *out, int blocks, int iters, int ops_per) {
	hipEvent_t a, b;
	hipEventCreate(&a);
	hipEventCreate(&b);
	k_rate<OP><<<blocks, 256>>>(seed, 10, out);
	hipEventRecord(a);
	k_rate<OP><<<blocks, 256>>>(seed, iters, out);
	hipEventRecord(b);
	hipEventSynchronize(b);
	float ms;
	hipEventElapsedTime(&ms, a, b);
	const double lane_ops = (double) blocks * 256 * iters * CH * ops_per;
	const double rate = lane_ops / (ms * 1e-3);
	printf("%-26s blocks %5d: %.3e instruction-lanes/s = %5.1f%% of nominal 7.86e13; %.2f cycles per wave64 "
	       "instruction per SIMD at 2.4 GHz\n",
	       name, blocks, rate, 100.0 * rate / 7.86432e13, 2.0 * 7.86432e13 / rate);
	hipEventDestroy(a);
	hipEventDestroy(b);
}

int main() {
	unsigned *seed, *out;
	hipMalloc(&seed, 256 * 4);
	hipMemset(seed, 0x5a, 256 * 4);
	hipMalloc(&out, 8192 * 256 * 4);
	const int iters = 20000;
	for(int blocks : {1024, 2048}) {
		run<0>("v_xor_b32", seed, out, blocks, iters, 1);
		run<3>("v_or_b32", seed, out, blocks, iters, 1);
		run<1>("v_bitop3_b32", seed, out, blocks, iters, 1);
		run<2>("v_bcnt_u32_b32 (acc)", seed, out, blocks, iters, 1);
		run<4>("mix xor+bitop3+bcnt", seed, out, blocks, iters, 3);
	}
	hipFree(seed);
	hipFree(out);
	return 0;
}
