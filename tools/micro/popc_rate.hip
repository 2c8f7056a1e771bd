// Calibration: VALU throughput of the SNP inner-loop op mix (2 xor, or,
// bcnt-accumulate per word pair) from registers, at several occupancies
// (development aid).
#include <hip/hip_runtime.h>
#include <stdio.h>
#pragma clang diagnostic ignored "-Wunused-value"

template <int WAVES_HINT>
__global__ __launch_bounds__(256) void k_popc(const uint4 *seed, int iters, unsigned *out) {
	uint4 a[4], b[4];
#pragma unroll
	for(int q = 0; q < 4; ++q) {
		a[q] = seed[(threadIdx.x + q) & 63];
		b[q] = seed[(threadIdx.x + 7 * q + 1) & 63];
	}
	unsigned acc[8][8];
#pragma unroll
	for(int i = 0; i < 8; ++i)
#pragma unroll
		for(int j = 0; j < 8; ++j) acc[i][j] = 0;
	for(int it = 0; it < iters; ++it) {
#pragma unroll
		for(int qa = 0; qa < 4; ++qa) {
#pragma unroll
			for(int qb = 0; qb < 4; ++qb) {
				acc[2 * qa][2 * qb] += __popc((a[qa].x ^ b[qb].x) | (a[qa].y ^ b[qb].y));
				acc[2 * qa][2 * qb + 1] += __popc((a[qa].x ^ b[qb].z) | (a[qa].y ^ b[qb].w));
				acc[2 * qa + 1][2 * qb] += __popc((a[qa].z ^ b[qb].x) | (a[qa].w ^ b[qb].y));
				acc[2 * qa + 1][2 * qb + 1] += __popc((a[qa].z ^ b[qb].z) | (a[qa].w ^ b[qb].w));
			}
		}
		// perturb so the loop is not hoisted
#pragma unroll
		for(int q = 0; q < 4; ++q) {
			a[q].x += it;
			a[q].y ^= it;
			a[q].z += 3;
			a[q].w ^= it * 5;
		}
	}
	unsigned s = 0;
#pragma unroll
	for(int i = 0; i < 8; ++i)
#pragma unroll
		for(int j = 0; j < 8; ++j) s += acc[i][j];
	out[blockIdx.x * 256 + threadIdx.x] = s;
}

int main() {
	uint4 *seed;
	unsigned *out;
	hipMalloc(&seed, 64 * sizeof(uint4));
	hipMemset(seed, 0x5a, 64 * sizeof(uint4));
	hipMalloc(&out, 4096 * 256 * 4);
	hipEvent_t a, b;
	hipEventCreate(&a);
	hipEventCreate(&b);
	const int iters = 20000;
	for(int blocks : {256, 512, 1024, 2048, 4096}) {
		k_popc<1><<<blocks, 256>>>(seed, 100, out);
		hipEventRecord(a);
		k_popc<1><<<blocks, 256>>>(seed, iters, out);
		hipEventRecord(b);
		hipEventSynchronize(b);
		float ms;
		hipEventElapsedTime(&ms, a, b);
		double ops = (double) blocks * 256 * iters * 64 * 4;   // 64 pairs x 4 ops per iteration (+16 perturbation ops)
		printf("blocks %5d: %.3f ms, %.3e lane-ops/s (%.1f%% of 256 CU x 128 lanes x 2.4 GHz)\n", blocks, ms,
		       ops / (ms * 1e-3), 100.0 * ops / (ms * 1e-3) / (256.0 * 128 * 2.4e9));
	}
	return 0;
}
