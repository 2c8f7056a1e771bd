// Calibration of the per-join cost model (development aid):
//   kernel A writes a pointer chain; kernel B (grid G) follows K dependent
//   links from block 0 wave 0 (others exit or do the same) and writes the end.
// Run under rocprofv3 --kernel-trace; durations of k_chase<K> give
// fixed cost + K x round-trip for data written by the previous kernel.
#include <hip/hip_runtime.h>
#include <stdio.h>
#pragma clang diagnostic ignored "-Wunused-value"

__global__ void k_write(int *chain, int n, int salt) {
	int i = blockIdx.x * blockDim.x + threadIdx.x;
	if(i < n) chain[i] = (int) (((long long) i * 7919 + 104729 + salt) % n);
}

template <int K>
__global__ void k_chase(const int *chain, int *out, int all, int base) {
	if(!all && blockIdx.x != 0) return;
	int p = (blockIdx.x * 97 + threadIdx.x) & 1023;
#pragma unroll 1
	for(int k = 0; k < K; ++k) p = chain[base + (p & 1023) * 64 + (threadIdx.x & 63)];
	if(threadIdx.x == 0) out[blockIdx.x] = p;
}

__global__ void k_empty(int *out) {
	if(threadIdx.x == 0 && blockIdx.x == 0) out[0] = 1;
}

int main() {
	const int n = 1 << 22;
	int *chain, *out;
	hipMalloc(&chain, n * 4);
	hipMalloc(&out, 4096 * 4);
	for(int rep = 0; rep < 200; ++rep) {
		for(int all = 0; all < 2; ++all) {
			int g = all ? 640 : 640;
			k_write<<<n / 256, 256>>>(chain, n, rep);
			k_empty<<<g, 256>>>(out);
			k_chase<0><<<g, 256>>>(chain, out, all, 0);
			k_chase<1><<<g, 256>>>(chain, out, all, 1 << 16);
			k_chase<2><<<g, 256>>>(chain, out, all, 2 << 16);
			k_chase<4><<<g, 256>>>(chain, out, all, 3 << 16);
			k_chase<8><<<g, 256>>>(chain, out, all, 4 << 16);
			k_chase<16><<<g, 256>>>(chain, out, all, 5 << 16);
			k_chase<16><<<g, 256>>>(chain, out, all, 5 << 16);   // L2-warm repeat
		}
	}
	hipDeviceSynchronize();
	printf("done\n");
	return 0;
}
