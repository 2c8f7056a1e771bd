// Calibration for a persistent DNJ join loop: the cost of one grid-wide
// barrier in a co-resident (cooperative) grid against a kernel boundary.
//   bar:   every block arrives (agent-scope atomic add), the last arriver bumps
//          the generation, the others poll it (bounded: a poll that gives up
//          sets an error flag and the grid exits, never a hang)
//   hand:  the same plus a phase handoff: block 0 writes a value before the
//          barrier, every block reads it after (the pattern a persistent
//          plan -> scan -> join -> requeue chain needs)
//   chain: a dependent kernel chain (one launch per phase, k_dep-like) for the
//          same number of phases, for comparison
// hipcc --offload-arch=gfx950 -O3 -o tools/micro/gridbar tools/micro/gridbar.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define SPIN_MAX (1 << 22)

struct Bar {
	unsigned *count;   // arrivals of the current generation
	unsigned *gen;     // generation
	int *err;
};

__device__ __forceinline__ bool grid_bar(const Bar &b, unsigned &g, unsigned nblk) {
	__syncthreads();
	bool ok = true;
	if(threadIdx.x == 0) {
		const unsigned want = g + 1;
		// release this block's writes, arrive
		const unsigned seen = __hip_atomic_fetch_add(b.count, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
		if(seen == nblk - 1) {
			__hip_atomic_store(b.count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
			__hip_atomic_store(b.gen, want, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
		} else {
			int spin = 0;
			while(__hip_atomic_load(b.gen, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) != want) {
				if(++spin > SPIN_MAX) {
					__hip_atomic_store(b.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
					ok = false;
					break;
				}
				__builtin_amdgcn_s_sleep(1);
			}
		}
		g = want;
	}
	__shared__ int s_ok;
	if(threadIdx.x == 0) s_ok = ok;
	__syncthreads();
	return s_ok;
}

__global__ __launch_bounds__(256) void k_bar(Bar b, int iters, int hand, int *val, int *out) {
	unsigned g = 0;
	int acc = 0;
	for(int it = 0; it < iters; ++it) {
		if(hand && blockIdx.x == 0 && threadIdx.x == 0) val[it & 1] = it;
		if(!grid_bar(b, g, gridDim.x)) return;
		if(__hip_atomic_load(b.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
		if(hand) acc += __hip_atomic_load(val + (it & 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
	}
	if(threadIdx.x == 0) out[blockIdx.x] = acc;
}

__global__ __launch_bounds__(256) void k_phase(int *val, int it) {
	const int v = val[it & 1];
	if(blockIdx.x == 0 && threadIdx.x == 0) val[(it + 1) & 1] = v + 1;
}

int main(int argc, char **argv) {
	int dev = 0;
	hipDeviceProp_t p;
	hipGetDeviceProperties(&p, dev);
	int per = 0;
	hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, (const void *) k_bar, 256, 0);
	printf("device %s, %d CUs, k_bar resident blocks per CU %d, cooperative %d\n", p.name, p.multiProcessorCount, per,
	       p.cooperativeLaunch);
	unsigned *cnt, *gen;
	int *err, *val, *out;
	hipMalloc(&cnt, 256);
	hipMalloc(&gen, 256);
	hipMalloc(&err, 256);
	hipMalloc(&val, 256);
	hipMalloc(&out, 4096 * 4);
	hipEvent_t a, z;
	hipEventCreate(&a);
	hipEventCreate(&z);
	hipStream_t st;
	hipStreamCreate(&st);
	const int iters = 20000;
	for(int nb : {64, 128, 256, 512}) {
		if(nb > per * p.multiProcessorCount) continue;
		for(int hand = 0; hand < 2; ++hand) {
			hipMemset(cnt, 0, 256);
			hipMemset(gen, 0, 256);
			hipMemset(err, 0, 256);
			Bar b{cnt, gen, err};
			int it = iters;
			void *args[] = {&b, &it, &hand, &val, &out};
			hipEventRecord(a, st);
			hipError_t e = hipLaunchCooperativeKernel((const void *) k_bar, dim3(nb), dim3(256), args, 0, st);
			hipEventRecord(z, st);
			hipEventSynchronize(z);
			float ms = 0;
			hipEventElapsedTime(&ms, a, z);
			int herr = 0;
			hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost);
			printf("grid barrier%s: %4d blocks x 256: %.3f us per barrier (launch %s, err %d)\n",
			       hand ? " + handoff" : "          ", nb, 1000.0 * ms / iters, hipGetErrorString(e), herr);
		}
	}
	for(int nb : {1, 64, 256, 1024}) {
		for(int r = 0; r < 100; ++r) k_phase<<<nb, 256, 0, st>>>(val, r);
		hipEventRecord(a, st);
		for(int r = 0; r < iters; ++r) k_phase<<<nb, 256, 0, st>>>(val, r);
		hipEventRecord(z, st);
		hipEventSynchronize(z);
		float ms = 0;
		hipEventElapsedTime(&ms, a, z);
		printf("kernel chain:          %4d blocks x 256: %.3f us per launch\n", nb, 1000.0 * ms / iters);
	}
	return 0;
}
