// Calibration: per-launch cost of back-to-back kernels on one stream, timed
// with HIP events (no profiler): empty kernels vs grid/block size, and a
// chain where each kernel reads what the previous one wrote (development aid).
#include <hip/hip_runtime.h>
#include <stdio.h>
#pragma clang diagnostic ignored "-Wunused-value"

template <int BS>
__global__ __launch_bounds__(BS) void k_empty(int *out, int g) {
	if(threadIdx.x == 0 && blockIdx.x == 0) out[0] = g;
}

// block 0 reads K dependent values written by the previous launch, every
// block reads one value, block 0 writes the next
template <int BS, int K>
__global__ __launch_bounds__(BS) void k_dep(int *buf, int it) {
	const int *src = buf + (it & 1) * 4096;
	int *dst = buf + ((it + 1) & 1) * 4096;
	int p = src[threadIdx.x & 63];
	if(blockIdx.x == 0) {
#pragma unroll 1
		for(int k = 1; k < K; ++k) p = src[(p + k) & 4095];
		if(threadIdx.x < 64) dst[threadIdx.x] = (p + threadIdx.x) & 4095;
	} else if(p == -12345) {
		dst[0] = 0;
	}
}

static float time_it(hipStream_t st, hipEvent_t a, hipEvent_t b, int reps, void (*f)(hipStream_t, int)) {
	for(int r = 0; r < 20; ++r) f(st, r);
	hipEventRecord(a, st);
	for(int r = 0; r < reps; ++r) f(st, r);
	hipEventRecord(b, st);
	hipEventSynchronize(b);
	float ms;
	hipEventElapsedTime(&ms, a, b);
	return ms * 1000.0f / reps;
}

// the same sequence captured once in a hipGraph and replayed (no host submission cost)
static float time_graph(hipStream_t st, hipEvent_t a, hipEvent_t b, int reps, void (*f)(hipStream_t, int)) {
	hipGraph_t g;
	hipGraphExec_t ge;
	hipStreamBeginCapture(st, hipStreamCaptureModeGlobal);
	for(int r = 0; r < reps; ++r) f(st, r);
	hipStreamEndCapture(st, &g);
	hipGraphInstantiate(&ge, g, NULL, NULL, 0);
	hipGraphLaunch(ge, st);
	hipEventRecord(a, st);
	hipGraphLaunch(ge, st);
	hipEventRecord(b, st);
	hipEventSynchronize(b);
	float ms;
	hipEventElapsedTime(&ms, a, b);
	hipGraphExecDestroy(ge);
	hipGraphDestroy(g);
	return ms * 1000.0f / reps;
}

static int *g_out;
static int g_grid;
template <int BS> void launch_empty(hipStream_t st, int) { k_empty<BS><<<g_grid, BS, 0, st>>>(g_out, g_grid); }
template <int BS, int K> void launch_dep(hipStream_t st, int r) { k_dep<BS, K><<<g_grid, BS, 0, st>>>(g_out, r); }

int main() {
	hipMalloc(&g_out, 3 * 4096 * 4);
	hipMemset(g_out, 0, 3 * 4096 * 4);
	hipStream_t st;
	hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
	hipEvent_t a, b;
	hipEventCreate(&a);
	hipEventCreate(&b);
	const int grids[] = {1, 64, 256, 640, 1024, 4096};
	for(int g : grids) {
		g_grid = g;
		printf("graph grid %5d: empty256 %6.2f  dep256(K=1) %6.2f  dep256(K=4) %6.2f  dep256(K=16) %6.2f  dep256(K=64) %6.2f us/launch\n",
		       g, time_graph(st, a, b, 500, launch_empty<256>), time_graph(st, a, b, 500, launch_dep<256, 1>),
		       time_graph(st, a, b, 500, launch_dep<256, 4>), time_graph(st, a, b, 500, launch_dep<256, 16>),
		       time_graph(st, a, b, 500, launch_dep<256, 64>));
	}
	for(int g : grids) {
		g_grid = g;
		printf("grid %5d: empty64 %6.2f  empty256 %6.2f  empty1024 %6.2f  dep256(K=1) %6.2f  dep256(K=4) %6.2f  dep256(K=16) %6.2f us/launch\n",
		       g, time_it(st, a, b, 2000, launch_empty<64>), time_it(st, a, b, 2000, launch_empty<256>),
		       time_it(st, a, b, 2000, launch_empty<1024>), time_it(st, a, b, 2000, launch_dep<256, 1>),
		       time_it(st, a, b, 2000, launch_dep<256, 4>), time_it(st, a, b, 2000, launch_dep<256, 16>));
	}
	return 0;
}
