// CU-masked streams on gfx950, with no torch and no engine in the process.
//
//   map LAYOUT K [WORDS]   launch 16384 one-wave blocks on a stream masked to
//                          K CUs (LAYOUT low: CUs 0..K-1; stride: every
//                          (256/K)-th; xcd: K/8 at the start of each 32-CU
//                          group), each block records s_getreg HW_ID and
//                          XCC_ID; prints the XCC / SE / CU slots that ran
//                          blocks and the time of a fixed spin workload.
//                          WORDS: the mask words handed to the runtime
//                          (default: enough for the highest CU; the engine's
//                          Device.configure passes the same).
//   destroy WORDS          create a masked stream (the first 64 CUs over WORDS
//                          words), run a kernel on it, destroy it, then run a
//                          kernel on a stream created before it, on a stream
//                          created after it and on the null stream
//   exit WORDS             create a masked stream, run on it, and return from
//                          main with the stream alive (runtime teardown)
//   engine WORDS POOL [MASK DESTROY PRIO TEARDOWN]
//                          the engine probe's stream sequence, then POOL
//                          streams as torch creates them (PRIO: alternating
//                          high / low priority), a kernel on each; MASK 0: a
//                          plain stream in the masked one's place; DESTROY 0:
//                          it stays; TEARDOWN 1: return from main with every
//                          stream alive
//
// hipcc --offload-arch=gfx950 -O3 -o tools/micro/cu_mask tools/micro/cu_mask.hip
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>
#include <set>
#include <map>

#define CK(x)                                                                                 \
	do {                                                                                      \
		hipError_t e_ = (x);                                                                  \
		if(e_ != hipSuccess) {                                                                \
			fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
			exit(2);                                                                          \
		}                                                                                     \
	} while(0)

// HW_ID (reg 4) and XCC_ID (reg 20), whole registers; vector stores only
__global__ __launch_bounds__(64) void k_where(unsigned *rec, int spin) {
	const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
	const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);
	long long t0 = __builtin_amdgcn_s_memrealtime();
	// a fixed amount of work per block: ~spin x 100 ns of wall on its CU
	while(__builtin_amdgcn_s_memrealtime() - t0 < spin) __builtin_amdgcn_s_sleep(2);
	if(threadIdx.x == 0) {
		rec[2 * blockIdx.x] = hw;
		rec[2 * blockIdx.x + 1] = xcc;
	}
}

__global__ void k_touch(int *p, int n) {
	const int i = blockIdx.x * blockDim.x + threadIdx.x;
	if(i < n) p[i] += 1;
}

static std::vector<uint32_t> mask_of(const char *layout, int k, int ncu, int words) {
	std::vector<int> cus;
	if(!strcmp(layout, "stride")) {
		const int step = ncu / k;
		for(int c = 0; c < ncu && (int) cus.size() < k; c += step) cus.push_back(c);
	} else if(!strcmp(layout, "xcd")) {
		const int per = k / 8 > 0 ? k / 8 : 1;
		for(int g = 0; g < 8; ++g)
			for(int i = 0; i < per; ++i) cus.push_back(g * (ncu / 8) + i);
	} else {
		for(int c = 0; c < k; ++c) cus.push_back(c);
	}
	int hi = 0;
	for(int c : cus) hi = c > hi ? c : hi;
	if(words <= 0) words = hi / 32 + 1;
	std::vector<uint32_t> m(words, 0u);
	for(int c : cus)
		if(c / 32 < words) m[c / 32] |= 1u << (c % 32);
	return m;
}

static int run_map(const char *layout, int k, int words) {
	hipDeviceProp_t p;
	CK(hipGetDeviceProperties(&p, 0));
	const int ncu = p.multiProcessorCount;
	std::vector<uint32_t> m = k >= ncu ? std::vector<uint32_t>() : mask_of(layout, k, ncu, words);
	hipStream_t s;
	if(m.empty()) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
	else CK(hipExtStreamCreateWithCUMask(&s, (uint32_t) m.size(), m.data()));
	const int nb = 16384;
	unsigned *d;
	CK(hipMalloc(&d, (size_t) nb * 8));
	CK(hipMemsetAsync(d, 0xff, (size_t) nb * 8, s));
	hipEvent_t e0, e1;
	CK(hipEventCreate(&e0));
	CK(hipEventCreate(&e1));
	k_where<<<nb, 64, 0, s>>>(d, 2000);   // warm
	CK(hipEventRecord(e0, s));
	k_where<<<nb, 64, 0, s>>>(d, 2000);   // 20 us per block
	CK(hipEventRecord(e1, s));
	CK(hipStreamSynchronize(s));
	float ms = 0;
	CK(hipEventElapsedTime(&ms, e0, e1));
	std::vector<unsigned> h((size_t) nb * 2);
	CK(hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost));
	std::map<unsigned, std::set<unsigned>> per_xcc;   // xcc -> {se:sh:cu}
	std::set<unsigned> slots;
	for(int b = 0; b < nb; ++b) {
		const unsigned hw = h[2 * b], xcc = h[2 * b + 1] & 0xf;
		const unsigned cu = (hw >> 8) & 0xf, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
		const unsigned key = (se << 5) | (sh << 4) | cu;
		per_xcc[xcc].insert(key);
		slots.insert((xcc << 8) | key);
	}
	printf("map %s k=%d words=%zu:", layout, k, m.size());
	for(size_t w = 0; w < m.size(); ++w) printf(" %08x", m[w]);
	printf("\n  distinct CU slots %zu over %zu XCCs; 16384 sleeping 20 us blocks in %.3f ms\n", slots.size(),
	       per_xcc.size(), ms);
	for(auto &x : per_xcc) {
		printf("  xcc %u: %zu CUs [", x.first, x.second.size());
		int c = 0;
		for(unsigned key : x.second) {
			if(c++) printf(" ");
			printf("%u.%u.%u", key >> 5, (key >> 4) & 1, key & 15);
		}
		printf("]\n");
	}
	CK(hipFree(d));
	CK(hipStreamDestroy(s));
	return 0;
}

static int run_destroy(int words, bool teardown) {
	std::vector<uint32_t> m(words, 0u);
	for(int c = 0; c < 64; ++c)
		if(c / 32 < words) m[c / 32] |= 1u << (c % 32);
	const int n = 1 << 20;
	int *d;
	CK(hipMalloc(&d, n * 4));
	CK(hipMemset(d, 0, n * 4));
	hipStream_t before;
	CK(hipStreamCreateWithFlags(&before, hipStreamNonBlocking));
	hipStream_t ms;
	CK(hipExtStreamCreateWithCUMask(&ms, (uint32_t) words, m.data()));
	k_touch<<<n / 256, 256, 0, ms>>>(d, n);
	CK(hipGetLastError());
	CK(hipStreamSynchronize(ms));
	printf("%s words=%d: kernel on the masked stream ok\n", teardown ? "exit" : "destroy", words);
	fflush(stdout);
	if(teardown) {
		printf("exit: returning from main with the masked stream alive\n");
		fflush(stdout);
		return 0;
	}
	CK(hipStreamDestroy(ms));
	printf("destroy: masked stream destroyed\n");
	fflush(stdout);
	k_touch<<<n / 256, 256, 0, before>>>(d, n);
	CK(hipGetLastError());
	CK(hipStreamSynchronize(before));
	printf("destroy: kernel on a stream created before it ok\n");
	fflush(stdout);
	hipStream_t after;
	CK(hipStreamCreateWithFlags(&after, hipStreamNonBlocking));
	k_touch<<<n / 256, 256, 0, after>>>(d, n);
	CK(hipGetLastError());
	CK(hipStreamSynchronize(after));
	printf("destroy: kernel on a stream created after it ok\n");
	fflush(stdout);
	k_touch<<<n / 256, 256, 0, 0>>>(d, n);
	CK(hipGetLastError());
	CK(hipDeviceSynchronize());
	printf("destroy: kernel on the null stream ok\n");
	std::vector<int> h(n);
	CK(hipMemcpy(h.data(), d, n * 4, hipMemcpyDeviceToHost));
	int bad = 0;
	for(int i = 0; i < n; ++i) bad += h[i] != 4;
	printf("destroy: values %s\n", bad ? "WRONG" : "ok (4 increments)");
	CK(hipStreamDestroy(before));
	CK(hipStreamDestroy(after));
	CK(hipFree(d));
	return bad ? 1 : 0;
}

// the engine probe's sequence (tools/cu_mask_probe.py close) without the
// engine: context A (plain stream), context B (plain stream, then replaced by
// a masked one, the plain one destroyed), work on the masked stream, the
// masked stream destroyed; then what torch does at its first use: a pool of
// streams at two priorities, a kernel on each
static int run_engine_seq(int words, int pool, int use_mask, int destroy, int prio, int teardown) {
	std::vector<uint32_t> m(words, 0u);
	for(int c = 0; c < 64; ++c)
		if(c / 32 < words) m[c / 32] |= 1u << (c % 32);
	const int n = 1 << 20;
	int *d;
	CK(hipMalloc(&d, n * 4));
	CK(hipMemset(d, 0, n * 4));
	hipStream_t a, b, ms;
	CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
	CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
	hipEvent_t e0, e1;
	CK(hipEventCreate(&e0));
	CK(hipEventCreate(&e1));
	if(use_mask) CK(hipExtStreamCreateWithCUMask(&ms, (uint32_t) words, m.data()));
	else CK(hipStreamCreateWithFlags(&ms, hipStreamNonBlocking));
	CK(hipStreamSynchronize(b));
	CK(hipStreamDestroy(b));
	CK(hipEventRecord(e0, ms));
	for(int k = 0; k < 3000; ++k) k_touch<<<n / 256, 256, 0, ms>>>(d, n);
	CK(hipEventRecord(e1, ms));
	CK(hipStreamSynchronize(ms));
	CK(hipEventDestroy(e0));
	CK(hipEventDestroy(e1));
	if(destroy) CK(hipStreamDestroy(ms));
	printf("engine-seq words=%d mask=%d destroy=%d prio=%d: 3000 kernels on the stream%s\n", words, use_mask, destroy,
	       prio, destroy ? ", stream destroyed" : ", stream kept");
	fflush(stdout);
	int lo = 0, hi = 0;
	CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
	std::vector<hipStream_t> ps;
	for(int k = 0; k < pool; ++k) {
		hipStream_t s;
		CK(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, prio && k % 2 ? hi : lo));
		ps.push_back(s);
		k_touch<<<n / 256, 256, 0, s>>>(d, n);
		CK(hipGetLastError());
		CK(hipStreamSynchronize(s));
		printf("  stream %d (priority %d): kernel done\n", k, prio && k % 2 ? hi : lo);
		fflush(stdout);
	}
	CK(hipDeviceSynchronize());
	printf("engine-seq: %d priority streams created after it, a kernel on each ok\n", pool);
	k_touch<<<n / 256, 256, 0, a>>>(d, n);
	CK(hipStreamSynchronize(a));
	k_touch<<<n / 256, 256, 0, 0>>>(d, n);
	CK(hipDeviceSynchronize());
	std::vector<int> h(n);
	CK(hipMemcpy(h.data(), d, n * 4, hipMemcpyDeviceToHost));
	int bad = 0;
	for(int i = 0; i < n; ++i) bad += h[i] != 3000 + pool + 2;
	printf("engine-seq: values %s\n", bad ? "WRONG" : "ok");
	fflush(stdout);
	if(teardown) {
		printf("engine-seq: returning from main with the streams alive\n");
		fflush(stdout);
		return bad ? 1 : 0;
	}
	for(hipStream_t s : ps) CK(hipStreamDestroy(s));
	CK(hipStreamDestroy(a));
	CK(hipFree(d));
	return bad ? 1 : 0;
}

int main(int argc, char **argv) {
	if(argc < 2) {
		fprintf(stderr, "usage: cu_mask map LAYOUT K [WORDS] | destroy WORDS | exit WORDS\n");
		return 2;
	}
	if(!strcmp(argv[1], "map") && argc >= 4) return run_map(argv[2], atoi(argv[3]), argc > 4 ? atoi(argv[4]) : 0);
	if(!strcmp(argv[1], "destroy")) return run_destroy(argc > 2 ? atoi(argv[2]) : 8, false);
	if(!strcmp(argv[1], "exit")) return run_destroy(argc > 2 ? atoi(argv[2]) : 8, true);
	if(!strcmp(argv[1], "engine"))
		return run_engine_seq(argc > 2 ? atoi(argv[2]) : 2, argc > 3 ? atoi(argv[3]) : 64, argc > 4 ? atoi(argv[4]) : 1,
		                      argc > 5 ? atoi(argv[5]) : 1, argc > 6 ? atoi(argv[6]) : 1, argc > 7 ? atoi(argv[7]) : 0);
	fprintf(stderr, "unknown mode\n");
	return 2;
}
