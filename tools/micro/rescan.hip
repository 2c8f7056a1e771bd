// Calibration: cost of one DNJ rescan launch (R rows x C cells in U-cell units
// over the grid, reduce per unit, store the partial) vs unit size and loads,
// graph-replayed (development aid).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <float.h>
#pragma clang diagnostic ignored "-Wunused-value"

template <int NT, int UNR, bool SD>
__global__ __launch_bounds__(NT) void k_rescan(const double *D, const double *sD, int rows, int len, double *out) {
	__shared__ double sq[NT / 64];
	constexpr int SEGC = NT * UNR;
	const int upr = (len + SEGC - 1) / SEGC;
	for(int u = blockIdx.x; u < rows * upr; u += gridDim.x) {
		const int r = u / upr, c0 = (u % upr) * SEGC;
		const double *row = D + (size_t) r * len;
		double q = DBL_MAX;
		double v[UNR], s[UNR];
#pragma unroll
		for(int m = 0; m < UNR; ++m) {
			int c = c0 + m * NT + threadIdx.x;
			if(c < len) {
				v[m] = row[c];
				s[m] = SD ? sD[c] : 1.0;
			}
		}
#pragma unroll
		for(int m = 0; m < UNR; ++m) {
			int c = c0 + m * NT + threadIdx.x;
			if(c < len) {
				double x = 3.0 * v[m] - s[m] - 0.5;
				q = x < q ? x : q;
			}
		}
		for(int off = 32; off > 0; off >>= 1) {
			double o = __shfl_xor(q, off, 64);
			q = o < q ? o : q;
		}
		if((threadIdx.x & 63) == 0) sq[threadIdx.x >> 6] = q;
		__syncthreads();
		if(threadIdx.x == 0) {
			for(int w = 1; w < NT / 64; ++w) q = sq[w] < q ? sq[w] : q;
			out[u] = q;
		}
		__syncthreads();
	}
}

typedef void (*LF)(hipStream_t, const double *, const double *, int, int, double *, int);
template <int NT, int UNR, bool SD>
void launch(hipStream_t st, const double *D, const double *sD, int rows, int len, double *out, int off) {
	const int upr = (len + NT * UNR - 1) / (NT * UNR);
	int g = rows * upr;
	if(g > 2048) g = 2048;
	// rotate the rows so replays read fresh lines (no L2 reuse across launches)
	k_rescan<NT, UNR, SD><<<g, NT, 0, st>>>(D + (size_t) off * len, sD, rows, len, out);
}

static float time_graph(hipStream_t st, LF f, const double *D, const double *sD, int rows, int len, double *out) {
	hipGraph_t g;
	hipGraphExec_t ge;
	hipEvent_t a, b;
	hipEventCreate(&a);
	hipEventCreate(&b);
	const int reps = 100;
	hipStreamBeginCapture(st, hipStreamCaptureModeGlobal);
	for(int r = 0; r < reps; ++r) f(st, D, sD, rows, len, out, (r % 16) * rows);
	hipStreamEndCapture(st, &g);
	hipGraphInstantiate(&ge, g, NULL, NULL, 0);
	hipGraphLaunch(ge, st);
	hipEventRecord(a, st);
	hipGraphLaunch(ge, st);
	hipEventRecord(b, st);
	hipEventSynchronize(b);
	float ms;
	hipEventElapsedTime(&ms, a, b);
	return ms * 1000.0f / reps;
}

int main() {
	const int len = 9000, maxrows = 16 * 256;
	double *D, *sD, *out;
	hipMalloc(&D, (size_t) maxrows * len * 8);
	hipMalloc(&sD, len * 8);
	hipMalloc(&out, 1 << 20);
	hipMemset(D, 0, (size_t) maxrows * len * 8);
	hipMemset(sD, 0, len * 8);
	hipStream_t st;
	hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
	const int rowsv[] = {1, 16, 64, 128, 256};
	for(int rows : rowsv) {
		double mb = rows * (double) len * 8 / 1e6;
		float t1 = time_graph(st, launch<256, 8, true>, D, sD, rows, len, out);
		float t2 = time_graph(st, launch<256, 8, false>, D, sD, rows, len, out);
		float t3 = time_graph(st, launch<256, 2, true>, D, sD, rows, len, out);
		float t4 = time_graph(st, launch<1024, 8, true>, D, sD, rows, len, out);
		float t5 = time_graph(st, launch<256, 32, true>, D, sD, rows, len, out);
		printf("rows %4d (%6.2f MB of D): 256x8+sD %6.2f  256x8 noSD %6.2f  256x2+sD %6.2f  1024x8+sD %6.2f  256x32+sD %6.2f us | %5.0f GB/s best\n",
		       rows, mb, t1, t2, t3, t4, t5, mb * 1e3 / (t1 < t4 ? t1 : t4));
	}
	return 0;
}
