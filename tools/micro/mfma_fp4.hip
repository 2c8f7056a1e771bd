// MX-fp4 MFMA (v_mfma_scale_f32_32x32x64_f8f6f4, both operands e2m1, unit
// scales) on gfx950: operand lane map and issue rate (development aid for an
// MFMA form of the non-pair SNP distance, DESIGN.md "dist").
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/micro/mfma_fp4 tools/micro/mfma_fp4.hip
//   tools/micro/mfma_fp4
//
// 1. map: A holds +1 (e2m1 0x2) in one nibble of one lane, B is all +1; the
//    output row that reads 1 names the A row of that (lane, nibble); the same
//    with the roles swapped names the B column.  Prints the (row | col, k)
//    decoding rule it finds for every (lane, nibble).
// 2. rate: 4 independent accumulators per wave, operands in registers,
//    blocks x 4 waves, MACs/s and position-pairs/s for the 3-MAC tetrahedron
//    form (diff = (3 L - dot) / 4).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));

#define FMT_FP4 4
#define SCALE_ONE 127   // E8M0 exponent of 1.0

__global__ void k_map(const int *a, const int *bm, float *out) {
	const int lane = threadIdx.x;
	v8i A, B;
	for(int r = 0; r < 8; ++r) {
		A[r] = a[lane * 8 + r];
		B[r] = bm[lane * 8 + r];
	}
	v16f C = {};
	C = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(A, B, C, FMT_FP4, FMT_FP4, 0, SCALE_ONE, 0, SCALE_ONE);
	for(int r = 0; r < 16; ++r) out[lane * 16 + r] = C[r];
}

__global__ void k_rate(int iters, float *sink) {
	v8i A, B;
	for(int r = 0; r < 8; ++r) {
		A[r] = 0x22222222 ^ (threadIdx.x * 0x01010101 * r);
		B[r] = 0x2a2a2a2a ^ (threadIdx.x * 0x10101010 * r);
	}
	v16f c0 = {}, c1 = {}, c2 = {}, c3 = {};
	for(int i = 0; i < iters; ++i) {
		c0 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(A, B, c0, FMT_FP4, FMT_FP4, 0, SCALE_ONE, 0, SCALE_ONE);
		c1 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(B, A, c1, FMT_FP4, FMT_FP4, 0, SCALE_ONE, 0, SCALE_ONE);
		c2 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(A, A, c2, FMT_FP4, FMT_FP4, 0, SCALE_ONE, 0, SCALE_ONE);
		c3 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(B, B, c3, FMT_FP4, FMT_FP4, 0, SCALE_ONE, 0, SCALE_ONE);
	}
	float s = 0;
	for(int r = 0; r < 16; ++r) s += c0[r] + c1[r] + c2[r] + c3[r];
	if(s == 1234.5f) sink[threadIdx.x] = s;
}

#define CK(x)                                                                   \
	do {                                                                        \
		hipError_t e_ = (x);                                                    \
		if(e_ != hipSuccess) {                                                  \
			fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));             \
			exit(1);                                                            \
		}                                                                       \
	} while(0)

// C/D layout of 32x32 (cdna_hip_programming.md 3): col = lane & 31,
// row = (reg & 3) + 8 (reg >> 2) + 4 (lane >> 5)
static void find_one(const float *out, int *row, int *col, int *cnt, float *val) {
	*cnt = 0;
	for(int l = 0; l < 64; ++l)
		for(int r = 0; r < 16; ++r)
			if(out[l * 16 + r] != 0.0f) {
				*row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5);
				*col = l & 31;
				*val = out[l * 16 + r];
				++*cnt;
			}
}

int main() {
	int *da, *db;
	float *dout;
	CK(hipMalloc(&da, 64 * 8 * 4));
	CK(hipMalloc(&db, 64 * 8 * 4));
	CK(hipMalloc(&dout, 64 * 16 * 4));
	static int ha[64 * 8], hb[64 * 8];
	static float ho[64 * 16];
	// 1. A: one +1 at (lane, nibble); B: +1 in a single column c0 = 5 only?
	// B all +1 makes every column light up; use B = +1 everywhere and read the
	// row, then A all +1 with one B nibble to read the column.
	int bad = 0;
	printf("A operand: (lane, nibble) -> row, k-range check\n");
	for(int l = 0; l < 64; ++l) {
		for(int nib = 0; nib < 32; nib += 31) {   // first and last nibble of the 4 used dwords
			for(int x = 0; x < 64 * 8; ++x) ha[x] = hb[x] = 0;
			ha[l * 8 + nib / 8] = 0x2 << (4 * (nib % 8));
			for(int x = 0; x < 64 * 8; ++x) hb[x] = (x % 8) < 4 ? 0x22222222 : 0;
			CK(hipMemcpy(da, ha, sizeof(ha), hipMemcpyHostToDevice));
			CK(hipMemcpy(db, hb, sizeof(hb), hipMemcpyHostToDevice));
			k_map<<<1, 64>>>(da, db, dout);
			CK(hipMemcpy(ho, dout, sizeof(ho), hipMemcpyDeviceToHost));
			int lit = 0;
			for(int x = 0; x < 64 * 16; ++x) lit += ho[x] != 0.0f;
			// a row of 32 ones
			int row = -1;
			for(int ll = 0; ll < 64; ++ll)
				for(int r = 0; r < 16; ++r)
					if(ho[ll * 16 + r] != 0.0f) row = (r & 3) + 8 * (r >> 2) + 4 * (ll >> 5);
			if(l < 3 || l == 31 || l == 32 || l == 63) printf("  lane %2d nibble %2d: %d outputs lit, row %d\n", l, nib, lit, row);
			if(lit != 32 || row != (l & 31)) ++bad;
		}
	}
	printf("A rows = lane & 31: %s\n", bad ? "NO" : "yes");
	// k mapping: A lane l nibble m and B lane l' nibble m' meet iff same k.
	// Find, for A (lane 0, nibble m), which B (lane, nibble) pairs with it.
	printf("k map (A lane 0 / 32 nibble m pairs with B lane L nibble m'):\n");
	for(int al = 0; al < 64; al += 32) {
		for(int m = 0; m < 32; m += 7) {
			int found = 0;
			for(int bl = 0; bl < 64 && !found; bl += 32) {
				for(int mb = 0; mb < 32 && !found; ++mb) {
					for(int x = 0; x < 64 * 8; ++x) ha[x] = hb[x] = 0;
					ha[al * 8 + m / 8] = 0x2 << (4 * (m % 8));
					hb[bl * 8 + mb / 8] = 0x2 << (4 * (mb % 8));
					CK(hipMemcpy(da, ha, sizeof(ha), hipMemcpyHostToDevice));
					CK(hipMemcpy(db, hb, sizeof(hb), hipMemcpyHostToDevice));
					k_map<<<1, 64>>>(da, db, dout);
					CK(hipMemcpy(ho, dout, sizeof(ho), hipMemcpyDeviceToHost));
					int row, col, cnt;
					float v;
					find_one(ho, &row, &col, &cnt, &v);
					if(cnt == 1) {
						printf("  A(lane %2d, nib %2d) x B(lane %2d, nib %2d) -> out[%d][%d] = %g\n", al, m, bl, mb, row,
						       col, v);
						found = 1;
					}
				}
			}
			if(!found) printf("  A(lane %2d, nib %2d): no partner found\n", al, m);
		}
	}
	// sign: -1 is 0xA
	for(int x = 0; x < 64 * 8; ++x) ha[x] = hb[x] = 0;
	ha[0] = 0xA;
	hb[0] = 0x2;
	CK(hipMemcpy(da, ha, sizeof(ha), hipMemcpyHostToDevice));
	CK(hipMemcpy(db, hb, sizeof(hb), hipMemcpyHostToDevice));
	k_map<<<1, 64>>>(da, db, dout);
	CK(hipMemcpy(ho, dout, sizeof(ho), hipMemcpyDeviceToHost));
	{
		int row, col, cnt;
		float v;
		find_one(ho, &row, &col, &cnt, &v);
		printf("(-1) x (+1) -> %d outputs, value %g\n", cnt, v);
	}
	// 2. rate
	int dev_cus = 0;
	hipDeviceProp_t p;
	CK(hipGetDeviceProperties(&p, 0));
	dev_cus = p.multiProcessorCount;
	float *sink;
	CK(hipMalloc(&sink, 4096));
	const int iters = 20000;
	for(int bpc = 1; bpc <= 2; ++bpc) {
		const int blocks = dev_cus * bpc;
		k_rate<<<blocks, 256>>>(100, sink);
		CK(hipDeviceSynchronize());
		hipEvent_t e0, e1;
		CK(hipEventCreate(&e0));
		CK(hipEventCreate(&e1));
		CK(hipEventRecord(e0));
		k_rate<<<blocks, 256>>>(iters, sink);
		CK(hipEventRecord(e1));
		CK(hipEventSynchronize(e1));
		float ms;
		CK(hipEventElapsedTime(&ms, e0, e1));
		const double macs = (double) blocks * 4 /*waves*/ * iters * 4 /*mfma*/ * 32.0 * 32 * 64;
		printf("rate: %d blocks x 4 waves: %.3f ms, %.3e MAC/s = %.1f%% of 5e15; tetrahedron %.3e position-pairs/s\n",
		       blocks, ms, macs / (ms * 1e-3), 100.0 * macs / (ms * 1e-3) / 5e15, macs / (ms * 1e-3) / 3);
	}
	return 0;
}
