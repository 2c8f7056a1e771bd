// Which bitop3 truth table computes (a ^ b) | c on gfx950 (development aid).
#include <hip/hip_runtime.h>
#include <stdio.h>
#pragma clang diagnostic ignored "-Wunused-value"
__global__ void k(unsigned *o) {
	const unsigned a = 0xF0F0F0F0u, b = 0xCCCCCCCCu, c = 0xAAAAAAAAu;
	o[0] = __builtin_amdgcn_bitop3_b32(a, b, c, 0xBE);
	o[1] = __builtin_amdgcn_bitop3_b32(a, b, c, 0xF6);
	o[2] = (a ^ b) | c;
}
int main() {
	unsigned *d, h[3];
	hipMalloc(&d, 12);
	k<<<1, 1>>>(d);
	hipMemcpy(h, d, 12, hipMemcpyDeviceToHost);
	printf("0xBE -> %08x, 0xF6 -> %08x, expected %08x\n", h[0], h[1], h[2]);
	return 0;
}
