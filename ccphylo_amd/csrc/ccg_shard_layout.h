// ccg_shard_layout.h -- the row-sharded LT layout (bands of SB rows dealt
// round-robin over the ranks, each rank's rows back to back), shared by the
// sharded tree engines (ccg_shard.h) and the sharded dist (snp.hip).
#pragma once
#include "ccg_internal.h"

#define SB CCG_SHARD_BAND

struct Shard {
	int rank, world;
	__host__ __device__ __forceinline__ bool owns(long long r) const { return (int) ((r / SB) % world) == rank; }
	__host__ __device__ __forceinline__ long long row(long long r) const { return off(r); }
	// elements before owned row r in the rank's buffer: full owned bands below
	// r's band (band g holds SB*SB*g + SB*(SB-1)/2 elements), then r's
	// predecessors in its band
	__host__ __device__ __forceinline__ long long off(long long r) const {
		const long long gb = r / SB, t = r - gb * SB, lb = gb / world;
		return (long long) SB * SB * world * (lb * (lb - 1) / 2) + (long long) SB * SB * rank * lb +
		       lb * (SB * (SB - 1) / 2) + SB * gb * t + t * (t - 1) / 2;
	}
};

