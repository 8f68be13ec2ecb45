// work_queue.hpp -- the work queue of wave-tiles the coding, fused and
// checksum kernels take their tiles from: device side.
#pragma once

#ifndef __HIPCC_RTC__  // hiprtc (jit.cpp) provides the HIP runtime itself
#include <hip/hip_runtime.h>
#endif

#include <cstdint>

#include "ec_kernels.hpp"  // kMixedQueues, kMixedQueueStride

namespace hec {
namespace {  // per translation unit, as gf_device.hpp

// The counter set a launch zeroes for the stream's NEXT launch (round 6,
// DESIGN.md §3.1 "Counter sets"): a stream alternates between two sets, and
// launch i zeroes the set launch i+1 will use -- the set launch i-1 used,
// which is complete (one stream runs its launches in order).  So a launch
// never depends on how the previous one counted: the counters are zero at
// every launch's start by construction, whatever state an earlier launch
// left them in.  Block 0's first kMixedQueues lanes, vector stores.  Graph
// launches get a private set zeroed by a memset node instead (zero ==
// nullptr).
__device__ __forceinline__ void queue_zero_next(uint32_t* zero) {
    if (zero && blockIdx.x == 0 && threadIdx.x < kMixedQueues) zero[threadIdx.x * (kMixedQueueStride / 4)] = 0u;
}

// Work queue of wave-tiles, one round per atomic (the
// register kernel's gf_matmul_v16 runs the batched form): the tile order is
// dealt round-robin to n = min(grid, kMixedQueues) launch counters, block b
// takes from counter b % n (tile = round * n + counter), and lane 0 fetches
// the wave's next round when it takes one, so the fetch is in flight while
// the tile is coded.  peek() reads that next tile early (a kernel that
// prefetches the next tile's inputs) without fetching again.  The counters
// start at zero (queue_zero_next / the graph's memset node); nothing here
// resets them, so no count of fetches has to come out exact.
struct WaveQueue {
    uint32_t* ctr;
    uint32_t n, q, total, pend, peek_v;
    bool peeked;
    __device__ __forceinline__ void init(uint32_t* queue, uint32_t total_tiles) {
        n = gridDim.x < kMixedQueues ? gridDim.x : kMixedQueues;
        q = blockIdx.x % n;
        total = total_tiles;
        ctr = queue + q * (kMixedQueueStride / 4);
        peeked = false;
        // defined in every lane (lane 0's is the one read): no merge of the
        // atomic's result with an undefined value
        asm volatile("" : "=v"(pend));
        if ((threadIdx.x & 63u) == 0) pend = atomicAdd(ctr, 1u);
    }
    __device__ __forceinline__ uint32_t tile_of(uint32_t v) const {
        const uint64_t t = uint64_t(v) * n + q;
        return t < total ? uint32_t(t) : total;
    }
    __device__ __forceinline__ uint32_t peek() {
        if (!peeked) {
            peek_v = uint32_t(__builtin_amdgcn_readfirstlane(int(pend)));
            peeked = true;
        }
        return tile_of(peek_v);
    }
    __device__ __forceinline__ uint32_t next() {
        const uint32_t v = peeked ? peek_v : uint32_t(__builtin_amdgcn_readfirstlane(int(pend)));
        peeked = false;
        const uint32_t t = tile_of(v);
        if (t < total && (threadIdx.x & 63u) == 0) pend = atomicAdd(ctr, 1u);
        return t;
    }
};

}  // namespace
}  // namespace hec
