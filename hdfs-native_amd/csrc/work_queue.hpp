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

// Work queue of wave-tiles, one round per atomic (the
// register kernel's gf_matmul_v16 runs the batched form): the tile order is
// dealt round-robin to n = min(grid, kMixedQueues) launch counters, block b
// takes from counter b % n (tile = round * n + counter), and lane 0 fetches
// the wave's next round when it takes one, so the fetch is in flight while
// the tile is coded.  peek() reads that next tile early (a kernel that
// prefetches the next tile's inputs) without fetching again.  Every fetch is
// read back, the one past the end included, so a counter's last value is
// known (its rounds + its waves - 1) and the wave that draws it zeroes the
// counter for the stream's next launch.
struct WaveQueue {
    uint32_t* ctr;
    uint32_t n, q, total, last, pend, peek_v;
    bool peeked;
    __device__ __forceinline__ void init(uint32_t* queue, uint32_t total_tiles, uint32_t waves_per_block) {
        n = gridDim.x < kMixedQueues ? gridDim.x : kMixedQueues;
        q = blockIdx.x % n;
        total = total_tiles;
        ctr = queue + q * (kMixedQueueStride / 4);
        const uint32_t rounds = total > q ? (total - 1 - q) / n + 1 : 0;
        const uint32_t blocks = (gridDim.x - 1 - q) / n + 1;
        last = rounds + blocks * waves_per_block - 1;
        peeked = false;
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
        if ((threadIdx.x & 63u) == 0) {
            if (t < total)
                pend = atomicAdd(ctr, 1u);
            else if (v == last)
                (void)atomicExch(ctr, 0u);  // every fetch of this counter is done
        }
        return t;
    }
};

}  // namespace
}  // namespace hec
