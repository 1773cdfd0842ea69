// Shared host/device helpers for the gfx950 tracker library.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <string>

#include "../../include/yolo_tracking_amd.h"

namespace yta {

// ------------------------------------------------------------------ host error plumbing
void set_error(const char *fmt, ...);

#define YTA_HIP(call)                                                                     \
    do {                                                                                  \
        hipError_t _e = (call);                                                           \
        if (_e != hipSuccess) {                                                           \
            ::yta::set_error("%s:%d %s -> %s", __FILE__, __LINE__, #call,                 \
                             hipGetErrorString(_e));                                      \
            return YTA_ERR_HIP;                                                           \
        }                                                                                 \
    } while (0)

#define YTA_CHECK(cond, code, ...)                                                        \
    do {                                                                                  \
        if (!(cond)) {                                                                    \
            ::yta::set_error(__VA_ARGS__);                                                \
            return (code);                                                                \
        }                                                                                 \
    } while (0)

int select_device(int device);

// ------------------------------------------------------------------ device helpers
constexpr int WAVE = 64;

// Block barrier for kernels that hand data between threads through GLOBAL memory: every wave
// drains its outstanding vector-memory operations before the barrier.  (__syncthreads() alone
// lowers to a bare s_barrier on gfx950 for workgroup scope; a global store still in flight could
// then be overtaken by another thread's load of the same address after the barrier.)
__device__ __forceinline__ void block_sync() {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __syncthreads();
}

__device__ __forceinline__ int lane_id() { return __lane_id(); }

__device__ __forceinline__ unsigned long long lanemask_lt() {
    return (1ull << lane_id()) - 1ull;
}

// Exclusive prefix sum over the whole block (blockDim.x multiple of 64, <= 1024).  `wsum` is a
// shared scratch of >= 17 ints.  Returns the exclusive prefix; *total gets the block sum.
__device__ __forceinline__ int block_exclusive_scan(int v, int *wsum, int *total) {
    const int lane = lane_id();
    const int wid = threadIdx.x / WAVE;
    const int nw = (blockDim.x + WAVE - 1) / WAVE;
    int incl = v;
#pragma unroll
    for (int off = 1; off < WAVE; off <<= 1) {
        int t = __shfl_up(incl, off, WAVE);
        if (lane >= off) incl += t;
    }
    if (lane == WAVE - 1) wsum[wid] = incl;
    block_sync();
    if (threadIdx.x == 0) {
        int run = 0;
        for (int w = 0; w < nw; ++w) {
            int t = wsum[w];
            wsum[w] = run;
            run += t;
        }
        wsum[16] = run;
    }
    __syncthreads();
    int excl = incl - v + wsum[wid];
    if (total) *total = wsum[16];
    __syncthreads();
    return excl;
}

// Order-preserving compaction of indices [0, n) where pred(i) holds, appended to out[*]
// starting at `base`.  All threads of the block must call it.  Returns the count.
template <typename Pred, typename Emit>
__device__ int block_compact(int n, int *wsum, Pred pred, Emit emit) {
    int count = 0;
    for (int start = 0; start < n; start += blockDim.x) {
        int i = start + threadIdx.x;
        int f = (i < n && pred(i)) ? 1 : 0;
        int tot;
        int pos = block_exclusive_scan(f, wsum, &tot);
        if (f) emit(i, count + pos);
        count += tot;
    }
    return count;
}

// NumPy's np.maximum / np.minimum for float64 (NaN-propagating; first operand wins on ties).
__host__ __device__ __forceinline__ double np_max(double a, double b) { return (a >= b || a != a) ? a : b; }
__host__ __device__ __forceinline__ double np_min(double a, double b) { return (a <= b || a != a) ? a : b; }

}  // namespace yta
