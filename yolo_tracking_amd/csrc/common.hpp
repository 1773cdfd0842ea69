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

// Wait for everything queued on `s` without spinning a host core: a blocking-sync event recorded
// on the stream (hipStreamSynchronize may busy-wait; on a host with a CPU quota the spinning
// threads of a synchronous update() then get the whole process throttled).  One event per host
// thread and device.
hipError_t host_wait(hipStream_t s);

// ------------------------------------------------------------------ device helpers
constexpr int WAVE = 64;

// address-space-qualified pointers for __builtin_amdgcn_global_load_lds (global -> LDS, no VGPRs)
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void glob_void;

// Block barrier for kernels that hand data between threads through GLOBAL memory: every wave
// drains its outstanding vector-memory operations before the barrier.  (__syncthreads() alone
// lowers to a bare s_barrier on gfx950 for workgroup scope; a global store still in flight could
// then be overtaken by another thread's load of the same address after the barrier.)
__device__ __forceinline__ void block_sync() {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __syncthreads();
}

// XCD-aware placement of a (gx x gy) tile grid (blockIdx.x: column tiles, blockIdx.y: row tiles,
// one grid slice per blockIdx.z).  Workgroups are dispatched round-robin over the 8 XCDs, each
// with its own L2, so launch-order neighbours share nothing.  Instead XCD x (linear id mod 8)
// takes row band x (gy / 8 row tiles) and walks it column by column: the band's row operands
// stay in its L2 and each column operand is fetched once per XCD and reused band-rows times.
// A bijection whenever gy is a multiple of 8; otherwise the launch order is kept.
__device__ __forceinline__ void xcd_tile(int &bx, int &by) {
    bx = blockIdx.x;
    by = blockIdx.y;
    const int gx = gridDim.x, gy = gridDim.y;
    if ((gy & 7) == 0) {
        const int lin = bx + gx * by, xcd = lin & 7, k = lin >> 3, band = gy >> 3;
        by = xcd * band + k % band;
        bx = k / band;
    }
}

// Diagnostic build only (-DYTA_STAMPS, tools/diag_stamps.py): wall-clock stamps (100 MHz) of
// block 0's phases, read back with yta_debug_stamps.
#ifdef YTA_STAMPS
static __device__ unsigned long long g_stamps[128];
static __device__ int g_stamp_off;
#define YTA_STAMP(k)                                                                        \
    do {                                                                                    \
        if (blockIdx.x == 0 && threadIdx.x == 0) g_stamps[g_stamp_off + (k)] = wall_clock64(); \
    } while (0)
#define YTA_STAMP_BASE(b)                                        \
    do {                                                         \
        if (blockIdx.x == 0 && threadIdx.x == 0) g_stamp_off = (b); \
    } while (0)
#define YTA_STAMP_ABS(k)                                                       \
    do {                                                                       \
        if (blockIdx.x == 0 && threadIdx.x == 0) g_stamps[(k)] = wall_clock64(); \
    } while (0)
#define YTA_COUNT(k)                                                           \
    do {                                                                       \
        if (blockIdx.x == 0 && threadIdx.x == 0) g_stamps[(k)] += 1;            \
    } while (0)
// per-block timeline of the block/stream kernels: start (e = 0) and end (e = 1) of block b of
// kernel k, read back with yta_debug_blocks
constexpr int YTA_BLK_MAX = 4096;
static __device__ unsigned long long g_blk[8][YTA_BLK_MAX][2];
// k_apply phases of blocks (x, y < 256): start, decision level 0, records in LDS, computed, stored
static __device__ unsigned long long g_apl[4096][5];
#define YTA_APL(k)                                                                          \
    do {                                                                                    \
        if (threadIdx.x == 0 && blockIdx.y < 256 && blockIdx.x < 16)                        \
            g_apl[blockIdx.y * 16 + blockIdx.x][k] = wall_clock64();                        \
    } while (0)
#define YTA_BLK(k, e)                                                                \
    do {                                                                             \
        if (threadIdx.x == 0 && blockIdx.x < YTA_BLK_MAX) g_blk[k][blockIdx.x][e] = wall_clock64(); \
    } while (0)
#else
#define YTA_APL(k) \
    do {           \
    } while (0)
#define YTA_BLK(k, e) \
    do {              \
    } while (0)
#define YTA_COUNT(k) \
    do {             \
    } while (0)
#define YTA_STAMP(k) \
    do {             \
    } while (0)
#define YTA_STAMP_BASE(b) \
    do {                  \
    } while (0)
#define YTA_STAMP_ABS(k) \
    do {                 \
    } while (0)
#endif

__device__ __forceinline__ int lane_id() { return __lane_id(); }

__device__ __forceinline__ unsigned long long lanemask_lt() {
    return (1ull << lane_id()) - 1ull;
}

// ------------------------------------------------------------------ DPP cross-lane primitives
// gfx950 (GFX9 DPP): quad_perm, row_shr:n (0x110+n), row_ror:n (0x120+n), row_bcast:15 (0x142),
// row_bcast:31 (0x143).  All lanes of the wave must be active.
template <int CTRL>
__device__ __forceinline__ int dpp_i32(int v) {
    return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false);
}
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(v);
    const unsigned lo = (unsigned)dpp_i32<CTRL>((int)(unsigned)b);
    const unsigned hi = (unsigned)dpp_i32<CTRL>((int)(unsigned)(b >> 32));
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
__device__ __forceinline__ double readlane_f64(double v, int lane) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)b, lane);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(b >> 32), lane);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// Inclusive prefix sum over the 64 lanes.
__device__ __forceinline__ int wave_inclusive_scan(int x) {
    const int l = lane_id(), rl = l & 15;
    int t;
    t = dpp_i32<0x111>(x); if (rl >= 1) x += t;
    t = dpp_i32<0x112>(x); if (rl >= 2) x += t;
    t = dpp_i32<0x114>(x); if (rl >= 4) x += t;
    t = dpp_i32<0x118>(x); if (rl >= 8) x += t;
    t = dpp_i32<0x142>(x); if ((l & 31) >= 16) x += t;
    t = dpp_i32<0x143>(x); if (l >= 32) x += t;
    return x;
}

enum { RED_MIN = 0, RED_MAX = 1, RED_SUM = 2 };
__device__ __forceinline__ double red_op(int op, double a, double b) {
    return op == RED_MIN ? fmin(a, b) : (op == RED_MAX ? fmax(a, b) : a + b);
}
__device__ __forceinline__ double red_ident(int op) {
    return op == RED_MIN ? INFINITY : (op == RED_MAX ? -INFINITY : 0.0);
}
// All-reduce within each 16-lane row (every lane of the row gets the row's result).
__device__ __forceinline__ double row_allreduce(int op, double v) {
    v = red_op(op, v, dpp_f64<0xB1>(v));    // quad_perm [1,0,3,2]
    v = red_op(op, v, dpp_f64<0x4E>(v));    // quad_perm [2,3,0,1]
    v = red_op(op, v, dpp_f64<0x124>(v));   // row_ror:4
    v = red_op(op, v, dpp_f64<0x128>(v));   // row_ror:8
    return v;
}
// Wave-uniform reduction of the 64 lanes.
__device__ __forceinline__ double wave_reduce(int op, double v) {
    v = row_allreduce(op, v);
    return red_op(op, red_op(op, readlane_f64(v, 0), readlane_f64(v, 16)),
                  red_op(op, readlane_f64(v, 32), readlane_f64(v, 48)));
}

// Block barrier for hand-offs through LDS only: outstanding global stores are not waited for
// (block_sync drains them, which costs a full memory round trip under load).
__device__ __forceinline__ void lds_sync() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();
}

// Exclusive prefix sum over the whole block (blockDim.x a multiple of 64, <= 1024).  `wsum` is a
// shared scratch of >= 16 ints.  Returns the exclusive prefix; *total gets the block sum.
// GSYNC: the barrier also drains global memory operations (block_sync), else LDS only.
template <bool GSYNC = true>
__device__ __forceinline__ int block_exclusive_scan(int v, int *wsum, int *total) {
    const int lane = lane_id();
    const int wid = threadIdx.x / WAVE;
    const int nw = blockDim.x / WAVE;
    const int incl = wave_inclusive_scan(v);
    if (lane == WAVE - 1) wsum[wid] = incl;
    if (GSYNC) block_sync();
    else lds_sync();
    int p = lane < nw ? wsum[lane] : 0;
    p = wave_inclusive_scan(p);
    const int before = wid > 0 ? __builtin_amdgcn_readlane(p, wid - 1) : 0;
    if (total) *total = __builtin_amdgcn_readlane(p, nw - 1);
    __syncthreads();   // wsum is reused by the next scan
    return incl - v + before;
}

// Order-preserving compaction of indices [0, n) where pred(i) holds: emit(i, position).  All
// threads of the block must call it.  Returns the count.  Each thread owns a contiguous run of
// up to 32 indices (predicate bits in a register), so one block scan covers n <= 32 * blockDim;
// beyond that the range is processed in such super-chunks.
template <bool GSYNC = true, typename Pred, typename Emit>
__device__ __forceinline__ int block_compact(int n, int *wsum, Pred pred, Emit emit) {
    const int nt = blockDim.x, t = threadIdx.x;
    int count = 0;
    for (int base = 0; base < n; base += 32 * nt) {
        const int m = n - base < 32 * nt ? n - base : 32 * nt;
        const int per = (m + nt - 1) / nt;
        const int lo = base + t * per;
        const int hi = lo + per < base + m ? lo + per : base + m;
        unsigned bits = 0;
        for (int i = lo; i < hi; ++i)
            if (pred(i)) bits |= 1u << (i - lo);
        int tot;
        int pos = count + block_exclusive_scan<GSYNC>(__popc(bits), wsum, &tot);
        while (bits) {
            const int k = __ffs(bits) - 1;
            bits &= bits - 1;
            emit(lo + k, pos++);
        }
        count += tot;
    }
    return count;
}

// Two order-preserving compactions of [0, n) in one pass (one block scan of packed counts):
// cat(i) -> 0 (neither), 1 or 2; emit(i, cat, position within its category).  Returns the two
// counts.  Same ownership scheme as block_compact.
template <bool GSYNC = true, typename Cat, typename Emit>
__device__ __forceinline__ int2 block_compact2(int n, int *wsum, Cat cat, Emit emit) {
    const int nt = blockDim.x, t = threadIdx.x;
    int c1 = 0, c2 = 0;
    for (int base = 0; base < n; base += 32 * nt) {
        const int m = n - base < 32 * nt ? n - base : 32 * nt;
        const int per = (m + nt - 1) / nt;
        const int lo = base + t * per;
        const int hi = lo + per < base + m ? lo + per : base + m;
        unsigned b1 = 0, b2 = 0;
        for (int i = lo; i < hi; ++i) {
            const int c = cat(i);
            if (c == 1) b1 |= 1u << (i - lo);
            else if (c == 2) b2 |= 1u << (i - lo);
        }
        int tot;   // counts <= 32 * 1024 each: 16 bits apiece
        const int ex = block_exclusive_scan<GSYNC>(__popc(b1) | (__popc(b2) << 16), wsum, &tot);
        int p1 = c1 + (ex & 0xFFFF), p2 = c2 + (ex >> 16);
        while (b1 | b2) {
            const int k1 = b1 ? __ffs(b1) - 1 : 32, k2 = b2 ? __ffs(b2) - 1 : 32;
            if (k1 < k2) {
                b1 &= b1 - 1;
                emit(lo + k1, 1, p1++);
            } else {
                b2 &= b2 - 1;
                emit(lo + k2, 2, p2++);
            }
        }
        c1 += tot & 0xFFFF;
        c2 += tot >> 16;
    }
    return make_int2(c1, c2);
}

// block_compact for items whose predicate needs memory loads, as a two-level gather: a thread owns
// a contiguous run of <= PER indices per pass, issues every first-level load of its run
// (first(i) -> K, typically a list entry), then every second-level load (second(i, k) -> V, the
// entry's record), and only then tests them (pred(i, v)); emit(i, v, position) gets the loaded
// value.  A load chain written inside one per-item call would cost a round trip per item: the
// compiler cannot issue item b + 1's index load ahead of item b's dependent load.
// One block scan per PER * blockDim items.
template <int PER, bool GSYNC = true, typename First, typename Second, typename Pred,
          typename Emit>
__device__ __forceinline__ int block_compact_ld(int n, int *wsum, First first, Second second,
                                                Pred pred, Emit emit) {
    const int nt = blockDim.x, t = threadIdx.x;
    using K = decltype(first(0));
    using V = decltype(second(0, first(0)));
    int count = 0;
    for (int base = 0; base < n; base += PER * nt) {
        const int m = n - base < PER * nt ? n - base : PER * nt;
        const int per = (m + nt - 1) / nt;
        const int lo = base + t * per;
        const int hi = lo + per < base + m ? lo + per : base + m;
        K kk[PER];
        V v[PER];
        if (lo < hi) {   // loads unconditional within the run (items past it load the run's last
                         // item, unused): a guarded load compiles to a branch and a wait per item
#pragma unroll
            for (int k = 0; k < PER; ++k) kk[k] = first(lo + k < hi ? lo + k : hi - 1);
#pragma unroll
            for (int k = 0; k < PER; ++k) v[k] = second(lo + k < hi ? lo + k : hi - 1, kk[k]);
        }
        unsigned bits = 0;
#pragma unroll
        for (int k = 0; k < PER; ++k)
            if (lo + k < hi && pred(lo + k, v[k])) bits |= 1u << k;
        int tot;
        int pos = count + block_exclusive_scan<GSYNC>(__popc(bits), wsum, &tot);
#pragma unroll
        for (int k = 0; k < PER; ++k)
            if ((bits >> k) & 1u) emit(lo + k, v[k], pos++);
        count += tot;
    }
    return count;
}

// Strided loop over [0, n) as a two-level gather (see block_compact_ld): B items per thread per
// step, first-level loads of all of them, then their second-level loads, then use(i, v).
template <int B, typename First, typename Second, typename Use>
__device__ __forceinline__ void batched_for2(int n, First first, Second second, Use use) {
    const int t = threadIdx.x, nt = blockDim.x;
    using K = decltype(first(0));
    using V = decltype(second(0, first(0)));
    for (int base = t; base < n; base += B * nt) {
        K kk[B];
        V v[B];
        // unconditional loads (items past n load item `base`, unused): see block_compact_ld
#pragma unroll
        for (int b = 0; b < B; ++b) kk[b] = first(base + b * nt < n ? base + b * nt : base);
#pragma unroll
        for (int b = 0; b < B; ++b) v[b] = second(base + b * nt < n ? base + b * nt : base, kk[b]);
#pragma unroll
        for (int b = 0; b < B; ++b)
            if (base + b * nt < n) use(base + b * nt, v[b]);
    }
}

// Strided loop over [0, n) that issues the loads of B iterations before using any of them, so
// their latencies overlap: load(i) -> value, use(i, value).
template <int B, typename Load, typename Use>
__device__ __forceinline__ void batched_for(int n, Load load, Use use) {
    const int t = threadIdx.x, nt = blockDim.x;
    using V = decltype(load(0));
    for (int base = t; base < n; base += B * nt) {
        V v[B];
#pragma unroll
        for (int b = 0; b < B; ++b) {   // unconditional loads: see block_compact_ld
            const int i = base + b * nt;
            v[b] = load(i < n ? i : base);
        }
#pragma unroll
        for (int b = 0; b < B; ++b) {
            const int i = base + b * nt;
            if (i < n) use(i, v[b]);
        }
    }
}

// NumPy's np.maximum / np.minimum for float64 (NaN-propagating; first operand wins on ties).
__host__ __device__ __forceinline__ double np_max(double a, double b) { return (a >= b || a != a) ? a : b; }
__host__ __device__ __forceinline__ double np_min(double a, double b) { return (a <= b || a != a) ? a : b; }

}  // namespace yta
