// FETCH_SIZE calibration (tools only): known byte counts in k_apply's access pattern, so the
// rocprofv3 HBM counters of the tracker kernels can be read in bytes (MI355X_MICROARCH.md §HBM:
// "other access widths are uncalibrated: calibrate on a known byte count").
//   hipcc --offload-arch=gfx950 -O3 -o tools/_diag/fetch_calib tools/fetch_calib.hip
//   rocprofv3 --pmc FETCH_SIZE -- tools/_diag/fetch_calib    (then WRITE_SIZE in its own pass)
// Kernels (each reads a known number of bytes from buffers far beyond the 256 MiB Infinity Cache):
//   k_stream   1 GiB read, 16 B per lane, consecutive lanes on consecutive 16-B pieces
//   k_gather   N random 256-B records, the first 240 B of each (15 pieces) loaded straight into LDS
//              with consecutive lanes on consecutive pieces (k_apply's global_load_lds gather)
//   k_scatter  the same records written back from LDS (WRITE_SIZE)
//   k_line0_32 k_finish's duplicate-removal read: one lane per random record, the record's first
//              32 B (the Kalman mean's box half: two 16-B loads) - N distinct 128-B lines touched
//   k_line0_80 k_finish's output-row read: one lane per random record, 32 B at offset 0 and the
//              48-B meta at offset 64 (five 16-B loads) - N distinct 128-B lines touched
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <numeric>
#include <random>
#include <vector>

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void glob_void;

constexpr int T = 128, P = 15, STRIDE = 16;   // pieces read per record, pieces per record

__global__ __launch_bounds__(256) void k_stream(const double2 *src, long long n, double *sink) {
    double acc = 0.0;
    for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
        const double2 v = src[i];
        acc += v.x + v.y;
    }
    if (acc == 12345.678) sink[0] = acc;   // never true: keeps the loads
}

__global__ __launch_bounds__(T) void k_gather(const double2 *rec, const int *slot, int n,
                                              double *sink) {
    __shared__ double2 buf[T][P];
    __shared__ int s_slot[T];
    const int i0 = blockIdx.x * T, t = threadIdx.x;
    s_slot[t] = i0 + t < n ? slot[i0 + t] : -1;
    __syncthreads();
    char *ldsb = reinterpret_cast<char *>(&buf[0][0]);
    const int wb = __builtin_amdgcn_readfirstlane(t & ~63);
#pragma unroll
    for (int q = 0; q < P; ++q) {
        const int p = t + q * T, r = p / P, k = p - r * P;
        const int rs = s_slot[r];
        if (rs >= 0)
            __builtin_amdgcn_global_load_lds((glob_void *)(rec + (long long)rs * STRIDE + k),
                                             (lds_void *)(ldsb + (wb + q * T) * 16), 16, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    double acc = 0.0;
    for (int k = 0; k < P; ++k) acc += buf[t][k].x;
    if (acc == 12345.678) sink[0] = acc;
}

__global__ __launch_bounds__(T) void k_scatter(double2 *rec, const int *slot, int n) {
    const int i0 = blockIdx.x * T, t = threadIdx.x;
    for (int p = t; p < T * P; p += T) {
        const int r = p / P, k = p - r * P;
        if (i0 + r < n) rec[(long long)slot[i0 + r] * STRIDE + k] = make_double2(r, k);
    }
}

__global__ __launch_bounds__(256) void k_line0_32(const double2 *rec, const int *slot, int n,
                                                   double *sink) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const double2 *r = rec + (long long)slot[i] * STRIDE;
    const double2 a = r[0], b = r[1];
    if (a.x + a.y + b.x + b.y == 12345.678) sink[0] = a.x;
}

__global__ __launch_bounds__(256) void k_line0_80(const double2 *rec, const int *slot, int n,
                                                   double *sink) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const double2 *r = rec + (long long)slot[i] * STRIDE;
    const double2 a = r[0], b = r[1], m0 = r[4], m1 = r[5], m2 = r[6];
    if (a.x + a.y + b.x + b.y + m0.x + m1.y + m2.x == 12345.678) sink[0] = a.x;
}

int main() {
    const long long NS = (1LL << 30) / 16;   // 1 GiB of 16-B pieces
    const int CAP = 1 << 21, N = 1 << 20;    // 512 MiB of 256-B records, 1 Mi of them gathered
    double2 *src, *rec;
    double *sink;
    int *dslot;
    hipMalloc(&src, 16 * NS);
    hipMalloc(&rec, 256LL * CAP);
    hipMalloc(&sink, 8);
    hipMalloc(&dslot, 4LL * N);
    hipMemset(src, 0, 16 * NS);
    hipMemset(rec, 0, 256LL * CAP);
    std::vector<int> perm(CAP);
    std::iota(perm.begin(), perm.end(), 0);
    std::shuffle(perm.begin(), perm.end(), std::mt19937(7));
    hipMemcpy(dslot, perm.data(), 4LL * N, hipMemcpyHostToDevice);
    hipDeviceSynchronize();
    k_stream<<<4096, 256>>>(src, NS, sink);
    k_gather<<<N / T, T>>>(rec, dslot, N, sink);
    k_scatter<<<N / T, T>>>(rec, dslot, N);
    // fresh records for the line-0 reads (the scatter's lines may still sit in the caches)
    hipMemcpy(dslot, perm.data() + N, 4LL * N, hipMemcpyHostToDevice);
    k_line0_32<<<N / 256, 256>>>(rec, dslot, N, sink);
    std::shuffle(perm.begin(), perm.end(), std::mt19937(11));
    hipMemcpy(dslot, perm.data(), 4LL * N, hipMemcpyHostToDevice);
    k_stream<<<4096, 256>>>(src, NS, sink);   // flush the 256 MiB Infinity Cache between them
    k_line0_80<<<N / 256, 256>>>(rec, dslot, N, sink);
    hipDeviceSynchronize();
    printf("k_stream reads %lld B; k_gather reads %lld B (%d records x %d B); k_scatter writes %lld B\n",
           16 * NS, 240LL * N, N, 240, 240LL * N);
    printf("k_line0_32 reads %d records x 32 B (%d lines of 128 B); k_line0_80 reads %d x 80 B\n", N,
           N, N);
    return 0;
}
