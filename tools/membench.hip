// Memory-pattern microbenchmark (tools only): what k_apply's access pattern can reach on MI355X.
//   hipcc --offload-arch=gfx950 -O3 -o tools/_diag/membench tools/membench.hip
// Patterns (N records of 240 B = 15 x 16 B, read + written in place):
//   seq      record r at slot r
//   sorted   slots increasing with random gaps (a live tracker's slot order)
//   random   random permutation of slots
// Two code shapes: "lane" (each lane moves its own record: 15 strided 16-B loads/stores) and
// "coop" (consecutive lanes on consecutive 16-B pieces, staged through LDS).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <numeric>
#include <random>
#include <vector>

constexpr int P = 15;
constexpr int T = 128;

__global__ __launch_bounds__(T) void k_lane(double2 *buf, const int *slot, int n) {
    const int i = blockIdx.x * T + threadIdx.x;
    if (i >= n) return;
    double2 *r = buf + (long long)slot[i] * P;
    double2 v[P];
#pragma unroll
    for (int k = 0; k < P; ++k) v[k] = r[k];
#pragma unroll
    for (int k = 0; k < P; ++k) { v[k].x += 1.0; v[k].y *= 0.5; }
#pragma unroll
    for (int k = 0; k < P; ++k) r[k] = v[k];
}

__global__ __launch_bounds__(T) void k_coop(double2 *buf, const int *slot, int n) {
    __shared__ double2 rec[T][P];
    __shared__ int s_slot[T];
    const int i0 = blockIdx.x * T, t = threadIdx.x;
    const int nloc = min(T, n - i0);
    if (t < nloc) s_slot[t] = slot[i0 + t];
    __syncthreads();
    for (int p = t; p < nloc * P; p += T) {
        const int r = p / P, k = p - r * P;
        rec[r][k] = buf[(long long)s_slot[r] * P + k];
    }
    __syncthreads();
    if (t < nloc)
        for (int k = 0; k < P; ++k) { rec[t][k].x += 1.0; rec[t][k].y *= 0.5; }
    __syncthreads();
    for (int p = t; p < nloc * P; p += T) {
        const int r = p / P, k = p - r * P;
        buf[(long long)s_slot[r] * P + k] = rec[r][k];
    }
}

int main() {
    const int N = 1 << 21;              // 2M records (~1.4M live tracks at 1024 streams)
    const int CAP = 3 * N / 2;          // slots
    double2 *buf;
    int *dslot;
    hipMalloc(&buf, sizeof(double2) * P * (size_t)CAP);
    hipMemset(buf, 0, sizeof(double2) * P * (size_t)CAP);
    hipMalloc(&dslot, sizeof(int) * N);
    std::mt19937 rng(1);
    std::vector<int> seq(N), sorted(N), rnd(N);
    std::iota(seq.begin(), seq.end(), 0);
    {
        std::vector<int> all(CAP);
        std::iota(all.begin(), all.end(), 0);
        std::shuffle(all.begin(), all.end(), rng);
        std::copy(all.begin(), all.begin() + N, sorted.begin());
        std::sort(sorted.begin(), sorted.end());
        std::copy(all.begin(), all.begin() + N, rnd.begin());
    }
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const double bytes = 2.0 * N * P * 16;
    for (int shape = 0; shape < 2; ++shape)
        for (auto &pr : {std::make_pair("seq", &seq), std::make_pair("sorted", &sorted),
                         std::make_pair("random", &rnd)}) {
            hipMemcpy(dslot, pr.second->data(), sizeof(int) * N, hipMemcpyHostToDevice);
            const int blocks = (N + T - 1) / T;
            float best = 1e30f;
            for (int rep = 0; rep < 6; ++rep) {
                hipEventRecord(e0);
                if (shape == 0) hipLaunchKernelGGL(k_lane, dim3(blocks), dim3(T), 0, 0, buf, dslot, N);
                else hipLaunchKernelGGL(k_coop, dim3(blocks), dim3(T), 0, 0, buf, dslot, N);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms;
                hipEventElapsedTime(&ms, e0, e1);
                if (rep > 0) best = std::min(best, ms);
            }
            printf("%-5s %-7s %8.1f us  %7.0f GB/s (read+write)\n", shape ? "coop" : "lane", pr.first,
                   best * 1e3, bytes / (best * 1e-3) / 1e9);
        }
    return 0;
}
