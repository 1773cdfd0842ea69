// Microbenchmark (tools only): k_apply's record pass with 256-B aligned records, read + written in
// place at random (or sorted) slots, writing 15 of the 16 16-B pieces (the pad untouched: the
// first line is written partially) or all 16.  Does a partial-line write cost extra on MI355X?
// hipcc --offload-arch=gfx950 -O3 -o tools/_diag/rmwbench tools/rmwbench.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <numeric>
#include <random>
#include <vector>

constexpr int T = 128;

template <int R, int W>   // pieces read / written per record (of 16)
__global__ __launch_bounds__(T) void k_coop(double2 *buf, const int *slot, int n) {
    __shared__ double2 rec[T][17];
    __shared__ int s_slot[T];
    const int i0 = blockIdx.x * T, t = threadIdx.x;
    const int nloc = min(T, n - i0);
    if (t < nloc) s_slot[t] = slot[i0 + t];
    __syncthreads();
    for (int p = t; p < nloc * R; p += T) {
        const int r = p / R, k = p - r * R;
        rec[r][k] = buf[(long long)s_slot[r] * 16 + k];
    }
    __syncthreads();
    if (t < nloc)
        for (int k = 0; k < 16; ++k) { rec[t][k].x += 1.0; rec[t][k].y *= 0.5; }
    __syncthreads();
    for (int p = t; p < nloc * W; p += T) {
        const int r = p / W, k = p - r * W;
        buf[(long long)s_slot[r] * 16 + k] = rec[r][k];
    }
}

int main() {
    const int N = 1 << 21;
    const int CAP = 2 * N;
    double2 *buf;
    int *dslot;
    hipMalloc(&buf, sizeof(double2) * 16 * (size_t)CAP);
    hipMemset(buf, 0, sizeof(double2) * 16 * (size_t)CAP);
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
    auto run = [&](const char *name, auto kern, double pieces) {
        const int blocks = (N + T - 1) / T;
        float best = 1e30f;
        for (int rep = 0; rep < 8; ++rep) {
            hipEventRecord(e0);
            hipLaunchKernelGGL(kern, dim3(blocks), dim3(T), 0, 0, buf, dslot, N);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            if (rep > 1) best = std::min(best, ms);
        }
        printf("%-22s %8.1f us  %7.0f GB/s (pieces moved)\n", name, best * 1e3,
               pieces * 16.0 * N / (best * 1e-3) / 1e9);
    };
    for (auto &pr : {std::make_pair("seq", &seq), std::make_pair("sorted", &sorted),
                     std::make_pair("random", &rnd)}) {
        hipMemcpy(dslot, pr.second->data(), sizeof(int) * N, hipMemcpyHostToDevice);
        printf("-- %s\n", pr.first);
        run("read 15 write 15", k_coop<15, 15>, 30);
        run("read 15 write 16", k_coop<15, 16>, 31);
        run("read 16 write 16", k_coop<16, 16>, 32);
        run("read 15 write 14", k_coop<15, 14>, 29);
    }
    return 0;
}
