// Microbenchmark (tools only): does a random 64-B read of a 128-B line cost 64 B or 128 B of HBM
// traffic on MI355X?  N records of 256 B (two lines) at random slots; each record read as
//   full   its first 128-B line (8 lanes x 16 B)
//   half   the first 64 B of that line (4 lanes x 16 B)
//   two    both lines (16 lanes x 16 B)
// hipcc --offload-arch=gfx950 -O3 -o tools/_diag/halfline tools/halfline.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <numeric>
#include <random>
#include <vector>

template <int L>   // lanes (16-B pieces) per record
__global__ __launch_bounds__(256) void k_gather(const double2 *buf, const int *slot, int n,
                                                double *out) {
    const int g = (blockIdx.x * 256 + threadIdx.x);
    const int rec = g / L, piece = g % L;
    double acc = 0.0;
    if (rec < n) {
        const double2 v = buf[(long long)slot[rec] * 16 + piece];
        acc = v.x + v.y;
    }
    if (acc == 1.2345e300) out[0] = acc;   // keeps the loads
}

int main() {
    const int n = 4 << 20;                  // 4 M records of 256 B = 1 GiB
    double2 *buf;
    int *slot;
    double *out;
    hipMalloc(&buf, (size_t)n * 256);
    hipMalloc(&slot, (size_t)n * 4);
    hipMalloc(&out, 8);
    hipMemset(buf, 0, (size_t)n * 256);
    std::vector<int> h(n);
    std::iota(h.begin(), h.end(), 0);
    std::shuffle(h.begin(), h.end(), std::mt19937(1));
    hipMemcpy(slot, h.data(), (size_t)n * 4, hipMemcpyHostToDevice);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto run = [&](const char *name, int L, auto kern) {
        const int blocks = (int)(((long long)n * L + 255) / 256);
        for (int it = 0; it < 3; ++it) hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, buf, slot, n, out);
        hipEventRecord(e0);
        const int reps = 10;
        for (int it = 0; it < reps; ++it) hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, buf, slot, n, out);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        const double us = 1e3 * ms / reps;
        printf("%-5s %8.1f us  %6.0f M records/s  %7.0f GB/s requested\n", name, us, n / us,
               (double)n * L * 16 / us / 1e3);
    };
    run("half", 4, k_gather<4>);
    run("full", 8, k_gather<8>);
    run("two", 16, k_gather<16>);
    return 0;
}
