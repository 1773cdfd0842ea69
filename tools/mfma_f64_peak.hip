// Measured f64 MFMA ceiling of the box (v_mfma_f64_16x16x4_f64, 8 independent accumulator
// chains per wave, no memory traffic in the loop): the peak the C3-C5 embedding-cost GEMMs
// (k_hs_emb / k_doc_emb / BoT-SORT stage 1) are priced against.  Build: hipcc --offload-arch=gfx950
// -O3 tools/mfma_f64_peak.hip -o tools/mfma_f64_peak; run on the GPU box.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double dbl4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_peak(double *out, int iters, double a0) {
    dbl4 acc[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) acc[c] = dbl4{0.0, 0.0, 0.0, 0.0};
    double a = a0 + threadIdx.x * 1e-9, b = a0 - threadIdx.x * 1e-9;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int c = 0; c < 8; ++c) acc[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[c], 0, 0, 0);
    }
    double s = 0.0;
#pragma unroll
    for (int c = 0; c < 8; ++c) s += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
    const int blocks = 256 * 8, threads = 256, iters = 4096;
    double *d;
    if (hipMalloc(&d, sizeof(double) * blocks * threads) != hipSuccess) return 1;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int rep = 0; rep < 4; ++rep) {
        hipEventRecord(e0);
        hipLaunchKernelGGL(k_peak, dim3(blocks), dim3(threads), 0, 0, d, iters, 1.0);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0.f;
        hipEventElapsedTime(&ms, e0, e1);
        const double flops = 2.0 * 16 * 16 * 4 * 8.0 * iters * (double)blocks * (threads / 64);
        printf("{\"kernel\": \"v_mfma_f64_16x16x4_f64\", \"rep\": %d, \"ms\": %.3f, \"tflops\": %.2f}\n",
               rep, ms, flops / (ms * 1e-3) / 1e12);
    }
    hipFree(d);
    return 0;
}
