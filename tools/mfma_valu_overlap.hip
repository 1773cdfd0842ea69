// Can f64 MFMA and f64 VALU work of different waves overlap on one SIMD (gfx950)?  The
// k_hs_emb question: its tile GEMM (v_mfma_f64_16x16x4_f64) and its f64 epilogue (div, sqrt,
// acos per corner) run back to back in every wave.  Four variants of the same total work per
// block (8 waves): A = every wave GEMM then epilogue-like VALU chain; B = waves 0-3 twice the GEMM,
// waves 4-7 twice the VALU chain (wave-specialised); C = GEMM only; D = VALU only.  B close to
// max(C, D) means a specialised kernel can hide the epilogue.  Build: hipcc --offload-arch=gfx950
// -O3 tools/mfma_valu_overlap.hip -o tools/mfma_valu_overlap; run on the GPU box.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double dbl4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void gemm_part(dbl4 *acc, double a, double b, int iters) {
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[c], 0, 0, 0);
    }
}

__device__ __forceinline__ double valu_part(double x, int iters) {
    double y = x + 0.25, z = x + 0.5, w = x + 0.75;
    for (int it = 0; it < iters; ++it) {   // four independent div / sqrt / acos chains
        x = acos(fmin(fmax(x / (sqrt(x * x + 1.0) + 1e-6), -1.0), 1.0)) * 0.3;
        y = acos(fmin(fmax(y / (sqrt(y * y + 1.0) + 1e-6), -1.0), 1.0)) * 0.3;
        z = acos(fmin(fmax(z / (sqrt(z * z + 1.0) + 1e-6), -1.0), 1.0)) * 0.3;
        w = acos(fmin(fmax(w / (sqrt(w * w + 1.0) + 1e-6), -1.0), 1.0)) * 0.3;
    }
    return x + y + z + w;
}

template <int MODE>
__global__ __launch_bounds__(512) void k_mix(double *out, int gi, int vi, double a0) {
    const int w = threadIdx.x >> 6;
    dbl4 acc[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[c] = dbl4{0.0, 0.0, 0.0, 0.0};
    double a = a0 + threadIdx.x * 1e-9, b = a0 - threadIdx.x * 1e-9, v = 0.0;
    if (MODE == 0) {
        gemm_part(acc, a, b, gi);
        v = valu_part(a, vi);
    } else if (MODE == 1) {
        if (w < 4) gemm_part(acc, a, b, 2 * gi);
        else v = valu_part(a, 2 * vi);
    } else if (MODE == 2) {
        gemm_part(acc, a, b, gi);
    } else {
        v = valu_part(a, vi);
    }
    double s = v;
#pragma unroll
    for (int c = 0; c < 4; ++c) s += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
    const int blocks = 256 * 4, threads = 512, gi = 512, vi = 48;
    double *d;
    if (hipMalloc(&d, sizeof(double) * blocks * threads) != hipSuccess) return 1;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const char *names[4] = {"A_seq_per_wave", "B_specialised", "C_gemm_only", "D_valu_only"};
    for (int rep = 0; rep < 3; ++rep)
        for (int m = 0; m < 4; ++m) {
            hipEventRecord(e0);
            switch (m) {
                case 0: hipLaunchKernelGGL(k_mix<0>, dim3(blocks), dim3(threads), 0, 0, d, gi, vi, 0.3); break;
                case 1: hipLaunchKernelGGL(k_mix<1>, dim3(blocks), dim3(threads), 0, 0, d, gi, vi, 0.3); break;
                case 2: hipLaunchKernelGGL(k_mix<2>, dim3(blocks), dim3(threads), 0, 0, d, gi, vi, 0.3); break;
                default: hipLaunchKernelGGL(k_mix<3>, dim3(blocks), dim3(threads), 0, 0, d, gi, vi, 0.3); break;
            }
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0.f;
            hipEventElapsedTime(&ms, e0, e1);
            printf("{\"variant\": \"%s\", \"rep\": %d, \"ms\": %.3f}\n", names[m], rep, ms);
        }
    hipFree(d);
    return 0;
}
