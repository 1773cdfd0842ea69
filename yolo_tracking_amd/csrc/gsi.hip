// GSI post-processing (boxmot/postprocessing/gsi.py:12-72) on gfx950: gap interpolation of the
// MOT result table and one Gaussian-process smoother per track.
//
//   k_gsi_gaps    [grid]  per sorted row: frames missing between it and the previous row of the
//                         same id (gsi.py:18-21), inclusive scan (hipCUB) -> output positions
//   k_gsi_fill    [grid]  every row copied to its output position, the missing frames written in
//                         front of it: row_pre + ((row - row_pre) / (f_curr - f_pre)) * i (:22-23)
//   k_gsi_gp      [block / track]  GaussianProcessRegressor(RBF(l, 'fixed')).fit(t, y).predict(t)
//                         for the 4 box columns at once (:40-54): K + 1e-10 I in band storage,
//                         right-looking Cholesky, forward / backward substitution, K_trans @ alpha
//
// Band storage.  K(i, j) = exp(-0.5 (t_i / l - t_j / l)^2) (sklearn kernels.py:1556-1565).  The
// host passes per track the band width w = max(i - j) over the pairs with (t_i/l - t_j/l)^2 <= 120;
// every pair outside the band has K < e^-60 (8.8e-27) and is dropped.  The Cholesky factor of a
// banded matrix stays inside the band, so the factorisation is exact on the stored entries; the
// dropped entries move a prediction by less than 1e-10 px even at the 1e-10 regulariser's
// condition number.  Row i of a track holds K(i, i - w .. i) at
// band[i * (w + 1) + (i - j)].
#include <hipcub/hipcub.hpp>

#include <vector>

#include "common.hpp"

namespace yta {
namespace {

constexpr double GP_ALPHA = 1e-10;   // GaussianProcessRegressor(alpha=1e-10), the default
constexpr int GP_T = 256;

struct GsiBuf {
    std::vector<void *> ptrs;
    ~GsiBuf() {
        for (void *p : ptrs) (void)hipFree(p);
    }
    template <typename T>
    hipError_t get(T **p, size_t n) {
        void *q = nullptr;
        hipError_t e = hipMalloc(&q, sizeof(T) * (n ? n : 1));
        if (e == hipSuccess) ptrs.push_back(q);
        *p = (T *)q;
        return e;
    }
};

// frame / id of a row as gsi.py:18 reads them: row[:2].astype(int) (truncation)
__device__ __forceinline__ long long as_int(double v) { return (long long)v; }

// gaps[i] = rows to insert in front of sorted row i.  virt0: the first row's id is -1, which
// equals the initial id_pre (gsi.py:16), so it pairs with a zero row at frame -1.
__global__ void k_gsi_gaps(const double *rows, int n, int ncol, int interval, int virt0,
                           long long *gaps) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double *row = rows + (long long)i * ncol;
    const long long f = as_int(row[0]), id = as_int(row[1]);
    long long fp, idp;
    if (i > 0) {
        fp = as_int(row[-ncol]);
        idp = as_int(row[1 - ncol]);
    } else if (virt0) {
        fp = -1;
        idp = -1;
    } else {
        gaps[i] = 0;
        return;
    }
    gaps[i] = (id == idp && fp + 1 < f && f < fp + interval) ? f - fp - 1 : 0;
}

__global__ void k_gsi_fill(const double *rows, int n, int ncol, int virt0, const long long *gaps,
                           const long long *incl, double *out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double *row = rows + (long long)i * ncol;
    const long long g = gaps[i], pos = i + incl[i];
    double *dst = out + pos * ncol;
    for (int c = 0; c < ncol; ++c) dst[c] = row[c];
    if (g == 0) return;
    const bool zero_prev = i == 0;   // virt0 (gaps[0] > 0 only then)
    (void)virt0;
    const double *prev = zero_prev ? nullptr : row - ncol;
    const long long f = as_int(row[0]), fp = zero_prev ? -1 : as_int(prev[0]);
    const double d = (double)(f - fp);
    for (long long m = 1; m <= g; ++m) {
        double *o = out + (pos - g + m - 1) * ncol;
        for (int c = 0; c < ncol; ++c) {
            const double p = zero_prev ? 0.0 : prev[c];
            o[c] = p + ((row[c] - p) / d) * (double)m;   // row_pre + (row - row_pre) / d * i
        }
    }
}

// One block per track.  t (frames), y (n x 4 box columns) and out (n x 4) at the track's row
// offset; band its workspace (n * (w + 1) doubles); rhs n x 4 doubles of workspace.
__global__ __launch_bounds__(GP_T) void k_gsi_gp(const double *t_all, const double *y_all,
                                                 const int *off, const double *lscale,
                                                 const int *width, const long long *band_off,
                                                 double *band_all, double *rhs_all,
                                                 double *out_all, int *err) {
    const int k = blockIdx.x, tid = threadIdx.x;
    const int r0 = off[k], n = off[k + 1] - r0, w = width[k];
    if (n <= 0) return;
    const double l = lscale[k];
    const double *t = t_all + r0;
    const double *y = y_all + (long long)r0 * 4;
    double *z = rhs_all + (long long)r0 * 4;
    double *o = out_all + (long long)r0 * 4;
    double *B = band_all + band_off[k];
    const int W = w + 1;
    auto kern = [&](int i, int j) {                       // RBF with fill_diagonal(K, 1)
        if (i == j) return 1.0;
        const double d = t[i] / l - t[j] / l;
        return exp(-0.5 * (d * d));
    };
    // K + alpha I on the band, the right-hand sides copied
    for (long long e = tid; e < (long long)n * W; e += GP_T) {
        const int i = (int)(e / W), q = (int)(e - (long long)i * W), j = i - q;
        B[e] = j < 0 ? 0.0 : (q == 0 ? 1.0 + GP_ALPHA : kern(i, j));
    }
    for (int e = tid; e < 4 * n; e += GP_T) z[e] = y[e];
    block_sync();
    // Cholesky, column by column: L_kk = sqrt(A_kk), L_ik = A_ik / L_kk, then the trailing band
    // A_ij -= L_ik L_jk for k < j <= i <= k + w
    for (int c = 0; c < n; ++c) {
        const double akk = B[(long long)c * W];
        if (!(akk > 0.0)) {                               // not positive definite
            if (tid == 0) atomicOr(err, 1);
            return;                                       // block-uniform
        }
        const double lkk = sqrt(akk);
        const int hi = c + w < n - 1 ? c + w : n - 1;    // rows c+1 .. hi hold column c
        for (int i = c + 1 + tid; i <= hi; i += GP_T) B[(long long)i * W + (i - c)] /= lkk;
        if (tid == 0) B[(long long)c * W] = lkk;
        block_sync();
        const int m = hi - c;                             // trailing rows
        for (int e = tid; e < m * m; e += GP_T) {
            const int ii = e / m, jj = e - ii * m;
            if (jj > ii) continue;
            const int i = c + 1 + ii, j = c + 1 + jj;
            B[(long long)i * W + (i - j)] -= B[(long long)i * W + (i - c)] * B[(long long)j * W + (j - c)];
        }
        block_sync();
    }
    // forward: L z = y (4 columns)
    for (int c = 0; c < n; ++c) {
        const double lkk = B[(long long)c * W];
        const int hi = c + w < n - 1 ? c + w : n - 1;
        double zc[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) zc[r] = z[4 * c + r] / lkk;
        block_sync();
        if (tid == 0)
            for (int r = 0; r < 4; ++r) z[4 * c + r] = zc[r];
        for (int e = tid; e < 4 * (hi - c); e += GP_T) {
            const int i = c + 1 + e / 4, r = e & 3;
            z[4 * i + r] -= B[(long long)i * W + (i - c)] * zc[r];
        }
        block_sync();
    }
    // backward: L^T a = z
    for (int c = n - 1; c >= 0; --c) {
        const double lkk = B[(long long)c * W];
        const int lo = c - w > 0 ? c - w : 0;
        double ac[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) ac[r] = z[4 * c + r] / lkk;
        block_sync();
        if (tid == 0)
            for (int r = 0; r < 4; ++r) z[4 * c + r] = ac[r];
        for (int e = tid; e < 4 * (c - lo); e += GP_T) {
            const int j = lo + e / 4, r = e & 3;
            z[4 * j + r] -= B[(long long)c * W + (c - j)] * ac[r];   // (L^T)_jc = L_cj
        }
        block_sync();
    }
    // predict at the training inputs: y_mean_i = sum_j K(i, j) alpha_j (_gpr.py:444)
    for (int i = tid; i < n; i += GP_T) {
        double s[4] = {0.0, 0.0, 0.0, 0.0};
        for (int j = 0; j < n; ++j) {
            const double d = t[i] / l - t[j] / l;
            const double kij = exp(-0.5 * (d * d));
#pragma unroll
            for (int r = 0; r < 4; ++r) s[r] += kij * z[4 * j + r];
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) o[4 * i + r] = s[r];
    }
}

}  // namespace
}  // namespace yta

using namespace yta;

extern "C" {

int yta_gsi_interpolate(int device, const double *rows, int n, int ncol, int interval, int virt0,
                        double *out, long long out_cap, long long *n_out) {
    YTA_CHECK(n >= 0 && ncol >= 2 && n_out, YTA_ERR_INVALID, "bad arguments");
    *n_out = n;
    if (n == 0) return YTA_OK;
    YTA_CHECK(rows, YTA_ERR_INVALID, "null rows");
    int rc = select_device(device);
    if (rc) return rc;
    GsiBuf m;
    double *d_rows, *d_out;
    long long *d_gaps, *d_incl;
    YTA_HIP(m.get(&d_rows, (size_t)n * ncol));
    YTA_HIP(m.get(&d_gaps, n));
    YTA_HIP(m.get(&d_incl, n));
    YTA_HIP(hipMemcpy(d_rows, rows, sizeof(double) * n * ncol, hipMemcpyHostToDevice));
    const int T = 256, G = (n + T - 1) / T;
    hipLaunchKernelGGL(k_gsi_gaps, dim3(G), dim3(T), 0, 0, d_rows, n, ncol, interval, virt0,
                       d_gaps);
    YTA_HIP(hipGetLastError());
    size_t tmp_bytes = 0;
    YTA_HIP(hipcub::DeviceScan::InclusiveSum(nullptr, tmp_bytes, d_gaps, d_incl, n));
    char *d_tmp;
    YTA_HIP(m.get(&d_tmp, tmp_bytes));
    YTA_HIP(hipcub::DeviceScan::InclusiveSum(d_tmp, tmp_bytes, d_gaps, d_incl, n));
    long long extra = 0;
    YTA_HIP(hipMemcpy(&extra, d_incl + (n - 1), sizeof(long long), hipMemcpyDeviceToHost));
    *n_out = n + extra;
    YTA_CHECK(*n_out <= out_cap, YTA_ERR_CAPACITY, "output needs %lld rows (capacity %lld)",
              *n_out, out_cap);
    YTA_CHECK(out, YTA_ERR_INVALID, "null out");
    YTA_HIP(m.get(&d_out, (size_t)(*n_out) * ncol));
    hipLaunchKernelGGL(k_gsi_fill, dim3(G), dim3(T), 0, 0, d_rows, n, ncol, virt0, d_gaps, d_incl,
                       d_out);
    YTA_HIP(hipGetLastError());
    YTA_HIP(hipMemcpy(out, d_out, sizeof(double) * (*n_out) * ncol, hipMemcpyDeviceToHost));
    return YTA_OK;
}

int yta_gsi_smooth(int device, const double *t, const double *y, const int *track_off,
                   const double *len_scale, const int *band_width, int n_tracks, double *out) {
    YTA_CHECK(n_tracks >= 0, YTA_ERR_INVALID, "negative track count");
    if (n_tracks == 0) return YTA_OK;
    YTA_CHECK(t && y && track_off && len_scale && band_width && out, YTA_ERR_INVALID,
              "null buffer");
    const int N = track_off[n_tracks];
    YTA_CHECK(track_off[0] == 0 && N >= 0, YTA_ERR_INVALID, "bad track offsets");
    std::vector<long long> band_off(n_tracks + 1, 0);
    for (int k = 0; k < n_tracks; ++k) {
        const int n = track_off[k + 1] - track_off[k], w = band_width[k];
        YTA_CHECK(n >= 0 && w >= 0 && (n == 0 || w < n), YTA_ERR_INVALID,
                  "track %d: %d rows, band width %d", k, n, w);
        YTA_CHECK(len_scale[k] > 0.0, YTA_ERR_INVALID, "track %d: length scale %g", k, len_scale[k]);
        band_off[k + 1] = band_off[k] + (long long)n * (w + 1);
    }
    if (N == 0) return YTA_OK;
    int rc = select_device(device);
    if (rc) return rc;
    GsiBuf m;
    double *d_t, *d_y, *d_ls, *d_band, *d_rhs, *d_out;
    int *d_off, *d_w, *d_err;
    long long *d_boff;
    YTA_HIP(m.get(&d_t, N));
    YTA_HIP(m.get(&d_y, (size_t)N * 4));
    YTA_HIP(m.get(&d_ls, n_tracks));
    YTA_HIP(m.get(&d_off, n_tracks + 1));
    YTA_HIP(m.get(&d_w, n_tracks));
    YTA_HIP(m.get(&d_boff, n_tracks + 1));
    YTA_HIP(m.get(&d_band, band_off[n_tracks]));
    YTA_HIP(m.get(&d_rhs, (size_t)N * 4));
    YTA_HIP(m.get(&d_out, (size_t)N * 4));
    YTA_HIP(m.get(&d_err, 1));
    YTA_HIP(hipMemcpy(d_t, t, sizeof(double) * N, hipMemcpyHostToDevice));
    YTA_HIP(hipMemcpy(d_y, y, sizeof(double) * N * 4, hipMemcpyHostToDevice));
    YTA_HIP(hipMemcpy(d_ls, len_scale, sizeof(double) * n_tracks, hipMemcpyHostToDevice));
    YTA_HIP(hipMemcpy(d_off, track_off, sizeof(int) * (n_tracks + 1), hipMemcpyHostToDevice));
    YTA_HIP(hipMemcpy(d_w, band_width, sizeof(int) * n_tracks, hipMemcpyHostToDevice));
    YTA_HIP(hipMemcpy(d_boff, band_off.data(), sizeof(long long) * (n_tracks + 1),
                      hipMemcpyHostToDevice));
    YTA_HIP(hipMemset(d_err, 0, sizeof(int)));
    hipLaunchKernelGGL(k_gsi_gp, dim3(n_tracks), dim3(GP_T), 0, 0, d_t, d_y, d_off, d_ls, d_w,
                       d_boff, d_band, d_rhs, d_out, d_err);
    YTA_HIP(hipGetLastError());
    int herr = 0;
    YTA_HIP(hipMemcpy(&herr, d_err, sizeof(int), hipMemcpyDeviceToHost));
    YTA_CHECK(herr == 0, YTA_ERR_INVALID,
              "the kernel matrix of a track is not positive definite (sklearn raises LinAlgError)");
    YTA_HIP(hipMemcpy(out, d_out, sizeof(double) * N * 4, hipMemcpyDeviceToHost));
    return YTA_OK;
}

}  // extern "C"
