// Host helpers for stream-subset updates of the OCSORT-family engines (SURVEY.md §8(b):
// update(ctx, n_streams, stream_ids, ...)).  In the reference every camera stream is its own
// tracker (examples/track.py:43-57); a stream without a new frame is simply not called.  The
// engines run one launch per kernel over all S streams; a [S] mask makes the kernels of the
// streams not listed return at once (Args::active), so their state is untouched.
#pragma once
#include <hip/hip_runtime.h>

#include <cstring>
#include <vector>

#include "common.hpp"

namespace yta {

struct StreamMask {
    const int *req_host = nullptr;   // host mask [S] for the next host-buffer update
    const int *req_dev = nullptr;    // device mask [S] for the next device-buffer update
    int *d = nullptr, *h = nullptr;  // device copy of req_host and its pinned staging

    void release() {
        if (d) (void)hipFree(d);
        if (h) (void)hipHostFree(h);
        d = h = nullptr;
    }
    // The mask of the launch being enqueued on `st` (nullptr: every stream).  The host update
    // calls are synchronous, so the pinned staging is free whenever this runs.
    int stage(int S, hipStream_t st, const int **active) {
        *active = req_dev;
        if (!req_host) return YTA_OK;
        if (!d) {
            YTA_HIP(hipMalloc((void **)&d, sizeof(int) * S));
            YTA_HIP(hipHostMalloc((void **)&h, sizeof(int) * S, hipHostMallocDefault));
        }
        memcpy(h, req_host, sizeof(int) * S);
        YTA_HIP(hipMemcpyAsync(d, h, sizeof(int) * S, hipMemcpyHostToDevice, st));
        *active = d;
        return YTA_OK;
    }
};

// A subset call expanded to the engine's S streams: the mask, the S + 1 detection offsets (0
// detections for the streams not listed), and the position of each listed stream.
inline int subset_expand(int S, int n, const int *ids, const int *det_offsets,
                         std::vector<int> &mask, std::vector<int> &off) {
    YTA_CHECK(ids && det_offsets, YTA_ERR_INVALID, "null argument");
    YTA_CHECK(n >= 1 && n <= S, YTA_ERR_INVALID, "n_streams %d outside 1..%d", n, S);
    YTA_CHECK(det_offsets[0] == 0, YTA_ERR_INVALID, "det_offsets[0] must be 0");
    for (int k = 0; k < n; ++k)
        YTA_CHECK(ids[k] >= 0 && ids[k] < S && (k == 0 || ids[k] > ids[k - 1]), YTA_ERR_INVALID,
                  "stream_ids must be ascending and within 0..%d", S - 1);
    mask.assign(S, 0);
    off.assign(S + 1, 0);
    for (int k = 0; k < n; ++k) mask[ids[k]] = 1;
    for (int s = 0, k = 0; s < S; ++s) {
        int m = 0;
        if (mask[s]) {
            m = det_offsets[k + 1] - det_offsets[k];
            YTA_CHECK(m >= 0, YTA_ERR_INVALID, "det_offsets must be non-decreasing");
            ++k;
        }
        off[s + 1] = off[s] + m;
    }
    return YTA_OK;
}

// Per-stream rows of `width` values for the listed streams, spread over all S (fill elsewhere).
template <typename T>
std::vector<T> subset_spread(int S, int n, const int *ids, const T *v, int width, T fill) {
    std::vector<T> out((size_t)S * width, fill);
    for (int k = 0; k < n; ++k)
        for (int c = 0; c < width; ++c) out[(size_t)ids[k] * width + c] = v[(size_t)k * width + c];
    return out;
}

// The S + 1 output offsets of the full call compacted to the listed streams (the others have no
// rows, so the packed rows are already the subset's).
inline void subset_compact(int n, const int *ids, const std::vector<int> &full, int *out_offsets) {
    out_offsets[0] = 0;
    for (int k = 0; k < n; ++k)
        out_offsets[k + 1] = out_offsets[k] + (full[ids[k] + 1] - full[ids[k]]);
}

}  // namespace yta
