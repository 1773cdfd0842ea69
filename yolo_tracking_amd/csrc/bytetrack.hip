// ByteTrack update() for S independent streams on gfx950, all state resident in HBM.
//
// Follows boxmot/trackers/bytetrack/byte_tracker.py:132-325.  One frame = 8 launches, each
// covering all S streams ("block/stream" kernels do the order-preserving list algebra with
// block-wide scans; "grid" kernels spread per-track work over the whole chip):
//   k_begin   [block/stream]  frame_id++, confidence split (:149-158), STrack box conversions
//                             (:14-25), grids over high / low detections, tracked -> activated /
//                             unconfirmed, pool = act ++ lost (:169-178), predicted pool boxes
//                             (mean only, :35-48), unconfirmed boxes (not predicted)
//   edges     [grid]          stage 1: pool x high, fused IoU (:181-183)
//   lap       [block/stream]  lapjv cost_limit = match_thresh (:184-186)
//   k_prep23  [block/stream]  leftovers = unmatched Tracked rows (:205-209), rest = unmatched
//                             high dets (:229)
//   edges     [grid]          stage 2: leftovers x low dets, IoU (:210); stage 3: unconfirmed x
//                             rest, fused IoU (:230-232)
//   lap       [block/problem] cost_limit 0.5 (:211) and 0.7 (:233)
//   k_apply   [grid]          Kalman predict of every pool track + update of every matched track
//                             (stages 1-3; :188-196, :212-220, :234-236), mark lost (:222-226) /
//                             removed (:237-240); each track's state is read and written once
//   k_finish  [block/stream]  births (:242-248), lost expiry (:250-253), joint/sub list algebra
//                             incl. the removed_stracks quirk (:257-265), duplicate removal
//                             (:312-325) through a grid over the lost list, output rows (:270-281),
//                             free-slot list
#include <chrono>
#include <algorithm>
#include <cmath>
#include <cstring>
#include <memory>
#include <new>
#include <thread>
#include <vector>

#include "bytetrack.hpp"
#include "host_pool.hpp"

namespace yta {
namespace {

// Threads per block of the block/stream kernels.  k_stage1 is one long latency-bound chain per
// stream: the widest block shortens it.  k_stage23 (small problems) and k_finish run better as
// several narrower blocks per CU.
#ifndef YTA_BLK1
#define YTA_BLK1 1024
#endif
#ifndef YTA_BLK23
#define YTA_BLK23 256
#endif
#ifndef YTA_BLKF
#define YTA_BLKF 256
#endif
constexpr int BLK1 = YTA_BLK1, BLK23 = YTA_BLK23, BLKF = YTA_BLKF;
constexpr int BLK_MAX = 1024;
constexpr int SLAB_WAVES = BLK_MAX / WAVE;   // solver slabs per stream (any block size)
static_assert(2 * YTA_BLK23 / WAVE <= SLAB_WAVES, "k_stage23's two blocks take disjoint slabs");

__device__ __forceinline__ void store_kf(double *kf, long long slot, const KfState &s) {
    double2 *dst = reinterpret_cast<double2 *>(kf + slot * TRK_STRIDE);
#pragma unroll
    for (int k = 0; k < 12; ++k) {   // mean: pieces 0-3, covariance: pieces 8-15
        const double *src = k < 4 ? s.m + 2 * k : s.c + 2 * (k - 4);
        dst[k < 4 ? k : TRK_COV / 2 + (k - 4)] = make_double2(src[0], src[1]);
    }
}

// STrack.xyxy of a track's current mean: ByteTrack (xc, yc, a, h) (byte_tracker.py:100-111),
// BoT-SORT (xc, yc, w, h) (bot_sort.py:173-182)
template <int V>
__device__ __forceinline__ Box kf_box(const double *kf, long long slot) {
    const double2 *m = reinterpret_cast<const double2 *>(kf + slot * TRK_STRIDE);
    const double2 a = m[0], b = m[1];
    if (V == VAR_BOTSORT) {
        const double xywh[4] = {a.x, a.y, b.x, b.y};
        return xywh_to_box(xywh);
    }
    return xyah_mean_to_box(a.x, a.y, b.x, b.y);
}

template <int V> constexpr int kf_model() { return V == VAR_BOTSORT ? KF_XYWH : KF_XYAH; }

// A detection's normalised ReID feature as the reference holds it: the row e of get_features,
// divided in place by its norm twice at STrack construction (bot_sort.py:40-48):
// curr_feat = (e / n1) / n2, elementwise in float32.
struct DetFeat {
    const float *e;
    float n1, n2;
    __device__ __forceinline__ float operator()(int k) const { return (e[k] / n1) / n2; }
};
__device__ __forceinline__ DetFeat det_feat(const BtArgs &a, int s, long long db, int d) {
    const float *fn = a.det_fn + (db + d) * 4;
    return DetFeat{a.det_feat + ((long long)a.det_off[s] + d) * a.D, fn[0], fn[1]};
}

__device__ __forceinline__ int st_of(int flags) { return flags & FL_STATE; }

__host__ __device__ __forceinline__ TrackMeta &bt_meta(const BtArgs &a, long long slot) {
    return *reinterpret_cast<TrackMeta *>(a.kf + slot * TRK_STRIDE + TRK_META);
}


// ------------------------------------------------------------------------------------ k_stage1
// Per stream: frame_id++, confidence split (:149-158), STrack box conversions (:14-25),
// tracked -> activated / unconfirmed, pool = act ++ lost (:169-178), predicted pool boxes (mean
// only, multi_predict :35-48 zeroes vh of non-tracked tracks; the covariance is advanced in
// k_apply), unconfirmed boxes (not predicted), then stage 1: pool x high detections, fused IoU
// (:181-183), lapjv with cost_limit = match_thresh (:184-186).
__device__ __forceinline__ LapSlab slab_of(const BtArgs &a, int s) {
    LapSlab l = a.slab;
    l.i += (long long)s * SLAB_WAVES * l.i_stride;
    l.d += (long long)s * SLAB_WAVES * l.d_stride;
    return l;
}

struct StageShared {
    AssocShared as;
};

// The lists of stage 1 (everything before the association): detections split, pool and
// unconfirmed lists with their boxes.
struct S1Lists {
    int nd, n_high, n_second, n_act, n_unc, n_pool;
    Box *hbox;       // the high detections' boxes / scores staged in the arena (or nullptr)
    double *hw;
};

template <int V>
__device__ __forceinline__ S1Lists stage1_lists(const BtArgs &a, int s, Arena &ar,
                                                StageShared &sh) {
    int *wsum = sh.as.lap.wsum;
    const int t = threadIdx.x, nt = blockDim.x;
    BtCounters *c = a.cnt + s;
    const long long db = (long long)s * a.MAXD, tb = (long long)s * a.CAP;
    int nd = a.det_off[s + 1] - a.det_off[s];
    if (nd > a.MAXD || nd < 0) {
        if (t == 0) atomicOr(&c->err, ERR_DET_CAPACITY);
        nd = nd < 0 ? 0 : a.MAXD;
    }
    const double *din = a.det_in + (long long)a.det_off[s] * 6;
    const double thr = a.track_thresh;
    auto det_box = [&](int i) {                          // STrack.xyxy with mean None (:105-106)
        const double *d = din + (long long)i * 6;
        double xywh[4];
        det_xyxy_to_xywh(d, xywh);
        return xywh_to_box(xywh);
    };
    // the high detections' boxes / scores staged in the arena for the stage-1 grid (top end,
    // sized for every detection; skipped when the arena has no room)
    Box *hbox = ar.try_alloc_top<Box>(nd);
    double *hw = hbox ? ar.try_alloc_top<double>(nd) : nullptr;
    if (!hw) hbox = nullptr;
    // detections: STrack conversions (:16-18) and the confidence split (:149-158), one pass
    const int2 hs = block_compact2(
        nd, wsum,
        [&](int i) {
            const double conf = din[(long long)i * 6 + 4];
            // byte_tracker.py:149-158 (low bound 0.1) / bot_sort.py:263-269 (track_low_thresh)
            return conf > thr ? 1 : (conf > a.low_thresh && conf < thr ? 2 : 0);
        },
        [&](int i, int cat, int pos) {
            const Box b = det_box(i);
            if (cat == 1) {
                const double conf = din[(long long)i * 6 + 4];
                a.high[db + pos] = i;
                a.high_box[db + pos] = b;
                a.high_score[db + pos] = conf;
                if (hbox) {
                    hbox[pos] = b;
                    hw[pos] = conf;
                }
            } else {
                a.second[db + pos] = i;
                a.second_box[db + pos] = b;
            }
        });
    const int n_high = hs.x, n_second = hs.y;
    YTA_STAMP(2);
    // tracked -> activated (pool head) / unconfirmed (:169-178), with their boxes: predicted for
    // the pool (mean only; multi_predict :35-48 zeroes vh of non-tracked tracks, the covariance is
    // advanced in k_apply), current for the unconfirmed (not predicted)
    const int n_tracked = c->n_tracked, n_lost = c->n_lost;
    const int *tracked = a.tracked + tb;
    // BoT-SORT: this frame's camera warp (multi_gmc after multi_predict, bot_sort.py:290-295)
    const double *H = V == VAR_BOTSORT ? a.warp + 6LL * s : nullptr;
    const bool gmc = V == VAR_BOTSORT && !warp_is_identity(H);
    auto warped = [&](double *p) {     // kron(I4, R) on (x, y), (w, h); t on (x, y) (kf_gmc)
        const double x = p[0], y = p[1], w = p[2], h = p[3];
        p[0] = (H[0] * x + H[1] * y) + H[2];
        p[1] = (H[3] * x + H[4] * y) + H[5];
        p[2] = H[0] * w + H[1] * h;
        p[3] = H[3] * w + H[4] * h;
    };
    auto pred_box = [&](long long slot, bool lost_list) {
        const double *m = a.kf + slot * TRK_STRIDE;
        const bool trk = st_of(a.flags[slot]) == ST_TRACKED;
        if (V == VAR_BYTETRACK && lost_list) {   // lazily predicted (kf_xyah.hpp)
            double ml[8];
            for (int k = 0; k < 8; ++k) ml[k] = m[k];
            kf_predict_lost_mean(ml, c->frame_id - a.kf_frame[slot]);
            return xyah_mean_to_box(ml[0] + ml[4], ml[1] + ml[5], ml[2] + ml[6], ml[3]);
        }
        const double vh = trk ? m[7] : 0.0;
        if (V == VAR_BOTSORT) {   // multi_predict zeroes vw and vh of non-tracked (:80-93)
            double p[4] = {m[0] + m[4], m[1] + m[5], m[2] + (trk ? m[6] : 0.0), m[3] + vh};
            if (gmc) warped(p);
            return xywh_to_box(p);
        }
        return xyah_mean_to_box(m[0] + m[4], m[1] + m[5], m[2] + m[6], m[3] + vh);
    };
    auto unc_box_of = [&](long long slot) {   // unconfirmed: not predicted, warped (:295)
        if (V == VAR_BOTSORT && gmc) {
            const double *m = a.kf + slot * TRK_STRIDE;
            double p[4] = {m[0], m[1], m[2], m[3]};
            warped(p);
            return xywh_to_box(p);
        }
        return kf_box<V>(a.kf, slot);
    };
    const int2 au = block_compact2(
        n_tracked, wsum,
        [&](int i) { return (a.flags[tb + tracked[i]] & FL_ACTIVATED) ? 1 : 2; },
        [&](int i, int cat, int pos) {
            const int slot = tracked[i];
            if (cat == 1) {
                a.pool[tb + pos] = slot;
                a.pool_box[tb + pos] = pred_box(tb + slot, false);
            } else {
                a.unc[tb + pos] = slot;
                a.unc_box[tb + pos] = unc_box_of(tb + slot);
            }
        });
    const int n_act = au.x, n_unc = au.y;
    for (int i = t; i < n_lost; i += nt) {
        const int slot = a.lost[tb + i];
        a.pool[tb + n_act + i] = slot;
        a.pool_box[tb + n_act + i] = pred_box(tb + slot, true);
    }
    const int n_pool = n_act + n_lost;
    block_sync();
    YTA_STAMP(4);
    return S1Lists{nd, n_high, n_second, n_act, n_unc, n_pool, hbox, hw};
}

// Stage 1's association over the lists (bot_sort.py:307-322 / byte_tracker.py:181-186).
template <int V>
__device__ __forceinline__ bool stage1_assoc(const BtArgs &a, int s, const S1Lists &L, Arena &ar,
                                             StageShared &sh) {
    BtCounters *c = a.cnt + s;
    const long long db = (long long)s * a.MAXD, tb = (long long)s * a.CAP;
    const int n_pool = L.n_pool, n_high = L.n_high;
    Box *hbox = L.hbox;
    double *hw = L.hw;
    bool ok;
    if (V == VAR_BOTSORT && a.D > 0)   // min(iou, gated appearance) (bot_sort.py:307-322)
        ok = assoc_block_emb(
            n_pool, [&](int i) { return a.pool_box[tb + i]; }, n_high,
            [&](int j) { return a.high_box[db + j]; }, a.fuse_first != 0,
            [&](int j) { return a.high_score[db + j]; },
            [&](int i) { return a.feat + (tb + a.pool[tb + i]) * a.D; },
            [&](int j) { return det_feat(a, s, db, a.high[db + j]); }, a.D, a.prox_thresh,
            a.app_thresh, a.match_thresh, a.x1 + tb, a.y1 + db, &c->err, &c->n_edges[0], ar,
            slab_of(a, s), sh.as);
    else   // ByteTrack: fused IoU (:181-183); BoT-SORT without ReID: IoU, fused if fuse_first
        ok = assoc_block(
            n_pool, [&](int i) { return a.pool_box[tb + i]; }, n_high,
            [&](int j) { return a.high_box[db + j]; }, V == VAR_BYTETRACK || a.fuse_first != 0,
            [&](int j) { return a.high_score[db + j]; }, a.match_thresh, a.x1 + tb, a.y1 + db,
            &c->err, &c->n_edges[0], ar, slab_of(a, s), sh.as, hbox, hw);
    return ok;
}

// The frame's stage-1 counters (frame_id advances with them unless `advance` is false: the split
// BoT-SORT stage 1 advances it in k_bs_lap, after the solve)
__device__ __forceinline__ void stage1_commit(BtCounters *c, const S1Lists &L, bool advance) {
    if (threadIdx.x != 0) return;
    if (advance) c->frame_id += 1;
    c->n_dets = L.nd;
    c->n_high = L.n_high;
    c->n_second = L.n_second;
    c->n_act = L.n_act;
    c->n_unc = L.n_unc;
    c->n_pool = L.n_pool;
    c->n_left = 0;
    c->n_rest = 0;
    c->n_births = 0;
    c->n_lazy = 0;
    c->n_res1 = 0;
    c->n_ref = 0;
}

template <int V>
__device__ __forceinline__ bool stage1_body(const BtArgs &a, int s, Arena &ar, StageShared &sh) {
    const S1Lists L = stage1_lists<V>(a, s, ar, sh);
    if (!stage1_assoc<V>(a, s, L, ar, sh)) return false;
    stage1_commit(a.cnt + s, L, true);
    return true;
}

// ------------------------------------------------------------------------------------ k_stage23
// Per stream: leftovers = unmatched Tracked pool rows (:205-209) x low detections, IoU, cost_limit
// 0.5 (:210-211); rest = unmatched high detections (:229); unconfirmed x rest, fused IoU,
// cost_limit 0.7 (:230-233).
// role -1: both stages in this block; 0: stage 2 only (leftovers, re-found); 1: stage 3 only (the
// rest of the high detections), its solver slabs after stage 2's (split23: one block each).
template <int V>
__device__ __forceinline__ bool stage23_body(const BtArgs &a, int s, Arena &ar, StageShared &sh,
                                             int role = -1) {
    int *wsum = sh.as.lap.wsum;
    const int t = threadIdx.x, nt = blockDim.x;
    BtCounters *c = a.cnt + s;
    const long long tb = (long long)s * a.CAP, db = (long long)s * a.MAXD;
    const int n_pool = c->n_pool, n_high = c->n_high, n_second = c->n_second, n_unc = c->n_unc;
    const int n_act = c->n_act;
    LapSlab slab = slab_of(a, s);
    if (role == 1) {
        slab.i += (long long)(nt / WAVE) * slab.i_stride;
        slab.d += (long long)(nt / WAVE) * slab.d_stride;
    }
    int n_left = 0, n_ref = 0, n_rest = 0;
    bool ok = true;
    if (role <= 0) {
        for (int i = t; i < n_pool; i += nt) a.left_of_pool[tb + i] = -1;
        block_sync();
        // leftovers: the pool's Tracked rows (its head, the activated tracks: pool = act ++ lost)
        // left unmatched in stage 1 (:205-209)
        n_left = block_compact_ld<8>(
            n_act, wsum, [&](int i) { return a.x1[tb + i]; }, [&](int, int h) { return h; },
            [&](int, int h) { return h < 0; },
            [&](int i, int, int pos) {
                a.left[tb + pos] = i;
                a.left_of_pool[tb + i] = pos;
            });
        // re-found: the pool's Lost rows matched in stage 1 (refind_stracks, :193-196), pool order,
        // with their slot and detection (k_apply visits these and no other Lost row)
        n_ref = block_compact_ld<8>(
            n_pool - n_act, wsum,
            [&](int k) { return make_int2(a.pool[tb + n_act + k], a.x1[tb + n_act + k]); },
            [&](int, int2 v) { return v; }, [&](int, const int2 &v) { return v.y >= 0; },
            [&](int, const int2 &v, int pos) { a.refound[tb + pos] = v; });
    }
    if (role != 0)
        n_rest = block_compact(n_high, wsum, [&](int h) { return a.y1[db + h] < 0; },
                               [&](int h, int pos) {
                                   a.rest[db + pos] = h;
                                   a.rest_score[db + pos] = a.high_score[db + h];
                               });
    block_sync();
    YTA_STAMP(4);
    if (role <= 0) {
        ok = assoc_block(
            n_left, [&](int k) { return a.pool_box[tb + a.left[tb + k]]; }, n_second,
            [&](int q) { return a.second_box[db + q]; }, false, [&](int) { return 1.0; }, 0.5,
            a.x2 + tb, a.y2 + db, &c->err, &c->n_edges[1], ar, slab, sh.as);
        if (!ok) return false;
        ar.reset();
    }
    if (role == 0) {
        if (t == 0) {
            c->n_left = n_left;
            c->n_ref = n_ref;
            c->n_lazy = V == VAR_BYTETRACK ? n_pool - n_act - n_ref : 0;
        }
        return true;
    }
    YTA_STAMP_BASE(40);
    YTA_STAMP(0);
    if (V == VAR_BOTSORT && a.D > 0)   // bot_sort.py:355-370
        ok = assoc_block_emb(
            n_unc, [&](int j) { return a.unc_box[tb + j]; }, n_rest,
            [&](int r) { return a.high_box[db + a.rest[db + r]]; }, true,
            [&](int r) { return a.rest_score[db + r]; },
            [&](int j) { return a.feat + (tb + a.unc[tb + j]) * a.D; },
            [&](int r) { return det_feat(a, s, db, a.high[db + a.rest[db + r]]); }, a.D,
            a.prox_thresh, a.app_thresh, 0.7, a.x3 + tb, a.y3 + db, &c->err, &c->n_edges[2], ar,
            slab, sh.as);
    else
        ok = assoc_block(
            n_unc, [&](int j) { return a.unc_box[tb + j]; }, n_rest,
            [&](int r) { return a.high_box[db + a.rest[db + r]]; }, true,
            [&](int r) { return a.rest_score[db + r]; }, 0.7, a.x3 + tb, a.y3 + db, &c->err,
            &c->n_edges[2], ar, slab, sh.as);
    if (!ok) return false;
    YTA_STAMP(15);
    if (t == 0) {
        c->n_rest = n_rest;
        if (role < 0) {
            c->n_left = n_left;
            c->n_ref = n_ref;
            // ByteTrack: the Lost rows k_apply leaves untouched (lazy prediction)
            c->n_lazy = V == VAR_BYTETRACK ? n_pool - n_act - n_ref : 0;
        }
    }
    return true;
}

// ---- pooled global fallback arenas ---------------------------------------------------------
// A stream-frame whose association does not fit its LDS arena is redone over a global arena.
// Sized for the worst case (every pair a candidate edge), one such arena per stream costs
// S x O(CAP x MAXD) bytes (154 GB for 2048 streams at CAP 3072 x MAXD 2048); fallbacks are rare
// (none in the headline's steady state), so the engine keeps a pool of ws_slots arenas.  A
// launch with no more blocks than arenas (few streams) redoes in place over arena blockIdx; in a
// larger launch the block that falls back queues its block id (redo_queue) and returns, and the
// launch's redo kernel (k_redo_*, ws_slots blocks, right behind it on the same stream) takes
// queued block q, q + ws_slots, ... on arena blockIdx.x (redo_drain).  The last redo block out
// clears the queue for the next launch.  (An in-kernel claim of a pooled arena - a bitmap,
// released after the redo - put code behind the second inlined body: k_stage23 went from 120
// VGPRs to 167 with 696 B of scratch, k_s1_lap and k_finish spilled, and the headline fell from
// 2.0 M to 1.5 M calls/s, gpurun_out/r6t.)
// A launch of at most ws_slots association blocks (few streams) has an arena per block: its blocks
// redo in place over arena `block` and no redo kernel is launched (redo_launch).
__device__ __forceinline__ bool redo_in_place(const BtArgs &a, int blocks) { return blocks <= a.ws_slots; }
__device__ __forceinline__ unsigned char *redo_arena(const BtArgs &a, int block) {
    return a.ws + (long long)block * a.ws_stride;
}
__device__ __forceinline__ void redo_queue(const BtArgs &a, int block) {
    const int q = atomicAdd(&a.redo_q[0], 1);
    a.redo_q[2 + q] = block;
}
// redo(block id, arena) -> false: the arena was too small as well (ERR_EDGE_OVERFLOW)
template <class Redo>
__device__ __forceinline__ void redo_drain(const BtArgs &a, Redo &&redo) {
    const int n = __builtin_amdgcn_readfirstlane(a.redo_q[0]);
    for (int q = blockIdx.x; q < n; q += gridDim.x) {
        Arena ag(redo_arena(a, blockIdx.x), a.ws_stride);
        redo(__builtin_amdgcn_readfirstlane(a.redo_q[2 + q]), ag);
        block_sync();
    }
    __syncthreads();   // every thread has read the count
    if (threadIdx.x == 0) {
        __threadfence();
        if (atomicAdd(&a.redo_q[1], 1) == (int)gridDim.x - 1) {
            atomicExch(&a.redo_q[0], 0);
            atomicExch(&a.redo_q[1], 0);
        }
    }
}

// LDS first; a frame whose association does not fit is redone by k_redo_stage1 over a global
// arena (the body only writes values that the redo rewrites identically, and bumps the frame
// counter only on success).
template <int V>
__global__ __launch_bounds__(BLK1) void k_stage1(BtArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    __shared__ StageShared sh;
    const int s = blockIdx.x;
    if (stream_skipped(a, s)) return;
    YTA_STAMP_BASE(0);
    YTA_STAMP(0);
    Arena ar(smem, a.lds_bytes);
    if (stage1_body<V>(a, s, ar, sh)) return;
    block_sync();
    if (threadIdx.x == 0) a.cnt[s].n_fallback[0] += 1;
    if (redo_in_place(a, a.S)) {
        Arena ag(redo_arena(a, s), a.ws_stride);
        if (!stage1_body<V>(a, s, ag, sh) && threadIdx.x == 0)
            atomicOr(&a.cnt[s].err, ERR_EDGE_OVERFLOW);
    } else if (threadIdx.x == 0) {
        redo_queue(a, s);
    }
}
template <int V>
__global__ __launch_bounds__(BLK1) void k_redo_stage1(BtArgs a) {
    __shared__ StageShared sh;
    redo_drain(a, [&](int s, Arena &ag) {
        if (!stage1_body<V>(a, s, ag, sh) && threadIdx.x == 0)
            atomicOr(&a.cnt[s].err, ERR_EDGE_OVERFLOW);
    });
}

// SPLIT (a.split23): two blocks per stream, block 2s + r running role r; else one block per
// stream with both stages (role -1 a constant: the one-block kernel keeps its registers).
// The split blocks take BLK23S threads (few streams: the chip is idle but for them).
constexpr int BLK23S = 512;
static_assert(2 * BLK23S / WAVE <= SLAB_WAVES, "k_stage23's two blocks take disjoint slabs");
template <int V, bool SPLIT>
__global__ __launch_bounds__(SPLIT ? BLK23S : BLK23) void k_stage23(BtArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    __shared__ StageShared sh;
    const int s = SPLIT ? blockIdx.x >> 1 : blockIdx.x;
    const int role = SPLIT ? (int)(blockIdx.x & 1) : -1;
    if (stream_skipped(a, s)) return;
    YTA_STAMP_BASE(20);
    YTA_STAMP(0);
    YTA_BLK(3, 0);
    Arena ar(smem, a.lds_bytes23);
    if (stage23_body<V>(a, s, ar, sh, role)) {
        YTA_BLK(3, 1);
        return;
    }
    block_sync();
    // a stream-frame is counted once: the split blocks mark it, k_finish counts the mark
    if (threadIdx.x == 0) {
        if (SPLIT) atomicOr(&a.cnt[s].fb23_mark, 1);
        else atomicAdd(&a.cnt[s].n_fallback[1], 1);
    }
    if (redo_in_place(a, SPLIT ? 2 * a.S : a.S)) {
        Arena ag(redo_arena(a, blockIdx.x), a.ws_stride);
        if (!stage23_body<V>(a, s, ag, sh, role) && threadIdx.x == 0)
            atomicOr(&a.cnt[s].err, ERR_EDGE_OVERFLOW);
    } else if (threadIdx.x == 0) {
        redo_queue(a, blockIdx.x);
    }
}
template <int V, bool SPLIT>
__global__ __launch_bounds__(SPLIT ? BLK23S : BLK23) void k_redo_stage23(BtArgs a) {
    __shared__ StageShared sh;
    redo_drain(a, [&](int b, Arena &ag) {
        const int s = SPLIT ? b >> 1 : b;
        if (!stage23_body<V>(a, s, ag, sh, SPLIT ? (b & 1) : -1) && threadIdx.x == 0)
            atomicOr(&a.cnt[s].err, ERR_EDGE_OVERFLOW);
    });
}

// ------------------------------------------------------------------ ByteTrack stage 1, split
// k_stage1's work for ByteTrack (match_thresh <= 1) as three launches that keep several streams
// on every CU (the fused kernel holds one 1024-thread stream per CU, its 150 KiB arena, for the
// whole latency chain of the frame).  Under load a dependent HBM round trip costs microseconds,
// so every pass issues all of a thread's loads before using any, and hand-offs that go through
// LDS only do not drain global stores (lds_sync):
//   k_s1_prep  [block/stream, 256 thr, 32 KiB static LDS] detection pass and confidence split
//              (:149-158), tracked -> activated / unconfirmed, pool = act ++ lost with predicted
//              boxes (:169-178, multi_predict's mean :35-48); coalesced loads, items staged in
//              LDS per pass (holding a run of items per thread in registers measured 1.6x slower:
//              strided rows, uncoalesced stores)
//   k_s1_edges [block/stream, 512 thr, <= 58 KiB LDS] grid over the high detections built in
//              LDS from two register-held detections per thread, then every pool row's candidate
//              edges, fused IoU cost (:181-183, matching.py:117, :216-220) below match_thresh:
//              count + the first E_SLOTS edges to HBM (the grid goes to HBM too when some row
//              has more)
//   k_s1_lap   [block/stream, 256 thr] CSR of the edges in LDS (rows with more edges query the
//              grid in HBM), lap_block with cost_limit = match_thresh (:184-186) on LDS, the
//              assignment written out; a frame that does not fit the LDS arena is redone over
//              global memory
// Same results as k_stage1: edges are exactly the pairs with cost < match_thresh whatever the
// grid's cell order, and lap_block's result does not depend on the order of a row's edges.
constexpr int PREP_T = 256;          // k_s1_prep threads
#ifndef YTA_PREP_CH
#define YTA_PREP_CH 768
#endif
constexpr int PREP_CH = YTA_PREP_CH;  // items staged in LDS per pass of k_s1_prep
#ifndef YTA_BLKE
#define YTA_BLKE 512
#endif
constexpr int BLKE = YTA_BLKE;       // k_s1_edges threads
#ifndef YTA_BLKL
#define YTA_BLKL 256
#endif
constexpr int BLKL = YTA_BLKL;       // k_s1_lap threads

struct PrepShared {
    union {
        struct {
            Box box[PREP_CH];
#if YTA_PREP_CH <= 768
            double conf[PREP_CH];
#endif
            unsigned char cat[PREP_CH];
        } d;                          // detections of the current pass
        struct {
            Box box[PREP_CH];
            int slot[PREP_CH];
            unsigned char cat[PREP_CH];
        } t;                          // tracked tracks of the current pass
    } u;
    int wsum[32];
};

struct DetRow {
    double v[6];
};
struct TrkRec {
    int slot, flags;
    double m[8];
};

// STrack.xyxy of multi_predict's mean (zeroed vh unless Tracked), byte_tracker.py:35-48, :100-111
__device__ __forceinline__ Box bt_pred_box(const TrkRec &r) {
    const double vh = st_of(r.flags) == ST_TRACKED ? r.m[7] : 0.0;
    return xyah_mean_to_box(r.m[0] + r.m[4], r.m[1] + r.m[5], r.m[2] + r.m[6], r.m[3] + vh);
}
__device__ __forceinline__ TrkRec bt_trk_rec(const BtArgs &a, long long tb, int slot) {
    TrkRec r;
    r.slot = slot;
    r.flags = a.flags[tb + slot];
    const double2 *m = reinterpret_cast<const double2 *>(a.kf + (tb + slot) * TRK_STRIDE);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const double2 q = m[k];
        r.m[2 * k] = q.x;
        r.m[2 * k + 1] = q.y;
    }
    return r;
}

// The stage-1 pool of the NEXT frame from the current tracked / lost lists (:169-178): tracked ->
// activated (pool head, multi_predict's predicted box :35-48) / unconfirmed (current box), pool
// tail = the lost tracks, lazily predicted (kf_xyah.hpp).  k_finish builds it at the end of every
// frame from the rows it already has in registers (finish_next_pool); this block-per-stream form
// (k_pool_build) rebuilds it after a reserve, which moves the records.
__device__ __forceinline__ void s1_pool_build(const BtArgs &a, int s, PrepShared &sh) {
    const int t = threadIdx.x;
    BtCounters *c = a.cnt + s;
    const long long tb = (long long)s * a.CAP;
    // tracked -> activated (pool head, predicted box) / unconfirmed (current box) (:169-178)
    const int n_tracked = c->n_tracked, n_lost = c->n_lost;
    int n_act = 0, n_unc = 0;
    for (int c0 = 0; c0 < n_tracked; c0 += PREP_CH) {
        const int m = n_tracked - c0 < PREP_CH ? n_tracked - c0 : PREP_CH;
        batched_for2<3>(
            m, [&](int i) { return a.tracked[tb + c0 + i]; },
            [&](int, int slot) { return bt_trk_rec(a, tb, slot); },
            [&](int i, const TrkRec &r) {
                const bool act = (r.flags & FL_ACTIVATED) != 0;
                sh.u.t.cat[i] = act ? 1 : 2;
                sh.u.t.slot[i] = r.slot;
                sh.u.t.box[i] = act ? bt_pred_box(r) : xyah_mean_to_box(r.m[0], r.m[1], r.m[2], r.m[3]);
            });
        lds_sync();
        const int2 au = block_compact2<false>(
            m, sh.wsum, [&](int i) { return (int)sh.u.t.cat[i]; },
            [&](int i, int cat, int pos) {
                if (cat == 1) {
                    const long long p = tb + n_act + pos;
                    a.pool[p] = sh.u.t.slot[i];
                    a.pool_box[p] = sh.u.t.box[i];
                } else {
                    const long long p = tb + n_unc + pos;
                    a.unc[p] = sh.u.t.slot[i];
                    a.unc_box[p] = sh.u.t.box[i];
                }
            });
        n_act += au.x;
        n_unc += au.y;
        lds_sync();
    }
    // pool tail: the lost tracks, predicted (their predicts since they were lost replayed first)
    const int fid_prev = c->frame_id;
    batched_for2<3>(
        n_lost, [&](int i) { return a.lost[tb + i]; },
        [&](int, int slot) {
            TrkRec r = bt_trk_rec(a, tb, slot);
            r.flags = fid_prev - a.kf_frame[tb + slot];   // pending predicts (state is Lost)
            return r;
        },
        [&](int i, TrkRec r) {
            kf_predict_lost_mean(r.m, r.flags);
            r.flags = ST_LOST;
            a.pool[tb + n_act + i] = r.slot;
            a.pool_box[tb + n_act + i] = bt_pred_box(r);
        });
    if (t == 0) {
        c->n_act = n_act;
        c->n_unc = n_unc;
        c->n_pool = n_act + n_lost;
    }
}

__global__ __launch_bounds__(PREP_T) void k_pool_build(BtArgs a) {
    __shared__ PrepShared sh;
    const int s = blockIdx.x;
    if (stream_skipped(a, s)) return;
    s1_pool_build(a, s, sh);
}

// NT: PREP_T, or 1024 with few streams (split23: one block per stream takes the lists)
template <int NT>
__global__ __launch_bounds__(NT) void k_s1_prep(BtArgs a) {
    __shared__ PrepShared sh;
    const int s = blockIdx.x, t = threadIdx.x;
    if (stream_skipped(a, s)) return;
    YTA_STAMP_BASE(60);
    YTA_STAMP(0);
    YTA_BLK(0, 0);
    BtCounters *c = a.cnt + s;
    const long long db = (long long)s * a.MAXD;
    int nd = a.det_off[s + 1] - a.det_off[s];
    if (nd > a.MAXD || nd < 0) {
        if (t == 0) atomicOr(&c->err, ERR_DET_CAPACITY);
        nd = nd < 0 ? 0 : a.MAXD;
    }
    const double *din = a.det_in + (long long)a.det_off[s] * 6;
    const double thr = a.track_thresh;
    // detections, PREP_CH per pass (coalesced loads, 3 rows in flight per thread): STrack
    // conversions (:16-18), measurement, confidence split (:149-158), boxes staged in LDS, then
    // the order-preserving high / second lists
    int n_high = 0, n_second = 0;
    for (int c0 = 0; c0 < nd; c0 += PREP_CH) {
        const int m = nd - c0 < PREP_CH ? nd - c0 : PREP_CH;
        batched_for<3>(
            m,
            [&](int i) {
                DetRow r;
                const double *d = din + (long long)(c0 + i) * 6;
#pragma unroll
                for (int k = 0; k < 6; ++k) r.v[k] = d[k];
                return r;
            },
            [&](int i, const DetRow &r) {
                double xywh[4];
                det_xyxy_to_xywh(r.v, xywh);
                const double conf = r.v[4];
                sh.u.d.cat[i] = conf > thr ? 1 : (conf > a.low_thresh && conf < thr ? 2 : 0);
                sh.u.d.box[i] = xywh_to_box(xywh);
#if YTA_PREP_CH <= 768
                sh.u.d.conf[i] = conf;
#endif
            });
        lds_sync();
        const int2 hs = block_compact2<false>(
            m, sh.wsum, [&](int i) { return (int)sh.u.d.cat[i]; },
            [&](int i, int cat, int pos) {
                if (cat == 1) {
                    const long long p = db + n_high + pos;
                    a.high[p] = c0 + i;
                    a.high_box[p] = sh.u.d.box[i];
#if YTA_PREP_CH <= 768
                    a.high_score[p] = sh.u.d.conf[i];
#else
                    a.high_score[p] = din[(long long)(c0 + i) * 6 + 4];   // L2-resident
#endif
                } else {
                    const long long p = db + n_second + pos;
                    a.second[p] = c0 + i;
                    a.second_box[p] = sh.u.d.box[i];
                }
            });
        n_high += hs.x;
        n_second += hs.y;
        lds_sync();   // the staging area is reused
    }
    YTA_STAMP(1);
    if (t == 0) {   // the pool (n_act / n_unc / n_pool) was built by the last k_finish
        c->frame_id += 1;
        c->n_dets = nd;
        c->n_high = n_high;
        c->n_second = n_second;
        c->n_left = 0;
        c->n_rest = 0;
        c->n_births = 0;
        c->n_lazy = 0;
        c->n_res1 = 0;
        c->n_ref = 0;
    }
    YTA_STAMP(3);
    YTA_BLK(0, 1);
}

// Every candidate edge of pool row box rb: f(high position, fused IoU cost) for cost <
// match_thresh.  gv: the stream's grid over its high detections (LDS or HBM); big items' boxes
// come from the high lists.
template <typename F>
__device__ __forceinline__ void s1_row_edges(const BtArgs &a, int s, const GridView &gv,
                                             const GridHdr &h, const Box &rb, F f) {
    const long long db = (long long)s * a.MAXD;
    const double thresh = a.match_thresh;
    auto scored = [&](int j, const Box &cb, double w) {
        const double dist = 1 - iou(rb, cb);                              // matching.py:117
        const double cost = 1 - (1 - dist) * w;                           // matching.py:216-220
        if (cost < thresh) f(j, cost);
    };
    grid_query(gv, h, rb, scored, [&](int j) {
        const Box cb = a.high_box[db + j];
        if (intersects(rb, cb)) scored(j, cb, a.high_score[db + j]);
    });
}

__device__ __forceinline__ GridView s1_grid_hbm(const BtArgs &a, int s) {
    const long long db = (long long)s * a.MAXD;
    return GridView{a.g_hdr + s, a.g_cell + (long long)s * (GRID_MAX_CELLS + 1), a.g_ids + db,
                    a.g_boxes + db, a.g_w + db, a.g_big + db};
}

// LDS bytes of a grid over C detections in k_s1_edges.
__host__ __device__ inline long long s1_grid_bytes(long long C) {
    return 4 * (GRID_MAX_CELLS + 1) + C * (4 + 32 + 8 + 4) + 5 * 16;
}

// k_s1_edges body over a grid whose storage (LDS or HBM) the caller fixed: inlined once per
// storage so that every grid access compiles to ds_* or global_* instructions, not flat ones.
// cdeg[nc]: every high detection's candidate-edge count (column degree), zeroed by the caller.
template <typename HBox, typename HW>
__device__ __forceinline__ void s1_edges_body(const BtArgs &a, int s, int nc, int nr,
                                              const GridView &gv, HBox hbox, HW hw,
                                              GridScratch &gs, int *wsum, int &spill, int *cdeg,
                                              int &n_edges, int (&rn)[4], int (&rc)[4]) {
    const int t = threadIdx.x, nt = blockDim.x;
    const long long tb = (long long)s * a.CAP, SC = (long long)a.S * a.CAP;
    grid_build(nc, hbox, hw, gv, gs, wsum);
    const GridHdr h = gs.hdr;
    YTA_STAMP(1);
    // pool rows, four per thread in flight
    for (int base = t; base < nr; base += 4 * nt) {
        Box rb[4];
#pragma unroll
        for (int b = 0; b < 4; ++b)
            if (base + b * nt < nr) rb[b] = a.pool_box[tb + base + b * nt];
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const int i = base + b * nt;
            if (i >= nr) continue;
            int n = 0, first = -1;
            s1_row_edges(a, s, gv, h, rb[b], [&](int j, double cost) {
                if (n == 0) first = j;
                if (n < E_SLOTS) {
                    a.e_col[n * SC + tb + i] = j;
                    a.e_cost[n * SC + tb + i] = cost;
                }
                ++n;
                atomicAdd(cdeg + j, 1);
            });
            a.e_cnt[tb + i] = n;
            if (n > E_SLOTS) spill = 1;
            if (n) atomicAdd(&n_edges, n);
            if (base == t) {   // rows t + b * nt: kept for the single-edge pass
                rn[b] = n;
                rc[b] = n == 1 ? first : -1;
            }
        }
    }
}

// The row phase of k_s1_edges over an LDS grid, one wave at a time on 64 pool rows (lane = row,
// rows t + m * blockDim as in s1_edges_body): each lane lists its row's grid candidates (the
// positions of the cells its window covers, contiguous per cell row) into the wave's queue at its
// prefix offset, then the wave scores the queue 64 candidates at a time, so a wave's trip count is
// its candidate total / 64 instead of its longest row, and consecutive lanes read consecutive
// grid positions (no LDS bank conflicts from 64 scattered 32-B boxes).  A row's box reaches the
// lane scoring its candidate by ds_bpermute.  Edges land in per-row LDS counters; their order
// within a row does not matter (lap_block, the single-edge pass and k_s1_lap's re-query are
// order-free).  Queues hold WQ_CAP entries; a larger candidate total is listed and scored in
// windows.  Big items (larger than 4 x the mean box) are visited per lane, as grid_query does.
constexpr int WQ_CAP = 384;
#ifndef YTA_S1_P1
#define YTA_S1_P1 1   // k_s1_edges' queue passes: two chunks per trip, branch-free tests (round 6)
#endif
#ifndef YTA_S1_SOA
#define YTA_S1_SOA 1   // k_s1_edges' LDS grid keeps its boxes as four arrays (GridView::sx)
#endif
__device__ __forceinline__ Box s1_box(const GridView &gv, int k) {
#if YTA_S1_SOA
    const double *x = gv.sx;
    const int n = gv.sn;
    return Box{x[k], x[n + k], x[2 * n + k], x[3 * n + k]};
#else
    return gv.boxes[k];
#endif
}
struct EdgeWaveQ {
    unsigned q[WQ_CAP];   // lane << 24 | grid position
    int cnt[WAVE];        // edges of the wave's row `lane`
    int first[WAVE];      // its first edge's detection
};

__device__ __forceinline__ double bperm_f64(double v, int src_lane) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_ds_bpermute(src_lane << 2, (int)b);
    const int hi = __builtin_amdgcn_ds_bpermute(src_lane << 2, (int)(b >> 32));
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

__device__ __forceinline__ void s1_edges_rows_wave(const BtArgs &a, int s, int nr,
                                                   const GridView &gv, const GridHdr &h,
                                                   EdgeWaveQ &wq, int &spill, int *cdeg,
                                                   int &n_edges, int (&rn)[4], int (&rc)[4]) {
    const int t = threadIdx.x, nt = blockDim.x, lane = lane_id();
    const long long tb = (long long)s * a.CAP, db = (long long)s * a.MAXD;
    const long long SC = (long long)a.S * a.CAP;
    const double thresh = a.match_thresh;
    int m = 0;
    for (int base = t - lane; base < nr; base += nt, ++m) {   // wave-uniform loop
        const int i = base + lane;
        const bool on = i < nr;
        Box rb{0.0, 0.0, 0.0, 0.0};
        if (on) rb = a.pool_box[tb + i];
        int cx0 = 0, cx1 = -1, cy0 = 0, cy1 = -1;
        if (!on || !grid_scan_window(h, rb, cx0, cx1, cy0, cy1)) cy1 = cy0 - 1;
        // this row's candidate count (cells of a grid row are contiguous)
        int cnt = 0;
        for (int cy = cy0; cy <= cy1; ++cy)
            cnt += gv.cell_start[cy * h.gx + cx1 + 1] - gv.cell_start[cy * h.gx + cx0];
        const int incl = wave_inclusive_scan(cnt);
        const int off = incl - cnt;
        const int total = __builtin_amdgcn_readlane(incl, WAVE - 1);
        wq.cnt[lane] = 0;
        wq.first[lane] = -1;
        for (int lo = 0; lo < total; lo += WQ_CAP) {
            const int hi = lo + WQ_CAP;
            // list this row's candidates whose wave index falls in [lo, hi)
            if (off < hi && off + cnt > lo) {
                int idx = off;
                for (int cy = cy0; cy <= cy1 && idx < hi; ++cy) {
                    const int b = gv.cell_start[cy * h.gx + cx0], e = gv.cell_start[cy * h.gx + cx1 + 1];
                    const int k0 = idx < lo ? lo - idx : 0;
                    const int k1 = idx + (e - b) < hi ? e - b : hi - idx;
                    for (int k = k0; k < k1; ++k) wq.q[idx + k - lo] = ((unsigned)lane << 24) | (unsigned)(b + k);
                    idx += e - b;
                }
            }
            __builtin_amdgcn_wave_barrier();
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            const int n = total - lo < WQ_CAP ? total - lo : WQ_CAP;
            // pass 1: keep the intersecting candidates (compacted in place: a survivor's new index
            // is at most its old one, and a chunk is read before any of it is overwritten)
            int ns = 0;
#if YTA_S1_P1
            // Two chunks of 64 per trip, every load of both issued before any test, and the test
            // branch-free: a queued row box has x2 > x1 and y2 > y1 (grid_scan_window lists
            // nothing otherwise, NaN included) and a binned box is usable, so intersects()
            // reduces to its four cross comparisons - the same predicate on every queued pair.
            // (The short-circuit form compiled to a chain of exec-masked LDS round trips.)
            const unsigned long long lt = (1ull << lane) - 1ull;
            for (int k0 = 0; k0 < n; k0 += 2 * WAVE) {   // wave-uniform trip count
                const int ka = k0 + lane, kb = ka + WAVE;
                const unsigned ea = wq.q[ka < n ? ka : 0], eb = wq.q[kb < n ? kb : 0];
                const int ra = (int)(ea >> 24), pa = (int)(ea & 0xFFFFFFu);
                const int rb_ = (int)(eb >> 24), pb = (int)(eb & 0xFFFFFFu);
                const Box A{bperm_f64(rb.x1, ra), bperm_f64(rb.y1, ra), bperm_f64(rb.x2, ra),
                            bperm_f64(rb.y2, ra)};
                const Box B{bperm_f64(rb.x1, rb_), bperm_f64(rb.y1, rb_), bperm_f64(rb.x2, rb_),
                            bperm_f64(rb.y2, rb_)};
                const Box ca = s1_box(gv, pa), cb = s1_box(gv, pb);
                const bool ha = (ka < n) & (A.x2 > ca.x1) & (ca.x2 > A.x1) & (A.y2 > ca.y1) &
                                (ca.y2 > A.y1);
                const bool hb = (kb < n) & (B.x2 > cb.x1) & (cb.x2 > B.x1) & (B.y2 > cb.y1) &
                                (cb.y2 > B.y1);
                const unsigned long long ba = __ballot(ha), bb = __ballot(hb);
                const int na = __popcll(ba);
                if (ha) wq.q[ns + __popcll(ba & lt)] = ea;
                if (hb) wq.q[ns + na + __popcll(bb & lt)] = eb;
                ns += na + __popcll(bb);
            }
#else
            for (int k0 = 0; k0 < n; k0 += WAVE) {   // wave-uniform trip count
                const int k = k0 + lane;
                const unsigned ent = k < n ? wq.q[k] : 0u;
                const int r = (int)(ent >> 24), pos = (int)(ent & 0xFFFFFFu);
                const Box tb_{bperm_f64(rb.x1, r), bperm_f64(rb.y1, r), bperm_f64(rb.x2, r),
                              bperm_f64(rb.y2, r)};
                const bool hit = k < n && intersects(tb_, s1_box(gv, pos));
                const unsigned long long bal = __ballot(hit);
                if (hit) wq.q[ns + __popcll(bal & ((1ull << lane) - 1ull))] = ent;
                ns += __popcll(bal);
            }
#endif
            __builtin_amdgcn_wave_barrier();
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            // pass 2: score the survivors (full lanes for the float64 IoU)
            for (int k0 = 0; k0 < ns; k0 += WAVE) {
                const int k = k0 + lane;
#if YTA_S1_P1   // every operand's load issued before the row box arrives and before any branch
                const unsigned ent = wq.q[k < ns ? k : 0];
                const int r = (int)(ent >> 24), pos = (int)(ent & 0xFFFFFFu);
                const Box cb = s1_box(gv, pos);
                const double wj = gv.w[pos];
                const int j = gv.ids[pos];
                const Box tb_{bperm_f64(rb.x1, r), bperm_f64(rb.y1, r), bperm_f64(rb.x2, r),
                              bperm_f64(rb.y2, r)};
                if (k >= ns) continue;
                const double dist = 1 - iou(tb_, cb);                   // matching.py:117
                const double cost = 1 - (1 - dist) * wj;                // matching.py:216-220
                if (!(cost < thresh)) continue;
#else
                const unsigned ent = k < ns ? wq.q[k] : 0u;
                const int r = (int)(ent >> 24), pos = (int)(ent & 0xFFFFFFu);
                const Box tb_{bperm_f64(rb.x1, r), bperm_f64(rb.y1, r), bperm_f64(rb.x2, r),
                              bperm_f64(rb.y2, r)};
                if (k >= ns) continue;
                const Box cb = s1_box(gv, pos);
                const double dist = 1 - iou(tb_, cb);                   // matching.py:117
                const double cost = 1 - (1 - dist) * gv.w[pos];         // matching.py:216-220
                if (!(cost < thresh)) continue;
                const int j = gv.ids[pos];
#endif
                const int c = atomicAdd(&wq.cnt[r], 1);
                if (c < E_SLOTS) {
                    a.e_col[c * SC + tb + base + r] = j;
                    a.e_cost[c * SC + tb + base + r] = cost;
                }
                if (c == 0) wq.first[r] = j;
                atomicAdd(cdeg + j, 1);
            }
            __builtin_amdgcn_wave_barrier();
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
        int nn = wq.cnt[lane];
        int first = wq.first[lane];
        // big items: every query visits them (grid_query), boxes from the high lists
        if (on)
            for (int k = 0; k < h.n_big; ++k) {
                const int j = gv.big[k];
                const Box cb = a.high_box[db + j];
                if (!intersects(rb, cb)) continue;
                const double dist = 1 - iou(rb, cb);
                const double cost = 1 - (1 - dist) * a.high_score[db + j];
                if (!(cost < thresh)) continue;
                if (nn < E_SLOTS) {
                    a.e_col[nn * SC + tb + i] = j;
                    a.e_cost[nn * SC + tb + i] = cost;
                }
                if (nn == 0) first = j;
                ++nn;
                atomicAdd(cdeg + j, 1);
            }
        if (on) {
            a.e_cnt[tb + i] = nn;
            if (nn > E_SLOTS) spill = 1;
            if (nn) atomicAdd(&n_edges, nn);
            if (m < 4) {   // rows t + m * nt: kept for the single-edge pass
                rn[m] = nn;
                rc[m] = nn == 1 ? first : -1;
            }
        }
        __builtin_amdgcn_wave_barrier();   // wq.cnt / first are reset by the next pass
    }
}

// Single-edge components (a pool row whose only candidate edge goes to a high detection no other
// row reaches) are matched outright here, as lap_block's P1 would (lapjv with cost_limit takes an
// isolated pair with cost < thresh): x1 / y1 get them and -1 elsewhere, the row's edge count
// becomes 0, and k_s1_lap solves what is left (about half of the edges at 1024 x 1024), with a
// smaller LDS arena.  Removing a whole component leaves every other node's degree as it was.
__device__ __forceinline__ void s1_single_edges(const BtArgs &a, int s, int nc, int nr, int *cdeg,
                                                bool lds, const int (&rn)[4], const int (&rc)[4]) {
    const int t = threadIdx.x, nt = blockDim.x;
    const long long tb = (long long)s * a.CAP, db = (long long)s * a.MAXD;
    if (lds) lds_sync();
    else block_sync();
    auto row = [&](int i, int n, int c) {   // rows i = t mod nt: this thread found their edges
        int x = -1;
        if (n == 1 && ald(cdeg + c) == 1) {
            x = c;
            cdeg[c] = ~i;   // the column's only row
            a.e_cnt[tb + i] = 0;
        }
        a.x1[tb + i] = x;
    };
#pragma unroll
    for (int b = 0; b < 4; ++b)
        if (t + b * nt < nr) row(t + b * nt, rn[b], rc[b]);
    for (int i = t + 4 * nt; i < nr; i += nt) {
        const int n = a.e_cnt[tb + i];
        row(i, n, n == 1 ? a.e_col[tb + i] : -1);
    }
    if (lds) lds_sync();
    else block_sync();
    for (int j = t; j < nc; j += nt) {
        const int d = ald(cdeg + j);
        a.y1[db + j] = d < 0 ? ~d : -1;
    }
}

// two 512-thread blocks per CU: <= 128 VGPRs (the diagnostic build's stamps would add some);
// NT 1024 with few streams (split23)
template <int NT>
__global__ __launch_bounds__(NT, NT == BLKE ? 4 : 1) void k_s1_edges(BtArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    __shared__ GridScratch gs;
    __shared__ int wsum[32];
    __shared__ int spill, n_edges;
    __shared__ EdgeWaveQ ewq[NT / WAVE];
    const int s = blockIdx.x, t = threadIdx.x, nt = blockDim.x;
    if (stream_skipped(a, s)) return;
    YTA_STAMP_BASE(66);
    YTA_STAMP(0);
    YTA_BLK(1, 0);
    BtCounters *c = a.cnt + s;
    const long long db = (long long)s * a.MAXD;
    const int nc = c->n_high, nr = c->n_pool;
    // this thread's detections t and t + blockDim held in registers (nc <= 2 blockDim: every box
    // load in flight at once; the grid build reads them three times)
    Box hb0{0.0, 0.0, 0.0, 0.0}, hb1{0.0, 0.0, 0.0, 0.0};
    double hw0 = 0.0, hw1 = 0.0;
    if (t < nc) {
        hb0 = a.high_box[db + t];
        hw0 = a.high_score[db + t];
    }
    if (t + nt < nc) {
        hb1 = a.high_box[db + t + nt];
        hw1 = a.high_score[db + t + nt];
    }
    if (t == 0) {
        spill = 0;
        n_edges = 0;
    }
    int rn[4] = {0, 0, 0, 0}, rc[4] = {-1, -1, -1, -1};   // rows t + b * nt (s1_single_edges)
    if (nc > 2 * nt || s1_grid_bytes(nc) + 4LL * nc > (long long)a.lds_bytes_e) {   // HBM grid
        int *cdeg = a.g_deg + db;
        for (int j = t; j < nc; j += nt) cdeg[j] = 0;
        block_sync();
        s1_edges_body(
            a, s, nc, nr, s1_grid_hbm(a, s), [&](int j) { return a.high_box[db + j]; },
            [&](int j) { return a.high_score[db + j]; }, gs, wsum, spill, cdeg, n_edges, rn, rc);
        s1_single_edges(a, s, nc, nr, cdeg, false, rn, rc);
        if (t == 0) c->n_edges[0] = n_edges;
        YTA_BLK(1, 1);
        return;
    }
    // grid_build visits item j only from thread j mod blockDim: a register select, no memory
    auto hbox = [&](int j) { return j == t ? hb0 : hb1; };
    auto hw = [&](int j) { return j == t ? hw0 : hw1; };
    Arena ar(smem, a.lds_bytes_e);
    GridView gv;
    gv.hdr = nullptr;
    gv.cell_start = ar.alloc<int>(grid_cells_for(nc) + 1);
    gv.ids = ar.alloc<int>(nc);
#if YTA_S1_SOA
    gv.boxes = nullptr;   // the boxes as four arrays (GridView::sx): conflict-free wave reads
    gv.sx = ar.alloc<double>(4LL * nc);
    gv.sn = nc;
#else
    gv.boxes = ar.alloc<Box>(nc);
#endif
    gv.w = ar.alloc<double>(nc);
    gv.big = ar.alloc<int>(nc);
    int *cdeg = ar.alloc<int>(nc);
    for (int j = t; j < nc; j += nt) cdeg[j] = 0;   // grid_build's barriers order these
    grid_build(nc, hbox, hw, gv, gs, wsum);
    YTA_STAMP(1);
    s1_edges_rows_wave(a, s, nr, gv, gs.hdr, ewq[t / WAVE], spill, cdeg, n_edges, rn, rc);
    s1_single_edges(a, s, nc, nr, cdeg, true, rn, rc);
    if (t == 0) c->n_edges[0] = n_edges;
    YTA_STAMP(2);
    YTA_BLK(1, 1);
    if (!spill) return;
    // some row has more edges than slots: k_s1_lap queries the grid again, from HBM
    const GridHdr h = gs.hdr;
    const GridView gg = s1_grid_hbm(a, s);
    const int ncell = h.gx * h.gy;
    if (t == 0) *gg.hdr = h;
    for (int q = t; q <= ncell; q += nt) gg.cell_start[q] = gv.cell_start[q];
    for (int q = t; q < h.n_binned; q += nt) {
        gg.ids[q] = gv.ids[q];
        gg.boxes[q] = s1_box(gv, q);
        gg.w[q] = gv.w[q];
    }
    for (int q = t; q < h.n_big; q += nt) gg.big[q] = gv.big[q];
}

// Arena bytes that always suffice for s1_lap_body (the global fallback arena's size): compact
// rows (ids, offsets, matches), column bitmap + word prefix, compact columns (ids, degrees,
// matches), the CSR, lap_block's work arrays.
__host__ __device__ inline long long s1_lap_arena_bytes(long long R, long long C, long long E) {
    return 4 * (R + 1) + 8 * R + 8 * ((C + 31) / 32 + 1) + 12 * C + 12 * E + 4 * (R + C) * 3 +
           4 * 6 * (R + C + 1) + 16 * 16 + 512;
}

// The residual problem (pool rows with edges left after k_s1_edges' single-edge components,
// high detections they reach) is solved on compact, order-preserving renumberings of its rows and
// columns: lap_block's results depend on node ids only through their order, so the assignment is
// the one it finds on the full index ranges, while its arrays (union-find over rows + columns, the
// CSR offsets) cover the ~30 % of pool rows and ~40 % of detections that are in play instead of all
// of them (the steady state's 1600-row pools otherwise overflow the 38 KiB arena).
__device__ __forceinline__ bool s1_lap_body(const BtArgs &a, int s, Arena &ar, LapShared &lsh) {
    const int t = threadIdx.x, nt = blockDim.x;
    BtCounters *c = a.cnt + s;
    const long long db = (long long)s * a.MAXD, tb = (long long)s * a.CAP;
    const long long SC = (long long)a.S * a.CAP;
    const int nr = c->n_pool, nc = c->n_high;
    YTA_STAMP_BASE(90);
    YTA_STAMP(0);
    // k_s1_edges filled x1 / y1 with its single-edge matches and -1; only the residual problem's
    // matches are written below
    int *X = a.x1 + tb;
    int *Y = a.y1 + db;
    // rows in play and their edge total
    int myr = 0, mye = 0;
    for (int i = t; i < nr; i += nt) {
        const int n = a.e_cnt[tb + i];
        myr += n > 0;
        mye += n;
    }
    int R, E;
    block_exclusive_scan<false>(myr, lsh.wsum, &R);
    block_exclusive_scan<false>(mye, lsh.wsum, &E);
    if (E == 0) {
        if (t == 0) c->n_res1 = 0;
        return true;
    }
    const int words = (nc + 31) >> 5;
    int *rid = ar.alloc_top<int>(R);
    int *row_off = ar.alloc_top<int>(R + 1);
    unsigned *cbits = ar.alloc_top<unsigned>(words);
    int *cpre = ar.alloc_top<int>(words + 1);
    int *csr_col = ar.alloc_top<int>(E);
    double *csr_cost = ar.alloc_top<double>(E);
    if (ar.fail) return false;
    for (int w = t; w < words; w += nt) cbits[w] = 0u;
    // compact rows in pool order (each thread a contiguous run of <= 8 rows) and their offsets
    int runR = 0, runE = 0;
    for (int base = 0; base < nr; base += 8 * nt) {
        const int m = nr - base < 8 * nt ? nr - base : 8 * nt;
        const int per = (m + nt - 1) / nt;
        const int lo = base + t * per;
        const int hi = lo + per < base + m ? lo + per : base + m;
        int cnt[8], mr = 0, me = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            cnt[k] = lo + k < hi ? a.e_cnt[tb + lo + k] : 0;
            mr += cnt[k] > 0;
            me += cnt[k];
        }
        int totR, totE;
        int pr = runR + block_exclusive_scan<false>(mr, lsh.wsum, &totR);
        int pe = runE + block_exclusive_scan<false>(me, lsh.wsum, &totE);
#pragma unroll
        for (int k = 0; k < 8; ++k)
            if (cnt[k] > 0) {
                rid[pr] = lo + k;
                row_off[pr] = pe;
                ++pr;
                pe += cnt[k];
            }
        runR += totR;
        runE += totE;
    }
    if (t == 0) row_off[R] = E;
    block_sync();
    YTA_STAMP(1);
    // CSR fill from the edge slots (runs of compact rows, four rows' slot loads in flight); a row
    // with more edges than slots queries the stream's grid in HBM again.  Columns in play: bitmap.
    {
        const GridView gg = s1_grid_hbm(a, s);
        for (int base = 0; base < R; base += 8 * nt) {
            const int m = R - base < 8 * nt ? R - base : 8 * nt;
            const int per = (m + nt - 1) / nt;
            const int lo = base + t * per;
            const int hi = lo + per < base + m ? lo + per : base + m;
#pragma unroll
          for (int half = 0; half < 8; half += 4) {
            int col[4][E_SLOTS];
            double cost[4][E_SLOTS];
            int n[4], gi[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int r = lo + half + k;
                n[k] = r < hi ? row_off[r + 1] - row_off[r] : 0;
                gi[k] = r < hi ? rid[r] : 0;
#pragma unroll
                for (int q = 0; q < E_SLOTS; ++q)
                    if (q < n[k]) {
                        col[k][q] = a.e_col[q * SC + tb + gi[k]];
                        cost[k][q] = a.e_cost[q * SC + tb + gi[k]];
                    }
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                if (n[k] == 0) continue;
                const int r = lo + half + k;
                int e = row_off[r];
                if (n[k] <= E_SLOTS) {
#pragma unroll
                    for (int q = 0; q < E_SLOTS; ++q)
                        if (q < n[k]) {
                            csr_col[e + q] = col[k][q];
                            csr_cost[e + q] = cost[k][q];
                            atomicOr(&cbits[col[k][q] >> 5], 1u << (col[k][q] & 31));
                        }
                } else {
                    const int eend = row_off[r + 1];
                    s1_row_edges(a, s, gg, *gg.hdr, a.pool_box[tb + gi[k]], [&](int j, double cj) {
                        if (e >= eend) return;
                        csr_col[e] = j;
                        csr_cost[e] = cj;
                        ++e;
                        atomicOr(&cbits[j >> 5], 1u << (j & 31));
                    });
                }
            }
          }
        }
    }
    block_sync();
    YTA_STAMP(2);
    // compact columns in detection order: prefix over the bitmap words (written by atomics: read
    // around the L1 when the arena is global)
    auto cword = [&](int w) { return (unsigned)ald(reinterpret_cast<const int *>(cbits + w)); };
    int C = 0;
    for (int base = 0; base < words; base += nt) {
        const int w = base + t;
        const int pc = w < words ? __popc(cword(w)) : 0;
        int tot;
        const int ex = block_exclusive_scan<false>(pc, lsh.wsum, &tot);
        if (w < words) cpre[w] = C + ex;
        C += tot;
    }
    int *cols = ar.alloc_top<int>(C);
    int *cdeg = ar.alloc_top<int>(C);
    int *Xc = ar.alloc_top<int>(R);
    int *Yc = ar.alloc_top<int>(C);
    if (ar.fail) return false;
    block_sync();
    for (int w = t; w < words; w += nt) {
        unsigned b = cword(w);
        int p = cpre[w];
        while (b) {
            const int k = __ffs(b) - 1;
            b &= b - 1;
            cols[p] = w * 32 + k;
            cdeg[p] = 0;
            ++p;
        }
    }
    block_sync();
    for (int e = t; e < E; e += nt) {
        const int j = csr_col[e];
        const int w = j >> 5;
        const int cc = cpre[w] + __popc(cword(w) & ((1u << (j & 31)) - 1u));
        csr_col[e] = cc;
        atomicAdd(&cdeg[cc], 1);
    }
    block_sync();
    if (!lap_block(R, C, row_off, csr_col, csr_cost, cdeg, a.match_thresh, Xc, Yc, &c->err, ar,
                   slab_of(a, s), lsh, true))
        return false;
    YTA_STAMP(3);
    // the residual matches, in the original numbering
    for (int r = t; r < R; r += nt) {
        const int x = Xc[r];
        if (x >= 0) {
            X[rid[r]] = cols[x];
            Y[cols[x]] = rid[r];
        }
    }
    if (t == 0) c->n_res1 = E;   // edges left after the single-edge components
    return true;
}

// four 256-thread blocks per CU: <= 128 VGPRs (4 waves per SIMD) and a <= 36 KiB arena; NT 1024
// with few streams (split23)
template <int NT>
__global__ __launch_bounds__(NT, NT == BLKL ? 4 : 1) void k_s1_lap(BtArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    __shared__ LapShared lsh;
    const int s = blockIdx.x;
    if (stream_skipped(a, s)) return;
    YTA_BLK(2, 0);
    Arena ar(smem, a.lds_bytes_l);
    if (!s1_lap_body(a, s, ar, lsh)) {
        block_sync();
        if (threadIdx.x == 0) a.cnt[s].n_fallback[0] += 1;
        // the many-stream kernel always queues: a redo in place costs it 48 B more scratch
        if (NT == 1024 && redo_in_place(a, a.S)) {
            Arena ag(redo_arena(a, s), a.ws_stride);
            if (!s1_lap_body(a, s, ag, lsh) && threadIdx.x == 0)
                atomicOr(&a.cnt[s].err, ERR_EDGE_OVERFLOW);
        } else if (threadIdx.x == 0) {
            redo_queue(a, s);
        }
    }
    YTA_BLK(2, 1);
}
template <int NT>
__global__ __launch_bounds__(NT) void k_redo_s1_lap(BtArgs a) {
    __shared__ LapShared lsh;
    redo_drain(a, [&](int s, Arena &ag) {
        if (!s1_lap_body(a, s, ag, lsh) && threadIdx.x == 0)
            atomicOr(&a.cnt[s].err, ERR_EDGE_OVERFLOW);
    });
}

// ------------------------------------------------------------------------------ k_feat / k_ema
// BoT-SORT features, one wave per row.  Norms follow np.linalg.norm on a float32 row (the sum of
// squares rounded to float32, then sqrt in float32); the sum is accumulated in float64 here,
// where OpenBLAS sdot accumulates in float32 lanes, so a norm may differ from the reference's in
// its last bit (the parity tests compare features with a tolerance).
__device__ __forceinline__ float f32_norm(double sumsq) { return sqrtf((float)sumsq); }

// k_feat: per high detection (conf > track_high_thresh, the stage-1 predicate) the norms of the
// in-place normalisations the reference applies to its row: n1 = |e|, n2 = |e/n1| (STrack
// construction, :40-48) and n3 = |(e/n1)/n2| (when a track takes it, :40-41).
constexpr int FEAT_T = 256;
__host__ __device__ __forceinline__ int feat_blocks(int maxd, int threads = FEAT_T) {
    return (maxd + threads / WAVE - 1) / (threads / WAVE);
}
__device__ __forceinline__ void feat_body(const BtArgs &a, int s, int bx) {
    const int lane = lane_id();
    if (stream_skipped(a, s)) return;
    const int d = bx * (int)(blockDim.x / WAVE) + threadIdx.x / WAVE;
    const int nd = min(a.det_off[s + 1] - a.det_off[s], a.MAXD);
    if (d >= nd) return;
    const long long row = (long long)a.det_off[s] + d;
    if (!(a.det_in[row * 6 + 4] > a.track_thresh)) return;
    const float *e = a.det_feat + row * a.D;
    double q = 0.0;
    for (int k = lane; k < a.D; k += WAVE) q += (double)e[k] * (double)e[k];
    const float n1 = f32_norm(wave_reduce(RED_SUM, q));
    q = 0.0;
    for (int k = lane; k < a.D; k += WAVE) {
        const float f = e[k] / n1;
        q += (double)f * (double)f;
    }
    const float n2 = f32_norm(wave_reduce(RED_SUM, q));
    q = 0.0;
    for (int k = lane; k < a.D; k += WAVE) {
        const float f = (e[k] / n1) / n2;
        q += (double)f * (double)f;
    }
    const float n3 = f32_norm(wave_reduce(RED_SUM, q));
    if (lane == 0) {
        float *fn = a.det_fn + ((long long)s * a.MAXD + d) * 4;
        fn[0] = n1;
        fn[1] = n2;
        fn[2] = n3;
        fn[3] = 0.f;
    }
}
__global__ __launch_bounds__(FEAT_T) void k_feat(BtArgs a) { feat_body(a, blockIdx.y, blockIdx.x); }

// k_ema: update_features of every track that took a high detection this frame (bot_sort.py:40-48):
// f = curr / |curr| with curr = (e/n1)/n2, smooth = 0.9 * smooth + 0.1 * f (float32), then
// smooth /= |smooth|.
constexpr int EMA_T = 256;
__host__ __device__ __forceinline__ int ema_blocks(int cap, int threads = EMA_T) {
    return (cap + threads / WAVE - 1) / (threads / WAVE);
}
__device__ __forceinline__ void ema_body(const BtArgs &a, int s, int bx) {
    const int lane = lane_id();
    if (stream_skipped(a, s)) return;
    const BtCounters *c = a.cnt + s;
    const int n_pool = c->n_pool, n_items = n_pool + c->n_unc;
    const int item = bx * (int)(blockDim.x / WAVE) + threadIdx.x / WAVE;
    if (item >= n_items) return;
    const long long tb = (long long)s * a.CAP, db = (long long)s * a.MAXD;
    const int h = a.ema_job[tb + item];
    if (h < 0) return;
    const int slot = item < n_pool ? a.pool[tb + item] : a.unc[tb + item - n_pool];
    const int d = a.high[db + h];
    const float *fn = a.det_fn + (db + d) * 4;
    const float n1 = fn[0], n2 = fn[1], n3 = fn[2];
    const float *e = a.det_feat + ((long long)a.det_off[s] + d) * a.D;
    float *sm = a.feat + (tb + slot) * a.D;
    double q = 0.0;
    for (int k = lane; k < a.D; k += WAVE) {
        const float f = ((e[k] / n1) / n2) / n3;
        const float v = 0.9f * sm[k] + 0.1f * f;
        sm[k] = v;
        q += (double)v * (double)v;
    }
    const float nrm = f32_norm(wave_reduce(RED_SUM, q));
    for (int k = lane; k < a.D; k += WAVE) sm[k] = sm[k] / nrm;
}
__global__ __launch_bounds__(EMA_T) void k_ema(BtArgs a) { ema_body(a, blockIdx.y, blockIdx.x); }

// ------------------------------------------------------------ BoT-SORT stage 1, split (C3)
// With ReID features, k_stage1's block per stream spends most of a few-stream frame on the
// appearance costs of the candidate pairs (bot_sort.py:307-322: ~2.5 D-long dot products per pool
// row, read through one CU).  For few streams the stage runs as three launches instead:
//   k_bs_prep  block / stream: the lists and boxes of stage 1 (stage1_lists)
//   k_bs_edges chip-wide, one wave per pool row: the row against every high detection (f64 box
//              test), the IoU cost, and for pairs inside proximity_thresh the cosine distance of
//              the features with the same 16-lane reduction k_stage1 uses (cosine_dist16), so
//              every cost has the same bits; edges with cost < match_thresh into the row's
//              E_SLOTS slots (e_cnt / e_col / e_cost, the layout k_s1_lap reads)
//   k_bs_lap   block / stream: lap_block over the edges (s1_lap_body, which solves the problem on
//              order-preserving renumberings: the same assignment as k_stage1's lap_block); a
//              stream with a row of more than E_SLOTS edges runs k_stage1's association instead.
// Same results as k_stage1 on every stream.
constexpr int BSE_T = 256;   // k_bs_edges threads: 4 waves = 4 pool rows per block

constexpr int BS_PREP_T = 1024;   // k_bs_prep (few streams: one block per stream takes the lists)
__global__ __launch_bounds__(BS_PREP_T) void k_bs_prep(BtArgs a) {
    __shared__ StageShared sh;
    if ((int)blockIdx.x >= a.S) {   // k_feat's blocks, launched with this grid (independent work)
        const int b = blockIdx.x - a.S, fb = feat_blocks(a.MAXD, BS_PREP_T);
        feat_body(a, b / fb, b % fb);
        return;
    }
    const int s = blockIdx.x;
    if (stream_skipped(a, s)) return;
    YTA_STAMP_BASE(0);
    YTA_STAMP(0);
    Arena none(nullptr, 0);   // no staged high boxes (the embedding association does not use them)
    const S1Lists L = stage1_lists<VAR_BOTSORT>(a, s, none, sh);
    stage1_commit(a.cnt + s, L, false);
    if (threadIdx.x == 0) {
        a.cnt[s].bs_spill = 0;
        a.cnt[s].n_edges[0] = 0;
    }
    // stage 1's results start unmatched (s1_lap_body writes only the residual matches; the fused
    // association, taken on a spill, writes every entry): cleared here, off k_bs_lap's chain
    const long long tb = (long long)s * a.CAP, db = (long long)s * a.MAXD;
    for (int q = threadIdx.x; q < L.n_pool; q += blockDim.x) a.x1[tb + q] = -1;
    for (int q = threadIdx.x; q < L.n_high; q += blockDim.x) a.y1[db + q] = -1;
}

// A pool row's pairs that need the appearance cost (inside proximity_thresh) are queued per wave
// while the row's column passes run, then costed four at a time (one 16-lane group each) with their
// feature rows' loads in flight together, instead of one dependent chain per column pass.
constexpr int BS_PQ = 64;   // queued pairs per wave (a full queue is costed before more are added)
struct BsPend {
    int j, dj;   // high position, detection index
    double cc;   // the (fused) IoU cost
};

__global__ __launch_bounds__(BSE_T) void k_bs_edges(BtArgs a) {
    __shared__ BsPend pq[BSE_T / WAVE][BS_PQ];
    const int s = blockIdx.y;
    if (stream_skipped(a, s)) return;
    BtCounters *c = a.cnt + s;
    const int i = blockIdx.x * (BSE_T / WAVE) + threadIdx.x / WAVE;   // pool row (wave-uniform)
    const int n_pool = c->n_pool, nh = c->n_high;
    if (i >= n_pool) return;
    const int lane = lane_id(), grp = lane >> 4;
    const long long tb = (long long)s * a.CAP, db = (long long)s * a.MAXD;
    const long long SC = (long long)a.S * a.CAP;
    const long long doff = a.det_off[s];
    const double prox = a.prox_thresh, app = a.app_thresh, thresh = a.match_thresh;
    const bool fused = a.fuse_first != 0;
    const Box rb = a.pool_box[tb + i];
    const float *rfeat = a.feat + (tb + a.pool[tb + i]) * a.D;
    BsPend *q = pq[threadIdx.x / WAVE];
    int n = 0;    // the row's edges (wave-uniform)
    int nq = 0;   // queued pairs (wave-uniform)
    auto put = [&](bool e, int j, double cost) {   // edges of this pass in lane order
        const unsigned long long m = __ballot(e);
        if (e) {
            const int k = n + __popcll(m & ((1ull << lane) - 1ull));
            if (k < E_SLOTS) {
                a.e_col[k * SC + tb + i] = j;
                a.e_cost[k * SC + tb + i] = cost;
            }
        }
        n += __popcll(m);
    };
    auto flush = [&]() {   // the queued pairs' appearance costs, four at a time
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        for (int p0 = 0; p0 < nq; p0 += 4) {
            const int p = p0 + grp;
            const bool v = p < nq;
            const BsPend e = q[v ? p : p0];
            const float *fn = a.det_fn + (db + e.dj) * 4;
            const DetFeat f{a.det_feat + (doff + e.dj) * a.D, fn[0], fn[1]};
            const double cd = cosine_dist16(rfeat, f, a.D);
            double cost = 1.0;
            if (v) {
                double emb = np_max(0.0, cd) / 2.0;                           // matching.py:164-166
                if (emb > app) emb = 1.0;                                       // bot_sort.py:318
                cost = np_min(e.cc, emb);                                       // bot_sort.py:320
            }
            put((lane & 15) == 0 && v && cost < thresh, e.j, cost);
        }
        __builtin_amdgcn_wave_barrier();   // the queue is rewritten next
        nq = 0;
    };
    constexpr int BOX_BATCH = 4;   // column boxes of 4 passes loaded at once (one round trip)
    Box cbs[BOX_BATCH];
    int hds[BOX_BATCH];   // the columns' detection indices (their feature rows), loaded alongside
    for (int j0 = 0; j0 < nh; j0 += WAVE) {
        const int j = j0 + lane;
        const int kb = (j0 / WAVE) % BOX_BATCH;
        if (kb == 0) {
#pragma unroll
            for (int k = 0; k < BOX_BATCH; ++k) {
                const int jk = j + k * WAVE < nh ? j + k * WAVE : 0;
                cbs[k] = a.high_box[db + jk];
                hds[k] = a.high[db + jk];
            }
        }
        Box cb = cbs[0];
        int hd = hds[0];
#pragma unroll
        for (int k = 1; k < BOX_BATCH; ++k)
            if (kb == k) {
                cb = cbs[k];
                hd = hds[k];
            }
        bool hit = false;
        double d = 1.0, cc = 1.0;
        if (j < nh) {
            if (intersects(rb, cb)) {
                hit = true;
                d = 1 - iou(rb, cb);                                        // matching.py:117
                cc = fused ? 1 - (1 - d) * a.high_score[db + j] : d;       // matching.py:216-220
            }
        }
        const bool masked = hit && d > prox;                               // emb masked (:319)
        const double mc = np_min(cc, 1.0);
        put(masked && mc < thresh, j, mc);
        const bool pend = hit && !masked;
        const unsigned long long pm = __ballot(pend);
        if (pm) {
            if (nq + __popcll(pm) > BS_PQ) flush();
            if (pend) q[nq + __popcll(pm & ((1ull << lane) - 1ull))] = BsPend{j, hd, cc};
            nq += __popcll(pm);
        }
    }
    if (nq) flush();
    if (lane == 0) {
        a.e_cnt[tb + i] = n;
        if (n > E_SLOTS) atomicOr(&c->bs_spill, 1);
        if (n) atomicAdd(&c->n_edges[0], n);
    }
}

__global__ __launch_bounds__(BLK1) void k_bs_lap(BtArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    __shared__ StageShared sh;
    const int s = blockIdx.x, t = threadIdx.x, nt = blockDim.x;
    if (stream_skipped(a, s)) return;
    BtCounters *c = a.cnt + s;
    const long long tb = (long long)s * a.CAP, db = (long long)s * a.MAXD;
    const int n_pool = c->n_pool, n_high = c->n_high;
    const bool spill = c->bs_spill != 0;
    const S1Lists L{c->n_dets, n_high, c->n_second, c->n_act, c->n_unc, n_pool, nullptr, nullptr};
    // x1 / y1 were cleared by k_bs_prep
    Arena ar(smem, a.lds_bytes);
    bool ok = spill ? stage1_assoc<VAR_BOTSORT>(a, s, L, ar, sh) : s1_lap_body(a, s, ar, sh.as.lap);
    if (!ok) {   // a global arena: here, or by k_redo_bs_lap (which then advances the frame)
        block_sync();
        if (t == 0) c->n_fallback[0] += 1;
        if (!redo_in_place(a, a.S)) {
            if (t == 0) redo_queue(a, s);
            return;
        }
        if (!spill) {
            for (int q = t; q < n_pool; q += nt) a.x1[tb + q] = -1;
            for (int q = t; q < n_high; q += nt) a.y1[db + q] = -1;
            block_sync();
        }
        Arena ag(redo_arena(a, s), a.ws_stride);
        ok = spill ? stage1_assoc<VAR_BOTSORT>(a, s, L, ag, sh) : s1_lap_body(a, s, ag, sh.as.lap);
        if (!ok && t == 0) atomicOr(&c->err, ERR_EDGE_OVERFLOW);
    }
    block_sync();
    if (t == 0) {
        c->frame_id += 1;
        c->n_res1 = 0;   // a ByteTrack statistic (s1_lap_body sets it): 0, as the fused k_stage1
    }
}
__global__ __launch_bounds__(BLK1) void k_redo_bs_lap(BtArgs a) {
    __shared__ StageShared sh;
    const int t = threadIdx.x, nt = blockDim.x;
    redo_drain(a, [&](int s, Arena &ag) {
        BtCounters *c = a.cnt + s;
        const long long tb = (long long)s * a.CAP, db = (long long)s * a.MAXD;
        const int n_pool = c->n_pool, n_high = c->n_high;
        const bool spill = c->bs_spill != 0;
        const S1Lists L{c->n_dets, n_high, c->n_second, c->n_act, c->n_unc, n_pool, nullptr, nullptr};
        if (!spill) {
            for (int q = t; q < n_pool; q += nt) a.x1[tb + q] = -1;
            for (int q = t; q < n_high; q += nt) a.y1[db + q] = -1;
            block_sync();
        }
        const bool ok = spill ? stage1_assoc<VAR_BOTSORT>(a, s, L, ag, sh)
                              : s1_lap_body(a, s, ag, sh.as.lap);
        block_sync();
        if (t == 0) {
            if (!ok) atomicOr(&c->err, ERR_EDGE_OVERFLOW);
            c->frame_id += 1;
            c->n_res1 = 0;
        }
    });
}

// ------------------------------------------------------------------------------------ k_apply
// BoT-SORT STrack.update_cls (bot_sort.py:50-67): per-class summed scores, the first strict
// maximum wins; a class not seen before is appended and taken as is.
__device__ __forceinline__ double vote_cls(double2 *h, int &n, double cls, double score,
                                           int *err) {
    double out = cls;
    if (n > 0) {
        double maxf = 0.0;
        bool found = false;
        for (int e = 0; e < n; ++e) {
            double2 c = h[e];
            if (cls == c.x) {
                c.y += score;
                h[e] = c;
                found = true;
            }
            if (c.y > maxf) {
                maxf = c.y;
                out = c.x;
            }
        }
        if (!found) {
            if (n < CLS_K) h[n++] = make_double2(cls, score);
            else atomicOr(err, ERR_CLS_HIST);
            out = cls;
        }
    } else {
        h[0] = make_double2(cls, score);
        n = 1;
    }
    return out;
}

// A detection's Kalman measurement (ByteTrack xyah, BoT-SORT xywh: STrack's conversions,
// ops.py:7-97), confidence and class, computed from its input row where a track takes it (one
// 48-B row instead of three per-detection arrays written by the detection pass and gathered back).
struct DetMeas {
    double z[4];
    double conf, cls;
};
template <int V>
__device__ __forceinline__ DetMeas det_meas(const BtArgs &a, int s, int d) {
    const double *r = a.det_in + ((long long)a.det_off[s] + d) * 6;
    double v[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) v[k] = r[k];
    DetMeas m;
    double xywh[4];
    det_xyxy_to_xywh(v, xywh);
    if (V == VAR_BOTSORT) {
#pragma unroll
        for (int k = 0; k < 4; ++k) m.z[k] = xywh[k];
    } else {
        xywh_to_xyah(xywh, m.z);
    }
    m.conf = v[4];
    m.cls = v[5];
    return m;
}

// STrack.update / re_activate (byte_tracker.py:70-98; bot_sort.py:125-170) minus the feature EMA
// (k_ema)
template <int V>
__device__ __forceinline__ void take_detection(const BtArgs &a, KfState &st, TrackMeta &m,
                                               int &flags, const DetMeas &dm, int det_local,
                                               int fid, long long slot, int *err,
                                               double *xc = nullptr) {
    if (V == VAR_BOTSORT && xc) kf_update_x(st, xc, dm.z);   // warped track
    else kf_update<kf_model<V>()>(st, dm.z);
    const bool reactivate = st_of(flags) != ST_TRACKED;
    m.tracklet_len = reactivate ? 0 : m.tracklet_len + 1;
    flags = (flags & ~FL_STATE) | ST_TRACKED | FL_ACTIVATED;
    m.frame_id = fid;
    m.score = dm.conf;
    m.cls = dm.cls;
    m.det_ind = det_local;
    if (V == VAR_BOTSORT) m.cls = vote_cls(a.cls_hist + slot * CLS_K, m.n_cls, m.cls, m.score, err);
}

// Records move between HBM and LDS in whole 16-B pieces with consecutive lanes on consecutive
// pieces of a record (full-line reads and writes); each thread then runs the Kalman step of one
// track out of LDS.  LDS row: pieces 0-3 the mean, 4-6 the meta, 7-14 the covariance (record
// pieces 0-6 and 8-15: the padding piece 7 is skipped).
constexpr int APPLY_T = 128;              // tracks (= threads) per block
constexpr int REC_PIECES = 15;            // 16-B pieces of a record that carry data
constexpr int L_META = 8, L_COV = 14;     // doubles: meta / covariance in an LDS row
__device__ __forceinline__ int rec_piece(int k) { return k < 7 ? k : k + 1; }   // LDS -> record
__device__ __forceinline__ bool piece_is_meta(int k) { return k >= 4 && k < 7; }

template <int V>
__global__ __launch_bounds__(APPLY_T) void k_apply(BtArgs a) {
    __shared__ double2 rec[APPLY_T][REC_PIECES];   // 60-dword rows: no bank conflicts
    static_assert(APPLY_T % WAVE == 0, "whole waves per block (LDS-direct load tiling)");
    __shared__ int s_slot[APPLY_T];
    __shared__ int s_wmask[APPLY_T];      // bit 0: write the Kalman record, bit 1: write the meta
    const int s = blockIdx.y, t = threadIdx.x;
    if (stream_skipped(a, s)) return;
    BtCounters *c = a.cnt + s;
    const int n_pool = c->n_pool, n_unc = c->n_unc, fid = c->frame_id;
    const int i0 = blockIdx.x * APPLY_T;
    const int n_items = n_pool + n_unc;
    if (i0 >= n_items) return;                                       // block-uniform
    YTA_APL(0);
    const int nloc = n_items - i0 < APPLY_T ? n_items - i0 : APPLY_T;
    const long long tb = (long long)s * a.CAP, db = (long long)s * a.MAXD;
    const int i = i0 + t;
    // per-track decision (small loads only)
    // act: 0 predict only, 1 predict + stage-1 update, 2 predict + stage-2 update, 3 predict +
    // mark lost, 4 update (unconfirmed, stage 3), 5 remove (unconfirmed)
    // The decision reads a short chain of small arrays; its loads are issued level by level with
    // the record loads in flight from level 1 on.
    // level 0 (by pool position): slot, stage-1 row result / leftover index, stage-3 result
    const bool live = t < nloc, in_pool = i < n_pool;
    int slot = -1, h = -1, L = -1, r3 = -1;
    if (live) {
        if (in_pool) {
            slot = a.pool[tb + i];
            h = a.x1[tb + i];
            L = a.left_of_pool[tb + i];
        } else {
            slot = a.unc[tb + (i - n_pool)];
            r3 = a.x3[tb + (i - n_pool)];
        }
    }
    // ByteTrack: a Lost track (the pool's tail) left unmatched in stage 1 (the only stage that
    // can re-find it) is predicted lazily (kf_xyah.hpp): its record is neither read nor written
    const bool lazy = V == VAR_BYTETRACK && live && in_pool && i >= c->n_act && h < 0;
    if (live) s_slot[t] = lazy ? -1 : slot;
    __syncthreads();
    YTA_APL(1);
    // level 1: flags, the stage-1 detection, the stage-2 result
    const int flags0 = live && !lazy ? a.flags[tb + slot] : 0;
    const int det1 = h >= 0 ? a.high[db + h] : -1;
    const int q2 = h < 0 && L >= 0 ? a.x2[tb + L] : -1;
    // Cooperative load straight into LDS (global_load_lds_dwordx4: no VGPRs, nothing the compiler
    // can sink behind the decision chain below): piece p = t + q * APPLY_T is piece p % 15 of
    // record p / 15, so each wave-instruction writes 1 KiB of rec linearly and consecutive lanes
    // read consecutive pieces of a record.  All 15 are in flight while the decision runs.
    {
        const double2 *rec2 = reinterpret_cast<const double2 *>(a.kf);
        char *ldsb = reinterpret_cast<char *>(&rec[0][0]);
        const int wb = __builtin_amdgcn_readfirstlane(t & ~(WAVE - 1));
#pragma unroll
        for (int q = 0; q < REC_PIECES; ++q) {
            const int p = t + q * APPLY_T;
            const int r = p / REC_PIECES, k = p - r * REC_PIECES;
            const int rs = s_slot[r < nloc ? r : 0];   // rows past nloc: row 0 again
            const long long sl = tb + (rs < 0 ? 0 : rs);
            const double2 *src = rec2 + sl * (TRK_STRIDE / 2) + rec_piece(k);
            if (rs >= 0)   // lazy rows: nothing loaded, their LDS row is never read
                __builtin_amdgcn_global_load_lds((glob_void *)src,
                                                 (lds_void *)(ldsb + (wb + q * APPLY_T) * 16), 16,
                                                 0, 0);
        }
    }
    // level 2 (3 for stage 3): the stage-2 / stage-3 detections
    // act: 0 predict only, 1 predict + stage-1 update, 2 predict + stage-2 update, 3 predict +
    // mark lost, 4 update (unconfirmed, stage 3), 5 remove (unconfirmed)
    int det = -1, act = 0, hpos = -1;
    DetMeas dm{};
    if (live) {
        if (in_pool) {
            if (h >= 0) {                                            // stage 1 (:188-196)
                act = 1;
                hpos = h;
                det = det1;
            } else if (L >= 0) {
                if (q2 >= 0) {                                       // stage 2 (:212-220)
                    act = 2;
                    det = a.second[db + q2];
                } else {
                    act = 3;                                         // mark_lost (:222-226)
                }
            }
        } else if (r3 >= 0) {                                        // stage 3 (:234-236)
            act = 4;
            hpos = a.rest[db + r3];
            det = a.high[db + hpos];
        } else {
            act = 5;                                                 // :237-240
        }
        // BoT-SORT: tracks taking a high detection also take its feature (k_ema)
        if (V == VAR_BOTSORT && a.D > 0) a.ema_job[tb + i] = hpos;
        if (det >= 0) dm = det_meas<V>(a, s, det);   // in flight beside the records
        // pieces this track rewrites: bit 0 the Kalman record, bit 1 the meta
        s_wmask[t] = act == 5 ? 0 : (act == 1 || act == 2 || act == 4 ? 3 : 1);
    }
    if (lazy) s_wmask[t] = 0;
    __syncthreads();
    YTA_APL(2);
    if (!lazy && t < nloc) {
        KfState st;
        double *row = reinterpret_cast<double *>(rec[t]);
        TrackMeta m;
        memcpy(&m, row + L_META, sizeof(TrackMeta));
        int flags = flags0;
        int wmask = 0;
        // BoT-SORT camera warp (multi_gmc, bot_sort.py:293-295; kf_xyah.hpp): a warped track
        // carries covariance cross terms in kfx from then on
        const double *H = V == VAR_BOTSORT ? a.warp + 6LL * s : nullptr;
        const bool gmc = V == VAR_BOTSORT && !warp_is_identity(H);
        const bool cross = V == VAR_BOTSORT && act != 5 && (gmc || (flags0 & FL_CROSS));
        double xc[16];
        if (V == VAR_BOTSORT && cross) {
            const double2 *src = reinterpret_cast<const double2 *>(a.kfx + (tb + slot) * 16);
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const double2 v = (flags0 & FL_CROSS) ? src[k] : make_double2(0.0, 0.0);
                xc[2 * k] = v.x;
                xc[2 * k + 1] = v.y;
            }
        }
        if (act <= 3) {
#pragma unroll
            for (int k = 0; k < 8; ++k) st.m[k] = row[k];
#pragma unroll
            for (int k = 0; k < 16; ++k) st.c[k] = row[L_COV + k];
            const bool tracked = st_of(flags) == ST_TRACKED;
            if (V == VAR_BYTETRACK && in_pool && i >= c->n_act)   // re-found from the lost list:
                kf_predict_lost(st, fid - 1 - a.kf_frame[tb + slot]);   // replay the lazy predicts
            if (!tracked) {                                          // :41-42 / bot_sort.py:85-87
                st.m[7] = 0;
                if (V == VAR_BOTSORT) st.m[6] = 0;
            }
            if (V == VAR_BOTSORT && cross) {
                kf_predict_x(st, xc);
                if (gmc) kf_gmc(st, xc, H);
            } else {
                kf_predict<kf_model<V>()>(st);
            }
            wmask = 1;
            if (act == 1 || act == 2) {
                take_detection<V>(a, st, m, flags, dm, det, fid, tb + slot, &c->err,
                                  cross ? xc : nullptr);
                wmask = 3;
            } else if (act == 3) {
                flags = (flags & ~FL_STATE) | ST_LOST;
                if (V == VAR_BYTETRACK) a.kf_frame[tb + slot] = fid;
            }
        } else if (act == 4) {
#pragma unroll
            for (int k = 0; k < 8; ++k) st.m[k] = row[k];
#pragma unroll
            for (int k = 0; k < 16; ++k) st.c[k] = row[L_COV + k];
            if (V == VAR_BOTSORT && gmc) kf_gmc(st, xc, H);        // unconfirmed: warped only
            take_detection<V>(a, st, m, flags, dm, det, fid, tb + slot, &c->err,
                              cross ? xc : nullptr);
            wmask = 3;
        } else {
            flags = (flags & ~FL_STATE) | ST_REMOVED | FL_REMOVED_NOW;
        }
        if (V == VAR_BOTSORT && cross) {
            double2 *dst = reinterpret_cast<double2 *>(a.kfx + (tb + slot) * 16);
#pragma unroll
            for (int k = 0; k < 8; ++k) dst[k] = make_double2(xc[2 * k], xc[2 * k + 1]);
            flags |= FL_CROSS;
        }
        if (flags != flags0) a.flags[tb + slot] = flags;
        if (wmask & 1) {
#pragma unroll
            for (int k = 0; k < 8; ++k) row[k] = st.m[k];
#pragma unroll
            for (int k = 0; k < 16; ++k) row[L_COV + k] = st.c[k];
        }
        if (wmask & 2) memcpy(row + L_META, &m, sizeof(TrackMeta));
    }
    __syncthreads();
    YTA_APL(3);
    // cooperative store of what changed, in whole lines or aligned half lines: a written Kalman
    // record takes its (maybe unchanged) meta and the zero padding piece with it, a meta-only
    // change the padding (a partially written line costs a read-modify-write: 3-5 % on the
    // record pass, profiles/r03q_rmwbench.txt)
    double2 *recw = reinterpret_cast<double2 *>(a.kf);
    for (int p = t; p < nloc * 16; p += APPLY_T) {
        const int r = p >> 4, k = p & 15;   // record piece
        const int wm = s_wmask[r];
        const bool meta_half = k >= 4 && k < 8;
        if (!(meta_half ? (wm & 3) : (wm & 1))) continue;
        const long long sl = tb + s_slot[r];
        recw[sl * (TRK_STRIDE / 2) + k] = k == 7 ? make_double2(0.0, 0.0) : rec[r][k < 7 ? k : k - 1];
    }
    YTA_APL(4);
}

// ------------------------------------------------------------------------------------ k_finish
// Per stream: births (:242-248), lost expiry (:250-253), joint/sub list algebra incl. the
// removed_stracks quirk (:257-265), duplicate removal (:312-325) through a grid over lost' (in an
// LDS arena, or the stream's global workspace when lost' is too large), output rows (:270-281),
// free slots.  Live / drop flags are LDS bitsets.
struct FinishShared {
    GridScratch gs;
    int wsum[32];
    int cur;   // the free list's cyclic start (read before the old list is overwritten)
};

// lost' float boxes (by position) + a grid of ids over them (cell starts, ids, big list)
__host__ __device__ inline long long dedup_arena_bytes(long long n) {
    return 4 * (grid_cells_for((int)(n < GRID_MAX_CELLS ? n : GRID_MAX_CELLS)) + 1) +
           n * (16 + 4 + 4) + 4 * 16;
}

__device__ __forceinline__ int track_age(const BtArgs &a, long long slot) {
    return bt_meta(a, slot).frame_id - bt_meta(a, slot).start_frame;   // end_frame - start_frame
}

// Every pass issues all of a thread's loads before using any (block_compact_ld, batched_for):
// the block's chain is a sequence of dependent HBM round trips, each microseconds under load.
struct SlotFlags {
    int slot, flags;
};

// PRE (the few-stream 1024-thread variant): when tracked' and lost' each fit one item per
// thread, the duplicate removal's tracked' boxes are loaded beside the lost' boxes (two dependent
// round trips for both instead of two each, before and after the grid build).
template <int V, bool PRE = false>
__device__ __forceinline__ void finish_body(const BtArgs &a, int s, unsigned *bits, Arena &ar,
                                            FinishShared &sh, bool lds_ar) {
    int *wsum = sh.wsum;
    const int t = threadIdx.x, nt = blockDim.x;
    BtCounters *c = a.cnt + s;
    const long long tb = (long long)s * a.CAP, db = (long long)s * a.MAXD;
    // Barriers: the compactions' scans hand off LDS only (GSYNC false); the global lists and
    // records this kernel writes and reads back are handed over at two block_syncs, before the
    // duplicate removal (births' records and flags, t2, l2, l2pos, expiry flags) and before the
    // output rows (tracked, unc, lost, t2 when the slot list is not in the arena).  A block_sync
    // waits for every outstanding store of the block - a memory round trip per barrier on a
    // one-stream frame's chain.  lds_ar: the arena is LDS.
    const int fid = c->frame_id;
    const int n_tracked = c->n_tracked, n_lost = c->n_lost;
    const int n_rest = c->n_rest, n_left = c->n_left, n_free = c->n_free;
    const long long next_id = c->next_id;
    const int words = (a.CAP + 31) / 32;
    unsigned *live = bits, *dropA = bits + words, *dropB = bits + 2 * words;
    for (int w = t; w < 3 * words; w += nt) bits[w] = 0u;
    YTA_STAMP(1);

    // births in ascending order of the still-unmatched high detections (:242-248), each
    // initiated by the thread that lists it
    struct RestItem {
        int y3, det;
        double score;
    };
    // BoT-SORT births' feature rows are copied by the whole block below from (slot, detection)
    // pairs staged in the (not yet used) dedup arena: one pass of independent loads instead of a
    // chain of index loads per birth on one wave
    int2 *bstage = V == VAR_BOTSORT && a.D > 0 && ar.cap >= (size_t)8 * (n_rest > 0 ? n_rest : 1)
                       ? reinterpret_cast<int2 *>(ar.base)
                       : nullptr;
    const int n_births_all = block_compact_ld<4, false>(
        n_rest, wsum,
        [&](int j) {
            RestItem r;
            r.y3 = a.y3[db + j];
            r.score = a.rest_score[db + j];
            r.det = a.rest[db + j];   // high position, resolved below
            return r;
        },
        [&](int, RestItem r) {
            r.det = a.high[db + r.det];
            return r;
        },
        [&](int, const RestItem &r) { return r.y3 < 0 && r.score >= a.det_thresh; },
        [&](int j, const RestItem &r, int b) {
            a.birth[db + b] = j;
            if (b >= n_free) return;   // capacity (flagged below)
            const int slot = a.free_list[tb + b];
            const int d = r.det;
            if (bstage) bstage[b] = make_int2(slot, d);
            const DetMeas dm = det_meas<V>(a, s, d);
            KfState st;
            kf_initiate<kf_model<V>()>(dm.z, st);
            store_kf(a.kf, tb + slot, st);
            TrackMeta m;
            m.score = dm.conf;
            m.cls = dm.cls;
            m.id = next_id + 1 + b;
            m.det_ind = d;
            m.n_cls = 0;
            if (V == VAR_BOTSORT) {   // the detection's own STrack: cls_hist [[cls, score]] (:28)
                a.cls_hist[(tb + slot) * CLS_K] = make_double2(m.cls, m.score);
                m.n_cls = 1;
            }
            a.flags[tb + slot] = ST_TRACKED | (fid == 1 ? FL_ACTIVATED : 0);
            m.frame_id = fid;
            m.start_frame = fid;
            m.tracklet_len = 0;
            m.pad = 0;
            bt_meta(a, tb + slot) = m;
        });
    int n_births = n_births_all;
    if (n_births > n_free) {
        if (t == 0) atomicOr(&c->err, ERR_TRACK_CAPACITY);
        n_births = n_free;
    }
    if (V == VAR_BOTSORT && a.D > 0 && bstage) {   // smooth_feat of a birth = its curr_feat
        if (lds_ar) lds_sync();
        else block_sync();
        if ((a.D & 3) == 0) {   // 16-B pieces: rows of D floats stay 16-B aligned
            const int D4 = a.D >> 2;
            struct Piece {
                float4 e;
                float n1, n2;
                int slot;
            };
            batched_for<4>(
                n_births * D4,
                [&](int q) {
                    const int2 sd = bstage[q / D4];
                    const DetFeat f = det_feat(a, s, db, sd.y);
                    return Piece{reinterpret_cast<const float4 *>(f.e)[q % D4], f.n1, f.n2, sd.x};
                },
                [&](int q, const Piece &p) {
                    const float4 e = p.e;
                    reinterpret_cast<float4 *>(a.feat + (tb + p.slot) * a.D)[q % D4] =
                        make_float4((e.x / p.n1) / p.n2, (e.y / p.n1) / p.n2, (e.z / p.n1) / p.n2,
                                    (e.w / p.n1) / p.n2);
                });
        } else {
            batched_for<8>(
                n_births * a.D,
                [&](int q) {
                    const int2 sd = bstage[q / a.D];
                    return det_feat(a, s, db, sd.y)(q % a.D);
                },
                [&](int q, float v) { a.feat[(tb + bstage[q / a.D].x) * a.D + q % a.D] = v; });
        }
        if (lds_ar) lds_sync();   // the arena is the dedup grid's next
        else block_sync();
    } else if (V == VAR_BOTSORT && a.D > 0) {
        block_sync();
        const int lane = lane_id(), nw = nt / WAVE;
        for (int b = t / WAVE; b < n_births; b += nw) {
            const int slot = a.free_list[tb + b];
            const DetFeat f = det_feat(a, s, db, a.high[db + a.rest[db + a.birth[db + b]]]);
            float *dst = a.feat + (tb + slot) * a.D;
            for (int k = lane; k < a.D; k += WAVE) dst[k] = f(k);
        }
    }
    YTA_STAMP(2);
    // tracked' = [Tracked survivors of tracked_stracks] ++ births ++ re-found (:257-261)
    auto with_flags = [&](int, int slot) { return SlotFlags{slot, a.flags[tb + slot]}; };
    int n_t2 = block_compact_ld<8, false>(
        n_tracked, wsum, [&](int i) { return a.tracked[tb + i]; }, with_flags,
        [&](int, const SlotFlags &v) { return st_of(v.flags) == ST_TRACKED; },
        [&](int, const SlotFlags &v, int pos) { a.t2[tb + pos] = v.slot; });
    for (int b = t; b < n_births; b += nt) a.t2[tb + n_t2 + b] = a.free_list[tb + b];
    n_t2 += n_births;
    const int n_ref = c->n_ref;   // re-found, pool order (k_stage23)
    for (int k = t; k < n_ref; k += nt) a.t2[tb + n_t2 + k] = a.refound[tb + k].x;
    n_t2 += n_ref;
    // lost' = sub(lost, tracked') ++ newly lost, minus ids already in removed_stracks (:262-264);
    // this frame's removals join removed_stracks only now (:265).  The lost-track expiry
    // (:250-253, end_frame == frame_id) is decided in the same pass: ByteTrack: a Lost track was
    // last updated the frame before it was marked lost (an activated Tracked track takes a
    // detection every frame until then), so frame_id = kf_frame - 1 unless it was re-found this
    // frame (frame_id = fid), from the dense array instead of the record's meta line.  l2pos: each
    // lost' track's pool position (its predicted box is pool_box there).
    const int n_act = c->n_act;
    struct LostItem {
        int slot, flags, frame;
    };
    int n_l2 = block_compact_ld<8, false>(
        n_lost, wsum, [&](int i) { return a.lost[tb + i]; },
        [&](int, int sl) {
            LostItem v;
            v.slot = sl;
            v.flags = a.flags[tb + sl];
            v.frame = V == VAR_BYTETRACK ? a.kf_frame[tb + sl] - 1 : bt_meta(a, tb + sl).frame_id;
            return v;
        },
        [&](int, const LostItem &v) {
            int f = v.flags;
            const int frame = V == VAR_BYTETRACK && st_of(f) == ST_TRACKED ? fid : v.frame;
            if (fid - frame > a.max_time_lost) f = (f & ~FL_STATE) | ST_REMOVED | FL_REMOVED_NOW;
            const bool keep = st_of(f) != ST_TRACKED && !(f & FL_EVER_REMOVED);
            if (f & FL_REMOVED_NOW) f = (f & ~FL_REMOVED_NOW) | FL_EVER_REMOVED;
            if (f != v.flags) a.flags[tb + v.slot] = f;
            return keep;
        },
        [&](int i, const LostItem &v, int pos) {
            a.l2[tb + pos] = v.slot;
            a.l2pos[tb + pos] = n_act + i;   // pool = act ++ lost, in list order
        });
    struct LeftItem {
        int x2, pos;
        SlotFlags sf;
    };
    n_l2 += block_compact_ld<4, false>(
        n_left, wsum,
        [&](int i) {
            LeftItem v;
            v.x2 = a.x2[tb + i];
            v.pos = a.left[tb + i];
            v.sf.slot = a.pool[tb + v.pos];
            return v;
        },
        [&](int, LeftItem v) {
            v.sf.flags = a.flags[tb + v.sf.slot];
            return v;
        },
        [&](int, const LeftItem &v) { return v.x2 < 0 && !(v.sf.flags & FL_EVER_REMOVED); },
        [&](int, const LeftItem &v, int pos) {
            a.l2[tb + n_l2 + pos] = v.sf.slot;
            a.l2pos[tb + n_l2 + pos] = v.pos;
        });
    block_sync();
    YTA_STAMP(4);
    // remove_duplicate_stracks (:312-325): pairs with 1 - IoU < 0.15 drop the younger track (set
    // semantics, so pairs are visited in any order).  The grid over lost' keeps outward-rounded
    // float boxes (16 B each: a steady-state lost' list of ~800 fits the LDS arena); a candidate
    // passing the conservative float pre-test is decided on its exact box, read again.
    if (n_t2 > 0 && n_l2 > 0) {
        const int ncell = grid_cells_for(n_l2);
        float4 *lcache = ar.alloc<float4>(n_l2);   // the grid reads boxes through its ids here
        GridView gv{nullptr, ar.alloc<int>(ncell + 1), ar.alloc<int>(n_l2), nullptr, nullptr,
                    ar.alloc<int>(n_l2), nullptr};
        // a lost' box: ByteTrack's lost' tracks are lazily predicted (kf_xyah.hpp)
        struct LostMean {
            double m[8];
            int lag;
        };
        auto lmean_of = [&](int slot_local) {
            LostMean v;
            const long long slot = tb + slot_local;
            const double2 *src = reinterpret_cast<const double2 *>(a.kf + slot * TRK_STRIDE);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const double2 x = src[k];
                v.m[2 * k] = x.x;
                v.m[2 * k + 1] = x.y;
            }
            v.lag = V == VAR_BYTETRACK ? fid - a.kf_frame[slot] : 0;
            return v;
        };
        auto lbox_of = [&](LostMean v) {
            if (V == VAR_BYTETRACK) kf_predict_lost_mean(v.m, v.lag);
            return V == VAR_BOTSORT ? xywh_to_box(v.m) : xyah_mean_to_box(v.m[0], v.m[1], v.m[2], v.m[3]);
        };
        // a lost' track's box is the one stage 1 used, pool_box at its pool position: ByteTrack's
        // lazily predicted mean (k_s1_prep / the last k_finish), BoT-SORT's predicted and warped
        // mean (stage1_lists: the same x + v and kron(I4, R) x + t operations as k_apply's
        // kf_predict / kf_predict_x and kf_gmc on the record, so the same bits, and no record read)
        // each entry's pool position kept beside its float box (one global round trip, not two,
        // for a candidate's exact box) when the arena has room
        int *lpos = ar.try_alloc<int>(n_l2);
        auto exact_lbox = [&](int q) {
            return a.pool_box[tb + (lpos ? lpos[q] : a.l2pos[tb + q])];
        };
        const bool pre = PRE && n_t2 <= nt && n_l2 <= nt;   // block-uniform
        long long pslot = 0;
        Box pbox{0.0, 0.0, 0.0, 0.0};
        if (pre) {
            const int sl = t < n_t2 ? a.t2[tb + t] : 0;
            const int lp = t < n_l2 ? a.l2pos[tb + t] : 0;
            const Box lb = a.pool_box[tb + lp];
            pslot = tb + sl;
            pbox = kf_box<V>(a.kf, pslot);
            if (t < n_l2) {
                lcache[t] = box_outer_f32(lb);
                if (lpos) lpos[t] = lp;
            }
        } else if (V == VAR_BYTETRACK || V == VAR_BOTSORT)
            batched_for2<4>(
                n_l2, [&](int q) { return a.l2pos[tb + q]; },
                [&](int, int pos) {
                    struct PB {
                        Box b;
                        int pos;
                    };
                    return PB{a.pool_box[tb + pos], pos};
                },
                [&](int q, const auto &v) {
                    lcache[q] = box_outer_f32(v.b);
                    if (lpos) lpos[q] = v.pos;
                });
        else
            batched_for2<3>(
                n_l2, [&](int q) { return a.l2[tb + q]; },
                [&](int, int sl) { return lmean_of(sl); },
                [&](int q, const LostMean &v) { lcache[q] = box_outer_f32(lbox_of(v)); });
        block_sync();   // lcache may be the global arena
        grid_build(n_l2, [&](int q) { return box_of_f4(lcache[q]); }, [](int) { return 1.0; }, gv,
                   sh.gs, wsum);
        const GridHdr gh = sh.gs.hdr;
        YTA_STAMP(5);
        struct TBox {
            long long slot;
            Box b;
        };
        auto query = [&](int p, const TBox &v) {
                if (p == 0) YTA_STAMP_ABS(126);   // diagnostic: thread 0's boxes have arrived
#ifdef YTA_STAMPS
                if (p == 0) g_stamps[127] = gh.n_big + 1000000ull * gh.gx * gh.gy;
#endif
                const Box &tbx = v.b;
                auto pair = [&](int q, const float4 &lf) {
#ifdef YTA_STAMPS
                    if (blockIdx.x == 0 && threadIdx.x == 0) g_stamps[125] += 1;
#endif
                    if (!iou_may_exceed(tbx, lf, 0.85)) return;
                    const Box lb = exact_lbox(q);
                    if (!intersects(tbx, lb)) return;
                    if (1 - iou(tbx, lb) < 0.15) {
                        if (track_age(a, v.slot) > track_age(a, tb + a.l2[tb + q]))
                            atomicOr(&dropB[q >> 5], 1u << (q & 31));
                        else
                            atomicOr(&dropA[p >> 5], 1u << (p & 31));
                    }
                };
                // 1 - IoU < 0.15  <=>  IoU > 0.85: only corners within 0.18 w of tbx's
                grid_query_iou_above_f4(gv, gh, lcache, tbx, 0.85, pair,
                                        [&](int q) { pair(q, lcache[q]); });
            };
        if (pre) {
            if (t < n_t2) query(t, TBox{pslot, pbox});
        } else {
            batched_for2<5>(
                n_t2, [&](int p) { return a.t2[tb + p]; },
                [&](int, int sl) {
                    TBox v;
                    v.slot = tb + sl;
                    v.b = kf_box<V>(a.kf, v.slot);
                    return v;
                },
                query);
        }
    }
    lds_sync();
    YTA_STAMP(6);
    // final lists (tracked, lost) and the output slots (activated tracked, in order) in one pass
    // over tracked' (one scan of packed counts), output rows, free slots.  ByteTrack (split stage
    // 1): the next frame's stage-1 pool too (NP): its head = the output slots with their predicted
    // boxes (the output pass holds their means), the unconfirmed = the kept non-activated entries
    // (births), the tail = the final lost list, lazily predicted - what k_s1_prep gathered from the
    // records at the start of the next frame (s1_pool_build), from rows this kernel already reads.
    constexpr bool NPV = V == VAR_BYTETRACK;
    const bool NP = NPV && a.match_thresh <= 1.0;
    ar.lo = 0;   // the dedup grid is dead: its arena holds the output slot list
    int *outslot = reinterpret_cast<int *>(ar.base);
    const bool os_arena = ar.hi >= (size_t)4 * (n_t2 > 0 ? n_t2 : 1);
    int n_tr = 0, n_out = 0;
    for (int base = 0; base < n_t2; base += 8 * nt) {
        const int m = n_t2 - base < 8 * nt ? n_t2 - base : 8 * nt;
        const int per = (m + nt - 1) / nt;
        const int lo = base + t * per;
        const int hi = lo + per < base + m ? lo + per : base + m;
        int sl[8];
        SlotFlags v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k)
            if (lo + k < hi) sl[k] = a.t2[tb + lo + k];
#pragma unroll
        for (int k = 0; k < 8; ++k)
            if (lo + k < hi) v[k] = with_flags(0, sl[k]);
        unsigned keep = 0, outb = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int p = lo + k;
            if (p < hi && !((dropA[p >> 5] >> (p & 31)) & 1u)) {
                keep |= 1u << k;
                if (v[k].flags & FL_ACTIVATED) outb |= 1u << k;
            }
        }
        int tot;   // counts <= 8 * 1024 each: 16 bits apiece
        const int ex = block_exclusive_scan<false>(__popc(keep) | (__popc(outb) << 16), wsum, &tot);
        int pk = n_tr + (ex & 0xFFFF), po = n_out + (ex >> 16);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            if (!((keep >> k) & 1u)) continue;
            const int slot = v[k].slot;
            const int kidx = pk++;
            a.tracked[tb + kidx] = slot;
            atomicOr(&live[slot >> 5], 1u << (slot & 31));
            if ((outb >> k) & 1u) {
                if (os_arena) outslot[po] = slot;
                else a.t2[tb + po] = slot;   // t2 entries < po were all read above
                ++po;
            } else if (NP) {
                a.unc[tb + (kidx - po)] = slot;   // the next pool's unconfirmed, in tracked order
            }
        }
        n_tr += tot & 0xFFFF;
        n_out += tot >> 16;
    }
    const int n_lo = block_compact_ld<8, false>(
        n_l2, wsum, [&](int q) { return a.l2[tb + q]; }, [&](int, int slot) { return slot; },
        [&](int q, int) { return !((dropB[q >> 5] >> (q & 31)) & 1u); },
        [&](int, int slot, int pos) {
            a.lost[tb + pos] = slot;
            atomicOr(&live[slot >> 5], 1u << (slot & 31));
        });
    // free slots below start in cyclic order from the slot after this frame's last birth: births
    // then take ascending slots across frames, so the tracked list (survivors in order, births
    // appended) stays sorted by slot up to a rotation, and the record gathers of k_s1_prep /
    // k_apply / k_finish walk memory in (gapped) ascending order instead of at random.  Read here,
    // so that only LDS is handed over between the output rows and the free-list pass.
    if (t == 0) sh.cur = n_births > 0 ? (a.free_list[tb + n_births - 1] + 1) % a.CAP : c->slot_cursor;
    block_sync();
    YTA_STAMP(7);
    double *out = a.out + tb * 8;
    struct Row {
        Box b;
        TrackMeta m;
    };
    auto put_row = [&](int pos, const Box &b, const TrackMeta &m) {
        double2 *o = reinterpret_cast<double2 *>(out + (long long)pos * 8);
        o[0] = make_double2(b.x1, b.y1);
        o[1] = make_double2(b.x2, b.y2);
        o[2] = make_double2((double)m.id, m.score);
        o[3] = make_double2(m.cls, (double)m.det_ind);
    };
    if (NPV && NP) {
        // output rows + the next pool's head: mean (8 f64) and meta of line 0 per row
        struct MRow {
            double m[8];
            TrackMeta meta;
            int slot;
        };
        batched_for<2>(
            n_out,
            [&](int pos) {
                MRow r;
                r.slot = os_arena ? outslot[pos] : a.t2[tb + pos];
                const double2 *src = reinterpret_cast<const double2 *>(a.kf + (tb + r.slot) * TRK_STRIDE);
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const double2 q = src[k];
                    r.m[2 * k] = q.x;
                    r.m[2 * k + 1] = q.y;
                }
                r.meta = bt_meta(a, tb + r.slot);
                return r;
            },
            [&](int pos, const MRow &r) {
                put_row(pos, xyah_mean_to_box(r.m[0], r.m[1], r.m[2], r.m[3]), r.meta);
                a.pool[tb + pos] = r.slot;   // activated Tracked: multi_predict keeps vh (:35-48)
                a.pool_box[tb + pos] = xyah_mean_to_box(r.m[0] + r.m[4], r.m[1] + r.m[5],
                                                        r.m[2] + r.m[6], r.m[3] + r.m[7]);
            });
        // the next pool's unconfirmed (current box) and its tail: the final lost list, predicted
        // through the frames since each was lost (fid - kf_frame, as s1_pool_build next frame)
        batched_for2<4>(
            n_tr - n_out, [&](int q) { return a.unc[tb + q]; },
            [&](int, int sl) { return kf_box<V>(a.kf, tb + sl); },
            [&](int q, const Box &b) { a.unc_box[tb + q] = b; });
        batched_for2<3>(
            n_lo, [&](int q) { return a.lost[tb + q]; },
            [&](int, int slot) {
                TrkRec r = bt_trk_rec(a, tb, slot);
                r.flags = fid - a.kf_frame[tb + slot];   // pending predicts (state is Lost)
                return r;
            },
            [&](int q, TrkRec r) {
                kf_predict_lost_mean(r.m, r.flags);
                r.flags = ST_LOST;
                a.pool[tb + n_out + q] = r.slot;
                a.pool_box[tb + n_out + q] = bt_pred_box(r);
            });
    } else {
        batched_for<4>(
            n_out,
            [&](int pos) {
                const long long slot = tb + (os_arena ? outslot[pos] : a.t2[tb + pos]);
                Row r;
                r.b = kf_box<V>(a.kf, slot);
                r.m = bt_meta(a, slot);
                return r;
            },
            [&](int pos, const Row &r) { put_row(pos, r.b, r.m); });
    }
    YTA_STAMP(8);
    // every read of the old free list was consumed before the block_sync above (births, t2,
    // sh.cur); the live bits are LDS
    lds_sync();
    const int cur = sh.cur;
    const int n_fr = block_compact<false>(
        a.CAP, wsum,
        [&](int i) {
            const int slot = i + cur < a.CAP ? i + cur : i + cur - a.CAP;
            return !((live[slot >> 5] >> (slot & 31)) & 1u);
        },
        [&](int i, int pos) { a.free_list[tb + pos] = i + cur < a.CAP ? i + cur : i + cur - a.CAP; });
    YTA_STAMP(9);
    if (t == 0) {
        c->n_births = n_births;
        c->next_id = next_id + n_births;
        c->n_t2 = n_t2;
        c->n_l2 = n_l2;
        c->n_tracked = n_tr;
        c->n_lost = n_lo;
        c->n_free = n_fr;
        c->slot_cursor = cur;
        c->n_out = n_out;
        if (c->fb23_mark) {   // split k_stage23 redone over global memory (either block)
            c->n_fallback[1] += 1;
            c->fb23_mark = 0;
        }
        if (a.out_counts) a.out_counts[s] = n_out;
        if (NP) {   // the next frame's stage-1 pool (built above)
            c->n_act = n_out;
            c->n_unc = n_tr - n_out;
            c->n_pool = n_out + n_lo;
        }
        if (a.cnt_mirror) a.cnt_mirror[s] = *c;   // every field above is final
    }
}

// four 256-thread blocks per CU: <= 128 VGPRs (the diagnostic build's stamps would add some)
// NT: threads per block - BLKF (four blocks per CU: many streams) or 1024 (few streams: the
// single block of a stream then takes every pass's items one or two per thread)
template <int V, int NT>
__global__ __launch_bounds__(NT, NT == BLKF ? 4 : 1) void k_finish(BtArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char fsmem[];
    __shared__ FinishShared sh;
    if (V == VAR_BOTSORT && (int)blockIdx.x >= a.S) {
        // split BoT-SORT: k_ema's blocks in this grid.  Independent of the finish work: the EMA
        // rewrites the smoothed features of tracks that took a detection this frame, the finish
        // writes only births' (free slots') features and reads none
        const int b = blockIdx.x - a.S, eb = ema_blocks(a.CAP, NT);
        ema_body(a, b / eb, b % eb);
        return;
    }
    const int s = blockIdx.x;
    if (stream_skipped(a, s)) {   // not updated this frame: no output rows
        if (threadIdx.x == 0) {
            a.cnt[s].n_out = 0;
            if (a.out_counts) a.out_counts[s] = 0;
        }
        return;
    }
    const int words = (a.CAP + 31) / 32;
    const size_t bits_bytes = ((size_t)12 * words + 15) & ~(size_t)15;
    unsigned *bits = reinterpret_cast<unsigned *>(fsmem);
    // the dedup grid's arena: LDS when lost' (<= lost + leftovers) fits, else global
    YTA_STAMP_BASE(80);
    YTA_STAMP(0);
    const BtCounters *c = a.cnt + s;
    const long long need = dedup_arena_bytes(c->n_lost + c->n_left);
    YTA_BLK(5, 0);
    if (need <= (long long)a.lds_bytes_f) {
        Arena ar(fsmem + bits_bytes, a.lds_bytes_f);
        finish_body<V, NT == 1024>(a, s, bits, ar, sh, true);
    } else {   // a global arena: here, or by k_redo_finish
        if (threadIdx.x == 0) a.cnt[s].n_fallback_f += 1;
        if (redo_in_place(a, a.S)) {
            Arena ag(redo_arena(a, s), a.ws_stride);
            finish_body<V>(a, s, bits, ag, sh, false);
        } else if (threadIdx.x == 0) {
            redo_queue(a, s);
        }
    }
    YTA_BLK(5, 1);
}
template <int V, int NT>
__global__ __launch_bounds__(NT) void k_redo_finish(BtArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char fsmem[];
    __shared__ FinishShared sh;
    unsigned *bits = reinterpret_cast<unsigned *>(fsmem);
    redo_drain(a, [&](int s, Arena &ag) { finish_body<V>(a, s, bits, ag, sh, false); });
}

// Rebuild the free-slot list of every stream from its tracked + lost lists (after a reserve).
// Host-buffer update: every stream's output rows (a.out + s * CAP * 8) packed back to back at the
// prefix offsets, so one copy returns them.  Block per stream, 16-B pieces.  Rows at or past
// `limit` (the destination's capacity) are not written: the host compares the offsets with it.
__global__ __launch_bounds__(256) void k_pack_out(const double *src, long long cap_rows,
                                                   const int *off, double *dst, long long limit) {
    const int s = blockIdx.x;
    const long long end = min((long long)off[s + 1], limit);
    const long long n2 = max(end - (long long)off[s], 0LL) * 4;   // double2 pieces
    const double2 *a = reinterpret_cast<const double2 *>(src + s * cap_rows * 8);
    double2 *b = reinterpret_cast<double2 *>(dst + (long long)off[s] * 8);
    for (long long k = threadIdx.x; k < n2; k += blockDim.x) b[k] = a[k];
}

// Host-buffer update of a small engine: the packed rows' offsets from the streams' output counts
// on the device (one thread: S is small here), so rows and counters come back in one round trip.
__global__ void k_out_offsets(const BtCounters *cnt, int S, int cap, int *off) {
    if (threadIdx.x != 0) return;
    int r = 0;
    off[0] = 0;
    for (int s = 0; s < S; ++s) {   // clamped: a stream with error flags may hold any count
        r += min(max(cnt[s].n_out, 0), cap);
        off[s + 1] = r;
    }
}

// float32 detection rows (what a float32 detector hands over; the reference promotes them to
// float64 exactly, byte_tracker.py:143) widened to the float64 rows the kernels read: n values,
// two per thread (8-B loads, 16-B stores).
__global__ __launch_bounds__(256) void k_widen_f32(const float *src, double *dst, long long n) {
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; 2 * i < n; i += stride) {
        if (2 * i + 1 < n) {
            const float2 v = reinterpret_cast<const float2 *>(src)[i];
            reinterpret_cast<double2 *>(dst)[i] = make_double2((double)v.x, (double)v.y);
        } else {
            dst[2 * i] = (double)src[2 * i];
        }
    }
}

// Pipelined host-buffer update (any S): the same prefix offsets from one 1024-thread block, each
// thread summing a run of streams, then a block scan.
constexpr int OFFS_T = 1024;
__global__ __launch_bounds__(OFFS_T) void k_out_offsets_scan(const BtCounters *cnt, int S, int cap,
                                                              int *off, int *off_host) {
    __shared__ int part[OFFS_T];
    const int t = threadIdx.x;
    const int per = (S + OFFS_T - 1) / OFFS_T, s0 = min(S, t * per), s1 = min(S, s0 + per);
    int sum = 0;
    for (int s = s0; s < s1; ++s) sum += min(max(cnt[s].n_out, 0), cap);
    part[t] = sum;
    __syncthreads();
    for (int d = 1; d < OFFS_T; d <<= 1) {   // inclusive Hillis-Steele scan
        const int v = t >= d ? part[t - d] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    int r = part[t] - sum;   // exclusive prefix of this thread's run
    if (t == 0) {
        off[0] = 0;
        if (off_host) off_host[0] = 0;
    }
    for (int s = s0; s < s1; ++s) {
        r += min(max(cnt[s].n_out, 0), cap);
        off[s + 1] = r;
        if (off_host) off_host[s + 1] = r;   // mapped host memory: no copy on the copy-out stream
    }
}

// Pipelined path: a frame's packed rows (off[S] of them, 64 B each) stored by the copy-out
// stream's kernel straight into mapped page-locked host memory (the caller's buffer or the slot's
// staging), 16-B pieces a lane, so a wave writes 1 KiB runs over PCIe.  Replaces the copy engine's
// device -> host copy, whose enqueue held the host until that stream drained (r05e:
// yta_bytetrack_pipe_stats host_d2h_call_ms ~1.7-1.8 ms a frame).  tools/pcie_bench.hip: 55 GB/s
// from 64 blocks, as the copy engines, and 88 GB/s beside a copy-engine host -> device copy.
// Round 6 (traces: tools/pipe_timeline.py, tools/trace_dump.py, gpurun_out/r6d-r6s): with 128
// blocks of plain stores, every other command completing while the rows streamed out took ~1 ms
// longer (an empty kernel on the copy-in stream ran 1.1 ms; the event the compute stream waited on
// behind it followed), so each frame's kernels started ~1.3 ms after their copy-in had ended;
// with system-coherent write-through stores (sc0 sc1: no dirty host lines left in L2 for another
// command's release to flush) the completions were prompt but the frame's first kernel ran
// 1.7 ms beside them.  Fewer blocks keep fewer host stores in flight: 2048 streams, 3 frames in
// flight, page-locked buffers, same box: 128 blocks 574 k calls/s, 64 620 k, 48 700 k, 32 750 k,
// 24 743 k, 16 717 k, 8 605 k; 32 blocks with plain stores 563 k.
constexpr int ROWS_H_BLOCKS = 32;
#ifndef YTA_D2H_STORE
#define YTA_D2H_STORE 2   // k_rows_to_host's stores: 0 plain, 1 nontemporal, 2 sc0 sc1, 3 sc0 sc1 nt
#endif
__global__ __launch_bounds__(1024) void k_copy_ints(const int *src, int *dst, int n) {
    for (int i = threadIdx.x; i < n; i += blockDim.x) dst[i] = src[i];
}
__global__ __launch_bounds__(256) void k_rows_to_host(const double *src, const int *off, int S,
                                                      long long limit, int4 *dst) {
    // int4 pieces of the packed rows, never past the destination's `limit` rows (the collect
    // compares off[S] with it and reports the frame)
    const long long n = min((long long)off[S], limit) * 4;
    const int4 *s4 = reinterpret_cast<const int4 *>(src);
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x) {
#if YTA_D2H_STORE >= 1
        typedef int v4i __attribute__((ext_vector_type(4)));
        const v4i v = reinterpret_cast<const v4i *>(s4)[i];
        v4i *d = reinterpret_cast<v4i *>(dst) + i;
#if YTA_D2H_STORE == 1
        __builtin_nontemporal_store(v, d);
#elif YTA_D2H_STORE == 2
        asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(d), "v"(v) : "memory");
#else
        asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1 nt" ::"v"(d), "v"(v) : "memory");
#endif
#else
        dst[i] = s4[i];
#endif
    }
}

// Pipelined path: the frame's counters stored straight into mapped, coherent host memory (16-B
// pieces over PCIe) by the compute stream, so the copy-out stream carries only the rows: a small
// hipMemcpyAsync device -> host there held the host until that stream drained (r05d:
// yta_bytetrack_pipe_stats host_small_d2h_ms ~1-2 ms a frame, which serialised the pipeline).
__global__ __launch_bounds__(256) void k_cnt_to_host(const BtCounters *cnt, int S, int4 *dst) {
    const int4 *src = reinterpret_cast<const int4 *>(cnt);
    const long long n = (long long)S * (long long)(sizeof(BtCounters) / sizeof(int4));
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

__global__ __launch_bounds__(BLKF) void k_rebuild_free(BtArgs a) {
    __shared__ int wsum[32];
    extern __shared__ __attribute__((aligned(16))) unsigned int live[];
    const int s = blockIdx.x, t = threadIdx.x;
    BtCounters *c = a.cnt + s;
    const long long tb = (long long)s * a.CAP;
    const int words = (a.CAP + 31) / 32;
    for (int w = t; w < words; w += (int)blockDim.x) live[w] = 0u;
    block_sync();
    for (int i = t; i < c->n_tracked; i += (int)blockDim.x) {
        const int slot = a.tracked[tb + i];
        atomicOr(&live[slot >> 5], 1u << (slot & 31));
    }
    for (int i = t; i < c->n_lost; i += (int)blockDim.x) {
        const int slot = a.lost[tb + i];
        atomicOr(&live[slot >> 5], 1u << (slot & 31));
    }
    block_sync();
    const int cur = c->slot_cursor < a.CAP ? c->slot_cursor : 0;   // cyclic order, as k_finish
    const int n_free = block_compact(
        a.CAP, wsum,
        [&](int i) {
            const int slot = i + cur < a.CAP ? i + cur : i + cur - a.CAP;
            return !((live[slot >> 5] >> (slot & 31)) & 1u);
        },
        [&](int i, int pos) { a.free_list[tb + pos] = i + cur < a.CAP ? i + cur : i + cur - a.CAP; });
    if (t == 0) c->n_free = n_free;
}

__global__ void k_reset(BtArgs a, int s0) {
    const int s = s0 + blockIdx.x;
    const long long tb = (long long)s * a.CAP;
    for (int i = threadIdx.x; i < a.CAP; i += blockDim.x) a.free_list[tb + i] = i;
    if (threadIdx.x == 0) {
        BtCounters z;
        memset(&z, 0, sizeof(z));
        z.n_free = a.CAP;
        a.cnt[s] = z;
    }
}

}  // namespace
}  // namespace yta

// ================================================================================== host engine
using namespace yta;

#ifndef YTA_PIPE_DEPTH
#define YTA_PIPE_DEPTH 3
#endif
constexpr int PIPE_DEPTH = YTA_PIPE_DEPTH;   // frames in flight of the pipelined host-buffer update
// yta_bytetrack_pipe_stats slots (include/yolo_tracking_amd.h): frames collected; detection
// bytes DMA'd straight from the caller / staged through pinned buffers; row bytes DMA'd straight
// into the caller / staged; host ms staging detections, in submit, waiting in collect, copying
// rows out; GPU ms of the copy-in, the kernels (+ row snapshot), the copy-out (per frame, from
// its events) and of a frame's whole span (copy-in start to copy-out end)
enum {
    PS_FRAMES, PS_IN_DIRECT, PS_IN_STAGED, PS_OUT_DIRECT, PS_OUT_STAGED, PS_STAGE_IN_MS,
    PS_SUBMIT_MS, PS_WAIT_MS, PS_COPY_OUT_MS, PS_GPU_IN_MS, PS_GPU_KERN_MS, PS_GPU_OUT_MS,
    PS_GPU_SPAN_MS, PS_H2D_CALL_MS, PS_LAUNCH_MS, PS_D2H_CALL_MS, PS_SMALL_H2D_MS, PS_SMALL_D2H_MS,
    PS_PINNED_CHECK_MS, PS_CAP_WAITS, PS_CAP_DRAINS, PS_N
};
static_assert(PS_N <= 24, "pstat holds 24 slots");
// Direct copies of the pipelined path in pieces of YTA_PIPE_CHUNK_MB (0: one copy each way)
static size_t pipe_chunk_bytes() {
    static const size_t c = [] {
        const char *v = getenv("YTA_PIPE_CHUNK_MB");
        return v ? (size_t)atoi(v) << 20 : (size_t)0;
    }();
    return c;
}
static bool env_flag(const char *name, bool dflt) {
    const char *v = getenv(name);
    return v ? atoi(v) != 0 : dflt;
}
static int env_int(const char *name, int dflt) {
    const char *v = getenv(name);
    return v ? atoi(v) : dflt;
}
// Per-frame GPU timing events of the pipelined path (yta_bytetrack_pipe_stats' GPU columns)
static bool pipe_timing() {
    static const bool k = env_flag("YTA_PIPE_TIMING", false);
    return k;
}
// Each frame slot copies in on its own stream (else one copy-in stream for all)
static bool pipe_slot_streams() {
    static const bool k = env_flag("YTA_PIPE_SLOT_STREAMS", false);
    return k;
}
// The copy-in / copy-out streams at the device's greatest stream priority (YTA_PIPE_PRIO: bit 0
// copy-in, bit 1 copy-out; default 3 = both).  The HIP runtime maps a process's streams onto at
// most GPU_MAX_HW_QUEUES hardware queues per priority (4 on the pool) and, past that, shares the
// least-used one.  In bench.py's process (two headline engines alive) the pipelined engine's
// streams shared queues: a frame's copy-in waited behind the previous frame's kernels and
// k_rows_to_host's ~2.4 ms of host stores ran beside nothing - 535 k calls/s page-locked against
// 711 k with GPU_MAX_HW_QUEUES=8.  The greater priority draws from its own pool of queues, which
// no compute stream uses (gpurun_out/r6z2: both 710 k, copy-out alone 534 k, a dedicated queue
// per stream through an every-CU mask 708 k).
static hipError_t pipe_stream_create(hipStream_t *st, int which) {
    static const int prio = env_int("YTA_PIPE_PRIO", 3);
    if (!(prio & (1 << which))) return hipStreamCreateWithFlags(st, hipStreamNonBlocking);
    int lo = 0, hi = 0;
    const hipError_t r = hipDeviceGetStreamPriorityRange(&lo, &hi);
    if (r != hipSuccess) return r;
    return hipStreamCreateWithPriority(st, hipStreamNonBlocking, hi);
}
// A frame's detection offsets read by the compute stream from the slot's mapped host copy
// (k_copy_ints) instead of a small copy on the copy-in stream
static bool pipe_off_kernel() {
    static const bool k = env_flag("YTA_PIPE_OFF_KERNEL", false);
    return k;
}
// k_rows_to_host's grid (YTA_PIPE_D2H_BLOCKS overrides ROWS_H_BLOCKS, for A/B runs)
static int pipe_d2h_blocks() {
    static const int k = [] {
        const char *v = getenv("YTA_PIPE_D2H_BLOCKS");
        const int b = v ? atoi(v) : ROWS_H_BLOCKS;
        return b < 1 ? 1 : (b > 4096 ? 4096 : b);
    }();
    return k;
}
// Rows device -> host by k_rows_to_host (1, default) or by the copy engines (YTA_PIPE_KERNEL_D2H=0)
static bool pipe_kernel_d2h() {
    static const bool k = [] {
        const char *v = getenv("YTA_PIPE_KERNEL_D2H");
        return !v || atoi(v) != 0;
    }();
    return k;
}
static hipError_t copy_pieces(void *dst, const void *src, size_t bytes, hipMemcpyKind kind,
                              hipStream_t st) {
    const size_t ch = pipe_chunk_bytes() ? pipe_chunk_bytes() : bytes;
    for (size_t o = 0; o < bytes; o += ch) {
        const hipError_t e = hipMemcpyAsync((char *)dst + o, (const char *)src + o,
                                            std::min(ch, bytes - o), kind, st);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

struct yta_bytetrack {
    int device = 0, S = 0, CAP = 0, MAXD = 0;
    int variant = VAR_BYTETRACK, D = 0;
    yta_bytetrack_params prm{};
    yta_botsort_params bprm{};
    // BoT-SORT: per-frame ReID rows aligned with the detections (host staging + device)
    float *h_feat = nullptr, *d_feat_in = nullptr;
    long long feat_cap = 0;
    hipStream_t stream = nullptr;
    double *d_warp = nullptr, *d_warp_id = nullptr;   // BoT-SORT: staged warps / identity warps
    std::vector<void *> allocs;
    BtArgs a{};
    // host staging
    double *h_dets = nullptr;
    // host-buffer outputs: the streams' rows packed on the device, one copy back
    double *d_pack = nullptr, *h_pack = nullptr;
    int *d_pack_off = nullptr, *h_pack_off = nullptr;
    long long pack_cap = 0;
    int *h_off = nullptr;
    BtCounters *h_cnt = nullptr;
    double *d_det_in = nullptr;
    long long d_det_cap = 0;
    int *d_det_off = nullptr;
    float *d_det32 = nullptr, *h_det32 = nullptr;   // float32 detection rows (before widening)
    long long det32_cap = 0;
    // BoT-SORT with ReID: stage 1 as k_bs_prep / k_bs_edges / k_bs_lap (few streams) instead of
    // the fused k_stage1 (set at create; YTA_BS_SPLIT=0 / 1 overrides)
    bool bs_split = false;
    // few streams: k_stage23's two stages in two blocks per stream (set at create; YTA_SPLIT23=0 / 1
    // overrides)
    bool split23 = false;
    // stream-subset updates: the [S] mask on the device and its pinned staging
    int *d_active = nullptr, *h_active = nullptr;
    // the engine's own [S * CAP][8] output rows (the host-buffer paths); a.out is whatever buffer
    // the last launch wrote (the caller's on the device-buffer path)
    double *out_own = nullptr;
    // pipelined host-buffer updates (yta_bytetrack_submit / _collect): PIPE_DEPTH frame slots, a
    // copy-in and a copy-out stream beside the compute stream
    struct PipeSlot {
        double *d_in = nullptr, *h_in = nullptr;     // detections (pinned staging for pageable)
        long long in_cap = 0;
        float *d_in32 = nullptr, *h_in32 = nullptr;  // float32 detections (before widening)
        long long in32_cap = 0;
        int *d_off = nullptr, *h_off = nullptr;      // S + 1 detection offsets
        double *d_pack = nullptr, *h_pack = nullptr; // packed output rows
        long long pack_cap = 0;
        int *d_pack_off = nullptr, *h_pack_off = nullptr;   // S + 1 row offsets
        BtCounters *d_cnt = nullptr, *h_cnt = nullptr;      // counters after this frame (d_cnt unused)
        BtCounters *m_cnt = nullptr;                 // h_cnt as the device sees it (mapped)
        int *m_pack_off = nullptr;                   // h_pack_off as the device sees it
        double *m_pack = nullptr;                    // h_pack as the device sees it
        long long *h_nid = nullptr;                  // next_id staging
        hipEvent_t in_done = nullptr, kern_done = nullptr, out_done = nullptr;   // dependencies
        // timing events (YTA_PIPE_TIMING=1 only): start / end of the slot's copy-in, kernels and
        // copy-out, for yta_bytetrack_pipe_stats
        hipEvent_t t_ev[6] = {};
        int *m_off = nullptr;                        // h_off as the device sees it (mapped)
        hipStream_t s_in = nullptr;                  // this slot's copy-in stream
        bool own_s_in = false;                       // (its own, YTA_PIPE_SLOT_STREAMS=1)
        double *user_out = nullptr;                  // the caller's buffer
        long long rows_bound = 0;                    // det_offsets[S] of the frame
        bool direct_out = false;                     // DMA straight into user_out
        long long in_bytes = 0;                      // detection bytes over the link
        bool direct_in = false;                      // DMA straight from the caller's buffer
        bool dirty = false;                          // an enqueue failed part way: wait first
    };
    PipeSlot pipe[PIPE_DEPTH];
    int pipe_head = 0, pipe_count = 0;
    hipStream_t s_in = nullptr, s_out = nullptr;
    // pipelined-path accounting (yta_bytetrack_pipe_stats): PIPE_STATS doubles
    double pstat[24] = {};
    // optional per-kernel timing with HIP events on the engine stream
    bool prof = false;
    // small host-buffer updates: the frame's launches, the packing and the copies back replayed
    // as one HIP graph, captured with the arguments below and re-captured when they change
    // (YTA_GRAPHS=0 disables)
    bool graphs = true;
    hipGraph_t g_graph = nullptr;
    hipGraphExec_t g_exec = nullptr;
    BtArgs g_args{};
    const void *g_ptrs[5] = {};
    long long g_cap = -1;
    long long g_captures = 0, g_replays = 0;   // yta_bytetrack_modes
    std::vector<hipEvent_t> ev;
    size_t ev_used = 0;
    // host-buffer staging copies: persistent worker threads (created on the first large copy)
    std::unique_ptr<CopyPool> pool;
};

namespace {

constexpr int BT_PHASES = 6;   // timed phases per frame, see yta_bytetrack_profile_collect
#ifndef YTA_LDS1_KB
#define YTA_LDS1_KB 150
#endif
constexpr size_t BT_LDS_BYTES = YTA_LDS1_KB * 1024;   // k_stage1 arena (one 1024-thread block per CU)
constexpr size_t BT_LDS23_BYTES = 32 * 1024;  // k_stage23 arena (several blocks per CU)
#ifndef YTA_LDSF_KB
#define YTA_LDSF_KB 32
#endif
constexpr size_t BT_LDSF_BYTES = YTA_LDSF_KB * 1024;   // k_finish dedup arena (four blocks per
                                                      // CU; lost' of 650 at 1024 x 1024)
#ifndef YTA_LDSL_KB
#define YTA_LDSL_KB 38
#endif
constexpr size_t BT_LDSL_BYTES = YTA_LDSL_KB * 1024;   // k_s1_lap arena (four blocks per CU)
#ifndef YTA_LDSE_KB
#define YTA_LDSE_KB 62
#endif
constexpr size_t BT_LDSE_BYTES = YTA_LDSE_KB * 1024;   // k_s1_edges grid (1024 high detections)

// Host-buffer ABI staging: copies between the caller's (pageable) buffers and the pinned staging
// buffers, split over up to 8 host threads, and chunked so that each chunk's DMA overlaps the next
// chunk's host copy.
#ifndef YTA_STAGE_THREADS
#define YTA_STAGE_THREADS 8
#endif
#ifndef YTA_STAGE_CHUNKS
#define YTA_STAGE_CHUNKS 4
#endif
void par_copy(yta_bytetrack *e, void *dst, const void *src, size_t bytes) {
    constexpr size_t MIN_PIECE = 2u << 20;
    const unsigned hw = std::thread::hardware_concurrency();
    const size_t T = std::min<size_t>(std::min<unsigned>(hw ? hw : 1, YTA_STAGE_THREADS),
                                      bytes / MIN_PIECE);
    if (T <= 1) {
        memcpy(dst, src, bytes);
        return;
    }
    if (!e->pool) e->pool.reset(new CopyPool(std::min<unsigned>(hw, YTA_STAGE_THREADS) - 1));
    e->pool->copy(dst, src, bytes, (int)T);
}
constexpr int STAGE_CHUNKS = YTA_STAGE_CHUNKS;

// True when the caller's buffer [p, p + bytes) is page-locked host memory (hipHostMalloc'd or
// hipHostRegister'ed, e.g. a pinned torch tensor's numpy view): the DMA engines then read / write
// it directly and the staging copy is skipped.  Pageable memory makes the query fail; its error
// is cleared.
// Is [p, p + bytes) one page-locked host allocation?  Both ends page-locked is not enough (a
// view spanning two pinned allocations with pageable pages between them): the whole range must
// lie inside the allocation that holds p.  Anything the runtime cannot vouch for is staged.
// dev (optional): the address the GPU's kernels use for p (mapped page-locked memory), or null.
bool host_pinned(const void *p, size_t bytes, void **dev = nullptr) {
    if (dev) *dev = nullptr;
    if (!p || !bytes) return false;
    hipPointerAttribute_t at;
    if (hipPointerGetAttributes(&at, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    if (at.type != hipMemoryTypeHost) return false;
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    if (hipPointerGetAttribute(&base, HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR,
                               (hipDeviceptr_t)p) != hipSuccess ||
        hipPointerGetAttribute(&size, HIP_POINTER_ATTRIBUTE_RANGE_SIZE, (hipDeviceptr_t)p) !=
            hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    const char *b = (const char *)base, *q = (const char *)p;
    const bool inside = b && q >= b && bytes <= size && (size_t)(q - b) <= size - bytes;
    if (inside && dev) *dev = at.devicePointer;
    return inside;
}
inline size_t stage_chunk(size_t bytes) {
    const int n = bytes >= (16u << 20) ? STAGE_CHUNKS : 1;
    return ((bytes + n - 1) / n + 63) & ~(size_t)63;
}

template <typename T>
int dalloc(yta_bytetrack *e, T **p, long long n) {
    void *q = nullptr;
    if (n <= 0) n = 1;
    hipError_t err = hipMalloc(&q, sizeof(T) * (size_t)n);
    if (err != hipSuccess) {
        set_error("hipMalloc(%lld bytes) failed: %s", (long long)(sizeof(T) * n),
                  hipGetErrorString(err));
        return YTA_ERR_NOMEM;
    }
    e->allocs.push_back(q);
    *p = static_cast<T *>(q);
    return YTA_OK;
}

#define DALLOC(ptr, n)                    \
    do {                                  \
        int _rc = dalloc(e, &(ptr), (n)); \
        if (_rc) return _rc;              \
    } while (0)

int bt_alloc(yta_bytetrack *e) {
    const long long S = e->S, CAP = e->CAP, MAXD = e->MAXD;
    BtArgs &a = e->a;
    a.S = e->S;
    a.CAP = e->CAP;
    a.MAXD = e->MAXD;
    if (e->variant == VAR_BOTSORT) {   // bot_sort.py:185-229
        const yta_botsort_params &b = e->bprm;
        a.track_thresh = b.track_high_thresh;
        a.low_thresh = b.track_low_thresh;
        a.det_thresh = b.new_track_thresh;
        a.match_thresh = b.match_thresh;
        a.max_time_lost = (int)(b.frame_rate / 30.0 * b.track_buffer);
        a.prox_thresh = b.proximity_thresh;
        a.app_thresh = b.appearance_thresh;
        a.fuse_first = b.fuse_first_associate;
        a.D = e->D;
    } else {
        a.track_thresh = e->prm.track_thresh;
        a.low_thresh = 0.1;                                                      // :150
        a.match_thresh = e->prm.match_thresh;
        a.det_thresh = e->prm.track_thresh;                                      // :127
        a.max_time_lost = (int)(e->prm.frame_rate / 30.0 * e->prm.track_buffer); // :128-129
        a.D = 0;
    }
    DALLOC(a.kf, S * CAP * TRK_STRIDE);
    if (e->variant == VAR_BOTSORT) {
        DALLOC(a.kfx, S * CAP * 16);
        DALLOC(e->d_warp, S * 6);
        DALLOC(e->d_warp_id, S * 6);
        std::vector<double> id((size_t)S * 6);
        for (int q = 0; q < S; ++q) {
            const double h[6] = {1, 0, 0, 0, 1, 0};
            std::copy(h, h + 6, id.begin() + 6 * q);
        }
        YTA_HIP(hipMemcpy(e->d_warp_id, id.data(), sizeof(double) * 6 * S, hipMemcpyHostToDevice));
        a.warp = e->d_warp_id;
    }
    DALLOC(a.flags, S * CAP);
    DALLOC(a.kf_frame, S * CAP);
    DALLOC(a.tracked, S * CAP);
    DALLOC(a.lost, S * CAP);
    DALLOC(a.free_list, S * CAP);
    DALLOC(a.cnt, S);
    DALLOC(a.high, S * MAXD);
    DALLOC(a.second, S * MAXD);
    DALLOC(a.rest, S * MAXD);
    DALLOC(a.birth, S * MAXD);
    DALLOC(a.high_box, S * MAXD);
    DALLOC(a.second_box, S * MAXD);
    DALLOC(a.high_score, S * MAXD);
    DALLOC(a.rest_score, S * MAXD);
    DALLOC(a.pool, S * CAP);
    DALLOC(a.unc, S * CAP);
    DALLOC(a.left, S * CAP);
    DALLOC(a.left_of_pool, S * CAP);
    DALLOC(a.t2, S * CAP);
    DALLOC(a.l2, S * CAP);
    DALLOC(a.refound, S * CAP);
    DALLOC(a.l2pos, S * CAP);
    DALLOC(a.pool_box, S * CAP);
    DALLOC(a.unc_box, S * CAP);
    DALLOC(a.x1, S * CAP);
    DALLOC(a.x2, S * CAP);
    DALLOC(a.x3, S * CAP);
    DALLOC(a.y1, S * MAXD);
    DALLOC(a.y2, S * MAXD);
    DALLOC(a.y3, S * MAXD);
    DALLOC(a.out, S * CAP * 8 + 16 * S);   // + the counters' mirror (BtArgs::cnt_mirror)
    e->out_own = a.out;
    if (e->variant == VAR_BOTSORT) {
        DALLOC(a.cls_hist, S * CAP * CLS_K);
        if (e->D > 0) {
            DALLOC(a.feat, S * CAP * e->D);
            DALLOC(a.det_fn, S * MAXD * 4);
            DALLOC(a.ema_job, S * CAP);
        }
    }
    // association: LDS arena first; the global fallback arena holds the worst case (every pair a
    // candidate edge), so no frame can overflow it
    a.lds_bytes = BT_LDS_BYTES;
    a.lds_bytes23 = BT_LDS23_BYTES;
    a.lds_bytes_f = BT_LDSF_BYTES;
    a.lds_bytes_l = BT_LDSL_BYTES;
    a.lds_bytes_e = BT_LDSE_BYTES;
    a.ws_stride = assoc_arena_bytes(CAP, MAXD, CAP * MAXD);
    if (e->variant == VAR_BOTSORT && e->D > 0) {   // split stage 1 (k_bs_edges / k_bs_lap)
        a.ws_stride = std::max(a.ws_stride, s1_lap_arena_bytes(CAP, MAXD, CAP * MAXD));
        DALLOC(a.e_cnt, S * CAP);
        DALLOC(a.e_col, E_SLOTS * S * CAP);
        DALLOC(a.e_cost, E_SLOTS * S * CAP);
    }
    if (e->variant == VAR_BYTETRACK) {   // stage 1 as k_s1_prep / k_s1_edges / k_s1_lap
        a.ws_stride = std::max(a.ws_stride, s1_lap_arena_bytes(CAP, MAXD, CAP * MAXD));
        DALLOC(a.g_cell, S * (GRID_MAX_CELLS + 1));
        DALLOC(a.g_ids, S * MAXD);
        DALLOC(a.g_big, S * MAXD);
        DALLOC(a.g_boxes, S * MAXD);
        DALLOC(a.g_w, S * MAXD);
        DALLOC(a.g_hdr, S);
        DALLOC(a.e_cnt, S * CAP);
        DALLOC(a.g_deg, S * MAXD);
        DALLOC(a.e_col, E_SLOTS * S * CAP);
        DALLOC(a.e_cost, E_SLOTS * S * CAP);
    }
    if (e->variant == VAR_BOTSORT && e->D > 0)
        a.ws_stride = std::max(a.ws_stride, assoc_emb_arena_bytes(CAP, MAXD));
    a.ws_stride = (a.ws_stride + 255) & ~255LL;
    a.split23 = e->split23;
    a.ws3 = nullptr;
    {   // pooled fallback arenas (redo_drain): enough for every block of a few-stream engine, a
        // bounded pool for many streams (YTA_WS_POOL overrides the bound, 2..256)
        int pool = 32;
        if (const char *v = getenv("YTA_WS_POOL")) pool = std::max(2, std::min(256, atoi(v)));
        a.ws_slots = (int)std::min<long long>(S * (a.split23 ? 2 : 1), pool);
    }
    DALLOC(a.ws, (long long)a.ws_slots * a.ws_stride);
    DALLOC(a.redo_q, 2 + 2 * S);
    YTA_HIP(hipMemset(a.redo_q, 0, 2 * sizeof(int)));
    a.slab.R = (int)CAP;
    a.slab.C = (int)MAXD;
    a.slab.i_stride = lap_slab_ints((int)CAP, (int)MAXD);
    a.slab.d_stride = lap_slab_doubles((int)CAP, (int)MAXD);
    DALLOC(a.slab.i, S * SLAB_WAVES * a.slab.i_stride);
    DALLOC(a.slab.d, S * SLAB_WAVES * a.slab.d_stride);
    DALLOC(e->d_det_off, S + 1);
    DALLOC(e->d_active, S);
    YTA_HIP(hipHostMalloc((void **)&e->h_off, sizeof(int) * (S + 1), hipHostMallocDefault));
    YTA_HIP(hipHostMalloc((void **)&e->h_cnt, sizeof(BtCounters) * S, hipHostMallocDefault));
    return YTA_OK;
}

int mark(yta_bytetrack *e) {
    if (!e->prof) return YTA_OK;
    if (e->ev_used == e->ev.size()) {
        hipEvent_t h;
        YTA_HIP(hipEventCreate(&h));
        e->ev.push_back(h);
    }
    YTA_HIP(hipEventRecord(e->ev[e->ev_used++], e->stream));
    return YTA_OK;
}

#define MARK()             \
    do {                   \
        int _m = mark(e);  \
        if (_m) return _m; \
    } while (0)

int set_lds_limits(size_t bytes) {
    const int b = (int)bytes;
    for (const void *k : {(const void *)k_stage1<VAR_BYTETRACK>, (const void *)k_stage1<VAR_BOTSORT>,
                          (const void *)k_bs_lap, (const void *)k_stage23<VAR_BYTETRACK, false>,
                          (const void *)k_stage23<VAR_BOTSORT, false>,
                          (const void *)k_stage23<VAR_BYTETRACK, true>,
                          (const void *)k_stage23<VAR_BOTSORT, true>, (const void *)k_s1_lap<BLKL>,
                          (const void *)k_s1_lap<1024>})
        YTA_HIP(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, b));
    // k_s1_edges never launches with more than BT_LDSE_BYTES (its wave queues are static LDS)
    for (const void *k : {(const void *)k_s1_edges<BLKE>, (const void *)k_s1_edges<1024>})
        YTA_HIP(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)std::min(bytes, BT_LDSE_BYTES)));
    return YTA_OK;
}

// One frame of every stream: 6 launches (ByteTrack), 4 + k_feat and k_ema (BoT-SORT, fused stage
// 1); with more streams than pooled fallback arenas each association kernel is followed by its
// redo kernel (ws_slots blocks that return at once unless a stream fell back).  Profiling marks bracket the phases s1_prep / s1_edges / s1_lap (BoT-SORT: k_feat + k_stage1,
// empty, empty), stage23, apply (k_apply + k_ema), finish.
// a launch of more association blocks than pooled arenas queues its fallbacks for a redo kernel
// (redo_in_place on the device)
#ifndef YTA_REDO_LAUNCH
#define YTA_REDO_LAUNCH 1   // 0: an A/B build without the redo launches (unsafe if a stream falls back)
#endif
static bool redo_launch(const BtArgs &a, int blocks) { return YTA_REDO_LAUNCH && blocks > a.ws_slots; }

template <int V>
int launch_frame(yta_bytetrack *e) {
    BtArgs &a = e->a;
    const bool reid = V == VAR_BOTSORT && a.D > 0;
    // split BoT-SORT stage 1 (few streams): k_feat's blocks ride in k_bs_prep's grid and k_ema's
    // in k_finish's (two launches fewer on a latency-bound chain)
    const bool bs = V == VAR_BOTSORT && reid && e->bs_split && a.prox_thresh < 1.0 &&
                    a.match_thresh <= 1.0;
    MARK();
    if (reid && !bs) {
        const dim3 gf((a.MAXD + FEAT_T / WAVE - 1) / (FEAT_T / WAVE), a.S);
        hipLaunchKernelGGL(k_feat, gf, dim3(FEAT_T), 0, e->stream, a);
        YTA_HIP(hipGetLastError());
    }
    if (V == VAR_BYTETRACK && a.match_thresh <= 1.0) {   // grid-exact candidates (assoc.hpp)
        if (e->split23)
            hipLaunchKernelGGL(k_s1_prep<1024>, dim3(a.S), dim3(1024), 0, e->stream, a);
        else
            hipLaunchKernelGGL(k_s1_prep<PREP_T>, dim3(a.S), dim3(PREP_T), 0, e->stream, a);
        YTA_HIP(hipGetLastError());
        MARK();
        if (e->split23)
            hipLaunchKernelGGL(k_s1_edges<1024>, dim3(a.S), dim3(1024), a.lds_bytes_e, e->stream, a);
        else
            hipLaunchKernelGGL(k_s1_edges<BLKE>, dim3(a.S), dim3(BLKE), a.lds_bytes_e, e->stream, a);
        YTA_HIP(hipGetLastError());
        MARK();
        if (e->split23) {
            hipLaunchKernelGGL(k_s1_lap<1024>, dim3(a.S), dim3(1024), a.lds_bytes_l, e->stream, a);
            if (redo_launch(a, a.S))
                hipLaunchKernelGGL(k_redo_s1_lap<1024>, dim3(a.ws_slots), dim3(1024), 0, e->stream, a);
        } else {
            hipLaunchKernelGGL(k_s1_lap<BLKL>, dim3(a.S), dim3(BLKL), a.lds_bytes_l, e->stream, a);
            if (YTA_REDO_LAUNCH)
                hipLaunchKernelGGL(k_redo_s1_lap<BLKL>, dim3(a.ws_slots), dim3(BLKL), 0, e->stream, a);
        }
    } else if (bs) {   // split stage 1 (k_bs_*): few streams
        hipLaunchKernelGGL(k_bs_prep, dim3(a.S + a.S * feat_blocks(a.MAXD, BS_PREP_T)),
                           dim3(BS_PREP_T), 0, e->stream, a);
        YTA_HIP(hipGetLastError());
        MARK();
        const dim3 ge((a.CAP + BSE_T / WAVE - 1) / (BSE_T / WAVE), a.S);
        hipLaunchKernelGGL(k_bs_edges, ge, dim3(BSE_T), 0, e->stream, a);
        YTA_HIP(hipGetLastError());
        MARK();
        hipLaunchKernelGGL(k_bs_lap, dim3(a.S), dim3(BLK1), a.lds_bytes, e->stream, a);
        if (redo_launch(a, a.S))
            hipLaunchKernelGGL(k_redo_bs_lap, dim3(a.ws_slots), dim3(BLK1), 0, e->stream, a);
    } else {   // fused stage 1: the whole stage in the first phase, the next two empty
        hipLaunchKernelGGL(k_stage1<V>, dim3(a.S), dim3(BLK1), a.lds_bytes, e->stream, a);
        if (redo_launch(a, a.S))
            hipLaunchKernelGGL(k_redo_stage1<V>, dim3(a.ws_slots), dim3(BLK1), 0, e->stream, a);
        YTA_HIP(hipGetLastError());
        MARK();
        MARK();
    }
    YTA_HIP(hipGetLastError());
    MARK();
    if (a.split23) {
        hipLaunchKernelGGL((k_stage23<V, true>), dim3(2 * a.S), dim3(BLK23S), a.lds_bytes23,
                           e->stream, a);
        if (redo_launch(a, 2 * a.S))
            hipLaunchKernelGGL((k_redo_stage23<V, true>), dim3(a.ws_slots), dim3(BLK23S), 0,
                               e->stream, a);
    } else {
        hipLaunchKernelGGL((k_stage23<V, false>), dim3(a.S), dim3(BLK23), a.lds_bytes23,
                           e->stream, a);
        if (redo_launch(a, a.S))
            hipLaunchKernelGGL((k_redo_stage23<V, false>), dim3(a.ws_slots), dim3(BLK23), 0,
                               e->stream, a);
    }
    YTA_HIP(hipGetLastError());
    MARK();
    const dim3 gt((a.CAP + APPLY_T - 1) / APPLY_T, a.S);
    hipLaunchKernelGGL(k_apply<V>, gt, dim3(APPLY_T), 0, e->stream, a);
    YTA_HIP(hipGetLastError());
    if (reid && !bs) {
        const dim3 ge(ema_blocks(a.CAP), a.S);
        hipLaunchKernelGGL(k_ema, ge, dim3(EMA_T), 0, e->stream, a);
        YTA_HIP(hipGetLastError());
    }
    MARK();
    const size_t bits_bytes = ((size_t)12 * ((a.CAP + 31) / 32) + 15) & ~(size_t)15;
    // few streams: 1024-thread finish blocks (k_ema's blocks in its grid take 16 tracks each)
    if (e->split23) {
        constexpr int FT = 1024;
        hipLaunchKernelGGL((k_finish<V, FT>), dim3(a.S + (bs ? a.S * ema_blocks(a.CAP, FT) : 0)),
                           dim3(FT), bits_bytes + a.lds_bytes_f, e->stream, a);
        if (redo_launch(a, a.S))
            hipLaunchKernelGGL((k_redo_finish<V, FT>), dim3(a.ws_slots), dim3(FT), bits_bytes,
                               e->stream, a);
    } else {
        hipLaunchKernelGGL((k_finish<V, BLKF>), dim3(a.S + (bs ? a.S * ema_blocks(a.CAP, BLKF) : 0)),
                           dim3(BLKF), bits_bytes + a.lds_bytes_f, e->stream, a);
        if (redo_launch(a, a.S))
            hipLaunchKernelGGL((k_redo_finish<V, BLKF>), dim3(a.ws_slots), dim3(BLKF), bits_bytes,
                               e->stream, a);
    }
    YTA_HIP(hipGetLastError());
    MARK();
    return YTA_OK;
}

int launch_pipeline(yta_bytetrack *e, const double *det_in, const int *det_off, double *out,
                    int *out_counts, const float *det_feat = nullptr) {
    BtArgs &a = e->a;
    a.det_in = det_in;
    a.det_off = det_off;
    a.out = out;
    a.out_counts = out_counts;
    a.det_feat = det_feat;
    return e->variant == VAR_BOTSORT ? launch_frame<VAR_BOTSORT>(e)
                                     : launch_frame<VAR_BYTETRACK>(e);
}

void release_buffers(yta_bytetrack *e) {
    for (void *p : e->allocs) (void)hipFree(p);
    e->allocs.clear();
    if (e->h_off) (void)hipHostFree(e->h_off);
    if (e->h_cnt) (void)hipHostFree(e->h_cnt);
    e->h_off = nullptr;
    e->h_cnt = nullptr;
}

// Grow track capacity and/or max detections, keeping every stream's tracker state.
int reserve(yta_bytetrack *e, int cap, int maxd) {
    if (cap <= e->CAP && maxd <= e->MAXD) return YTA_OK;
    cap = std::max(cap, e->CAP);
    maxd = std::max(maxd, e->MAXD);
    YTA_HIP(host_wait(e->stream));
    yta_bytetrack *n = new (std::nothrow) yta_bytetrack();
    YTA_CHECK(n, YTA_ERR_NOMEM, "out of host memory");
    n->device = e->device;
    n->S = e->S;
    n->CAP = cap;
    n->MAXD = maxd;
    n->prm = e->prm;
    n->variant = e->variant;
    n->D = e->D;
    n->bprm = e->bprm;
    n->stream = e->stream;
    // every create-time mode bt_alloc reads (the split stage 2 / 3 blocks, the fallback pool size)
    n->split23 = e->split23;
    n->bs_split = e->bs_split;
    n->graphs = e->graphs;
    int rc = bt_alloc(n);
    const size_t S = e->S, oc = e->CAP, nc = cap;
    auto copy2d = [&](void *dst, size_t dpitch, const void *src, size_t spitch, size_t width,
                      size_t height) -> int {
        YTA_HIP(hipMemcpy2DAsync(dst, dpitch, src, spitch, width, height, hipMemcpyDeviceToDevice,
                                 e->stream));
        return YTA_OK;
    };
    if (!rc)
        rc = copy2d(n->a.kf, nc * TRK_STRIDE * 8, e->a.kf, oc * TRK_STRIDE * 8,
                    oc * TRK_STRIDE * 8, S);
    if (!rc && e->a.kfx) rc = copy2d(n->a.kfx, nc * 16 * 8, e->a.kfx, oc * 16 * 8, oc * 16 * 8, S);
    if (!rc) rc = copy2d(n->a.flags, nc * 4, e->a.flags, oc * 4, oc * 4, S);
    if (!rc) rc = copy2d(n->a.kf_frame, nc * 4, e->a.kf_frame, oc * 4, oc * 4, S);
    if (!rc && e->a.cls_hist)
        rc = copy2d(n->a.cls_hist, nc * CLS_K * 16, e->a.cls_hist, oc * CLS_K * 16,
                    oc * CLS_K * 16, S);
    if (!rc && e->a.feat) {
        const size_t row = (size_t)e->D * 4;
        rc = copy2d(n->a.feat, nc * row, e->a.feat, oc * row, oc * row, S);
    }
    if (!rc) rc = copy2d(n->a.tracked, nc * 4, e->a.tracked, oc * 4, oc * 4, S);
    if (!rc) rc = copy2d(n->a.lost, nc * 4, e->a.lost, oc * 4, oc * 4, S);
    if (!rc) {
        hipError_t he = hipMemcpyAsync(n->a.cnt, e->a.cnt, sizeof(BtCounters) * S,
                                       hipMemcpyDeviceToDevice, e->stream);
        if (he != hipSuccess) {
            set_error("reserve copy: %s", hipGetErrorString(he));
            rc = YTA_ERR_HIP;
        }
    }
    if (!rc) {
        const size_t live_bytes = sizeof(unsigned int) * ((nc + 31) / 32);
        hipLaunchKernelGGL(k_rebuild_free, dim3(e->S), dim3(BLKF), live_bytes, e->stream, n->a);
        hipError_t he = hipGetLastError();
        if (he == hipSuccess) he = host_wait(e->stream);
        if (he != hipSuccess) {
            set_error("reserve: %s", hipGetErrorString(he));
            rc = YTA_ERR_HIP;
        }
    }
    if (rc) {
        n->stream = nullptr;
        release_buffers(n);
        delete n;
        return rc;
    }
    memcpy(n->h_cnt, e->h_cnt, sizeof(BtCounters) * S);
    release_buffers(e);
    e->CAP = n->CAP;
    e->MAXD = n->MAXD;
    e->allocs.swap(n->allocs);
    n->a.lds_bytes = e->a.lds_bytes;
    n->a.lds_bytes23 = e->a.lds_bytes23;
    n->a.lds_bytes_f = e->a.lds_bytes_f;
    n->a.lds_bytes_l = e->a.lds_bytes_l;
    n->a.lds_bytes_e = e->a.lds_bytes_e;
    e->a = n->a;
    e->out_own = n->out_own;
    e->d_warp = n->d_warp;
    e->d_warp_id = n->d_warp_id;
    e->h_off = n->h_off;
    e->h_cnt = n->h_cnt;
    e->d_det_off = n->d_det_off;
    e->d_active = n->d_active;
    n->h_off = nullptr;
    n->h_cnt = nullptr;
    n->stream = nullptr;
    delete n;
    if (e->variant == VAR_BYTETRACK && e->a.match_thresh <= 1.0) {
        // the next frame's stage-1 pool (k_finish builds it each frame) from the moved records
        hipLaunchKernelGGL(k_pool_build, dim3(e->S), dim3(PREP_T), 0, e->stream, e->a);
        YTA_HIP(hipGetLastError());
    }
    return YTA_OK;
}

int check_errors(yta_bytetrack *e) {
    for (int s = 0; s < e->S; ++s) {
        const int err = e->h_cnt[s].err;
        if (err) {
            set_error("stream %d: device error flags 0x%x (%s%s%s%s%s)", s, err,
                      err & ERR_EDGE_OVERFLOW ? "edge pool overflow " : "",
                      err & ERR_SOLVER ? "assignment solver failure " : "",
                      err & ERR_TRACK_CAPACITY ? "track capacity exceeded " : "",
                      err & ERR_DET_CAPACITY ? "too many detections " : "",
                      err & ERR_CLS_HIST ? "class histogram full " : "");
            return (err & (ERR_TRACK_CAPACITY | ERR_DET_CAPACITY | ERR_EDGE_OVERFLOW | ERR_CLS_HIST))
                       ? YTA_ERR_CAPACITY
                       : YTA_ERR_HIP;
        }
    }
    return YTA_OK;
}

int read_counters(yta_bytetrack *e) {
    YTA_HIP(hipMemcpyAsync(e->h_cnt, e->a.cnt, sizeof(BtCounters) * e->S, hipMemcpyDeviceToHost,
                           e->stream));
    YTA_HIP(host_wait(e->stream));
    return YTA_OK;
}


template <typename Init>
int create_engine(int device, int n_streams, int track_capacity, int max_dets,
                  yta_bytetrack **engine, Init init) {
    YTA_CHECK(n_streams > 0 && track_capacity > 0 && max_dets > 0, YTA_ERR_INVALID,
              "n_streams, track_capacity and max_dets must be positive");
    *engine = nullptr;
    int rc = select_device(device);
    if (rc) return rc;
    yta_bytetrack *e = new (std::nothrow) yta_bytetrack();
    YTA_CHECK(e, YTA_ERR_NOMEM, "out of host memory");
    e->device = device;
    e->S = n_streams;
    e->CAP = track_capacity;
    e->MAXD = max_dets;
    e->split23 = n_streams <= 64;
    if (const char *v = getenv("YTA_SPLIT23")) e->split23 = atoi(v) != 0;
    if (const char *v = getenv("YTA_GRAPHS")) e->graphs = atoi(v) != 0;
    init(e);
    hipError_t he;
    {   // A/B (round 6): YTA_ENGINE_PRIO=1 gives every other engine created a high-priority
        // compute stream (its dispatches go first when CU resources free up)
        static int n_created = 0;
        const char *v = getenv("YTA_ENGINE_PRIO");
        int lo = 0, hi = 0;
        if (v && atoi(v) && (n_created++ & 1) == 0 &&
            hipDeviceGetStreamPriorityRange(&lo, &hi) == hipSuccess)
            he = hipStreamCreateWithPriority(&e->stream, hipStreamNonBlocking, hi);
        else
            he = hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking);
    }
    if (he != hipSuccess) {
        set_error("hipStreamCreate: %s", hipGetErrorString(he));
        delete e;
        return YTA_ERR_HIP;
    }
    rc = bt_alloc(e);
    if (!rc) rc = set_lds_limits(BT_LDS_BYTES);
    if (!rc) rc = yta_bytetrack_reset(e);
    if (rc) {
        yta_bytetrack_destroy(e);
        return rc;
    }
    *engine = e;
    return YTA_OK;
}

// Host-buffer update shared by both trackers.  feats (BoT-SORT with ReID): per stream, the rows
// get_features returned for that stream's high detections (conf > track_high_thresh, in
// detection order), streams concatenated; staged here aligned with the detection rows.
static bool identity_warps(const double *w, int S) {
    if (!w) return true;
    for (int s = 0; s < S; ++s) {
        const double *h = w + 6LL * s;
        if (!(h[0] == 1.0 && h[1] == 0.0 && h[2] == 0.0 && h[3] == 0.0 && h[4] == 1.0 &&
              h[5] == 0.0))
            return false;
    }
    return true;
}

constexpr long long SMALL_PACK_BYTES = 1LL << 20;   // single-round-trip host update below this

// Device / pinned buffers for packed output rows (at least `rows`; grown to twice that, so a
// slowly growing output does not reallocate every frame) and the S + 1 offsets.
int ensure_pack(yta_bytetrack *e, long long rows) {
    if (rows <= e->pack_cap && e->d_pack_off) return YTA_OK;
    if (e->d_pack) (void)hipFree(e->d_pack);
    if (e->h_pack) (void)hipHostFree(e->h_pack);
    if (e->d_pack_off) (void)hipFree(e->d_pack_off);
    if (e->h_pack_off) (void)hipHostFree(e->h_pack_off);
    e->d_pack = e->h_pack = nullptr;
    e->d_pack_off = e->h_pack_off = nullptr;
    e->pack_cap = 0;
    const long long cap = std::max<long long>(2 * rows, 1024);
    const int S = e->S;
    YTA_HIP(hipMalloc((void **)&e->d_pack, sizeof(double) * 8 * cap));
    YTA_HIP(hipHostMalloc((void **)&e->h_pack, sizeof(double) * 8 * cap, hipHostMallocDefault));
    YTA_HIP(hipMalloc((void **)&e->d_pack_off, sizeof(int) * (S + 1)));
    YTA_HIP(hipHostMalloc((void **)&e->h_pack_off, sizeof(int) * (S + 1), hipHostMallocDefault));
    e->pack_cap = cap;
    return YTA_OK;
}

// float32 detection rows into a device buffer of `cap` floats (grown, contents dropped), through
// page-locked staging when the caller's buffer is pageable; enqueued on `st`.
int stage_f32(yta_bytetrack *e, const float *src, long long n, float **dbuf, float **hbuf,
              long long *cap, hipStream_t st) {
    if (n > *cap) {
        if (*dbuf) (void)hipFree(*dbuf);
        if (*hbuf) (void)hipHostFree(*hbuf);
        *dbuf = *hbuf = nullptr;
        *cap = 0;
        const long long c = std::max<long long>(n + n / 8, 6144);
        YTA_HIP(hipMalloc((void **)dbuf, sizeof(float) * c));
        YTA_HIP(hipHostMalloc((void **)hbuf, sizeof(float) * c, hipHostMallocDefault));
        *cap = c;
    }
    const size_t bytes = sizeof(float) * n;
    if (host_pinned(src, bytes)) {
        YTA_HIP(hipMemcpyAsync(*dbuf, src, bytes, hipMemcpyHostToDevice, st));
        return YTA_OK;
    }
    const size_t ch = stage_chunk(bytes);
    for (size_t o = 0; o < bytes; o += ch) {
        const size_t m = std::min(ch, bytes - o);
        par_copy(e, (char *)*hbuf + o, (const char *)src + o, m);
        YTA_HIP(hipMemcpyAsync((char *)*dbuf + o, (char *)*hbuf + o, m, hipMemcpyHostToDevice, st));
    }
    return YTA_OK;
}

int widen_f32(const float *src, double *dst, long long n, hipStream_t st) {
    const long long pairs = (n + 1) / 2;
    const unsigned blocks = (unsigned)std::min<long long>(4096, (pairs + 255) / 256);
    hipLaunchKernelGGL(k_widen_f32, dim3(std::max(1u, blocks)), dim3(256), 0, st, src, dst, n);
    YTA_HIP(hipGetLastError());
    return YTA_OK;
}

// Run `work` (the stream-ordered device work of one small host-buffer frame) through the engine's
// cached graph: replayed when the launch arguments and buffers are the ones it was captured with,
// else captured anew.  Kernel arguments are fixed at capture, so the comparison covers every
// pointer and scalar the launches read on the host side (BtArgs, the packing buffers, S / CAP).
// A capture failure turns graphs off for the engine and runs `work` directly.
template <typename Work>
int graph_run(yta_bytetrack *e, long long worst, Work work) {
    BtArgs cur = e->a;   // the arguments launch_pipeline will set
    cur.det_in = e->d_det_in;
    cur.det_off = e->d_det_off;
    cur.out = e->out_own;
    cur.out_counts = nullptr;
    cur.det_feat = e->d_feat_in;
    const void *ptrs[5] = {e->d_pack, e->h_pack, e->d_pack_off, e->h_cnt, e->out_own};
    const bool same = e->g_exec && e->g_cap == worst && memcmp(&cur, &e->g_args, sizeof cur) == 0 &&
                      memcmp(ptrs, e->g_ptrs, sizeof ptrs) == 0;
    if (!same) {
        if (e->g_exec) (void)hipGraphExecDestroy(e->g_exec);
        if (e->g_graph) (void)hipGraphDestroy(e->g_graph);
        e->g_exec = nullptr;
        e->g_graph = nullptr;
        if (hipStreamBeginCapture(e->stream, hipStreamCaptureModeThreadLocal) != hipSuccess) {
            (void)hipGetLastError();
            e->graphs = false;
            return work();
        }
        const int r = work();
        hipGraph_t g = nullptr;
        const hipError_t he = hipStreamEndCapture(e->stream, &g);
        if (r || he != hipSuccess || !g ||
            hipGraphInstantiate(&e->g_exec, g, nullptr, nullptr, 0) != hipSuccess) {
            if (g) (void)hipGraphDestroy(g);
            e->g_exec = nullptr;
            (void)hipGetLastError();
            e->graphs = false;
            return r ? r : work();   // not captured: run it as plain launches
        }
        e->g_graph = g;
        e->g_args = e->a;
        memcpy(e->g_ptrs, ptrs, sizeof ptrs);
        e->g_cap = worst;
        ++e->g_captures;
    }
    ++e->g_replays;
    YTA_HIP(hipGraphLaunch(e->g_exec, e->stream));
    return YTA_OK;
}

int update_host(yta_bytetrack *e, const double *dets, const int *det_offsets, const float *feats,
                long long *next_id, double *out, int out_capacity, int *out_offsets,
                const double *warps = nullptr, const int *active = nullptr,
                const float *dets32 = nullptr) {
    YTA_CHECK(e && det_offsets && out_offsets, YTA_ERR_INVALID, "null argument");
    YTA_CHECK(!dets32 || (e->variant == VAR_BYTETRACK && !dets), YTA_ERR_INVALID,
              "float32 detections: ByteTrack engines, instead of the float64 rows");
    YTA_CHECK(e->pipe_count == 0, YTA_ERR_INVALID, "pipelined frames in flight: collect them first");
    YTA_HIP(hipSetDevice(e->device));
    const int S = e->S;
    YTA_CHECK(det_offsets[0] == 0, YTA_ERR_INVALID, "det_offsets[0] must be 0");
    int need_d = e->MAXD, need_c = e->CAP;
    for (int s = 0; s < S; ++s) {
        const int m = det_offsets[s + 1] - det_offsets[s];
        YTA_CHECK(m >= 0, YTA_ERR_INVALID, "det_offsets must be non-decreasing");
        need_d = std::max(need_d, m);
        need_c = std::max(need_c, e->h_cnt[s].n_tracked + e->h_cnt[s].n_lost + m);
    }
    // every output row is a track matched to or born from one of this frame's detections, so
    // det_offsets[S] rows always suffice; checked before anything moves (the frame is not consumed)
    YTA_CHECK(out_capacity >= det_offsets[S], YTA_ERR_CAPACITY,
              "out holds %d rows, the call needs det_offsets[S] = %d", out_capacity, det_offsets[S]);
    if (need_d > e->MAXD || need_c > e->CAP) {   // grow geometrically, keeping all state
        const int rc = reserve(e, need_c > e->CAP ? std::max(need_c, 2 * e->CAP) : e->CAP,
                               need_d > e->MAXD ? std::max(need_d, 2 * e->MAXD) : e->MAXD);
        if (rc) return rc;
    }
    if (e->variant == VAR_BOTSORT) {   // this frame's camera warps (staged after any reserve)
        e->a.warp = e->d_warp_id;
        if (warps && !identity_warps(warps, S)) {
            for (long long k = 0; k < 6LL * S; ++k)
                YTA_CHECK(std::isfinite(warps[k]), YTA_ERR_INVALID, "non-finite warp entry");
            YTA_HIP(hipMemcpyAsync(e->d_warp, warps, sizeof(double) * 6 * S,
                                   hipMemcpyHostToDevice, e->stream));
            e->a.warp = e->d_warp;
        }
    }
    const long long total = det_offsets[S];
    YTA_CHECK(total == 0 || dets || dets32, YTA_ERR_INVALID, "null dets");
    if (total > e->d_det_cap) {
        if (e->d_det_in) (void)hipFree(e->d_det_in);
        if (e->h_dets) (void)hipHostFree(e->h_dets);
        e->d_det_in = nullptr;
        e->h_dets = nullptr;
        e->d_det_cap = 0;
        const long long cap = std::max<long long>(2 * total, 1024);
        YTA_HIP(hipMalloc((void **)&e->d_det_in, sizeof(double) * 6 * cap));
        YTA_HIP(hipHostMalloc((void **)&e->h_dets, sizeof(double) * 6 * cap, hipHostMallocDefault));
        e->d_det_cap = cap;
    }
    if (total && dets32) {   // float32 rows: half the bytes over the link, widened on the device
        int src = stage_f32(e, dets32, 6 * total, &e->d_det32, &e->h_det32, &e->det32_cap,
                            e->stream);
        if (!src) src = widen_f32(e->d_det32, e->d_det_in, 6 * total, e->stream);
        if (src) return src;
    } else if (total && host_pinned(dets, sizeof(double) * 6 * total)) {   // straight from the caller
        YTA_HIP(hipMemcpyAsync(e->d_det_in, dets, sizeof(double) * 6 * total,
                               hipMemcpyHostToDevice, e->stream));
    } else if (total) {   // chunk k's DMA overlaps chunk k+1's host copy
        const size_t bytes = sizeof(double) * 6 * total, ch = stage_chunk(bytes);
        for (size_t o = 0; o < bytes; o += ch) {
            const size_t n = std::min(ch, bytes - o);
            par_copy(e, (char *)e->h_dets + o, (const char *)dets + o, n);
            YTA_HIP(hipMemcpyAsync((char *)e->d_det_in + o, (char *)e->h_dets + o, n,
                                   hipMemcpyHostToDevice, e->stream));
        }
    }
    const int D = e->a.D;
    if (D > 0 && total) {
        if (total > e->feat_cap) {
            if (e->d_feat_in) (void)hipFree(e->d_feat_in);
            if (e->h_feat) (void)hipHostFree(e->h_feat);
            e->d_feat_in = nullptr;
            e->h_feat = nullptr;
            e->feat_cap = 0;
            const long long cap = std::max<long long>(2 * total, 1024);
            YTA_HIP(hipMalloc((void **)&e->d_feat_in, sizeof(float) * D * cap));
            YTA_HIP(hipHostMalloc((void **)&e->h_feat, sizeof(float) * D * cap,
                                  hipHostMallocDefault));
            e->feat_cap = cap;
        }
        long long k = 0;   // next high row of feats
        for (long long r = 0; r < total; ++r)
            if (dets[r * 6 + 4] > e->a.track_thresh) {
                YTA_CHECK(feats, YTA_ERR_INVALID, "null feats with high detections");
                memcpy(e->h_feat + r * D, feats + k * D, sizeof(float) * D);
                ++k;
            }
        YTA_HIP(hipMemcpyAsync(e->d_feat_in, e->h_feat, sizeof(float) * D * total,
                               hipMemcpyHostToDevice, e->stream));
    }
    memcpy(e->h_off, det_offsets, sizeof(int) * (S + 1));
    YTA_HIP(hipMemcpyAsync(e->d_det_off, e->h_off, sizeof(int) * (S + 1), hipMemcpyHostToDevice,
                           e->stream));
    if (next_id) {
        for (int s = 0; s < S; ++s) e->h_cnt[s].next_id = next_id[s];
        YTA_HIP(hipMemcpy2DAsync(&e->a.cnt[0].next_id, sizeof(BtCounters), &e->h_cnt[0].next_id,
                                 sizeof(BtCounters), sizeof(long long), S, hipMemcpyHostToDevice,
                                 e->stream));
    }
    if (active) {   // stream subset: the others' kernels return at once (BtArgs::active)
        if (!e->h_active) {
            YTA_HIP(hipHostMalloc((void **)&e->h_active, sizeof(int) * S, hipHostMallocDefault));
        }
        memcpy(e->h_active, active, sizeof(int) * S);
        YTA_HIP(hipMemcpyAsync(e->d_active, e->h_active, sizeof(int) * S, hipMemcpyHostToDevice,
                               e->stream));
        e->a.active = e->d_active;
    }
    // Small engines (every stream's worst-case rows <= 1 MiB, e.g. one camera stream): rows packed
    // at device-computed offsets and copied back with the counters, one round trip per frame
    const long long worst = (long long)S * e->CAP;
    const bool small = worst * 64 <= SMALL_PACK_BYTES;
    int rc = YTA_OK;
    if (small) {
        rc = ensure_pack(e, worst);
        if (rc) return rc;
    }
    // one stream: its rows already start at row 0 of out_own, so the packing launches (two
    // dependent kernels on a one-camera frame's chain, ~9 us) are skipped, and k_finish mirrors
    // the counters right after the rows, so one copy returns both
    const bool one = small && S == 1 && !active;
    if (one) {
        rc = ensure_pack(e, worst + 2);
        if (rc) return rc;
    }
    e->a.cnt_mirror = one ? reinterpret_cast<BtCounters *>(e->out_own + worst * 8) : nullptr;
    auto device_work = [&]() -> int {   // the frame's launches (+ packing and copies back)
        int r = launch_pipeline(e, e->d_det_in, e->d_det_off, e->out_own, nullptr, e->d_feat_in);
        if (r || !small) return r;
        if (one) {
            YTA_HIP(hipMemcpyAsync(e->h_pack, e->out_own, sizeof(double) * 8 * (worst + 2),
                                   hipMemcpyDeviceToHost, e->stream));
            return YTA_OK;
        }
        const double *src = e->out_own;
        if (S > 1) {
            hipLaunchKernelGGL(k_out_offsets, dim3(1), dim3(64), 0, e->stream, e->a.cnt, S,
                               e->CAP, e->d_pack_off);
            hipLaunchKernelGGL(k_pack_out, dim3(S), dim3(256), 0, e->stream, e->out_own,
                               (long long)e->CAP, e->d_pack_off, e->d_pack, e->pack_cap);
            YTA_HIP(hipGetLastError());
            src = e->d_pack;
        }
        YTA_HIP(hipMemcpyAsync(e->h_cnt, e->a.cnt, sizeof(BtCounters) * S, hipMemcpyDeviceToHost,
                               e->stream));
        YTA_HIP(hipMemcpyAsync(e->h_pack, src, sizeof(double) * 8 * worst,
                               hipMemcpyDeviceToHost, e->stream));
        return YTA_OK;
    };
    if (small && e->graphs && !e->prof && !active) {
        rc = graph_run(e, worst, device_work);
    } else {
        rc = device_work();
    }
    e->a.active = nullptr;
    e->a.cnt_mirror = nullptr;
    if (rc) return rc;
    if (small) {
        YTA_HIP(host_wait(e->stream));
        if (one) memcpy(e->h_cnt, e->h_pack + worst * 8, sizeof(BtCounters));
        if (next_id)   // the device counters have advanced: hand them back even on an error below
            for (int q = 0; q < S; ++q) next_id[q] = e->h_cnt[q].next_id;
        rc = check_errors(e);
        if (rc) return rc;
        long long rows = 0;
        out_offsets[0] = 0;
        for (int q = 0; q < S; ++q) {
            rows += e->h_cnt[q].n_out;
            out_offsets[q + 1] = (int)rows;
        }
        YTA_CHECK(rows <= out_capacity, YTA_ERR_CAPACITY, "output needs %lld rows > capacity %d",
                  rows, out_capacity);
        YTA_CHECK(rows == 0 || out, YTA_ERR_INVALID, "null out");
        if (rows > 0) memcpy(out, e->h_pack, sizeof(double) * 8 * rows);
        return YTA_OK;
    }
    rc = read_counters(e);
    if (rc) return rc;
    if (next_id)   // the device counters have advanced: hand them back even on an error below
        for (int s = 0; s < S; ++s) next_id[s] = e->h_cnt[s].next_id;
    rc = check_errors(e);
    if (rc) return rc;
    long long rows = 0;
    out_offsets[0] = 0;
    for (int s = 0; s < S; ++s) {
        rows += e->h_cnt[s].n_out;
        out_offsets[s + 1] = (int)rows;
    }
    YTA_CHECK(rows <= out_capacity, YTA_ERR_CAPACITY, "output needs %lld rows > capacity %d", rows,
              out_capacity);
    YTA_CHECK(rows == 0 || out, YTA_ERR_INVALID, "null out");
    if (rows > 0) {   // pack on the device, one copy back through pinned staging
        rc = ensure_pack(e, rows);
        if (rc) return rc;
        memcpy(e->h_pack_off, out_offsets, sizeof(int) * (S + 1));
        YTA_HIP(hipMemcpyAsync(e->d_pack_off, e->h_pack_off, sizeof(int) * (S + 1),
                               hipMemcpyHostToDevice, e->stream));
        hipLaunchKernelGGL(k_pack_out, dim3(S), dim3(256), 0, e->stream, e->out_own,
                           (long long)e->CAP, e->d_pack_off, e->d_pack, e->pack_cap);
        YTA_HIP(hipGetLastError());
        const size_t bytes = sizeof(double) * 8 * rows, ch = stage_chunk(bytes);
        if (host_pinned(out, bytes)) {   // straight into the caller's buffer
            YTA_HIP(hipMemcpyAsync(out, e->d_pack, bytes, hipMemcpyDeviceToHost, e->stream));
            YTA_HIP(host_wait(e->stream));
            return YTA_OK;
        }
        // chunked copy back: the host copies chunk k out while chunk k+1 is in flight
        hipEvent_t ev[STAGE_CHUNKS];
        int nev = 0;
        hipError_t err = hipSuccess;
        for (size_t o = 0; o < bytes && err == hipSuccess; o += ch) {
            err = hipEventCreateWithFlags(&ev[nev], hipEventDisableTiming | hipEventBlockingSync);
            if (err != hipSuccess) break;
            ++nev;
            err = hipMemcpyAsync((char *)e->h_pack + o, (char *)e->d_pack + o,
                                 std::min(ch, bytes - o), hipMemcpyDeviceToHost, e->stream);
            if (err == hipSuccess) err = hipEventRecord(ev[nev - 1], e->stream);
        }
        size_t o = 0;
        for (int k = 0; k < nev && err == hipSuccess; ++k, o += ch) {
            err = hipEventSynchronize(ev[k]);
            if (err == hipSuccess)
                par_copy(e, (char *)out + o, (const char *)e->h_pack + o, std::min(ch, bytes - o));
        }
        for (int k = 0; k < nev; ++k) (void)hipEventDestroy(ev[k]);
        YTA_HIP(err);
    }
    YTA_HIP(host_wait(e->stream));
    return YTA_OK;
}

// Host-buffer update of a subset of the streams: n ascending stream ids; dets / det_offsets (n+1)
// / feats / warps (n x 6) / next_id (n) / out_offsets (n+1) cover those streams only, in id
// order.  Expanded to the engine's S streams (zero detections, identity warp and the engine's
// own counter for the others, which the stream mask leaves untouched), run, and compacted.
int update_host_subset(yta_bytetrack *e, int n, const int *ids, const double *dets,
                       const int *det_offsets, const float *feats, long long *next_id,
                       double *out, int out_capacity, int *out_offsets, const double *warps) {
    YTA_CHECK(e && ids && det_offsets && out_offsets, YTA_ERR_INVALID, "null argument");
    const int S = e->S;
    YTA_CHECK(n >= 1 && n <= S, YTA_ERR_INVALID, "n_streams %d outside 1..%d", n, S);
    for (int k = 0; k < n; ++k)
        YTA_CHECK(ids[k] >= 0 && ids[k] < S && (k == 0 || ids[k] > ids[k - 1]), YTA_ERR_INVALID,
                  "stream_ids must be ascending and within 0..%d", S - 1);
    YTA_CHECK(det_offsets[0] == 0, YTA_ERR_INVALID, "det_offsets[0] must be 0");
    std::vector<int> active(S, 0), off(S + 1, 0), full_oo(S + 1, 0);
    std::vector<long long> nid(S);
    std::vector<double> w;
    if (next_id) {   // the skipped streams keep their device counters: read them first (a device
                     // update since the last host call may have advanced them)
        YTA_HIP(hipSetDevice(e->device));
        const int rc = read_counters(e);
        if (rc) return rc;
    }
    for (int s = 0; s < S; ++s) nid[s] = e->h_cnt[s].next_id;
    if (warps && e->variant == VAR_BOTSORT) {
        w.assign((size_t)6 * S, 0.0);
        for (int s = 0; s < S; ++s) w[6 * s] = w[6 * s + 4] = 1.0;
    }
    for (int k = 0; k < n; ++k) {
        active[ids[k]] = 1;
        if (next_id) nid[ids[k]] = next_id[k];
        if (!w.empty()) std::copy(warps + 6LL * k, warps + 6LL * k + 6, w.begin() + 6LL * ids[k]);
    }
    for (int s = 0, k = 0; s < S; ++s) {
        int m = 0;
        if (active[s]) {
            m = det_offsets[k + 1] - det_offsets[k];
            YTA_CHECK(m >= 0, YTA_ERR_INVALID, "det_offsets must be non-decreasing");
            ++k;
        }
        off[s + 1] = off[s] + m;
    }
    const int rc = update_host(e, dets, off.data(), feats, next_id ? nid.data() : nullptr, out,
                               out_capacity, full_oo.data(), w.empty() ? nullptr : w.data(),
                               active.data());
    if (e->variant == VAR_BOTSORT) e->a.warp = e->d_warp_id;
    // the device counters have advanced for the active streams: hand them back even on an error
    if (next_id)
        for (int k = 0; k < n; ++k) next_id[k] = nid[ids[k]];
    if (rc) return rc;
    out_offsets[0] = 0;
    for (int k = 0; k < n; ++k)   // skipped streams have 0 rows: the packing is the subset's
        out_offsets[k + 1] = out_offsets[k] + (full_oo[ids[k] + 1] - full_oo[ids[k]]);
    return YTA_OK;
}

// ---- pipelined host-buffer update --------------------------------------------------------------
// Frame f's detections go host -> device on s_in while frame f-1's kernels run on the compute
// stream and frame f-2's rows come back on s_out (PIPE_DEPTH frames in flight) (both PCIe directions and the kernels at once).
// The compute stream snapshots every frame's rows (k_pack_out into the slot) and counters before
// the next frame's kernels can touch them, so the copy-out of frame f never races frame f+1.
void pipe_free(yta_bytetrack *e) {
    for (auto &p : e->pipe) {
        for (void *d : {(void *)p.d_in, (void *)p.d_off, (void *)p.d_pack, (void *)p.d_pack_off,
                        (void *)p.d_cnt, (void *)p.d_in32})
            if (d) (void)hipFree(d);
        for (void *h : {(void *)p.h_in, (void *)p.h_off, (void *)p.h_pack, (void *)p.h_pack_off,
                        (void *)p.h_cnt, (void *)p.h_nid, (void *)p.h_in32})
            if (h) (void)hipHostFree(h);
        for (hipEvent_t ev : {p.in_done, p.kern_done, p.out_done, p.t_ev[0], p.t_ev[1], p.t_ev[2],
                              p.t_ev[3], p.t_ev[4], p.t_ev[5]})
            if (ev) (void)hipEventDestroy(ev);
        if (p.own_s_in && p.s_in) (void)hipStreamDestroy(p.s_in);
        p = yta_bytetrack::PipeSlot{};
    }
    for (auto &p : e->pipe) p = yta_bytetrack::PipeSlot{};
    for (hipStream_t st : {e->s_in, e->s_out})
        if (st) (void)hipStreamDestroy(st);
    e->s_in = e->s_out = nullptr;
    e->pipe_count = 0;
    e->pipe_head = 0;
}

int pipe_slot_ready(yta_bytetrack *e, yta_bytetrack::PipeSlot &p, long long dets) {
    const int S = e->S;
    if (!p.s_in && pipe_slot_streams()) {
        YTA_HIP(pipe_stream_create(&p.s_in, 0));
        p.own_s_in = true;
    }
    if (!e->s_in) {
        YTA_HIP(pipe_stream_create(&e->s_in, 0));
        YTA_HIP(pipe_stream_create(&e->s_out, 1));
    }
    if (!p.s_in) p.s_in = e->s_in;
    if (!p.in_done) {
        for (hipEvent_t *ev : {&p.in_done, &p.kern_done, &p.out_done})
            YTA_HIP(hipEventCreateWithFlags(ev, hipEventDisableTiming));
        if (pipe_timing())
            for (hipEvent_t &ev : p.t_ev) YTA_HIP(hipEventCreateWithFlags(&ev, hipEventDefault));
        YTA_HIP(hipMalloc((void **)&p.d_off, sizeof(int) * (S + 1)));
        YTA_HIP(hipHostMalloc((void **)&p.h_off, sizeof(int) * (S + 1),
                              hipHostMallocMapped | hipHostMallocCoherent));
        YTA_HIP(hipHostGetDevicePointer((void **)&p.m_off, p.h_off, 0));
        YTA_HIP(hipMalloc((void **)&p.d_pack_off, sizeof(int) * (S + 1)));
        // counters and row offsets: written by the compute stream's kernels straight into mapped,
        // coherent host memory (k_out_offsets_scan, k_cnt_to_host)
        const unsigned mf = hipHostMallocMapped | hipHostMallocCoherent;
        YTA_HIP(hipHostMalloc((void **)&p.h_pack_off, sizeof(int) * (S + 1), mf));
        YTA_HIP(hipHostMalloc((void **)&p.h_cnt, sizeof(BtCounters) * S, mf));
        YTA_HIP(hipHostGetDevicePointer((void **)&p.m_pack_off, p.h_pack_off, 0));
        YTA_HIP(hipHostGetDevicePointer((void **)&p.m_cnt, p.h_cnt, 0));
        YTA_HIP(hipHostMalloc((void **)&p.h_nid, sizeof(long long) * S, hipHostMallocDefault));
    }
    if (dets > p.in_cap) {   // detections and packed rows: both bounded by the frame's dets
        for (void *d : {(void *)p.d_in, (void *)p.d_pack})
            if (d) (void)hipFree(d);
        for (void *h : {(void *)p.h_in, (void *)p.h_pack})
            if (h) (void)hipHostFree(h);
        p.d_in = p.h_in = p.d_pack = p.h_pack = nullptr;
        p.in_cap = p.pack_cap = 0;
        const long long cap = std::max<long long>(dets + dets / 8, 1024);
        YTA_HIP(hipMalloc((void **)&p.d_in, sizeof(double) * 6 * cap));
        YTA_HIP(hipHostMalloc((void **)&p.h_in, sizeof(double) * 6 * cap, hipHostMallocDefault));
        YTA_HIP(hipMalloc((void **)&p.d_pack, sizeof(double) * 8 * cap));
        YTA_HIP(hipHostMalloc((void **)&p.h_pack, sizeof(double) * 8 * cap,
                              hipHostMallocMapped | hipHostMallocCoherent));
        YTA_HIP(hipHostGetDevicePointer((void **)&p.m_pack, p.h_pack, 0));
        p.in_cap = p.pack_cap = cap;
    }
    return YTA_OK;
}

// The frame's copy-in (s_in): offsets and detections into the slot.
int pipe_enqueue_in(yta_bytetrack *e, yta_bytetrack::PipeSlot &p, const double *dets,
                    const int *det_offsets, long long total, const float *dets32) {
    const int S = e->S;
    int rc = YTA_OK;
    // this slot's last frame was collected (its events completed): its buffers are free
    if (p.t_ev[0]) YTA_HIP(hipEventRecord(p.t_ev[0], p.s_in));
    memcpy(p.h_off, det_offsets, sizeof(int) * (S + 1));
    auto ts = std::chrono::steady_clock::now();
    if (!pipe_off_kernel())   // else the compute stream reads them from the mapped h_off
        YTA_HIP(hipMemcpyAsync(p.d_off, p.h_off, sizeof(int) * (S + 1), hipMemcpyHostToDevice,
                               p.s_in));
    e->pstat[PS_SMALL_H2D_MS] += std::chrono::duration<double, std::milli>(
                                     std::chrono::steady_clock::now() - ts)
                                     .count();
    p.direct_in = false;
    p.in_bytes = 0;
    if (total && dets32) {   // float32 rows: half the bytes over the link, widened on the device
        p.in_bytes = (long long)sizeof(float) * 6 * total;
        p.direct_in = host_pinned(dets32, (size_t)p.in_bytes);
        rc = stage_f32(e, dets32, 6 * total, &p.d_in32, &p.h_in32, &p.in32_cap, p.s_in);
        if (rc) return rc;
    } else if (total) {
        const size_t bytes = sizeof(double) * 6 * total;
        p.in_bytes = (long long)bytes;
        ts = std::chrono::steady_clock::now();
        const bool pinned_in = host_pinned(dets, bytes);
        e->pstat[PS_PINNED_CHECK_MS] += std::chrono::duration<double, std::milli>(
                                            std::chrono::steady_clock::now() - ts)
                                            .count();
        if (pinned_in) {   // straight from the caller (kept until collected)
            p.direct_in = true;
            const auto t0 = std::chrono::steady_clock::now();
            YTA_HIP(copy_pieces(p.d_in, dets, bytes, hipMemcpyHostToDevice, p.s_in));
            e->pstat[PS_H2D_CALL_MS] += std::chrono::duration<double, std::milli>(
                                            std::chrono::steady_clock::now() - t0)
                                            .count();
        } else {   // staged: chunk k's DMA overlaps chunk k+1's host copy
            const auto t0 = std::chrono::steady_clock::now();
            const size_t ch = stage_chunk(bytes);
            for (size_t o = 0; o < bytes; o += ch) {
                const size_t n = std::min(ch, bytes - o);
                par_copy(e, (char *)p.h_in + o, (const char *)dets + o, n);
                YTA_HIP(hipMemcpyAsync((char *)p.d_in + o, (char *)p.h_in + o, n,
                                       hipMemcpyHostToDevice, p.s_in));
            }
            e->pstat[PS_STAGE_IN_MS] += std::chrono::duration<double, std::milli>(
                                            std::chrono::steady_clock::now() - t0)
                                            .count();
        }
    }
    e->pstat[p.direct_in ? PS_IN_DIRECT : PS_IN_STAGED] += (double)p.in_bytes;
    if (p.t_ev[1]) YTA_HIP(hipEventRecord(p.t_ev[1], p.s_in));
    YTA_HIP(hipEventRecord(p.in_done, p.s_in));
    return YTA_OK;
}

// The frame's kernels + row / counter snapshot (compute stream) and copy-out (s_out).
int pipe_enqueue_run(yta_bytetrack *e, yta_bytetrack::PipeSlot &p, const long long *next_id,
                     double *out, long long total, const float *dets32) {
    const int S = e->S;
    int rc = YTA_OK;
    // compute stream: the frame, then its rows and counters snapshotted into the slot
    YTA_HIP(hipStreamWaitEvent(e->stream, p.in_done, 0));
    if (p.t_ev[2]) YTA_HIP(hipEventRecord(p.t_ev[2], e->stream));
    if (pipe_off_kernel()) {
        hipLaunchKernelGGL(k_copy_ints, dim3(1), dim3(1024), 0, e->stream, p.m_off, p.d_off, S + 1);
        YTA_HIP(hipGetLastError());
    }
    if (next_id) {
        memcpy(p.h_nid, next_id, sizeof(long long) * S);
        YTA_HIP(hipMemcpy2DAsync(&e->a.cnt[0].next_id, sizeof(BtCounters), p.h_nid,
                                 sizeof(long long), sizeof(long long), S, hipMemcpyHostToDevice,
                                 e->stream));
    }
    if (total && dets32) {
        rc = widen_f32(p.d_in32, p.d_in, 6 * total, e->stream);
        if (rc) return rc;
    }
    const auto tl = std::chrono::steady_clock::now();
    rc = launch_pipeline(e, p.d_in, p.d_off, e->out_own, nullptr);
    if (rc) return rc;
    e->pstat[PS_LAUNCH_MS] += std::chrono::duration<double, std::milli>(
                                  std::chrono::steady_clock::now() - tl)
                                  .count();
    hipLaunchKernelGGL(k_out_offsets_scan, dim3(1), dim3(OFFS_T), 0, e->stream, e->a.cnt, S,
                       e->CAP, p.d_pack_off, p.m_pack_off);
    hipLaunchKernelGGL(k_pack_out, dim3(S), dim3(256), 0, e->stream, e->out_own, (long long)e->CAP,
                       p.d_pack_off, p.d_pack, p.pack_cap);
    hipLaunchKernelGGL(k_cnt_to_host, dim3((S * 8 + 255) / 256), dim3(256), 0, e->stream,
                       e->a.cnt, S, (int4 *)p.m_cnt);
    YTA_HIP(hipGetLastError());
    if (p.t_ev[3]) YTA_HIP(hipEventRecord(p.t_ev[3], e->stream));
    YTA_HIP(hipEventRecord(p.kern_done, e->stream));
    // copy-out stream: counters, offsets and at most det_offsets[S] rows (every output row is a
    // track matched to or born from one of the frame's detections)
    YTA_HIP(hipStreamWaitEvent(e->s_out, p.kern_done, 0));
    if (p.t_ev[4]) YTA_HIP(hipEventRecord(p.t_ev[4], e->s_out));
    p.user_out = out;
    p.rows_bound = total;
    auto ts = std::chrono::steady_clock::now();
    void *out_dev = nullptr;
    p.direct_out = total > 0 && host_pinned(out, sizeof(double) * 8 * total, &out_dev);
    e->pstat[PS_PINNED_CHECK_MS] += std::chrono::duration<double, std::milli>(
                                        std::chrono::steady_clock::now() - ts)
                                        .count();
    if (total) {
        const auto t0 = std::chrono::steady_clock::now();
        void *dst_dev = p.direct_out ? out_dev : (void *)p.m_pack;
        if (pipe_kernel_d2h() && dst_dev) {   // the rows stored by a kernel (k_rows_to_host)
            hipLaunchKernelGGL(k_rows_to_host, dim3(pipe_d2h_blocks()), dim3(256), 0, e->s_out,
                               p.d_pack, p.d_pack_off, S, total, (int4 *)dst_dev);
            YTA_HIP(hipGetLastError());
        } else {
            YTA_HIP(copy_pieces(p.direct_out ? out : p.h_pack, p.d_pack,
                                sizeof(double) * 8 * total, hipMemcpyDeviceToHost, e->s_out));
        }
        e->pstat[PS_D2H_CALL_MS] += std::chrono::duration<double, std::milli>(
                                        std::chrono::steady_clock::now() - t0)
                                        .count();
    }
    if (p.t_ev[5]) YTA_HIP(hipEventRecord(p.t_ev[5], e->s_out));
    YTA_HIP(hipEventRecord(p.out_done, e->s_out));
    return YTA_OK;
}

// Track capacity for the next frame of the pipeline.  Each stream's tracked + lost lists after it
// are at most the live tracks after some earlier frame plus every detection from that frame on
// (every tracked track is matched to or born from one of its frame's detections; lost tracks were
// tracked before).  The counters used: the newest frame in flight whose kernels have run (the
// compute stream stored them into its slot's mapped h_cnt, k_cnt_to_host), else the last
// collected ones; if that bound does not fit, wait for the newest frame's kernels (not its
// copies) and use its exact counters; only a frame that still does not fit drains the pipeline
// and grows the engine.  (Round 4 bounded from the last COLLECTED frame only: at the bench's
// 3N capacity that never fit with two frames in flight, so every submit drained the compute
// stream and read the counters synchronously - the pipeline ran one frame at a time.)
int pipe_capacity(yta_bytetrack *e, const int *det_offsets) {
    const int S = e->S;
    int need_d = e->MAXD;
    for (int s = 0; s < S; ++s) {
        const int m = det_offsets[s + 1] - det_offsets[s];
        YTA_CHECK(m >= 0, YTA_ERR_INVALID, "det_offsets must be non-decreasing");
        need_d = std::max(need_d, m);
    }
    auto slot = [&](int k) -> yta_bytetrack::PipeSlot & {
        return e->pipe[(e->pipe_head + k) % PIPE_DEPTH];
    };
    // k0: the in-flight frame (in flight order) whose counters are used, -1 for e->h_cnt
    auto fits = [&](int k0) {
        const BtCounters *c = k0 < 0 ? e->h_cnt : slot(k0).h_cnt;
        for (int s = 0; s < S; ++s) {
            long long bound = (long long)c[s].n_tracked + c[s].n_lost +
                              (det_offsets[s + 1] - det_offsets[s]);
            for (int k = k0 + 1; k < e->pipe_count; ++k)
                bound += slot(k).h_off[s + 1] - slot(k).h_off[s];
            if (bound > e->CAP) return false;
        }
        return true;
    };
    if (need_d <= e->MAXD) {
        int k0 = -1;
        for (int k = e->pipe_count - 1; k >= 0; --k) {
            const hipError_t q = hipEventQuery(slot(k).kern_done);
            if (q == hipSuccess) {
                k0 = k;
                break;
            }
            (void)hipGetLastError();   // hipErrorNotReady
        }
        if (fits(k0)) return YTA_OK;
        if (k0 != e->pipe_count - 1) {
            YTA_HIP(hipEventSynchronize(slot(e->pipe_count - 1).kern_done));
            ++e->pstat[PS_CAP_WAITS];
            if (fits(e->pipe_count - 1)) return YTA_OK;
        }
    }
    // drain the kernels in flight, then the exact need
    ++e->pstat[PS_CAP_DRAINS];
    YTA_HIP(host_wait(e->stream));   // every frame in flight has run: a.cnt is current
    std::vector<BtCounters> c(S);
    YTA_HIP(hipMemcpy(c.data(), e->a.cnt, sizeof(BtCounters) * S, hipMemcpyDeviceToHost));
    int need_c = e->CAP;
    for (int s = 0; s < S; ++s)
        need_c = std::max(need_c, c[s].n_tracked + c[s].n_lost +
                                      (det_offsets[s + 1] - det_offsets[s]));
    if (need_d > e->MAXD || need_c > e->CAP)
        return reserve(e, need_c > e->CAP ? std::max(need_c, 2 * e->CAP) : e->CAP,
                       need_d > e->MAXD ? std::max(need_d, 2 * e->MAXD) : e->MAXD);
    return YTA_OK;
}

int pipe_submit(yta_bytetrack *e, const double *dets, const int *det_offsets,
                const long long *next_id, double *out, long long out_capacity,
                const float *dets32 = nullptr) {
    YTA_CHECK(e && det_offsets, YTA_ERR_INVALID, "null argument");
    YTA_CHECK(e->variant == VAR_BYTETRACK, YTA_ERR_INVALID, "pipelined updates: ByteTrack engines");
    YTA_HIP(hipSetDevice(e->device));
    YTA_CHECK(e->pipe_count < PIPE_DEPTH, YTA_ERR_INVALID, "%d frames in flight: collect one first",
              PIPE_DEPTH);
    const int S = e->S;
    YTA_CHECK(det_offsets[0] == 0, YTA_ERR_INVALID, "det_offsets[0] must be 0");
    const long long total = det_offsets[S];
    YTA_CHECK(total == 0 || dets || dets32, YTA_ERR_INVALID, "null dets");
    YTA_CHECK(out_capacity >= total && (total == 0 || out), YTA_ERR_CAPACITY,
              "out holds %lld rows, the frame needs det_offsets[S] = %lld", out_capacity, total);
    for (int s = 0; s < S; ++s)
        YTA_CHECK(det_offsets[s + 1] >= det_offsets[s], YTA_ERR_INVALID,
                  "det_offsets must be non-decreasing");
    auto &p = e->pipe[(e->pipe_head + e->pipe_count) % PIPE_DEPTH];
    if (p.dirty) {   // a failed submit may have left copies from this slot's buffers queued
        YTA_HIP(hipStreamSynchronize(p.s_in ? p.s_in : e->s_in));
        YTA_HIP(hipStreamSynchronize(e->stream));
        YTA_HIP(hipStreamSynchronize(e->s_out));
        p.dirty = false;
    }
    int rc = pipe_slot_ready(e, p, total);
    if (rc) return rc;
    const auto t0 = std::chrono::steady_clock::now();
    // the copy-in first (it needs only the slot), so it overlaps any wait for capacity below
    rc = pipe_enqueue_in(e, p, dets, det_offsets, total, dets32);
    if (!rc) rc = pipe_capacity(e, det_offsets);
    if (!rc) rc = pipe_enqueue_run(e, p, next_id, out, total, dets32);
    if (rc) {   // copies from the slot's pinned staging may be in flight: the next use waits
        p.dirty = true;
        return rc;
    }
    e->pstat[PS_SUBMIT_MS] +=
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    ++e->pipe_count;
    return YTA_OK;
}

int pipe_collect(yta_bytetrack *e, long long *next_id, int *out_offsets) {
    YTA_CHECK(e && out_offsets, YTA_ERR_INVALID, "null argument");
    YTA_CHECK(e->pipe_count > 0, YTA_ERR_INVALID, "no frame in flight");
    YTA_HIP(hipSetDevice(e->device));
    auto &p = e->pipe[e->pipe_head];
    e->pipe_head = (e->pipe_head + 1) % PIPE_DEPTH;
    --e->pipe_count;
    const auto t0 = std::chrono::steady_clock::now();
    YTA_HIP(hipEventSynchronize(p.out_done));
    const auto t1 = std::chrono::steady_clock::now();
    e->pstat[PS_WAIT_MS] += std::chrono::duration<double, std::milli>(t1 - t0).count();
    if (p.t_ev[0]) {   // the frame's GPU-side phases from its timing events (all complete)
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, p.t_ev[0], p.t_ev[1]) == hipSuccess)
            e->pstat[PS_GPU_IN_MS] += ms;
        if (hipEventElapsedTime(&ms, p.t_ev[2], p.t_ev[3]) == hipSuccess)
            e->pstat[PS_GPU_KERN_MS] += ms;
        if (hipEventElapsedTime(&ms, p.t_ev[4], p.t_ev[5]) == hipSuccess)
            e->pstat[PS_GPU_OUT_MS] += ms;
        if (hipEventElapsedTime(&ms, p.t_ev[0], p.t_ev[5]) == hipSuccess)
            e->pstat[PS_GPU_SPAN_MS] += ms;
        (void)hipGetLastError();
    }
    e->pstat[PS_FRAMES] += 1;
    const int S = e->S;
    memcpy(e->h_cnt, p.h_cnt, sizeof(BtCounters) * S);   // the latest known counters
    if (next_id)
        for (int s = 0; s < S; ++s) next_id[s] = p.h_cnt[s].next_id;
    const int rc = check_errors(e);
    if (rc) return rc;
    memcpy(out_offsets, p.h_pack_off, sizeof(int) * (S + 1));
    const long long rows = out_offsets[S];
    YTA_CHECK(rows <= p.rows_bound, YTA_ERR_HIP, "%lld output rows > %lld detections", rows,
              p.rows_bound);
    e->pstat[p.direct_out ? PS_OUT_DIRECT : PS_OUT_STAGED] += 64.0 * (double)rows;
    if (rows > 0 && !p.direct_out) {
        par_copy(e, p.user_out, p.h_pack, sizeof(double) * 8 * rows);
        e->pstat[PS_COPY_OUT_MS] += std::chrono::duration<double, std::milli>(
                                        std::chrono::steady_clock::now() - t1)
                                        .count();
    }
    return YTA_OK;
}

}  // namespace

extern "C" {

int yta_bytetrack_create(int device, int n_streams, int track_capacity, int max_dets,
                         const yta_bytetrack_params *params, yta_bytetrack **engine) {
    YTA_CHECK(engine && params, YTA_ERR_INVALID, "null engine/params");
    YTA_CHECK(params->frame_rate > 0 && params->track_buffer >= 0, YTA_ERR_INVALID,
              "frame_rate must be > 0 and track_buffer >= 0");
    yta_bytetrack_params prm = *params;
    return create_engine(device, n_streams, track_capacity, max_dets, engine,
                         [&](yta_bytetrack *e) { e->prm = prm; });
}

int yta_botsort_create(int device, int n_streams, int track_capacity, int max_dets, int feat_dim,
                       const yta_botsort_params *params, yta_botsort **engine) {
    YTA_CHECK(engine && params, YTA_ERR_INVALID, "null engine/params");
    YTA_CHECK(params->frame_rate > 0 && params->track_buffer >= 0, YTA_ERR_INVALID,
              "frame_rate must be > 0 and track_buffer >= 0");
    YTA_CHECK(params->with_reid == 0 || feat_dim > 0, YTA_ERR_INVALID,
              "with_reid needs feat_dim > 0");
    yta_botsort_params prm = *params;
    const int D = prm.with_reid ? feat_dim : 0;
    return create_engine(device, n_streams, track_capacity, max_dets, engine,
                         [&](yta_bytetrack *e) {
                             e->variant = VAR_BOTSORT;
                             e->bprm = prm;
                             e->D = D;
                             // few streams: the appearance costs chip-wide (k_bs_edges)
                             e->bs_split = D > 0 && n_streams <= 64;
                             if (const char *v = getenv("YTA_BS_SPLIT")) e->bs_split = D > 0 && atoi(v);
                         });
}

int yta_bytetrack_destroy(yta_bytetrack *e) {
    if (!e) return YTA_OK;
    (void)hipSetDevice(e->device);
    if (e->stream) (void)host_wait(e->stream);
    // pipelined frames submitted and not collected: their copy-in (slot / shared s_in) and
    // copy-out (s_out, k_rows_to_host into the caller's or the slot's mapped memory) may still be
    // running; drain every copy stream before any buffer they touch is freed
    for (auto &p : e->pipe)
        if (p.s_in) (void)hipStreamSynchronize(p.s_in);
    for (hipStream_t st : {e->s_in, e->s_out})
        if (st) (void)hipStreamSynchronize(st);
    if (e->g_exec) (void)hipGraphExecDestroy(e->g_exec);
    if (e->g_graph) (void)hipGraphDestroy(e->g_graph);
    release_buffers(e);
    if (e->h_dets) (void)hipHostFree(e->h_dets);
    if (e->d_det_in) (void)hipFree(e->d_det_in);
    if (e->d_pack) (void)hipFree(e->d_pack);
    if (e->h_pack) (void)hipHostFree(e->h_pack);
    if (e->d_pack_off) (void)hipFree(e->d_pack_off);
    if (e->h_pack_off) (void)hipHostFree(e->h_pack_off);
    if (e->h_feat) (void)hipHostFree(e->h_feat);
    if (e->d_feat_in) (void)hipFree(e->d_feat_in);
    if (e->h_active) (void)hipHostFree(e->h_active);
    if (e->d_det32) (void)hipFree(e->d_det32);
    if (e->h_det32) (void)hipHostFree(e->h_det32);
    pipe_free(e);
    for (hipEvent_t h : e->ev) (void)hipEventDestroy(h);
    if (e->stream) (void)hipStreamDestroy(e->stream);
    delete e;
    return YTA_OK;
}

int yta_bytetrack_reset(yta_bytetrack *e) {
    YTA_CHECK(e, YTA_ERR_INVALID, "null engine");
    YTA_CHECK(e->pipe_count == 0, YTA_ERR_INVALID, "pipelined frames in flight: collect them first");
    YTA_HIP(hipSetDevice(e->device));
    hipLaunchKernelGGL(k_reset, dim3(e->S), dim3(256), 0, e->stream, e->a, 0);
    YTA_HIP(hipGetLastError());
    YTA_HIP(hipMemsetAsync(e->a.kf, 0, sizeof(double) * TRK_STRIDE * (size_t)e->S * e->CAP,
                           e->stream));
    YTA_HIP(hipMemsetAsync(e->a.flags, 0, sizeof(int) * (size_t)e->S * e->CAP, e->stream));
    YTA_HIP(host_wait(e->stream));
    memset(e->h_cnt, 0, sizeof(BtCounters) * e->S);
    return YTA_OK;
}

int yta_bytetrack_reset_stream(yta_bytetrack *e, int stream) {
    YTA_CHECK(e, YTA_ERR_INVALID, "null engine");
    YTA_CHECK(e->pipe_count == 0, YTA_ERR_INVALID, "pipelined frames in flight: collect them first");
    YTA_CHECK(stream >= 0 && stream < e->S, YTA_ERR_INVALID, "stream %d outside 0..%d", stream,
              e->S - 1);
    YTA_HIP(hipSetDevice(e->device));
    hipLaunchKernelGGL(k_reset, dim3(1), dim3(256), 0, e->stream, e->a, stream);
    YTA_HIP(hipGetLastError());
    const size_t tb = (size_t)stream * e->CAP;
    YTA_HIP(hipMemsetAsync(e->a.kf + tb * TRK_STRIDE, 0, sizeof(double) * TRK_STRIDE * e->CAP,
                           e->stream));
    YTA_HIP(hipMemsetAsync(e->a.flags + tb, 0, sizeof(int) * e->CAP, e->stream));
    YTA_HIP(host_wait(e->stream));
    memset(&e->h_cnt[stream], 0, sizeof(BtCounters));
    return YTA_OK;
}

int yta_bytetrack_reserve(yta_bytetrack *e, int track_capacity, int max_dets) {
    YTA_CHECK(e, YTA_ERR_INVALID, "null engine");
    YTA_CHECK(e->pipe_count == 0, YTA_ERR_INVALID, "pipelined frames in flight: collect them first");
    YTA_HIP(hipSetDevice(e->device));
    return reserve(e, track_capacity, max_dets);
}

int yta_bytetrack_capacity(yta_bytetrack *e, int *track_capacity, int *max_dets) {
    YTA_CHECK(e && track_capacity && max_dets, YTA_ERR_INVALID, "null argument");
    *track_capacity = e->CAP;
    *max_dets = e->MAXD;
    return YTA_OK;
}

int yta_bytetrack_update(yta_bytetrack *e, const double *dets, const int *det_offsets,
                         long long *next_id, double *out, int out_capacity, int *out_offsets) {
    return update_host(e, dets, det_offsets, nullptr, next_id, out, out_capacity, out_offsets);
}

int yta_bytetrack_update_device(yta_bytetrack *e, const double *d_dets, const int *d_det_offsets,
                                double *d_out, int *d_out_counts) {
    YTA_CHECK(e && d_det_offsets && d_out, YTA_ERR_INVALID, "null argument");
    YTA_CHECK(e->pipe_count == 0, YTA_ERR_INVALID, "pipelined frames in flight: collect them first");
    return launch_pipeline(e, d_dets, d_det_offsets, d_out, d_out_counts);
}

int yta_bytetrack_update_streams(yta_bytetrack *e, int n_streams, const int *stream_ids,
                                 const double *dets, const int *det_offsets, long long *next_id,
                                 double *out, int out_capacity, int *out_offsets) {
    return update_host_subset(e, n_streams, stream_ids, dets, det_offsets, nullptr, next_id, out,
                              out_capacity, out_offsets, nullptr);
}

int yta_bytetrack_update_device_masked(yta_bytetrack *e, const int *d_active,
                                       const double *d_dets, const int *d_det_offsets,
                                       double *d_out, int *d_out_counts) {
    YTA_CHECK(e && d_det_offsets && d_out, YTA_ERR_INVALID, "null argument");
    YTA_CHECK(e->pipe_count == 0, YTA_ERR_INVALID, "pipelined frames in flight: collect them first");
    e->a.active = d_active;
    const int rc = launch_pipeline(e, d_dets, d_det_offsets, d_out, d_out_counts);
    e->a.active = nullptr;
    return rc;
}

int yta_bytetrack_submit(yta_bytetrack *e, const double *dets, const int *det_offsets,
                         const long long *next_id, double *out, int out_capacity) {
    return pipe_submit(e, dets, det_offsets, next_id, out, out_capacity);
}

int yta_bytetrack_submit_f32(yta_bytetrack *e, const float *dets, const int *det_offsets,
                             const long long *next_id, double *out, int out_capacity) {
    return pipe_submit(e, nullptr, det_offsets, next_id, out, out_capacity, dets);
}

int yta_bytetrack_update_f32(yta_bytetrack *e, const float *dets, const int *det_offsets,
                             long long *next_id, double *out, int out_capacity,
                             int *out_offsets) {
    return update_host(e, nullptr, det_offsets, nullptr, next_id, out, out_capacity, out_offsets,
                       nullptr, nullptr, dets);
}

int yta_bytetrack_collect(yta_bytetrack *e, long long *next_id, int *out_offsets) {
    return pipe_collect(e, next_id, out_offsets);
}

int yta_bytetrack_pipe_stats(yta_bytetrack *e, double *stats, int n, int reset) {
    YTA_CHECK(e && (stats || n == 0), YTA_ERR_INVALID, "null argument");
    for (int k = 0; k < n; ++k) stats[k] = k < PS_N ? e->pstat[k] : 0.0;
    if (reset)
        for (double &v : e->pstat) v = 0.0;
    return YTA_OK;
}

int yta_bytetrack_next_ids(yta_bytetrack *e, long long *next_id) {
    YTA_CHECK(e && next_id, YTA_ERR_INVALID, "null argument");
    YTA_CHECK(e->pipe_count == 0, YTA_ERR_INVALID, "pipelined frames in flight: collect them first");
    YTA_HIP(hipSetDevice(e->device));
    const int rc = read_counters(e);
    if (rc) return rc;
    for (int s = 0; s < e->S; ++s) next_id[s] = e->h_cnt[s].next_id;
    return YTA_OK;
}

int yta_bytetrack_sync(yta_bytetrack *e) {
    YTA_CHECK(e, YTA_ERR_INVALID, "null engine");
    YTA_CHECK(e->pipe_count == 0, YTA_ERR_INVALID, "pipelined frames in flight: collect them first");
    const int rc = read_counters(e);
    if (rc) return rc;
    return check_errors(e);
}

int yta_bytetrack_get_state(yta_bytetrack *e, int stream, int *n_tracks, long long *ints,
                            double *mean, double *cov) {
    YTA_CHECK(e && n_tracks && ints && mean && cov, YTA_ERR_INVALID, "null argument");
    YTA_CHECK(stream >= 0 && stream < e->S, YTA_ERR_INVALID, "bad stream %d", stream);
    YTA_CHECK(e->pipe_count == 0, YTA_ERR_INVALID, "pipelined frames in flight: collect them first");
    YTA_HIP(hipSetDevice(e->device));
    const int rc = read_counters(e);
    if (rc) return rc;
    const BtCounters c = e->h_cnt[stream];
    const long long tb = (long long)stream * e->CAP;
    std::vector<int> tr(c.n_tracked), lo(c.n_lost);
    std::vector<double> kf((size_t)e->CAP * TRK_STRIDE);
    std::vector<int> flags(e->CAP);
    if (c.n_tracked)
        YTA_HIP(hipMemcpy(tr.data(), e->a.tracked + tb, sizeof(int) * c.n_tracked,
                          hipMemcpyDeviceToHost));
    if (c.n_lost)
        YTA_HIP(hipMemcpy(lo.data(), e->a.lost + tb, sizeof(int) * c.n_lost, hipMemcpyDeviceToHost));
    YTA_HIP(hipMemcpy(kf.data(), e->a.kf + tb * TRK_STRIDE,
                      sizeof(double) * TRK_STRIDE * e->CAP, hipMemcpyDeviceToHost));
    YTA_HIP(hipMemcpy(flags.data(), e->a.flags + tb, sizeof(int) * e->CAP, hipMemcpyDeviceToHost));
    std::vector<int> kf_frame(e->CAP);
    YTA_HIP(hipMemcpy(kf_frame.data(), e->a.kf_frame + tb, sizeof(int) * e->CAP,
                      hipMemcpyDeviceToHost));
    std::vector<double> kfx(e->a.kfx ? (size_t)e->CAP * 16 : 0);
    if (e->a.kfx)
        YTA_HIP(hipMemcpy(kfx.data(), e->a.kfx + tb * 16, sizeof(double) * 16 * e->CAP,
                          hipMemcpyDeviceToHost));
    int n = 0;
    for (int which = 0; which < 2; ++which) {
        const std::vector<int> &lst = which ? lo : tr;
        for (int slot : lst) {
            TrackMeta m;
            memcpy(&m, kf.data() + (size_t)slot * TRK_STRIDE + TRK_META, sizeof(TrackMeta));
            long long *ii = ints + (long long)n * 7;
            ii[0] = which;
            ii[1] = m.id;
            ii[2] = flags[slot] & FL_STATE;
            ii[3] = (flags[slot] & FL_ACTIVATED) ? 1 : 0;
            ii[4] = m.frame_id;
            ii[5] = m.start_frame;
            ii[6] = m.tracklet_len;
            KfState st;
            memcpy(st.m, kf.data() + (size_t)slot * TRK_STRIDE, sizeof(double) * 8);
            memcpy(st.c, kf.data() + (size_t)slot * TRK_STRIDE + TRK_COV, sizeof(double) * 16);
            if (e->variant == VAR_BYTETRACK && which)   // lost list: lazily predicted
                kf_predict_lost(st, c.frame_id - kf_frame[slot]);
            for (int k = 0; k < 8; ++k) mean[(long long)n * 8 + k] = st.m[k];
            double *P = cov + (long long)n * 64;
            kf_cov_full(st, P);
            if (!kfx.empty() && (flags[slot] & FL_CROSS))   // BoT-SORT warped track
                for (int g = 0; g < 2; ++g)
                    for (int k = 0; k < 8; ++k) {
                        int r, q;
                        xcross(k, r, q);
                        P[grp_global(g, r) * 8 + grp_global(g, q)] = kfx[(size_t)slot * 16 + 8 * g + k];
                    }
            ++n;
        }
    }
    *n_tracks = n;
    return YTA_OK;
}

int yta_bytetrack_profile(yta_bytetrack *e, int enable) {
    YTA_CHECK(e, YTA_ERR_INVALID, "null engine");
    YTA_HIP(host_wait(e->stream));
    e->prof = enable != 0;
    e->ev_used = 0;
    return YTA_OK;
}

// Per-launch time summed over the frames run since profiling was enabled / last collected:
// ms[k] for the 4 launches of one frame in order (stage1, stage23, apply, finish); *frames =
// frames covered.
int yta_bytetrack_profile_collect(yta_bytetrack *e, double *ms, int *frames) {
    YTA_CHECK(e && ms && frames, YTA_ERR_INVALID, "null argument");
    YTA_HIP(host_wait(e->stream));
    const size_t per = BT_PHASES + 1;
    for (int k = 0; k < BT_PHASES; ++k) ms[k] = 0.0;
    *frames = (int)(e->ev_used / per);
    for (int f = 0; f < *frames; ++f)
        for (int k = 0; k < BT_PHASES; ++k) {
            float t = 0.f;
            YTA_HIP(hipEventElapsedTime(&t, e->ev[f * per + k], e->ev[f * per + k + 1]));
            ms[k] += t;
        }
    e->ev_used = 0;
    return YTA_OK;
}

int yta_bytetrack_stats(yta_bytetrack *e, long long *stats) {
    YTA_CHECK(e && stats, YTA_ERR_INVALID, "null argument");
    YTA_HIP(hipSetDevice(e->device));
    const int rc = read_counters(e);
    if (rc) return rc;
    constexpr int NS = 21;
    for (int k = 0; k < NS; ++k) stats[k] = 0;
    for (int s = 0; s < e->S; ++s) {
        const BtCounters &c = e->h_cnt[s];
        const long long v[NS] = {c.n_dets, c.n_high, c.n_second, c.n_pool, c.n_act, c.n_unc,
                                 c.n_left, c.n_rest, c.n_births, c.n_t2, c.n_l2, c.n_tracked,
                                 c.n_lost, c.n_out, (long long)c.n_edges[0],
                                 (long long)c.n_edges[1] + c.n_edges[2], c.n_fallback[0],
                                 c.n_fallback[1], c.n_lazy, c.n_res1, c.n_fallback_f};
        for (int k = 0; k < NS; ++k) stats[k] += v[k];
    }
    return YTA_OK;
}

int yta_bytetrack_modes(yta_bytetrack *e, long long *out, int n) {
    YTA_CHECK(e && (out || n <= 0), YTA_ERR_INVALID, "null argument");
    const long long v[YTA_BT_MODES] = {e->split23,          e->a.split23,   e->a.ws_slots,
                                       e->graphs,           e->bs_split,    e->g_captures,
                                       e->g_replays,        e->CAP,         e->MAXD};
    for (int k = 0; k < n && k < YTA_BT_MODES; ++k) out[k] = v[k];
    return YTA_OK;
}

int yta_bytetrack_set_lds(yta_bytetrack *e, int bytes) {
    YTA_CHECK(e, YTA_ERR_INVALID, "null engine");
    YTA_CHECK(bytes >= 0 && bytes <= 150 * 1024, YTA_ERR_INVALID, "LDS bytes must be in [0, 150 KiB]");
    YTA_HIP(hipSetDevice(e->device));
    YTA_HIP(host_wait(e->stream));
    e->a.lds_bytes = (size_t)bytes & ~(size_t)15;
    e->a.lds_bytes23 = std::min(e->a.lds_bytes, BT_LDS23_BYTES);
    e->a.lds_bytes_f = std::min(e->a.lds_bytes, BT_LDSF_BYTES);
    e->a.lds_bytes_l = std::min(e->a.lds_bytes, BT_LDSL_BYTES);
    e->a.lds_bytes_e = std::min(e->a.lds_bytes, BT_LDSE_BYTES);
    return set_lds_limits(std::max<size_t>(e->a.lds_bytes, BT_LDS_BYTES));
}

int yta_bytetrack_hip_stream(yta_bytetrack *e, void **stream) {
    YTA_CHECK(e && stream, YTA_ERR_INVALID, "null argument");
    *stream = (void *)e->stream;
    return YTA_OK;
}

int yta_botsort_update(yta_botsort *e, const double *dets, const int *det_offsets,
                       const float *feats, const double *warps, long long *next_id, double *out,
                       int out_capacity, int *out_offsets) {
    YTA_CHECK(e && e->variant == VAR_BOTSORT, YTA_ERR_INVALID, "not a BoT-SORT engine");
    const int rc = update_host(e, dets, det_offsets, feats, next_id, out, out_capacity, out_offsets,
                               warps);
    e->a.warp = e->d_warp_id;
    return rc;
}

int yta_botsort_update_device(yta_botsort *e, const double *d_dets, const int *d_det_offsets,
                              const float *d_feats, const double *d_warps, double *d_out,
                              int *d_out_counts) {
    YTA_CHECK(e && e->variant == VAR_BOTSORT && d_det_offsets && d_out, YTA_ERR_INVALID,
              "null argument / not a BoT-SORT engine");
    YTA_CHECK(e->D == 0 || d_feats, YTA_ERR_INVALID, "null feats");
    e->a.warp = d_warps ? d_warps : e->d_warp_id;
    const int rc = launch_pipeline(e, d_dets, d_det_offsets, d_out, d_out_counts, d_feats);
    e->a.warp = e->d_warp_id;
    return rc;
}

int yta_botsort_update_streams(yta_botsort *e, int n_streams, const int *stream_ids,
                               const double *dets, const int *det_offsets, const float *feats,
                               const double *warps, long long *next_id, double *out,
                               int out_capacity, int *out_offsets) {
    YTA_CHECK(e && e->variant == VAR_BOTSORT, YTA_ERR_INVALID, "not a BoT-SORT engine");
    return update_host_subset(e, n_streams, stream_ids, dets, det_offsets, feats, next_id, out,
                              out_capacity, out_offsets, warps);
}

int yta_botsort_get_features(yta_botsort *e, int stream, int *n_tracks, float *feats,
                             double *cls_hist, int *n_cls) {
    YTA_CHECK(e && e->variant == VAR_BOTSORT && n_tracks, YTA_ERR_INVALID,
              "null argument / not a BoT-SORT engine");
    YTA_CHECK(stream >= 0 && stream < e->S, YTA_ERR_INVALID, "bad stream %d", stream);
    YTA_HIP(hipSetDevice(e->device));
    const int rc = read_counters(e);
    if (rc) return rc;
    const BtCounters c = e->h_cnt[stream];
    const long long tb = (long long)stream * e->CAP;
    std::vector<int> lst(c.n_tracked + c.n_lost);
    if (c.n_tracked)
        YTA_HIP(hipMemcpy(lst.data(), e->a.tracked + tb, sizeof(int) * c.n_tracked,
                          hipMemcpyDeviceToHost));
    if (c.n_lost)
        YTA_HIP(hipMemcpy(lst.data() + c.n_tracked, e->a.lost + tb, sizeof(int) * c.n_lost,
                          hipMemcpyDeviceToHost));
    const int D = e->D;
    int n = 0;
    for (int slot : lst) {
        if (feats && D)
            YTA_HIP(hipMemcpy(feats + (long long)n * D, e->a.feat + (tb + slot) * D,
                              sizeof(float) * D, hipMemcpyDeviceToHost));
        if (cls_hist)
            YTA_HIP(hipMemcpy(cls_hist + (long long)n * CLS_K * 2, e->a.cls_hist + (tb + slot) * CLS_K,
                              sizeof(double2) * CLS_K, hipMemcpyDeviceToHost));
        if (n_cls) {
            TrackMeta m;
            YTA_HIP(hipMemcpy(&m, e->a.kf + (tb + slot) * TRK_STRIDE + TRK_META, sizeof(TrackMeta),
                              hipMemcpyDeviceToHost));
            n_cls[n] = m.n_cls;
        }
        ++n;
    }
    *n_tracks = n;
    return YTA_OK;
}

#ifdef YTA_STAMPS
int yta_debug_stamps(unsigned long long *out) {
    YTA_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * 128));
    return YTA_OK;
}
int yta_debug_apply(unsigned long long *out) {   // [4096][5]
    YTA_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_apl), sizeof(g_apl)));
    return YTA_OK;
}
int yta_debug_blocks(unsigned long long *out) {   // [8][YTA_BLK_MAX][2]
    YTA_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_blk), sizeof(g_blk)));
    return YTA_OK;
}
#endif

}  // extern "C"
