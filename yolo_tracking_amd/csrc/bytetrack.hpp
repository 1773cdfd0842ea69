// Tracker engine (ByteTrack, BoT-SORT): device-resident state for S independent streams (see
// bytetrack.hip).
#pragma once
#include "assoc.hpp"
#include "kf_xyah.hpp"

namespace yta {

// Track states (boxmot/trackers/bytetrack/basetrack.py:8-12) and flag bits.
constexpr int ST_NEW = 0, ST_TRACKED = 1, ST_LOST = 2, ST_REMOVED = 3;
constexpr int FL_STATE = 3;
constexpr int FL_ACTIVATED = 4;      // STrack.is_activated
constexpr int FL_EVER_REMOVED = 8;   // track_id is in BYTETracker.removed_stracks
constexpr int FL_REMOVED_NOW = 16;   // marked removed in the current frame (joins removed_stracks at its end)
constexpr int FL_CROSS = 32;         // BoT-SORT: a camera warp coupled the axes, kfx holds the cross terms

struct TrackMeta {                   // 48 B, one per slot
    double score;
    double cls;
    long long id;
    int det_ind;
    int n_cls;                       // BoT-SORT: entries of the class histogram (update_cls)
    int frame_id;
    int start_frame;
    int tracklet_len;
    int pad;
};

static_assert(sizeof(TrackMeta) == 48, "TrackMeta layout");

// One 256-B record per slot, two aligned 128-B lines: line 0 = the Kalman mean (8 f64) + the meta
// (6 f64) + 16 B of padding, line 1 = the four 2x2 covariance blocks (16 f64).  Everything an
// output row, a predicted box or duplicate removal needs is in line 0 (mean + score, cls, id,
// det_ind, frames); only the Kalman pass reads line 1.  (A 192-B record alone straddles a third
// line half of the time, a separate 48-B meta costs a line of its own.)
constexpr int TRK_STRIDE = 32;       // doubles per slot
constexpr int TRK_META = 8;          // offset of the meta in a record (doubles)
constexpr int TRK_COV = 16;          // offset of the covariance (doubles)
static_assert(TRK_META + 6 <= TRK_COV && TRK_COV + 16 == TRK_STRIDE, "record layout");

struct BtCounters {                  // one per stream, 128 B
    long long next_id;               // last issued track id (BaseTrack._count)
    int frame_id;
    int n_tracked, n_lost, n_free;
    int n_dets, n_high, n_second;
    int n_pool, n_act, n_unc;
    int n_left, n_rest, n_births;
    int n_t2, n_l2, n_out;
    int err;
    int n_edges[3];
    int n_fallback[2];               // cumulative: association redone over global memory
    int n_lazy;                      // ByteTrack: lost-list records k_apply left untouched
    int n_res1;                      // ByteTrack: stage-1 edges left to k_s1_lap
    int n_ref;                       // re-found Lost tracks (refound list)
    int n_fallback_f;                // cumulative: k_finish's duplicate-removal grid over global
    int slot_cursor;                 // births take free slots from here on, cyclically
    int bs_spill;                    // BoT-SORT split stage 1: a pool row had more than E_SLOTS
                                     // edges (k_bs_lap then runs the fused association)
    int fb23_mark;                   // split k_stage23: a block of this frame fell back (k_finish
                                     // counts the stream-frame once in n_fallback[1])
};
static_assert(sizeof(BtCounters) == 128, "BtCounters layout");


// Tracker variants (template parameter V of the kernels).
constexpr int VAR_BYTETRACK = 0, VAR_BOTSORT = 1;
constexpr int CLS_K = 8;             // BoT-SORT class-histogram entries per track
#ifndef YTA_ESLOTS
#define YTA_ESLOTS 4
#endif
constexpr int E_SLOTS = YTA_ESLOTS;  // candidate edges kept per pool row by k_s1_edges

struct BtArgs {
    int S, CAP, MAXD;
    double track_thresh, match_thresh, det_thresh;   // det_thresh: births (BoT-SORT new_track_thresh)
    double low_thresh;        // second-stage lower confidence bound (ByteTrack 0.1)
    int max_time_lost;
    // BoT-SORT
    double prox_thresh, app_thresh;
    int fuse_first;           // fuse_first_associate
    int D;                    // appearance feature length (0: with_reid off)
    const float *det_feat;    // per frame: [rows of det_in][D] ReID features (high rows read)
    float *det_fn;            // [S*MAXD][4] per high detection: the norms n1, n2, n3 of its row
    float *feat;              // [S*CAP][D] smoothed track features
    double2 *cls_hist;        // [S*CAP][CLS_K] (class, summed score)
    int *ema_job;             // [S*CAP] per k_apply item: high position of the detection taken
                              // with its feature, else -1
    // inputs
    const double *det_in;     // packed rows of 6
    const int *det_off;       // S+1
    // persistent state
    double *kf;               // [S*CAP][TRK_STRIDE]: Kalman state + TrackMeta per slot
    double *kfx;              // BoT-SORT: [S*CAP][16] covariance cross terms (kf_xyah.hpp, FL_CROSS)
    const double *warp;       // BoT-SORT: [S][6] this frame's camera warps (multi_gmc), row-major 2x3
    int *flags;               // [S*CAP] state + FL_* bits, dense: every list scan reads these
    int *kf_frame;            // [S*CAP] ByteTrack, Lost tracks: the frame their stored Kalman
                              // state belongs to (later predicts replayed lazily, kf_xyah.hpp)
    int *tracked, *lost, *free_list;   // [S*CAP]
    BtCounters *cnt;          // [S]
    // per-frame: detections [S*MAXD]
    int *high, *second, *rest, *birth;
    Box *high_box, *second_box;
    double *high_score, *rest_score;
    // per-frame: tracks [S*CAP]
    int *pool, *unc, *left, *left_of_pool, *t2, *l2;
    int2 *refound;            // [S*CAP] (slot, stage-1 high position) of each re-found Lost track
    int *l2pos;               // [S*CAP] per lost' entry: its pool position (k_finish)
    Box *pool_box, *unc_box;
    // association results
    int *x1, *y1, *x2, *y2, *x3, *y3;   // x*: [S*CAP], y*: [S*MAXD]
    // association workspace: LDS arena size, per-stream global fallback arena, solver slabs
    size_t lds_bytes, lds_bytes23, lds_bytes_f;   // arenas of k_stage1 / k_stage23 / k_finish
    unsigned char *ws;
    long long ws_stride;
    // few streams: k_stage23 runs stage 2 and stage 3 (independent given stage 1) in two blocks
    // per stream; stage 3's block has its own fallback arena [S * ws_stride] and solver slabs
    int split23;
    unsigned char *ws3;       // unused (round 6: the stage-3 block claims from the pool below)
    // the global fallback arenas are a pool of ws_slots arenas of ws_stride bytes shared by the
    // engine's streams: a block whose LDS arena is too small queues its stream in redo_q and the
    // launch's redo kernel (bytetrack.hip k_redo_*, ws_slots blocks) redoes it over arena
    // blockIdx.x; worst-case arenas for every stream cost O(S * CAP * MAXD) bytes of HBM
    int ws_slots;
    int *redo_q;              // [2 + 2S]: queued count, redo blocks done, queued block ids
    LapSlab slab;             // per stream: (threads / 64) slabs
    // ByteTrack stage 1 as three launches (k_s1_prep / k_s1_edges / k_s1_lap): the per-stream
    // grid over the high detections and every pool row's first candidate edges, in HBM
    int *g_cell;              // [S][GRID_MAX_CELLS + 1] cell starts
    int *g_ids, *g_big;       // [S*MAXD] binned high positions in cell order / big items
    Box *g_boxes;             // [S*MAXD] their boxes, cell order
    double *g_w;              // [S*MAXD] their scores (fuse_score weights), cell order
    GridHdr *g_hdr;           // [S]
    int *e_cnt;               // [S*CAP] candidate edges per pool row (0 once matched outright)
    int *g_deg;               // [S*MAXD] candidate edges per high detection (HBM-grid path)
    int *e_col;               // [E_SLOTS][S*CAP] the first E_SLOTS edges' high positions
    double *e_cost;           // [E_SLOTS][S*CAP] and costs
    size_t lds_bytes_l;       // k_s1_lap arena
    size_t lds_bytes_e;       // k_s1_edges grid
    // outputs
    double *out;              // [S*CAP][8]
    int *out_counts;          // optional [S]
    BtCounters *cnt_mirror;   // optional [S]: k_finish copies each stream's final counters here
                              // (one-stream host update: right after the rows, so one copy
                              // returns both)
    // stream subset: [S] nonzero = update this stream this frame; nullptr = every stream.  A
    // skipped stream's kernels return at once (its state, frame counter and ID counter are not
    // touched); k_finish reports 0 output rows for it.
    const int *active;
};

__device__ __forceinline__ bool stream_skipped(const BtArgs &a, int s) {
    return a.active != nullptr && a.active[s] == 0;
}

}  // namespace yta
