// HybridSORT update() for S independent streams on gfx950, all tracker state resident in HBM.
//
// Follows boxmot/trackers/hybridsort/hybridsort.py:373-570 (HybridSORT.update without its
// PerClassDecorator, which the host side replays call by call) with the association of
// boxmot/trackers/hybridsort/association.py:495-581 as HybridSORT configures it (hard-wired,
// hybridsort.py:346-360): TCM weight 0, ReID weight 1.3 on the short-term embedding cost,
// long-term ReID weight 0, long-term correction at 0.4, no BYTE round (hybridsort.yaml).  One
// frame (one undecorated update call) =
//   k_hs_predict [grid]          predict every tracker (:296-320: velocity clamp, 9-d Kalman
//                                predict, kalman / simple scores) and its column inputs (box,
//                                kalman score, 4 corner velocities, k-previous and last
//                                observations), one thread per tracker
//   k_hs_pre     [block/stream]  NaN cull (:406-416: compacts the column inputs when a tracker
//                                goes), confidence split (:391-404)
//   k_hs_emb     [grid]          stage-1 cost tiles: dets_feats x smooth_feats on f64 MFMA
//                                (v_mfma_f64_16x16x4_f64) with the row norms, cosine distance
//                                max(0, 1 - uv / sqrt(uu vv)) (association.py:667-684), and in the
//                                same epilogue the asso function, the four corner angle costs
//                                (:314-383, :507-518) and the fused cost
//                                -(iou + angle) + 1.3 emb (:531-539)
//   k_hs_assoc   [block/stream]  padded LAP (lapx semantics, no limit), long-term correction
//                                (:557-567), tracker updates (Kalman + ORU replay, corner
//                                velocities, observations), OCR round on the last observations
//                                (:512-542), misses, births, outputs in reversed tracker order,
//                                removal (:544-570)
//   k_hs_ema     [grid]          update_features of first-round matches (EMA alpha 0.8, float32)
//                                and the smooth features of births (:197-214)
#include <algorithm>
#include <cstring>
#include <new>
#include <vector>

#include "kf_hybrid.hpp"
#include "kf_ocsort.hpp"   // np_sum5
#include "ocsort_common.hpp"
#include "subset.hpp"

namespace yta {
namespace {

constexpr int HF_CPRE = 8;          // confidence_pre is not None
constexpr int ERR_INF_ROW = 64;     // a predicted box with an inf but no NaN (the reference's
                                    // trks / trackers lists would disagree, hybridsort.py:412-416)
constexpr int HS_RING = OC_DT_MAX + 1;
constexpr double HS_TRACK_THRESH = 0.6;     // predict(track_thresh=0.6) (:296)
constexpr double HS_EG_WEIGHT = 1.3;        // EG_weight_high_score (:347)
constexpr double HS_CORR_THRESH = 0.4;      // longterm_reid_correction_thresh (:355)

struct HsTrack {
    Kf9 kf;
    Kf9 fz;                         // frozen filter (attr_saved x / P)
    double hist_z[5];               // the filter's last measurement kept in history_obs
    double last_obs[5];
    double vel[8];                  // velocity_lt, _rt, _lb, _rb: (dy, dx) each
    double conf, cls, det_ind;      // det_ind holds the detection's score (dets0[:, 6])
    double confidence, conf_pre;
    double obs[HS_RING][5];
    long long id;
    int obs_age[HS_RING];
    int obs_n;
    int age, hits, hit_streak, tsu, flags, hist_since;
};

struct HsCounters {
    long long next_id;
    int frame;
    int n_trk, n_free;
    int n_dets, n_high, n_out, n_births;
    int lap_calls, corrections;
    int n_ema;
    int err;
    int lap_done;                  // first round solved by k_hs_lap this frame
    LapStats ls;                   // cumulative solver counters
    int n_ud, n_ut, n_upd;         // k_hs_assoc -> k_hs_ocr -> k_hs_assoc_b: the OCR round's sizes
    int ocr_nan;                   // the OCR matrix holds a NaN (its max is then NaN)
    unsigned long long ocr_max;    // its maximum, order-preserving bits (hs_ord)
    int pad[7];
};
static_assert(sizeof(HsCounters) == 128, "HsCounters layout");

// per-tracker association inputs, one 160-B record (k_hs_pre -> k_hs_emb / k_hs_assoc)
struct HsCol {
    double box[4];
    double kscore;                  // clip(x[3], 0.6, 1)
    double kobs[5];                 // k_previous_obs
    double vel[8];
    double valid;                   // k_previous_obs[4] >= 0 (valid_mask)
    double pad;
};

struct HsArgs {
    int S, CAP, MAXD, D;
    double det_thresh, thr, inertia;
    int max_age, min_hits, delta_t, asso;
    const double *det_in;
    const int *det_off;
    const float *det_feat;          // [rows of det_in][D] get_features output
    HsTrack *rec;                   // [S*CAP]
    float *feat;                    // [S*CAP][D] smooth_feat (float32)
    int *list, *free_list;          // [S*CAP]
    HsCounters *cnt;
    // per frame
    int *hi_row;                    // [S*MAXD]
    int *corr;                      // [S*MAXD] first-round pair undone by the long-term correction
    HsCol *col;                     // [S*CAP]
    double *clast;                  // [S*CAP][5] last observations
    int *nan_flag, *cslot;          // [S*CAP]
    double *cost, *emat;            // [S*MAXD*CAP]
    int *rmatch, *cmatched;
    int *udet, *utrk, *tmp;         // [S*(MAXD+CAP)]
    int *upd;                       // [S*CAP] kept-detection index updating each tracker or -1
    int *ema_slot, *ema_row;        // [S*(CAP+MAXD)] feature jobs: slot, kept index (birth: ~p)
    unsigned char *lap_ws;
    unsigned char *lap_csr;         // per stream: the replay's row entries (nullptr: n < LAPB_MIN_N)
    long long lap_csr_stride;
    long long lap_ws_stride;
    double *pre_u, *pre_s2;        // [S*MAXD] first-round row pre-pass (lap_rect.hpp)
    int *pre_x;
    double *out;
    int *out_counts;
    int arr_chip;                  // first rounds solved with the chip-wide bidding rounds
    const int *active;             // [S] nonzero = update the stream this frame; null = all
};

__device__ __forceinline__ long long hs_mb(const HsArgs &a, int s) {
    return (long long)s * (a.MAXD > 4 ? a.MAXD : 4) * a.CAP;
}

// corner (x column, y column) of velocity_lt, _rt, _lb, _rb (hybridsort.py:74-103,
// association.py:338-383)
__device__ __forceinline__ int hs_cx(int c) { return c < 2 ? 0 : 2; }
__device__ __forceinline__ int hs_cy(int c) { return (c & 1) ? 3 : 1; }

// speed_direction_{lt,rt,lb,rb}(prev, cur) (hybridsort.py:74-103) -> (dy, dx)
__device__ __forceinline__ void hs_dir(const double *p, const double *b, int c, double &vy,
                                       double &vx) {
    const double cx1 = p[hs_cx(c)], cy1 = p[hs_cy(c)];
    const double cx2 = b[hs_cx(c)], cy2 = b[hs_cy(c)];
    const double sy = cy2 - cy1, sx = cx2 - cx1;
    const double nrm = sqrt(sy * sy + sx * sx) + 1e-6;
    vy = sy / nrm;
    vx = sx / nrm;
}

// k_previous_obs (hybridsort.py:22-30) from the ring
__device__ __forceinline__ void hs_prev_obs(const HsTrack &r, int dt, double *o) {
    if (r.obs_n == 0) {
        for (int k = 0; k < 5; ++k) o[k] = -1.0;
        return;
    }
    const int m = r.obs_n < HS_RING ? r.obs_n : HS_RING;
    for (int i = 0; i < dt; ++i) {
        const int want = r.age - (dt - i);
        for (int e = 0; e < m; ++e)
            if (r.obs_age[e] == want) {
                for (int k = 0; k < 5; ++k) o[k] = r.obs[e][k];
                return;
            }
    }
    const int newest = (r.obs_n - 1) % HS_RING;
    for (int k = 0; k < 5; ++k) o[k] = r.obs[newest][k];
}

// KalmanBoxTracker.update (hybridsort.py:230-294) + KalmanFilter.update (hybridsort_kf.py:439-528).
// bbox = dets[p] (x1, y1, x2, y2, score); cls / det_ind = dets0[p, 5] / dets0[p, 6].
__device__ void hs_update(HsTrack &r, const double *bbox, double cls, double det_ind, int dt) {
    if (!bbox) {
        if (r.flags & OF_OBSERVED) {          // freeze
            r.fz = r.kf;
            r.flags |= OF_SAVED;
        }
        r.flags &= ~(OF_OBSERVED | HF_CPRE);  // confidence_pre = None
        r.hist_since += 1;
        return;
    }
    r.conf = bbox[4];
    r.cls = cls;
    r.det_ind = det_ind;
    if (np_sum5(r.last_obs) >= 0) {
        const int m = r.obs_n < HS_RING ? r.obs_n : HS_RING;
        bool found = false;
        double acc[8];
        for (int i = 0; i < dt; ++i) {        // every stored observation within delta_t (no break)
            const int want = r.age - i - 1;
            for (int e = 0; e < m; ++e)
                if (r.obs_age[e] == want) {
                    for (int c = 0; c < 4; ++c) {
                        double vy, vx;
                        hs_dir(r.obs[e], bbox, c, vy, vx);
                        if (found) {
                            acc[2 * c] = acc[2 * c] + vy;
                            acc[2 * c + 1] = acc[2 * c + 1] + vx;
                        } else {
                            acc[2 * c] = vy;
                            acc[2 * c + 1] = vx;
                        }
                    }
                    found = true;
                    break;
                }
        }
        if (!found)
            for (int c = 0; c < 4; ++c) hs_dir(r.last_obs, bbox, c, acc[2 * c], acc[2 * c + 1]);
        for (int k = 0; k < 8; ++k) r.vel[k] = acc[k];
        r.flags |= OF_VELOCITY;
    }
    for (int k = 0; k < 5; ++k) r.last_obs[k] = bbox[k];
    const int slot = r.obs_n % HS_RING;
    for (int k = 0; k < 5; ++k) r.obs[slot][k] = bbox[k];
    r.obs_age[slot] = r.age;
    r.obs_n += 1;
    r.tsu = 0;
    r.hits += 1;
    r.hit_streak += 1;
    double z[5];
    hs_bbox_to_z(bbox, z);
    if (!(r.flags & OF_OBSERVED) && (r.flags & OF_SAVED)) {   // unfreeze: restore, replay
        r.kf = r.fz;
        r.flags &= ~OF_SAVED;
        kf9_replay(r.kf, r.hist_z, z, r.hist_since + 1, r.hist_z);
    } else {
        for (int k = 0; k < 5; ++k) r.hist_z[k] = z[k];
    }
    r.hist_since = 0;
    r.flags |= OF_OBSERVED;
    kf9_correct(r.kf, z);
    r.conf_pre = r.confidence;                // confidence_pre = confidence (never None here)
    r.flags |= HF_CPRE;
    r.confidence = bbox[4];
}

// KalmanBoxTracker.predict (hybridsort.py:296-320): returns the predicted box; kalman / simple
// scores through ks / ss
__device__ void hs_predict(HsTrack &r, double *b, double &ks, double &ss) {
    if (r.kf.x[7] + r.kf.x[2] <= 0) r.kf.x[7] = r.kf.x[7] * 0.0;
    kf9_predict(r.kf);
    r.age += 1;
    if (r.tsu > 0) r.hit_streak = 0;
    r.tsu += 1;
    hs_x_to_bbox(r.kf.x, b);
    ks = np_min(np_max(r.kf.x[3], HS_TRACK_THRESH), 1.0);
    const bool pre = (r.flags & HF_CPRE) && r.conf_pre != 0.0;   // `if not self.confidence_pre`
    const double v = pre ? r.confidence - (r.conf_pre - r.confidence) : r.confidence;
    ss = np_min(np_max(v, 0.1), HS_TRACK_THRESH);
}

// KalmanBoxTracker.__init__ (hybridsort.py:112-194)
__device__ void hs_birth(HsTrack &out, const double *bbox, double cls, double det_ind, long long id) {
    HsTrack r;
    double z[5];
    hs_bbox_to_z(bbox, z);
    kf9_init(z, r.kf);
    r.fz = r.kf;
    for (int k = 0; k < 5; ++k) {
        r.hist_z[k] = 0.0;
        r.last_obs[k] = -1.0;
    }
    for (int k = 0; k < 8; ++k) r.vel[k] = 0.0;
    r.conf = bbox[4];
    r.cls = cls;
    r.det_ind = det_ind;
    r.confidence = bbox[4];
    r.conf_pre = 0.0;
    r.id = id;
    r.obs_n = 0;
    for (int e = 0; e < HS_RING; ++e) r.obs_age[e] = -1;
    r.age = r.hits = r.hit_streak = r.tsu = 0;
    r.flags = 0;
    r.hist_since = 0;
    out = r;
}

// predict (hybridsort.py:406-413) of every tracker, chip-wide: boxes and scores into the column
// records (by list position); k_hs_pre compacts the survivors per stream.
// One wave per block, as k_hs_upd (HS_UPD_T): the trackers spread over 4x the CUs.
__global__ __launch_bounds__(64) void k_hs_predict(HsArgs a) {
    const int s = blockIdx.y;
    if (a.active && !a.active[s]) return;   // stream not updated this frame
    HsCounters *c = a.cnt + s;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= c->n_trk) return;
    const long long tb = (long long)s * a.CAP;
    HsTrack &r = a.rec[tb + a.list[tb + i]];
    double b[4], ks, ss;
    hs_predict(r, b, ks, ss);
    const double sc = r.kf.x[3];
    const bool nan = (b[0] != b[0]) || (b[1] != b[1]) || (b[2] != b[2]) || (b[3] != b[3]) ||
                     (sc != sc);
    if (!nan && !(fabs(b[0]) < INFINITY && fabs(b[1]) < INFINITY && fabs(b[2]) < INFINITY &&
                  fabs(b[3]) < INFINITY && fabs(sc) < INFINITY))
        atomicOr(&c->err, ERR_INF_ROW);
    a.nan_flag[tb + i] = nan;
    // the column record at the tracker's list position, complete (k_hs_pre keeps it in place
    // when no tracker is culled, the steady state; otherwise it compacts the survivors' records)
    HsCol q;
    for (int k = 0; k < 4; ++k) q.box[k] = b[k];
    q.kscore = ks;
    (void)ss;   // simple score: trks[:, 5], read only by the BYTE round (use_byte = False)
    double ko[5];
    hs_prev_obs(r, a.delta_t, ko);
    for (int k = 0; k < 5; ++k) q.kobs[k] = ko[k];
    const bool hv = (r.flags & OF_VELOCITY) != 0;
    for (int k = 0; k < 8; ++k) q.vel[k] = hv ? r.vel[k] : 0.0;
    q.valid = ko[4] < 0 ? 0.0 : 1.0;
    q.pad = 0.0;
    a.col[tb + i] = q;
    for (int k = 0; k < 5; ++k) a.clast[(tb + i) * 5 + k] = r.last_obs[k];
    a.cslot[tb + i] = a.list[tb + i];
    a.cmatched[tb + i] = 0;
    a.upd[tb + i] = -1;
}

__global__ __launch_bounds__(OC_T) void k_hs_pre(HsArgs a) {
    __shared__ OcShared sh;
    const int s = blockIdx.x, t = threadIdx.x, nt = blockDim.x;
    if (a.active && !a.active[s]) return;   // stream not updated this frame
    HsCounters *c = a.cnt + s;
    const long long tb = (long long)s * a.CAP, db = (long long)s * a.MAXD;
    const long long ub = (long long)s * (a.MAXD + a.CAP);
    int nd = a.det_off[s + 1] - a.det_off[s];
    if (nd > a.MAXD || nd < 0) {
        if (t == 0) atomicOr(&c->err, ERR_DET_CAPACITY);
        nd = nd < 0 ? 0 : a.MAXD;
    }
    const double *din = a.det_in + (long long)a.det_off[s] * 6;
    int n_trk = c->n_trk;
    int *list = a.list + tb;
    HsCol *col = a.col + tb;
    // predict and the column records ran chip-wide in k_hs_predict (by list position)
    int n_free = c->n_free;
    const int n_nan = block_compact(n_trk, sh.wsum, [&](int i) { return a.nan_flag[tb + i] != 0; },
                                    [&](int i, int pos) { a.tmp[ub + pos] = list[i]; });
    if (n_nan > 0) {   // cull: the survivors' records compacted
        block_sync();   // the compaction's tmp stores (other threads' runs) before their reads
        for (int k = t; k < n_nan; k += nt) a.free_list[tb + n_free + k] = a.tmp[ub + k];
        n_free += n_nan;
        block_sync();
        const int n_keep = block_compact(n_trk, sh.wsum, [&](int i) { return a.nan_flag[tb + i] == 0; },
                                         [&](int i, int pos) {
                                             a.tmp[ub + pos] = list[i];
                                             a.upd[tb + pos] = i;
                                         });
        block_sync();
        // kept trackers' column records, compacted (scratch: the cost matrix)
        HsCol *scratch = reinterpret_cast<HsCol *>(a.cost + hs_mb(a, s));
        for (int j = t; j < n_keep; j += nt) {
            const HsTrack &r = a.rec[tb + a.tmp[ub + j]];
            scratch[j] = col[a.upd[tb + j]];
            for (int k = 0; k < 5; ++k) a.clast[(tb + j) * 5 + k] = r.last_obs[k];
        }
        block_sync();
        for (int j = t; j < n_keep; j += nt) {
            list[j] = a.tmp[ub + j];
            a.cslot[tb + j] = a.tmp[ub + j];
            col[j] = scratch[j];
            a.cmatched[tb + j] = 0;
            a.nan_flag[tb + j] = 0;
            a.upd[tb + j] = -1;
        }
        n_trk = n_keep;
        if (t == 0) c->n_free = n_free;
        block_sync();
    }
    // detections kept for association (:401-404)
    const int n_hi = block_compact(nd, sh.wsum, [&](int i) { return din[i * 6 + 4] > a.det_thresh; },
                                   [&](int i, int pos) { a.hi_row[db + pos] = i; });
    for (int i = t; i < n_hi; i += nt) a.rmatch[db + i] = -1;
    if (t == 0) {
        c->n_trk = n_trk;
        c->n_high = n_hi;
        c->n_dets = nd;
    }
}

// ---------------------------------------------------------------------------------- k_hs_emb
// 64 (detections) x 64 (trackers) cost tiles per block, 4 waves of 32 x 32 (2 x 2 MFMA tiles of
// v_mfma_f64_16x16x4_f64: A[l&15][k = l>>4], B[k = l>>4][l&15], D[row (l>>4) + 4 r][col l&15]).
// The embedding dimension streams through LDS in chunks of 32 floats, double-buffered (one
// barrier per chunk: a chunk is stored into the other buffer while this one's MFMAs run) and
// widened to float64 as the MFMA operands are read (exact); the row norms accumulate from the
// same chunks.  Rows are 36 floats apart, so the 16 rows x 4 k of one operand read hit 64
// distinct banks.  The epilogue's column records reuse the GEMM buffers (LDS 47.6 -> 38 KiB:
// four blocks per CU), and the association function is a template argument.  Tiles are placed
// by XCD row bands (xcd_tile): C5 1049 -> 861 us per 4096^2 launch, 7.16 -> 5.65 ms at 8 streams.
typedef double dbl4 __attribute__((ext_vector_type(4)));
constexpr int HE_TILE = 64, HE_KC = 32, HE_LDF = 36;

struct HsDetCol {                   // per detection row of the tile
    double box[4], score;
};

union HeLds {
    struct {
        float A[2][HE_TILE * HE_LDF], B[2][HE_TILE * HE_LDF];
    } g;
    struct {
        HsDetCol d[HE_TILE];
        HsCol t[HE_TILE];
    } c;
};

template <int ASSO>
__global__ __launch_bounds__(256, 4) void k_hs_emb(HsArgs a) {
    __shared__ __attribute__((aligned(16))) HeLds L;
    __shared__ double nA[HE_TILE], nB[HE_TILE];
    const int s = blockIdx.z;
    if (a.active && !a.active[s]) return;   // stream not updated this frame
    const HsCounters *c = a.cnt + s;
    const int n_trk = c->n_trk, n_hi = c->n_high, D = a.D;
    int bx, by;
    xcd_tile(bx, by);                                         // row bands per XCD (common.hpp)
    const int r0 = by * HE_TILE, c0 = bx * HE_TILE;
    if (r0 >= n_hi || c0 >= n_trk) return;                   // block-uniform
    const long long tb = (long long)s * a.CAP, db = (long long)s * a.MAXD, mb = hs_mb(a, s);
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int wr = (w >> 1) * 32, wc = (w & 1) * 32;
    // staging: thread t loads 8 consecutive k of row t >> 2 (A: detection, B: tracker)
    const int lr = t >> 2, lk = (t & 3) * 8;
    const bool a_ok = r0 + lr < n_hi, b_ok = c0 + lr < n_trk;
    const float *arow = a_ok ? a.det_feat + ((long long)a.det_off[s] + a.hi_row[db + r0 + lr]) * D
                             : nullptr;
    const float *brow = b_ok ? a.feat + (tb + a.cslot[tb + c0 + lr]) * D : nullptr;
    double qa = 0.0, qb = 0.0;
    dbl4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = dbl4{0.0, 0.0, 0.0, 0.0};
    // the next chunk's 8 + 8 floats are loaded into registers while this chunk's MFMAs run
    // (float4 pairs when D is a multiple of the chunk: rows then start 128-B aligned)
    float4 pa[2], pb[2];
    const bool vec = (D % HE_KC) == 0;
    auto fetch = [&](int k0) {
        const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
        if (vec) {
            pa[0] = a_ok ? *reinterpret_cast<const float4 *>(arow + k0 + lk) : z;
            pa[1] = a_ok ? *reinterpret_cast<const float4 *>(arow + k0 + lk + 4) : z;
            pb[0] = b_ok ? *reinterpret_cast<const float4 *>(brow + k0 + lk) : z;
            pb[1] = b_ok ? *reinterpret_cast<const float4 *>(brow + k0 + lk + 4) : z;
        } else {
            float ta[8], tb8[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int k = k0 + lk + u;
                ta[u] = (a_ok && k < D) ? arow[k] : 0.f;
                tb8[u] = (b_ok && k < D) ? brow[k] : 0.f;
            }
            pa[0] = make_float4(ta[0], ta[1], ta[2], ta[3]);
            pa[1] = make_float4(ta[4], ta[5], ta[6], ta[7]);
            pb[0] = make_float4(tb8[0], tb8[1], tb8[2], tb8[3]);
            pb[1] = make_float4(tb8[4], tb8[5], tb8[6], tb8[7]);
        }
    };
    // norms in k order (u = 0..7 of this thread's 8), then the chunk into LDS buffer b
    auto stash = [&](int b) {
        const float va[8] = {pa[0].x, pa[0].y, pa[0].z, pa[0].w, pa[1].x, pa[1].y, pa[1].z, pa[1].w};
        const float vb[8] = {pb[0].x, pb[0].y, pb[0].z, pb[0].w, pb[1].x, pb[1].y, pb[1].z, pb[1].w};
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const double av = (double)va[u], bv = (double)vb[u];
            qa += av * av;
            qb += bv * bv;
        }
        float4 *da = reinterpret_cast<float4 *>(&L.g.A[b][lr * HE_LDF + lk]);
        float4 *dbp = reinterpret_cast<float4 *>(&L.g.B[b][lr * HE_LDF + lk]);
        da[0] = pa[0];
        da[1] = pa[1];
        dbp[0] = pb[0];
        dbp[1] = pb[1];
    };
    fetch(0);
    stash(0);
    __syncthreads();
    int buf = 0;
    for (int k0 = 0; k0 < D; k0 += HE_KC) {
        const bool more = k0 + HE_KC < D;
        if (more) fetch(k0 + HE_KC);
        const float *As = L.g.A[buf], *Bs = L.g.B[buf];
#pragma unroll
        for (int ks = 0; ks < HE_KC; ks += 4) {
            const int kk = ks + (lane >> 4);
            double af[2], bf[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) af[i] = (double)As[(wr + 16 * i + (lane & 15)) * HE_LDF + kk];
#pragma unroll
            for (int j = 0; j < 2; ++j) bf[j] = (double)Bs[(wc + 16 * j + (lane & 15)) * HE_LDF + kk];
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[i], bf[j], acc[i][j], 0, 0, 0);
        }
        // the other buffer was last read before the previous barrier
        if (more) stash(buf ^ 1);
        __syncthreads();
        buf ^= 1;
    }
    // row norms (4 threads per row)
    qa += __shfl_xor(qa, 1);
    qa += __shfl_xor(qa, 2);
    qb += __shfl_xor(qb, 1);
    qb += __shfl_xor(qb, 2);
    if ((t & 3) == 0) {
        nA[lr] = qa;
        nB[lr] = qb;
    }
    // column records over the GEMM buffers (every MFMA read is behind the loop's last barrier)
    HsDetCol *dcol = L.c.d;
    HsCol *tcol = L.c.t;
    if (t < HE_TILE) {
        const int p = r0 + t;
        if (p < n_hi) {
            const double *dr = a.det_in + ((long long)a.det_off[s] + a.hi_row[db + p]) * 6;
            HsDetCol dc;
#pragma unroll
            for (int k = 0; k < 4; ++k) dc.box[k] = dr[k];
            dc.score = dr[4];
            dcol[t] = dc;
        }
    } else if (t < 2 * HE_TILE) {
        const int j = c0 + t - HE_TILE;
        if (j < n_trk) {   // 20 doubles, copied as such (a struct copy goes through scratch)
            const double *src = reinterpret_cast<const double *>(a.col + tb + j);
            double *dst = reinterpret_cast<double *>(tcol + (t - HE_TILE));
#pragma unroll
            for (int k = 0; k < (int)(sizeof(HsCol) / 8); ++k) dst[k] = src[k];
        }
    }
    __syncthreads();
    // epilogue: cosine distance, asso function, corner angle costs, fused cost
    bool giou_bad = false;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) {
                const int lrow = wr + 16 * i + (lane >> 4) + 4 * rr;
                const int lcol = wc + 16 * j + (lane & 15);
                const int p = r0 + lrow, q = c0 + lcol;
                if (p >= n_hi || q >= n_trk) continue;
                const double uv = acc[i][j][rr];
                const double emb = np_max(0.0, 1.0 - uv / sqrt(nA[lrow] * nB[lcol]));
                const HsDetCol &dc = dcol[lrow];
                const HsCol &tc = tcol[lcol];
                const Box db_{dc.box[0], dc.box[1], dc.box[2], dc.box[3]};
                const Box tb_{tc.box[0], tc.box[1], tc.box[2], tc.box[3]};
                const double v = asso_of(ASSO, db_, tb_, 0.0, 0.0);
                if (ASSO == 1 && v != v) giou_bad = true;
                double angle = 0.0;
#pragma unroll
                for (int cc = 0; cc < 4; ++cc) {
                    const double dx = dc.box[hs_cx(cc)] - tc.kobs[hs_cx(cc)];
                    const double dy = dc.box[hs_cy(cc)] - tc.kobs[hs_cy(cc)];
                    const double nrm = sqrt(dx * dx + dy * dy) + 1e-6;
                    const double X = dx / nrm, Y = dy / nrm;
                    double cs = tc.vel[2 * cc + 1] * X + tc.vel[2 * cc] * Y;
                    cs = np_min(np_max(cs, -1.0), 1.0);
                    const double ang = (M_PI / 2.0 - fabs(acos(cs))) / M_PI;
                    const double term = ((tc.valid * ang) * a.inertia) * dc.score;
                    angle = cc == 0 ? term : angle + term;
                }
                double cost = -(v + angle);
                cost = cost + HS_EG_WEIGHT * emb;
                cost = cost + 0.0;                            // + 0 * long-term cost
                const long long o = mb + (long long)p * n_trk + q;
                a.emat[o] = emb;
                a.cost[o] = cost;
            }
    if (giou_bad) atomicOr(&a.cnt[s].err, ERR_GIOU);
}

// -------------------------------------------------------------------------------- k_hs_assoc
// Row pre-pass of the first-round solve, chip-wide (lap_rect.hpp).
__global__ __launch_bounds__(OC_T) void k_hs_rowpre(HsArgs a) {
    const int s = blockIdx.y;
    if (a.active && !a.active[s]) return;   // stream not updated this frame
    const HsCounters *c = a.cnt + s;
    const long long db = (long long)s * a.MAXD;
    main_lap_pre(a.cost + hs_mb(a, s), c->n_high, c->n_trk, a.pre_u + db, a.pre_x + db,
                 a.pre_s2 + db);
}

// First-round solve, one LAP_T-thread block per stream (ocsort_common.hpp first_round_lap).
__global__ __launch_bounds__(LAP_T) void k_hs_lap(HsArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int s = blockIdx.x;
    if (a.active && !a.active[s]) return;   // stream not updated this frame
    HsCounters *c = a.cnt + s;
    const long long tb = (long long)s * a.CAP, db = (long long)s * a.MAXD;
    first_round_lap(a.cost + hs_mb(a, s), c->n_high, c->n_trk, a.rmatch + db, a.cmatched + tb, false,
                    a.pre_u + db, a.pre_x + db, a.pre_s2 + db, a.rmatch + db, lds,
                    lap_kernel_lds(a.CAP, a.MAXD), a.lap_ws + s * a.lap_ws_stride, &c->err,
                    &c->lap_done, &c->ls, a.lap_ws + (s + 1) * a.lap_ws_stride - tight_ws_bytes(),
                    nullptr, a.arr_chip != 0);
}

// The chip-wide bidding rounds of the first round (ocsort_common.hpp fr_arr_*), when a.arr_chip.
__global__ __launch_bounds__(OC_T) void k_hs_arr0(HsArgs a) {
    __shared__ int wsum[32];
    const int s = blockIdx.x;
    if (a.active && !a.active[s]) return;   // stream not updated this frame
    const HsCounters *c = a.cnt + s;
    const long long tb = (long long)s * a.CAP, db = (long long)s * a.MAXD;
    fr_arr_round0(a.cost + hs_mb(a, s), c->n_high, c->n_trk, a.rmatch + db, a.cmatched + tb, false,
                  a.pre_u + db, a.pre_x + db, a.pre_s2 + db,
                  a.lap_ws + (s + 1) * a.lap_ws_stride - tight_ws_bytes(), wsum);
}
__global__ __launch_bounds__(ARR_SCAN_WPB * WAVE) void k_hs_arrscan(HsArgs a) {
    const int s = blockIdx.y;
    if (a.active && !a.active[s]) return;
    const HsCounters *c = a.cnt + s;
    fr_arr_scan(a.cost + hs_mb(a, s), c->n_high, c->n_trk, a.lap_ws + (s + 1) * a.lap_ws_stride - tight_ws_bytes(),
                blockIdx.x, gridDim.x);
}
__global__ __launch_bounds__(OC_T) void k_hs_arrapply(HsArgs a) {
    __shared__ int wsum[32];
    const int s = blockIdx.x;
    if (a.active && !a.active[s]) return;
    const HsCounters *c = a.cnt + s;
    fr_arr_apply(a.cost + hs_mb(a, s), c->n_high, c->n_trk, a.lap_ws + (s + 1) * a.lap_ws_stride - tight_ws_bytes(),
                 wsum);
}

// HybridSORT's long-term correction (hybridsort/association.py:557-567): a first-round pair (kept
// detection i, tracker k) is undone when emb > 0.4 and iou - |kalman score - score| < thr.
__device__ __forceinline__ bool hs_corrected(const HsArgs &a, int s, int i, int k, int n_trk) {
    const long long tb = (long long)s * a.CAP, db = (long long)s * a.MAXD;
    const double e = a.emat[hs_mb(a, s) + (long long)i * n_trk + k];
    if (!(e > HS_CORR_THRESH)) return false;
    const double *dr = a.det_in + ((long long)a.det_off[s] + a.hi_row[db + i]) * 6;
    const HsCol &q = a.col[tb + k];
    const double v = asso_of(a.asso, box5(dr), Box{q.box[0], q.box[1], q.box[2], q.box[3]}, 0.0,
                             0.0);
    const double sd = fabs(q.kscore - dr[4]);
    return (v - sd) < a.thr;
}

// First-round Kalman updates (hybridsort.py:462-464) chip-wide, one thread per kept detection,
// when k_hs_lap solved the first round (else k_hs_assoc updates after its own solve).  A tracker
// is matched at most once and the updates only touch its record, so they are independent.
// One wave per block: a 4096-detection frame spreads over 64 CUs instead of 16, so the record
// gathers of each update (one record per lane) go through 4x as many CUs' memory pipes.
constexpr int HS_UPD_T = 64;
__global__ __launch_bounds__(HS_UPD_T) void k_hs_upd(HsArgs a) {
    const int s = blockIdx.y;
    if (a.active && !a.active[s]) return;   // stream not updated this frame
    const HsCounters *c = a.cnt + s;
    const int n_trk = c->n_trk, n_hi = c->n_high;
    const int i = blockIdx.x * HS_UPD_T + threadIdx.x;
    if (!c->lap_done || i >= n_hi || n_trk == 0) return;
    const long long tb = (long long)s * a.CAP, db = (long long)s * a.MAXD;
    const int k = a.rmatch[db + i];
    const bool corr = k >= 0 && hs_corrected(a, s, i, k, n_trk);
    a.corr[db + i] = corr;   // for k_hs_assoc's lists
    if (k < 0 || corr) return;
    const double *din = a.det_in + (long long)a.det_off[s] * 6;
    // cls / det_ind from dets0 row i of the input (filtered position, :464)
    hs_update(a.rec[tb + a.list[tb + k]], din + (long long)a.hi_row[db + i] * 6,
              din[(long long)i * 6 + 5], din[(long long)i * 6 + 4], a.delta_t);
}

__global__ __launch_bounds__(OC_T) void k_hs_assoc(HsArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    __shared__ OcShared sh;
    const int s = blockIdx.x, t = threadIdx.x, nt = blockDim.x;
    if (a.active && !a.active[s]) {   // not updated this frame: no output rows
        if (threadIdx.x == 0) {
            a.cnt[s].n_out = 0;
            if (a.out_counts) a.out_counts[s] = 0;
        }
        return;
    }
    HsCounters *c = a.cnt + s;
    const long long tb = (long long)s * a.CAP, db = (long long)s * a.MAXD, mb = hs_mb(a, s);
    const long long ub = (long long)s * (a.MAXD + a.CAP);
    unsigned char *gws = a.lap_ws + s * a.lap_ws_stride;
    const long long lds_bytes = oc_lds_bytes(a.CAP, a.MAXD);
    const double *din = a.det_in + (long long)a.det_off[s] * 6;
    int n_trk = c->n_trk;
    const int n_hi = c->n_high;
    const int dt = a.delta_t;
    int *list = a.list + tb;
    double *cost = a.cost + mb;
    int *udet = a.udet + ub, *utrk = a.utrk + ub;
    int n_ud = 0, n_ut = 0;
    int n_corr = 0;
    // dets[p] (x1, y1, x2, y2, score) of kept detection p: input row hi_row[p]
    auto hrow = [&](int p) { return din + (long long)a.hi_row[db + p] * 6; };
    YTA_STAMP_BASE(40);
    YTA_STAMP(0);
    // ---- first round (association.py:495-581)
    if (n_trk == 0 || n_hi == 0) {
        for (int i = t; i < n_hi; i += nt) udet[i] = i;
        for (int j = t; j < n_trk; j += nt) utrk[j] = j;
        n_ud = n_hi;
        n_ut = n_trk;
        if (t == 0) c->lap_calls = 0;
        block_sync();
    } else {
        block_sync();
        if (!c->lap_done)   // else solved by k_hs_lap
            main_lap(LapMat{cost, n_hi, n_trk, false}, a.pre_u + db, a.pre_x + db, a.pre_s2 + db,
                 a.rmatch + db, lds, lds_bytes, gws, &c->err, &c->ls,
                     a.lap_csr ? a.lap_csr + s * a.lap_csr_stride : nullptr);
        YTA_STAMP(1);
        if (t == 0) c->lap_calls = 1;
        for (int j = t; j < n_trk; j += nt) a.cmatched[tb + j] = 0;
        block_sync();
        for (int i = t; i < n_hi; i += nt) {
            const int k = a.rmatch[db + i];
            if (k >= 0) a.cmatched[tb + k] = 1;
        }
        block_sync();
        n_ud = block_compact(n_hi, sh.wsum, [&](int i) { return a.rmatch[db + i] < 0; },
                             [&](int i, int pos) { udet[pos] = i; });
        n_ut = block_compact(n_trk, sh.wsum, [&](int j) { return a.cmatched[tb + j] == 0; },
                             [&](int j, int pos) { utrk[pos] = j; });
        // long-term correction (:557-567): emb > 0.4 and iou - |kalman score - score| < thr
        // (decided by k_hs_upd when k_hs_lap solved the round)
        if (!c->lap_done) {
            for (int i = t; i < n_hi; i += nt) {
                const int k = a.rmatch[db + i];
                a.corr[db + i] = k >= 0 && hs_corrected(a, s, i, k, n_trk);
            }
            block_sync();
        }
        auto corrected = [&](int i) { return a.corr[db + i] != 0; };
        n_corr = block_compact(n_hi, sh.wsum, corrected, [&](int i, int pos) {
            udet[n_ud + pos] = i;
            utrk[n_ut + pos] = a.rmatch[db + i];
        });
        for (int i = t; i < n_hi; i += nt) {
            const int k = a.rmatch[db + i];
            if (k >= 0 && !corrected(i)) a.upd[tb + k] = i;
        }
        n_ud += n_corr;
        n_ut += n_corr;
        block_sync();
    }
    YTA_STAMP(2);
    // first-round updates with features (:462-464); feature jobs for k_hs_ema
    const long long eb = (long long)s * (a.CAP + a.MAXD);
    const int n_upd = block_compact(n_trk, sh.wsum, [&](int j) { return a.upd[tb + j] >= 0; },
                                    [&](int j, int pos) {
                                        a.ema_slot[eb + pos] = list[j];
                                        a.ema_row[eb + pos] = a.upd[tb + j];
                                    });
    if (!c->lap_done) {   // else applied chip-wide by k_hs_upd
        for (int j = t; j < n_trk; j += nt) {
            const int p = a.upd[tb + j];
            if (p >= 0) {
                // cls / det_ind from dets0 row p of the input (filtered position, :464)
                hs_update(a.rec[tb + list[j]], hrow(p), din[(long long)p * 6 + 5],
                          din[(long long)p * 6 + 4], dt);
            }
        }
    }
    block_sync();
    YTA_STAMP(3);
    // the OCR round's matrix is filled chip-wide (k_hs_ocr); k_hs_assoc_b solves and finishes
    if (t == 0) {
        c->n_ud = n_ud;
        c->n_ut = n_ut;
        c->n_upd = n_upd;
        c->corrections = n_corr;
        c->ocr_nan = 0;
        c->ocr_max = 0ull;
    }
}

// Order-preserving bits of a double (larger value, larger bits), for the OCR matrix's maximum.
__device__ __forceinline__ unsigned long long hs_ord(double v) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(v);
    return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
__device__ __forceinline__ double hs_unord(unsigned long long o) {
    const unsigned long long b = (o >> 63) ? (o & 0x7FFFFFFFFFFFFFFFull) : ~o;
    return __longlong_as_double((long long)b);
}

// OCR round matrix (:512-542): asso_func(left dets, last observations) over the chip, one entry per
// thread, with its maximum (np.max: NaN-propagating, ocr_nan) for k_hs_assoc_b.
__global__ __launch_bounds__(256) void k_hs_ocr(HsArgs a) {
    __shared__ OcShared sh;
    const int s = blockIdx.y;
    if (a.active && !a.active[s]) return;
    HsCounters *c = a.cnt + s;
    const int n_ud = c->n_ud, n_ut = c->n_ut;
    if (n_ud <= 0 || n_ut <= 0) return;
    const long long tb = (long long)s * a.CAP, db = (long long)s * a.MAXD, mb = hs_mb(a, s);
    const long long ub = (long long)s * (a.MAXD + a.CAP);
    const double *din = a.det_in + (long long)a.det_off[s] * 6;
    const int *udet = a.udet + ub, *utrk = a.utrk + ub;
    double *mat = a.emat + mb;   // the embedding costs are no longer needed
    const long long nm = (long long)n_ud * n_ut;
    double mx = -INFINITY;
    bool bad = false, nan = false;
    for (long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x; q < nm;
         q += (long long)gridDim.x * blockDim.x) {
        const int p = (int)(q / n_ut), k = (int)(q % n_ut);
        const Box db_ = box5(din + (long long)a.hi_row[db + udet[p]] * 6);
        const Box tb_ = box5(a.clast + (tb + utrk[k]) * 5);
        const double v = asso_of(a.asso, db_, tb_, 0.0, 0.0);
        bad |= a.asso == 1 && v != v;
        nan |= v != v;
        mat[q] = v;
        if (v == v) mx = v > mx ? v : mx;
    }
    if (bad) atomicOr(&c->err, ERR_GIOU);
    if (nan) atomicOr(&c->ocr_nan, 1);
    mx = block_max(mx, sh);
    if (threadIdx.x == 0 && mx > -INFINITY) atomicMax(&c->ocr_max, hs_ord(mx));
}

// The OCR solve's row pre-pass over the grid (main_lap_pre, as k_hs_rowpre for the first round),
// when the solve runs (max > thr).  The first round's pre-pass arrays are free by now.
__global__ __launch_bounds__(OC_T) void k_hs_ocr_pre(HsArgs a) {
    const int s = blockIdx.y;
    if (a.active && !a.active[s]) return;
    const HsCounters *c = a.cnt + s;
    const int n_ud = c->n_ud, n_ut = c->n_ut;
    if (n_ud <= 0 || n_ut <= 0 || c->ocr_nan || !(hs_unord(c->ocr_max) > a.thr)) return;
    const long long db = (long long)s * a.MAXD;
    main_lap_pre(a.emat + hs_mb(a, s), n_ud, n_ut, a.pre_u + db, a.pre_x + db, a.pre_s2 + db,
                 true);   // the -IoU round solves -mat
}

// The rest of the association after k_hs_ocr: the OCR round's solve (:512-542), misses, births,
// outputs, removal (:544-570).
__global__ __launch_bounds__(OC_T) void k_hs_assoc_b(HsArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    __shared__ OcShared sh;
    const int s = blockIdx.x, t = threadIdx.x, nt = blockDim.x;
    if (a.active && !a.active[s]) return;   // (k_hs_assoc reported no rows)
    HsCounters *c = a.cnt + s;
    const long long tb = (long long)s * a.CAP, db = (long long)s * a.MAXD, mb = hs_mb(a, s);
    const long long ub = (long long)s * (a.MAXD + a.CAP);
    unsigned char *gws = a.lap_ws + s * a.lap_ws_stride;
    const long long lds_bytes = oc_lds_bytes(a.CAP, a.MAXD);
    const double *din = a.det_in + (long long)a.det_off[s] * 6;
    const int frame = c->frame + 1;
    int n_trk = c->n_trk;
    const int n_hi = c->n_high;
    const int dt = a.delta_t;
    int *list = a.list + tb;
    double *emat = a.emat + mb;
    int *udet = a.udet + ub, *utrk = a.utrk + ub;
    int n_ud = 0, n_ut = 0;
    int n_corr = 0;
    // dets[p] (x1, y1, x2, y2, score) of kept detection p: input row hi_row[p]
    auto hrow = [&](int p) { return din + (long long)a.hi_row[db + p] * 6; };
    YTA_STAMP_BASE(40);
    YTA_STAMP_BASE(40);
    n_ud = c->n_ud;
    n_ut = c->n_ut;
    n_corr = c->corrections;
    const int n_upd = c->n_upd;
    const long long eb = (long long)s * (a.CAP + a.MAXD);
    // ---- OCR round (:512-542): asso_func(left dets, last observations), no feature update
    if (n_ud > 0 && n_ut > 0) {
        double *mat = emat;   // filled by k_hs_ocr
        const double mx = c->ocr_nan ? NAN : hs_unord(c->ocr_max);
        YTA_STAMP(8);
#ifdef YTA_STAMPS
        const unsigned long long fr0 = g_stamps[100], st0 = g_stamps[101];
        if (blockIdx.x == 0 && t == 0) {
            g_stamps[49] = n_ud;
            g_stamps[50] = n_ut;
        }
#endif
        if (mx > a.thr) {
            iou_lap<1024>(LapMat{mat, n_ud, n_ut, true}, a.rmatch + db, lds, lds_bytes, gws, &c->err, &c->ls,
                          a.lap_ws + (s + 1) * a.lap_ws_stride - tight_ws_bytes(), a.pre_u + db,
                          a.pre_x + db, a.pre_s2 + db, a.thr);   // row pre-pass: k_hs_ocr_pre
#ifdef YTA_STAMPS
            if (blockIdx.x == 0 && t == 0) {   // this solve's free rows and search steps
                g_stamps[51] = g_stamps[100] - fr0;
                g_stamps[52] = g_stamps[101] - st0;
            }
#endif
            for (int i = t; i < n_hi; i += nt) a.tmp[ub + i] = 0;
            for (int j = t; j < n_trk; j += nt) a.nan_flag[tb + j] = 0;
            block_sync();
            for (int p = t; p < n_ud; p += nt) a.tmp[ub + udet[p]] = 1;
            for (int k = t; k < n_ut; k += nt) a.nan_flag[tb + utrk[k]] = 1;
            block_sync();
            for (int p = t; p < n_ud; p += nt) {
                const int k = a.rmatch[db + p];
                if (k >= 0 && !(mat[(long long)p * n_ut + k] < a.thr)) {
                    const int di = udet[p], tj = utrk[k];
                    hs_update(a.rec[tb + list[tj]], hrow(di), din[(long long)di * 6 + 5],
                              din[(long long)di * 6 + 4], dt);
                    a.tmp[ub + di] = 0;
                    a.nan_flag[tb + tj] = 0;
                }
            }
            block_sync();
            n_ud = block_compact(n_hi, sh.wsum, [&](int i) { return a.tmp[ub + i] == 1; },
                                 [&](int i, int pos) { udet[pos] = i; });
            n_ut = block_compact(n_trk, sh.wsum, [&](int j) { return a.nan_flag[tb + j] == 1; },
                                 [&](int j, int pos) { utrk[pos] = j; });
            for (int j = t; j < n_trk; j += nt) a.nan_flag[tb + j] = 0;
            if (t == 0) c->lap_calls += 1;
            block_sync();
        }
    }
    YTA_STAMP(4);
    // ---- misses (:544-545)
    for (int k = t; k < n_ut; k += nt) hs_update(a.rec[tb + list[utrk[k]]], nullptr, 0.0, 0.0, dt);
    block_sync();
    YTA_STAMP(5);
    // ---- births in unmatched-list order (:548-550)
    int n_free = c->n_free;
    int n_b = n_ud;
    if (n_b > n_free) {
        if (t == 0) atomicOr(&c->err, ERR_TRACK_CAPACITY);
        n_b = n_free;
    }
    const long long next_id = c->next_id;
    // a birth's record is built in LDS (the solver's arena is free by now) by its thread and
    // stored by the whole block in 16-B pieces, consecutive lanes on consecutive pieces (one
    // thread storing its record word by word beside the others' touched a line per birth and
    // store instruction); 8-B pieces (the record is a multiple of 8 B)
    static_assert(sizeof(HsTrack) % 8 == 0, "HsTrack is stored in 8-B pieces");
    constexpr int REC_Q = (int)(sizeof(HsTrack) / 8);
    HsTrack *bstage = reinterpret_cast<HsTrack *>(lds);
    int bch = (int)(lds_bytes / (long long)sizeof(HsTrack));
    bch = bch < 1 ? 1 : (bch > nt ? nt : bch);
    for (int b0 = 0; b0 < n_b; b0 += bch) {
        const int m = n_b - b0 < bch ? n_b - b0 : bch;
        for (int r = t; r < m; r += nt) {
            const int b = b0 + r;
            const int slot = a.free_list[tb + n_free - 1 - b];
            const int p = udet[b];
            hs_birth(bstage[r], hrow(p), din[(long long)p * 6 + 5], din[(long long)p * 6 + 4],
                     next_id + b);
            list[n_trk + b] = slot;
            a.ema_slot[eb + n_upd + b] = slot;
            a.ema_row[eb + n_upd + b] = ~p;
        }
        lds_sync();
        for (int q = t; q < m * REC_Q; q += nt) {
            const int r = q / REC_Q, k = q - r * REC_Q;
            const int slot = a.free_list[tb + n_free - 1 - (b0 + r)];
            reinterpret_cast<double *>(&a.rec[tb + slot])[k] =
                reinterpret_cast<const double *>(&bstage[r])[k];
        }
        lds_sync();
    }
    n_free -= n_b;
    n_trk += n_b;
    block_sync();
    YTA_STAMP(6);
    // ---- outputs in reversed tracker order, then removal (:551-570); ids + 1 (:563).  Every
    // record read is batched (block_compact_ld / batched_for2): a per-item chain of list ->
    // record loads would cost a round trip per tracker.  The removal flags of the pass
    // (nan_flag: 0 on entry) feed the two removal compactions.
    double *out = a.out + tb * 8;
    struct TrkState {
        int slot, tsu, hit_streak;
    };
    int *oslot = a.tmp + ub;   // the output trackers' slots, in output order
    const int n_out = block_compact_ld<8>(
        n_trk, sh.wsum, [&](int q) { return list[n_trk - 1 - q]; },
        [&](int, int slot) {
            const HsTrack &r = a.rec[tb + slot];
            return TrkState{slot, r.tsu, r.hit_streak};
        },
        [&](int q, const TrkState &v) {
            a.nan_flag[tb + n_trk - 1 - q] = v.tsu > a.max_age;
            return v.tsu < 1 && (v.hit_streak >= a.min_hits || frame <= a.min_hits);
        },
        [&](int, const TrkState &v, int pos) { oslot[pos] = v.slot; });
    block_sync();   // the slots (other threads' runs) before their reads
    struct OutRow {
        double b[4], id, conf, cls, det_ind;
    };
    batched_for2<4>(
        n_out, [&](int pos) { return oslot[pos]; },
        [&](int, int slot) {
            const HsTrack &r = a.rec[tb + slot];
            OutRow o;
            if (np_sum5(r.last_obs) < 0) hs_x_to_bbox(r.kf.x, o.b);
            else for (int k = 0; k < 4; ++k) o.b[k] = r.last_obs[k];
            o.id = (double)(r.id + 1);
            o.conf = r.conf;
            o.cls = r.cls;
            o.det_ind = r.det_ind;
            return o;
        },
        [&](int pos, const OutRow &o) {
            double *d = out + (long long)pos * 8;
            for (int k = 0; k < 4; ++k) d[k] = o.b[k];
            d[4] = o.id;
            d[5] = o.conf;
            d[6] = o.cls;
            d[7] = o.det_ind;
        });
    block_sync();   // oslot (tmp) is reused below
    const int n_dead = block_compact(n_trk, sh.wsum, [&](int j) { return a.nan_flag[tb + j] != 0; },
                                     [&](int j, int pos) { a.tmp[ub + pos] = list[j]; });
    block_sync();   // the compaction's tmp stores (other threads' runs) before their reads
    for (int k = t; k < n_dead; k += nt) a.free_list[tb + n_free + k] = a.tmp[ub + k];
    block_sync();
    const int n_live = block_compact(n_trk, sh.wsum, [&](int j) { return a.nan_flag[tb + j] == 0; },
                                     [&](int j, int pos) { a.tmp[ub + pos] = list[j]; });
    block_sync();
    for (int j = t; j < n_live; j += nt) list[j] = a.tmp[ub + j];
    for (int j = t; j < n_trk; j += nt) a.nan_flag[tb + j] = 0;
    if (t == 0) {
        c->frame = frame;
        c->n_trk = n_live;
        c->n_free = n_free + n_dead;
        c->n_out = n_out;
        c->n_births = n_b;
        c->n_ema = n_upd + n_b;
        c->corrections = n_corr;
        c->next_id = next_id + n_b;
        if (a.out_counts) a.out_counts[s] = n_out;
    }
    YTA_STAMP(7);
}

// ---------------------------------------------------------------------------------- k_hs_ema
// update_features (hybridsort.py:197-214), float32 as the reference: f = e / |e| (in place on the
// detection's row), smooth = 0.8 smooth + 0.2 f, smooth /= |smooth|; a birth's smooth_feat is its
// row normalised twice (feat is smooth_feat).  Norms: np.linalg.norm of a float32 row, the sum of
// squares accumulated in float64 here (OpenBLAS sdot sums in float32 lanes, so a norm may differ
// from the reference's in its last bit; the tests compare features with a tolerance).  One wave
// per job.
__device__ __forceinline__ float hs_f32_norm(double sumsq) { return sqrtf((float)sumsq); }

__global__ __launch_bounds__(256) void k_hs_ema(HsArgs a) {
    const int s = blockIdx.y, lane = lane_id();
    if (a.active && !a.active[s]) return;   // stream not updated this frame
    const HsCounters *c = a.cnt + s;
    const int job = blockIdx.x * 4 + threadIdx.x / WAVE;
    if (job >= c->n_ema) return;
    const long long tb = (long long)s * a.CAP, db = (long long)s * a.MAXD;
    const long long eb = (long long)s * (a.CAP + a.MAXD);
    const int slot = a.ema_slot[eb + job], code = a.ema_row[eb + job];
    const int p = code >= 0 ? code : ~code;
    const float *e = a.det_feat + ((long long)a.det_off[s] + a.hi_row[db + p]) * a.D;
    float *sm = a.feat + (tb + slot) * a.D;
    double q = 0.0;
    for (int k = lane; k < a.D; k += WAVE) q += (double)e[k] * (double)e[k];
    const float n1 = hs_f32_norm(wave_reduce(RED_SUM, q));
    q = 0.0;
    if (code < 0) {
        for (int k = lane; k < a.D; k += WAVE) {
            const float f = e[k] / n1;
            q += (double)f * (double)f;
        }
        const float n2 = hs_f32_norm(wave_reduce(RED_SUM, q));
        for (int k = lane; k < a.D; k += WAVE) sm[k] = (e[k] / n1) / n2;
        return;
    }
    for (int k = lane; k < a.D; k += WAVE) {
        const float f = e[k] / n1;
        const float v = 0.8f * sm[k] + 0.2f * f;
        sm[k] = v;
        q += (double)v * (double)v;
    }
    const float nrm = hs_f32_norm(wave_reduce(RED_SUM, q));
    for (int k = lane; k < a.D; k += WAVE) sm[k] = sm[k] / nrm;
}

// KalmanBoxTracker KAT: one thread per track, steps of predict, update(box | None)
__global__ void k_kf9_run(int n, int steps, const double *b0, const double *b, double *x_out,
                          double *P_out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    HsTrack r;
    hs_birth(r, b0 + 5LL * i, 0.0, 0.0, 0);
    for (int st = 0; st < steps; ++st) {
        double bb[4], ks, ss;
        hs_predict(r, bb, ks, ss);
        const double *z = b + ((long long)st * n + i) * 5;
        hs_update(r, z[0] != z[0] ? nullptr : z, 0.0, 0.0, 3);
    }
    for (int k = 0; k < 9; ++k) x_out[9LL * i + k] = r.kf.x[k];
    double *M = P_out + 81LL * i;
    for (int k = 0; k < 81; ++k) M[k] = 0.0;
    for (int g = 0; g < 4; ++g) {
        M[g * 9 + g] = r.kf.p[4 * g];
        M[g * 9 + g + 5] = r.kf.p[4 * g + 1];
        M[(g + 5) * 9 + g] = r.kf.p[4 * g + 2];
        M[(g + 5) * 9 + g + 5] = r.kf.p[4 * g + 3];
    }
    M[4 * 9 + 4] = r.kf.p[16];
}

__global__ void k_hs_reset(HsArgs a, int s0) {
    const int s = s0 + blockIdx.x;
    const long long tb = (long long)s * a.CAP;
    for (int i = threadIdx.x; i < a.CAP; i += blockDim.x) a.free_list[tb + i] = a.CAP - 1 - i;
    if (threadIdx.x == 0) {
        HsCounters z;
        memset(&z, 0, sizeof(z));
        z.n_free = a.CAP;
        z.next_id = 0;                         // KalmanBoxTracker.count = 0 (:361)
        a.cnt[s] = z;
    }
}

}  // namespace
}  // namespace yta

// ================================================================================== host engine
using namespace yta;

struct yta_hybridsort {
    int device = 0, S = 0, CAP = 0, MAXD = 0, D = 0;
    yta_hybridsort_params prm{};
    hipStream_t stream = nullptr;
    std::vector<void *> allocs;
    HsArgs a{};
    double *h_dets = nullptr, *d_det_in = nullptr;
    long long det_cap = 0;
    float *h_feat = nullptr, *d_feat = nullptr;
    long long feat_cap = 0;
    int *h_off = nullptr, *d_off = nullptr;
    HsCounters *h_cnt = nullptr;
    size_t lds = 0;
    StreamMask mask;   // stream-subset updates (subset.hpp)
};

namespace {

template <typename T>
int hs_dalloc(yta_hybridsort *e, T **p, long long n) {
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

#define HSALLOC(ptr, n)                      \
    do {                                     \
        int _rc = hs_dalloc(e, &(ptr), (n)); \
        if (_rc) return _rc;                 \
    } while (0)

int hs_alloc(yta_hybridsort *e) {
    const long long S = e->S, CAP = e->CAP, MAXD = e->MAXD, D = e->D;
    HsArgs &a = e->a;
    const yta_hybridsort_params &p = e->prm;
    a.S = e->S;
    a.CAP = e->CAP;
    a.MAXD = e->MAXD;
    a.D = e->D;
    a.det_thresh = p.det_thresh;
    a.thr = p.iou_threshold;
    a.inertia = p.inertia;
    a.max_age = p.max_age;
    a.min_hits = p.min_hits;
    a.delta_t = p.delta_t;
    a.asso = p.asso_func;
    HSALLOC(a.rec, S * CAP);
    HSALLOC(a.feat, S * CAP * D);
    HSALLOC(a.list, S * CAP);
    HSALLOC(a.free_list, S * CAP);
    HSALLOC(a.cnt, S);
    HSALLOC(a.hi_row, S * MAXD);
    HSALLOC(a.corr, S * MAXD);
    HSALLOC(a.col, S * CAP);
    HSALLOC(a.clast, S * CAP * 5);
    HSALLOC(a.nan_flag, S * CAP);
    HSALLOC(a.cslot, S * CAP);
    // the cost matrix doubles as the column-record scratch of k_hs_pre (CAP records of 160 B)
    const long long mat = std::max<long long>(MAXD, (long long)sizeof(HsCol) / 8) * CAP;
    HSALLOC(a.cost, S * mat);
    HSALLOC(a.emat, S * mat);
    HSALLOC(a.rmatch, S * MAXD);
    HSALLOC(a.pre_u, S * MAXD);
    HSALLOC(a.pre_s2, S * MAXD);
    HSALLOC(a.pre_x, S * MAXD);
    HSALLOC(a.cmatched, S * CAP);
    HSALLOC(a.udet, S * (MAXD + CAP));
    HSALLOC(a.utrk, S * (MAXD + CAP));
    HSALLOC(a.tmp, S * (MAXD + CAP));
    HSALLOC(a.upd, S * CAP);
    HSALLOC(a.ema_slot, S * (MAXD + CAP));
    HSALLOC(a.ema_row, S * (MAXD + CAP));
    HSALLOC(a.out, S * CAP * 8);
    const long long n = std::max(CAP, MAXD);
    a.lap_ws_stride = oc_lap_ws_stride(n);
    a.arr_chip = MAXD >= ARR_CHIP_MIN_DETS;
    if (const char *v = getenv("YTA_ARR_CHIP")) a.arr_chip = atoi(v);
    HSALLOC(a.lap_ws, S * a.lap_ws_stride);
    a.lap_csr = nullptr;
    a.lap_csr_stride = n >= LAPB_MIN_N && lap_sparse_on() ? (lap_csr_bytes(n) + 255) & ~255LL : 0;
    if (a.lap_csr_stride) HSALLOC(a.lap_csr, S * a.lap_csr_stride);
    e->lds = (size_t)oc_lds_bytes(CAP, MAXD);
    HSALLOC(e->d_off, S + 1);
    YTA_HIP(hipHostMalloc((void **)&e->h_off, sizeof(int) * (S + 1), hipHostMallocDefault));
    YTA_HIP(hipHostMalloc((void **)&e->h_cnt, sizeof(HsCounters) * S, hipHostMallocDefault));
    YTA_HIP(hipFuncSetAttribute((const void *)k_hs_lap, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)LAP_LDS_MAX));
    YTA_HIP(hipFuncSetAttribute((const void *)k_hs_assoc,
                                hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)dense_lap_ws_bytes(OC_LDS_LAP_N)));
    YTA_HIP(hipFuncSetAttribute((const void *)k_hs_assoc_b,
                                hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)dense_lap_ws_bytes(OC_LDS_LAP_N)));
    return YTA_OK;
}

void hs_release(yta_hybridsort *e) {
    for (void *p : e->allocs) (void)hipFree(p);
    e->allocs.clear();
    if (e->h_off) (void)hipHostFree(e->h_off);
    if (e->h_cnt) (void)hipHostFree(e->h_cnt);
    e->h_off = nullptr;
    e->h_cnt = nullptr;
}

int hs_launch(yta_hybridsort *e, const double *d_dets, const int *d_off, const float *d_feat,
              double *out, int *out_counts) {
    HsArgs &a = e->a;
    a.det_in = d_dets;
    a.det_off = d_off;
    a.det_feat = d_feat;
    a.out = out;
    a.out_counts = out_counts;
    {
        const int mrc = e->mask.stage(a.S, e->stream, &a.active);
        if (mrc) return mrc;
    }
    hipLaunchKernelGGL(k_hs_predict, dim3((a.CAP + 63) / 64, a.S), dim3(64), 0, e->stream, a);
    YTA_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_hs_pre, dim3(a.S), dim3(OC_T), 0, e->stream, a);
    YTA_HIP(hipGetLastError());
    const dim3 ge((a.CAP + HE_TILE - 1) / HE_TILE, (a.MAXD + HE_TILE - 1) / HE_TILE, a.S);
    switch (a.asso) {
        case 0: hipLaunchKernelGGL(k_hs_emb<0>, ge, dim3(256), 0, e->stream, a); break;
        case 1: hipLaunchKernelGGL(k_hs_emb<1>, ge, dim3(256), 0, e->stream, a); break;
        case 2: hipLaunchKernelGGL(k_hs_emb<2>, ge, dim3(256), 0, e->stream, a); break;
        case 3: hipLaunchKernelGGL(k_hs_emb<3>, ge, dim3(256), 0, e->stream, a); break;
        default: hipLaunchKernelGGL(k_hs_emb<4>, ge, dim3(256), 0, e->stream, a); break;
    }
    YTA_HIP(hipGetLastError());
    {
        const long long rows = (a.MAXD + OC_T / WAVE - 1) / (OC_T / WAVE);
        const long long rcap = std::max<long long>(4, 4096 / a.S);
        hipLaunchKernelGGL(k_hs_rowpre, dim3((unsigned)std::max<long long>(1, std::min(rows, rcap)), a.S),
                           dim3(OC_T), 0, e->stream, a);
        YTA_HIP(hipGetLastError());
    }
    if (a.arr_chip) {   // the first round's bidding rounds over the chip
        hipLaunchKernelGGL(k_hs_arr0, dim3(a.S), dim3(OC_T), 0, e->stream, a);
        for (int r = 0; r < ARR_CHIP_ROUNDS; ++r) {
            hipLaunchKernelGGL(k_hs_arrscan, dim3(ARR_SCAN_BLOCKS, a.S), dim3(ARR_SCAN_WPB * WAVE), 0,
                               e->stream, a);
            hipLaunchKernelGGL(k_hs_arrapply, dim3(a.S), dim3(OC_T), 0, e->stream, a);
        }
        YTA_HIP(hipGetLastError());
    }
    hipLaunchKernelGGL(k_hs_lap, dim3(a.S), dim3(LAP_T), (size_t)lap_kernel_lds(a.CAP, a.MAXD),
                       e->stream, a);
    YTA_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_hs_upd, dim3((a.MAXD + HS_UPD_T - 1) / HS_UPD_T, a.S), dim3(HS_UPD_T), 0,
                       e->stream, a);
    YTA_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_hs_assoc, dim3(a.S), dim3(OC_T), e->lds, e->stream, a);
    YTA_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_hs_ocr, dim3((unsigned)std::max(4, 2048 / a.S), a.S), dim3(256), 0, e->stream,
                       a);
    YTA_HIP(hipGetLastError());
    {
        const long long rows = (a.MAXD + OC_T / WAVE - 1) / (OC_T / WAVE);
        const long long rcap = std::max<long long>(4, 4096 / a.S);
        hipLaunchKernelGGL(k_hs_ocr_pre, dim3((unsigned)std::max<long long>(1, std::min(rows, rcap)), a.S),
                           dim3(OC_T), 0, e->stream, a);
        YTA_HIP(hipGetLastError());
    }
    hipLaunchKernelGGL(k_hs_assoc_b, dim3(a.S), dim3(OC_T), e->lds, e->stream, a);
    YTA_HIP(hipGetLastError());
    const dim3 gj((a.CAP + a.MAXD + 3) / 4, a.S);
    hipLaunchKernelGGL(k_hs_ema, gj, dim3(256), 0, e->stream, a);
    YTA_HIP(hipGetLastError());
    return YTA_OK;
}

int hs_read_counters(yta_hybridsort *e) {
    YTA_HIP(hipMemcpyAsync(e->h_cnt, e->a.cnt, sizeof(HsCounters) * e->S, hipMemcpyDeviceToHost,
                           e->stream));
    YTA_HIP(host_wait(e->stream));
    return YTA_OK;
}

int hs_check_errors(yta_hybridsort *e) {
    for (int s = 0; s < e->S; ++s) {
        const int err = e->h_cnt[s].err;
        if (err) {
            set_error("stream %d: device error flags 0x%x (%s%s%s%s%s)", s, err,
                      err & ERR_GIOU ? "giou enclosure not positive (iou.py:58 assert) " : "",
                      err & ERR_SOLVER ? "assignment solver failure " : "",
                      err & ERR_TRACK_CAPACITY ? "track capacity exceeded " : "",
                      err & ERR_DET_CAPACITY ? "too many detections " : "",
                      err & ERR_INF_ROW ? "infinite predicted box without NaN " : "");
            return (err & (ERR_TRACK_CAPACITY | ERR_DET_CAPACITY)) ? YTA_ERR_CAPACITY
                   : (err & (ERR_GIOU | ERR_INF_ROW))               ? YTA_ERR_INVALID
                                                                   : YTA_ERR_HIP;
        }
    }
    return YTA_OK;
}

int hs_reserve(yta_hybridsort *e, int cap, int maxd) {
    if (cap <= e->CAP && maxd <= e->MAXD) return YTA_OK;
    cap = std::max(cap, e->CAP);
    maxd = std::max(maxd, e->MAXD);
    YTA_HIP(host_wait(e->stream));
    yta_hybridsort *n = new (std::nothrow) yta_hybridsort();
    YTA_CHECK(n, YTA_ERR_NOMEM, "out of host memory");
    n->device = e->device;
    n->S = e->S;
    n->CAP = cap;
    n->MAXD = maxd;
    n->D = e->D;
    n->prm = e->prm;
    n->stream = e->stream;
    int rc = hs_alloc(n);
    const size_t S = e->S, oc = e->CAP, nc = cap, Dd = e->D;
    auto copy2d = [&](void *dst, size_t dp, const void *src, size_t sp, size_t w) -> int {
        YTA_HIP(hipMemcpy2DAsync(dst, dp, src, sp, w, S, hipMemcpyDeviceToDevice, e->stream));
        return YTA_OK;
    };
    if (!rc) rc = copy2d(n->a.rec, nc * sizeof(HsTrack), e->a.rec, oc * sizeof(HsTrack),
                         oc * sizeof(HsTrack));
    if (!rc) rc = copy2d(n->a.feat, nc * Dd * 4, e->a.feat, oc * Dd * 4, oc * Dd * 4);
    if (!rc) rc = copy2d(n->a.list, nc * 4, e->a.list, oc * 4, oc * 4);
    if (!rc) {
        std::vector<int> fl(nc * S), old(oc * S);
        std::vector<HsCounters> cnt(S);
        hipError_t he = hipMemcpyAsync(old.data(), e->a.free_list, sizeof(int) * oc * S,
                                       hipMemcpyDeviceToHost, e->stream);
        if (he == hipSuccess)
            he = hipMemcpyAsync(cnt.data(), e->a.cnt, sizeof(HsCounters) * S,
                                hipMemcpyDeviceToHost, e->stream);
        if (he == hipSuccess) he = host_wait(e->stream);
        if (he == hipSuccess) {
            for (size_t s = 0; s < S; ++s) {
                int k = 0;
                for (int q = (int)nc - 1; q >= (int)oc; --q) fl[s * nc + k++] = q;
                for (int q = 0; q < cnt[s].n_free; ++q) fl[s * nc + k++] = old[s * oc + q];
                cnt[s].n_free = k;
            }
            he = hipMemcpy(n->a.free_list, fl.data(), sizeof(int) * nc * S, hipMemcpyHostToDevice);
            if (he == hipSuccess)
                he = hipMemcpy(n->a.cnt, cnt.data(), sizeof(HsCounters) * S,
                               hipMemcpyHostToDevice);
        }
        if (he != hipSuccess) {
            set_error("reserve: %s", hipGetErrorString(he));
            rc = YTA_ERR_HIP;
        }
    }
    if (rc) {
        n->stream = nullptr;
        hs_release(n);
        delete n;
        return rc;
    }
    memcpy(n->h_cnt, e->h_cnt, sizeof(HsCounters) * S);
    hs_release(e);
    e->CAP = n->CAP;
    e->MAXD = n->MAXD;
    e->allocs.swap(n->allocs);
    e->a = n->a;
    e->lds = n->lds;
    e->h_off = n->h_off;
    e->h_cnt = n->h_cnt;
    e->d_off = n->d_off;
    n->h_off = nullptr;
    n->h_cnt = nullptr;
    n->stream = nullptr;
    delete n;
    return YTA_OK;
}

}  // namespace

extern "C" {

int yta_hybridsort_create(int device, int n_streams, int track_capacity, int max_dets,
                          int feat_dim, const yta_hybridsort_params *params,
                          yta_hybridsort **engine) {
    YTA_CHECK(engine && params, YTA_ERR_INVALID, "null engine/params");
    YTA_CHECK(n_streams > 0 && track_capacity > 0 && max_dets > 0, YTA_ERR_INVALID,
              "n_streams, track_capacity and max_dets must be positive");
    YTA_CHECK(params->delta_t >= 0 && params->delta_t <= OC_DT_MAX, YTA_ERR_INVALID,
              "delta_t must be in [0, %d]", OC_DT_MAX);
    YTA_CHECK(params->asso_func >= 0 && params->asso_func <= 3, YTA_ERR_INVALID,
              "asso_func must be 0..3 (iou, giou, diou, ciou): HybridSORT calls it without the "
              "image size centroid needs (hybridsort.py:516)");
    YTA_CHECK(feat_dim > 0, YTA_ERR_INVALID, "HybridSORT needs embeddings (feat_dim > 0)");
    *engine = nullptr;
    int rc = select_device(device);
    if (rc) return rc;
    yta_hybridsort *e = new (std::nothrow) yta_hybridsort();
    YTA_CHECK(e, YTA_ERR_NOMEM, "out of host memory");
    e->device = device;
    e->S = n_streams;
    e->CAP = track_capacity;
    e->MAXD = max_dets;
    e->D = feat_dim;
    e->prm = *params;
    hipError_t he = hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking);
    if (he != hipSuccess) {
        set_error("hipStreamCreate: %s", hipGetErrorString(he));
        delete e;
        return YTA_ERR_HIP;
    }
    rc = hs_alloc(e);
    if (!rc) rc = yta_hybridsort_reset(e);
    if (rc) {
        yta_hybridsort_destroy(e);
        return rc;
    }
    *engine = e;
    return YTA_OK;
}

int yta_hybridsort_destroy(yta_hybridsort *e) {
    if (!e) return YTA_OK;
    (void)hipSetDevice(e->device);
    if (e->stream) (void)host_wait(e->stream);
    hs_release(e);
    e->mask.release();
    if (e->h_dets) (void)hipHostFree(e->h_dets);
    if (e->d_det_in) (void)hipFree(e->d_det_in);
    if (e->h_feat) (void)hipHostFree(e->h_feat);
    if (e->d_feat) (void)hipFree(e->d_feat);
    if (e->stream) (void)hipStreamDestroy(e->stream);
    delete e;
    return YTA_OK;
}

int yta_hybridsort_reset(yta_hybridsort *e) {
    YTA_CHECK(e, YTA_ERR_INVALID, "null engine");
    YTA_HIP(hipSetDevice(e->device));
    hipLaunchKernelGGL(k_hs_reset, dim3(e->S), dim3(256), 0, e->stream, e->a, 0);
    YTA_HIP(hipGetLastError());
    YTA_HIP(host_wait(e->stream));
    memset(e->h_cnt, 0, sizeof(HsCounters) * e->S);
    return YTA_OK;
}

int yta_hybridsort_capacity(yta_hybridsort *e, int *track_capacity, int *max_dets) {
    YTA_CHECK(e && track_capacity && max_dets, YTA_ERR_INVALID, "null argument");
    *track_capacity = e->CAP;
    *max_dets = e->MAXD;
    return YTA_OK;
}

int yta_hybridsort_update(yta_hybridsort *e, const double *dets, const int *det_offsets,
                          const float *feats, long long *next_id, double *out, int out_capacity,
                          int *out_offsets) {
    YTA_CHECK(e && det_offsets && out_offsets, YTA_ERR_INVALID, "null argument");
    YTA_HIP(hipSetDevice(e->device));
    const int S = e->S;
    YTA_CHECK(det_offsets[0] == 0, YTA_ERR_INVALID, "det_offsets[0] must be 0");
    int need_d = e->MAXD, need_c = e->CAP;
    for (int s = 0; s < S; ++s) {
        const int m = det_offsets[s + 1] - det_offsets[s];
        YTA_CHECK(m >= 0, YTA_ERR_INVALID, "det_offsets must be non-decreasing");
        need_d = std::max(need_d, m);
        need_c = std::max(need_c, e->h_cnt[s].n_trk + m);
    }
    // every output row is a track matched to or born from one of this frame's detections, so
    // det_offsets[S] rows always suffice; checked before anything moves (the frame is not consumed)
    YTA_CHECK(out_capacity >= det_offsets[S], YTA_ERR_CAPACITY,
              "out holds %d rows, the call needs det_offsets[S] = %d", out_capacity, det_offsets[S]);
    if (need_d > e->MAXD || need_c > e->CAP) {
        const int rc = hs_reserve(e, need_c > e->CAP ? std::max(need_c, 2 * e->CAP) : e->CAP,
                                  need_d > e->MAXD ? std::max(need_d, 2 * e->MAXD) : e->MAXD);
        if (rc) return rc;
    }
    const long long total = det_offsets[S];
    YTA_CHECK(total == 0 || (dets && feats), YTA_ERR_INVALID, "null dets / feats");
    const int D = e->D;
    if (total > e->det_cap) {
        if (e->d_det_in) (void)hipFree(e->d_det_in);
        if (e->h_dets) (void)hipHostFree(e->h_dets);
        if (e->d_feat) (void)hipFree(e->d_feat);
        if (e->h_feat) (void)hipHostFree(e->h_feat);
        e->d_det_in = nullptr;
        e->h_dets = nullptr;
        e->d_feat = nullptr;
        e->h_feat = nullptr;
        e->det_cap = 0;
        const long long cap = std::max<long long>(2 * total, 1024);
        YTA_HIP(hipMalloc((void **)&e->d_det_in, sizeof(double) * 6 * cap));
        YTA_HIP(hipHostMalloc((void **)&e->h_dets, sizeof(double) * 6 * cap, hipHostMallocDefault));
        YTA_HIP(hipMalloc((void **)&e->d_feat, sizeof(float) * D * cap));
        YTA_HIP(hipHostMalloc((void **)&e->h_feat, sizeof(float) * D * cap, hipHostMallocDefault));
        e->det_cap = cap;
    }
    if (total) {
        memcpy(e->h_dets, dets, sizeof(double) * 6 * total);
        YTA_HIP(hipMemcpyAsync(e->d_det_in, e->h_dets, sizeof(double) * 6 * total,
                               hipMemcpyHostToDevice, e->stream));
        memcpy(e->h_feat, feats, sizeof(float) * D * total);
        YTA_HIP(hipMemcpyAsync(e->d_feat, e->h_feat, sizeof(float) * D * total,
                               hipMemcpyHostToDevice, e->stream));
    }
    memcpy(e->h_off, det_offsets, sizeof(int) * (S + 1));
    YTA_HIP(hipMemcpyAsync(e->d_off, e->h_off, sizeof(int) * (S + 1), hipMemcpyHostToDevice,
                           e->stream));
    if (next_id) {
        for (int s = 0; s < S; ++s) e->h_cnt[s].next_id = next_id[s];
        YTA_HIP(hipMemcpy2DAsync(&e->a.cnt[0].next_id, sizeof(HsCounters), &e->h_cnt[0].next_id,
                                 sizeof(HsCounters), sizeof(long long), S, hipMemcpyHostToDevice,
                                 e->stream));
    }
    int rc = hs_launch(e, e->d_det_in, e->d_off, e->d_feat, e->a.out, nullptr);
    if (rc) return rc;
    rc = hs_read_counters(e);
    if (rc) return rc;
    if (next_id)   // the device counters have advanced: hand them back even on an error below
        for (int s = 0; s < S; ++s) next_id[s] = e->h_cnt[s].next_id;
    rc = hs_check_errors(e);
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
    for (int s = 0; s < S; ++s) {
        const int n = e->h_cnt[s].n_out;
        if (n)
            YTA_HIP(hipMemcpyAsync(out + (long long)out_offsets[s] * 8,
                                   e->a.out + (long long)s * e->CAP * 8, sizeof(double) * 8 * n,
                                   hipMemcpyDeviceToHost, e->stream));
    }
    YTA_HIP(host_wait(e->stream));
    return YTA_OK;
}

int yta_hybridsort_update_device(yta_hybridsort *e, const double *d_dets, const int *d_det_offsets,
                                 const float *d_feats, double *d_out, int *d_out_counts) {
    YTA_CHECK(e && d_det_offsets && d_out && d_feats, YTA_ERR_INVALID, "null argument");
    return hs_launch(e, d_dets, d_det_offsets, d_feats, d_out, d_out_counts);
}

int yta_hybridsort_sync(yta_hybridsort *e) {
    YTA_CHECK(e, YTA_ERR_INVALID, "null engine");
    const int rc = hs_read_counters(e);
    if (rc) return rc;
    return hs_check_errors(e);
}

int yta_hybridsort_get_state(yta_hybridsort *e, int stream, int *n_tracks, long long *ints,
                             double *dbl, double *x, double *P, float *feat) {
    YTA_CHECK(e && n_tracks && ints && dbl && x && P, YTA_ERR_INVALID, "null argument");
    YTA_CHECK(stream >= 0 && stream < e->S, YTA_ERR_INVALID, "bad stream %d", stream);
    YTA_HIP(hipSetDevice(e->device));
    const int rc = hs_read_counters(e);
    if (rc) return rc;
    const HsCounters c = e->h_cnt[stream];
    const long long tb = (long long)stream * e->CAP;
    std::vector<int> lst(c.n_trk);
    std::vector<HsTrack> rec(e->CAP);
    if (c.n_trk)
        YTA_HIP(hipMemcpy(lst.data(), e->a.list + tb, sizeof(int) * c.n_trk, hipMemcpyDeviceToHost));
    YTA_HIP(hipMemcpy(rec.data(), e->a.rec + tb, sizeof(HsTrack) * e->CAP, hipMemcpyDeviceToHost));
    for (int i = 0; i < c.n_trk; ++i) {
        const HsTrack &r = rec[lst[i]];
        long long *ii = ints + 6LL * i;
        ii[0] = r.id;
        ii[1] = r.age;
        ii[2] = r.hits;
        ii[3] = r.hit_streak;
        ii[4] = r.tsu;
        ii[5] = (r.flags & OF_OBSERVED) ? 1 : 0;
        double *dd = dbl + 3LL * i;
        dd[0] = r.conf;
        dd[1] = r.cls;
        dd[2] = r.det_ind;
        for (int k = 0; k < 9; ++k) x[9LL * i + k] = r.kf.x[k];
        double *M = P + 81LL * i;
        for (int k = 0; k < 81; ++k) M[k] = 0.0;
        for (int g = 0; g < 4; ++g) {
            M[g * 9 + g] = r.kf.p[4 * g];
            M[g * 9 + g + 5] = r.kf.p[4 * g + 1];
            M[(g + 5) * 9 + g] = r.kf.p[4 * g + 2];
            M[(g + 5) * 9 + g + 5] = r.kf.p[4 * g + 3];
        }
        M[4 * 9 + 4] = r.kf.p[16];
        if (feat)
            YTA_HIP(hipMemcpy(feat + (long long)i * e->D, e->a.feat + (tb + lst[i]) * e->D,
                              sizeof(float) * e->D, hipMemcpyDeviceToHost));
    }
    *n_tracks = c.n_trk;
    return YTA_OK;
}

int yta_hybridsort_classes(yta_hybridsort *e, int stream, double *cls, int cap, int *n) {
    YTA_CHECK(e && n && (cls || cap == 0), YTA_ERR_INVALID, "null argument");
    YTA_CHECK(stream >= 0 && stream < e->S, YTA_ERR_INVALID, "bad stream %d", stream);
    YTA_HIP(hipSetDevice(e->device));
    const int rc = hs_read_counters(e);
    if (rc) return rc;
    const int nt = e->h_cnt[stream].n_trk;
    YTA_CHECK(nt <= cap, YTA_ERR_CAPACITY, "%d trackers > capacity %d", nt, cap);
    const long long tb = (long long)stream * e->CAP;
    std::vector<int> lst(nt);
    if (nt)
        YTA_HIP(hipMemcpy(lst.data(), e->a.list + tb, sizeof(int) * nt, hipMemcpyDeviceToHost));
    for (int i = 0; i < nt; ++i)
        YTA_HIP(hipMemcpy(cls + i, (const char *)(e->a.rec + tb + lst[i]) + offsetof(HsTrack, cls),
                          sizeof(double), hipMemcpyDeviceToHost));
    *n = nt;
    return YTA_OK;
}

int yta_hybridsort_stats(yta_hybridsort *e, long long *stats) {
    YTA_CHECK(e && stats, YTA_ERR_INVALID, "null argument");
    const int rc = hs_read_counters(e);
    if (rc) return rc;
    for (int k = 0; k < 8; ++k) stats[k] = 0;
    for (int s = 0; s < e->S; ++s) {
        const HsCounters &c = e->h_cnt[s];
        const long long v[8] = {c.n_dets, c.n_high, c.n_trk, c.n_out, c.n_births, c.lap_calls,
                                c.corrections, c.n_ema};
        for (int k = 0; k < 8; ++k) stats[k] += v[k];
    }
    return YTA_OK;
}

int yta_kf9_run(int device, int n, int steps, const double *b0, const double *b, double *x_out,
                double *P_out) {
    YTA_CHECK(n > 0 && steps >= 0 && b0 && (b || steps == 0) && x_out && P_out, YTA_ERR_INVALID,
              "bad arguments");
    int rc = select_device(device);
    if (rc) return rc;
    double *d_b0 = nullptr, *d_b = nullptr, *d_x = nullptr, *d_P = nullptr;
    const size_t nb = sizeof(double) * 5 * (size_t)n * std::max(steps, 1);
    hipError_t he = hipMalloc((void **)&d_b0, sizeof(double) * 5 * n);
    if (he == hipSuccess) he = hipMalloc((void **)&d_b, nb);
    if (he == hipSuccess) he = hipMalloc((void **)&d_x, sizeof(double) * 9 * n);
    if (he == hipSuccess) he = hipMalloc((void **)&d_P, sizeof(double) * 81 * n);
    if (he == hipSuccess) he = hipMemcpy(d_b0, b0, sizeof(double) * 5 * n, hipMemcpyHostToDevice);
    if (he == hipSuccess && steps)
        he = hipMemcpy(d_b, b, sizeof(double) * 5 * (size_t)n * steps, hipMemcpyHostToDevice);
    if (he == hipSuccess) {
        hipLaunchKernelGGL(k_kf9_run, dim3((n + 63) / 64), dim3(64), 0, 0, n, steps, d_b0, d_b,
                           d_x, d_P);
        he = hipGetLastError();
    }
    if (he == hipSuccess) he = hipMemcpy(x_out, d_x, sizeof(double) * 9 * n, hipMemcpyDeviceToHost);
    if (he == hipSuccess) he = hipMemcpy(P_out, d_P, sizeof(double) * 81 * n, hipMemcpyDeviceToHost);
    (void)hipFree(d_b0);
    (void)hipFree(d_b);
    (void)hipFree(d_x);
    (void)hipFree(d_P);
    if (he != hipSuccess) {
        set_error("yta_kf9_run: %s", hipGetErrorString(he));
        return YTA_ERR_HIP;
    }
    return YTA_OK;
}

int yta_hybridsort_lap_stats(yta_hybridsort *e, long long *stats, int n) {
    YTA_CHECK(e && (stats || n <= 0), YTA_ERR_INVALID, "null argument");
    const int rc = hs_read_counters(e);
    if (rc) return rc;
    long long v[YTA_LAP_STATS] = {};
    for (int s = 0; s < e->S; ++s) {
        const LapStats &l = e->h_cnt[s].ls;
        v[0] += l.transposed;
        v[1] += l.uncertified;
        v[2] += l.replays;
        v[3] += l.reduced;
    }
    for (int k = 0; k < n && k < YTA_LAP_STATS; ++k) stats[k] = v[k];
    return YTA_OK;
}

int yta_hybridsort_hip_stream(yta_hybridsort *e, void **stream) {
    YTA_CHECK(e && stream, YTA_ERR_INVALID, "null argument");
    *stream = (void *)e->stream;
    return YTA_OK;
}

#ifdef YTA_STAMPS
int yta_hybridsort_debug_stamps(unsigned long long *out) {
    YTA_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * 128));
    return YTA_OK;
}
#endif

#ifdef YTA_STAMPS
// diagnostic build only: this file's stamps (k_hs_lap's rectangular solver phases)
int yta_hs_debug_stamps(unsigned long long *out) {
    YTA_HIP(hipDeviceSynchronize());
    YTA_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), 128 * sizeof(unsigned long long)));
    return YTA_OK;
}
int yta_hs_debug_stamps_reset() {
    unsigned long long z[128] = {};
    YTA_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), z, sizeof(z)));
    return YTA_OK;
}
#endif


// ---- stream subsets (subset.hpp): the listed streams updated, every other stream untouched
int yta_hybridsort_reset_stream(yta_hybridsort *e, int stream) {
    YTA_CHECK(e, YTA_ERR_INVALID, "null engine");
    YTA_CHECK(stream >= 0 && stream < e->S, YTA_ERR_INVALID, "stream %d outside 0..%d", stream,
              e->S - 1);
    YTA_HIP(hipSetDevice(e->device));
    hipLaunchKernelGGL(k_hs_reset, dim3(1), dim3(256), 0, e->stream, e->a, stream);
    YTA_HIP(hipGetLastError());
    YTA_HIP(host_wait(e->stream));
    return hs_read_counters(e);
}

int yta_hybridsort_update_device_masked(yta_hybridsort *e, const int *d_active, const double *d_dets, const int *d_det_offsets, const float *d_feats, double *d_out, int *d_out_counts) {
    YTA_CHECK(e, YTA_ERR_INVALID, "null engine");
    e->mask.req_dev = d_active;
    const int rc = yta_hybridsort_update_device(e, d_dets, d_det_offsets, d_feats, d_out, d_out_counts);
    e->mask.req_dev = nullptr;
    return rc;
}

int yta_hybridsort_update_streams(yta_hybridsort *e, int n_streams, const int *stream_ids, const double *dets, const int *det_offsets, const float *feats,
                           long long *next_id, double *out, int out_capacity, int *out_offsets) {
    YTA_CHECK(e && out_offsets, YTA_ERR_INVALID, "null argument");
    YTA_HIP(hipSetDevice(e->device));
    const int S = e->S;
    std::vector<int> mask, off, full_oo(S + 1, 0);
    int rc = subset_expand(S, n_streams, stream_ids, det_offsets, mask, off);
    if (rc) return rc;
    std::vector<long long> nid(S);
    if (next_id) {   // the skipped streams keep their device counters: read them first
        rc = hs_read_counters(e);
        if (rc) return rc;
        for (int s = 0; s < S; ++s) nid[s] = e->h_cnt[s].next_id;
        for (int k = 0; k < n_streams; ++k) nid[stream_ids[k]] = next_id[k];
    }

    e->mask.req_host = mask.data();
    rc = yta_hybridsort_update(e, dets, off.data(), feats, next_id ? nid.data() : nullptr, out,
                        out_capacity, full_oo.data());
    e->mask.req_host = nullptr;
    if (next_id)
        for (int k = 0; k < n_streams; ++k) next_id[k] = nid[stream_ids[k]];
    if (rc) return rc;
    subset_compact(n_streams, stream_ids, full_oo, out_offsets);
    return YTA_OK;
}

}  // extern "C"
