// DeepOCSORT update() for S independent streams on gfx950, all tracker state resident in HBM.
//
// Follows boxmot/trackers/deepocsort/deep_ocsort.py:357-520 (new-KF branch, the only live one)
// with the embedding-aware association of boxmot/utils/association.py:79-201.  One frame =
//   k_doc_predict [grid]         CMC correction of every tracker (:250-267, last observation,
//                                observations within delta_t ages, Kalman state and its frozen
//                                copy), predict (:269-293), column inputs; one thread per tracker
//   k_doc_pre    [block/stream]  NaN cull (compacts the column inputs when a tracker goes),
//                                confidence split, embedding weights
//                                alpha = af + (1 - af)(1 - trust) (:395-398)
//   k_doc_cost   [grid]          dense asso (dets x trackers) and iou + angle (association.py:
//                                111-170), per-row / per-column counts for the fast path
//   k_doc_emb    [grid]          stage-1 embedding cost dets_embs @ trk_embs^T (float64 MFMA tiles)
//   k_doc_aw     [grid]          emb[iou <= 0] = 0, per-row / per-column top-2 weights
//                                (compute_aw_max_metric :79-108) or the flat weight (aw_off)
//   k_doc_final  [grid]          cost = -(iou + angle + w_r w_c w emb)
//   k_doc_assoc  [block/stream]  fast path or padded LAP, filtered matches, OCR round on the last
//                                observations (:470-493), tracker updates (Kalman + ORU replay),
//                                births, outputs in reversed tracker order, removal
//   k_doc_ema    [grid]          update_emb of every matched tracker (:243-245), embeddings of births
#include <algorithm>
#include <cstring>
#include <new>
#include <vector>

#include "aw.hpp"
#include "kf_deep.hpp"
#include "kf_ocsort.hpp"
#include "ocsort_common.hpp"
#include "subset.hpp"

namespace yta {
namespace {

constexpr int OF_FROZEN = 8;        // KalmanBoxTracker.frozen
constexpr int DOC_RING = OC_DT_MAX + 1;   // observations of ages age - delta_t .. age

struct DocTrack {
    Kf8 kf;
    Kf8 fz;                         // frozen filter (attr_saved x / P)
    double lm[4];                   // attr_saved last_measurement
    double hist_z[4];               // the filter's last measurement (history_obs[-1] when observed)
    double last_obs[5];
    double vel[2];
    double conf, cls;
    double obs[DOC_RING][5];
    long long id;
    int obs_age[DOC_RING];
    int obs_n;
    int det_ind, age, hits, hit_streak, tsu, flags, hist_since;
};

struct DocCounters {
    long long next_id;
    unsigned long long ocr_max;    // k_doc_ocr -> k_doc_assoc_b: the OCR matrix's maximum (hs_ord)
    int n_trk, n_free;
    int n_dets, n_high, n_out, n_births;
    int lap_calls, fast_path;
    int n_ema;
    int err;
    int lap_done;                  // first round solved by k_doc_lap this frame
    int n_ud, n_upd;               // k_doc_assoc -> k_doc_finish: unmatched detections, updates
    LapStats ls;                   // cumulative solver counters
    int frame;
    int n_ut;                      // k_doc_assoc -> k_doc_ocr -> k_doc_assoc_b: OCR round columns
    int ocr_nan;                   // the OCR matrix holds a NaN (its max is then NaN)
    int n_pos;                     // k_doc_cost -> k_doc_emb*: some row has more than POS_K pairs
                                   // whose asso value is not <= 0 (the dense tiles run)
    int col_ovf;                   // k_doc_emb_pairs -> k_doc_aw*: a column listed more than POS_K
    int pad[6];
};
static_assert(sizeof(DocCounters) == 128, "DocCounters layout");

constexpr int POS_K = 16;   // listed embedding pairs per detection row (k_doc_cost)

struct DocArgs {
    int S, CAP, MAXD, D;
    double det_thresh, thr, inertia, w_emb, af, aw_param;
    int max_age, min_hits, delta_t, asso, embedding_off, cmc_off, aw_off;
    const double *det_in;
    const int *det_off;
    const int *img_wh;              // S x (w, h) or null
    const double *warp;             // S x 6 or null (identity)
    const float *det_feat;          // [rows of det_in][D]
    DocTrack *rec;                  // [S*CAP]
    double *emb;                    // [S*CAP][D] tracker embeddings (float64)
    int *list, *free_list;          // [S*CAP]
    DocCounters *cnt;
    // per frame
    int *hi_row;                    // [S*MAXD]
    double *alpha;                  // [S*MAXD] embedding weight of each kept detection
    Box *cbox;                      // [S*CAP]
    double *cvel, *ckobs, *clast;   // [S*CAP] x 2 / 5 / 5
    int *nan_flag, *cslot;          // [S*CAP]
    double *mat, *mat2, *emat;      // [S*MAXD*CAP]: asso, cost, embedding cost
    double *rw, *cw;                // [S*MAXD], [S*CAP] AW weights
    double *cw_part;                // [S*AW_CHUNKS*CAP*2] per-row-chunk column top-2
    int *rmatch, *cmatched;
    int *udet, *utrk, *tmp;         // [S*(MAXD+CAP)]
    int *upd;                       // [S*CAP] update source per tracker (input row) or -1
    int *ema_slot, *ema_row;        // [S*(CAP+MAXD)] embedding jobs: slot, input row (birth: ~row)
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
    int *pos_q;                    // [S*MAXD*POS_K] per kept detection: trackers whose pair's
    int *pos_cnt;                  // embedding term is used; [S*MAXD] their count
    double *col_e;                 // [S*CAP*POS_K] per tracker: its listed pairs' embedding terms
    int *col_cnt;                  // [S*CAP] their count
    int force_dense;               // YTA_DOC_DENSE=1: every frame on the dense tiles / AW scans
                                   // (tests/test_gpu_deepocsort.py compares both paths)
};

__device__ __forceinline__ long long doc_mb(const DocArgs &a, int s) {
    return (long long)s * (a.MAXD > 4 ? a.MAXD : 4) * a.CAP;
}

// affine of a box's two corners (deep_ocsort.py:253-256): ps = b[:4].reshape(2, 2).T, m ps + t
__device__ __forceinline__ void doc_affine_box(double *b, const double *m, const double *t) {
    const double x1 = b[0], y1 = b[1], x2 = b[2], y2 = b[3];
    b[0] = (m[0] * x1 + m[1] * y1) + t[0];
    b[1] = (m[2] * x1 + m[3] * y1) + t[1];
    b[2] = (m[0] * x2 + m[1] * y2) + t[0];
    b[3] = (m[2] * x2 + m[3] * y2) + t[1];
}

// KalmanBoxTracker.apply_affine_correction (deep_ocsort.py:250-267).  last_observation is the
// same array as the newest stored observation (update() assigns both), so when that one is in
// the delta_t window it is corrected twice.
__device__ void doc_apply_affine(DocTrack &r, const double *aff, int dt) {
    const double m[4] = {aff[0], aff[1], aff[3], aff[4]};
    const double t[2] = {aff[2], aff[5]};
    const bool lo_pos = np_sum5(r.last_obs) > 0;
    if (lo_pos) doc_affine_box(r.last_obs, m, t);
    const int nring = r.obs_n < DOC_RING ? r.obs_n : DOC_RING;
    const int newest = r.obs_n > 0 ? (r.obs_n - 1) % DOC_RING : -1;
    for (int e = 0; e < nring; ++e) {
        if (r.obs_age[e] < r.age - dt || r.obs_age[e] > r.age) continue;
        if (e == newest) {
            // the shared array: its current value is last_obs (already corrected if sum > 0)
            doc_affine_box(r.last_obs, m, t);
            for (int k = 0; k < 4; ++k) r.obs[e][k] = r.last_obs[k];
        } else {
            doc_affine_box(r.obs[e], m, t);
        }
    }
    if (newest >= 0 && !(r.obs_age[newest] >= r.age - dt && r.obs_age[newest] <= r.age) && lo_pos)
        for (int k = 0; k < 4; ++k) r.obs[newest][k] = r.last_obs[k];
    kf8_affine(r.kf, m, t);
    if (!(r.flags & OF_OBSERVED) && (r.flags & OF_SAVED)) {   // the frozen copy too (:398-405)
        kf8_affine(r.fz, m, t);
        const double a0 = r.lm[0], a1 = r.lm[1], b0 = r.lm[2], b1 = r.lm[3];
        r.lm[0] = (m[0] * a0 + m[1] * a1) + t[0];
        r.lm[1] = (m[2] * a0 + m[3] * a1) + t[1];
        r.lm[2] = m[0] * b0 + m[1] * b1;
        r.lm[3] = m[2] * b0 + m[3] * b1;
    }
}

__device__ __forceinline__ void doc_x_to_bbox(const double *x, double *b) {   // :50-52
    b[0] = x[0] - x[2] / 2;
    b[1] = x[1] - x[3] / 2;
    b[2] = x[0] + x[2] / 2;
    b[3] = x[1] + x[3] / 2;
}

// k_previous_obs (deep_ocsort.py:16-24) from the ring
__device__ __forceinline__ void doc_prev_obs(const DocTrack &r, int dt, double *o) {
    if (r.obs_n == 0) {
        for (int k = 0; k < 5; ++k) o[k] = -1.0;
        return;
    }
    const int m = r.obs_n < DOC_RING ? r.obs_n : DOC_RING;
    for (int i = 0; i < dt; ++i) {
        const int want = r.age - (dt - i);
        for (int e = 0; e < m; ++e)
            if (r.obs_age[e] == want) {
                for (int k = 0; k < 5; ++k) o[k] = r.obs[e][k];
                return;
            }
    }
    for (int k = 0; k < 5; ++k) o[k] = r.last_obs[k];
}

// KalmanBoxTracker.update (deep_ocsort.py:198-241) + KalmanFilterNew.update (deepocsort_kf.py)
__device__ void doc_update(DocTrack &r, const double *det, int det_local, int dt) {
    if (!det) {
        if (r.flags & OF_OBSERVED) {          // freeze: last_measurement = history_obs[-2]
            r.fz = r.kf;
            for (int k = 0; k < 4; ++k) r.lm[k] = r.hist_z[k];
            r.flags |= OF_SAVED;
        }
        r.flags &= ~OF_OBSERVED;
        r.flags |= OF_FROZEN;
        r.hist_since += 1;
        return;
    }
    const double bbox[5] = {det[0], det[1], det[2], det[3], det[4]};
    r.conf = det[4];
    r.cls = det[5];
    r.det_ind = det_local;
    r.flags &= ~OF_FROZEN;
    if (np_sum5(r.last_obs) >= 0) {
        const double *prev = r.last_obs;
        const int m = r.obs_n < DOC_RING ? r.obs_n : DOC_RING;
        bool found = false;
        for (int dd = dt; dd >= 1 && !found; --dd) {
            const int want = r.age - dd;
            for (int e = 0; e < m; ++e)
                if (r.obs_age[e] == want) {
                    prev = r.obs[e];
                    found = true;
                    break;
                }
        }
        const double cx1 = (prev[0] + prev[2]) / 2.0, cy1 = (prev[1] + prev[3]) / 2.0;
        const double cx2 = (bbox[0] + bbox[2]) / 2.0, cy2 = (bbox[1] + bbox[3]) / 2.0;
        const double sy = cy2 - cy1, sx = cx2 - cx1;
        const double nrm = sqrt(sy * sy + sx * sx) + 1e-6;
        r.vel[0] = sy / nrm;
        r.vel[1] = sx / nrm;
        r.flags |= OF_VELOCITY;
    }
    for (int k = 0; k < 5; ++k) r.last_obs[k] = bbox[k];
    const int slot = r.obs_n % DOC_RING;
    for (int k = 0; k < 5; ++k) r.obs[slot][k] = bbox[k];
    r.obs_age[slot] = r.age;
    r.obs_n += 1;
    r.tsu = 0;
    r.hits += 1;
    r.hit_streak += 1;
    // R from the predicted w, h (deep_ocsort.py:236-237)
    const double rw = DK_P * r.kf.x[2], rh = DK_P * r.kf.x[3];
    const double rd[4] = {rw * rw, rh * rh, rw * rw, rh * rh};
    const double w = bbox[2] - bbox[0], h = bbox[3] - bbox[1];
    const double z[4] = {bbox[0] + w / 2.0, bbox[1] + h / 2.0, w, h};
    if (!(r.flags & OF_OBSERVED) && (r.flags & OF_SAVED)) {
        r.kf = r.fz;
        r.flags &= ~OF_SAVED;
        kf8_replay(r.kf, r.lm, z, r.hist_since + 1, r.hist_z);
    } else {
        for (int k = 0; k < 4; ++k) r.hist_z[k] = z[k];
    }
    r.hist_since = 0;
    r.flags |= OF_OBSERVED;
    kf8_correct(r.kf, z, rd);
}

// KalmanBoxTracker.predict (deep_ocsort.py:269-293): velocity clamps, Q(w, h) from the current
// state, age / streak bookkeeping
__device__ void doc_predict(DocTrack &r) {
    if (r.kf.x[2] + r.kf.x[6] <= 0) r.kf.x[6] = 0;
    if (r.kf.x[3] + r.kf.x[7] <= 0) r.kf.x[7] = 0;
    if (r.flags & OF_FROZEN) r.kf.x[6] = r.kf.x[7] = 0;
    double qd[8];
    for (int k = 0; k < 8; ++k) qd[k] = dk_q(k, r.kf.x[2], r.kf.x[3]);
    kf8_predict(r.kf, qd);
    r.age += 1;
    if (r.tsu > 0) r.hit_streak = 0;
    r.tsu += 1;
}

// KalmanBoxTracker.__init__ (deep_ocsort.py:103-196, new KF)
__device__ void doc_birth(DocTrack &out, const double *dr, long long id, int det_ind) {
    DocTrack r;
    const double w = dr[2] - dr[0], h = dr[3] - dr[1];
    const double z[4] = {dr[0] + w / 2.0, dr[1] + h / 2.0, w, h};
    kf8_init(z, r.kf);
    r.fz = r.kf;
    for (int k = 0; k < 4; ++k) r.lm[k] = r.hist_z[k] = 0.0;
    for (int k = 0; k < 5; ++k) r.last_obs[k] = -1.0;
    r.vel[0] = r.vel[1] = 0.0;
    r.conf = dr[4];
    r.cls = dr[5];
    r.id = id;
    r.obs_n = 0;
    for (int e = 0; e < DOC_RING; ++e) r.obs_age[e] = -1;
    r.det_ind = det_ind;
    r.age = r.hits = r.hit_streak = r.tsu = 0;
    r.flags = 0;
    r.hist_since = 0;
    out = r;
}

// CMC (deep_ocsort.py:385-389), then predict (:269-293) of every tracker, chip-wide; k_doc_pre
// compacts the survivors per stream.
// Per-tracker kernels (predict, Kalman updates) run one wave per block: a frame's trackers spread
// over 4x the CUs of 256-thread blocks (k_hs_upd's A/B: profiles/r03zi_ab_hs_upd_wave_blocks.txt).
constexpr int DOC_TRK_T = 64;
__global__ __launch_bounds__(DOC_TRK_T) void k_doc_predict(DocArgs a) {
    const int s = blockIdx.y;
    if (a.active && !a.active[s]) return;   // stream not updated this frame
    const DocCounters *c = a.cnt + s;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= c->n_trk) return;
    const long long tb = (long long)s * a.CAP;
    const double *aff = a.warp ? a.warp + 6LL * s : nullptr;
    DocTrack &r = a.rec[tb + a.list[tb + i]];
    if (!a.cmc_off && aff) doc_apply_affine(r, aff, a.delta_t);   // identity when no warp is given
    doc_predict(r);
    double b[4];
    doc_x_to_bbox(r.kf.x, b);
    a.nan_flag[tb + i] = (b[0] != b[0]) || (b[1] != b[1]) || (b[2] != b[2]) || (b[3] != b[3]);
    a.cbox[tb + i] = Box{b[0], b[1], b[2], b[3]};
    // the rest of the column inputs at the tracker's list position (k_doc_pre keeps them in place
    // when no tracker is culled, the steady state, and recomputes the survivors' otherwise)
    double ko[5];
    doc_prev_obs(r, a.delta_t, ko);
    for (int k = 0; k < 5; ++k) {
        a.ckobs[(tb + i) * 5 + k] = ko[k];
        a.clast[(tb + i) * 5 + k] = r.last_obs[k];
    }
    const bool hv = (r.flags & OF_VELOCITY) != 0;
    a.cvel[(tb + i) * 2] = hv ? r.vel[0] : 0.0;
    a.cvel[(tb + i) * 2 + 1] = hv ? r.vel[1] : 0.0;
    a.cslot[tb + i] = a.list[tb + i];
    a.cmatched[tb + i] = 0;
    a.upd[tb + i] = -1;
}

__global__ __launch_bounds__(OC_T) void k_doc_pre(DocArgs a) {
    __shared__ OcShared sh;
    const int s = blockIdx.x, t = threadIdx.x, nt = blockDim.x;
    if (a.active && !a.active[s]) return;   // stream not updated this frame
    DocCounters *c = a.cnt + s;
    const long long tb = (long long)s * a.CAP, db = (long long)s * a.MAXD;
    const long long ub = (long long)s * (a.MAXD + a.CAP);
    int nd = a.det_off[s + 1] - a.det_off[s];
    if (nd > a.MAXD || nd < 0) {
        if (t == 0) atomicOr(&c->err, ERR_DET_CAPACITY);
        nd = nd < 0 ? 0 : a.MAXD;
    }
    const double *din = a.det_in + (long long)a.det_off[s] * 6;
    int n_trk = c->n_trk;
    const int dt = a.delta_t;
    int *list = a.list + tb;
    // CMC + predict and the column inputs ran chip-wide in k_doc_predict (by list position)
    int n_free = c->n_free;
    const int n_nan = block_compact(n_trk, sh.wsum, [&](int i) { return a.nan_flag[tb + i] != 0; },
                                    [&](int i, int pos) { a.tmp[ub + pos] = list[i]; });
    if (n_nan > 0) {   // cull: the survivors' inputs compacted
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
        Box *bscratch = reinterpret_cast<Box *>(a.mat2 + doc_mb(a, s));
        for (int j = t; j < n_keep; j += nt) {
            const DocTrack &r = a.rec[tb + a.tmp[ub + j]];
            bscratch[j] = a.cbox[tb + a.upd[tb + j]];
            double ko[5];
            doc_prev_obs(r, dt, ko);
            for (int k = 0; k < 5; ++k) {
                a.ckobs[(tb + j) * 5 + k] = ko[k];
                a.clast[(tb + j) * 5 + k] = r.last_obs[k];
            }
            const bool hv = (r.flags & OF_VELOCITY) != 0;
            a.cvel[(tb + j) * 2] = hv ? r.vel[0] : 0.0;
            a.cvel[(tb + j) * 2 + 1] = hv ? r.vel[1] : 0.0;
        }
        block_sync();
        for (int j = t; j < n_keep; j += nt) {
            list[j] = a.tmp[ub + j];
            a.cslot[tb + j] = a.tmp[ub + j];
            a.cbox[tb + j] = bscratch[j];
            a.cmatched[tb + j] = 0;
            a.nan_flag[tb + j] = 0;
            a.upd[tb + j] = -1;
        }
        n_trk = n_keep;
        if (t == 0) c->n_free = n_free;
        block_sync();
    }
    // detections kept for association (:374-377) and their embedding weights (:395-398)
    const int n_hi = block_compact(nd, sh.wsum, [&](int i) { return din[i * 6 + 4] > a.det_thresh; },
                                   [&](int i, int pos) {
                                       a.hi_row[db + pos] = i;
                                       const double trust = (din[i * 6 + 4] - a.det_thresh) /
                                                            (1 - a.det_thresh);
                                       a.alpha[db + pos] = a.af + (1 - a.af) * (1 - trust);
                                   });
    for (int i = t; i < n_hi; i += nt) {
        a.rmatch[db + i] = 0;
        a.pos_cnt[db + i] = 0;
    }
    for (int j = t; j < n_trk; j += nt) a.col_cnt[tb + j] = 0;
    if (t == 0) {
        c->n_trk = n_trk;
        c->n_high = n_hi;
        c->n_dets = nd;
        c->n_pos = a.force_dense ? 1 : 0;
        c->col_ovf = 0;
    }
}

__global__ __launch_bounds__(OC_T) void k_doc_cost(DocArgs a) {
    const int s = blockIdx.y;
    if (a.active && !a.active[s]) return;   // stream not updated this frame
    DocCounters *c = a.cnt + s;
    const int n_trk = c->n_trk, n_hi = c->n_high;
    const long long nm = (long long)n_hi * n_trk;
    const long long tb = (long long)s * a.CAP, db = (long long)s * a.MAXD, mb = doc_mb(a, s);
    const double *din = a.det_in + (long long)a.det_off[s] * 6;
    const double img_w = a.img_wh ? (double)a.img_wh[2 * s] : 0.0;
    const double img_h = a.img_wh ? (double)a.img_wh[2 * s + 1] : 0.0;
    double *mat = a.mat + mb, *mat2 = a.mat2 + mb;
    bool giou_bad = false;
    for (long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x; q < nm;
         q += (long long)gridDim.x * blockDim.x) {
        const int i = (int)(q / n_trk), j = (int)(q % n_trk);
        const double *dr = din + (long long)a.hi_row[db + i] * 6;
        const double v = asso_of(a.asso, box5(dr), a.cbox[tb + j], img_w, img_h);
        if (a.asso == 1 && v != v) giou_bad = true;
        const double *ko = a.ckobs + (tb + j) * 5;
        const double dx = (dr[0] + dr[2]) / 2.0 - (ko[0] + ko[2]) / 2.0;
        const double dy = (dr[1] + dr[3]) / 2.0 - (ko[1] + ko[3]) / 2.0;
        const double nrm = sqrt(dx * dx + dy * dy) + 1e-6;
        const double X = dx / nrm, Y = dy / nrm;
        const double vy = a.cvel[(tb + j) * 2], vx = a.cvel[(tb + j) * 2 + 1];
        double cs = vx * X + vy * Y;
        cs = np_min(np_max(cs, -1.0), 1.0);
        const double ang = (M_PI / 2.0 - fabs(acos(cs))) / M_PI;
        const double valid = ko[4] < 0 ? 0.0 : 1.0;
        const double angle = ((valid * ang) * a.inertia) * dr[4];
        mat[q] = v;
        mat2[q] = v + angle;            // iou + angle; the embedding term joins in k_doc_final
        // emb_cost[iou_matrix <= 0] = 0 (association.py:165): only these pairs' dot products
        // are read (k_doc_aw, k_doc_final); listed per detection row
        if (!(v <= 0)) {
            const int k = atomicAdd(&a.pos_cnt[db + i], 1);
            if (k < POS_K) a.pos_q[(db + i) * POS_K + k] = j;
            else c->n_pos = 1;   // a row with more: the dense tiles
        }
        if (v > a.thr) {
            atomicAdd(&a.rmatch[db + i], 1);
            atomicAdd(&a.cmatched[tb + j], 1);
        }
    }
    if (giou_bad) atomicOr(&c->err, ERR_GIOU);
}

// dets_embs @ trk_embs^T (deep_ocsort.py:432), float64 accumulation.
constexpr int EMB_TILE = 64;
// 64 (detections) x 64 (trackers) tiles per block, 4 waves of 32 x 32 (2 x 2 MFMA tiles of
// v_mfma_f64_16x16x4_f64: A[l&15][k = l>>4], B[k = l>>4][l&15], D[row (l>>4) + 4 r][col l&15]);
// K streams through LDS in chunks of 32, the next chunk held in registers while the current
// chunk's MFMAs run.  Detection rows are float32 (promoted exactly), tracker rows float64.
typedef double dbl4 __attribute__((ext_vector_type(4)));
constexpr int DE_KC = 32, DE_LD = DE_KC + 1;
__global__ __launch_bounds__(256) void k_doc_emb(DocArgs a) {
    __shared__ double As[EMB_TILE * DE_LD], Bs[EMB_TILE * DE_LD];
    const int s = blockIdx.z;
    if (a.active && !a.active[s]) return;   // stream not updated this frame
    const DocCounters *c = a.cnt + s;
    if (c->n_pos == 0) return;               // the listed pairs only (k_doc_emb_pairs)
    const int n_trk = c->n_trk, n_hi = c->n_high, D = a.D;
    int bx, by;
    xcd_tile(bx, by);                                         // row bands per XCD (common.hpp)
    const int r0 = by * EMB_TILE, c0 = bx * EMB_TILE;
    if (r0 >= n_hi || c0 >= n_trk) return;                   // block-uniform
    const long long tb = (long long)s * a.CAP, db = (long long)s * a.MAXD, mb = doc_mb(a, s);
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int wr = (w >> 1) * 32, wc = (w & 1) * 32;
    const int lr = t >> 2, lk = (t & 3) * 8;   // staging: 8 consecutive k of row lr
    const bool a_ok = r0 + lr < n_hi, b_ok = c0 + lr < n_trk;
    const float *arow = a_ok ? a.det_feat + ((long long)a.det_off[s] + a.hi_row[db + r0 + lr]) * D
                             : nullptr;
    const double *brow = b_ok ? a.emb + (tb + a.cslot[tb + c0 + lr]) * D : nullptr;
    double pa[8], pb[8];
    auto fetch = [&](int k0) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int k = k0 + lk + u;
            pa[u] = (a_ok && k < D) ? (double)arow[k] : 0.0;
            pb[u] = (b_ok && k < D) ? brow[k] : 0.0;
        }
    };
    dbl4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = dbl4{0.0, 0.0, 0.0, 0.0};
    fetch(0);
    for (int k0 = 0; k0 < D; k0 += DE_KC) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            As[lr * DE_LD + lk + u] = pa[u];
            Bs[lr * DE_LD + lk + u] = pb[u];
        }
        __syncthreads();
        if (k0 + DE_KC < D) fetch(k0 + DE_KC);
#pragma unroll
        for (int ks = 0; ks < DE_KC; ks += 4) {
            const int kk = ks + (lane >> 4);
            double af[2], bf[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) af[i] = As[(wr + 16 * i + (lane & 15)) * DE_LD + kk];
#pragma unroll
            for (int j = 0; j < 2; ++j) bf[j] = Bs[(wc + 16 * j + (lane & 15)) * DE_LD + kk];
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[i], bf[j], acc[i][j], 0, 0, 0);
        }
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) {
                const int p = r0 + wr + 16 * i + (lane >> 4) + 4 * rr;
                const int q = c0 + wc + 16 * j + (lane & 15);
                if (p < n_hi && q < n_trk) a.emat[mb + (long long)p * n_trk + q] = acc[i][j][rr];
            }
}

// The embedding term is read only where the asso value is not <= 0 (association.py:165): a few
// pairs per detection, listed per row by k_doc_cost.  One wave per detection row, its pairs four at
// a time (a 16-lane group each: float64 accumulation, cosine_dist16's reduction), written at their
// positions of emat; with AW on, the row's top two of emb (zero elsewhere) give its weight here,
// and every column's listed values for k_doc_aw_cols (k_doc_aw's dense scans then do not run).
// The dense tiles (k_doc_emb) and scans run instead when a row or column listed more than POS_K.
constexpr int EMBP_T = 256;
__global__ __launch_bounds__(EMBP_T) void k_doc_emb_pairs(DocArgs a) {
    const int s = blockIdx.y;
    if (a.active && !a.active[s]) return;   // stream not updated this frame
    const DocCounters *c = a.cnt + s;
    if (c->n_pos != 0) return;               // dense path
    const int n_trk = c->n_trk, n_hi = c->n_high, D = a.D;
    const int i = blockIdx.x * (EMBP_T / WAVE) + threadIdx.x / WAVE;
    if (i >= n_hi) return;
    const long long tb = (long long)s * a.CAP, db = (long long)s * a.MAXD, mb = doc_mb(a, s);
    const int lane = lane_id(), grp = lane >> 4, l16 = lane & 15;
    const int cnt = a.pos_cnt[db + i];   // <= POS_K (n_pos == 0)
    const float *ar = a.det_feat + ((long long)a.det_off[s] + a.hi_row[db + i]) * D;
    double m1 = -INFINITY, m2 = -INFINITY;
    for (int p0 = 0; p0 < cnt; p0 += 4) {
        const int p = p0 + grp;
        const bool v = p < cnt;
        const int j = a.pos_q[(db + i) * POS_K + (v ? p : p0)];
        const double *br = a.emb + (tb + a.cslot[tb + j]) * D;
        double acc = 0.0;
        constexpr int CB = 16;
        int k = l16;
        for (; k + 16 * (CB - 1) < D; k += 16 * CB) {
            float av[CB];
            double bv[CB];
#pragma unroll
            for (int u = 0; u < CB; ++u) {
                av[u] = ar[k + 16 * u];
                bv[u] = br[k + 16 * u];
            }
#pragma unroll
            for (int u = 0; u < CB; ++u) acc += (double)av[u] * bv[u];
        }
        for (; k < D; k += 16) acc += (double)ar[k] * br[k];
        acc = row_allreduce(RED_SUM, acc);
        if (v && l16 == 0) {
            a.emat[mb + (long long)i * n_trk + j] = acc;
            top2_push(acc, m1, m2);
            if (!a.aw_off) {   // the column's share for k_doc_aw_cols
                const int kc = atomicAdd(&a.col_cnt[tb + j], 1);
                if (kc < POS_K) a.col_e[(tb + j) * POS_K + kc] = acc;
                else atomicOr(const_cast<int *>(&c->col_ovf), 1);
            }
        }
    }
    if (a.aw_off) return;
    for (int o = 32; o >= 1; o >>= 1) {   // merge the lanes' top-2
        const double o1 = __shfl_xor(m1, o), o2 = __shfl_xor(m2, o);
        top2_push(o1, m1, m2);
        top2_push(o2, m1, m2);
    }
    // the row's other entries are 0 (emb zeroed where the asso value is <= 0)
    if (n_trk - cnt >= 1) top2_push(0.0, m1, m2);
    if (n_trk - cnt >= 2) top2_push(0.0, m1, m2);
    if (lane == 0) a.rw[db + i] = aw_weight(m1, m2, a.aw_param, n_trk);
}

// compute_aw_max_metric (association.py:79-108) on emb[iou <= 0] = 0: the top two values of each
// row (blockIdx.x < row blocks) or column; one wave per row / per 64 columns.
// compute_aw_max_metric (association.py:79-108) on emb (zeroed where iou <= 0).  Rows: one wave
// per detection row.  Columns: AW_CHUNKS row chunks x 64-column tiles, 4 waves per tile (lanes =
// columns, coalesced rows), partial top-2 merged in LDS, then k_doc_aw_cols merges the chunks
// (top-2 selection is exact and order-free).
constexpr int AW_CHUNKS = 8;
__global__ __launch_bounds__(256) void k_doc_aw(DocArgs a) {
    const int s = blockIdx.y;
    if (a.active && !a.active[s]) return;   // stream not updated this frame
    const DocCounters *c = a.cnt + s;
    const int n_trk = c->n_trk, n_hi = c->n_high;
    const long long db = (long long)s * a.MAXD, mb = doc_mb(a, s);
    const double *E = a.emat + mb, *I = a.mat + mb;
    const int lane = lane_id(), wv = threadIdx.x / WAVE;
    const int row_blocks = (a.MAXD + 3) / 4;
    auto val = [&](int r, int cc) {
        const long long q = (long long)r * n_trk + cc;
        return I[q] <= 0 ? 0.0 : E[q];
    };
    if ((int)blockIdx.x < row_blocks) {
        if (c->n_pos == 0) return;   // the row weights came with the listed pairs (k_doc_emb_pairs)
        const int r = blockIdx.x * 4 + wv;
        if (r >= n_hi) return;
        double m1 = -INFINITY, m2 = -INFINITY;
        constexpr int RB = 8;   // a lane's next 8 entries loaded before any is used
        int cc = lane;
        for (; cc + WAVE * (RB - 1) < n_trk; cc += WAVE * RB) {
            double iv[RB];
#pragma unroll
            for (int u = 0; u < RB; ++u) iv[u] = I[(long long)r * n_trk + cc + WAVE * u];
#pragma unroll
            for (int u = 0; u < RB; ++u)   // the embedding term only where it is kept
                top2_push(iv[u] <= 0 ? 0.0 : E[(long long)r * n_trk + cc + WAVE * u], m1, m2);
        }
        for (; cc < n_trk; cc += WAVE) top2_push(val(r, cc), m1, m2);
        for (int o = 32; o >= 1; o >>= 1) {   // merge the lanes' top-2
            const double o1 = __shfl_xor(m1, o), o2 = __shfl_xor(m2, o);
            top2_push(o1, m1, m2);
            top2_push(o2, m1, m2);
        }
        if (lane == 0) a.rw[db + r] = aw_weight(m1, m2, a.aw_param, n_trk);
    } else {
        __shared__ double part[4][WAVE][2];
        if (c->n_pos == 0 && c->col_ovf == 0) return;   // listed columns (k_doc_aw_cols)
        const int q = (int)blockIdx.x - row_blocks;
        const int tile = q / AW_CHUNKS, chunk = q % AW_CHUNKS;
        const int cc = tile * WAVE + lane;
        const int per = (n_hi + AW_CHUNKS - 1) / AW_CHUNKS;
        const int r0 = chunk * per, r1 = r0 + per < n_hi ? r0 + per : n_hi;
        double m1 = -INFINITY, m2 = -INFINITY;
        if (cc < n_trk) {
            int r = r0 + wv;
            for (; r + 12 < r1; r += 16) {   // 4 independent rows per step
                const double v0 = val(r, cc), v1 = val(r + 4, cc), v2 = val(r + 8, cc),
                             v3 = val(r + 12, cc);
                top2_push(v0, m1, m2);
                top2_push(v1, m1, m2);
                top2_push(v2, m1, m2);
                top2_push(v3, m1, m2);
            }
            for (; r < r1; r += 4) top2_push(val(r, cc), m1, m2);
        }
        part[wv][lane][0] = m1;
        part[wv][lane][1] = m2;
        __syncthreads();
        if (wv == 0 && cc < n_trk) {
            for (int k = 1; k < 4; ++k) {
                top2_push(part[k][lane][0], m1, m2);
                top2_push(part[k][lane][1], m1, m2);
            }
            double *o = a.cw_part + ((long long)s * AW_CHUNKS + chunk) * a.CAP * 2 + 2LL * cc;
            o[0] = m1;
            o[1] = m2;
        }
    }
}
__global__ __launch_bounds__(256) void k_doc_aw_cols(DocArgs a) {
    const int s = blockIdx.y;
    if (a.active && !a.active[s]) return;   // stream not updated this frame
    const DocCounters *c = a.cnt + s;
    const int n_trk = c->n_trk, n_hi = c->n_high;
    const int cc = blockIdx.x * blockDim.x + threadIdx.x;
    if (cc >= n_trk) return;
    double m1 = -INFINITY, m2 = -INFINITY;
    if (c->n_pos == 0 && c->col_ovf == 0) {   // the column's listed values, zeros elsewhere
        const long long tb = (long long)s * a.CAP;
        const int cnt = a.col_cnt[tb + cc];
        for (int k = 0; k < cnt; ++k) top2_push(a.col_e[(tb + cc) * POS_K + k], m1, m2);
        if (n_hi - cnt >= 1) top2_push(0.0, m1, m2);
        if (n_hi - cnt >= 2) top2_push(0.0, m1, m2);
        a.cw[tb + cc] = aw_weight(m1, m2, a.aw_param, n_hi);
        return;
    }
    for (int k = 0; k < AW_CHUNKS; ++k) {
        const double *o = a.cw_part + ((long long)s * AW_CHUNKS + k) * a.CAP * 2 + 2LL * cc;
        top2_push(o[0], m1, m2);
        top2_push(o[1], m1, m2);
    }
    a.cw[(long long)s * a.CAP + cc] = aw_weight(m1, m2, a.aw_param, n_hi);
}

// final cost -(iou + angle + emb_term) (association.py:170); emb_term = ((w rw) cw) emb (AW) or
// emb * w (aw_off), emb zeroed where iou <= 0.
__global__ __launch_bounds__(256) void k_doc_final(DocArgs a) {
    const int s = blockIdx.y;
    if (a.active && !a.active[s]) return;   // stream not updated this frame
    const DocCounters *c = a.cnt + s;
    const int n_trk = c->n_trk, n_hi = c->n_high;
    const long long nm = (long long)n_hi * n_trk;
    const long long tb = (long long)s * a.CAP, db = (long long)s * a.MAXD, mb = doc_mb(a, s);
    const bool use_emb = !a.embedding_off && a.D > 0 && n_hi > 0 && n_trk > 0;
    for (long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x; q < nm;
         q += (long long)gridDim.x * blockDim.x) {
        double term = 0.0;
        if (use_emb) {
            const double e = a.mat[mb + q] <= 0 ? 0.0 : a.emat[mb + q];
            if (a.aw_off) term = e * a.w_emb;
            else {
                const int i = (int)(q / n_trk), j = (int)(q % n_trk);
                term = ((a.w_emb * a.rw[db + i]) * a.cw[tb + j]) * e;
            }
        }
        a.mat2[mb + q] = -(a.mat2[mb + q] + term);
    }
}

// Row pre-pass of the first-round solve, chip-wide (lap_rect.hpp).
__global__ __launch_bounds__(OC_T) void k_doc_rowpre(DocArgs a) {
    const int s = blockIdx.y;
    if (a.active && !a.active[s]) return;   // stream not updated this frame
    const DocCounters *c = a.cnt + s;
    const long long db = (long long)s * a.MAXD;
    main_lap_pre(a.mat2 + doc_mb(a, s), c->n_high, c->n_trk, a.pre_u + db, a.pre_x + db,
                 a.pre_s2 + db);
}

// First-round solve, one LAP_T-thread block per stream (ocsort_common.hpp first_round_lap).
__global__ __launch_bounds__(LAP_T) void k_doc_lap(DocArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int s = blockIdx.x;
    if (a.active && !a.active[s]) return;   // stream not updated this frame
    DocCounters *c = a.cnt + s;
    const long long tb = (long long)s * a.CAP, db = (long long)s * a.MAXD;
    first_round_lap(a.mat2 + doc_mb(a, s), c->n_high, c->n_trk, a.rmatch + db, a.cmatched + tb, true,
                    a.pre_u + db, a.pre_x + db, a.pre_s2 + db, a.rmatch + db, lds,
                    lap_kernel_lds(a.CAP, a.MAXD), a.lap_ws + s * a.lap_ws_stride, &c->err,
                    &c->lap_done, &c->ls, a.lap_ws + (s + 1) * a.lap_ws_stride - tight_ws_bytes(),
                    nullptr, a.arr_chip != 0);
}

// The chip-wide bidding rounds of the first round (ocsort_common.hpp fr_arr_*), when a.arr_chip.
__global__ __launch_bounds__(OC_T) void k_doc_arr0(DocArgs a) {
    __shared__ int wsum[32];
    const int s = blockIdx.x;
    if (a.active && !a.active[s]) return;   // stream not updated this frame
    const DocCounters *c = a.cnt + s;
    const long long tb = (long long)s * a.CAP, db = (long long)s * a.MAXD;
    fr_arr_round0(a.mat2 + doc_mb(a, s), c->n_high, c->n_trk, a.rmatch + db, a.cmatched + tb, true,
                  a.pre_u + db, a.pre_x + db, a.pre_s2 + db,
                  a.lap_ws + (s + 1) * a.lap_ws_stride - tight_ws_bytes(), wsum);
}
__global__ __launch_bounds__(ARR_SCAN_WPB * WAVE) void k_doc_arrscan(DocArgs a) {
    const int s = blockIdx.y;
    if (a.active && !a.active[s]) return;
    const DocCounters *c = a.cnt + s;
    fr_arr_scan(a.mat2 + doc_mb(a, s), c->n_high, c->n_trk, a.lap_ws + (s + 1) * a.lap_ws_stride - tight_ws_bytes(),
                blockIdx.x, gridDim.x);
}
__global__ __launch_bounds__(OC_T) void k_doc_arrapply(DocArgs a) {
    __shared__ int wsum[32];
    const int s = blockIdx.x;
    if (a.active && !a.active[s]) return;
    const DocCounters *c = a.cnt + s;
    fr_arr_apply(a.mat2 + doc_mb(a, s), c->n_high, c->n_trk, a.lap_ws + (s + 1) * a.lap_ws_stride - tight_ws_bytes(),
                 wsum);
}

__global__ __launch_bounds__(OC_T) void k_doc_assoc(DocArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    __shared__ OcShared sh;
    const int s = blockIdx.x, t = threadIdx.x, nt = blockDim.x;
    if (a.active && !a.active[s]) return;   // stream not updated this frame
    DocCounters *c = a.cnt + s;
    const long long tb = (long long)s * a.CAP, db = (long long)s * a.MAXD, mb = doc_mb(a, s);
    const long long ub = (long long)s * (a.MAXD + a.CAP);
    unsigned char *gws = a.lap_ws + s * a.lap_ws_stride;
    const long long lds_bytes = oc_lds_bytes(a.CAP, a.MAXD);
    const double *din = a.det_in + (long long)a.det_off[s] * 6;
    int n_trk = c->n_trk;
    const int n_hi = c->n_high;
    int *list = a.list + tb;
    double *mat = a.mat + mb, *mat2 = a.mat2 + mb;
    int *udet = a.udet + ub, *utrk = a.utrk + ub;
    int n_ud = 0, n_ut = 0;
    auto hbox = [&](int i) { return box5(din + (long long)a.hi_row[db + i] * 6); };
    YTA_STAMP_BASE(40);
    YTA_STAMP(0);
    // ---- first round (association.py:111-201)
    if (n_trk == 0) {
        for (int i = t; i < n_hi; i += nt) udet[i] = i;
        n_ud = n_hi;
        if (t == 0) { c->fast_path = 0; c->lap_calls = 0; }
    } else {
        if (t < 8) sh.cnt[t] = 0;
        block_sync();
        int over = 0, bad = 0;
        for (int i = t; i < n_hi; i += nt) {
            const int k = ald(a.rmatch + db + i);
            over += k;
            bad |= k > 1;
        }
        for (int j = t; j < n_trk; j += nt) bad |= ald(a.cmatched + tb + j) > 1;
        if (over) atomicAdd(&sh.cnt[0], over);
        if (bad) atomicOr(&sh.cnt[1], 1);
        block_sync();
        const bool solved = c->lap_done != 0;   // by k_*_lap
        const bool fast = !solved && sh.cnt[1] == 0 && sh.cnt[0] > 0;
        if (fast) {
            for (int i = t; i < n_hi; i += nt) {
                int col = -1;
                if (ald(a.rmatch + db + i) == 1)
                    for (int j = 0; j < n_trk; ++j)
                        if (mat[(long long)i * n_trk + j] > a.thr) { col = j; break; }
                a.rmatch[db + i] = col;
            }
            block_sync();
        } else if (n_hi > 0 && !solved) {
            block_sync();
            main_lap(LapMat{mat2, n_hi, n_trk, false}, a.pre_u + db, a.pre_x + db, a.pre_s2 + db,
                     a.rmatch + db, lds, lds_bytes, gws, &c->err, &c->ls,
                     a.lap_csr ? a.lap_csr + s * a.lap_csr_stride : nullptr);
        }
        YTA_STAMP(1);
        if (t == 0) { c->fast_path = fast; c->lap_calls = (fast || n_hi == 0) ? 0 : 1; }
        for (int j = t; j < n_trk; j += nt) a.cmatched[tb + j] = 0;
        block_sync();
        for (int i = t; i < n_hi; i += nt) {
            const int col = a.rmatch[db + i];
            if (col >= 0) a.cmatched[tb + col] = 1;
        }
        block_sync();
        n_ud = block_compact(n_hi, sh.wsum, [&](int i) { return a.rmatch[db + i] < 0; },
                             [&](int i, int pos) { udet[pos] = i; });
        n_ut = block_compact(n_trk, sh.wsum, [&](int j) { return a.cmatched[tb + j] == 0; },
                             [&](int j, int pos) { utrk[pos] = j; });
        auto filtered = [&](int i) {
            const int col = a.rmatch[db + i];
            return col >= 0 && mat[(long long)i * n_trk + col] < a.thr;
        };
        const int nf = block_compact(n_hi, sh.wsum, filtered, [&](int i, int pos) {
            udet[n_ud + pos] = i;
            utrk[n_ut + pos] = a.rmatch[db + i];
        });
        for (int i = t; i < n_hi; i += nt) {
            const int col = a.rmatch[db + i];
            if (col >= 0 && !filtered(i)) a.upd[tb + col] = i;   // kept-detection index
        }
        n_ud += nf;
        n_ut += nf;
        block_sync();
    }
    YTA_STAMP(2);
    // the OCR round's matrix is filled chip-wide (k_doc_ocr); k_doc_assoc_b solves the round
    if (t == 0) {
        c->n_ud = n_ud;
        c->n_ut = n_ut;
        c->ocr_nan = 0;
        c->ocr_max = 0ull;
    }
}

// Order-preserving bits of a double (larger value, larger bits), for the OCR matrix's maximum.
__device__ __forceinline__ unsigned long long doc_ord(double v) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(v);
    return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
__device__ __forceinline__ double doc_unord(unsigned long long o) {
    const unsigned long long b = (o >> 63) ? (o & 0x7FFFFFFFFFFFFFFFull) : ~o;
    return __longlong_as_double((long long)b);
}

// OCR round matrix (:470-493): asso_func(left dets, last observations) over the chip, one entry
// per thread, with its maximum (np.max: NaN-propagating) for k_doc_assoc_b.  In the block it was
// one thread per ~60 entries of f64 GIoU (C4: ~40 x 400 entries, ~90 us for the round).
__global__ __launch_bounds__(256) void k_doc_ocr(DocArgs a) {
    __shared__ OcShared sh;
    const int s = blockIdx.y;
    if (a.active && !a.active[s]) return;
    DocCounters *c = a.cnt + s;
    const int n_ud = c->n_ud, n_ut = c->n_ut;
    if (n_ud <= 0 || n_ut <= 0) return;
    const long long tb = (long long)s * a.CAP, db = (long long)s * a.MAXD, mb = doc_mb(a, s);
    const long long ub = (long long)s * (a.MAXD + a.CAP);
    const double *din = a.det_in + (long long)a.det_off[s] * 6;
    const int *udet = a.udet + ub, *utrk = a.utrk + ub;
    double *mat = a.mat + mb;
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
    if (threadIdx.x == 0 && mx > -INFINITY) atomicMax(&c->ocr_max, doc_ord(mx));
}

// The OCR round's solve (:470-493) after k_doc_ocr, then the update jobs.
__global__ __launch_bounds__(OC_T) void k_doc_assoc_b(DocArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    __shared__ OcShared sh;
    const int s = blockIdx.x, t = threadIdx.x, nt = blockDim.x;
    if (a.active && !a.active[s]) return;   // stream not updated this frame
    DocCounters *c = a.cnt + s;
    const long long tb = (long long)s * a.CAP, db = (long long)s * a.MAXD, mb = doc_mb(a, s);
    const long long ub = (long long)s * (a.MAXD + a.CAP);
    unsigned char *gws = a.lap_ws + s * a.lap_ws_stride;
    const long long lds_bytes = oc_lds_bytes(a.CAP, a.MAXD);
    const int n_trk = c->n_trk;
    const int n_hi = c->n_high;
    int *list = a.list + tb;
    double *mat = a.mat + mb;
    int *udet = a.udet + ub, *utrk = a.utrk + ub;
    int n_ud = c->n_ud, n_ut = c->n_ut;
    YTA_STAMP_BASE(40);
    if (n_ud > 0 && n_ut > 0) {
        const double mx = c->ocr_nan ? NAN : doc_unord(c->ocr_max);
        if (mx > a.thr) {
            iou_lap(LapMat{mat, n_ud, n_ut, true}, a.rmatch + db, lds, lds_bytes, gws, &c->err, &c->ls,
                    a.lap_ws + (s + 1) * a.lap_ws_stride - tight_ws_bytes(), nullptr, nullptr,
                    nullptr, a.thr);
            for (int i = t; i < n_hi; i += nt) a.tmp[ub + i] = 0;
            for (int j = t; j < n_trk; j += nt) a.nan_flag[tb + j] = 0;
            block_sync();
            for (int p = t; p < n_ud; p += nt) a.tmp[ub + udet[p]] = 1;
            for (int k = t; k < n_ut; k += nt) a.nan_flag[tb + utrk[k]] = 1;
            block_sync();
            for (int p = t; p < n_ud; p += nt) {
                const int k = a.rmatch[db + p];
                if (k >= 0 && !(mat[(long long)p * n_ut + k] < a.thr)) {
                    a.upd[tb + utrk[k]] = udet[p];
                    a.tmp[ub + udet[p]] = 0;
                    a.nan_flag[tb + utrk[k]] = 0;
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
    YTA_STAMP(3);
    // ---- tracker updates; embedding jobs for k_doc_ema
    const long long eb = (long long)s * (a.CAP + a.MAXD);
    const int n_upd = block_compact(n_trk, sh.wsum, [&](int j) { return a.upd[tb + j] >= 0; },
                                    [&](int j, int pos) {
                                        a.ema_slot[eb + pos] = list[j];
                                        a.ema_row[eb + pos] = a.upd[tb + j];
                                    });
    if (t == 0) {
        c->n_ud = n_ud;
        c->n_upd = n_upd;
    }
    YTA_STAMP(4);
}

// Every tracker's update (deep_ocsort.py:461-467, :480-493: a matched tracker takes its
// detection, the others update(None)) chip-wide, one thread per tracker: each touches only its
// own record.
__global__ __launch_bounds__(DOC_TRK_T) void k_doc_upd(DocArgs a) {
    const int s = blockIdx.y;
    if (a.active && !a.active[s]) return;   // stream not updated this frame
    const DocCounters *c = a.cnt + s;
    const int j = blockIdx.x * DOC_TRK_T + threadIdx.x;
    if (j >= c->n_trk) return;
    const long long tb = (long long)s * a.CAP, db = (long long)s * a.MAXD;
    const double *din = a.det_in + (long long)a.det_off[s] * 6;
    const int hi = a.upd[tb + j];
    const int row = hi >= 0 ? a.hi_row[db + hi] : -1;
    doc_update(a.rec[tb + a.list[tb + j]], row >= 0 ? din + (long long)row * 6 : nullptr, row,
               a.delta_t);
}

constexpr int DOC_BIRTH_CH = 16;   // births staged in LDS at a time (k_doc_finish)

// Births, outputs, removal (deep_ocsort.py:495-520), after k_doc_upd.
__global__ __launch_bounds__(OC_T) void k_doc_finish(DocArgs a) {
    __shared__ OcShared sh;
    const int s = blockIdx.x, t = threadIdx.x, nt = blockDim.x;
    if (a.active && !a.active[s]) {   // not updated this frame: no output rows
        if (threadIdx.x == 0) {
            a.cnt[s].n_out = 0;
            if (a.out_counts) a.out_counts[s] = 0;
        }
        return;
    }
    DocCounters *c = a.cnt + s;
    const long long tb = (long long)s * a.CAP, db = (long long)s * a.MAXD;
    const long long ub = (long long)s * (a.MAXD + a.CAP);
    const double *din = a.det_in + (long long)a.det_off[s] * 6;
    const int frame = c->frame + 1;
    int n_trk = c->n_trk;
    int *list = a.list + tb;
    const int *udet = a.udet + ub;
    const int n_ud = c->n_ud, n_upd = c->n_upd;
    const long long eb = (long long)s * (a.CAP + a.MAXD);
    YTA_STAMP_BASE(40);
    // ---- births in unmatched-list order (:495-503)
    int n_free = c->n_free;
    int n_b = n_ud;
    if (n_b > n_free) {
        if (t == 0) atomicOr(&c->err, ERR_TRACK_CAPACITY);
        n_b = n_free;
    }
    const long long next_id = c->next_id;
    // a birth's 1216-B record is built in LDS by its thread and stored by the whole block in
    // 16-B pieces, consecutive lanes on consecutive pieces: one thread storing its record word by
    // word beside the others' made every store instruction touch a line per birth (C4: ~33 us for
    // 33 births)
    static_assert(sizeof(DocTrack) % 16 == 0, "DocTrack is stored in 16-B pieces");
    constexpr int REC_Q = (int)(sizeof(DocTrack) / 16);
    __shared__ DocTrack bstage[DOC_BIRTH_CH];
    for (int b0 = 0; b0 < n_b; b0 += DOC_BIRTH_CH) {
        const int m = n_b - b0 < DOC_BIRTH_CH ? n_b - b0 : DOC_BIRTH_CH;
        for (int r = t; r < m; r += nt) {
            const int b = b0 + r;
            const int slot = a.free_list[tb + n_free - 1 - b];
            const double *dr = din + (long long)a.hi_row[db + udet[b]] * 6;
            doc_birth(bstage[r], dr, next_id + b, a.hi_row[db + udet[b]]);
            list[n_trk + b] = slot;
            a.ema_slot[eb + n_upd + b] = slot;
            a.ema_row[eb + n_upd + b] = ~udet[b];   // birth: copy the detection's embedding
        }
        lds_sync();
        for (int q = t; q < m * REC_Q; q += nt) {
            const int r = q / REC_Q, k = q - r * REC_Q;
            const int slot = a.free_list[tb + n_free - 1 - (b0 + r)];
            reinterpret_cast<double2 *>(&a.rec[tb + slot])[k] =
                reinterpret_cast<const double2 *>(&bstage[r])[k];
        }
        lds_sync();
    }
    n_free -= n_b;
    n_trk += n_b;
    block_sync();
    YTA_STAMP(5);
    // ---- outputs in reversed tracker order, then removal (:505-520); ids as stored (:513).
    // Every record read is batched (block_compact_ld / batched_for2): a per-item chain of list ->
    // record loads would cost a round trip per tracker.  The pass leaves the removal flags in
    // nan_flag for the two removal compactions.
    double *out = a.out + tb * 8;
    struct TrkState {
        int slot, tsu, hit_streak;
    };
    int *oslot = a.tmp + ub;   // the output trackers' slots, in output order
    const int n_out = block_compact_ld<8>(
        n_trk, sh.wsum, [&](int q) { return list[n_trk - 1 - q]; },
        [&](int, int slot) {
            const DocTrack &r = a.rec[tb + slot];
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
            const DocTrack &r = a.rec[tb + slot];
            OutRow o;
            if (np_sum5(r.last_obs) < 0) doc_x_to_bbox(r.kf.x, o.b);
            else for (int k = 0; k < 4; ++k) o.b[k] = r.last_obs[k];
            o.id = (double)r.id;
            o.conf = r.conf;
            o.cls = r.cls;
            o.det_ind = (double)r.det_ind;
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
        c->next_id = next_id + n_b;
        if (a.out_counts) a.out_counts[s] = n_out;
    }
    YTA_STAMP(7);
}

// update_emb (deep_ocsort.py:243-245) for every tracker updated this frame - emb = alpha emb +
// (1 - alpha) det_emb, then emb /= |emb| (float64) - and the embeddings of births (the
// detection's row).  One wave per job.
__global__ __launch_bounds__(256) void k_doc_ema(DocArgs a) {
    const int s = blockIdx.y, lane = lane_id();
    if (a.active && !a.active[s]) return;   // stream not updated this frame
    const DocCounters *c = a.cnt + s;
    const int job = blockIdx.x * 4 + threadIdx.x / WAVE;
    if (job >= c->n_ema) return;
    const long long tb = (long long)s * a.CAP, db = (long long)s * a.MAXD;
    const long long eb = (long long)s * (a.CAP + a.MAXD);
    const int slot = a.ema_slot[eb + job], code = a.ema_row[eb + job];
    const int hi = code >= 0 ? code : ~code;
    const float *e = a.det_feat + ((long long)a.det_off[s] + a.hi_row[db + hi]) * a.D;
    double *emb = a.emb + (tb + slot) * a.D;
    if (code < 0) {
        for (int k = lane; k < a.D; k += WAVE) emb[k] = (double)e[k];
        return;
    }
    const double al = a.alpha[db + hi];
    double q = 0.0;
    for (int k = lane; k < a.D; k += WAVE) {
        const double v = al * emb[k] + (1 - al) * (double)e[k];
        emb[k] = v;
        q += v * v;
    }
    const double nrm = sqrt(wave_reduce(RED_SUM, q));
    for (int k = lane; k < a.D; k += WAVE) emb[k] = emb[k] / nrm;
}

// KalmanBoxTracker KAT: one thread per track, steps of [affine], predict, update(box | None)
__global__ void k_kf8_run(int n, int steps, int dt, const double *b0, const double *b,
                          const double *warps, double *x_out, double *P_out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    DocTrack r;
    const double d0[6] = {b0[4 * i], b0[4 * i + 1], b0[4 * i + 2], b0[4 * i + 3], 0.9, 0.0};
    doc_birth(r, d0, 1, 0);
    for (int st = 0; st < steps; ++st) {
        if (warps) doc_apply_affine(r, warps + ((long long)st * n + i) * 6, dt);
        doc_predict(r);
        const double *z = b + ((long long)st * n + i) * 4;
        const double d[6] = {z[0], z[1], z[2], z[3], 0.9, 0.0};
        doc_update(r, z[0] != z[0] ? nullptr : d, 0, dt);
    }
    for (int k = 0; k < 8; ++k) x_out[8LL * i + k] = r.kf.x[k];
    double *M = P_out + 64LL * i;
    for (int k = 0; k < 64; ++k) M[k] = 0.0;
    for (int g = 0; g < 2; ++g)
        for (int a0 = 0; a0 < 4; ++a0)
            for (int b1 = 0; b1 < 4; ++b1) M[dk_glob(g, a0) * 8 + dk_glob(g, b1)] = r.kf.p[g][4 * a0 + b1];
}

__global__ void k_doc_reset(DocArgs a, int s0) {
    const int s = s0 + blockIdx.x;
    const long long tb = (long long)s * a.CAP;
    for (int i = threadIdx.x; i < a.CAP; i += blockDim.x) a.free_list[tb + i] = a.CAP - 1 - i;
    if (threadIdx.x == 0) {
        DocCounters z;
        memset(&z, 0, sizeof(z));
        z.n_free = a.CAP;
        z.next_id = 1;                         // KalmanBoxTracker.count = 1 (:347)
        a.cnt[s] = z;
    }
}

}  // namespace
}  // namespace yta

// ================================================================================== host engine
using namespace yta;

struct yta_deepocsort {
    int device = 0, S = 0, CAP = 0, MAXD = 0, D = 0;
    yta_deepocsort_params prm{};
    hipStream_t stream = nullptr;
    std::vector<void *> allocs;
    DocArgs a{};
    double *h_dets = nullptr, *d_det_in = nullptr;
    long long det_cap = 0;
    float *h_feat = nullptr, *d_feat = nullptr;
    long long feat_cap = 0;
    int *h_off = nullptr, *d_off = nullptr, *h_wh = nullptr, *d_wh = nullptr;
    double *h_warp = nullptr, *d_warp = nullptr;
    DocCounters *h_cnt = nullptr;
    size_t lds = 0;
    StreamMask mask;   // stream-subset updates (subset.hpp)
};

namespace {

template <typename T>
int doc_dalloc(yta_deepocsort *e, T **p, long long n) {
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

#define DOCALLOC(ptr, n)                      \
    do {                                      \
        int _rc = doc_dalloc(e, &(ptr), (n)); \
        if (_rc) return _rc;                  \
    } while (0)

int doc_alloc(yta_deepocsort *e) {
    const long long S = e->S, CAP = e->CAP, MAXD = e->MAXD, D = e->D;
    DocArgs &a = e->a;
    const yta_deepocsort_params &p = e->prm;
    a.S = e->S;
    a.CAP = e->CAP;
    a.MAXD = e->MAXD;
    a.D = e->D;
    a.det_thresh = p.det_thresh;
    a.thr = p.iou_threshold;
    a.inertia = p.inertia;
    a.w_emb = p.w_association_emb;
    a.af = p.alpha_fixed_emb;
    a.aw_param = p.aw_param;
    a.max_age = p.max_age;
    a.min_hits = p.min_hits;
    a.delta_t = p.delta_t;
    a.asso = p.asso_func;
    a.embedding_off = p.embedding_off || D == 0;
    a.cmc_off = p.cmc_off;
    a.aw_off = p.aw_off;
    DOCALLOC(a.rec, S * CAP);
    DOCALLOC(a.emb, S * CAP * std::max<long long>(D, 1));
    DOCALLOC(a.list, S * CAP);
    DOCALLOC(a.free_list, S * CAP);
    DOCALLOC(a.cnt, S);
    DOCALLOC(a.hi_row, S * MAXD);
    DOCALLOC(a.alpha, S * MAXD);
    DOCALLOC(a.cbox, S * CAP);
    DOCALLOC(a.cvel, S * CAP * 2);
    DOCALLOC(a.ckobs, S * CAP * 5);
    DOCALLOC(a.clast, S * CAP * 5);
    DOCALLOC(a.nan_flag, S * CAP);
    DOCALLOC(a.cslot, S * CAP);
    const long long mat = std::max<long long>(MAXD, 4) * CAP;
    DOCALLOC(a.mat, S * mat);
    DOCALLOC(a.mat2, S * mat);
    DOCALLOC(a.emat, S * mat);
    DOCALLOC(a.pos_q, S * MAXD * POS_K);
    DOCALLOC(a.pos_cnt, S * MAXD);
    DOCALLOC(a.col_e, S * CAP * POS_K);
    DOCALLOC(a.col_cnt, S * CAP);
    DOCALLOC(a.rw, S * MAXD);
    DOCALLOC(a.cw, S * CAP);
    DOCALLOC(a.cw_part, S * AW_CHUNKS * CAP * 2);
    DOCALLOC(a.rmatch, S * MAXD);
    DOCALLOC(a.pre_u, S * MAXD);
    DOCALLOC(a.pre_s2, S * MAXD);
    DOCALLOC(a.pre_x, S * MAXD);
    DOCALLOC(a.cmatched, S * CAP);
    DOCALLOC(a.udet, S * (MAXD + CAP));
    DOCALLOC(a.utrk, S * (MAXD + CAP));
    DOCALLOC(a.tmp, S * (MAXD + CAP));
    DOCALLOC(a.upd, S * CAP);
    DOCALLOC(a.ema_slot, S * (MAXD + CAP));
    DOCALLOC(a.ema_row, S * (MAXD + CAP));
    DOCALLOC(a.out, S * CAP * 8);
    const long long n = std::max(CAP, MAXD);
    a.lap_ws_stride = oc_lap_ws_stride(n);
    a.arr_chip = MAXD >= ARR_CHIP_MIN_DETS;
    if (const char *v = getenv("YTA_ARR_CHIP")) a.arr_chip = atoi(v);
    if (const char *v = getenv("YTA_DOC_DENSE")) a.force_dense = atoi(v) != 0;
    DOCALLOC(a.lap_ws, S * a.lap_ws_stride);
    a.lap_csr = nullptr;
    a.lap_csr_stride = n >= LAPB_MIN_N && lap_sparse_on() ? (lap_csr_bytes(n) + 255) & ~255LL : 0;
    if (a.lap_csr_stride) DOCALLOC(a.lap_csr, S * a.lap_csr_stride);
    e->lds = (size_t)oc_lds_bytes(CAP, MAXD);
    DOCALLOC(e->d_off, S + 1);
    DOCALLOC(e->d_wh, 2 * S);
    DOCALLOC(e->d_warp, 6 * S);
    YTA_HIP(hipHostMalloc((void **)&e->h_off, sizeof(int) * (S + 1), hipHostMallocDefault));
    YTA_HIP(hipHostMalloc((void **)&e->h_wh, sizeof(int) * 2 * S, hipHostMallocDefault));
    YTA_HIP(hipHostMalloc((void **)&e->h_warp, sizeof(double) * 6 * S, hipHostMallocDefault));
    YTA_HIP(hipHostMalloc((void **)&e->h_cnt, sizeof(DocCounters) * S, hipHostMallocDefault));
    YTA_HIP(hipFuncSetAttribute((const void *)k_doc_lap, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)LAP_LDS_MAX));
    YTA_HIP(hipFuncSetAttribute((const void *)k_doc_assoc,
                                hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)dense_lap_ws_bytes(OC_LDS_LAP_N)));
    YTA_HIP(hipFuncSetAttribute((const void *)k_doc_assoc_b,
                                hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)dense_lap_ws_bytes(OC_LDS_LAP_N)));
    return YTA_OK;
}

void doc_release(yta_deepocsort *e) {
    for (void *p : e->allocs) (void)hipFree(p);
    e->allocs.clear();
    if (e->h_off) (void)hipHostFree(e->h_off);
    if (e->h_wh) (void)hipHostFree(e->h_wh);
    if (e->h_warp) (void)hipHostFree(e->h_warp);
    if (e->h_cnt) (void)hipHostFree(e->h_cnt);
    e->h_off = e->h_wh = nullptr;
    e->h_warp = nullptr;
    e->h_cnt = nullptr;
}

int doc_launch(yta_deepocsort *e, const double *d_dets, const int *d_off, const float *d_feat,
               const double *d_warp, const int *d_wh, double *out, int *out_counts) {
    DocArgs &a = e->a;
    a.det_in = d_dets;
    a.det_off = d_off;
    a.det_feat = d_feat;
    a.warp = d_warp;
    a.img_wh = d_wh;
    a.out = out;
    a.out_counts = out_counts;
    {
        const int mrc = e->mask.stage(a.S, e->stream, &a.active);
        if (mrc) return mrc;
    }
    hipLaunchKernelGGL(k_doc_predict, dim3((a.CAP + DOC_TRK_T - 1) / DOC_TRK_T, a.S), dim3(DOC_TRK_T), 0,
                       e->stream, a);
    YTA_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_doc_pre, dim3(a.S), dim3(OC_T), 0, e->stream, a);
    YTA_HIP(hipGetLastError());
    const long long per = ((long long)a.MAXD * a.CAP + OC_T - 1) / OC_T;
    const long long cap = std::max<long long>(4, 4096 / a.S);
    const dim3 gm((unsigned)std::max<long long>(1, std::min(per, cap)), a.S);
    hipLaunchKernelGGL(k_doc_cost, gm, dim3(OC_T), 0, e->stream, a);
    YTA_HIP(hipGetLastError());
    if (!a.embedding_off) {
        const dim3 gp((a.MAXD + EMBP_T / WAVE - 1) / (EMBP_T / WAVE), a.S);
        hipLaunchKernelGGL(k_doc_emb_pairs, gp, dim3(EMBP_T), 0, e->stream, a);
        YTA_HIP(hipGetLastError());
        const dim3 ge((a.CAP + EMB_TILE - 1) / EMB_TILE, (a.MAXD + EMB_TILE - 1) / EMB_TILE, a.S);
        hipLaunchKernelGGL(k_doc_emb, ge, dim3(256), 0, e->stream, a);
        YTA_HIP(hipGetLastError());
        if (!a.aw_off) {
            const dim3 ga((a.MAXD + 3) / 4 + (a.CAP + WAVE - 1) / WAVE * AW_CHUNKS, a.S);
            hipLaunchKernelGGL(k_doc_aw, ga, dim3(256), 0, e->stream, a);
            YTA_HIP(hipGetLastError());
            hipLaunchKernelGGL(k_doc_aw_cols, dim3((a.CAP + 255) / 256, a.S), dim3(256), 0,
                               e->stream, a);
            YTA_HIP(hipGetLastError());
        }
    }
    hipLaunchKernelGGL(k_doc_final, gm, dim3(256), 0, e->stream, a);
    YTA_HIP(hipGetLastError());
    {
        const long long rows = (a.MAXD + OC_T / WAVE - 1) / (OC_T / WAVE);
        const long long rcap = std::max<long long>(4, 4096 / a.S);
        hipLaunchKernelGGL(k_doc_rowpre, dim3((unsigned)std::max<long long>(1, std::min(rows, rcap)), a.S),
                           dim3(OC_T), 0, e->stream, a);
        YTA_HIP(hipGetLastError());
    }
    if (a.arr_chip) {   // the first round's bidding rounds over the chip
        hipLaunchKernelGGL(k_doc_arr0, dim3(a.S), dim3(OC_T), 0, e->stream, a);
        for (int r = 0; r < ARR_CHIP_ROUNDS; ++r) {
            hipLaunchKernelGGL(k_doc_arrscan, dim3(ARR_SCAN_BLOCKS, a.S), dim3(ARR_SCAN_WPB * WAVE), 0,
                               e->stream, a);
            hipLaunchKernelGGL(k_doc_arrapply, dim3(a.S), dim3(OC_T), 0, e->stream, a);
        }
        YTA_HIP(hipGetLastError());
    }
    hipLaunchKernelGGL(k_doc_lap, dim3(a.S), dim3(LAP_T), (size_t)lap_kernel_lds(a.CAP, a.MAXD),
                       e->stream, a);
    YTA_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_doc_assoc, dim3(a.S), dim3(OC_T), e->lds, e->stream, a);
    YTA_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_doc_ocr, dim3((unsigned)std::max(4, 2048 / a.S), a.S), dim3(256), 0,
                       e->stream, a);
    YTA_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_doc_assoc_b, dim3(a.S), dim3(OC_T), e->lds, e->stream, a);
    YTA_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_doc_upd, dim3((a.CAP + DOC_TRK_T - 1) / DOC_TRK_T, a.S), dim3(DOC_TRK_T), 0,
                       e->stream, a);
    YTA_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_doc_finish, dim3(a.S), dim3(OC_T), 0, e->stream, a);
    YTA_HIP(hipGetLastError());
    if (!a.embedding_off) {
        const dim3 gj((a.CAP + a.MAXD + 3) / 4, a.S);
        hipLaunchKernelGGL(k_doc_ema, gj, dim3(256), 0, e->stream, a);
        YTA_HIP(hipGetLastError());
    }
    return YTA_OK;
}

int doc_read_counters(yta_deepocsort *e) {
    YTA_HIP(hipMemcpyAsync(e->h_cnt, e->a.cnt, sizeof(DocCounters) * e->S, hipMemcpyDeviceToHost,
                           e->stream));
    YTA_HIP(host_wait(e->stream));
    return YTA_OK;
}

int doc_check_errors(yta_deepocsort *e) {
    for (int s = 0; s < e->S; ++s) {
        const int err = e->h_cnt[s].err;
        if (err) {
            set_error("stream %d: device error flags 0x%x (%s%s%s%s)", s, err,
                      err & ERR_GIOU ? "giou enclosure not positive (iou.py:58 assert) " : "",
                      err & ERR_SOLVER ? "assignment solver failure " : "",
                      err & ERR_TRACK_CAPACITY ? "track capacity exceeded " : "",
                      err & ERR_DET_CAPACITY ? "too many detections " : "");
            return (err & (ERR_TRACK_CAPACITY | ERR_DET_CAPACITY)) ? YTA_ERR_CAPACITY
                   : (err & ERR_GIOU)                              ? YTA_ERR_INVALID
                                                                   : YTA_ERR_HIP;
        }
    }
    return YTA_OK;
}

int doc_reserve(yta_deepocsort *e, int cap, int maxd) {
    if (cap <= e->CAP && maxd <= e->MAXD) return YTA_OK;
    cap = std::max(cap, e->CAP);
    maxd = std::max(maxd, e->MAXD);
    YTA_HIP(host_wait(e->stream));
    yta_deepocsort *n = new (std::nothrow) yta_deepocsort();
    YTA_CHECK(n, YTA_ERR_NOMEM, "out of host memory");
    n->device = e->device;
    n->S = e->S;
    n->CAP = cap;
    n->MAXD = maxd;
    n->D = e->D;
    n->prm = e->prm;
    n->stream = e->stream;
    int rc = doc_alloc(n);
    const size_t S = e->S, oc = e->CAP, nc = cap, Dd = std::max(e->D, 1);
    auto copy2d = [&](void *dst, size_t dp, const void *src, size_t sp, size_t w) -> int {
        YTA_HIP(hipMemcpy2DAsync(dst, dp, src, sp, w, S, hipMemcpyDeviceToDevice, e->stream));
        return YTA_OK;
    };
    if (!rc) rc = copy2d(n->a.rec, nc * sizeof(DocTrack), e->a.rec, oc * sizeof(DocTrack),
                         oc * sizeof(DocTrack));
    if (!rc) rc = copy2d(n->a.emb, nc * Dd * 8, e->a.emb, oc * Dd * 8, oc * Dd * 8);
    if (!rc) rc = copy2d(n->a.list, nc * 4, e->a.list, oc * 4, oc * 4);
    if (!rc) {
        std::vector<int> fl(nc * S), old(oc * S);
        std::vector<DocCounters> cnt(S);
        hipError_t he = hipMemcpyAsync(old.data(), e->a.free_list, sizeof(int) * oc * S,
                                       hipMemcpyDeviceToHost, e->stream);
        if (he == hipSuccess)
            he = hipMemcpyAsync(cnt.data(), e->a.cnt, sizeof(DocCounters) * S,
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
                he = hipMemcpy(n->a.cnt, cnt.data(), sizeof(DocCounters) * S,
                               hipMemcpyHostToDevice);
        }
        if (he != hipSuccess) {
            set_error("reserve: %s", hipGetErrorString(he));
            rc = YTA_ERR_HIP;
        }
    }
    if (rc) {
        n->stream = nullptr;
        doc_release(n);
        delete n;
        return rc;
    }
    memcpy(n->h_cnt, e->h_cnt, sizeof(DocCounters) * S);
    doc_release(e);
    e->CAP = n->CAP;
    e->MAXD = n->MAXD;
    e->allocs.swap(n->allocs);
    e->a = n->a;
    e->lds = n->lds;
    e->h_off = n->h_off;
    e->h_wh = n->h_wh;
    e->h_warp = n->h_warp;
    e->h_cnt = n->h_cnt;
    e->d_off = n->d_off;
    e->d_wh = n->d_wh;
    e->d_warp = n->d_warp;
    n->h_off = n->h_wh = nullptr;
    n->h_warp = nullptr;
    n->h_cnt = nullptr;
    n->stream = nullptr;
    delete n;
    return YTA_OK;
}

}  // namespace

extern "C" {

int yta_deepocsort_create(int device, int n_streams, int track_capacity, int max_dets,
                          int feat_dim, const yta_deepocsort_params *params,
                          yta_deepocsort **engine) {
    YTA_CHECK(engine && params, YTA_ERR_INVALID, "null engine/params");
    YTA_CHECK(n_streams > 0 && track_capacity > 0 && max_dets > 0, YTA_ERR_INVALID,
              "n_streams, track_capacity and max_dets must be positive");
    YTA_CHECK(params->delta_t >= 0 && params->delta_t <= OC_DT_MAX, YTA_ERR_INVALID,
              "delta_t must be in [0, %d]", OC_DT_MAX);
    YTA_CHECK(params->asso_func >= 0 && params->asso_func <= 4, YTA_ERR_INVALID,
              "asso_func must be 0..4 (iou, giou, diou, ciou, centroid)");
    YTA_CHECK(params->embedding_off || feat_dim > 0, YTA_ERR_INVALID,
              "embeddings need feat_dim > 0");
    YTA_CHECK(params->det_thresh < 1.0, YTA_ERR_INVALID, "det_thresh must be < 1 (trust weight)");
    *engine = nullptr;
    int rc = select_device(device);
    if (rc) return rc;
    yta_deepocsort *e = new (std::nothrow) yta_deepocsort();
    YTA_CHECK(e, YTA_ERR_NOMEM, "out of host memory");
    e->device = device;
    e->S = n_streams;
    e->CAP = track_capacity;
    e->MAXD = max_dets;
    e->D = params->embedding_off ? 0 : feat_dim;
    e->prm = *params;
    hipError_t he = hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking);
    if (he != hipSuccess) {
        set_error("hipStreamCreate: %s", hipGetErrorString(he));
        delete e;
        return YTA_ERR_HIP;
    }
    rc = doc_alloc(e);
    if (!rc) rc = yta_deepocsort_reset(e);
    if (rc) {
        yta_deepocsort_destroy(e);
        return rc;
    }
    *engine = e;
    return YTA_OK;
}

int yta_deepocsort_destroy(yta_deepocsort *e) {
    if (!e) return YTA_OK;
    (void)hipSetDevice(e->device);
    if (e->stream) (void)host_wait(e->stream);
    doc_release(e);
    e->mask.release();
    if (e->h_dets) (void)hipHostFree(e->h_dets);
    if (e->d_det_in) (void)hipFree(e->d_det_in);
    if (e->h_feat) (void)hipHostFree(e->h_feat);
    if (e->d_feat) (void)hipFree(e->d_feat);
    if (e->stream) (void)hipStreamDestroy(e->stream);
    delete e;
    return YTA_OK;
}

int yta_deepocsort_reset(yta_deepocsort *e) {
    YTA_CHECK(e, YTA_ERR_INVALID, "null engine");
    YTA_HIP(hipSetDevice(e->device));
    hipLaunchKernelGGL(k_doc_reset, dim3(e->S), dim3(256), 0, e->stream, e->a, 0);
    YTA_HIP(hipGetLastError());
    YTA_HIP(host_wait(e->stream));
    memset(e->h_cnt, 0, sizeof(DocCounters) * e->S);
    return YTA_OK;
}

int yta_deepocsort_capacity(yta_deepocsort *e, int *track_capacity, int *max_dets) {
    YTA_CHECK(e && track_capacity && max_dets, YTA_ERR_INVALID, "null argument");
    *track_capacity = e->CAP;
    *max_dets = e->MAXD;
    return YTA_OK;
}

int yta_deepocsort_update(yta_deepocsort *e, const double *dets, const int *det_offsets,
                          const float *feats, const double *warps, const int *img_wh,
                          long long *next_id, double *out, int out_capacity, int *out_offsets) {
    YTA_CHECK(e && det_offsets && out_offsets, YTA_ERR_INVALID, "null argument");
    YTA_HIP(hipSetDevice(e->device));
    const int S = e->S;
    YTA_CHECK(det_offsets[0] == 0, YTA_ERR_INVALID, "det_offsets[0] must be 0");
    YTA_CHECK(img_wh || e->prm.asso_func != 4, YTA_ERR_INVALID, "centroid needs img_wh");
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
        const int rc = doc_reserve(e, need_c > e->CAP ? std::max(need_c, 2 * e->CAP) : e->CAP,
                                   need_d > e->MAXD ? std::max(need_d, 2 * e->MAXD) : e->MAXD);
        if (rc) return rc;
    }
    const long long total = det_offsets[S];
    YTA_CHECK(total == 0 || dets, YTA_ERR_INVALID, "null dets");
    if (total > e->det_cap) {
        if (e->d_det_in) (void)hipFree(e->d_det_in);
        if (e->h_dets) (void)hipHostFree(e->h_dets);
        e->d_det_in = nullptr;
        e->h_dets = nullptr;
        e->det_cap = 0;
        const long long cap = std::max<long long>(2 * total, 1024);
        YTA_HIP(hipMalloc((void **)&e->d_det_in, sizeof(double) * 6 * cap));
        YTA_HIP(hipHostMalloc((void **)&e->h_dets, sizeof(double) * 6 * cap, hipHostMallocDefault));
        e->det_cap = cap;
    }
    if (total) {
        memcpy(e->h_dets, dets, sizeof(double) * 6 * total);
        YTA_HIP(hipMemcpyAsync(e->d_det_in, e->h_dets, sizeof(double) * 6 * total,
                               hipMemcpyHostToDevice, e->stream));
    }
    const int D = e->D;
    if (D > 0 && total) {   // feats: rows of the kept detections (conf > det_thresh), packed
        if (total > e->feat_cap) {
            if (e->d_feat) (void)hipFree(e->d_feat);
            if (e->h_feat) (void)hipHostFree(e->h_feat);
            e->d_feat = nullptr;
            e->h_feat = nullptr;
            e->feat_cap = 0;
            const long long cap = std::max<long long>(2 * total, 1024);
            YTA_HIP(hipMalloc((void **)&e->d_feat, sizeof(float) * D * cap));
            YTA_HIP(hipHostMalloc((void **)&e->h_feat, sizeof(float) * D * cap,
                                  hipHostMallocDefault));
            e->feat_cap = cap;
        }
        long long k = 0;
        for (long long r = 0; r < total; ++r)
            if (dets[r * 6 + 4] > e->prm.det_thresh) {
                YTA_CHECK(feats, YTA_ERR_INVALID, "null feats with kept detections");
                memcpy(e->h_feat + r * D, feats + k * D, sizeof(float) * D);
                ++k;
            }
        YTA_HIP(hipMemcpyAsync(e->d_feat, e->h_feat, sizeof(float) * D * total,
                               hipMemcpyHostToDevice, e->stream));
    }
    memcpy(e->h_off, det_offsets, sizeof(int) * (S + 1));
    YTA_HIP(hipMemcpyAsync(e->d_off, e->h_off, sizeof(int) * (S + 1), hipMemcpyHostToDevice,
                           e->stream));
    if (img_wh) {
        memcpy(e->h_wh, img_wh, sizeof(int) * 2 * S);
        YTA_HIP(hipMemcpyAsync(e->d_wh, e->h_wh, sizeof(int) * 2 * S, hipMemcpyHostToDevice,
                               e->stream));
    }
    if (warps) {
        memcpy(e->h_warp, warps, sizeof(double) * 6 * S);
        YTA_HIP(hipMemcpyAsync(e->d_warp, e->h_warp, sizeof(double) * 6 * S,
                               hipMemcpyHostToDevice, e->stream));
    }
    if (next_id) {
        for (int s = 0; s < S; ++s) e->h_cnt[s].next_id = next_id[s];
        YTA_HIP(hipMemcpy2DAsync(&e->a.cnt[0].next_id, sizeof(DocCounters),
                                 &e->h_cnt[0].next_id, sizeof(DocCounters), sizeof(long long), S,
                                 hipMemcpyHostToDevice, e->stream));
    }
    int rc = doc_launch(e, e->d_det_in, e->d_off, e->d_feat, warps ? e->d_warp : nullptr,
                        img_wh ? e->d_wh : nullptr, e->a.out, nullptr);
    if (rc) return rc;
    rc = doc_read_counters(e);
    if (rc) return rc;
    if (next_id)   // the device counters have advanced: hand them back even on an error below
        for (int s = 0; s < S; ++s) next_id[s] = e->h_cnt[s].next_id;
    rc = doc_check_errors(e);
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

int yta_deepocsort_update_device(yta_deepocsort *e, const double *d_dets,
                                 const int *d_det_offsets, const float *d_feats,
                                 const double *d_warps, const int *d_img_wh, double *d_out,
                                 int *d_out_counts) {
    YTA_CHECK(e && d_det_offsets && d_out, YTA_ERR_INVALID, "null argument");
    YTA_CHECK(e->D == 0 || d_feats, YTA_ERR_INVALID, "null feats");
    YTA_CHECK(d_img_wh || e->prm.asso_func != 4, YTA_ERR_INVALID, "centroid needs img_wh");
    return doc_launch(e, d_dets, d_det_offsets, d_feats, d_warps, d_img_wh, d_out, d_out_counts);
}

int yta_deepocsort_sync(yta_deepocsort *e) {
    YTA_CHECK(e, YTA_ERR_INVALID, "null engine");
    const int rc = doc_read_counters(e);
    if (rc) return rc;
    return doc_check_errors(e);
}

int yta_deepocsort_get_state(yta_deepocsort *e, int stream, int *n_tracks, long long *ints,
                             double *x, double *P, double *emb) {
    YTA_CHECK(e && n_tracks && ints && x && P, YTA_ERR_INVALID, "null argument");
    YTA_CHECK(stream >= 0 && stream < e->S, YTA_ERR_INVALID, "bad stream %d", stream);
    YTA_HIP(hipSetDevice(e->device));
    const int rc = doc_read_counters(e);
    if (rc) return rc;
    const DocCounters c = e->h_cnt[stream];
    const long long tb = (long long)stream * e->CAP;
    std::vector<int> lst(c.n_trk);
    std::vector<DocTrack> rec(e->CAP);
    if (c.n_trk)
        YTA_HIP(hipMemcpy(lst.data(), e->a.list + tb, sizeof(int) * c.n_trk, hipMemcpyDeviceToHost));
    YTA_HIP(hipMemcpy(rec.data(), e->a.rec + tb, sizeof(DocTrack) * e->CAP, hipMemcpyDeviceToHost));
    for (int i = 0; i < c.n_trk; ++i) {
        const DocTrack &r = rec[lst[i]];
        long long *ii = ints + 7LL * i;
        ii[0] = r.id;
        ii[1] = r.age;
        ii[2] = r.hits;
        ii[3] = r.hit_streak;
        ii[4] = r.tsu;
        ii[5] = (r.flags & OF_OBSERVED) ? 1 : 0;
        ii[6] = (r.flags & OF_FROZEN) ? 1 : 0;
        for (int k = 0; k < 8; ++k) x[8LL * i + k] = r.kf.x[k];
        double *M = P + 64LL * i;
        for (int k = 0; k < 64; ++k) M[k] = 0.0;
        for (int g = 0; g < 2; ++g)
            for (int a0 = 0; a0 < 4; ++a0)
                for (int b0 = 0; b0 < 4; ++b0)
                    M[dk_glob(g, a0) * 8 + dk_glob(g, b0)] = r.kf.p[g][4 * a0 + b0];
        if (emb && e->D)
            YTA_HIP(hipMemcpy(emb + (long long)i * e->D, e->a.emb + (tb + lst[i]) * e->D,
                              sizeof(double) * e->D, hipMemcpyDeviceToHost));
    }
    *n_tracks = c.n_trk;
    return YTA_OK;
}

int yta_deepocsort_stats(yta_deepocsort *e, long long *stats) {
    YTA_CHECK(e && stats, YTA_ERR_INVALID, "null argument");
    const int rc = doc_read_counters(e);
    if (rc) return rc;
    for (int k = 0; k < 8; ++k) stats[k] = 0;
    for (int s = 0; s < e->S; ++s) {
        const DocCounters &c = e->h_cnt[s];
        const long long v[8] = {c.n_dets, c.n_high, 0, c.n_trk, c.n_out, c.n_births, c.lap_calls,
                                c.fast_path};
        for (int k = 0; k < 8; ++k) stats[k] += v[k];
    }
    return YTA_OK;
}

int yta_kf8_run(int device, int n, int steps, const double *b0, const double *b,
                const double *warps, double *x_out, double *P_out) {
    YTA_CHECK(n > 0 && steps >= 0 && b0 && (b || steps == 0) && x_out && P_out, YTA_ERR_INVALID,
              "bad arguments");
    int rc = select_device(device);
    if (rc) return rc;
    double *d_b0 = nullptr, *d_b = nullptr, *d_w = nullptr, *d_x = nullptr, *d_P = nullptr;
    const size_t nb = sizeof(double) * 4 * (size_t)n * std::max(steps, 1);
    const size_t nw = sizeof(double) * 6 * (size_t)n * std::max(steps, 1);
    hipError_t he = hipMalloc((void **)&d_b0, sizeof(double) * 4 * n);
    if (he == hipSuccess) he = hipMalloc((void **)&d_b, nb);
    if (he == hipSuccess && warps) he = hipMalloc((void **)&d_w, nw);
    if (he == hipSuccess) he = hipMalloc((void **)&d_x, sizeof(double) * 8 * n);
    if (he == hipSuccess) he = hipMalloc((void **)&d_P, sizeof(double) * 64 * n);
    if (he == hipSuccess) he = hipMemcpy(d_b0, b0, sizeof(double) * 4 * n, hipMemcpyHostToDevice);
    if (he == hipSuccess && steps)
        he = hipMemcpy(d_b, b, sizeof(double) * 4 * (size_t)n * steps, hipMemcpyHostToDevice);
    if (he == hipSuccess && warps && steps)
        he = hipMemcpy(d_w, warps, sizeof(double) * 6 * (size_t)n * steps, hipMemcpyHostToDevice);
    if (he == hipSuccess) {
        hipLaunchKernelGGL(k_kf8_run, dim3((n + 63) / 64), dim3(64), 0, 0, n, steps, 3, d_b0, d_b,
                           d_w, d_x, d_P);
        he = hipGetLastError();
    }
    if (he == hipSuccess) he = hipMemcpy(x_out, d_x, sizeof(double) * 8 * n, hipMemcpyDeviceToHost);
    if (he == hipSuccess) he = hipMemcpy(P_out, d_P, sizeof(double) * 64 * n, hipMemcpyDeviceToHost);
    (void)hipFree(d_b0);
    (void)hipFree(d_b);
    (void)hipFree(d_w);
    (void)hipFree(d_x);
    (void)hipFree(d_P);
    if (he != hipSuccess) {
        set_error("yta_kf8_run: %s", hipGetErrorString(he));
        return YTA_ERR_HIP;
    }
    return YTA_OK;
}

int yta_deepocsort_lap_stats(yta_deepocsort *e, long long *stats, int n) {
    YTA_CHECK(e && (stats || n <= 0), YTA_ERR_INVALID, "null argument");
    const int rc = doc_read_counters(e);
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

int yta_deepocsort_hip_stream(yta_deepocsort *e, void **stream) {
    YTA_CHECK(e && stream, YTA_ERR_INVALID, "null argument");
    *stream = (void *)e->stream;
    return YTA_OK;
}

#ifdef YTA_STAMPS
int yta_deepocsort_debug_stamps(unsigned long long *out) {
    YTA_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * 128));
    return YTA_OK;
}
#endif


// ---- stream subsets (subset.hpp): the listed streams updated, every other stream untouched
int yta_deepocsort_reset_stream(yta_deepocsort *e, int stream) {
    YTA_CHECK(e, YTA_ERR_INVALID, "null engine");
    YTA_CHECK(stream >= 0 && stream < e->S, YTA_ERR_INVALID, "stream %d outside 0..%d", stream,
              e->S - 1);
    YTA_HIP(hipSetDevice(e->device));
    hipLaunchKernelGGL(k_doc_reset, dim3(1), dim3(256), 0, e->stream, e->a, stream);
    YTA_HIP(hipGetLastError());
    YTA_HIP(host_wait(e->stream));
    return doc_read_counters(e);
}

int yta_deepocsort_update_device_masked(yta_deepocsort *e, const int *d_active, const double *d_dets, const int *d_det_offsets, const float *d_feats, const double *d_warps, const int *d_img_wh, double *d_out, int *d_out_counts) {
    YTA_CHECK(e, YTA_ERR_INVALID, "null engine");
    e->mask.req_dev = d_active;
    const int rc = yta_deepocsort_update_device(e, d_dets, d_det_offsets, d_feats, d_warps, d_img_wh, d_out, d_out_counts);
    e->mask.req_dev = nullptr;
    return rc;
}

int yta_deepocsort_update_streams(yta_deepocsort *e, int n_streams, const int *stream_ids, const double *dets, const int *det_offsets, const float *feats, const double *warps, const int *img_wh,
                           long long *next_id, double *out, int out_capacity, int *out_offsets) {
    YTA_CHECK(e && out_offsets, YTA_ERR_INVALID, "null argument");
    YTA_HIP(hipSetDevice(e->device));
    const int S = e->S;
    std::vector<int> mask, off, full_oo(S + 1, 0);
    int rc = subset_expand(S, n_streams, stream_ids, det_offsets, mask, off);
    if (rc) return rc;
    std::vector<long long> nid(S);
    if (next_id) {   // the skipped streams keep their device counters: read them first
        rc = doc_read_counters(e);
        if (rc) return rc;
        for (int s = 0; s < S; ++s) nid[s] = e->h_cnt[s].next_id;
        for (int k = 0; k < n_streams; ++k) nid[stream_ids[k]] = next_id[k];
    }
    std::vector<int> wh;
    if (img_wh) wh = subset_spread<int>(S, n_streams, stream_ids, img_wh, 2, 1);
    std::vector<double> w;
    if (warps) {
        w = subset_spread<double>(S, n_streams, stream_ids, warps, 6, 0.0);
        for (int s = 0; s < S; ++s)
            if (!mask[s]) w[6 * s] = w[6 * s + 4] = 1.0;   // identity for the skipped streams
    }
    e->mask.req_host = mask.data();
    rc = yta_deepocsort_update(e, dets, off.data(), feats, warps ? w.data() : nullptr, img_wh ? wh.data() : nullptr, next_id ? nid.data() : nullptr, out,
                        out_capacity, full_oo.data());
    e->mask.req_host = nullptr;
    if (next_id)
        for (int k = 0; k < n_streams; ++k) next_id[k] = nid[stream_ids[k]];
    if (rc) return rc;
    subset_compact(n_streams, stream_ids, full_oo, out_offsets);
    return YTA_OK;
}

}  // extern "C"
