// OCSORT update() for S independent streams on gfx950, all tracker state resident in HBM.
//
// Follows boxmot/trackers/ocsort/ocsort.py:188-379 with boxmot/utils/association.py:8-28,
// :111-201 and the live paths of ocsort_kf.py (kf_ocsort.hpp).  One frame = one launch of
// three kernels (k_oc_pre: A-C, one block per stream; k_oc_cost: D over the whole chip;
// k_oc_assoc: E-J, one block per stream) whose phases keep the reference's list semantics:
//   A  predict every tracker (x[6] clamp, Kalman predict, age / hit_streak / time_since_update,
//      :168-181), predicted boxes; trackers whose box has a NaN are dropped (:254-264)
//   B  per-column association inputs in tracker order: box, velocity (or 0), k_previous_obs
//      (:14-22), last observation
//   C  detections: conf > det_thresh (first / OCR rounds), 0.1 < conf < det_thresh (BYTE round)
//   D  dense asso (iou / giou / diou / ciou / centroid, dets x trackers) and the OCSORT cost
//      -(asso + angle), angle = ((valid * (pi/2 - |acos(clip(v . dir))|) / pi) * inertia) * score
//   E  fast path when every row and column has at most one asso > thr (and one has exactly one),
//      else the padded dense LAP (lap_dense.hpp, one wave); matches filtered by asso >= thr; the
//      unmatched lists in the reference's order (scan order, then the filtered pairs)
//   F  BYTE round (use_byte) and G  OCR round: asso of the leftovers (OCR: against the trackers'
//      last observations), LAP on -asso when its max exceeds thr, lists replaced by the sorted
//      set differences (np.setdiff1d)
//   H  tracker updates, one thread per tracker: velocity from the observation delta_t ages back,
//      observation ring, Kalman update with the observation-centric re-update (freeze on the first
//      miss, restore + virtual-trajectory replay on re-acquisition)
//   I  births in unmatched-list order; J  output rows in reversed tracker order, then trackers
//      unseen for more than max_age frames are dropped.
#include <algorithm>
#include <cstring>
#include <new>
#include <vector>

#include "kf_ocsort.hpp"
#include "ocsort_common.hpp"
#include "subset.hpp"

namespace yta {
namespace {

struct OcTrack {                   // one slot
    Kf7 kf;                        // live filter
    Kf7 fz;                        // frozen copy (freeze, ocsort_kf.py:383-387)
    double hist_z[4];              // last non-None entry of history_obs
    double last_obs[5];            // last_observation (placeholder -1s)
    double vel[2];                 // velocity (dy, dx)
    double conf, cls;
    double obs[OC_DT_MAX][5];      // ring of the latest delta_t observations
    long long id;
    int obs_age[OC_DT_MAX];
    int obs_n;                     // observations inserted so far (ring position = n % delta_t)
    int det_ind, age, hits, hit_streak, tsu, flags, hist_since;
};

struct OcCounters {                // one per stream
    long long next_id;             // KalmanBoxTracker.count
    int frame;
    int n_trk, n_free;
    int n_dets, n_high, n_second, n_out, n_births;
    int lap_calls, fast_path;
    int err;
    int lap_done;                  // first round solved by k_oc_lap this frame
    LapStats ls;                   // cumulative solver counters
    int pad[13];
};
static_assert(sizeof(OcCounters) == 128, "OcCounters layout");

struct OcArgs {
    int S, CAP, MAXD;
    double det_thresh, thr, inertia;
    int max_age, min_hits, delta_t, asso, use_byte;
    const double *det_in;          // packed rows of 6
    const int *det_off;            // S + 1
    const int *img_wh;             // S x (w, h) or null
    OcTrack *rec;                  // [S*CAP]
    int *list, *free_list;         // [S*CAP]
    OcCounters *cnt;
    // per frame
    int *hi_row, *lo_row;          // [S*MAXD] input rows of the first / BYTE detections
    Box *cbox;                     // [S*CAP] predicted boxes (tracker order)
    double *cvel, *ckobs, *clast;  // [S*CAP] x 2 / 5 / 5
    int *nan_flag;                 // [S*CAP]
    double *mat, *mat2;            // [S*MAXD*CAP] asso, cost
    int *rmatch;                   // [S*MAXD] first-round column of each row (-1)
    int *cmatched;                 // [S*CAP]
    int *udet, *utrk, *tmp;        // [S*(MAXD+CAP)]
    int *upd;                      // [S*CAP] update source per tracker: input row, -1 none
    unsigned char *lap_ws;         // per stream (n > OC_LDS_LAP_N)
    unsigned char *lap_csr;         // per stream: the replay's row entries (nullptr: n < LAPB_MIN_N)
    long long lap_csr_stride;
    long long lap_ws_stride;
    double *pre_u, *pre_s2;        // [S*MAXD] first-round row pre-pass (lap_rect.hpp)
    int *pre_x;
    double *out;                   // [S*CAP*8]
    int *out_counts;
    const int *active;             // [S] nonzero = update the stream this frame; null = all
};

// k_previous_obs (ocsort.py:14-22) from the ring
__device__ __forceinline__ void k_prev_obs(const OcTrack &r, int dt, double *o) {
    if (r.obs_n == 0) {
        for (int k = 0; k < 5; ++k) o[k] = -1.0;
        return;
    }
    const int m = r.obs_n < dt ? r.obs_n : dt;
    for (int i = 0; i < dt; ++i) {
        const int want = r.age - (dt - i);
        for (int e = 0; e < m; ++e)
            if (r.obs_age[e] == want) {
                for (int k = 0; k < 5; ++k) o[k] = r.obs[e][k];
                return;
            }
    }
    for (int k = 0; k < 5; ++k) o[k] = r.last_obs[k];   // the newest observation
}

// KalmanBoxTracker.update (ocsort.py:130-166) + KalmanFilter.update (ocsort_kf.py:437-526)
__device__ void tracker_update(OcTrack &r, const double *det, int det_local, int dt) {
    if (!det) {                                   // update(None)
        r.det_ind = -1;
        if (r.flags & OF_OBSERVED) {              // freeze on the first miss
            r.fz = r.kf;
            r.flags |= OF_SAVED;
        }
        r.flags &= ~OF_OBSERVED;
        r.hist_since += 1;
        return;
    }
    double bbox[5] = {det[0], det[1], det[2], det[3], det[4]};
    r.det_ind = det_local;
    r.conf = bbox[4];
    r.cls = det[5];
    if (np_sum5(r.last_obs) >= 0) {
        const double *prev = r.last_obs;
        const int m = r.obs_n < dt ? r.obs_n : dt;
        bool found = false;
        for (int i = 0; i < dt && !found; ++i) {
            const int want = r.age - (dt - i);
            for (int e = 0; e < m; ++e)
                if (r.obs_age[e] == want) {
                    prev = r.obs[e];
                    found = true;
                    break;
                }
        }
        // speed_direction (ocsort.py:57-62)
        const double cx1 = (prev[0] + prev[2]) / 2.0, cy1 = (prev[1] + prev[3]) / 2.0;
        const double cx2 = (bbox[0] + bbox[2]) / 2.0, cy2 = (bbox[1] + bbox[3]) / 2.0;
        const double sy = cy2 - cy1, sx = cx2 - cx1;
        const double nrm = sqrt(sy * sy + sx * sx) + 1e-6;
        r.vel[0] = sy / nrm;
        r.vel[1] = sx / nrm;
        r.flags |= OF_VELOCITY;
    }
    for (int k = 0; k < 5; ++k) r.last_obs[k] = bbox[k];
    const int slot = r.obs_n % dt;
    for (int k = 0; k < 5; ++k) r.obs[slot][k] = bbox[k];
    r.obs_age[slot] = r.age;
    r.obs_n += 1;
    r.tsu = 0;
    r.hits += 1;
    r.hit_streak += 1;
    double z[4];
    oc_bbox_to_z(bbox, z);
    if (!(r.flags & OF_OBSERVED) && (r.flags & OF_SAVED)) {
        // unfreeze: restore, replay the virtual trajectory from the last kept observation
        r.kf = r.fz;
        r.flags &= ~OF_SAVED;   // the restored attr_saved is the one before the freeze: None
        kf7_replay(r.kf, r.hist_z, z, r.hist_since + 1, r.hist_z);
    } else {
        for (int k = 0; k < 4; ++k) r.hist_z[k] = z[k];
    }
    r.hist_since = 0;
    r.flags |= OF_OBSERVED;
    kf7_correct(r.kf, z);
}

// NT: OC_T, or 1024 with few streams (one block per stream takes the lists; only sh.wsum is
// shared state sized per wave)
template <int NT>
__global__ __launch_bounds__(NT) void k_oc_pre(OcArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    __shared__ OcShared sh;
    const int s = blockIdx.x, t = threadIdx.x, nt = blockDim.x;
    if (a.active && !a.active[s]) return;   // stream not updated this frame
    OcCounters *c = a.cnt + s;
    const long long tb = (long long)s * a.CAP, db = (long long)s * a.MAXD;
    const long long mb = (long long)s * (a.MAXD > 4 ? a.MAXD : 4) * a.CAP;
    const long long ub = (long long)s * (a.MAXD + a.CAP);
    unsigned char *gws = a.lap_ws + s * a.lap_ws_stride;
    int nd = a.det_off[s + 1] - a.det_off[s];
    if (nd > a.MAXD || nd < 0) {
        if (t == 0) atomicOr(&c->err, ERR_DET_CAPACITY);
        nd = nd < 0 ? 0 : a.MAXD;
    }
    const double *din = a.det_in + (long long)a.det_off[s] * 6;
    const double img_w = a.img_wh ? (double)a.img_wh[2 * s] : 0.0;
    const double img_h = a.img_wh ? (double)a.img_wh[2 * s + 1] : 0.0;
    const int frame = c->frame + 1;
    int n_trk = c->n_trk;
    const int dt = a.delta_t;
    int *list = a.list + tb;
    YTA_STAMP_BASE(0);
    YTA_STAMP(0);

    // ---- A: predict (:250-264)
    for (int i = t; i < n_trk; i += nt) {
        OcTrack &r = a.rec[tb + list[i]];
        if (r.kf.x[6] + r.kf.x[2] <= 0) r.kf.x[6] *= 0.0;
        kf7_predict(r.kf);
        r.age += 1;
        if (r.tsu > 0) r.hit_streak = 0;
        r.tsu += 1;
        double b[4];
        oc_x_to_bbox(r.kf.x, b);
        a.nan_flag[tb + i] = (b[0] != b[0]) || (b[1] != b[1]) || (b[2] != b[2]) || (b[3] != b[3]);
        a.cbox[tb + i] = Box{b[0], b[1], b[2], b[3]};
    }
    block_sync();
    // ---- B: drop NaN trackers (order kept), free their slots; column inputs in tracker order
    YTA_STAMP(1);
    {
        int n_free = c->n_free;
        const int n_nan = block_compact(n_trk, sh.wsum, [&](int i) { return a.nan_flag[tb + i] != 0; },
                                        [&](int i, int pos) { a.tmp[ub + pos] = list[i]; });
        block_sync();   // the compaction's tmp stores (other threads' runs) before their reads
        for (int k = t; k < n_nan; k += nt) a.free_list[tb + n_free + k] = a.tmp[ub + k];
        n_free += n_nan;
        block_sync();
        const int n_keep = block_compact(n_trk, sh.wsum, [&](int i) { return a.nan_flag[tb + i] == 0; },
                                         [&](int i, int pos) {
                                             a.tmp[ub + pos] = list[i];
                                             a.upd[tb + pos] = i;   // its old position
                                         });
        block_sync();
        Box *bscratch = reinterpret_cast<Box *>(a.mat2 + mb);
        for (int j = t; j < n_keep; j += nt) {
            const OcTrack &r = a.rec[tb + a.tmp[ub + j]];
            bscratch[j] = a.cbox[tb + a.upd[tb + j]];
            double ko[5];
            k_prev_obs(r, dt, ko);
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
            a.cbox[tb + j] = bscratch[j];
            a.cmatched[tb + j] = 0;
            a.nan_flag[tb + j] = 0;
        }
        n_trk = n_keep;
        if (t == 0) c->n_free = n_free;
        block_sync();
    }
    for (int j = t; j < n_trk; j += nt) a.upd[tb + j] = -1;
    // ---- C: detection split (:241-247)
    YTA_STAMP(2);
    const int n_hi = block_compact(nd, sh.wsum, [&](int i) { return din[i * 6 + 4] > a.det_thresh; },
                                   [&](int i, int pos) { a.hi_row[db + pos] = i; });
    const int n_lo = block_compact(
        nd, sh.wsum,
        [&](int i) { const double cf = din[i * 6 + 4]; return cf > 0.1 && cf < a.det_thresh; },
        [&](int i, int pos) { a.lo_row[db + pos] = i; });
    block_sync();
    for (int i = t; i < n_hi; i += nt) a.rmatch[db + i] = 0;
    if (t == 0) {
        c->n_trk = n_trk;          // NaN-culled
        c->n_high = n_hi;
        c->n_second = n_lo;
    }
    (void)img_w;
    (void)img_h;
    (void)frame;
    (void)lds;
    (void)gws;
}

// k_oc_cost: the first round's dense asso / cost matrices of every stream over the whole chip
// (association.py:111-150; costs -(asso + angle), :155-170), with the per-row / per-column counts
// of asso > thr that decide the fast path (:156-159).
__global__ __launch_bounds__(OC_T) void k_oc_cost(OcArgs a) {
    const int s = blockIdx.y;
    if (a.active && !a.active[s]) return;   // stream not updated this frame
    OcCounters *c = a.cnt + s;
    const int n_trk = c->n_trk, n_hi = c->n_high;
    const long long nm = (long long)n_hi * n_trk;
    const long long tb = (long long)s * a.CAP, db = (long long)s * a.MAXD;
    const long long mb = (long long)s * (a.MAXD > 4 ? a.MAXD : 4) * a.CAP;
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
        // speed_direction_batch (:8-17): k-obs centre -> detection centre
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
        mat2[q] = -((v + angle) + 0.0);
        if (v > a.thr) {
            atomicAdd(&a.rmatch[db + i], 1);
            atomicAdd(&a.cmatched[tb + j], 1);
        }
    }
    if (giou_bad) atomicOr(&c->err, ERR_GIOU);
}

// Row pre-pass of the first-round solve (row minima, argmins, second minima of the cost matrix),
// chip-wide, so the stream block only walks the augmenting paths.
__global__ __launch_bounds__(OC_T) void k_oc_rowpre(OcArgs a) {
    const int s = blockIdx.y;
    if (a.active && !a.active[s]) return;   // stream not updated this frame
    const OcCounters *c = a.cnt + s;
    const long long db = (long long)s * a.MAXD;
    const long long mb = (long long)s * (a.MAXD > 4 ? a.MAXD : 4) * a.CAP;
    main_lap_pre(a.mat2 + mb, c->n_high, c->n_trk, a.pre_u + db, a.pre_x + db, a.pre_s2 + db);
}

// First-round solve, one LAP_T-thread block per stream (ocsort_common.hpp first_round_lap).
__global__ __launch_bounds__(LAP_T) void k_oc_lap(OcArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int s = blockIdx.x;
    if (a.active && !a.active[s]) return;   // stream not updated this frame
    OcCounters *c = a.cnt + s;
    const long long tb = (long long)s * a.CAP, db = (long long)s * a.MAXD;
    first_round_lap(a.mat2 + (long long)s * (a.MAXD > 4 ? a.MAXD : 4) * a.CAP, c->n_high, c->n_trk, a.rmatch + db, a.cmatched + tb, true,
                    a.pre_u + db, a.pre_x + db, a.pre_s2 + db, a.rmatch + db, lds,
                    lap_kernel_lds(a.CAP, a.MAXD), a.lap_ws + s * a.lap_ws_stride, &c->err,
                    &c->lap_done, &c->ls, a.lap_ws + (s + 1) * a.lap_ws_stride - tight_ws_bytes());
}

__global__ __launch_bounds__(OC_T) void k_oc_assoc(OcArgs a) {
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
    OcCounters *c = a.cnt + s;
    const long long tb = (long long)s * a.CAP, db = (long long)s * a.MAXD;
    const long long mb = (long long)s * (a.MAXD > 4 ? a.MAXD : 4) * a.CAP;
    const long long ub = (long long)s * (a.MAXD + a.CAP);
    unsigned char *gws = a.lap_ws + s * a.lap_ws_stride;
    const long long lds_bytes = oc_lds_bytes(a.CAP, a.MAXD);
    int nd = a.det_off[s + 1] - a.det_off[s];
    if (nd > a.MAXD || nd < 0) {
        if (t == 0) atomicOr(&c->err, ERR_DET_CAPACITY);
        nd = nd < 0 ? 0 : a.MAXD;
    }
    const double *din = a.det_in + (long long)a.det_off[s] * 6;
    const double img_w = a.img_wh ? (double)a.img_wh[2 * s] : 0.0;
    const double img_h = a.img_wh ? (double)a.img_wh[2 * s + 1] : 0.0;
    const int frame = c->frame + 1;
    int n_trk = c->n_trk;
    const int n_hi = c->n_high, n_lo = c->n_second;
    const int dt = a.delta_t;
    int *list = a.list + tb;
    YTA_STAMP_BASE(40);
    YTA_STAMP(0);
    auto hbox = [&](int i) { return box5(din + (long long)a.hi_row[db + i] * 6); };
    double *mat = a.mat + mb, *mat2 = a.mat2 + mb;
    int *udet = a.udet + ub, *utrk = a.utrk + ub;
    int n_ud = 0, n_ut = 0;

    // ---- D / E: first round (association.py:111-201)
    if (n_trk == 0) {
        for (int i = t; i < n_hi; i += nt) udet[i] = i;
        n_ud = n_hi;
        n_ut = 0;
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
        YTA_STAMP(3);
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
        YTA_STAMP(4);
        if (t == 0) { c->fast_path = fast; c->lap_calls = (fast || n_hi == 0) ? 0 : 1; }
        // matched columns; unmatched lists: scan order, then the filtered pairs in row order
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
            if (col >= 0 && !filtered(i)) a.upd[tb + col] = a.hi_row[db + i];
        }
        n_ud += nf;
        n_ut += nf;
        block_sync();
    }

    // ---- F: BYTE round (:289-313)
    YTA_STAMP(5);
    if (a.use_byte && n_lo > 0 && n_ut > 0) {
        const double mx = asso_matrix(
            a.asso, n_lo, n_ut, [&](int p) { return box5(din + (long long)a.lo_row[db + p] * 6); },
            [&](int k) { return a.cbox[tb + utrk[k]]; }, img_w, img_h, mat, lds, lds_bytes, &c->err,
            sh);
        if (mx > a.thr) {
            iou_lap(LapMat{mat, n_lo, n_ut, true}, a.rmatch + db, lds, lds_bytes, gws, &c->err, &c->ls,
                    a.lap_ws + (s + 1) * a.lap_ws_stride - tight_ws_bytes(), nullptr, nullptr,
                    nullptr, a.thr);
            for (int k = t; k < n_ut; k += nt) a.tmp[ub + k] = 0;   // taken flags
            block_sync();
            for (int p = t; p < n_lo; p += nt) {
                const int k = a.rmatch[db + p];
                if (k >= 0 && !(mat[(long long)p * n_ut + k] < a.thr)) {
                    a.upd[tb + utrk[k]] = a.lo_row[db + p];
                    a.tmp[ub + k] = 1;
                }
            }
            block_sync();
            // setdiff1d: the remaining tracker indices, sorted
            for (int k = t; k < n_ut; k += nt) a.nan_flag[tb + utrk[k]] = a.tmp[ub + k] ? 0 : 1;
            block_sync();
            n_ut = block_compact(n_trk, sh.wsum, [&](int j) { return a.nan_flag[tb + j] == 1; },
                                 [&](int j, int pos) { utrk[pos] = j; });
            for (int j = t; j < n_trk; j += nt) a.nan_flag[tb + j] = 0;
            if (t == 0) c->lap_calls += 1;
            block_sync();
        }
    }
    // ---- G: OCR round (:315-342)
    YTA_STAMP(6);
    if (n_ud > 0 && n_ut > 0) {
        const double mx = asso_matrix(
            a.asso, n_ud, n_ut, [&](int p) { return hbox(udet[p]); },
            [&](int k) { return box5(a.clast + (tb + utrk[k]) * 5); }, img_w, img_h, mat, lds,
            lds_bytes, &c->err, sh);
        if (mx > a.thr) {
            iou_lap(LapMat{mat, n_ud, n_ut, true}, a.rmatch + db, lds, lds_bytes, gws, &c->err, &c->ls,
                    a.lap_ws + (s + 1) * a.lap_ws_stride - tight_ws_bytes(), nullptr, nullptr,
                    nullptr, a.thr);
            // removed dets / trackers -> flags, then sorted set differences
            for (int i = t; i < n_hi; i += nt) a.tmp[ub + i] = 0;
            for (int j = t; j < n_trk; j += nt) a.nan_flag[tb + j] = 0;
            block_sync();
            for (int p = t; p < n_ud; p += nt) a.tmp[ub + udet[p]] = 1;        // in udet
            for (int k = t; k < n_ut; k += nt) a.nan_flag[tb + utrk[k]] = 1;   // in utrk
            block_sync();
            for (int p = t; p < n_ud; p += nt) {
                const int k = a.rmatch[db + p];
                if (k >= 0 && !(mat[(long long)p * n_ut + k] < a.thr)) {
                    a.upd[tb + utrk[k]] = a.hi_row[db + udet[p]];
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
    // ---- H: tracker updates (matched: det row; the rest: None)
    YTA_STAMP(7);
    for (int j = t; j < n_trk; j += nt) {
        OcTrack &r = a.rec[tb + list[j]];
        const int row = a.upd[tb + j];
        tracker_update(r, row >= 0 ? din + (long long)row * 6 : nullptr, row, dt);
    }
    block_sync();
    // ---- I: births in unmatched-list order (:347-349)
    YTA_STAMP(8);
    int n_free = c->n_free;
    int n_b = n_ud;
    if (n_b > n_free) {
        if (t == 0) atomicOr(&c->err, ERR_TRACK_CAPACITY);
        n_b = n_free;
    }
    const long long next_id = c->next_id;
    // a birth's record is built in LDS (the solver's arena is free by now) by its thread and
    // stored by the whole block in 8-B pieces, consecutive lanes on consecutive pieces (one thread
    // storing its record word by word beside the others' touched a line per birth and store)
    static_assert(sizeof(OcTrack) % 8 == 0, "OcTrack is stored in 8-B pieces");
    constexpr int REC_Q = (int)(sizeof(OcTrack) / 8);
    OcTrack *bstage = reinterpret_cast<OcTrack *>(lds);
    int bch = (int)(lds_bytes / (long long)sizeof(OcTrack));
    bch = bch < 1 ? 1 : (bch > nt ? nt : bch);
    for (int b0 = 0; b0 < n_b; b0 += bch) {
      const int mb_ = n_b - b0 < bch ? n_b - b0 : bch;
      for (int rr = t; rr < mb_; rr += nt) {
        const int b = b0 + rr;
        const int slot = a.free_list[tb + n_free - 1 - b];
        const double *dr = din + (long long)a.hi_row[db + udet[b]] * 6;
        OcTrack r;
        double z[4];
        oc_bbox_to_z(dr, z);
        kf7_init(z, r.kf);
        r.fz = r.kf;
        for (int k = 0; k < 4; ++k) r.hist_z[k] = 0.0;
        for (int k = 0; k < 5; ++k) r.last_obs[k] = -1.0;
        r.vel[0] = r.vel[1] = 0.0;
        r.conf = dr[4];
        r.cls = dr[5];
        r.id = next_id + b;
        r.obs_n = 0;
        for (int e = 0; e < OC_DT_MAX; ++e) r.obs_age[e] = -1;
        r.det_ind = a.hi_row[db + udet[b]];
        r.age = r.hits = r.hit_streak = r.tsu = 0;
        r.flags = 0;
        r.hist_since = 0;
        bstage[rr] = r;
        list[n_trk + b] = slot;
      }
      lds_sync();
      for (int q = t; q < mb_ * REC_Q; q += nt) {
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
    // ---- J: outputs in reversed tracker order, then drop trackers unseen > max_age (:350-379)
    YTA_STAMP(9);
    // every record read batched (block_compact_ld / batched_for2); the removal flags of the
    // pass go to nan_flag for the two removal compactions
    double *out = a.out + tb * 8;
    struct TrkState {
        int slot, tsu, hit_streak;
    };
    int *oslot = a.tmp + ub;   // the output trackers' slots, in output order
    const int n_out = block_compact_ld<8>(
        n_trk, sh.wsum, [&](int q) { return list[n_trk - 1 - q]; },
        [&](int, int slot) {
            const OcTrack &r = a.rec[tb + slot];
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
            const OcTrack &r = a.rec[tb + slot];
            OutRow o;
            if (np_sum5(r.last_obs) < 0) oc_x_to_bbox(r.kf.x, o.b);
            else for (int k = 0; k < 4; ++k) o.b[k] = r.last_obs[k];
            o.id = (double)(r.id + 1);
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
    YTA_STAMP(10);
    if (t == 0) {
        c->frame = frame;
        c->n_trk = n_live;
        c->n_free = n_free + n_dead;
        c->n_dets = nd;
        c->n_high = n_hi;
        c->n_second = n_lo;
        c->n_out = n_out;
        c->n_births = n_b;
        c->next_id = next_id + n_b;
        if (a.out_counts) a.out_counts[s] = n_out;
    }
}

__global__ void k_oc_reset(OcArgs a, int s0) {
    const int s = s0 + blockIdx.x;
    const long long tb = (long long)s * a.CAP;
    // births pop from the end of the free list: store it descending so slots fill from 0
    for (int i = threadIdx.x; i < a.CAP; i += blockDim.x) a.free_list[tb + i] = a.CAP - 1 - i;
    if (threadIdx.x == 0) {
        OcCounters z;
        memset(&z, 0, sizeof(z));
        z.n_free = a.CAP;
        a.cnt[s] = z;
    }
}

}  // namespace
}  // namespace yta

// ================================================================================== host engine
using namespace yta;

struct yta_ocsort {
    int device = 0, S = 0, CAP = 0, MAXD = 0;
    yta_ocsort_params prm{};
    hipStream_t stream = nullptr;
    std::vector<void *> allocs;
    OcArgs a{};
    double *h_dets = nullptr, *d_det_in = nullptr;
    long long det_cap = 0;
    int *h_off = nullptr, *d_off = nullptr, *h_wh = nullptr, *d_wh = nullptr;
    OcCounters *h_cnt = nullptr;
    size_t lds = 0;
    StreamMask mask;   // stream-subset updates (subset.hpp)
};

namespace {

template <typename T>
int oc_dalloc(yta_ocsort *e, T **p, long long n) {
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

#define OCALLOC(ptr, n)                      \
    do {                                     \
        int _rc = oc_dalloc(e, &(ptr), (n)); \
        if (_rc) return _rc;                 \
    } while (0)

int oc_alloc(yta_ocsort *e) {
    const long long S = e->S, CAP = e->CAP, MAXD = e->MAXD;
    OcArgs &a = e->a;
    const yta_ocsort_params &p = e->prm;
    a.S = e->S;
    a.CAP = e->CAP;
    a.MAXD = e->MAXD;
    a.det_thresh = p.det_thresh;
    a.thr = p.asso_threshold;
    a.inertia = p.inertia;
    a.max_age = p.max_age;
    a.min_hits = p.min_hits;
    a.delta_t = p.delta_t;
    a.asso = p.asso_func;
    a.use_byte = p.use_byte;
    OCALLOC(a.rec, S * CAP);
    OCALLOC(a.list, S * CAP);
    OCALLOC(a.free_list, S * CAP);
    OCALLOC(a.cnt, S);
    OCALLOC(a.hi_row, S * MAXD);
    OCALLOC(a.lo_row, S * MAXD);
    OCALLOC(a.cbox, S * CAP);
    OCALLOC(a.cvel, S * CAP * 2);
    OCALLOC(a.ckobs, S * CAP * 5);
    OCALLOC(a.clast, S * CAP * 5);
    OCALLOC(a.nan_flag, S * CAP);
    const long long mat = std::max<long long>(MAXD * CAP, 4 * CAP);   // (mat2 doubles as a Box
    OCALLOC(a.mat, S * mat);                                            //  scratch of CAP boxes)
    OCALLOC(a.mat2, S * mat);
    OCALLOC(a.rmatch, S * MAXD);
    OCALLOC(a.pre_u, S * MAXD);
    OCALLOC(a.pre_s2, S * MAXD);
    OCALLOC(a.pre_x, S * MAXD);
    OCALLOC(a.cmatched, S * CAP);
    OCALLOC(a.udet, S * (MAXD + CAP));
    OCALLOC(a.utrk, S * (MAXD + CAP));
    OCALLOC(a.tmp, S * (MAXD + CAP));
    OCALLOC(a.upd, S * CAP);
    OCALLOC(a.out, S * CAP * 8);
    const long long n = std::max(CAP, MAXD);
    a.lap_ws_stride = oc_lap_ws_stride(n);
    OCALLOC(a.lap_ws, S * a.lap_ws_stride);
    a.lap_csr = nullptr;
    a.lap_csr_stride = n >= LAPB_MIN_N && lap_sparse_on() ? (lap_csr_bytes(n) + 255) & ~255LL : 0;
    if (a.lap_csr_stride) OCALLOC(a.lap_csr, S * a.lap_csr_stride);
    e->lds = (size_t)oc_lds_bytes(CAP, MAXD);
    OCALLOC(e->d_off, S + 1);
    OCALLOC(e->d_wh, 2 * S);
    YTA_HIP(hipHostMalloc((void **)&e->h_off, sizeof(int) * (S + 1), hipHostMallocDefault));
    YTA_HIP(hipHostMalloc((void **)&e->h_wh, sizeof(int) * 2 * S, hipHostMallocDefault));
    YTA_HIP(hipHostMalloc((void **)&e->h_cnt, sizeof(OcCounters) * S, hipHostMallocDefault));
    YTA_HIP(hipFuncSetAttribute((const void *)k_oc_lap, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)LAP_LDS_MAX));
    YTA_HIP(hipFuncSetAttribute((const void *)k_oc_assoc, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)dense_lap_ws_bytes(OC_LDS_LAP_N)));
    return YTA_OK;
}

void oc_release(yta_ocsort *e) {
    for (void *p : e->allocs) (void)hipFree(p);
    e->allocs.clear();
    if (e->h_off) (void)hipHostFree(e->h_off);
    if (e->h_wh) (void)hipHostFree(e->h_wh);
    if (e->h_cnt) (void)hipHostFree(e->h_cnt);
    e->h_off = e->h_wh = nullptr;
    e->h_cnt = nullptr;
}

int oc_launch(yta_ocsort *e, const double *d_dets, const int *d_off, const int *d_wh, double *out,
              int *out_counts) {
    OcArgs &a = e->a;
    a.det_in = d_dets;
    a.det_off = d_off;
    a.img_wh = d_wh;
    a.out = out;
    a.out_counts = out_counts;
    {
        const int mrc = e->mask.stage(a.S, e->stream, &a.active);
        if (mrc) return mrc;
    }
    if (a.S <= 64)
        hipLaunchKernelGGL(k_oc_pre<1024>, dim3(a.S), dim3(1024), 0, e->stream, a);
    else
        hipLaunchKernelGGL(k_oc_pre<OC_T>, dim3(a.S), dim3(OC_T), 0, e->stream, a);
    YTA_HIP(hipGetLastError());
    const long long per = ((long long)a.MAXD * a.CAP + OC_T - 1) / OC_T;
    const long long cap = std::max<long long>(4, 4096 / a.S);
    hipLaunchKernelGGL(k_oc_cost, dim3((unsigned)std::max<long long>(1, std::min(per, cap)), a.S),
                       dim3(OC_T), 0, e->stream, a);
    YTA_HIP(hipGetLastError());
    const long long rows = (a.MAXD + OC_T / WAVE - 1) / (OC_T / WAVE);
    hipLaunchKernelGGL(k_oc_rowpre, dim3((unsigned)std::max<long long>(1, std::min(rows, cap)), a.S),
                       dim3(OC_T), 0, e->stream, a);
    YTA_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_oc_lap, dim3(a.S), dim3(LAP_T), (size_t)lap_kernel_lds(a.CAP, a.MAXD),
                       e->stream, a);
    YTA_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_oc_assoc, dim3(a.S), dim3(OC_T), e->lds, e->stream, a);
    YTA_HIP(hipGetLastError());
    return YTA_OK;
}

int oc_read_counters(yta_ocsort *e) {
    YTA_HIP(hipMemcpyAsync(e->h_cnt, e->a.cnt, sizeof(OcCounters) * e->S, hipMemcpyDeviceToHost,
                           e->stream));
    YTA_HIP(host_wait(e->stream));
    return YTA_OK;
}

int oc_check_errors(yta_ocsort *e) {
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

// Grow capacity (tracks per stream / detections per stream), keeping every stream's state.
int oc_reserve(yta_ocsort *e, int cap, int maxd) {
    if (cap <= e->CAP && maxd <= e->MAXD) return YTA_OK;
    cap = std::max(cap, e->CAP);
    maxd = std::max(maxd, e->MAXD);
    YTA_HIP(host_wait(e->stream));
    yta_ocsort *n = new (std::nothrow) yta_ocsort();
    YTA_CHECK(n, YTA_ERR_NOMEM, "out of host memory");
    n->device = e->device;
    n->S = e->S;
    n->CAP = cap;
    n->MAXD = maxd;
    n->prm = e->prm;
    n->stream = e->stream;
    int rc = oc_alloc(n);
    const size_t S = e->S, oc = e->CAP, nc = cap;
    auto copy2d = [&](void *dst, size_t dp, const void *src, size_t sp, size_t w) -> int {
        YTA_HIP(hipMemcpy2DAsync(dst, dp, src, sp, w, S, hipMemcpyDeviceToDevice, e->stream));
        return YTA_OK;
    };
    if (!rc) rc = copy2d(n->a.rec, nc * sizeof(OcTrack), e->a.rec, oc * sizeof(OcTrack),
                         oc * sizeof(OcTrack));
    if (!rc) rc = copy2d(n->a.list, nc * 4, e->a.list, oc * 4, oc * 4);
    if (!rc) {
        // free slots: the old free list, then the new slots [oc, nc) (popped from the end:
        // written so the lowest new slot is used first after the old ones)
        std::vector<int> fl(nc * S);
        std::vector<int> old(oc * S);
        std::vector<OcCounters> cnt(S);
        hipError_t he = hipMemcpyAsync(old.data(), e->a.free_list, sizeof(int) * oc * S,
                                       hipMemcpyDeviceToHost, e->stream);
        if (he == hipSuccess)
            he = hipMemcpyAsync(cnt.data(), e->a.cnt, sizeof(OcCounters) * S,
                                hipMemcpyDeviceToHost, e->stream);
        if (he == hipSuccess) he = host_wait(e->stream);
        if (he != hipSuccess) {
            set_error("reserve: %s", hipGetErrorString(he));
            rc = YTA_ERR_HIP;
        } else {
            for (size_t s = 0; s < S; ++s) {
                int k = 0;
                for (int q = (int)nc - 1; q >= (int)oc; --q) fl[s * nc + k++] = q;
                for (int q = 0; q < cnt[s].n_free; ++q) fl[s * nc + k++] = old[s * oc + q];
                cnt[s].n_free = k;
            }
            he = hipMemcpy(n->a.free_list, fl.data(), sizeof(int) * nc * S, hipMemcpyHostToDevice);
            if (he == hipSuccess)
                he = hipMemcpy(n->a.cnt, cnt.data(), sizeof(OcCounters) * S,
                               hipMemcpyHostToDevice);
            if (he != hipSuccess) {
                set_error("reserve: %s", hipGetErrorString(he));
                rc = YTA_ERR_HIP;
            }
        }
    }
    if (rc) {
        n->stream = nullptr;
        oc_release(n);
        delete n;
        return rc;
    }
    memcpy(n->h_cnt, e->h_cnt, sizeof(OcCounters) * S);
    oc_release(e);
    e->CAP = n->CAP;
    e->MAXD = n->MAXD;
    e->allocs.swap(n->allocs);
    e->a = n->a;
    e->lds = n->lds;
    e->h_off = n->h_off;
    e->h_wh = n->h_wh;
    e->h_cnt = n->h_cnt;
    e->d_off = n->d_off;
    e->d_wh = n->d_wh;
    n->h_off = n->h_wh = nullptr;
    n->h_cnt = nullptr;
    n->stream = nullptr;
    delete n;
    return YTA_OK;
}

}  // namespace

extern "C" {

int yta_ocsort_create(int device, int n_streams, int track_capacity, int max_dets,
                      const yta_ocsort_params *params, yta_ocsort **engine) {
    YTA_CHECK(engine && params, YTA_ERR_INVALID, "null engine/params");
    YTA_CHECK(n_streams > 0 && track_capacity > 0 && max_dets > 0, YTA_ERR_INVALID,
              "n_streams, track_capacity and max_dets must be positive");
    YTA_CHECK(params->delta_t >= 1 && params->delta_t <= OC_DT_MAX, YTA_ERR_INVALID,
              "delta_t must be in [1, %d]", OC_DT_MAX);
    YTA_CHECK(params->asso_func >= 0 && params->asso_func <= 4, YTA_ERR_INVALID,
              "asso_func must be 0..4 (iou, giou, diou, ciou, centroid)");
    YTA_CHECK(!(params->use_byte && params->asso_func == 4), YTA_ERR_INVALID,
              "use_byte with centroid: the reference calls centroid_batch without w, h "
              "(ocsort.py:292) and raises");
    *engine = nullptr;
    int rc = select_device(device);
    if (rc) return rc;
    yta_ocsort *e = new (std::nothrow) yta_ocsort();
    YTA_CHECK(e, YTA_ERR_NOMEM, "out of host memory");
    e->device = device;
    e->S = n_streams;
    e->CAP = track_capacity;
    e->MAXD = max_dets;
    e->prm = *params;
    hipError_t he = hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking);
    if (he != hipSuccess) {
        set_error("hipStreamCreate: %s", hipGetErrorString(he));
        delete e;
        return YTA_ERR_HIP;
    }
    rc = oc_alloc(e);
    if (!rc) rc = yta_ocsort_reset(e);
    if (rc) {
        yta_ocsort_destroy(e);
        return rc;
    }
    *engine = e;
    return YTA_OK;
}

int yta_ocsort_destroy(yta_ocsort *e) {
    if (!e) return YTA_OK;
    (void)hipSetDevice(e->device);
    if (e->stream) (void)host_wait(e->stream);
    oc_release(e);
    e->mask.release();
    if (e->h_dets) (void)hipHostFree(e->h_dets);
    if (e->d_det_in) (void)hipFree(e->d_det_in);
    if (e->stream) (void)hipStreamDestroy(e->stream);
    delete e;
    return YTA_OK;
}

int yta_ocsort_reset(yta_ocsort *e) {
    YTA_CHECK(e, YTA_ERR_INVALID, "null engine");
    YTA_HIP(hipSetDevice(e->device));
    hipLaunchKernelGGL(k_oc_reset, dim3(e->S), dim3(256), 0, e->stream, e->a, 0);
    YTA_HIP(hipGetLastError());
    YTA_HIP(host_wait(e->stream));
    memset(e->h_cnt, 0, sizeof(OcCounters) * e->S);
    return YTA_OK;
}

int yta_ocsort_capacity(yta_ocsort *e, int *track_capacity, int *max_dets) {
    YTA_CHECK(e && track_capacity && max_dets, YTA_ERR_INVALID, "null argument");
    *track_capacity = e->CAP;
    *max_dets = e->MAXD;
    return YTA_OK;
}

int yta_ocsort_update(yta_ocsort *e, const double *dets, const int *det_offsets,
                      const int *img_wh, long long *next_id, double *out, int out_capacity,
                      int *out_offsets) {
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
        const int rc = oc_reserve(e, need_c > e->CAP ? std::max(need_c, 2 * e->CAP) : e->CAP,
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
    memcpy(e->h_off, det_offsets, sizeof(int) * (S + 1));
    YTA_HIP(hipMemcpyAsync(e->d_off, e->h_off, sizeof(int) * (S + 1), hipMemcpyHostToDevice,
                           e->stream));
    if (img_wh) {
        memcpy(e->h_wh, img_wh, sizeof(int) * 2 * S);
        YTA_HIP(hipMemcpyAsync(e->d_wh, e->h_wh, sizeof(int) * 2 * S, hipMemcpyHostToDevice,
                               e->stream));
    }
    if (next_id) {
        for (int s = 0; s < S; ++s) e->h_cnt[s].next_id = next_id[s];
        YTA_HIP(hipMemcpy2DAsync(&e->a.cnt[0].next_id, sizeof(OcCounters), &e->h_cnt[0].next_id,
                                 sizeof(OcCounters), sizeof(long long), S, hipMemcpyHostToDevice,
                                 e->stream));
    }
    int rc = oc_launch(e, e->d_det_in, e->d_off, img_wh ? e->d_wh : nullptr, e->a.out, nullptr);
    if (rc) return rc;
    rc = oc_read_counters(e);
    if (rc) return rc;
    if (next_id)   // the device counters have advanced: hand them back even on an error below
        for (int s = 0; s < S; ++s) next_id[s] = e->h_cnt[s].next_id;
    rc = oc_check_errors(e);
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

int yta_ocsort_update_device(yta_ocsort *e, const double *d_dets, const int *d_det_offsets,
                             const int *d_img_wh, double *d_out, int *d_out_counts) {
    YTA_CHECK(e && d_det_offsets && d_out, YTA_ERR_INVALID, "null argument");
    YTA_CHECK(d_img_wh || e->prm.asso_func != 4, YTA_ERR_INVALID, "centroid needs img_wh");
    return oc_launch(e, d_dets, d_det_offsets, d_img_wh, d_out, d_out_counts);
}

int yta_ocsort_sync(yta_ocsort *e) {
    YTA_CHECK(e, YTA_ERR_INVALID, "null engine");
    const int rc = oc_read_counters(e);
    if (rc) return rc;
    return oc_check_errors(e);
}

int yta_ocsort_get_state(yta_ocsort *e, int stream, int *n_tracks, long long *ints, double *x,
                         double *P) {
    YTA_CHECK(e && n_tracks && ints && x && P, YTA_ERR_INVALID, "null argument");
    YTA_CHECK(stream >= 0 && stream < e->S, YTA_ERR_INVALID, "bad stream %d", stream);
    YTA_HIP(hipSetDevice(e->device));
    const int rc = oc_read_counters(e);
    if (rc) return rc;
    const OcCounters c = e->h_cnt[stream];
    const long long tb = (long long)stream * e->CAP;
    std::vector<int> lst(c.n_trk);
    std::vector<OcTrack> rec(e->CAP);
    if (c.n_trk)
        YTA_HIP(hipMemcpy(lst.data(), e->a.list + tb, sizeof(int) * c.n_trk, hipMemcpyDeviceToHost));
    YTA_HIP(hipMemcpy(rec.data(), e->a.rec + tb, sizeof(OcTrack) * e->CAP, hipMemcpyDeviceToHost));
    for (int i = 0; i < c.n_trk; ++i) {
        const OcTrack &r = rec[lst[i]];
        long long *ii = ints + 7LL * i;
        ii[0] = r.id;
        ii[1] = r.age;
        ii[2] = r.hits;
        ii[3] = r.hit_streak;
        ii[4] = r.tsu;
        ii[5] = (r.flags & OF_OBSERVED) ? 1 : 0;
        ii[6] = (r.flags & OF_SAVED) ? 1 : 0;
        for (int k = 0; k < 7; ++k) x[7LL * i + k] = r.kf.x[k];
        double *M = P + 49LL * i;
        for (int k = 0; k < 49; ++k) M[k] = 0.0;
        for (int g = 0; g < 3; ++g) {
            const int a0 = g, b0 = g + 4;
            M[a0 * 7 + a0] = r.kf.p[4 * g];
            M[a0 * 7 + b0] = r.kf.p[4 * g + 1];
            M[b0 * 7 + a0] = r.kf.p[4 * g + 2];
            M[b0 * 7 + b0] = r.kf.p[4 * g + 3];
        }
        M[3 * 7 + 3] = r.kf.p[12];
    }
    *n_tracks = c.n_trk;
    return YTA_OK;
}

// Last frame's counts summed over streams: dets, first-round dets, BYTE dets, live trackers,
// output rows, births, LAP calls, fast-path frames (8 int64).
int yta_ocsort_stats(yta_ocsort *e, long long *stats) {
    YTA_CHECK(e && stats, YTA_ERR_INVALID, "null argument");
    const int rc = oc_read_counters(e);
    if (rc) return rc;
    for (int k = 0; k < 8; ++k) stats[k] = 0;
    for (int s = 0; s < e->S; ++s) {
        const OcCounters &c = e->h_cnt[s];
        const long long v[8] = {c.n_dets, c.n_high, c.n_second, c.n_trk,
                                c.n_out, c.n_births, c.lap_calls, c.fast_path};
        for (int k = 0; k < 8; ++k) stats[k] += v[k];
    }
    return YTA_OK;
}

int yta_ocsort_lap_stats(yta_ocsort *e, long long *stats, int n) {
    YTA_CHECK(e && (stats || n <= 0), YTA_ERR_INVALID, "null argument");
    const int rc = oc_read_counters(e);
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

int yta_ocsort_hip_stream(yta_ocsort *e, void **stream) {
    YTA_CHECK(e && stream, YTA_ERR_INVALID, "null argument");
    *stream = (void *)e->stream;
    return YTA_OK;
}

#ifdef YTA_STAMPS
int yta_ocsort_debug_stamps(unsigned long long *out) {
    YTA_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * 128));
    return YTA_OK;
}
#endif

// Kalman KAT: n tracks run `steps` steps of predict + update from z[step][track] (4 values; a
// NaN first value = missed update, i.e. update(None)); track i starts from z0[i].  Final x (7)
// and full P (49) per track.
int yta_kf7_run(int device, int n, int steps, const double *z0, const double *z, double *x_out,
                double *P_out);


// ---- stream subsets (subset.hpp): the listed streams updated, every other stream untouched
int yta_ocsort_reset_stream(yta_ocsort *e, int stream) {
    YTA_CHECK(e, YTA_ERR_INVALID, "null engine");
    YTA_CHECK(stream >= 0 && stream < e->S, YTA_ERR_INVALID, "stream %d outside 0..%d", stream,
              e->S - 1);
    YTA_HIP(hipSetDevice(e->device));
    hipLaunchKernelGGL(k_oc_reset, dim3(1), dim3(256), 0, e->stream, e->a, stream);
    YTA_HIP(hipGetLastError());
    YTA_HIP(host_wait(e->stream));
    return oc_read_counters(e);
}

int yta_ocsort_update_device_masked(yta_ocsort *e, const int *d_active, const double *d_dets, const int *d_det_offsets, const int *d_img_wh, double *d_out, int *d_out_counts) {
    YTA_CHECK(e, YTA_ERR_INVALID, "null engine");
    e->mask.req_dev = d_active;
    const int rc = yta_ocsort_update_device(e, d_dets, d_det_offsets, d_img_wh, d_out, d_out_counts);
    e->mask.req_dev = nullptr;
    return rc;
}

int yta_ocsort_update_streams(yta_ocsort *e, int n_streams, const int *stream_ids, const double *dets, const int *det_offsets, const int *img_wh,
                           long long *next_id, double *out, int out_capacity, int *out_offsets) {
    YTA_CHECK(e && out_offsets, YTA_ERR_INVALID, "null argument");
    YTA_HIP(hipSetDevice(e->device));
    const int S = e->S;
    std::vector<int> mask, off, full_oo(S + 1, 0);
    int rc = subset_expand(S, n_streams, stream_ids, det_offsets, mask, off);
    if (rc) return rc;
    std::vector<long long> nid(S);
    if (next_id) {   // the skipped streams keep their device counters: read them first
        rc = oc_read_counters(e);
        if (rc) return rc;
        for (int s = 0; s < S; ++s) nid[s] = e->h_cnt[s].next_id;
        for (int k = 0; k < n_streams; ++k) nid[stream_ids[k]] = next_id[k];
    }
    std::vector<int> wh;
    if (img_wh) wh = subset_spread<int>(S, n_streams, stream_ids, img_wh, 2, 1);
    e->mask.req_host = mask.data();
    rc = yta_ocsort_update(e, dets, off.data(), img_wh ? wh.data() : nullptr, next_id ? nid.data() : nullptr, out,
                        out_capacity, full_oo.data());
    e->mask.req_host = nullptr;
    if (next_id)
        for (int k = 0; k < n_streams; ++k) next_id[k] = nid[stream_ids[k]];
    if (rc) return rc;
    subset_compact(n_streams, stream_ids, full_oo, out_offsets);
    return YTA_OK;
}

}  // extern "C"

namespace {
__global__ void k_kf7_run(int n, int steps, const double *z0, const double *z, double *xo,
                          double *Po) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Kf7 kf, fz;
    kf7_init(z0 + 4LL * i, kf);
    fz = kf;
    double hz[4] = {0, 0, 0, 0};
    bool observed = false, saved = false;
    int since = 0;
    for (int st = 0; st < steps; ++st) {
        kf7_predict(kf);
        const double *zz = z + (4LL * n) * st + 4LL * i;
        if (zz[0] != zz[0]) {
            if (observed) { fz = kf; saved = true; }
            observed = false;
            since += 1;
            continue;
        }
        if (!observed && saved) {
            kf = fz;
            saved = false;
            kf7_replay(kf, hz, zz, since + 1, hz);
        } else {
            for (int k = 0; k < 4; ++k) hz[k] = zz[k];
        }
        since = 0;
        observed = true;
        kf7_correct(kf, zz);
    }
    for (int k = 0; k < 7; ++k) xo[7LL * i + k] = kf.x[k];
    double *M = Po + 49LL * i;
    for (int k = 0; k < 49; ++k) M[k] = 0.0;
    for (int g = 0; g < 3; ++g) {
        M[g * 7 + g] = kf.p[4 * g];
        M[g * 7 + g + 4] = kf.p[4 * g + 1];
        M[(g + 4) * 7 + g] = kf.p[4 * g + 2];
        M[(g + 4) * 7 + g + 4] = kf.p[4 * g + 3];
    }
    M[24] = kf.p[12];
}
}  // namespace

extern "C" int yta_kf7_run(int device, int n, int steps, const double *z0, const double *z,
                           double *x_out, double *P_out) {
    YTA_CHECK(n >= 0 && steps >= 0, YTA_ERR_INVALID, "negative size");
    if (n == 0) return YTA_OK;
    YTA_CHECK(z0 && (steps == 0 || z) && x_out && P_out, YTA_ERR_INVALID, "null buffer");
    int rc = select_device(device);
    if (rc) return rc;
    double *d_z0 = nullptr, *d_z = nullptr, *d_x = nullptr, *d_P = nullptr;
    auto cleanup = [&]() {
        if (d_z0) (void)hipFree(d_z0);
        if (d_z) (void)hipFree(d_z);
        if (d_x) (void)hipFree(d_x);
        if (d_P) (void)hipFree(d_P);
    };
    hipError_t he = hipMalloc(&d_z0, sizeof(double) * 4 * n);
    if (he == hipSuccess) he = hipMalloc(&d_z, sizeof(double) * 4 * n * (steps ? steps : 1));
    if (he == hipSuccess) he = hipMalloc(&d_x, sizeof(double) * 7 * n);
    if (he == hipSuccess) he = hipMalloc(&d_P, sizeof(double) * 49 * n);
    if (he == hipSuccess) he = hipMemcpy(d_z0, z0, sizeof(double) * 4 * n, hipMemcpyHostToDevice);
    if (he == hipSuccess && steps)
        he = hipMemcpy(d_z, z, sizeof(double) * 4 * n * steps, hipMemcpyHostToDevice);
    if (he == hipSuccess) {
        hipLaunchKernelGGL(k_kf7_run, dim3((n + 63) / 64), dim3(64), 0, 0, n, steps, d_z0, d_z, d_x,
                           d_P);
        he = hipGetLastError();
    }
    if (he == hipSuccess) he = hipMemcpy(x_out, d_x, sizeof(double) * 7 * n, hipMemcpyDeviceToHost);
    if (he == hipSuccess) he = hipMemcpy(P_out, d_P, sizeof(double) * 49 * n, hipMemcpyDeviceToHost);
    cleanup();
    YTA_CHECK(he == hipSuccess, YTA_ERR_HIP, "kf7 KAT: %s", hipGetErrorString(he));
    return YTA_OK;
}

// ----------------------------------------------------------------------------------------------
// First-round solve KAT (ocsort_common.hpp): the chip-wide row pre-pass and the LAP_T-thread
// solve exactly as the engines launch them, on one na x nb cost matrix (rows = detections,
// columns = trackers; no fast path).  rx[i] = tracker of detection i or -1 when solved; *done = 0
// when the association kernel would replay lapjv instead; *n_tight = the number of tight
// non-matching edges the uniqueness certificate of a transposed solve examined (na > nb), -1
// when the problem was solved in its normal orientation (no certificate).
namespace {
__global__ __launch_bounds__(OC_T) void k_kat_fr_pre(const double *m, int na, int nb, double *u,
                                                     int *x, double *s2) {
    main_lap_pre(m, na, nb, u, x, s2);
}
__global__ __launch_bounds__(LAP_T) void k_kat_fr(const double *m, int na, int nb, const double *u,
                                                  const int *x, const double *s2, int *rx,
                                                  long long lds_bytes, unsigned char *gws, int *st,
                                                  int *n_tight, int chip) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    LapStats ls{0, 0, 0, 0};
    if (threadIdx.x == 0) *n_tight = -1;
    __syncthreads();
    first_round_lap(m, na, nb, rx, rx, false, u, x, s2, rx, lds, lds_bytes, gws, st, st + 1, &ls,
                    gws + dense_lap_ws_bytes(na > nb ? na : nb) + arr_ws_region(na > nb ? na : nb),
                    n_tight, chip != 0);
}
// the engines' chip-wide bidding rounds (fr_arr_*) on the KAT's one problem
__global__ __launch_bounds__(OC_T) void k_kat_arr0(const double *m, int na, int nb, const int *rcnt,
                                                   const double *u, const int *x, const double *s2,
                                                   unsigned char *tws) {
    __shared__ int wsum[32];
    fr_arr_round0(m, na, nb, rcnt, rcnt, false, u, x, s2, tws, wsum);
}
__global__ __launch_bounds__(ARR_SCAN_WPB * WAVE) void k_kat_arrscan(const double *m, int na, int nb,
                                                                     unsigned char *tws) {
    fr_arr_scan(m, na, nb, tws, blockIdx.x, gridDim.x);
}
__global__ __launch_bounds__(OC_T) void k_kat_arrapply(const double *m, int na, int nb,
                                                       unsigned char *tws) {
    __shared__ int wsum[32];
    fr_arr_apply(m, na, nb, tws, wsum);
}
struct KatBuf {
    std::vector<void *> ptrs;
    ~KatBuf() {
        for (void *p : ptrs) (void)hipFree(p);
    }
    template <typename T>
    hipError_t get(T **p, size_t n) {
        void *q = nullptr;
        const hipError_t e = hipMalloc(&q, sizeof(T) * (n ? n : 1));
        if (e == hipSuccess) ptrs.push_back(q);
        *p = (T *)q;
        return e;
    }
};
}  // namespace

extern "C" int yta_lap_first_round(int device, int na, int nb, const double *cost, int *rx,
                                   int *done, int *n_tight) {
    YTA_CHECK(na > 0 && nb > 0 && cost && rx && done && n_tight, YTA_ERR_INVALID, "bad arguments");
    const int n = std::max(na, nb);
    YTA_CHECK(n <= RECT_CPT_MAX * LAP_T, YTA_ERR_INVALID, "more than %d rows or columns",
              RECT_CPT_MAX * LAP_T);
    int rc = select_device(device);
    if (rc) return rc;
    KatBuf m;
    double *dc, *u, *s2;
    int *x, *drx, *st, *dg;
    unsigned char *gws;
    YTA_HIP(m.get(&dc, (long long)na * nb));
    YTA_HIP(m.get(&u, n));
    YTA_HIP(m.get(&s2, n));
    YTA_HIP(m.get(&x, n));
    YTA_HIP(m.get(&drx, na));
    YTA_HIP(m.get(&st, 2));
    YTA_HIP(m.get(&dg, 1));
    YTA_HIP(m.get(&gws, (size_t)(dense_lap_ws_bytes(n) + arr_ws_region(n) + tight_ws_bytes())));
    YTA_HIP(hipMemcpy(dc, cost, sizeof(double) * na * nb, hipMemcpyHostToDevice));
    YTA_HIP(hipMemset(drx, 0, sizeof(int) * na));   // rcnt = 0: no fast path
    YTA_HIP(hipMemset(st, 0, sizeof(int) * 2));
    static bool attr = false;
    if (!attr) {
        YTA_HIP(hipFuncSetAttribute((const void *)k_kat_fr,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)LAP_LDS_MAX));
        attr = true;
    }
    const long long lds = lap_kernel_lds(nb, na);
    hipLaunchKernelGGL(k_kat_fr_pre, dim3(256), dim3(OC_T), 0, 0, dc, na, nb, u, x, s2);
    YTA_HIP(hipGetLastError());
    // as the engines: the chip-wide bidding rounds for first rounds of ARR_CHIP_MIN_DETS or more
    const int chip = n >= ARR_CHIP_MIN_DETS;
    if (chip) {
        unsigned char *tws = gws + dense_lap_ws_bytes(n) + arr_ws_region(n);
        hipLaunchKernelGGL(k_kat_arr0, dim3(1), dim3(OC_T), 0, 0, dc, na, nb, drx, u, x, s2, tws);
        for (int r = 0; r < ARR_CHIP_ROUNDS; ++r) {
            hipLaunchKernelGGL(k_kat_arrscan, dim3(ARR_SCAN_BLOCKS), dim3(ARR_SCAN_WPB * WAVE), 0, 0,
                               dc, na, nb, tws);
            hipLaunchKernelGGL(k_kat_arrapply, dim3(1), dim3(OC_T), 0, 0, dc, na, nb, tws);
        }
        YTA_HIP(hipGetLastError());
    }
    hipLaunchKernelGGL(k_kat_fr, dim3(1), dim3(LAP_T), (size_t)lds, 0, dc, na, nb, u, x, s2, drx,
                       lds, gws, st, dg, chip);
    YTA_HIP(hipGetLastError());
    int hst[2];
    YTA_HIP(hipMemcpy(hst, st, sizeof(hst), hipMemcpyDeviceToHost));
    YTA_HIP(hipMemcpy(rx, drx, sizeof(int) * na, hipMemcpyDeviceToHost));
    YTA_HIP(hipMemcpy(n_tight, dg, sizeof(int), hipMemcpyDeviceToHost));
    YTA_CHECK(hst[0] == 0, YTA_ERR_HIP, "solver error flags 0x%x", hst[0]);
    *done = hst[1];
    return YTA_OK;
}
