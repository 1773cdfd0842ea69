/*
 * yolo_tracking_amd — C ABI of the MI355X tracker.update() hot path.
 *
 * Every entry point returns an int status (YTA_OK = 0, negative = error; the message is available
 * from yta_last_error(), thread-local).  No torch / HIP types cross this boundary: plain pointers,
 * sizes and opaque handles only.  Host buffers are caller-owned; device buffers are owned by the
 * library (except in the *_device entry points, which take caller-owned device pointers).
 *
 * What each entry point replaces in the reference (BoxMOT 10.0.51, /root/reference):
 *   yta_bytetrack_*          boxmot/trackers/bytetrack/byte_tracker.py:114-281  BYTETracker.__init__/update
 *                            (created by boxmot/tracker_zoo.py:56-64 create_tracker('bytetrack', ...))
 *   yta_botsort_*            boxmot/trackers/botsort/bot_sort.py:185-420  BoTSORT.__init__/update
 *                            (created by boxmot/tracker_zoo.py:66-81 create_tracker('botsort', ...));
 *                            the ReID forward pass (reid_multibackend.py:303-311) and the CMC
 *                            estimator (sof.py) stay outside: their outputs are inputs here
 *   yta_ocsort_*             boxmot/trackers/ocsort/ocsort.py:188-379  OCSort.__init__/update
 *                            (created by boxmot/tracker_zoo.py:42-55 create_tracker('ocsort', ...))
 *   yta_deepocsort_*         boxmot/trackers/deepocsort/deep_ocsort.py:308-520  DeepOCSort.__init__/
 *                            update (created by boxmot/tracker_zoo.py:83-99); ReID and CMC outside
 *   yta_kf8_run              deep_ocsort.py:103-293 KalmanBoxTracker (new KF) + deepocsort_kf.py
 *   yta_hybridsort_*         boxmot/trackers/hybridsort/hybridsort.py:329-570  HybridSORT.__init__/
 *                            update without its PerClassDecorator (the host replays it call by
 *                            call, boxmot/utils/__init__.py:22-61; created by
 *                            boxmot/tracker_zoo.py:100-114); ReID outside
 *   yta_kf9_run              hybridsort.py:106-320 KalmanBoxTracker + hybridsort_kf.py:339-528
 *   yta_lap_padded           boxmot/utils/association.py:20-28 linear_assignment -> lap.lapjv(cost,
 *                            extend_cost=True)
 *   yta_lap_rect             the same call's optimum where ties cannot change the tracker result
 *                            (association.py:20-28 at ocsort.py:266-291, :315-342)
 *   yta_kf7_run              boxmot/motion/kalman_filters/ocsort_kf.py:339-526 predict / update incl.
 *                            freeze / unfreeze (observation-centric re-update)
 *   yta_box_affinity         boxmot/utils/iou.py:6-188  iou/giou/diou/ciou/centroid_batch
 *   yta_iou_distance         boxmot/utils/matching.py:94-119 iou_distance (+ fuse_score :213-221)
 *   yta_kf_xyah_initiate     boxmot/motion/kalman_filters/bytetrack_kf.py:55-86
 *   yta_kf_xyah_predict      boxmot/motion/kalman_filters/bytetrack_kf.py:155-192 (multi_predict)
 *   yta_kf_xyah_update       boxmot/motion/kalman_filters/bytetrack_kf.py:194-226 (+ project :126-153)
 *   yta_lap_limited          boxmot/utils/matching.py:56-71 linear_assignment -> lap.lapjv(cost,
 *                            extend_cost=True, cost_limit=thresh)
 *   yta_embedding_distance   boxmot/utils/matching.py:145-167 embedding_distance (max(0, cdist cosine))
 *   yta_aw_max_metric        boxmot/utils/association.py:79-108 compute_aw_max_metric
 *   yta_gsi_*                boxmot/postprocessing/gsi.py:12-72 linear_interpolation / gaussian_smooth
 *   yta_reid_preprocess*     boxmot/appearance/reid_multibackend.py:189-224
 *                            ReIDDetectMultiBackend.preprocess (crop, cv2.resize INTER_LINEAR,
 *                            BGR -> RGB, ImageNet standardisation, NCHW batch)
 *   yta_reid_normalize*      boxmot/appearance/reid_multibackend.py:303-311 get_features'
 *                            `features / np.linalg.norm(features)`
 */
#ifndef YOLO_TRACKING_AMD_H
#define YOLO_TRACKING_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define YTA_OK 0
#define YTA_ERR_INVALID (-1)   /* bad argument (shape, null pointer, unknown kind)        */
#define YTA_ERR_HIP (-2)       /* HIP runtime failure (no device, launch or copy failure)  */
#define YTA_ERR_CAPACITY (-3)  /* track / detection / output capacity exceeded            */
#define YTA_ERR_NOMEM (-4)     /* host or device allocation failed                        */

/* ---- library ---------------------------------------------------------------------------- */
int yta_version(void);                       /* returns the ABI version (positive) */
const char *yta_last_error(void);            /* message of the last failing call on this thread */
int yta_device_count(int *count);

/* ---- association primitives (parity / KAT entry points; synchronous, host buffers) ---------
 * Boxes are [x1, y1, x2, y2] float64 rows. */
#define YTA_AFF_IOU 0
#define YTA_AFF_GIOU 1
#define YTA_AFF_DIOU 2
#define YTA_AFF_CIOU 3
#define YTA_AFF_CENTROID 4
/* out[i*nb + j] = affinity(a_i, b_j), exactly iou.py's *_batch(a, b) (centroid uses img_w/img_h) */
int yta_box_affinity(int device, int kind, const double *a, int na, const double *b, int nb,
                     double img_w, double img_h, double *out);
/* out = 1 - iou_batch(a, b); if scores != NULL, then fuse_score: 1 - (1 - out) * scores[j] */
int yta_iou_distance(int device, const double *a, int na, const double *b, int nb,
                     const double *scores, double *out);

/* Grid-pruned pair search (the candidate machinery behind the tracker's association and
 * duplicate removal): every (i, j) with 1 - IoU(a_i, b_j) < thresh, thresh <= 1; pairs[2k] = i,
 * pairs[2k+1] = j in no particular order; *n_pairs = total found (only `cap` are written). */
int yta_grid_pairs(int device, const double *a, int na, const double *b, int nb, double thresh,
                   int *pairs, int cap, int *n_pairs);

/* ---- ByteTrack Kalman filter, xyah state (parity / KAT entry points) -----------------------
 * mean: n x 8, cov: n x 8 x 8 (row-major, full matrices), meas / z: n x 4 [xc, yc, a, h]. */
int yta_kf_xyah_initiate(int device, int n, const double *meas, double *mean, double *cov);
/* Camera-motion correction KAT (SURVEY.md §8(b) affine_apply), in place on n states (mean 8,
 * covariance 8 x 8 row-major, block-diagonal over {x, y, x', y'} / {w, h, w', h'} as every state
 * of these trackers is), warps n row-major 2x3, with the engines' own device functions:
 *   kind 0  BoT-SORT STrack.multi_gmc (bot_sort.py:95-111): kf_gmc (kf_xyah.hpp)
 *   kind 1  DeepOCSORT apply_affine_correction, new-KF branch (deepocsort_kf.py:387-405;
 *           deep_ocsort.py:250-267 calls it per tracker): kf8_affine (kf_deep.hpp) */
int yta_affine_apply(int device, int kind, int n, const double *warps, double *mean, double *cov);
/* in place; the caller applies the reference's `mean[7] = 0` for non-tracked tracks beforehand */
int yta_kf_xyah_predict(int device, int n, double *mean, double *cov);
int yta_kf_xyah_update(int device, int n, double *mean, double *cov, const double *z);

/* Device self-test of the block-wide scan / reduction primitives the kernels are built on (DPP
 * cross-lane operations) at several block sizes.  0 when every result matches a serial answer. */
int yta_selftest(int device);

/* ---- linear assignment with lapx cost_limit semantics -------------------------------------
 * Minimises sum(matched cost) + cost_limit/2 * (#unmatched rows + #unmatched cols); x[r] = col or
 * -1, y[c] = row or -1 (lap.lapjv(cost, extend_cost=True, cost_limit=cost_limit)). */
int yta_lap_limited(int device, int nr, int nc, const double *cost, double cost_limit, int *x,
                    int *y);

/* Padded dense assignment (association.py:20-28: lap.lapjv(cost, extend_cost=True), OCSORT
 * family): zero-padded to max(nr, nc) square, every row / column of the smaller side matched;
 * x[r] = col or -1, y[c] = row or -1.  The same operation and tie-breaking sequence as the
 * restated lapjv (oracle/lapjv.c). */
int yta_lap_padded(int device, int nr, int nc, const double *cost, int *x, int *y);

/* The optimum of the same padded problem by the rectangular solver the OCSORT-family engines use
 * where the result does not depend on lapjv's tie-breaking (lap_rect.hpp): warm
 * start from row minima, shortest augmenting paths with bound pruning.  Every row / column of the
 * smaller side is matched; equal to yta_lap_padded whenever the optimum is unique.  At most 8192
 * entries on the larger side. */
int yta_lap_rect(int device, int nr, int nc, const double *cost, int *x, int *y);
/* The OCSORT-family first-round solve (ocsort_common.hpp first_round_lap, association.py:20-28)
 * exactly as the engines launch it (chip-wide row pre-pass + one LAP_T-thread block), no fast
 * path: na x nb cost (rows = detections).  rx (na): tracker of each detection or -1; *done: 1 =
 * solved, 0 = the engine would replay lapjv (more detections than trackers and the optimum not
 * certified unique); *n_tight: tight non-matching edges the certificate examined (-1 unless
 * na > nb). */
int yta_lap_first_round(int device, int na, int nb, const double *cost, int *rx, int *done,
                        int *n_tight);

/* ---- ByteTrack engine: S independent streams, state resident in HBM -----------------------
 * One engine = S trackers with identical parameters (BYTETracker(track_thresh, match_thresh,
 * track_buffer, frame_rate)).  Stream s keeps its own tracks and its own ID counter. */
typedef struct yta_bytetrack yta_bytetrack;
typedef struct {
    double track_thresh;   /* bytetrack.yaml:1   (ctor default 0.45) */
    double match_thresh;   /* bytetrack.yaml:3   (ctor default 0.8)  */
    int track_buffer;      /* bytetrack.yaml:2   (ctor default 25)   */
    int frame_rate;        /* bytetrack.yaml:4   (ctor default 30)   */
} yta_bytetrack_params;

/* track_capacity: live (tracked + lost) tracks per stream; max_dets: detections per stream per
 * frame.  The host-buffer update grows both on demand; the device-buffer update treats them as
 * hard limits (YTA_ERR_CAPACITY from yta_bytetrack_sync). */
int yta_bytetrack_create(int device, int n_streams, int track_capacity, int max_dets,
                         const yta_bytetrack_params *params, yta_bytetrack **engine);
int yta_bytetrack_destroy(yta_bytetrack *engine);
int yta_bytetrack_reset(yta_bytetrack *engine);

/* Grow the per-stream track capacity / max detections (never shrinks), keeping every stream's
 * state.  yta_bytetrack_update() calls this itself when a frame would not fit. */
int yta_bytetrack_reserve(yta_bytetrack *engine, int track_capacity, int max_dets);
int yta_bytetrack_capacity(yta_bytetrack *engine, int *track_capacity, int *max_dets);

/* Host-buffer update of all S streams (one frame each).  dets: packed rows of
 * [x1, y1, x2, y2, conf, cls] float64 for stream 0, then stream 1, ...; det_offsets: S+1
 * prefix offsets (rows).  next_id: S counters (in: the last issued ID per stream, i.e. the
 * reference's BaseTrack._count; out: updated), may be NULL to use the engine's own counters.
 * out: caller buffer of out_capacity rows x 8 float64 [x1,y1,x2,y2,id,conf,cls,det_ind];
 * out_offsets: S+1 prefix offsets written by the call.  Synchronous.
 * out_capacity >= det_offsets[S] always suffices (every output row is a track matched to or born
 * from one of the frame's detections) and is required: a smaller buffer fails with
 * YTA_ERR_CAPACITY before anything is staged or launched, so the same call can be retried.  An
 * error reported after the launch (device error flags, HIP failure) means the frame HAS been
 * applied on the device; next_id is still written back then.  The same rules hold for every
 * tracker's host-buffer update below. */
int yta_bytetrack_update(yta_bytetrack *engine, const double *dets, const int *det_offsets,
                         long long *next_id, double *out, int out_capacity, int *out_offsets);

/* Device-resident update for throughput runs: d_dets / d_det_offsets are device pointers laid out
 * as above; results stay on the device: d_out holds S * track_capacity rows x 8, stream s at row
 * s * track_capacity, d_out_counts[s] rows.  Asynchronous on the engine's HIP stream. */
int yta_bytetrack_update_device(yta_bytetrack *engine, const double *d_dets,
                                const int *d_det_offsets, double *d_out, int *d_out_counts);
int yta_bytetrack_sync(yta_bytetrack *engine);      /* waits; reports device-side errors */
/* The S per-stream ID counters on the device (waits): the last ID each stream issued, i.e. the
 * reference's BaseTrack._count after that stream's frames (basetrack.py:37-40), for the
 * device-buffer path where no host copy follows the frames. */
int yta_bytetrack_next_ids(yta_bytetrack *engine, long long *next_id);

/* Pipelined host-buffer update (ByteTrack engines): submit enqueues one frame of every stream and
 * returns at once; collect waits for the OLDEST submitted frame and reports it.  Up to three
 * frames are in flight, so frame f's detections travel host -> device while frame f-1's kernels
 * run and frame f-2's rows travel back: both PCIe directions and the kernels overlap (the synchronous
 * yta_bytetrack_update does them one after the other).  Results are identical to
 * yta_bytetrack_update frame by frame.
 *   submit: dets / det_offsets as yta_bytetrack_update; next_id: S counters written to the device
 *     before the frame, or NULL to continue the engine's own (with frames in flight pass NULL:
 *     the host copies are a frame behind); out: out_capacity >= det_offsets[S] rows x 8, filled
 *     by the matching collect (rows beyond out_offsets[S] unspecified).  Page-locked dets / out
 *     are DMA'd directly and must stay untouched until the frame is collected; pageable dets are
 *     staged during the call (reusable at once).  A fourth submit before a collect fails with
 *     YTA_ERR_INVALID; so do the synchronous update / reset / reserve while frames are in flight.
 *   collect: next_id (S, may be NULL) receives the counters after that frame; out_offsets S + 1
 *     row offsets into that frame's out; device error flags are reported here. */
int yta_bytetrack_submit(yta_bytetrack *engine, const double *dets, const int *det_offsets,
                         const long long *next_id, double *out, int out_capacity);
int yta_bytetrack_collect(yta_bytetrack *engine, long long *next_id, int *out_offsets);
/* Accounting of the pipelined path since the last reset (n doubles, up to 21): frames collected;
 * detection bytes DMA'd straight from the caller's page-locked buffer / staged through the
 * engine's pinned buffers; output-row bytes DMA'd straight into the caller's buffer / staged;
 * host milliseconds spent staging detections, inside submit, waiting in collect, copying staged
 * rows out; GPU milliseconds (per frame, from its events, summed) of the copy-in, the kernels +
 * row snapshot, the copy-out, and the frame's whole span (copy-in start to copy-out end); host
 * milliseconds inside the direct copy-in call, the kernel launches and the copy-out call, the
 * small offset copy in, the small counter / offset copies out (0: the kernels store them), and
 * the page-locked checks; the submits that waited for the newest frame's kernels to bound the
 * track capacity, and the submits that drained the pipeline to check or grow it.
 * reset != 0 zeroes the accounting after the read. */
int yta_bytetrack_pipe_stats(yta_bytetrack *engine, double *stats, int n, int reset);
/* float32 detections (ultralytics hands BoxMOT float32 boxes; the reference promotes them to
 * float64 exactly, byte_tracker.py:143): packed rows of 6 float32 cross PCIe at half the bytes and
 * are widened on the device, so every result equals the float64 call on the promoted rows.  Same
 * contracts as yta_bytetrack_submit / yta_bytetrack_update otherwise. */
int yta_bytetrack_submit_f32(yta_bytetrack *engine, const float *dets, const int *det_offsets,
                             const long long *next_id, double *out, int out_capacity);
int yta_bytetrack_update_f32(yta_bytetrack *engine, const float *dets, const int *det_offsets,
                             long long *next_id, double *out, int out_capacity,
                             int *out_offsets);

/* Host-buffer update of a SUBSET of the streams (update(ctx, n_streams,
 * stream_ids, ...)).  In the reference every camera stream is its own tracker
 * (examples/track.py:43-57) and a stream without a new frame is simply not called
 * (examples/val.py:184-226 runs sequences of different lengths side by side).  stream_ids:
 * n_streams ascending ids in 0..S-1; dets / det_offsets (n_streams + 1) / next_id (n_streams) /
 * out / out_offsets (n_streams + 1) as yta_bytetrack_update, over those streams in id order.
 * Every other stream is left exactly as it was: tracks, Kalman state, frame counter, ID counter. */
int yta_bytetrack_update_streams(yta_bytetrack *engine, int n_streams, const int *stream_ids,
                                 const double *dets, const int *det_offsets, long long *next_id,
                                 double *out, int out_capacity, int *out_offsets);
/* Device form of the subset update: d_active = S ints on the device, nonzero = update that stream
 * this call (NULL = every stream); skipped streams report 0 rows in d_out_counts. */
int yta_bytetrack_update_device_masked(yta_bytetrack *engine, const int *d_active,
                                       const double *d_dets, const int *d_det_offsets,
                                       double *d_out, int *d_out_counts);
/* Reset ONE stream to a freshly created tracker (no tracks, frame and ID counters 0), as
 * constructing a new BYTETracker for that camera would (byte_tracker.py:115-130); the other
 * streams are untouched.  Also for BoT-SORT engines. */
int yta_bytetrack_reset_stream(yta_bytetrack *engine, int stream);

/* Parity introspection: copy stream s's live tracks, tracked list first then lost list, in list
 * order.  Per track: list (0 tracked / 1 lost), id, state (0 New 1 Tracked 2 Lost 3 Removed),
 * activated, frame_id, start_frame, tracklet_len (ints: 7 x int64 per track), mean (8 f64), cov
 * (64 f64).  *n_tracks receives the count; buffers must hold track_capacity entries. */
int yta_bytetrack_get_state(yta_bytetrack *engine, int stream, int *n_tracks, long long *ints,
                            double *mean, double *cov);
/* Measurement: when enabled, HIP events are recorded around each phase of a frame on the
 * engine's stream; collect returns per-phase milliseconds summed over the covered frames, 6 values
 * in launch order: k_s1_prep, k_s1_edges, k_s1_lap (BoT-SORT and match_thresh > 1: the fused
 * k_stage1 in the first, the next two 0), stage23, apply, finish. */
int yta_bytetrack_profile(yta_bytetrack *engine, int enable);
int yta_bytetrack_profile_collect(yta_bytetrack *engine, double *ms, int *frames);
/* Last frame's counts summed over streams (synchronises): dets, high, second, pool, activated,
 * unconfirmed, leftovers, rest, births, tracked', lost', tracked, lost, output rows, stage-1
 * candidate edges, stage-2+3 candidate edges, then the cumulative number of stream-frames whose
 * stage-1 / stage-2+3 association did not fit in LDS and ran over global memory, then (ByteTrack)
 * the lost-list Kalman records the last frame left untouched (lazy prediction), then (ByteTrack)
 * the stage-1 candidate edges left to the solver after the single-edge components, then the
 * cumulative number of stream-frames whose duplicate-removal grid (k_finish) did not fit in LDS
 * (21 int64). */
int yta_bytetrack_stats(yta_bytetrack *engine, long long *stats);
/* Introspection of the engine's launch modes (writes min(n, YTA_BT_MODES) int64): the few-stream
 * mode chosen at create (YTA_SPLIT23), the mode the kernel arguments carry (stage 2 / 3 in two
 * blocks per stream), the fallback arenas pooled, cached HIP graphs enabled (YTA_GRAPHS), BoT-SORT
 * split stage 1 (YTA_BS_SPLIT), graph captures and graph replays so far, track capacity, max
 * detections.  The third is the number of pooled global fallback arenas (a stream-frame whose
 * association does not fit in LDS is redone over one of them by the launch's redo kernel, which
 * runs that many blocks): two per stream in the split mode up to a bound of 32 (YTA_WS_POOL).  The first two agree for the engine's whole life, reserve() included. */
#define YTA_BT_MODES 9
int yta_bytetrack_modes(yta_bytetrack *engine, long long *out, int n);
/* Tuning / testing: bytes of LDS the association kernels may use per stream (default 150 KiB,
 * at most 150 KiB); a stream-frame that does not fit runs over global memory.  0 forces the
 * global-memory path for every stream. */
int yta_bytetrack_set_lds(yta_bytetrack *engine, int bytes);
/* Throughput helper: the engine's HIP stream (hipStream_t as void*) */
int yta_bytetrack_hip_stream(yta_bytetrack *engine, void **stream);

/* ---- BoT-SORT engine: S independent streams ----------------------------------------------
 * The same engine object as ByteTrack (yta_bytetrack_destroy / reset / reserve / capacity / sync /
 * get_state / profile / stats / set_lds / hip_stream all apply; get_state's mean is xywh) with
 * BoT-SORT's association (IoU + gated cosine appearance cost), xywh Kalman filter, feature EMA
 * and class vote.  IDs start from 0 per stream at creation (BaseTrack.clear_count, :205). */
typedef struct yta_bytetrack yta_botsort;
typedef struct {
    double track_high_thresh;     /* botsort.yaml / ctor default 0.5  */
    double track_low_thresh;      /* 0.1  */
    double new_track_thresh;      /* 0.6  */
    double match_thresh;          /* 0.8  */
    double proximity_thresh;      /* 0.5  */
    double appearance_thresh;     /* 0.25 */
    int track_buffer;             /* 30   */
    int frame_rate;               /* 30   */
    int fuse_first_associate;     /* 0    */
    int with_reid;                /* 1: feat_dim-wide float32 ReID features per high detection */
} yta_botsort_params;

int yta_botsort_create(int device, int n_streams, int track_capacity, int max_dets, int feat_dim,
                       const yta_botsort_params *params, yta_botsort **engine);
/* Host-buffer update (synchronous).  dets / det_offsets / next_id / out / out_offsets as
 * yta_bytetrack_update.  feats: for each stream in order, the rows get_features returned for its
 * detections with conf > track_high_thresh, in detection order (float32, feat_dim wide; NULL
 * when with_reid is 0).  warps: S camera-motion 2x3 affines (row-major) or NULL for identity;
 * applied as STrack.multi_gmc (bot_sort.py:95-111) to the predicted pool and the unconfirmed
 * tracks (:290-295). */
int yta_botsort_update(yta_botsort *engine, const double *dets, const int *det_offsets,
                       const float *feats, const double *warps, long long *next_id, double *out,
                       int out_capacity, int *out_offsets);
/* Device-resident update (asynchronous): d_feats holds feat_dim floats per detection row of
 * d_dets (only the high rows are read); d_warps S row-major 2x3 camera warps (multi_gmc,
 * bot_sort.py:95-111, 290-295) or NULL for the identity. */
int yta_botsort_update_device(yta_botsort *engine, const double *d_dets, const int *d_det_offsets,
                              const float *d_feats, const double *d_warps, double *d_out,
                              int *d_out_counts);
/* Subset update (see yta_bytetrack_update_streams): feats cover the listed streams' high
 * detections in id order, warps n_streams 2x3 affines (or NULL). */
int yta_botsort_update_streams(yta_botsort *engine, int n_streams, const int *stream_ids,
                               const double *dets, const int *det_offsets, const float *feats,
                               const double *warps, long long *next_id, double *out,
                               int out_capacity, int *out_offsets);
/* Parity introspection, in yta_bytetrack_get_state's track order: smoothed features
 * (feat_dim floats per track, may be NULL), class histograms (8 x (class, summed score) float64
 * per track, may be NULL) and their entry counts (may be NULL). */
int yta_botsort_get_features(yta_botsort *engine, int stream, int *n_tracks, float *feats,
                             double *cls_hist, int *n_cls);

/* ---- OCSORT engine: S independent streams ------------------------------------------------
 * OCSort(per_class, det_thresh, max_age, min_hits, asso_threshold, delta_t, asso_func, inertia,
 * use_byte) per stream; the KalmanBoxTracker.count ID counter per stream (next_id in / out as
 * for ByteTrack; the Python front-end shares one counter per process like the reference). */
typedef struct yta_ocsort yta_ocsort;
#define YTA_ASSO_IOU 0
#define YTA_ASSO_GIOU 1
#define YTA_ASSO_DIOU 2
#define YTA_ASSO_CIOU 3
#define YTA_ASSO_CENTROID 4
typedef struct {
    double det_thresh;       /* ocsort.yaml: 0      (ctor default 0.2)  */
    int max_age;             /* 30                                      */
    int min_hits;            /* 1                   (ctor default 3)    */
    double asso_threshold;   /* iou_thresh 0.3                          */
    int delta_t;             /* 3  (1..8)                               */
    int asso_func;           /* YTA_ASSO_*: giou    (ctor default iou)  */
    double inertia;          /* 0.2                                     */
    int use_byte;            /* 0                                       */
} yta_ocsort_params;

int yta_ocsort_create(int device, int n_streams, int track_capacity, int max_dets,
                      const yta_ocsort_params *params, yta_ocsort **engine);
int yta_ocsort_destroy(yta_ocsort *engine);
int yta_ocsort_reset(yta_ocsort *engine);
int yta_ocsort_capacity(yta_ocsort *engine, int *track_capacity, int *max_dets);
/* Host-buffer update (synchronous): dets / det_offsets / next_id / out / out_offsets as
 * yta_bytetrack_update; img_wh: S x (width, height) of the frames (img.shape[1], img.shape[0];
 * read by the centroid cost only, may be NULL otherwise).  Output rows per stream in the
 * reference's order (reversed tracker list), id = tracker id + 1. */
int yta_ocsort_update(yta_ocsort *engine, const double *dets, const int *det_offsets,
                      const int *img_wh, long long *next_id, double *out, int out_capacity,
                      int *out_offsets);
/* Device-resident update (asynchronous): d_out holds S * track_capacity rows x 8. */
int yta_ocsort_update_device(yta_ocsort *engine, const double *d_dets, const int *d_det_offsets,
                             const int *d_img_wh, double *d_out, int *d_out_counts);
int yta_ocsort_sync(yta_ocsort *engine);
/* Stream subsets (see yta_bytetrack_update_streams): the listed streams (ascending ids) updated,
 * every other stream left exactly as it was; per-stream arguments (dets, img_wh n x 2, next_id,
 * out_offsets n + 1) cover the listed streams in id order.  The device form takes an [S] mask on
 * the device (nonzero = update; skipped streams report 0 rows).  reset_stream: one stream back to
 * a freshly constructed tracker (ocsort.py:188-216), the others untouched.  The same three calls
 * exist for DeepOCSORT (feats of the listed streams' kept detections, warps n x 6) and
 * HybridSORT (feats of the listed streams' rows). */
int yta_ocsort_update_streams(yta_ocsort *engine, int n_streams, const int *stream_ids,
                              const double *dets, const int *det_offsets, const int *img_wh,
                              long long *next_id, double *out, int out_capacity,
                              int *out_offsets);
int yta_ocsort_update_device_masked(yta_ocsort *engine, const int *d_active, const double *d_dets,
                                    const int *d_det_offsets, const int *d_img_wh, double *d_out,
                                    int *d_out_counts);
int yta_ocsort_reset_stream(yta_ocsort *engine, int stream);
/* Parity introspection, tracker-list order: ints 7 x int64 per tracker (id, age, hits,
 * hit_streak, time_since_update, kf.observed, kf.attr_saved is not None), x (7 f64), P (49 f64). */
int yta_ocsort_get_state(yta_ocsort *engine, int stream, int *n_tracks, long long *ints,
                         double *x, double *P);
/* Last frame's counts summed over streams: dets, first-round dets, BYTE dets, live trackers,
 * output rows, births, LAP calls, fast-path frames (8 int64). */
int yta_ocsort_stats(yta_ocsort *engine, long long *stats);
/* Solver counters since create / reset, summed over streams (4 int64): first-round solves of the
 * transposed problem (more detections than trackers, association.py:20-28 with dummy columns),
 * those of them whose optimum was not certified unique (exact ties: lapjv replayed instead),
 * lapjv replays in any round (the single-wavefront restatement of lapx's tie-breaking), and -IoU
 * rounds (BYTE / OCR) solved on the rows and columns that have a positive entry. */
#define YTA_LAP_STATS 4
/* n: the length of stats; min(n, YTA_LAP_STATS) values are written (round 6: the n argument is
 * new - round 5 wrote 4 values with no length, round 4 three). */
int yta_ocsort_lap_stats(yta_ocsort *engine, long long *stats, int n);
int yta_ocsort_hip_stream(yta_ocsort *engine, void **stream);
/* OCSORT Kalman KAT: n tracks initialised from z0 (n x 4, [u, v, s, r]) run `steps` steps of
 * predict + update(z[step] (n x 4 per step); a NaN first value = update(None)), freeze /
 * unfreeze included; final x (n x 7) and full P (n x 49). */
int yta_kf7_run(int device, int n, int steps, const double *z0, const double *z, double *x_out,
                double *P_out);

/* ---- DeepOCSORT engine: S independent streams --------------------------------------------
 * DeepOCSort(det_thresh, max_age, min_hits, iou_threshold, delta_t, asso_func, inertia,
 * w_association_emb, alpha_fixed_emb, aw_param, embedding_off, cmc_off, aw_off) per stream
 * (boxmot/trackers/deepocsort/deep_ocsort.py:308-520; per_class is stored but unused by the
 * reference's update).  The ReID forward pass (:387 get_features) and the CMC estimator (:391
 * cmc.apply) stay outside: their outputs are inputs here.  KalmanBoxTracker.count starts at 1
 * and ids are reported as stored (no +1). */
typedef struct yta_deepocsort yta_deepocsort;
typedef struct {
    double det_thresh;          /* deepocsort.yaml: 0   (ctor default 0.3); must be < 1 */
    int max_age;                /* 30                                                  */
    int min_hits;               /* 1                    (ctor default 3)               */
    double iou_threshold;       /* iou_thresh 0.3                                      */
    int delta_t;                /* 3  (0..8)                                           */
    int asso_func;              /* YTA_ASSO_*: giou     (ctor default iou)             */
    double inertia;             /* 0.2                                                 */
    double w_association_emb;   /* 0.5 (create_tracker does not pass the yaml's 0.75)  */
    double alpha_fixed_emb;     /* 0.95                                                */
    double aw_param;            /* 0.5                                                 */
    int embedding_off;          /* 0                                                   */
    int cmc_off;                /* 0                                                   */
    int aw_off;                 /* 0                                                   */
} yta_deepocsort_params;

int yta_deepocsort_create(int device, int n_streams, int track_capacity, int max_dets,
                          int feat_dim, const yta_deepocsort_params *params,
                          yta_deepocsort **engine);
int yta_deepocsort_destroy(yta_deepocsort *engine);
int yta_deepocsort_reset(yta_deepocsort *engine);
int yta_deepocsort_capacity(yta_deepocsort *engine, int *track_capacity, int *max_dets);
/* Host-buffer update (synchronous).  dets / det_offsets / next_id / out / out_offsets as
 * yta_ocsort_update; feats: feat_dim float32 per detection with conf > det_thresh, in input order
 * (what get_features returns for dets[conf > det_thresh]); warps: S x 6 float64 row-major 2x3
 * affines from the CMC estimator (NULL = identity for every stream); img_wh as yta_ocsort_update. */
int yta_deepocsort_update(yta_deepocsort *engine, const double *dets, const int *det_offsets,
                          const float *feats, const double *warps, const int *img_wh,
                          long long *next_id, double *out, int out_capacity, int *out_offsets);
/* Device-resident update (asynchronous).  d_feats holds feat_dim float32 for EVERY input row
 * (rows at or below det_thresh are ignored); d_warps S x 6 or NULL; d_out S * track_capacity
 * rows x 8. */
int yta_deepocsort_update_device(yta_deepocsort *engine, const double *d_dets,
                                 const int *d_det_offsets, const float *d_feats,
                                 const double *d_warps, const int *d_img_wh, double *d_out,
                                 int *d_out_counts);
int yta_deepocsort_sync(yta_deepocsort *engine);
/* Stream subsets and per-stream reset: as yta_ocsort_update_streams / _update_device_masked /
 * _reset_stream (deep_ocsort.py:308-347 for a fresh tracker). */
int yta_deepocsort_update_streams(yta_deepocsort *engine, int n_streams, const int *stream_ids,
                                  const double *dets, const int *det_offsets, const float *feats,
                                  const double *warps, const int *img_wh, long long *next_id,
                                  double *out, int out_capacity, int *out_offsets);
int yta_deepocsort_update_device_masked(yta_deepocsort *engine, const int *d_active,
                                        const double *d_dets, const int *d_det_offsets,
                                        const float *d_feats, const double *d_warps,
                                        const int *d_img_wh, double *d_out, int *d_out_counts);
int yta_deepocsort_reset_stream(yta_deepocsort *engine, int stream);
/* Parity introspection, tracker-list order: ints 7 x int64 per tracker (id, age, hits,
 * hit_streak, time_since_update, kf.observed, frozen), x (8 f64), P (64 f64), emb (feat_dim f64
 * per tracker; may be NULL). */
int yta_deepocsort_get_state(yta_deepocsort *engine, int stream, int *n_tracks, long long *ints,
                             double *x, double *P, double *emb);
/* Last frame's counts summed over streams: dets, kept dets, 0, live trackers, output rows,
 * births, LAP calls, fast-path frames (8 int64). */
int yta_deepocsort_stats(yta_deepocsort *engine, long long *stats);
/* Solver counters since create / reset, summed over streams (4 int64): first-round solves of the
 * transposed problem (more detections than trackers, association.py:20-28 with dummy columns),
 * those of them whose optimum was not certified unique (exact ties: lapjv replayed instead),
 * lapjv replays in any round (the single-wavefront restatement of lapx's tie-breaking), and -IoU
 * rounds (BYTE / OCR) solved on the rows and columns that have a positive entry. */
int yta_deepocsort_lap_stats(yta_deepocsort *engine, long long *stats, int n);
int yta_deepocsort_hip_stream(yta_deepocsort *engine, void **stream);
/* DeepOCSORT Kalman KAT (deep_ocsort.py:103-136, 198-293 new-KF branch): n tracks initialised
 * from boxes b0 (n x 4, x1 y1 x2 y2) run `steps` steps of [affine (warps: steps x n x 6, NULL =
 * none)], predict + update(b[step] (n x 4); a NaN first value = update(None)) with the reference's
 * clamps, Q(w, h), R(w, h), freeze / unfreeze replay; final x (n x 8) and full P (n x 64). */
int yta_kf8_run(int device, int n, int steps, const double *b0, const double *b,
                const double *warps, double *x_out, double *P_out);

/* ---- HybridSORT engine: S independent streams --------------------------------------------
 * HybridSORT(det_thresh, max_age, min_hits, iou_threshold, delta_t, asso_func, inertia) per stream
 * (boxmot/trackers/hybridsort/hybridsort.py:329-570) with its hard-wired association settings
 * (:346-360: TCM weight 0, ReID weight 1.3, long-term ReID weight 0 with the 0.4 correction, no
 * BYTE round, no ECC).  One update call = one undecorated HybridSORT.update: the per-class
 * decorator's calls (one per class, each over all trackers) are issued by the caller.  The ReID
 * forward pass (:394 get_features) stays outside: its rows are inputs here.  KalmanBoxTracker.count
 * starts at 0 and ids are reported + 1; det_ind reports the detection's score (dets0[:, 6]). */
typedef struct yta_hybridsort yta_hybridsort;
typedef struct {
    double det_thresh;          /* hybridsort.yaml: 0                                      */
    int max_age;                /* 30                                                      */
    int min_hits;               /* 1                                                       */
    double iou_threshold;       /* iou_thresh 0.3                                          */
    int delta_t;                /* 3  (0..8)                                               */
    int asso_func;              /* YTA_ASSO_IOU..YTA_ASSO_CIOU: giou (centroid: the reference
                                   calls the asso function without the image size, :516)   */
    double inertia;             /* 0.2                                                     */
} yta_hybridsort_params;

int yta_hybridsort_create(int device, int n_streams, int track_capacity, int max_dets,
                          int feat_dim, const yta_hybridsort_params *params,
                          yta_hybridsort **engine);
int yta_hybridsort_destroy(yta_hybridsort *engine);
int yta_hybridsort_reset(yta_hybridsort *engine);
int yta_hybridsort_capacity(yta_hybridsort *engine, int *track_capacity, int *max_dets);
/* Host-buffer update (synchronous).  dets / det_offsets / next_id / out / out_offsets as
 * yta_ocsort_update; feats: feat_dim float32 for EVERY input row, in input order (what
 * get_features returns for the call's boxes). */
int yta_hybridsort_update(yta_hybridsort *engine, const double *dets, const int *det_offsets,
                          const float *feats, long long *next_id, double *out, int out_capacity,
                          int *out_offsets);
/* Device-resident update (asynchronous): d_feats feat_dim float32 per input row; d_out
 * S * track_capacity rows x 8; d_out_counts S ints (may be NULL). */
int yta_hybridsort_update_device(yta_hybridsort *engine, const double *d_dets,
                                 const int *d_det_offsets, const float *d_feats, double *d_out,
                                 int *d_out_counts);
int yta_hybridsort_sync(yta_hybridsort *engine);
/* Stream subsets and per-stream reset: as yta_ocsort_update_streams / _update_device_masked /
 * _reset_stream (hybridsort.py:329-361 for a fresh tracker). */
int yta_hybridsort_update_streams(yta_hybridsort *engine, int n_streams, const int *stream_ids,
                                  const double *dets, const int *det_offsets, const float *feats,
                                  long long *next_id, double *out, int out_capacity,
                                  int *out_offsets);
int yta_hybridsort_update_device_masked(yta_hybridsort *engine, const int *d_active,
                                        const double *d_dets, const int *d_det_offsets,
                                        const float *d_feats, double *d_out, int *d_out_counts);
int yta_hybridsort_reset_stream(yta_hybridsort *engine, int stream);
/* Parity introspection, tracker-list order: ints 6 x int64 per tracker (id, age, hits,
 * hit_streak, time_since_update, kf.observed), dbl 3 x f64 (conf, cls, det_ind), x (9 f64),
 * P (81 f64), feat (feat_dim float32 smooth_feat per tracker; may be NULL). */
int yta_hybridsort_get_state(yta_hybridsort *engine, int stream, int *n_tracks, long long *ints,
                             double *dbl, double *x, double *P, float *feat);
/* The cls of every live tracker of a stream in list order (PerClassDecorator's active classes,
 * boxmot/utils/__init__.py:38). */
int yta_hybridsort_classes(yta_hybridsort *engine, int stream, double *cls, int cap, int *n);
/* Last frame's counts summed over streams: dets, kept dets, live trackers, output rows, births,
 * LAP calls, long-term corrections, feature jobs (8 int64). */
int yta_hybridsort_stats(yta_hybridsort *engine, long long *stats);
/* Solver counters since create / reset, summed over streams (4 int64): first-round solves of the
 * transposed problem (more detections than trackers, association.py:20-28 with dummy columns),
 * those of them whose optimum was not certified unique (exact ties: lapjv replayed instead),
 * lapjv replays in any round (the single-wavefront restatement of lapx's tie-breaking), and -IoU
 * rounds (BYTE / OCR) solved on the rows and columns that have a positive entry. */
int yta_hybridsort_lap_stats(yta_hybridsort *engine, long long *stats, int n);
int yta_hybridsort_hip_stream(yta_hybridsort *engine, void **stream);
/* HybridSORT Kalman KAT (hybridsort.py:112-320): n tracks initialised from rows b0 (n x 5:
 * x1 y1 x2 y2 score) run `steps` steps of predict (velocity clamp) + update(b[step] (n x 5); a
 * NaN first value = update(None)) with the freeze / unfreeze replay; final x (n x 9) and full P
 * (n x 81). */
int yta_kf9_run(int device, int n, int steps, const double *b0, const double *b, double *x_out,
                double *P_out);

/* embedding_distance (matching.py:145-167): out (n x m) = max(0, 1 - t.d / (|t| |d|)) of float32
 * track / detection feature rows (dim wide) in float64, through the BoT-SORT engine's cosine. */
int yta_embedding_distance(int device, const float *track_feats, int n, const float *det_feats,
                           int m, int dim, double *out);
/* compute_aw_max_metric (association.py:79-108): out (nr x nc) = ((w * rw_i) * cw_j) * emb_ij with
 * the row / column weights 1 - max(second / top - bottom, 0) / (1 - bottom) (0 when top == 0, 1
 * when the row / column has fewer than two entries) — the DeepOCSORT engine's AW code. */
int yta_aw_max_metric(int device, const double *emb_cost, int nr, int nc, double w_association_emb,
                      double bottom, double *out);

/* ---- GSI post-processing (boxmot/postprocessing/gsi.py; synchronous, host buffers) ----------
 * linear_interpolation (gsi.py:12-30) of a MOT result table already sorted by (id, frame)
 * (np.lexsort, stable): rows n x ncol float64 (frame, id, ...); for consecutive rows of one id
 * with f_pre + 1 < f < f_pre + interval the missing frames are inserted in front of the row as
 * row_pre + ((row - row_pre) / (f - f_pre)) * i.  virt0 = 1 when the first row's id is -1 (it then
 * pairs with the reference's initial zero row at frame -1, gsi.py:16).  *n_out = rows of the
 * result (YTA_ERR_CAPACITY when > out_cap; out is then untouched). */
int yta_gsi_interpolate(int device, const double *rows, int n, int ncol, int interval, int virt0,
                        double *out, long long out_cap, long long *n_out);
/* gaussian_smooth (gsi.py:33-59): per track k (rows track_off[k] .. track_off[k+1]-1 of t / y),
 * GaussianProcessRegressor(RBF(len_scale[k], 'fixed')).fit(t, y).predict(t) for the 4 columns of
 * y (n x 4: x, y, w, h) -> out (n x 4).  band_width[k] = max(i - j) over the track's pairs with
 * (t_i / l - t_j / l)^2 <= 120 (pairs beyond it have K < e^-60 and are dropped).  A kernel matrix
 * that is not positive definite fails with YTA_ERR_INVALID (sklearn: LinAlgError). */
int yta_gsi_smooth(int device, const double *t, const double *y, const int *track_off,
                   const double *len_scale, const int *band_width, int n_tracks, double *out);

/* ---- ReID crop preprocessing (boxmot/appearance/reid_multibackend.py:189-224) ----------------
 * For each box (x1, y1, x2, y2 float64): box.astype(int) (truncation), x1 = max(0, x1),
 * y1 = max(0, y1), x2 = min(w - 1, x2), y2 = min(h - 1, y2), crop = img[y1:y2, x1:x2] (Python
 * slice semantics: a negative stop counts from the end); cv2.resize(crop, (out_w, out_h),
 * INTER_LINEAR) in OpenCV's fixed-point form (INTER_AREA when both scale factors are exactly 2);
 * BGR -> RGB; (v / 255 - mean) / std in float64 with the ImageNet mean / std of :214-215; stored as
 * float32 (half = 0) or float16 (half = 1, the reference's fp16 .to(torch.half)) into
 * out[n][3][out_h][out_w].  img: h x w x 3 uint8 BGR, row-major.
 * yta_reid_preprocess: synchronous, host buffers; an empty crop fails with YTA_ERR_INVALID naming
 * the box (cv2.resize asserts !ssize.empty()) and nothing is written. */
int yta_reid_preprocess(int device, const uint8_t *img, int h, int w, const double *xyxys, int n,
                        int out_h, int out_w, int half, void *out);
/* Asynchronous device-buffer form over a batch of images (one launch for every box of every
 * camera stream): box b reads image box_img[b] (box_img nullable = image 0) stored at
 * d_imgs + d_img_off[i] with dims d_img_hw[2 i] (h), d_img_hw[2 i + 1] (w).  An empty crop is
 * zero-filled and counted into *d_n_empty (nullable; the caller zeroes it).  stream: a
 * hipStream_t (NULL = the default stream). */
int yta_reid_preprocess_device(const uint8_t *d_imgs, const long long *d_img_off,
                               const int *d_img_hw, const double *d_xyxys, const int *d_box_img,
                               int n, int out_h, int out_w, int half, void *d_out, int *d_n_empty,
                               void *stream);
/* get_features (reid_multibackend.py:310): feats[0..count) /= ||feats||_2 over the whole batch,
 * float32 in place (sum of squares accumulated in float64).  Synchronous, host buffer. */
int yta_reid_normalize(int device, float *feats, long long count);
/* Device form: d_work holds >= 256 doubles of scratch. */
int yta_reid_normalize_device(float *d_feats, long long count, double *d_work, void *stream);

/* ---- Camera-motion compensation: SparseOptFlow (boxmot/motion/cmc/sof.py:15-162) -------------
 * The estimator BoTSORT (bot_sort.py:228, :293) and DeepOCSort (deep_ocsort.py:351, :391) call once
 * per frame: apply(img, dets) -> 2x3 float64 warp.  Per stream: gray (cvtColor BGR2GRAY), resize
 * by `scale` (INTER_LINEAR), on the first frame goodFeaturesToTrack(maxCorners 3000, quality
 * 0.01, minDistance 1, blockSize 3) under generate_mask (cmc_interface.py:13-24: a 2 % border and
 * every det box x scale); afterwards calcOpticalFlowPyrLK (21x21, 3 levels) of the stored corners
 * from the previous accepted frame, estimateAffinePartial2D(RANSAC 3 px, 2000 iters, 0.99) + LM
 * refinement, translation / scale.  The reference's quirks are kept: the corners are detected once
 * and only filtered (sof.py:155 stores the tracked points under another name), a failed estimate
 * returns the identity and keeps the previous frame.  S streams per engine, every stream's frame
 * in the same launches.  Restatement and parity: oracle/cmc_sof.py (unpinned against cv2 itself). */
typedef struct yta_sof yta_sof;
/* max_h / max_w: the largest input frame (pixels) any stream will pass (device-buffer form; the
 * host-buffer form grows them). */
int yta_sof_create(int device, int n_streams, double scale, int max_h, int max_w,
                   yta_sof **engine);
int yta_sof_destroy(yta_sof *engine);
int yta_sof_reset(yta_sof *engine);
/* Host-buffer apply (synchronous).  frames: stream s's h x w x 3 uint8 BGR frame at
 * frames + frame_off[s] (bytes), frame_hw[2 s] = h, frame_hw[2 s + 1] = w; dets: packed float64
 * rows of det_stride (>= 4) columns, x1 y1 x2 y2 first, stream s at rows det_off[s] ..
 * det_off[s+1]-1 (the rows the tracker passes to cmc.apply); warps: S x 6 float64 out. */
int yta_sof_apply(yta_sof *engine, const uint8_t *frames, const long long *frame_off,
                  const int *frame_hw, const double *dets, int det_stride, const int *det_off,
                  double *warps);
/* Device-buffer apply (asynchronous on the engine stream): the same layout in device memory;
 * d_warps (S x 6 float64) can be handed straight to yta_botsort_update_device /
 * yta_deepocsort_update_device. */
int yta_sof_apply_device(yta_sof *engine, const uint8_t *d_frames, const long long *d_frame_off,
                         const int *d_frame_hw, const double *d_dets, int det_stride,
                         const int *d_det_off, double *d_warps);
int yta_sof_sync(yta_sof *engine);
/* Parity introspection of stream s: the stored corners (prev_keypoints, n x 2 float32, up to
 * cap), whether the stream has its first frame, and the stored previous gray frame (h x w uint8,
 * may be NULL). */
int yta_sof_get_state(yta_sof *engine, int stream, int *initialized, int *n_kp, float *kp,
                      int cap, int *h, int *w, uint8_t *prev_img, int img_cap);
/* Last apply's per-stream outcome (S ints): 0 first frame (corners detected or none found),
 * 1 estimated (warp from RANSAC / 2-point model), 2 identity (no corners left / fewer than two
 * tracked / RANSAC found no model). */
int yta_sof_outcome(yta_sof *engine, int *outcome);
int yta_sof_hip_stream(yta_sof *engine, void **stream);

/* Known-answer entries for the estimator's stages (synchronous, host buffers, one image):
 * gray small image (preprocess) of an h x w x 3 BGR frame -> out (round(h*scale) x round(w*scale));
 * min-eigenvalue map (cornerMinEigenVal, blockSize 3, ksize 3) of a gray image -> float32;
 * goodFeaturesToTrack under a mask -> corners (n x 2 float32, up to 3000). */
int yta_sof_kat_preprocess(int device, const uint8_t *frame, int h, int w, double scale,
                           uint8_t *out, int *out_h, int *out_w);
int yta_sof_kat_min_eigen(int device, const uint8_t *gray, int h, int w, float *eig);
int yta_sof_kat_corners(int device, const uint8_t *gray, const uint8_t *mask, int h, int w,
                        float *corners, int *n);
/* calcOpticalFlowPyrLK of n points between two gray images (same size) -> next (n x 2 float32),
 * status (n uint8); estimateAffinePartial2D(RANSAC) + refinement of n point pairs -> M (2 x 3
 * float64), *ok = 0 when no model (fewer than 2 points). */
int yta_sof_kat_lk(int device, const uint8_t *prev, const uint8_t *next, int h, int w,
                   const float *pts, int n, float *next_pts, uint8_t *status);
int yta_sof_kat_affine(int device, const float *src, const float *dst, int n, double *M, int *ok);

/* ---- Camera-motion compensation: ECC (boxmot/motion/cmc/ecc.py:13-104) -------------------------
 * get_cmc_method('ecc') (motion/cmc/__init__.py:9-11, built by hybridsort.py:366): apply(img, dets)
 * -> 2x3 float32 warp = cv2.findTransformECC(prev, curr, eye(2, 3), warp_mode, (COUNT | EPS,
 * max_iter, eps), None, 1) (ecc.py:73-81) on the gray frames resized by `scale`, translation divided
 * by `scale` (ecc.py:87-89); the identity on the first frame (ecc.py:66-68) and when OpenCV raises
 * (NaN correlation, or a step that would minimise it; ecc.py:82-84: prev_img kept).  warp_mode:
 * MOTION_TRANSLATION 0, MOTION_EUCLIDEAN 1 (the reference's default), MOTION_AFFINE 2
 * (MOTION_HOMOGRAPHY is refused; align=True's preview image: yta_ecc_aligned).  S streams per engine, one 1024-thread block runs a stream's
 * whole Gauss-Newton loop.  Restatement and parity: oracle/cmc_ecc.py (unpinned against cv2). */
typedef struct yta_ecc yta_ecc;
int yta_ecc_create(int device, int n_streams, int warp_mode, double eps, int max_iter,
                   double scale, int max_h, int max_w, yta_ecc **engine);
int yta_ecc_destroy(yta_ecc *engine);
int yta_ecc_reset(yta_ecc *engine);
/* Host-buffer apply (synchronous): frames as yta_sof_apply; warps: S x 6 float32 out. */
int yta_ecc_apply(yta_ecc *engine, const uint8_t *frames, const long long *frame_off,
                  const int *frame_hw, float *warps);
/* Device-buffer apply (asynchronous on the engine stream), then yta_ecc_sync. */
int yta_ecc_apply_device(yta_ecc *engine, const uint8_t *d_frames, const long long *d_frame_off,
                         const int *d_frame_hw, float *d_warps);
int yta_ecc_sync(yta_ecc *engine);
/* Last apply per stream (each array S entries, may be NULL): outcome 0 first frame, 1 estimated,
 * 2 identity (OpenCV would have raised); Gauss-Newton iterations run; the final correlation rho. */
int yta_ecc_outcome(yta_ecc *engine, int *outcome, int *iters, double *rho);
/* Whether stream s has its first frame, and its stored previous gray frame (h x w uint8, may be
 * NULL). */
int yta_ecc_get_state(yta_ecc *engine, int stream, int *initialized, int *h, int *w,
                      uint8_t *prev_img, int img_cap);
/* align=True (ecc.py:91-98, replaces the cv2.warpAffine(prev_img, warp, (w, h), INTER_LINEAR)
 * call there): stream s's previous gray frame - the template its last estimate registered against
 * - warped by the returned matrix, h x w uint8 into out (cap bytes).  *h = *w = 0 and nothing
 * written when the last apply was not an estimate (first frame, or OpenCV would have raised: the
 * reference returns before ecc.py:91).  out = NULL: only *h / *w (size query). */
int yta_ecc_aligned(yta_ecc *engine, int stream, uint8_t *out, long long cap, int *h, int *w);
int yta_ecc_hip_stream(yta_ecc *engine, void **stream);

/* ---- OSNet omni-scale block kernels (boxmot/appearance/backbones/osnet.py LightConv3x3 /
 * ChannelGate / OSBlock; the ReID network's forward, appearance/osnet.py).  Device pointers,
 * asynchronous on `stream` (a hipStream_t; NULL = default), NCHW planes, float32 (half = 0) or
 * float16 (half = 1) storage, float32 arithmetic.
 * yta_osnet_dw3x3: per sample n and channel c (plane of H x W at x + n x_n_stride + c x_c_stride,
 * elements): depthwise 3x3 with zero padding 1 (w: C x 9 float32, BatchNorm folded) + b[c] +
 * ReLU; channels c < n_first go to plane c of y_first (sample stride yf_n_stride) and add their
 * plane sum to plane_sum[n ps_n_stride + c] (float32, may be NULL), the others to plane
 * c - n_first of y_rest.  yta_osnet_gate_sum: out[n][c] = sum_b stack[n][b][c] * gate[n][b][c]
 * for the 4 branches (stack N x 4 x C x P, gate N x 4 x C, out N x C x P). */
int yta_osnet_dw3x3(const void *x, long long x_n_stride, long long x_c_stride, const float *w,
                    const float *b, int N, int C, int H, int W, int half, void *y_first,
                    long long yf_n_stride, int n_first, void *y_rest, long long yr_n_stride,
                    float *plane_sum, long long ps_n_stride, void *stream);
int yta_osnet_gate_sum(const void *stack, const void *gate, int N, int C, int P, int half,
                       void *out, void *stream);
/* yta_osnet_pointwise: every 1x1 convolution of the network (osnet.py Conv1x1 / Conv1x1Linear /
 * LightConv3x3.conv1 / the ChannelGate-free layers, the fc) as an MFMA GEMM over strided tensors
 * (elements; sample n, channel c, pixel p of a tensor at base + n * sn + c * sc + p * sp):
 *   y[n][g cout_g + co][p] = relu?( sum_{k < k1} w[g][k][co] x1[n][g k1 + k][p]
 *                                 + sum_{k < k2} w[g][k1 + k][co] x2[n][k][p]
 *                                 + bias[g cout_g + co] + res[n][g cout_g + co][p] )
 * w: float32 [G][k1 + k2][cout_g] (k-major: BatchNorm folded, transposed); bias, x2 (k2 = 0),
 * res may be NULL. */
typedef struct yta_pw_args {
    const void *x1;
    long long x1n, x1c, x1p;
    const void *x2;
    long long x2n, x2c, x2p;
    const float *w;
    const float *bias;
    const void *res;
    long long rn, rc, rp;
    void *y;
    long long yn, yc, yp;
    int k1, k2, G, cout_g, P, N, relu, pad;
} yta_pw_args;
int yta_osnet_pointwise(const yta_pw_args *args, int half, void *stream);
/* yta_osnet_stem: conv1 (7x7, stride 2, padding 3, 3 -> C0 <= 128; w: float32 C0 x 3 x 7 x 7,
 * BatchNorm folded) + b + ReLU: x N x 3 x H x W -> y N x C0 x ((H-1)/2+1) x ((W-1)/2+1).
 * yta_osnet_pool: kind 0 max 3x3 stride 2 padding 1, 1 average 2x2 stride 2, 2 global mean
 * (y N x C).  yta_osnet_gate: the ChannelGate's fc1 + ReLU, fc2 + sigmoid on the four branches'
 * pooled planes (plane_sum N x 4 x mid float32 sums over P pixels; w1 hid x mid, b1 hid, w2
 * mid x hid, b2 mid in the storage type) -> gate N x 4 x mid. */
int yta_osnet_stem(const void *x, int N, int H, int W, const float *w, const float *b, int C0,
                   int half, void *y, void *stream);
int yta_osnet_pool(const void *x, int N, int C, int H, int W, int kind, int half, void *y,
                   void *stream);
int yta_osnet_gate(const float *plane_sum, int N, int mid, int hid, int P, const void *w1,
                   const void *b1, const void *w2, const void *b2, int half, void *gate,
                   void *stream);

#ifdef __cplusplus
}
#endif
#endif
