// Pairwise box affinities, float64, in boxmot/utils/iou.py's exact operation order.
// The library is compiled with -ffp-contract=off so that no a*b+c is fused: every cost is
// bit-identical to NumPy's (KAT: tests/test_kat_gpu.py against tests/golden/kat_iou.npz).
#pragma once
#include "common.hpp"

namespace yta {

struct Box {
    double x1, y1, x2, y2;
};

struct Overlap {
    double inter, iou;
};

// iou.py:13-24 (a = bboxes1 row box, b = bboxes2 column box)
__host__ __device__ __forceinline__ Overlap overlap(const Box &a, const Box &b) {
    double xx1 = np_max(a.x1, b.x1);
    double yy1 = np_max(a.y1, b.y1);
    double xx2 = np_min(a.x2, b.x2);
    double yy2 = np_min(a.y2, b.y2);
    double w = np_max(0.0, xx2 - xx1);
    double h = np_max(0.0, yy2 - yy1);
    double wh = w * h;
    double area_a = (a.x2 - a.x1) * (a.y2 - a.y1);
    double area_b = (b.x2 - b.x1) * (b.y2 - b.y1);
    Overlap o;
    o.inter = wh;
    o.iou = wh / (area_a + area_b - wh);
    return o;
}

__host__ __device__ __forceinline__ double iou(const Box &a, const Box &b) { return overlap(a, b).iou; }

// True when the intersection is non-empty, i.e. np_min(x2) - np_max(x1) > 0 on both axes.  If
// false, iou() is +-0 or NaN, so every "1 - iou < thresh" test with thresh <= 1 fails: such pairs
// can never be association edges.  Written as plain comparisons, which is the same predicate for
// every input: with a NaN both forms are false; otherwise min - max > 0 <=> min > max (the
// difference of two distinct doubles never rounds to 0, inf - inf = NaN fails like inf > inf).
__host__ __device__ __forceinline__ bool intersects(const Box &a, const Box &b) {
    return a.x2 > a.x1 && a.x2 > b.x1 && b.x2 > a.x1 && b.x2 > b.x1 &&
           a.y2 > a.y1 && a.y2 > b.y1 && b.y2 > a.y1 && b.y2 > b.y1;
}

// iou.py:28-62.  Returns NaN where the reference would raise on its enclosure assert (:58); the
// host wrapper turns that into an error.
__host__ __device__ __forceinline__ double giou(const Box &a, const Box &b) {
    Overlap o = overlap(a, b);
    double wc = np_max(a.x2, b.x2) - np_min(a.x1, b.x1);
    double hc = np_max(a.y2, b.y2) - np_min(a.y1, b.y1);
    double enc = wc * hc;
    double g = o.iou - (enc - o.inter) / enc;
    return (g + 1.0) / 2.0;
}

__host__ __device__ __forceinline__ void centre_terms(const Box &a, const Box &b, double &inner,
                                                      double &outer) {
    double cxa = (a.x1 + a.x2) / 2.0, cya = (a.y1 + a.y2) / 2.0;
    double cxb = (b.x1 + b.x2) / 2.0, cyb = (b.y1 + b.y2) / 2.0;
    double dx = cxa - cxb, dy = cya - cyb;
    inner = dx * dx + dy * dy;
    double ex = np_max(a.x2, b.x2) - np_min(a.x1, b.x1);
    double ey = np_max(a.y2, b.y2) - np_min(a.y1, b.y1);
    outer = ex * ex + ey * ey;
}

// iou.py:65-105
__host__ __device__ __forceinline__ double diou(const Box &a, const Box &b) {
    Overlap o = overlap(a, b);
    double inner, outer;
    centre_terms(a, b, inner, outer);
    double d = o.iou - inner / outer;
    return (d + 1) / 2.0;
}

// iou.py:108-161 (arctan is not correctly rounded on either side: KAT within 1e-12, not bitwise)
__host__ __device__ __forceinline__ double ciou(const Box &a, const Box &b) {
    Overlap o = overlap(a, b);
    double inner, outer;
    centre_terms(a, b, inner, outer);
    double wa = a.x2 - a.x1, ha = a.y2 - a.y1;
    double wb = b.x2 - b.x1, hb = b.y2 - b.y1;
    hb = hb + 1.0;
    ha = ha + 1.0;
    double at = atan(wb / hb) - atan(wa / ha);
    const double k4pi2 = 4.0 / (3.141592653589793 * 3.141592653589793);
    double v = k4pi2 * (at * at);
    double s = 1 - o.iou;
    double alpha = v / (s + v);
    double c = o.iou - inner / outer - alpha * v;
    return (c + 1) / 2.0;
}

// iou.py:164-188
__host__ __device__ __forceinline__ double centroid(const Box &a, const Box &b, double img_w,
                                                    double img_h) {
    double cxa = (a.x1 + a.x2) / 2, cya = (a.y1 + a.y2) / 2;
    double cxb = (b.x1 + b.x2) / 2, cyb = (b.y1 + b.y2) / 2;
    double dx = cxa - cxb, dy = cya - cyb;
    double dist = sqrt(dx * dx + dy * dy);
    double norm = sqrt(img_w * img_w + img_h * img_h);
    return 1 - dist / norm;
}

// ByteTrack detection boxes: STrack(det) stores xywh = xyxy2xywh(det) (ops.py:7-21) and its
// `xyxy` property converts back with xywh2xyxy (ops.py:24-40) - not the identity in float64.
__host__ __device__ __forceinline__ void det_xyxy_to_xywh(const double *d, double *xywh) {
    xywh[0] = (d[0] + d[2]) / 2;
    xywh[1] = (d[1] + d[3]) / 2;
    xywh[2] = d[2] - d[0];
    xywh[3] = d[3] - d[1];
}
__host__ __device__ __forceinline__ Box xywh_to_box(const double *b) {
    Box r;
    r.x1 = b[0] - b[2] / 2;
    r.y1 = b[1] - b[3] / 2;
    r.x2 = b[0] + b[2] / 2;
    r.y2 = b[1] + b[3] / 2;
    return r;
}
// ops.xywh2tlwh (:43-58) then ops.tlwh2xyah (:87-97)
__host__ __device__ __forceinline__ void xywh_to_xyah(const double *b, double *z) {
    double t = b[0] - b[2] / 2.0;
    double l = b[1] - b[3] / 2.0;
    z[0] = t + b[2] / 2;
    z[1] = l + b[3] / 2;
    z[2] = b[2] / b[3];
    z[3] = b[3];
}
// STrack.xyxy from a Kalman mean (byte_tracker.py:100-111): w = a*h, then xywh2xyxy
__host__ __device__ __forceinline__ Box xyah_mean_to_box(double xc, double yc, double a, double h) {
    double b[4] = {xc, yc, a * h, h};
    return xywh_to_box(b);
}

}  // namespace yta
