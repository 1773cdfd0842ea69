"""ctypes binding of the gfx950 C-ABI library (include/yolo_tracking_amd.h -> libyta.so).

There is no CPU fallback: if the library is missing, or no HIP device is present, every tracker
call raises `YTAError`.  `build()` in __graft_entry__.py (or `make -C yolo_tracking_amd/csrc`)
produces the library in-tree.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# YTA_LIBRARY: an alternative build of the same library (tuning experiments, tools/)
LIB_PATH = os.environ.get("YTA_LIBRARY") or os.path.join(_HERE, "libyta.so")


class PwArgs(ctypes.Structure):
    """yta_pw_args (include/yolo_tracking_amd.h): one 1x1 convolution / linear layer."""
    _fields_ = [("x1", ctypes.c_void_p), ("x1n", ctypes.c_longlong), ("x1c", ctypes.c_longlong),
                ("x1p", ctypes.c_longlong), ("x2", ctypes.c_void_p), ("x2n", ctypes.c_longlong),
                ("x2c", ctypes.c_longlong), ("x2p", ctypes.c_longlong), ("w", ctypes.c_void_p),
                ("bias", ctypes.c_void_p), ("res", ctypes.c_void_p), ("rn", ctypes.c_longlong),
                ("rc", ctypes.c_longlong), ("rp", ctypes.c_longlong), ("y", ctypes.c_void_p),
                ("yn", ctypes.c_longlong), ("yc", ctypes.c_longlong), ("yp", ctypes.c_longlong),
                ("k1", ctypes.c_int), ("k2", ctypes.c_int), ("G", ctypes.c_int),
                ("cout_g", ctypes.c_int), ("P", ctypes.c_int), ("N", ctypes.c_int),
                ("relu", ctypes.c_int), ("pad", ctypes.c_int)]


YTA_OK = 0
YTA_ERR_INVALID = -1
YTA_ERR_HIP = -2
YTA_ERR_CAPACITY = -3
YTA_ERR_NOMEM = -4

AFF_KINDS = {"iou": 0, "giou": 1, "diou": 2, "ciou": 3, "centroid": 4}


class YTAError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"yolo_tracking_amd error {code}: {msg}")
        self.code = code


class CapacityError(YTAError):
    pass


class BtParams(ctypes.Structure):
    _fields_ = [("track_thresh", ctypes.c_double), ("match_thresh", ctypes.c_double),
                ("track_buffer", ctypes.c_int), ("frame_rate", ctypes.c_int)]


class BotParams(ctypes.Structure):
    """yta_botsort_params (include/yolo_tracking_amd.h)."""
    _fields_ = [("track_high_thresh", ctypes.c_double), ("track_low_thresh", ctypes.c_double),
                ("new_track_thresh", ctypes.c_double), ("match_thresh", ctypes.c_double),
                ("proximity_thresh", ctypes.c_double), ("appearance_thresh", ctypes.c_double),
                ("track_buffer", ctypes.c_int), ("frame_rate", ctypes.c_int),
                ("fuse_first_associate", ctypes.c_int), ("with_reid", ctypes.c_int)]


class OcParams(ctypes.Structure):
    """yta_ocsort_params (include/yolo_tracking_amd.h)."""
    _fields_ = [("det_thresh", ctypes.c_double), ("max_age", ctypes.c_int),
                ("min_hits", ctypes.c_int), ("asso_threshold", ctypes.c_double),
                ("delta_t", ctypes.c_int), ("asso_func", ctypes.c_int),
                ("inertia", ctypes.c_double), ("use_byte", ctypes.c_int)]


class DocParams(ctypes.Structure):
    """yta_deepocsort_params (include/yolo_tracking_amd.h)."""
    _fields_ = [("det_thresh", ctypes.c_double), ("max_age", ctypes.c_int),
                ("min_hits", ctypes.c_int), ("iou_threshold", ctypes.c_double),
                ("delta_t", ctypes.c_int), ("asso_func", ctypes.c_int),
                ("inertia", ctypes.c_double), ("w_association_emb", ctypes.c_double),
                ("alpha_fixed_emb", ctypes.c_double), ("aw_param", ctypes.c_double),
                ("embedding_off", ctypes.c_int), ("cmc_off", ctypes.c_int),
                ("aw_off", ctypes.c_int)]


class HsParams(ctypes.Structure):
    """yta_hybridsort_params (include/yolo_tracking_amd.h)."""
    _fields_ = [("det_thresh", ctypes.c_double), ("max_age", ctypes.c_int),
                ("min_hits", ctypes.c_int), ("iou_threshold", ctypes.c_double),
                ("delta_t", ctypes.c_int), ("asso_func", ctypes.c_int),
                ("inertia", ctypes.c_double)]


ASSO_FUNCS = {"iou": 0, "giou": 1, "diou": 2, "ciou": 3, "centroid": 4}

_lib = None

_P = ctypes.c_void_p
_I = ctypes.c_int
_D = ctypes.c_double

_SIGS = {
    "yta_version": ([], _I),
    "yta_last_error": ([], ctypes.c_char_p),
    "yta_device_count": ([_P], _I),
    "yta_box_affinity": ([_I, _I, _P, _I, _P, _I, _D, _D, _P], _I),
    "yta_iou_distance": ([_I, _P, _I, _P, _I, _P, _P], _I),
    "yta_kf_xyah_initiate": ([_I, _I, _P, _P, _P], _I),
    "yta_kf_xyah_predict": ([_I, _I, _P, _P], _I),
    "yta_kf_xyah_update": ([_I, _I, _P, _P, _P], _I),
    "yta_grid_pairs": ([_I, _P, _I, _P, _I, _D, _P, _I, _P], _I),
    "yta_lap_limited": ([_I, _I, _I, _P, _D, _P, _P], _I),
    "yta_lap_padded": ([_I, _I, _I, _P, _P, _P], _I),
    "yta_lap_rect": ([_I, _I, _I, _P, _P, _P], _I),
    "yta_lap_first_round": ([_I, _I, _I, _P, _P, _P, _P], _I),
    "yta_affine_apply": ([_I, _I, _I, _P, _P, _P], _I),
    "yta_bytetrack_create": ([_I, _I, _I, _I, _P, _P], _I),
    "yta_bytetrack_destroy": ([_P], _I),
    "yta_bytetrack_reset": ([_P], _I),
    "yta_bytetrack_reserve": ([_P, _I, _I], _I),
    "yta_bytetrack_capacity": ([_P, _P, _P], _I),
    "yta_bytetrack_update": ([_P, _P, _P, _P, _P, _I, _P], _I),
    "yta_bytetrack_update_device": ([_P, _P, _P, _P, _P], _I),
    "yta_bytetrack_sync": ([_P], _I),
    "yta_bytetrack_update_streams": ([_P, _I, _P, _P, _P, _P, _P, _I, _P], _I),
    "yta_bytetrack_update_device_masked": ([_P, _P, _P, _P, _P, _P], _I),
    "yta_bytetrack_reset_stream": ([_P, _I], _I),
    "yta_bytetrack_submit": ([_P, _P, _P, _P, _P, _I], _I),
    "yta_bytetrack_collect": ([_P, _P, _P], _I),
    "yta_bytetrack_pipe_stats": ([_P, _P, _I, _I], _I),
    "yta_bytetrack_next_ids": ([_P, _P], _I),
    "yta_bytetrack_submit_f32": ([_P, _P, _P, _P, _P, _I], _I),
    "yta_bytetrack_update_f32": ([_P, _P, _P, _P, _P, _I, _P], _I),
    "yta_bytetrack_get_state": ([_P, _I, _P, _P, _P, _P], _I),
    "yta_bytetrack_profile": ([_P, _I], _I),
    "yta_bytetrack_profile_collect": ([_P, _P, _P], _I),
    "yta_bytetrack_stats": ([_P, _P], _I),
    "yta_bytetrack_modes": ([_P, _P, _I], _I),
    "yta_bytetrack_hip_stream": ([_P, _P], _I),
    "yta_bytetrack_set_lds": ([_P, _I], _I),
    "yta_selftest": ([_I], _I),
    "yta_botsort_create": ([_I, _I, _I, _I, _I, _P, _P], _I),
    "yta_botsort_update": ([_P, _P, _P, _P, _P, _P, _P, _I, _P], _I),
    "yta_botsort_update_device": ([_P, _P, _P, _P, _P, _P, _P], _I),
    "yta_botsort_get_features": ([_P, _I, _P, _P, _P, _P], _I),
    "yta_botsort_update_streams": ([_P, _I, _P, _P, _P, _P, _P, _P, _P, _I, _P], _I),
    "yta_ocsort_create": ([_I, _I, _I, _I, _P, _P], _I),
    "yta_ocsort_destroy": ([_P], _I),
    "yta_ocsort_reset": ([_P], _I),
    "yta_ocsort_capacity": ([_P, _P, _P], _I),
    "yta_ocsort_update": ([_P, _P, _P, _P, _P, _P, _I, _P], _I),
    "yta_ocsort_update_device": ([_P, _P, _P, _P, _P, _P], _I),
    "yta_ocsort_update_streams": ([_P, _I, _P, _P, _P, _P, _P, _P, _I, _P], _I),
    "yta_ocsort_update_device_masked": ([_P, _P, _P, _P, _P, _P, _P], _I),
    "yta_ocsort_reset_stream": ([_P, _I], _I),
    "yta_ocsort_sync": ([_P], _I),
    "yta_ocsort_get_state": ([_P, _I, _P, _P, _P, _P], _I),
    "yta_ocsort_stats": ([_P, _P], _I),
    "yta_ocsort_lap_stats": ([_P, _P, _I], _I),
    "yta_ocsort_hip_stream": ([_P, _P], _I),
    "yta_kf7_run": ([_I, _I, _I, _P, _P, _P, _P], _I),
    "yta_deepocsort_create": ([_I, _I, _I, _I, _I, _P, _P], _I),
    "yta_deepocsort_destroy": ([_P], _I),
    "yta_deepocsort_reset": ([_P], _I),
    "yta_deepocsort_capacity": ([_P, _P, _P], _I),
    "yta_deepocsort_update": ([_P, _P, _P, _P, _P, _P, _P, _P, _I, _P], _I),
    "yta_deepocsort_update_device": ([_P, _P, _P, _P, _P, _P, _P, _P], _I),
    "yta_deepocsort_update_streams": ([_P, _I, _P, _P, _P, _P, _P, _P, _P, _P, _I, _P], _I),
    "yta_deepocsort_update_device_masked": ([_P, _P, _P, _P, _P, _P, _P, _P, _P], _I),
    "yta_deepocsort_reset_stream": ([_P, _I], _I),
    "yta_deepocsort_sync": ([_P], _I),
    "yta_deepocsort_get_state": ([_P, _I, _P, _P, _P, _P, _P], _I),
    "yta_deepocsort_stats": ([_P, _P], _I),
    "yta_deepocsort_lap_stats": ([_P, _P, _I], _I),
    "yta_deepocsort_hip_stream": ([_P, _P], _I),
    "yta_kf8_run": ([_I, _I, _I, _P, _P, _P, _P, _P], _I),
    "yta_hybridsort_create": ([_I, _I, _I, _I, _I, _P, _P], _I),
    "yta_hybridsort_destroy": ([_P], _I),
    "yta_hybridsort_reset": ([_P], _I),
    "yta_hybridsort_capacity": ([_P, _P, _P], _I),
    "yta_hybridsort_update": ([_P, _P, _P, _P, _P, _P, _I, _P], _I),
    "yta_hybridsort_update_device": ([_P, _P, _P, _P, _P, _P], _I),
    "yta_hybridsort_update_streams": ([_P, _I, _P, _P, _P, _P, _P, _P, _I, _P], _I),
    "yta_hybridsort_update_device_masked": ([_P, _P, _P, _P, _P, _P, _P], _I),
    "yta_hybridsort_reset_stream": ([_P, _I], _I),
    "yta_hybridsort_sync": ([_P], _I),
    "yta_hybridsort_get_state": ([_P, _I, _P, _P, _P, _P, _P, _P], _I),
    "yta_hybridsort_classes": ([_P, _I, _P, _I, _P], _I),
    "yta_hybridsort_stats": ([_P, _P], _I),
    "yta_hybridsort_lap_stats": ([_P, _P, _I], _I),
    "yta_hybridsort_hip_stream": ([_P, _P], _I),
    "yta_kf9_run": ([_I, _I, _I, _P, _P, _P, _P], _I),
    "yta_gsi_interpolate": ([_I, _P, _I, _I, _I, _I, _P, ctypes.c_longlong, _P], _I),
    "yta_gsi_smooth": ([_I, _P, _P, _P, _P, _P, _I, _P], _I),
    "yta_embedding_distance": ([_I, _P, _I, _P, _I, _I, _P], _I),
    "yta_aw_max_metric": ([_I, _P, _I, _I, ctypes.c_double, ctypes.c_double, _P], _I),
    "yta_reid_preprocess": ([_I, _P, _I, _I, _P, _I, _I, _I, _I, _P], _I),
    "yta_reid_preprocess_device": ([_P, _P, _P, _P, _P, _I, _I, _I, _I, _P, _P, _P], _I),
    "yta_reid_normalize": ([_I, _P, ctypes.c_longlong], _I),
    "yta_reid_normalize_device": ([_P, ctypes.c_longlong, _P, _P], _I),
    "yta_sof_create": ([_I, _I, _D, _I, _I, _P], _I),
    "yta_sof_destroy": ([_P], _I),
    "yta_sof_reset": ([_P], _I),
    "yta_sof_apply": ([_P, _P, _P, _P, _P, _I, _P, _P], _I),
    "yta_sof_apply_device": ([_P, _P, _P, _P, _P, _I, _P, _P], _I),
    "yta_sof_sync": ([_P], _I),
    "yta_sof_get_state": ([_P, _I, _P, _P, _P, _I, _P, _P, _P, _I], _I),
    "yta_sof_outcome": ([_P, _P], _I),
    "yta_sof_hip_stream": ([_P, _P], _I),
    "yta_sof_kat_preprocess": ([_I, _P, _I, _I, _D, _P, _P, _P], _I),
    "yta_sof_kat_min_eigen": ([_I, _P, _I, _I, _P], _I),
    "yta_sof_kat_corners": ([_I, _P, _P, _I, _I, _P, _P], _I),
    "yta_sof_kat_lk": ([_I, _P, _P, _I, _I, _P, _I, _P, _P], _I),
    "yta_sof_kat_affine": ([_I, _P, _P, _I, _P, _P], _I),
    "yta_ecc_create": ([_I, _I, _I, _D, _I, _D, _I, _I, _P], _I),
    "yta_ecc_destroy": ([_P], _I),
    "yta_ecc_reset": ([_P], _I),
    "yta_ecc_apply": ([_P, _P, _P, _P, _P], _I),
    "yta_ecc_apply_device": ([_P, _P, _P, _P, _P], _I),
    "yta_ecc_sync": ([_P], _I),
    "yta_ecc_outcome": ([_P, _P, _P, _P], _I),
    "yta_ecc_get_state": ([_P, _I, _P, _P, _P, _P, _I], _I),
    "yta_ecc_aligned": ([_P, _I, _P, ctypes.c_longlong, _P, _P], _I),
    "yta_ecc_hip_stream": ([_P, _P], _I),
    "yta_osnet_dw3x3": ([_P, ctypes.c_longlong, ctypes.c_longlong, _P, _P, _I, _I, _I, _I, _I, _P,
                         ctypes.c_longlong, _I, _P, ctypes.c_longlong, _P, ctypes.c_longlong, _P],
                        _I),
    "yta_osnet_gate_sum": ([_P, _P, _I, _I, _I, _I, _P, _P], _I),
    "yta_osnet_pointwise": ([_P, _I, _P], _I),
    "yta_osnet_stem": ([_P, _I, _I, _I, _P, _P, _I, _I, _P, _P], _I),
    "yta_osnet_pool": ([_P, _I, _I, _I, _I, _I, _I, _P, _P], _I),
    "yta_osnet_gate": ([_P, _I, _I, _I, _I, _P, _P, _P, _P, _I, _P, _P], _I),
}

EXPORTED_SYMBOLS = tuple(_SIGS)


def load_library(path=None):
    """Load (once) and return the ctypes handle; raises if the library is absent."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise YTAError(YTA_ERR_HIP, f"HIP library not built: {p} (run __graft_entry__.build() "
                                    "or `make -C yolo_tracking_amd/csrc`)")
    lib = ctypes.CDLL(p)
    for name, (args, res) in _SIGS.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res
    if path is None:
        _lib = lib
    return lib


def check(rc):
    if rc != YTA_OK:
        msg = load_library().yta_last_error()
        msg = msg.decode() if msg else ""
        cls = CapacityError if rc == YTA_ERR_CAPACITY else YTAError
        raise cls(rc, msg)


def device_count():
    n = ctypes.c_int(0)
    check(load_library().yta_device_count(ctypes.byref(n)))
    return n.value


def ptr(a):
    return a.ctypes.data if a is not None else None


def parse_device(device):
    """Map the reference's `device` argument ('cpu', '0', 'cuda:1', 1, torch.device) to a HIP
    ordinal.  The tracker arithmetic always runs on an MI355X; 'cpu' (which in the reference only
    places the ReID model) selects device 0."""
    if device is None:
        return 0
    if isinstance(device, int):
        return device
    s = str(device).strip().lower()
    if s in ("", "cpu", "cuda", "gpu"):
        return 0
    if ":" in s:
        s = s.split(":", 1)[1]
    s = s.split(",")[0]
    try:
        return int(s)
    except ValueError:
        return 0


# ------------------------------------------------------------------------- primitive wrappers
def box_affinity(a, b, kind="iou", img_w=0.0, img_h=0.0, device=0):
    a = np.ascontiguousarray(a, dtype=np.float64).reshape(-1, 4)
    b = np.ascontiguousarray(b, dtype=np.float64).reshape(-1, 4)
    out = np.empty((len(a), len(b)), dtype=np.float64)
    check(load_library().yta_box_affinity(device, AFF_KINDS[kind], ptr(a), len(a), ptr(b), len(b),
                                          float(img_w), float(img_h), ptr(out)))
    return out


def iou_distance(a, b, scores=None, device=0):
    a = np.ascontiguousarray(a, dtype=np.float64).reshape(-1, 4)
    b = np.ascontiguousarray(b, dtype=np.float64).reshape(-1, 4)
    s = None if scores is None else np.ascontiguousarray(scores, dtype=np.float64)
    out = np.empty((len(a), len(b)), dtype=np.float64)
    check(load_library().yta_iou_distance(device, ptr(a), len(a), ptr(b), len(b), ptr(s), ptr(out)))
    return out


def kf_xyah_initiate(meas, device=0):
    meas = np.ascontiguousarray(meas, dtype=np.float64).reshape(-1, 4)
    n = len(meas)
    mean = np.empty((n, 8))
    cov = np.empty((n, 8, 8))
    check(load_library().yta_kf_xyah_initiate(device, n, ptr(meas), ptr(mean), ptr(cov)))
    return mean, cov


def kf_xyah_predict(mean, cov, device=0):
    mean = np.array(mean, dtype=np.float64, order="C").reshape(-1, 8)
    cov = np.array(cov, dtype=np.float64, order="C").reshape(-1, 8, 8)
    check(load_library().yta_kf_xyah_predict(device, len(mean), ptr(mean), ptr(cov)))
    return mean, cov


def kf_xyah_update(mean, cov, z, device=0):
    mean = np.array(mean, dtype=np.float64, order="C").reshape(-1, 8)
    cov = np.array(cov, dtype=np.float64, order="C").reshape(-1, 8, 8)
    z = np.ascontiguousarray(z, dtype=np.float64).reshape(-1, 4)
    check(load_library().yta_kf_xyah_update(device, len(mean), ptr(mean), ptr(cov), ptr(z)))
    return mean, cov


def grid_pairs(a, b, thresh, device=0):
    """All (i, j) with 1 - IoU(a_i, b_j) < thresh, found through the device grid (sorted)."""
    a = np.ascontiguousarray(a, dtype=np.float64).reshape(-1, 4)
    b = np.ascontiguousarray(b, dtype=np.float64).reshape(-1, 4)
    cap = max(16, 8 * (len(a) + len(b)))
    while True:
        pairs = np.empty((cap, 2), dtype=np.int32)
        n = ctypes.c_int()
        check(load_library().yta_grid_pairs(device, ptr(a), len(a), ptr(b), len(b), float(thresh),
                                            ptr(pairs), cap, ctypes.byref(n)))
        if n.value <= cap:
            p = pairs[:n.value]
            return p[np.lexsort((p[:, 1], p[:, 0]))]
        cap = n.value


def kf7_run(z0, z, device=0):
    """OCSORT Kalman KAT (yta_kf7_run): z0 (n, 4), z (steps, n, 4) with NaN rows = missed."""
    z0 = np.ascontiguousarray(z0, dtype=np.float64).reshape(-1, 4)
    n = len(z0)
    z = np.ascontiguousarray(z, dtype=np.float64).reshape(-1, n, 4)
    x = np.empty((n, 7))
    P = np.empty((n, 7, 7))
    check(load_library().yta_kf7_run(device, n, len(z), ptr(z0), ptr(z), ptr(x), ptr(P)))
    return x, P


def kf8_run(b0, b, warps=None, device=0):
    """DeepOCSORT KalmanBoxTracker KAT (yta_kf8_run): b0 (n, 4) boxes, b (steps, n, 4) with NaN
    rows = missed, warps (steps, n, 2, 3) or None."""
    b0 = np.ascontiguousarray(b0, dtype=np.float64).reshape(-1, 4)
    n = len(b0)
    b = np.ascontiguousarray(b, dtype=np.float64).reshape(-1, n, 4)
    w = None if warps is None else np.ascontiguousarray(warps, dtype=np.float64).reshape(-1, n, 6)
    x = np.empty((n, 8))
    P = np.empty((n, 8, 8))
    check(load_library().yta_kf8_run(device, n, len(b), ptr(b0), ptr(b), ptr(w), ptr(x), ptr(P)))
    return x, P


def kf9_run(b0, b, device=0):
    """HybridSORT KalmanBoxTracker KAT (yta_kf9_run): b0 (n, 5) rows x1 y1 x2 y2 score, b
    (steps, n, 5) with NaN rows = missed."""
    b0 = np.ascontiguousarray(b0, dtype=np.float64).reshape(-1, 5)
    n = len(b0)
    b = np.ascontiguousarray(b, dtype=np.float64).reshape(-1, n, 5)
    x = np.empty((n, 9))
    P = np.empty((n, 9, 9))
    check(load_library().yta_kf9_run(device, n, len(b), ptr(b0), ptr(b), ptr(x), ptr(P)))
    return x, P


def embedding_distance(track_feats, det_feats, device=0):
    """matching.py:145-167 embedding_distance on the device -> (n, m) float64."""
    t = np.ascontiguousarray(track_feats, dtype=np.float32)
    d = np.ascontiguousarray(det_feats, dtype=np.float32)
    n, m = len(t), len(d)
    out = np.zeros((n, m), dtype=np.float64)
    if n * m:
        assert t.shape[1] == d.shape[1]
        check(load_library().yta_embedding_distance(device, ptr(t), n, ptr(d), m, t.shape[1],
                                                    ptr(out)))
    return out


def aw_max_metric(emb_cost, w_association_emb, bottom=0.5, device=0):
    """association.py:79-108 compute_aw_max_metric on the device."""
    e = np.ascontiguousarray(emb_cost, dtype=np.float64)
    out = np.empty_like(e)
    check(load_library().yta_aw_max_metric(device, ptr(e), e.shape[0], e.shape[1],
                                           float(w_association_emb), float(bottom), ptr(out)))
    return out


def lap_padded(cost, device=0):
    """lap.lapjv(cost, extend_cost=True) -> (x, y) (association.py:20-28)."""
    c = np.ascontiguousarray(cost, dtype=np.float64)
    nr, nc = c.shape
    x = np.empty(nr, dtype=np.int32)
    y = np.empty(nc, dtype=np.int32)
    check(load_library().yta_lap_padded(device, nr, nc, ptr(c), ptr(x), ptr(y)))
    return x, y


def lap_rect(cost, device=0):
    """The padded problem's optimum by the OCSORT-family rectangular solver (lap_rect.hpp)."""
    c = np.ascontiguousarray(cost, dtype=np.float64)
    nr, nc = c.shape
    x = np.empty(nr, dtype=np.int32)
    y = np.empty(nc, dtype=np.int32)
    check(load_library().yta_lap_rect(device, nr, nc, ptr(c), ptr(x), ptr(y)))
    return x, y


def affine_apply(kind, warps, mean, cov, device=0):
    """Camera-motion correction of n Kalman states (yta_affine_apply): kind 0 BoT-SORT multi_gmc,
    kind 1 DeepOCSORT apply_affine_correction.  Returns new (mean (n, 8), cov (n, 8, 8))."""
    w = np.ascontiguousarray(warps, dtype=np.float64).reshape(-1, 6)
    m = np.array(mean, dtype=np.float64).reshape(-1, 8)
    c = np.array(cov, dtype=np.float64).reshape(-1, 8, 8)
    assert len(w) == len(m) == len(c)
    check(load_library().yta_affine_apply(device, int(kind), len(m), ptr(w), ptr(m), ptr(c)))
    return m, c


def lap_first_round(cost, device=0):
    """The OCSORT-family first-round solve as the engines run it -> (rx, done, n_tight): rx[i] =
    column of row i or -1; done = False when the engine would replay lapjv (rows > columns and
    the optimum not certified unique); n_tight = tight non-matching edges the uniqueness
    certificate examined (-1 unless rows > columns)."""
    c = np.ascontiguousarray(cost, dtype=np.float64)
    na, nb = c.shape
    rx = np.empty(na, dtype=np.int32)
    done = ctypes.c_int(0)
    nt = ctypes.c_int(0)
    check(load_library().yta_lap_first_round(device, na, nb, ptr(c), ptr(rx), ctypes.byref(done),
                                             ctypes.byref(nt)))
    return rx, bool(done.value), nt.value


def lap_limited(cost, cost_limit, device=0):
    """lap.lapjv(cost, extend_cost=True, cost_limit=cost_limit) -> (x, y)."""
    c = np.ascontiguousarray(cost, dtype=np.float64)
    nr, nc = c.shape
    x = np.empty(nr, dtype=np.int32)
    y = np.empty(nc, dtype=np.int32)
    check(load_library().yta_lap_limited(device, nr, nc, ptr(c), float(cost_limit), ptr(x), ptr(y)))
    return x, y
