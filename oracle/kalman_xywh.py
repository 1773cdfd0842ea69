"""ORACLE — test infrastructure only.  BoT-SORT's constant-velocity Kalman filter in (xc, yc, w, h)
space, restated from boxmot/motion/kalman_filters/botsort_kf.py with the same NumPy / SciPy
operations (so results are bit-identical to the reference on the same host), plus the camera-
motion compensation of STrack.multi_gmc (boxmot/trackers/botsort/bot_sort.py:95-111).

State  : [xc, yc, w, h, vxc, vyc, vw, vh] (8), covariance 8x8, dt = 1.
Noise  : std weights position 1/20, velocity 1/160 (botsort_kf.py:40-41); x / w terms scale with
         the width mean[2], y / h terms with the height mean[3].
"""
import numpy as np
import scipy.linalg

W_POS = 1.0 / 20
W_VEL = 1.0 / 160

F = np.eye(8)
for _i in range(4):
    F[_i, 4 + _i] = 1.0       # botsort_kf.py:35-37
H = np.eye(4, 8)              # botsort_kf.py:38


def initiate(z):
    """botsort_kf.py:43-73."""
    mean = np.r_[z, np.zeros_like(z)]
    std = [2 * W_POS * z[2], 2 * W_POS * z[3], 2 * W_POS * z[2], 2 * W_POS * z[3],
           10 * W_VEL * z[2], 10 * W_VEL * z[3], 10 * W_VEL * z[2], 10 * W_VEL * z[3]]
    return mean, np.diag(np.square(std))


def multi_predict(mean, cov):
    """botsort_kf.py:150-190 over N stacked states."""
    std_pos = [W_POS * mean[:, 2], W_POS * mean[:, 3], W_POS * mean[:, 2], W_POS * mean[:, 3]]
    std_vel = [W_VEL * mean[:, 2], W_VEL * mean[:, 3], W_VEL * mean[:, 2], W_VEL * mean[:, 3]]
    sqr = np.square(np.r_[std_pos, std_vel]).T
    motion_cov = np.asarray([np.diag(sqr[i]) for i in range(len(mean))])
    mean = np.dot(mean, F.T)
    left = np.dot(F, cov).transpose((1, 0, 2))
    cov = np.dot(left, F.T) + motion_cov
    return mean, cov


def project(mean, cov):
    """botsort_kf.py:110-148."""
    std = [W_POS * mean[2], W_POS * mean[3], W_POS * mean[2], W_POS * mean[3]]
    innovation_cov = np.diag(np.square(std))
    mean = np.dot(H, mean)
    cov = np.linalg.multi_dot((H, cov, H.T))
    return mean, cov + innovation_cov


def update(mean, cov, z):
    """botsort_kf.py:192-226."""
    projected_mean, projected_cov = project(mean, cov)
    chol, lower = scipy.linalg.cho_factor(projected_cov, lower=True, check_finite=False)
    gain = scipy.linalg.cho_solve((chol, lower), np.dot(cov, H.T).T, check_finite=False).T
    innovation = z - projected_mean
    new_mean = mean + np.dot(innovation, gain.T)
    new_cov = cov - np.linalg.multi_dot((gain, projected_cov, gain.T))
    return new_mean, new_cov


def gmc(mean, cov, warp):
    """STrack.multi_gmc for one track (bot_sort.py:95-111): R8 = kron(I4, R), mean <- R8 mean + t,
    cov <- R8 cov R8^T."""
    warp = np.asarray(warp, np.float64)
    r8 = np.kron(np.eye(4, dtype=float), warp[:2, :2])
    m = r8.dot(mean)
    m[:2] += warp[:2, 2]
    return m, r8.dot(cov).dot(r8.transpose())
