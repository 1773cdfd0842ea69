"""ORACLE — test infrastructure only.  ByteTrack's constant-velocity Kalman filter in (x, y, a, h)
space, restated from boxmot/motion/kalman_filters/bytetrack_kf.py.

State  : [xc, yc, a, h, vxc, vyc, va, vh]  (8), covariance 8x8, dt = 1.
Noise  : std weights position 1/20, velocity 1/160 (bytetrack_kf.py:52-53), all scaled by h.
"""
import numpy as np

W_POS = 1.0 / 20
W_VEL = 1.0 / 160

F = np.eye(8)
F[:4, 4:] = np.eye(4)        # bytetrack_kf.py:44-46
H = np.eye(4, 8)             # bytetrack_kf.py:47


def initiate(z):
    """bytetrack_kf.py:55-86."""
    h = z[3]
    mean = np.concatenate([np.asarray(z, np.float64), np.zeros(4)])
    std = np.array([2 * W_POS * h, 2 * W_POS * h, 1e-2, 2 * W_POS * h,
                    10 * W_VEL * h, 10 * W_VEL * h, 1e-5, 10 * W_VEL * h])
    return mean, np.diag(np.square(std))


def multi_predict(mean, cov):
    """bytetrack_kf.py:155-192 over N stacked states."""
    h = mean[:, 3]
    one = np.ones_like(h)
    std = np.stack([W_POS * h, W_POS * h, 1e-2 * one, W_POS * h,
                    W_VEL * h, W_VEL * h, 1e-5 * one, W_VEL * h], axis=1)
    q = np.zeros((len(mean), 8, 8))
    idx = np.arange(8)
    q[:, idx, idx] = np.square(std)
    new_mean = mean @ F.T
    new_cov = np.einsum("ij,njk,lk->nil", F, cov, F) + q
    return new_mean, new_cov


def update(mean, cov, z):
    """bytetrack_kf.py:194-226 (project :126-153; Cholesky solve for the gain)."""
    h = mean[3]
    r = np.diag(np.square([W_POS * h, W_POS * h, 1e-1, W_POS * h]))
    s = H @ cov @ H.T + r
    ph = cov @ H.T                        # 8x4
    chol = np.linalg.cholesky(s)
    gain = np.linalg.solve(chol.T, np.linalg.solve(chol, ph.T)).T
    innov = np.asarray(z, np.float64) - H @ mean
    new_mean = mean + innov @ gain.T
    new_cov = cov - gain @ s @ gain.T
    return new_mean, new_cov
