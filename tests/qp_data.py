"""QP test data: the OCP's Gauss-Newton QP at a given iterate, built with the oracle."""
import numpy as np


def build_qp(oracle, opts, X, U, yref, yref_e, x0, shape_id=None):
    N = opts.N
    nb = X.shape[0]
    A = np.zeros((nb, N, 4, 4))
    B = np.zeros((nb, N, 4, 2))
    b = np.zeros((nb, N, 4))
    H = np.zeros((nb, 6 * N + 4))
    g = np.zeros((nb, 6 * N + 4))
    lo = np.zeros((nb, N, 3))
    hi = np.zeros((nb, N, 3))
    act = np.ones((nb, N, 3), np.uint8)
    W = np.array(opts.W[:])
    We = np.array(opts.We[:])
    tau = opts.tau
    for k in range(N):
        xn, Ak, Bk = oracle.rk4(X[:, k], U[:, k], opts.Ts, shape_id)
        A[:, k], B[:, k], b[:, k] = Ak, Bk, xn - X[:, k + 1]
        H[:, 6 * k:6 * k + 6] = tau * W
        g[:, 6 * k:6 * k + 4] = tau * W[:4] * (X[:, k] - yref[:, k, :4])
        g[:, 6 * k + 4:6 * k + 6] = tau * W[4:] * (U[:, k] - yref[:, k, 4:])
        v = np.stack([X[:, k, 3], U[:, k, 0], U[:, k, 1]], 1)
        lo[:, k] = np.array(opts.lh[:]) - v
        hi[:, k] = np.array(opts.uh[:]) - v
    act[:, 0, 0] = 1 if opts.stage0_s_bound else 0
    H[:, 6 * N:] = We
    g[:, 6 * N:] = We * (X[:, N] - yref_e)
    dx0 = x0 - X[:, 0]
    return A, B, b, H, g, lo, hi, act, dx0
