"""CPU oracle (numpy, fp64) for the PhaseLift path: MyPhaseLift + TFOCS (AT, TraceLS).

TEST INFRASTRUCTURE ONLY -- imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, never by the product path.

Restates (paths relative to the reference root):
  main/src/my_recovery_algorithms/MyPhaseLift.m:69-107
  main/3rd_software_component/sparsepr/src/initializeLinopPR.m:50-66 (A(X) = diag(Phi X Phi'),
      A*(y) = Phi' diag(y) Phi)
  .../sparsepr/third/TFOCS/solver_TraceLS.m:1-42  (smooth_quad at A(X) - b, prox_trace(lambda),
      restart default 100)
  .../TFOCS/tfocs_AT.m:20-88                        (Auslender-Teboulle iteration)
  .../TFOCS/private/tfocs_initialize.m             (defaults: L0 1, alpha 0.9, beta 0.5,
      Lexact Inf, cntr_reset 50, stopCrit 1; x0 = 0 -> A_x = 0)
  .../TFOCS/private/tfocs_backtrack.m              (simple / non-simple Lipschitz backtracking)
  .../TFOCS/private/tfocs_iterate.m                (stopping tests, restart)
  .../TFOCS/private/tfocs_cleanup.m                (output x: no stopFcn, restart > 0)
  .../TFOCS/prox_trace.m:62-173                    (eig((X+X')/2), shrink eigenvalues by q*t)
Pinned by TFOCS's own known-answer tests (examples/smallscale/reference_solutions/
traceLS_problem{1,2}_noisy.mat, harness test_TraceLS.m: relative error to the CVX
solution below 1e-5), copied as fixtures into tests/golden/.
MATLAB eig of a Hermitian matrix -> numpy.linalg.eigh (ascending).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np

EPS = np.finfo(np.float64).eps


def _dot(a, b):
    """tfocs_dot: real(a(:)' * b(:))."""
    return float(np.real(np.vdot(a, b)))


def _nsq(a):
    """tfocs_normsq."""
    return _dot(a, a)


def prox_trace(q, X, t):
    """prox_trace.m:62-173 (LARGESCALE off, isReal false).  Returns (value, X)."""
    tau = q * t
    H = 0.5 * (X + X.conj().T)
    w, V = np.linalg.eigh(H)
    s = w - tau
    keep = s > 0
    s = s[keep]
    if s.size == 0:
        Xn = np.zeros_like(X)
    else:
        Vk = V[:, keep]
        Xn = (Vk * s[None, :]) @ Vk.conj().T
        Xn = 0.5 * (Xn + Xn.conj().T)
    return q * float(np.sum(s)), Xn


def prox_trace_value(q, X):
    """prox_trace value mode (nargin < 5): q * trace(X + X')/2."""
    return q * float(np.real(np.trace(X + X.conj().T))) / 2


@dataclass
class TfocsResult:
    x: np.ndarray
    niter: int
    status: str
    L: float
    restarts: int


def tfocs_at_tracels(Aop, Aadj, b, lam, x0, *, maxIts=math.inf, tol=1e-8, restart=100, L0=1.0, alpha=0.9,
                     beta=0.5, Lexact=math.inf, cntr_reset=50, want_hist=False):
    """solver_TraceLS(A, b, lambda, x0, opts) with tfocs_AT: min 0.5||A(X) - b||^2 + lam tr X, X >= 0.

    Aop(X) -> vector, Aadj(y) -> matrix.  x0 = zeros (the only start any caller uses)."""
    b = np.asarray(b)
    smooth = lambda Ax: (0.5 * _nsq(Ax - b), Ax - b)          # smooth_quad at A(x) - b
    # ---- tfocs_initialize
    L = L0
    theta = math.inf
    x = np.array(x0, dtype=np.result_type(x0, np.complex128) if np.iscomplexobj(x0) else np.float64)
    zero_x0 = not np.any(x)
    A_x = np.zeros_like(b, dtype=np.result_type(b, x)) if zero_x0 else Aop(x)
    C_x = prox_trace_value(lam, x)
    f_x, g_Ax = smooth(A_x)
    restart_iter = 0
    backtrack_simple = True
    backtrack_tol = 1e-10
    backtrack_steps = 0
    n_iter = 0
    y, z = x, x
    A_y, A_z = A_x, A_x
    f_y = f_x
    g_y = None
    g_Ay = g_Ax
    cntr_Ay = cntr_Ax = 0
    status = ""
    restarts = 0
    hist = []
    xy_sq = 0.0
    while True:
        x_old, A_x_old, z_old, A_z_old = x, A_x, z, A_z
        L_old = L
        L = L * alpha
        theta_old = theta
        while True:                                                     # tfocs_AT.m inner loop
            theta = 2.0 / (1.0 + math.sqrt(1.0 + 4.0 * (L / L_old) / theta_old ** 2))
            if theta < 1:
                y = (1 - theta) * x_old + theta * z_old
                if cntr_Ay >= cntr_reset:
                    A_y = Aop(y)
                    cntr_Ay = 0
                else:
                    cntr_Ay += 1
                    A_y = (1 - theta) * A_x_old + theta * A_z_old
                f_y = math.inf
                g_Ay = None
                g_y = None
            if g_y is None:
                if g_Ay is None:
                    f_y, g_Ay = smooth(A_y)
                g_y = Aadj(g_Ay)
            step = 1.0 / (theta * L)
            C_z, z = prox_trace(lam, z_old - step * g_y, step)
            A_z = Aop(z)
            if theta == 1:
                x, A_x, C_x = z, A_z, C_z
            else:
                x = (1 - theta) * x_old + theta * z
                if cntr_Ax >= cntr_reset:
                    cntr_Ax = 0
                    A_x = Aop(x)
                else:
                    cntr_Ax += 1
                    A_x = (1 - theta) * A_x_old + theta * A_z
                C_x = math.inf
            f_x = math.inf
            g_Ax = None
            # ---- tfocs_backtrack
            if beta >= 1:
                break
            xy = x - y
            xy_sq = _nsq(xy)
            if xy_sq == 0:
                break
            if xy_sq / _nsq(x) < EPS:
                cntr_Ax = math.inf
            if backtrack_simple:
                if math.isinf(f_x):
                    f_x = smooth(A_x)[0]
                q_x = f_y + _dot(xy, g_y) + 0.5 * L * xy_sq
                localL = L + 2 * max(f_x - q_x, 0.0) / xy_sq
                backtrack_simple = abs(f_y - f_x) >= backtrack_tol * max(abs(f_x), abs(f_y))
            else:
                if g_Ax is None:
                    f_x, g_Ax = smooth(A_x)
                localL = 2 * _dot(A_x - A_y, g_Ax - g_Ay) / xy_sq
            backtrack_steps += 1
            if localL <= L or L >= Lexact:
                break
            if not math.isinf(localL):
                L = min(Lexact, localL)
            else:
                localL = L
            L = min(Lexact, max(localL, L / beta))
        # ---- tfocs_iterate
        n_iter += 1
        norm_x = math.sqrt(_nsq(x))
        norm_dx = math.sqrt(_nsq(x - x_old))
        if want_hist:
            hist.append((n_iter, L, theta, norm_dx))
        if math.isnan(f_y):
            status = "NaN found -- aborting"
        elif norm_dx == 0:
            if n_iter > 1:
                status = "Step size tolerance reached (||dx||=0)"
        elif norm_dx < tol * max(norm_x, 1):
            status = "Step size tolerance reached"
        elif n_iter == maxIts:
            status = "Iteration limit reached"
        elif backtrack_steps > 0 and xy_sq == 0:
            status = "Unexpectedly small stepsize"
        if status:
            break
        backtrack_steps = 0
        if n_iter - restart_iter == abs(round(restart)):
            restart_iter = n_iter
            restarts += 1
            backtrack_simple = True
            theta = math.inf
            y, A_y, f_y, g_Ay, g_y = x, A_x, f_x, g_Ax, None
            z, A_z = x, A_x
    res = TfocsResult(x, n_iter, status, L, restarts)
    if want_hist:
        res.hist = hist
    return res


def phaselift_ops(Phi):
    """initializeLinopPR.m: A(X) = diag(Phi X Phi'), A*(y) = Phi' diag(y) Phi."""
    PhiH = Phi.conj().T

    def Aop(X):
        return np.einsum("ij,ji->i", Phi @ X, PhiH)

    def Aadj(yv):
        return PhiH @ (yv[:, None] * Phi)

    return Aop, Aadj


def my_phaselift(measurements, Phi, *, maxIts=4000, tol=1e-10, restart=200, lam=5e-2, want_hist=False):
    """MyPhaseLift.m:69-107: solver_TraceLS(PR operator, y, 5e-2, zeros(n), opts) then the
    leading eigenvector scaled by sqrt of its eigenvalue."""
    Phi = np.asarray(Phi, dtype=np.complex128)
    m, n = Phi.shape
    Aop, Aadj = phaselift_ops(Phi)
    res = tfocs_at_tracels(Aop, Aadj, np.asarray(measurements, dtype=np.float64).reshape(m), lam,
                           np.zeros((n, n), np.complex128), maxIts=maxIts, tol=tol, restart=restart,
                           want_hist=want_hist)
    w, V = np.linalg.eigh(res.x)                      # [recoveredSig, eVal] = eig(recoveredMat)
    sig = math.sqrt(w[-1]) * V[:, -1] if w[-1] >= 0 else np.sqrt(complex(w[-1])) * V[:, -1]
    return sig, res


def my_phaselift_reduced(measurements, Phi, *, maxIts=4000, tol=1e-10, restart=200, lam=5e-2):
    """my_phaselift in the coordinates of range(Phi^H) (m <= n, Phi of full row rank): with the zero
    start every TFOCS iterate is Q Xr Q^H, Phi^H = Q R (R = chol(Phi Phi^H)), A(Q Xr Q^H) =
    diag(R^H Xr R), A*(g) = Q (R diag(g) R^H) Q^H, and norms / inner products are preserved, so the
    same tfocs_at_tracels run on m x m matrices is the dense iteration up to rounding
    (tests/test_oracle.py::test_phaselift_reduction_is_exact).  Returns (sig, result) like
    my_phaselift, sig mapped back to n coordinates (Q u = Phi^H R^-1 u)."""
    Phi = np.asarray(Phi, dtype=np.complex128)
    m, n = Phi.shape
    if m > n:
        return my_phaselift(measurements, Phi, maxIts=maxIts, tol=tol, restart=restart, lam=lam)
    R = np.linalg.cholesky(Phi @ Phi.conj().T).conj().T          # upper, Phi Phi^H = R^H R
    Rc = R.conj()
    res = tfocs_at_tracels(lambda X: np.sum(Rc * (X @ R), axis=0), lambda g: (R * g[None, :]) @ R.conj().T,
                           np.asarray(measurements, dtype=np.float64).reshape(m), lam,
                           np.zeros((m, m), np.complex128), maxIts=maxIts, tol=tol, restart=restart)
    w, V = np.linalg.eigh(res.x)
    u = np.linalg.solve(R, V[:, -1])
    sig = Phi.conj().T @ u
    sig = (math.sqrt(w[-1]) if w[-1] >= 0 else np.sqrt(complex(w[-1]))) * sig
    return sig, res
