"""CPU oracle (numpy, fp64) for the 2ACE ADMM channel-recovery hot path.

TEST INFRASTRUCTURE ONLY.  Nothing on the product path imports this module:
only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may use it, and only as the checker.

Parity status: **parity unpinned against MATLAB.**  The reference's hot path is
MATLAB (``main/src/my_recovery_algorithms/ADMM_v2/*.m``); neither MATLAB nor
Octave exists in this image, and the reference ships no ADMM outputs to pin
against.  This file is a line-by-line restatement of the
``.m`` sources; every function cites the file:line it follows.  It is pinned
only by (a) its cross-check against the independent C restatement in
``oracle/ace_oracle.c`` and (b) property tests (exact recovery on noiseless
low-rank channels, phase equivariance) in ``tests/test_oracle.py``.

MATLAB built-ins are mapped to LAPACK through numpy:
``inv`` -> ``numpy.linalg.inv`` (zgesv/LU, as MATLAB's zgetrf/zgetri),
``eig`` of a Hermitian product -> ``numpy.linalg.eigh`` (ascending eigenvalues,
as MATLAB's zheev path), ``svd`` -> ``numpy.linalg.svd``.
Sort semantics: MATLAB ``sort(...,'descend')`` is stable; ``min`` returns the
first minimiser; ``sum`` over <=32 elements is taken sequentially.

Paths below are relative to the reference root.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np

REF_V4M = "main/src/my_recovery_algorithms/ADMM_v2/inferLowRankV4_multi.m"
REF_NUC = "main/src/my_recovery_algorithms/ADMM_v2/inferLowRank_Nuclear.m"

VARIANT_A2ONLY = 0
VARIANT_NUCLEAR = 1


def _seqsum(x):
    """Sequential left-to-right sum (MATLAB ``sum`` over a short vector)."""
    x = np.asarray(x, dtype=np.float64).ravel()
    return float(np.cumsum(x)[-1]) if x.size else 0.0


def _fro(x):
    return float(np.linalg.norm(x))


# ----------------------------------------------------------------------------
# Z-proximal steps
# ----------------------------------------------------------------------------
def rank_profile(tx, rx, m, n, use_rank_one):
    """Rank/variance profile of ArgMinZ (inferLowRankV4_multi.m:437-464)."""
    sz = min(rx, tx)
    r0 = math.ceil(math.sqrt(sz) * 0.5)
    r1 = math.ceil(math.sqrt(sz) * 0.7)
    r2 = math.ceil(math.sqrt(sz))
    r3 = min(sz, math.ceil(math.sqrt(sz) * 2.0))
    f0, f1, f2, f3 = 0.8, 0.9, 0.95, 0.995
    if use_rank_one:
        return [1], [0.95]
    if m >= n * 3:
        return [r3], [f3]
    if r1 <= 2:
        return [r2], [f2]
    if r0 <= 2:
        return [r1, r2, r3], [f1, f2, f3]
    return [r0, r1, r2, r3], [f0, f1, f2, f3]


def argmin_z_lowrank(X, N, mu, tx, rx, m, n, use_rank_one):
    """A2only Z-step: spectral tail rescaling of E=reshape(X+N/mu,tx,[])
    (inferLowRankV4_multi.m:423-485)."""
    Z = X + N / mu                                            # :424
    r = Z.shape[1]
    E = Z.reshape((tx, rx * r), order="F")                     # :426
    H = E @ E.conj().T
    H = 0.5 * (H + H.conj().T)                                 # E*E' is exactly Hermitian in MATLAB
    w, U = np.linalg.eigh(H)                                   # :428 eig, ascending
    s2 = np.maximum(0.0, np.real(w))                           # :429
    idx = np.argsort(-s2, kind="stable")                       # :430 stable descend
    s2 = s2[idx].copy()
    r_list, f_list = rank_profile(tx, rx, m, n, use_rank_one)  # :437-464
    s2_scale = np.ones_like(s2)                                # :469
    for rr, f in zip(r_list, f_list):                          # :470-480
        vr = _seqsum(s2[:rr])
        v = _seqsum(s2)
        if vr < v * f:
            scale = min(1.0, vr / (v - vr) * (1.0 / f - 1.0))
            s2[rr:] = s2[rr:] * scale
            s2_scale[idx[rr:]] = s2_scale[idx[rr:]] * scale
    if np.any(s2_scale < 1):                                   # :482-484
        Zr = ((U * np.sqrt(s2_scale)[None, :]) @ U.conj().T) @ E
        Z = Zr.reshape((tx * rx, r), order="F")
    return Z


def argmin_z_nuclear(X, N, mu):
    """A2nuclear Z-step: singular-value soft threshold of the n-by-r iterate
    (inferLowRank_Nuclear.m:411-419, Shrink :421-439)."""
    Z = X + N / mu
    if Z.shape[1] == 1:
        nz = _fro(Z)
        s = max(0.0, nz - 1.0 / mu)
        return Z * (s / nz) if nz > 0 else Z * 0.0
    U, S, Vh = np.linalg.svd(Z, full_matrices=False)
    S = np.sign(S) * np.maximum(0.0, np.abs(S) - 1.0 / mu)
    return (U * S[None, :]) @ Vh


# ----------------------------------------------------------------------------
# Y steps
# ----------------------------------------------------------------------------
def argmin_y(AX, B, M, mu, scale_by_row):
    """Magnitude projection (inferLowRankV4_multi.m:511-533)."""
    Y = AX + M / mu
    r = Y.shape[1]
    if scale_by_row:
        D = np.sqrt(np.sum(np.abs(Y) ** 2, axis=1))
        zero = D == 0
        if np.any(zero):
            Y[zero, :] = 1.0 / math.sqrt(r)
            D[zero] = 1.0
        BD = B / D
        return Y * ((BD + mu) / (1 + mu))[:, None]
    D = np.abs(Y)
    zero = D == 0
    if np.any(zero):
        Y[zero] = 1.0
        D[zero] = 1.0
    BD = B[:, None] / D
    return Y * ((BD + mu) / (1 + mu))


def normalize_rows(Y, B, scale_by_row):
    """inferLowRankV4_multi.m:538-559."""
    Y = Y.copy()
    r = Y.shape[1]
    if scale_by_row:
        D = np.sqrt(np.sum(np.abs(Y) ** 2, axis=1))
        zero = D == 0
        if np.any(zero):
            Y[zero, :] = 1.0 / math.sqrt(r)
            D[zero] = 1.0
        return Y * (B / D)[:, None]
    D = np.abs(Y)
    zero = D == 0
    if np.any(zero):
        Y[zero] = 1.0
        D[zero] = 1.0
    return Y * (B[:, None] / D)


# ----------------------------------------------------------------------------
# InferADMM
# ----------------------------------------------------------------------------
@dataclass
class AdmmResult:
    X: np.ndarray
    Y: np.ndarray
    converged: bool
    iters: int
    mu: float
    opt_obj: float
    trace: list = field(default_factory=list)


def make_U(A):
    """U = inv(A'*A + eye(n)) (inferLowRankV4_multi.m:242, :288)."""
    n = A.shape[1]
    return np.linalg.inv(A.conj().T @ A + np.eye(n))


def infer_admm(A, B, X0, scale_by_row, use_rank_one, tx, rx, *, mu0=1e-3, rho=1.03,
               tol_rel=1e-4, tol_abs=1e-8, maxiter=500, U=None,
               variant=VARIANT_A2ONLY, fixed_iters=False, want_trace=False):
    """InferADMM (inferLowRankV4_multi.m:281-386; nuclear variant
    inferLowRank_Nuclear.m:269-374 differs only in ArgMinZ).  lambda = 0
    (the only value any driver reaches: defaults :6).

    ``fixed_iters``: throughput mode of the build -- the
    convergence test is evaluated but never exits; ``maxiter`` iterations run.
    """
    B = np.asarray(B, dtype=np.float64).ravel()
    m, n = A.shape
    X = np.array(X0, dtype=np.complex128).reshape(n, -1)
    r = X.shape[1]
    if U is None:                                              # :286-294
        U = make_U(A)

    def zstep(Xv, Nv, muv):
        if variant == VARIANT_NUCLEAR:
            return argmin_z_nuclear(Xv, Nv, muv)
        return argmin_z_lowrank(Xv, Nv, muv, tx, rx, m, n, use_rank_one)

    M = np.zeros((m, r), np.complex128)                         # :296
    N = np.zeros((n, r), np.complex128)                         # :297
    AX = A @ X                                                  # :299
    nB = _fro(B)
    if scale_by_row:                                            # :300-306
        X = X * (nB / _fro(AX))
    else:
        for j in range(r):
            X[:, j] = X[:, j] * (nB / _fro(AX[:, j]))
    AX = A @ X                                                  # :307
    Y = normalize_rows(AX, B, scale_by_row)                     # :308
    Z = zstep(X, N, 1.0)                                        # :309
    AtY = A.conj().T @ Y                                        # :310

    mu = mu0
    opt_obj = math.inf
    opt_X = None
    opt_Y = None
    converged = False
    last_res = math.inf
    trace = []
    it = 0
    for it in range(1, maxiter + 1):                            # :318
        Y0, Z0, AtY0 = Y, Z, AtY
        X = U @ (A.conj().T @ (Y - M / mu) + (Z - N / mu))      # :325 ArgMinX :404
        AX = A @ X                                              # :326
        Y = argmin_y(AX, B, M, mu, scale_by_row)                # :329
        AtY = A.conj().T @ Y                                    # :330
        Z = zstep(X, N, mu)                                     # :333
        J_M = AX - Y                                            # :336
        M = M + mu * J_M
        J_N = X - Z                                             # :340
        N = N + mu * J_N
        if scale_by_row:                                        # :344-351
            obj = _fro(np.sqrt(np.sum(np.abs(AX) ** 2, axis=1)) - B)
            if obj < opt_obj:
                opt_obj, opt_X, opt_Y = obj, X.copy(), Y.copy()
        else:                                                   # :352-361
            objs = np.sqrt(np.sum((np.abs(AX) - B[:, None]) ** 2, axis=0))
            # MATLAB's min omits NaN and returns the first minimiser (index 1 if all NaN)
            j = 0 if np.all(np.isnan(objs)) else int(np.nanargmin(objs))
            obj = float(objs[j])
            if obj < opt_obj:
                opt_obj, opt_X, opt_Y = obj, X[:, [j]].copy(), Y[:, [j]].copy()
        nAX, nY, nX, nZ = _fro(AX), _fro(Y), _fro(X), _fro(Z)   # :364-370
        dZ2 = _fro(Z - Z0) ** 2
        res_prim = math.sqrt(_fro(J_M) ** 2 + _fro(J_N) ** 2)
        res_dual = mu * math.sqrt(_fro(AtY - AtY0) ** 2 + dZ2)
        res_comb = math.sqrt(res_prim ** 2 + _fro(Y - Y0) ** 2 + dZ2)
        t_prim = tol_abs * math.sqrt((m + n) * r) + tol_rel * math.sqrt(max(nAX, nY) ** 2 + max(nX, nZ) ** 2)
        t_dual = tol_abs * math.sqrt(n * r * 2) + tol_rel * math.sqrt(_fro(AtY) ** 2 + nZ ** 2)
        t_comb = tol_abs * math.sqrt((m + n) * r * 2) + tol_rel * math.sqrt(
            max(nAX, nY) ** 2 + max(nX, nZ) ** 2 + nY ** 2 + nZ ** 2)
        if want_trace:
            trace.append(dict(it=it, mu=mu, obj=obj, res_prim=res_prim, res_dual=res_dual,
                              res_comb=res_comb, t_prim=t_prim, t_dual=t_dual, t_comb=t_comb))
        if (res_prim < t_prim and res_dual < t_dual) or (res_comb < t_comb):   # :372
            converged = True
            if not fixed_iters:
                break
        if res_comb > last_res * 0.9:                           # :379-381
            mu = mu * rho
        last_res = res_comb
    if opt_X is None:          # reference would raise "undefined opt_X" (all objs NaN)
        opt_X, opt_Y = X, Y
    return AdmmResult(opt_X, opt_Y, converged, it, mu, opt_obj, trace)


# ----------------------------------------------------------------------------
# Pipeline pieces
# ----------------------------------------------------------------------------
def spectral_initialize(A, B, r):
    """inferLowRankV4_multi.m:561-574."""
    As = A.copy()
    for i in range(A.shape[0]):
        an = np.linalg.norm(A[i, :])
        if an != 0:
            As[i, :] = A[i, :] * (B[i] / an)
    AtA = As.conj().T @ As
    AtA = 0.5 * (AtA + AtA.conj().T)
    w, V = np.linalg.eigh(AtA)
    s2 = np.maximum(0.0, np.real(w))
    idx = np.argsort(-s2, kind="stable")
    s2 = s2[idx]
    return V[:, idx[:r]] * np.sqrt(s2[:r])[None, :]


def infer_low_rank_impl(A, B, Xs, tx, rx, r, use_rank_one, *, variant=VARIANT_A2ONLY, **kw):
    """inferLowRankV4_multi.m:111-271 (lambda = 0 branch)."""
    U = make_U(A)                                               # :242
    X = Xs                                                      # :252
    res1 = infer_admm(A, B, X, True, use_rank_one, tx, rx, U=U, variant=variant, **kw)   # :258
    X = res1.X
    G = X.conj().T @ X
    G = 0.5 * (G + G.conj().T)
    _, Vx = np.linalg.eigh(G)                                   # :263 (ascending, not re-sorted)
    X = X @ Vx                                                  # :264
    res2 = infer_admm(A, B, X, False, use_rank_one, tx, rx, U=U, variant=variant, **kw)  # :270
    return res2, (res1.iters, res2.iters)


@dataclass
class PipelineResult:
    X: np.ndarray
    Y: np.ndarray
    quality: float
    stage_iters: list
    restart_quality: list
    rolled_back: bool
    use_rank_one: bool = False     # the refinement's profile: the last restart's retry ran (:73-77, :92)
    X_max: np.ndarray = None       # the refinement's input (:90-92), rescaled like X (:106)


def infer_low_rank_pipeline(A, B, tx, rx, train_idx_list, *, variant=VARIANT_A2ONLY, r=20,
                            cc_frac=0.95, tol_abs=1e-8, **kw):
    """inferLowRankV4_multi (restarts = len(train_idx_list) = 3, :5-109),
    inferLowRankV4 (1 restart) and inferLowRank_Nuclear (1 restart,
    refinement from the last X, inferLowRank_Nuclear.m:76-89).

    ``train_idx_list``: one 0-based row-index array of length floor(m*cc_frac)
    per restart, in sampled order (stands in for MATLAB ``randsample``, :48).
    """
    A = np.asarray(A, np.complex128)
    B = np.asarray(B, np.float64).ravel()
    m, n = A.shape
    r = min(r, m, n)                                             # :19
    A_norm = _fro(A) / math.sqrt(m)                              # :27-30
    if A_norm < tol_abs:
        A_norm = 1.0
    B_norm = _fro(B)                                             # :32-35
    if B_norm < tol_abs:
        B_norm = 1.0
    A = A / A_norm
    B = B / B_norm
    max_quality = -1.0
    X_max = Y_max = None
    stage_iters = []
    qualities = []
    quality = None
    use_rank_one = False
    X = Y = None
    for tr in train_idx_list:                                    # :42
        tr = np.asarray(tr, dtype=np.int64)
        assert tr.size == math.floor(m * cc_frac)
        te = np.setdiff1d(np.arange(m), tr)                      # :49 (sorted)
        A_tr, B_tr, A_te, B_te = A[tr], B[tr], A[te], B[te]
        Xs = spectral_initialize(A_tr, B_tr, r)                  # :58
        use_rank_one = False                                     # :66
        res, its = infer_low_rank_impl(A_tr, B_tr, Xs, tx, rx, r, use_rank_one,
                                       variant=variant, tol_abs=tol_abs, **kw)
        X, Y = res.X, res.Y
        stage_iters.extend(its)
        quality = 1 - _fro(np.abs(A_te @ X).ravel() - B_te) / _fro(B_te)   # :68
        if quality < 0.6:                                        # :73-77
            use_rank_one = True
            res, its = infer_low_rank_impl(A_tr, B_tr, Xs, tx, rx, r, use_rank_one,
                                           variant=variant, tol_abs=tol_abs, **kw)
            X, Y = res.X, res.Y
            stage_iters.extend(its)
            quality = 1 - _fro(np.abs(A_te @ X).ravel() - B_te) / _fro(B_te)
        else:
            stage_iters.extend((0, 0))
        qualities.append(quality)
        if variant == VARIANT_A2ONLY and max_quality < quality:  # :79-83
            X_max, Y_max, max_quality = X, Y, quality
    if variant == VARIANT_NUCLEAR:                               # inferLowRank_Nuclear.m:78-88
        X_max, Y_max = X, Y
    rolled_back = False
    ref = infer_admm(A, B, X_max, True, use_rank_one, tx, rx, variant=variant, tol_abs=tol_abs, **kw)  # :92/:100
    Xf, Yf = ref.X, ref.Y
    stage_iters.append(ref.iters)
    if quality > 0.6:                                            # :89 (last restart's quality)
        sim = float(np.abs(X_max.conj().T @ Xf).ravel()[0]) / _fro(X_max) / _fro(Xf)   # :93
        if sim < 0.6:                                            # :94-98
            Xf, Yf = X_max, Y_max
            rolled_back = True
    Xf = Xf * (B_norm / A_norm)                                  # :106-107
    Yf = Yf * (B_norm / A_norm)
    return PipelineResult(Xf.ravel(), Yf.ravel(), float(quality), stage_iters, qualities, rolled_back,
                          bool(use_rank_one), (X_max * (B_norm / A_norm)).ravel())


# ----------------------------------------------------------------------------
# Metric
# ----------------------------------------------------------------------------
def phase_aligned_rel_err(x_hat, x):
    """Numerical_Simulation/src/evaluate_plot_results/Evaluation_H.m:81-89:
    ||x - (x_hat' x / x_hat' x_hat) x_hat|| / ||x||."""
    x_hat = np.asarray(x_hat).ravel()
    x = np.asarray(x).ravel()
    den = np.vdot(x_hat, x_hat)
    if den == 0:
        return 1.0 if np.linalg.norm(x) > 0 else 0.0
    a = np.vdot(x_hat, x) / den
    return float(np.linalg.norm(x - a * x_hat) / max(np.linalg.norm(x), 1e-300))


def unit_phase_aligned_rel_err(x_hat, x):
    """Relative error after aligning only the global PHASE (|a| forced to 1)."""
    x_hat = np.asarray(x_hat).ravel()
    x = np.asarray(x).ravel()
    c = np.vdot(x_hat, x)
    ph = c / abs(c) if abs(c) > 0 else 1.0
    return float(np.linalg.norm(x - ph * x_hat) / max(np.linalg.norm(x), 1e-300))
