"""ctypes loader for the C restatement oracle (oracle/ace_oracle.c).

TEST INFRASTRUCTURE ONLY (see oracle/ace_oracle.c header): used by tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg.  Parity unpinned vs
MATLAB (no MATLAB in the image).
"""
from __future__ import annotations

import ctypes as C
import pathlib
import subprocess

import numpy as np

HERE = pathlib.Path(__file__).resolve().parent
LIB_PATH = HERE / "libace_oracle.so"


def build():
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)


def load():
    if not LIB_PATH.exists():
        build()
    lib = C.CDLL(str(LIB_PATH))
    dp, ip = C.POINTER(C.c_double), C.POINTER(C.c_int)
    lib.aceo_make_U.argtypes = [C.c_int, C.c_int, dp, dp, C.c_int]
    lib.aceo_infer_admm_r1.argtypes = [C.c_int] * 7 + [C.c_double] * 4 + [C.c_int] + [dp] * 6 + [ip, ip, dp]
    lib.aceo_infer_admm_r1_batch.argtypes = ([C.c_int] * 7 + [C.c_double] * 4 + [C.c_int] * 3 + [dp] * 6 +
                                             [ip, ip, dp, C.c_int])
    lib.aceo_herm_eig.argtypes = [C.c_int, dp, dp, dp]
    return lib


_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        _LIB = load()
    return _LIB


def _dp(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def make_U(A, nthreads=8):
    A = np.ascontiguousarray(A, np.complex128)
    m, n = A.shape
    U = np.empty((n, n), np.complex128)
    lib().aceo_make_U(m, n, _dp(A.view(np.float64)), _dp(U.view(np.float64)), nthreads)
    return U


def infer_admm_r1_batch(A, U, B, X0, tx, rx, *, variant=0, use_rank_one=False, fixed_iters=False, mu0=1e-3,
                        rho=1.03, tol_rel=1e-4, tol_abs=1e-8, maxiter=500, nthreads=8):
    """Batch of InferADMM refinement solves (r = 1).  A/U: [1|batch] stacks."""
    A = np.ascontiguousarray(A, np.complex128)
    U = np.ascontiguousarray(U, np.complex128)
    B = np.ascontiguousarray(B, np.float64)
    X0 = np.ascontiguousarray(X0, np.complex128)
    batch, m = B.shape
    n = X0.shape[1]
    a_shared = 1 if A.shape[0] == 1 else 0
    X = np.empty((batch, n), np.complex128)
    Y = np.empty((batch, m), np.complex128)
    it = np.empty(batch, np.int32)
    cv = np.empty(batch, np.int32)
    mu = np.empty(batch, np.float64)
    rc = lib().aceo_infer_admm_r1_batch(
        int(variant), int(use_rank_one), int(fixed_iters), m, n, tx, rx, mu0, rho, tol_rel, tol_abs, maxiter,
        batch, a_shared, _dp(A.view(np.float64)), _dp(U.view(np.float64)), _dp(B), _dp(X0.view(np.float64)),
        _dp(X.view(np.float64)), _dp(Y.view(np.float64)), it.ctypes.data_as(C.POINTER(C.c_int)),
        cv.ctypes.data_as(C.POINTER(C.c_int)), _dp(mu), int(nthreads))
    if rc != 0:
        raise RuntimeError(f"oracle error {rc}")
    return X, Y, it, cv.astype(bool), mu


def herm_eig(H):
    H = np.ascontiguousarray(H, np.complex128)
    n = H.shape[0]
    w = np.empty(n)
    V = np.empty((n, n), np.complex128)
    lib().aceo_herm_eig(n, _dp(H.view(np.float64)), _dp(w), _dp(V.view(np.float64)))
    return w, V
