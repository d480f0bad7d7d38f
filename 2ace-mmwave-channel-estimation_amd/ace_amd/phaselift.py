"""Host-side mirror of the reference PhaseLift solver, backed by the HIP library.

Reference: recoveredSig = MyPhaseLift(measurements, measurementMat)
(main/src/my_recovery_algorithms/MyPhaseLift.m:69-107: TFOCS solver_TraceLS with
lambda = 5e-2, maxIts 4000, tol 1e-10, restart 200, x0 = zeros(n); then the leading
eigenvector scaled by the square root of its eigenvalue).  Recover_Channel.m:34 calls it
with measurements = (rss/2e5).^2*1e10 and rescales the result by 2e5/sqrt(1e10).

Entry points (no CPU fallback):
  * ``MyPhaseLift(measurements, measurementMat)`` -- MATLAB argument order, numpy in/out (n, 1).
  * ``phaselift_host(Phi, b)`` -- a batch of measurement vectors sharing Phi, host arrays.
  * ``phaselift_batch(Phi, b)`` -- device tensors already in HBM (the throughput path).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from ._lib import LIB, check


class PhaseLiftCfg(C.Structure):
    """Mirror of ``ace_phaselift_cfg`` (include/ace.h)."""
    _fields_ = [("maxIts", C.c_int), ("restart", C.c_int), ("cntr_reset", C.c_int), ("reserved", C.c_int),
                ("tol", C.c_double), ("lambda_", C.c_double), ("L0", C.c_double), ("alpha", C.c_double),
                ("beta", C.c_double)]


_cfgp = C.POINTER(PhaseLiftCfg)
_dp = C.POINTER(C.c_double)
LIB.ace_phaselift_cfg_default.argtypes = [_cfgp]
LIB.ace_phaselift_cfg_default.restype = None
LIB.ace_phaselift_workspace_size.argtypes = [_cfgp, C.c_int, C.c_int, C.c_int]
LIB.ace_phaselift_workspace_size.restype = C.c_size_t
LIB.ace_phaselift_solve_batch.argtypes = [_cfgp, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p,
                                          C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p]
LIB.ace_phaselift_solve_batch.restype = C.c_int
LIB.ace_phaselift_solve_host.argtypes = [_cfgp, C.c_int, C.c_int, C.c_int, _dp, _dp, _dp,
                                         C.POINTER(C.c_int32), C.POINTER(C.c_uint32)]
LIB.ace_phaselift_solve_host.restype = C.c_int
LIB.ace_phaselift_solve_host_x.argtypes = [_cfgp, C.c_int, C.c_int, C.c_int, _dp, _dp, _dp,
                                           C.POINTER(C.c_int32), C.POINTER(C.c_uint32), _dp]
LIB.ace_phaselift_solve_host_x.restype = C.c_int


LIB.ace_prox_eig_host.argtypes = [C.c_int, C.c_int, C.c_int, _dp, _dp, _dp, _dp, C.POINTER(C.c_int32)]
LIB.ace_prox_eig_host.restype = C.c_int


def prox_eig_host(A, tau, path=2):
    """The prox's eigensolver on host arrays (TFOCS/prox_trace.m:88-92): every eigenpair of the Hermitian A[b]
    above tau[b], descending.  path 0 / 1 / 2: unblocked one-stage / blocked one-stage / two-stage reduction; + 4:
    the smaller side of tau (k[b] < 0: V holds the -k[b] eigenpairs at or below tau, ascending).
    Returns (lam [batch][d], V [batch][d][d] with eigenvector q as row q, k [batch])."""
    A = np.ascontiguousarray(np.asarray(A, dtype=np.complex128).reshape((-1,) + np.shape(A)[-2:]))
    batch, d = A.shape[0], A.shape[1]
    tau = np.ascontiguousarray(np.broadcast_to(np.asarray(tau, dtype=np.float64), (batch,)))
    lam = np.zeros((batch, d))
    V = np.zeros((batch, d, d), np.complex128)
    k = np.zeros(batch, np.int32)
    check(LIB.ace_prox_eig_host(batch, d, int(path), A.view(np.float64).ctypes.data_as(_dp), tau.ctypes.data_as(_dp),
                                lam.ctypes.data_as(_dp), V.view(np.float64).ctypes.data_as(_dp),
                                k.ctypes.data_as(C.POINTER(C.c_int32))))
    return lam, V, k


def phaselift_cfg(maxIts=4000, tol=1e-10, restart=200, lam=5e-2, **kw) -> PhaseLiftCfg:
    cfg = PhaseLiftCfg()
    LIB.ace_phaselift_cfg_default(C.byref(cfg))
    cfg.maxIts, cfg.tol, cfg.restart, cfg.lambda_ = int(maxIts), float(tol), int(restart), float(lam)
    for k, v in kw.items():
        if not hasattr(cfg, k):
            raise TypeError(f"unknown ace_phaselift_cfg field {k!r}")
        setattr(cfg, k, v)
    return cfg


@dataclass
class PhaseLiftResult:
    sig: object      # [batch][n] complex128
    iters: object    # [batch] int32 (TFOCS iterations)
    status: object   # [batch] uint32 (ACE_ST_CONVERGED: step tolerance reached before maxIts)
    X: object = None  # [batch][d][d] complex128: the final TFOCS iterate, reduced coordinates (with_x=True)


def phaselift_host(Phi, b, with_x=False, **kw) -> PhaseLiftResult:
    """Batch of MyPhaseLift solves on host arrays: Phi [m][n] (shared), b [batch][m].  with_x: also return
    solver_TraceLS's iterate (MyPhaseLift.m:98 recoveredMat) in the coordinates of range(Phi^H)
    (ace_phaselift_solve_host_x; recoveredMat = Q X Q^H, Phi^H = Q R, R = chol(Phi Phi^H))."""
    Phi = np.ascontiguousarray(Phi, dtype=np.complex128)
    b = np.ascontiguousarray(np.atleast_2d(np.asarray(b, dtype=np.float64)))
    m, n = Phi.shape
    if b.shape[1] != m:
        raise ValueError(f"shape mismatch: Phi{Phi.shape} b{b.shape}")
    batch = b.shape[0]
    cfg = phaselift_cfg(**kw)
    sig = np.empty((batch, n), np.complex128)
    it = np.empty(batch, np.int32)
    stt = np.empty(batch, np.uint32)
    args = (C.byref(cfg), batch, m, n, Phi.view(np.float64).ctypes.data_as(_dp), b.ctypes.data_as(_dp),
            sig.view(np.float64).ctypes.data_as(_dp), it.ctypes.data_as(C.POINTER(C.c_int32)),
            stt.ctypes.data_as(C.POINTER(C.c_uint32)))
    if not with_x:
        check(LIB.ace_phaselift_solve_host(*args))
        return PhaseLiftResult(sig, it, stt)
    d = min(m, n)
    X = np.empty((batch, d, d), np.complex128)
    check(LIB.ace_phaselift_solve_host_x(*args, X.view(np.float64).ctypes.data_as(_dp)))
    return PhaseLiftResult(sig, it, stt, X)


def MyPhaseLift(measurements, measurementMat, **kw):
    """recoveredSig = MyPhaseLift(measurements, measurementMat) on the GPU, shape (n, 1)."""
    Phi = np.asarray(measurementMat, dtype=np.complex128)
    res = phaselift_host(Phi, np.asarray(measurements, dtype=np.float64).reshape(1, -1), **kw)
    return res.sig[0].reshape(-1, 1)


def phaselift_batch(Phi, b, *, workspace=None, stream=None, **kw) -> PhaseLiftResult:
    """Batch on device tensors: Phi [m][n] complex128, b [batch][m] float64."""
    import torch
    from .solver import _DEFAULT_WS
    if not (Phi.is_cuda and b.is_cuda):
        raise ValueError("phaselift_batch needs device tensors")
    Phi, b = Phi.contiguous(), b.contiguous()
    m, n = Phi.shape
    batch = b.shape[0]
    cfg = phaselift_cfg(**kw)
    dev = Phi.device
    out = PhaseLiftResult(torch.empty((batch, n), dtype=torch.complex128, device=dev),
                          torch.empty(batch, dtype=torch.int32, device=dev),
                          torch.empty(batch, dtype=torch.int32, device=dev))
    nbytes = int(LIB.ace_phaselift_workspace_size(C.byref(cfg), batch, m, n)) + 256
    ws = (workspace or _DEFAULT_WS).get(nbytes, dev)
    if stream is None:
        stream = torch.cuda.current_stream(dev)
    check(LIB.ace_phaselift_solve_batch(C.byref(cfg), batch, m, n, Phi.data_ptr(), b.data_ptr(), out.sig.data_ptr(),
                                        out.iters.data_ptr(), out.status.data_ptr(), ws.data_ptr(), ws.numel(),
                                        stream.cuda_stream))
    return out
