"""GPU parity of the tridiagonal top-K Z-step (topk_tri, ace_zprox1w.hip) of the full rank profile.

ArgMinZ (inferLowRankV4_multi.m:423-485) rescales the eigenvalue groups of E E^H (1..r_0, r_0+1..r_1, ...,
everything past the largest rank K by one factor), so it needs the top-K eigenpairs and any orthonormal
completion.  In the cold iterations the one-wave Z-step takes them from a Householder tridiagonalisation,
multisection and twisted factorisation (ZArgs::tkeig, ACE_TK_EIG) instead of full Jacobi sweeps; a failed
Ritz-residual check rebuilds H and runs the Jacobi eigensolver.  These tests hold the path to the Jacobi
solves (ACE_TK_EIG=0) and to the C oracle (oracle/ace_oracle.c, LAPACK's eig through numpy), at the unit's
shape and at the small geometries whose profiles differ, and drive the fallback with a clustered top
eigenvalue.
"""
import re

import numpy as np
import pytest

import ace_oracle as O
import ace_oracle_c as OC

pytestmark = pytest.mark.gpu

TOL = 1e-5


def _errs(Xg, Xo):
    return np.array([O.unit_phase_aligned_rel_err(Xg[b], Xo[b]) for b in range(Xg.shape[0])])


def _solve(A, B, X0, tx, monkeypatch, tk, **kw):
    from ace_amd import infer_admm_batch
    monkeypatch.setenv("ACE_TK_EIG", str(tk))
    r = infer_admm_batch(A, B, X0, tx, tx, **kw)
    return r.X.cpu().numpy(), r.iters.cpu().numpy()


@pytest.mark.parametrize("tx,m,batch,fixed", [(32, 256, 1024, True), (32, 256, 512, False), (16, 64, 256, False),
                                              (8, 192, 256, False)])
def test_tridiagonal_zstep_matches_jacobi_and_oracle(gpu, monkeypatch, tx, m, batch, fixed):
    """Default (tridiagonal through iteration 6) and always-tridiagonal against Jacobi throughout: equal
    iteration counts, X within 1e-10; a sample against the C oracle within 1e-5 with equal counts.
    (8, 192): m >= 3n, the one-entry profile [r3] / [0.995]; (16, 64): [3, 4, 6]; 32-ant: [3, 4, 6, 12]."""
    from ace_amd import synth_problem
    A, B, X0, _ = synth_problem(7301 + tx, 0, batch, m, tx, tx)
    kw = dict(maxiter=200 if fixed else 500, fixed_iters=fixed)
    Xj, ij = _solve(A, B, X0, tx, monkeypatch, 0, **kw)
    for tk in (6, 100000):
        Xt, it = _solve(A, B, X0, tx, monkeypatch, tk, **kw)
        assert np.array_equal(it, ij), (tk, it[it != ij][:8], ij[it != ij][:8])
        e = _errs(Xt, Xj)
        assert np.median(e) <= 1e-12 and e.max() <= 1e-10, (tk, np.median(e), e.max())
    idx = np.arange(0, batch, batch // 4)
    Xo, _, ito, _, _ = OC.infer_admm_r1_batch(A[0].cpu().numpy()[None], OC.make_U(A[0].cpu().numpy())[None],
                                              B.cpu().numpy()[idx], X0.cpu().numpy()[idx], tx, tx, variant=0,
                                              maxiter=kw["maxiter"], fixed_iters=fixed)
    assert np.array_equal(it[idx], ito), (it[idx], ito)
    assert _errs(Xt[idx], Xo).max() <= TOL


def test_clustered_top_eigenvalues_fall_back_to_jacobi(gpu, monkeypatch, capfd):
    """X0 = vec(U diag(s) V^H) with s = (3, 3, 3, 2, 1.5, ...): the init Z-step's E E^H has a triple top
    eigenvalue.  T then nearly splits (off-diagonals at rounding level) and the twisted vectors of the three
    equal Ritz values either land in different blocks (a valid orthonormal basis of the cluster: accepted)
    or repeat one vector (the QR's noise column fails the residual check and the realisation goes to the
    Jacobi eigensolver, H formed again from E).  Both kinds occur here (ACE_TK_TRACE counts the fallbacks);
    the results equal the Jacobi solve's and the oracle's."""
    import torch
    from ace_amd import synth_problem
    tx, m, batch = 32, 256, 64
    A, B, X0, _ = synth_problem(7411, 0, batch, m, tx, tx)
    rng = np.random.default_rng(7411)
    s = np.r_[3.0, 3.0, 3.0, 2.0, np.linspace(1.5, 0.1, tx - 4)]
    X0h = np.empty((batch, tx * tx), np.complex128)
    for b in range(batch):
        U, _ = np.linalg.qr(rng.standard_normal((tx, tx)) + 1j * rng.standard_normal((tx, tx)))
        V, _ = np.linalg.qr(rng.standard_normal((tx, tx)) + 1j * rng.standard_normal((tx, tx)))
        X0h[b] = ((U * s) @ V.conj().T).reshape(-1, order="F")
    X0 = torch.from_numpy(X0h).to(A.device)
    kw = dict(maxiter=200, fixed_iters=True)
    monkeypatch.setenv("ACE_TK_TRACE", "1")
    Xt, it = _solve(A, B, X0, tx, monkeypatch, 6, **kw)
    err = capfd.readouterr().err
    fb = [int(v) for v in re.findall(r"Jacobi fallbacks (\d+)", err)]
    assert fb and sum(fb) >= 1, err[-2000:]
    Xj, ij = _solve(A, B, X0, tx, monkeypatch, 0, **kw)
    assert np.array_equal(it, ij)
    assert _errs(Xt, Xj).max() <= 1e-10
    idx = np.arange(0, batch, 16)
    Xo, _, ito, _, _ = OC.infer_admm_r1_batch(A[0].cpu().numpy()[None], OC.make_U(A[0].cpu().numpy())[None],
                                              B.cpu().numpy()[idx], X0h[idx], tx, tx, variant=0, **kw)
    assert np.array_equal(it[idx], ito)
    assert _errs(Xt[idx], Xo).max() <= TOL


def test_tridiagonal_zstep_batch_position_invariance(gpu, monkeypatch):
    """A realisation's result does not depend on its batch neighbours (bit-identical to a batch of one)."""
    from ace_amd import synth_problem
    tx, m = 32, 256
    A, B, X0, _ = synth_problem(7507, 0, 130, m, tx, tx)
    Xf, _ = _solve(A, B, X0, tx, monkeypatch, 100000, maxiter=60, fixed_iters=True)
    for b in (0, 77, 129):
        Xb, _ = _solve(A, B[b:b + 1], X0[b:b + 1], tx, monkeypatch, 100000, maxiter=60, fixed_iters=True)
        assert np.array_equal(Xb[0], Xf[b]), b
