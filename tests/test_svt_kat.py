"""The nuclear-norm prox (A2nuclear ArgMinZ / Shrink, inferLowRank_Nuclear.m:411-439) pinned by
TFOCS's own known answer for nuclear-norm minimisation.

Fixture: main/3rd_software_component/sparsepr/third/TFOCS/examples/smallscale/reference_solutions/
nuclearNorm_problem1_noiseless.mat (a 30 x 30 rank-2 matrix observed on 580 entries, the CVX
minimiser X_reference of ||X||_* s.t. X(omega) = b), copied as data into
tests/golden/tfocs_nuclearNorm_problem1.npz by tests/golden/make_golden.py.

Harness (examples/smallscale/test_nuclearNorm.m): solver_sNuclearBP({M,N,omega}, b, mu = 1e-3,
X0 = 0, [], opts.alg = 'GRA') passes when ||x - X_reference||_F / ||X_reference||_F < 1e-5.
solver_sNuclearBP minimises ||X||_* + mu/2 ||X||_F^2 s.t. X(omega) = b through its smoothed dual;
its primal point for a dual z is X(z) = argmin ||X||_* + mu/2 ||X||^2 - <P*z, X> = Shrink(P*z, 1)/mu,
and the dual gradient is b - P X(z) with Lipschitz constant ||P||^2 / mu = 1/mu, so 'GRA' (plain
gradient ascent, fixed step mu) is z <- z + mu (b - P X(z)).  Every step is one singular-value soft
threshold of a 30 x 30 matrix: the prox under test (n = 30 rows, r = 30 columns).
"""
import numpy as np
import pytest

import ace_oracle as O
from conftest import ROOT

GOLD = ROOT / "tests" / "golden"
MU = 1e-3


def _kat():
    g = np.load(GOLD / "tfocs_nuclearNorm_problem1.npz")
    return g["omega"] - 1, g["b"], g["X_reference"]


def _gra(prox, om, b, shape, iters):
    """z <- z + mu (b - P Shrink(P* z, 1) / mu); returns the relative error history of X(z)."""
    M, N = shape
    z = np.zeros(len(b))
    X = None
    for _ in range(iters):
        Y = np.zeros(M * N)
        Y[om] = z
        X = prox(Y.reshape(N, M).T) / MU               # column-major vec, as MATLAB's X(omega)
        z = z + MU * (b - X.T.ravel()[om])
    return X


def test_oracle_svt_solves_nuclear_norm_kat():
    """The oracle's Shrink (ace_oracle.argmin_z_nuclear, numpy SVD) inside the harness's GRA
    iteration reaches the CVX solution within test_nuclearNorm.m's 1e-5."""
    om, b, Xr = _kat()
    X = _gra(lambda Y: O.argmin_z_nuclear(Y.astype(complex), np.zeros(Y.shape, complex), 1.0).real,
             om, b, Xr.shape, 4600)
    err = np.linalg.norm(X - Xr) / np.linalg.norm(Xr)
    assert err < 1e-5, err


@pytest.mark.gpu
def test_gpu_nuclear_prox_matches_oracle(gpu):
    """The GPU's r-general nuclear Z-prox (Gram r x r + Jacobi eigensolver) against numpy's SVD
    soft threshold: the r = 20 stage shape (n = 1024), the KAT shape (30 x 30), r = 32 and r = 1,
    thresholds that zero some singular values and that zero all of them."""
    import torch
    from ace_amd import nuclear_prox_batch
    rng = np.random.default_rng(3)
    for n, r, tau in ((1024, 20, 0.5), (30, 30, 1.0), (256, 32, 4.0), (64, 7, 0.25), (1024, 1, 0.5), (16, 4, 1e6)):
        E = (rng.standard_normal((5, r, n)) + 1j * rng.standard_normal((5, r, n))) / np.sqrt(n)
        E[1] = E[1, :1].repeat(r, axis=0) * np.linspace(1, 2, r)[:, None]     # rank one
        Z = nuclear_prox_batch(torch.from_numpy(E).cuda(), tau).cpu().numpy()
        for k in range(5):
            Zo = O.argmin_z_nuclear(E[k].T, np.zeros((n, r), complex), 1.0 / tau).T
            den = max(np.linalg.norm(Zo), 1e-300)
            assert np.linalg.norm(Z[k] - Zo) <= 1e-11 * max(den, np.linalg.norm(E[k])), (n, r, tau, k)


@pytest.mark.gpu
def test_gpu_svt_solves_nuclear_norm_kat(gpu):
    """The same harness with every Shrink on the GPU kernel: the CVX solution within 1e-5."""
    import torch
    from ace_amd import nuclear_prox_batch
    om, b, Xr = _kat()

    def prox(Y):
        E = torch.from_numpy(np.ascontiguousarray(Y.T).astype(complex)[None]).cuda()   # [1][r = N][n = M]
        return nuclear_prox_batch(E, 1.0).cpu().numpy()[0].T.real

    X = _gra(prox, om, b, Xr.shape, 4600)
    err = np.linalg.norm(X - Xr) / np.linalg.norm(Xr)
    assert err < 1e-5, err
