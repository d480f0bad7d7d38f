"""SpectralInitialize (inferLowRankV4_multi.m:561-574) on the GPU against the oracle
(oracle/ace_oracle.py::spectral_initialize, numpy eigh of As^H As), through both of the
pipeline's paths: the m x m dual Gram (m <= n) and the n x n primal Gram (m > n).

Eigenvectors are unique up to a unit phase (and up to a rotation inside clusters of equal
eigenvalues), so the comparison is the phase-free form X X^H = sum_k s_k v_k v_k^H (sensitive only
to the gap between the r-th and (r+1)-th eigenvalue, printed per case) plus each column after
aligning its phase.  Tolerances: 1e-10 relative for X X^H and the column norms (sqrt(s_k)), 1e-8 per
aligned column (eps ||C|| / gap for the closest neighbouring eigenvalue)."""
import math

import numpy as np
import pytest

import ace_oracle as O

pytestmark = pytest.mark.gpu


def _case(seed, tx, m, count, zero_row=False):
    from ace_amd import synth
    A, B, _, _ = synth.problem(seed, 0, count, m, tx, tx)
    B = B.copy()
    if zero_row:
        B[:, 3] = 0.0          # a zero magnitude (its row drops out of As)
    return A[0], B


@pytest.mark.parametrize("seed,tx,m,r,zero", [(3, 16, 200, 20, False),     # dual: m < n = 256
                                              (4, 16, 640, 20, True),      # primal: m > n
                                              (5, 32, 256, 20, False),     # config-2 geometry (dual)
                                              (6, 32, 1216, 12, False),    # primal, n = 1024
                                              (7, 8, 64, 20, True),        # dual, m = n
                                              # orders that are not multiples of the product's 64-column strips
                                              # or of the panel width (hetrd_blk's lower-triangle tasks, odd
                                              # trailing orders in its column-pair update)
                                              (10, 8, 17, 12, False), (11, 16, 130, 20, False),
                                              (12, 16, 255, 20, True)])
def test_spectral_initialize_matches_oracle(gpu, seed, tx, m, r, zero):
    from ace_amd import SpectralInitialize
    A, B = _case(seed, tx, m, 3, zero)
    X = SpectralInitialize(A, B, r)
    for b in range(B.shape[0]):
        Xo = O.spectral_initialize(A, B[b], r)
        As = A * (B[b] / np.linalg.norm(A, axis=1))[:, None]
        w = np.sort(np.linalg.eigvalsh(As.conj().T @ As))[::-1]
        gap = (w[r - 1] - w[r]) / w[0]
        P, Po = X[b] @ X[b].conj().T, Xo @ Xo.conj().T
        ep = np.linalg.norm(P - Po) / np.linalg.norm(Po)
        assert ep <= 1e-10, (b, ep, gap)
        np.testing.assert_allclose(np.linalg.norm(X[b], axis=0), np.linalg.norm(Xo, axis=0), rtol=1e-10)
        for k in range(r):
            x, xo = X[b][:, k], Xo[:, k]
            ph = np.vdot(x, xo)
            ph = ph / abs(ph) if abs(ph) > 0 else 1.0
            e = np.linalg.norm(x * ph - xo) / max(np.linalg.norm(xo), 1e-300)
            assert e <= 1e-8, (b, k, e)


def test_spectral_initialize_single_vector(gpu):
    from ace_amd import SpectralInitialize
    A, B = _case(9, 8, 100, 1)
    X = SpectralInitialize(A, B[0], 4)
    assert X.shape == (64, 4)
    P, Po = X @ X.conj().T, (lambda Xo: Xo @ Xo.conj().T)(O.spectral_initialize(A, B[0], 4))
    assert np.linalg.norm(P - Po) / np.linalg.norm(Po) <= 1e-10
