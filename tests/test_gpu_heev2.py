"""GPU parity of PhaseLift's prox eigensolver (TFOCS/prox_trace.m:88-92: every eigenpair of (X + X^H)/2 above
lambda * step) through ace_prox_eig_host, for the two-stage reduction (csrc/ace_heev2.hip: dense -> band on
the f64 matrix cores, band -> tridiagonal by bulge chasing, tools/proto_heev2.py is its numpy model) and the
one-stage ones it replaces.

The reference's eig (MATLAB, LAPACK zheevd) fixes eigenvectors only up to a unit phase each, so the checks are
on what prox_trace consumes: the kept count, the eigenvalues, and the shrunk projector
X = sum_q (lam_q - tau) v_q v_q^H (invariant to the phases and to rotations inside clusters), against numpy's
eigh (LAPACK zheevd as well), plus residuals and orthonormality of the vectors themselves.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _herm(rng, d, batch, rank=None):
    A = rng.standard_normal((batch, d, d)) + 1j * rng.standard_normal((batch, d, d))
    if rank is not None:   # low rank: zero columns and panels in the reduction
        U = A[:, :, :rank]
        return np.einsum("bik,bjk->bij", U, U.conj())
    return (A + np.conj(np.swapaxes(A, 1, 2))) / 2


def _tau_at(a, f):
    """A threshold halfway between two neighbouring eigenvalues (fraction f of the spectrum below it), so that the
    kept count is not decided by rounding."""
    w = np.linalg.eigvalsh(a)
    i = min(max(int(f * len(w)), 1), len(w) - 1)
    return 0.5 * (w[i - 1] + w[i])


def _projector(lam, V, k, tau):
    Vk = V[:k]                       # rows = eigenvectors
    return Vk.T @ np.diag(lam[:k] - tau) @ Vk.conj()


def _check(A, tau, lam, V, k, tol=1e-11):
    d = A.shape[0]
    w, U = np.linalg.eigh(A)
    keep = w > tau
    assert k == int(keep.sum())
    nrm = np.linalg.norm(A)
    ref_l = w[keep][::-1]
    assert np.abs(lam[:k] - ref_l).max(initial=0.0) <= tol * nrm
    Xr = U[:, keep] @ np.diag(w[keep] - tau) @ U[:, keep].conj().T
    X = _projector(lam, V, k, tau)
    assert np.linalg.norm(X - Xr) <= tol * max(nrm, 1.0), np.linalg.norm(X - Xr) / nrm
    if k:
        Vk = V[:k].T                 # columns = eigenvectors
        res = np.linalg.norm(A @ Vk - Vk * lam[:k], axis=0).max()
        assert res <= tol * nrm, res / nrm
        assert np.abs(Vk.conj().T @ Vk - np.eye(k)).max() <= 1e-10


@pytest.mark.parametrize("d", [32, 40, 64, 121, 200, 256])
def test_two_stage_matches_eigh(gpu, d):
    from ace_amd import prox_eig_host
    rng = np.random.default_rng(100 + d)
    A = _herm(rng, d, 3)
    tau = np.array([_tau_at(a, f) for a, f in zip(A, (0.4, 0.05, 0.9))])
    lam, V, k = prox_eig_host(A, tau, path=2)
    for b in range(3):
        _check(A[b], tau[b], lam[b], V[b], k[b])


@pytest.mark.parametrize("d", [48, 256])
def test_two_stage_low_rank_and_empty(gpu, d):
    """Rank-3 matrices (all but three panel columns vanish: zero reflectors, tau = 0) and a threshold above the
    spectrum (k = 0), as the prox meets them once z is near rank one."""
    from ace_amd import prox_eig_host
    rng = np.random.default_rng(7 + d)
    A = _herm(rng, d, 2, rank=3)
    A[1] *= 0.0
    tau = np.array([1e-3, 1e-3])
    lam, V, k = prox_eig_host(A, tau, path=2)
    _check(A[0], tau[0], lam[0], V[0], k[0])
    assert k[0] == 3 and k[1] == 0


def test_two_stage_agrees_with_one_stage(gpu):
    """The same prox inputs through the blocked one-stage reduction (the r05 default) and the two-stage one."""
    from ace_amd import prox_eig_host
    rng = np.random.default_rng(5)
    A = _herm(rng, 256, 4)
    tau = np.full(4, 0.5)
    l1, V1, k1 = prox_eig_host(A, tau, path=1)
    l2, V2, k2 = prox_eig_host(A, tau, path=2)
    assert np.array_equal(k1, k2)
    for b in range(4):
        nrm = np.linalg.norm(A[b])
        assert np.abs(l1[b, :k1[b]] - l2[b, :k2[b]]).max() <= 1e-12 * nrm
        X1, X2 = _projector(l1[b], V1[b], k1[b], 0.5), _projector(l2[b], V2[b], k2[b], 0.5)
        assert np.linalg.norm(X1 - X2) <= 1e-11 * nrm


def test_two_stage_batch_invariance(gpu):
    """A matrix's result does not depend on the rest of the batch (bit for bit)."""
    from ace_amd import prox_eig_host
    rng = np.random.default_rng(11)
    A = _herm(rng, 256, 5)
    tau = np.full(5, 0.3)
    lam, V, k = prox_eig_host(A, tau, path=2)
    l1, V1, k1 = prox_eig_host(A[3:4], tau[3:4], path=2)
    assert k1[0] == k[3] and np.array_equal(l1[0, :k[3]], lam[3, :k[3]]) and np.array_equal(V1[0, :k[3]], V[3, :k[3]])


@pytest.mark.parametrize("path", [1, 2])
def test_smaller_side(gpu, path):
    """PhaseLift's default (path + 4): with more than half of the eigenvalues above tau the solver returns the
    pairs at or below it, and X = (A - tau I) + sum_{lam <= tau} (tau - lam) v v^H is the same shrunk projector."""
    from ace_amd import prox_eig_host
    rng = np.random.default_rng(31)
    d = 256
    A = _herm(rng, d, 3)
    tau = np.array([_tau_at(a, f) for a, f in zip(A, (0.2, 0.7, 0.45))])
    lam, V, k = prox_eig_host(A, tau, path=path + 4)
    for b in range(3):
        w, U = np.linalg.eigh(A[b])
        above = int((w > tau[b]).sum())
        nrm = np.linalg.norm(A[b])
        Xr = U[:, w > tau[b]] @ np.diag(w[w > tau[b]] - tau[b]) @ U[:, w > tau[b]].conj().T
        if 2 * above > d:
            kc = -k[b]
            assert kc == d - above
            Vk = V[b, :kc]
            assert np.abs(lam[b, :kc] - w[:kc]).max() <= 1e-11 * nrm
            X = A[b] - tau[b] * np.eye(d) + Vk.T @ np.diag(tau[b] - lam[b, :kc]) @ Vk.conj()
        else:
            assert k[b] == above
            X = _projector(lam[b], V[b], k[b], tau[b])
        assert np.linalg.norm(X - Xr) <= 1e-11 * nrm, (b, np.linalg.norm(X - Xr) / nrm)
