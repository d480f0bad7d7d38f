"""CPU tests of the oracle (the checker): golden vectors, the two restatements
against each other, MATLAB-semantics units, and recovery properties.

Parity against MATLAB itself is unpinned (no MATLAB in the image, no reference
ADMM outputs) -- see DESIGN.md.
"""
import math
import pathlib

import numpy as np
import pytest

import ace_oracle as O
import ace_oracle_c as OC
from ace_amd import synth

GOLD = pathlib.Path(__file__).resolve().parent / "golden"


def _A(codes):
    n = codes.shape[-1]
    return (1j ** codes.astype(np.int64)).astype(np.complex128) / math.sqrt(n)


def _err(a, b):
    return O.unit_phase_aligned_rel_err(a, b)


# ---------------------------------------------------------------- golden vectors
@pytest.mark.parametrize("name", ["pipeline_v4_16ant_m64", "pipeline_v4multi_16ant_m64",
                                  "pipeline_nuclear_16ant_m64"])
def test_pipeline_golden(name):
    g = np.load(GOLD / f"{name}.npz")
    A = _A(g["codes"])
    tx = int(g["tx"])
    for b in range(g["B"].shape[0]):
        res = O.infer_low_rank_pipeline(A, g["B"][b], tx, tx, list(g["train_idx"][b]), variant=int(g["variant"]))
        assert res.stage_iters == list(g["stage_iters"][b])
        assert abs(res.quality - g["quality"][b]) <= 1e-9
        assert _err(res.X, g["X"][b]) <= 1e-9


@pytest.mark.parametrize("name", ["refine_a2only_16ant_m64", "refine_a2only_32ant_m256",
                                  "refine_a2only_32ant_m256_fixed200", "refine_nuclear_16ant_m64_fixed60"])
def test_refine_golden_numpy_and_c(name):
    """Both restatements reproduce the committed InferADMM (r = 1) vectors."""
    g = np.load(GOLD / f"{name}.npz")
    A = _A(g["codes"])
    tx = int(g["tx"])
    var, maxiter, fixed = int(g["variant"]), int(g["maxiter"]), bool(g["fixed"])
    U = O.make_U(A)
    Xc, Yc, itc, cvc, _ = OC.infer_admm_r1_batch(A[None], OC.make_U(A)[None], g["B"], g["X0"], tx, tx,
                                                 variant=var, maxiter=maxiter, fixed_iters=fixed)
    for b in range(g["B"].shape[0]):
        r = O.infer_admm(A, g["B"][b], g["X0"][b][:, None], True, False, tx, tx, U=U, variant=var,
                         maxiter=maxiter, fixed_iters=fixed)
        assert r.iters == g["iters"][b] == itc[b]
        assert r.converged == bool(g["converged"][b]) == bool(cvc[b])
        assert _err(r.X, g["X"][b]) <= 1e-9
        assert _err(Xc[b], g["X"][b]) <= 1e-9
        assert _err(Yc[b], g["Y"][b]) <= 1e-9


def test_synth_generator_pinned():
    g = np.load(GOLD / "synth_pin.npz")
    assert np.array_equal(synth.codebook_codes(58659179, 8, 16), g["codes"])
    assert np.allclose(synth.normal_pairs(58659179, 3, 4), g["normals"], rtol=1e-14, atol=0)
    assert np.allclose(synth.channel(58659179, 0, 4, 4), g["vecH"], rtol=1e-13, atol=1e-15)


def test_reference_codebook_layout():
    """The reference's probing codebook (codebook/codebook_mat/random_probe_cb_16x16.mat,
    3968 x 256, entries j^k) has the layout the synthetic codebook reproduces:
    unit-modulus 2-bit phase states, one row per probe, kron(tx, rx) columns."""
    g = np.load(GOLD / "ref_codebook_16x16_slice.npz")
    assert tuple(g["shape"]) == (3968, 256)
    head = g["codes_head"]
    assert head.dtype == np.uint8 and head.max() <= 3
    counts = np.bincount(head.ravel(), minlength=4) / head.size
    assert np.all(np.abs(counts - 0.25) < 0.05)          # uniform phase states
    ours = synth.codebook_codes(1, 64, 256)
    assert ours.shape == head.shape and ours.max() <= 3
    A = _A(head)
    assert np.allclose(np.linalg.norm(A, axis=1), 1.0)   # rows normalised like FW / sqrt(Nt*Nr)


# ----------------------------------------------------------------- MATLAB semantics
def test_rank_profiles():
    """inferLowRankV4_multi.m:437-464 for the reference's antenna counts."""
    assert O.rank_profile(32, 32, 256, 1024, False) == ([3, 4, 6, 12], [0.8, 0.9, 0.95, 0.995])
    assert O.rank_profile(16, 16, 64, 256, False) == ([3, 4, 8], [0.9, 0.95, 0.995])
    assert O.rank_profile(16, 16, 64, 256, True) == ([1], [0.95])
    assert O.rank_profile(16, 16, 768, 256, False) == ([8], [0.995])
    assert O.rank_profile(4, 4, 16, 16, False) == ([2], [0.95])


def test_c_jacobi_eig_matches_lapack():
    rng = np.random.default_rng(0)
    for n in (4, 16, 32):
        E = rng.standard_normal((n, n)) + 1j * rng.standard_normal((n, n))
        H = E @ E.conj().T
        w, V = OC.herm_eig(H)
        wl = np.linalg.eigvalsh(H)
        assert np.allclose(w, wl, rtol=0, atol=1e-12 * wl.max())
        assert np.allclose(V.conj().T @ V, np.eye(n), atol=1e-12)
        assert np.allclose(H @ V, V * w[None, :], atol=1e-10 * wl.max())


def test_argmin_y_zero_guards():
    Y = np.array([[0.0], [3 + 4j]])
    out = O.argmin_y(np.zeros((2, 1), complex), np.array([2.0, 5.0]), Y.copy(), 1.0, True)
    # C = AX + M/mu = [0, 3+4j]; zero row -> 1/sqrt(r) with D = 1; Y = C (B/D + mu)/(1 + mu)
    assert np.allclose(out[:, 0], [1.0 * (2.0 + 1.0) / 2.0, (3 + 4j) * (5.0 / 5.0 + 1.0) / 2.0])


def test_stable_descending_sort_ties():
    # MATLAB sort(...,'descend') is stable: equal values keep their original order
    s2 = np.array([1.0, 3.0, 3.0, 2.0])
    assert list(np.argsort(-s2, kind="stable")) == [1, 2, 3, 0]


# -------------------------------------------------------------- cross restatements
@pytest.mark.parametrize("tx,m", [(8, 64), (16, 64), (16, 256)])
def test_numpy_vs_c_a2only(tx, m):
    A, B, X0, _ = synth.problem(77, 0, 3, m, tx, tx)
    U = O.make_U(A[0])
    Xc, _, itc, _, _ = OC.infer_admm_r1_batch(A, U[None], B, X0, tx, tx)
    for b in range(3):
        r = O.infer_admm(A[0], B[b], X0[b][:, None], True, False, tx, tx, U=U)
        assert r.iters == itc[b]
        assert _err(r.X, Xc[b]) <= 1e-10


def test_c_private_codebooks():
    A, B, X0, _ = synth.problem(78, 0, 3, 64, 8, 8, a_shared=False)
    Us = np.stack([OC.make_U(a) for a in A])
    Xc, _, itc, _, _ = OC.infer_admm_r1_batch(A, Us, B, X0, 8, 8)
    for b in range(3):
        r = O.infer_admm(A[b], B[b], X0[b][:, None], True, False, 8, 8)
        assert r.iters == itc[b] and _err(r.X, Xc[b]) <= 1e-10


def test_nuclear_refinement_is_rounding_chaotic():
    """Documents why nuclear-variant parity is asserted on short horizons only:
    the ORACLE against itself, with B perturbed by one part in 1e15, diverges to
    O(1e-1) differences before converging (Lyapunov growth ~1.2x per iteration
    while mu is small).  No implementation can match MATLAB there to 1e-5."""
    A, B, X0, _ = synth.problem(7, 0, 1, 64, 16, 16)
    Bu = B[0] * np.linalg.norm(B[0]) ** 0  # already normalised
    U = O.make_U(A[0])
    r1 = O.infer_admm(A[0], Bu, X0[0][:, None], True, False, 16, 16, U=U, variant=1, want_trace=True)
    r2 = O.infer_admm(A[0], Bu * (1 + 1e-15), X0[0][:, None], True, False, 16, 16, U=U, variant=1,
                      want_trace=True)
    mid = max(abs(a["res_comb"] - b["res_comb"]) / a["res_comb"] for a, b in zip(r1.trace[:250], r2.trace[:250]))
    assert mid > 1e-3
    # ... while the first 60 iterations agree to ~1e-12
    early = max(abs(a["res_comb"] - b["res_comb"]) / a["res_comb"] for a, b in zip(r1.trace[:60], r2.trace[:60]))
    assert early < 1e-9


# ------------------------------------------------------------------- properties
@pytest.mark.parametrize("tx,m", [(4, 64), (8, 256)])
def test_pipeline_recovers_channel_with_many_measurements(tx, m):
    """With m = 4n magnitude measurements at 60 dB SNR the restated pipeline recovers
    the sparse multipath channel to ~1e-3 (phase-aligned, Evaluation_H.m:81-89)."""
    A, B, X0, H = synth.problem(5, 0, 1, m, tx, tx, snr_db=60.0)
    rng = np.random.default_rng(0)
    tr = [rng.permutation(m)[:math.floor(0.95 * m)] for _ in range(3)]
    r = O.infer_low_rank_pipeline(A[0], B[0], tx, tx, tr)
    assert r.quality > 0.99
    assert O.phase_aligned_rel_err(r.X, H[0]) < 5e-3


def test_phase_equivariance():
    """InferADMM is equivariant under a global phase of X0 (why parity is measured
    after phase alignment, Evaluation_H.m:81-82)."""
    A, B, X0, _ = synth.problem(9, 0, 1, 64, 8, 8)
    U = O.make_U(A[0])
    r1 = O.infer_admm(A[0], B[0], X0[0][:, None], True, False, 8, 8, U=U)
    r2 = O.infer_admm(A[0], B[0], X0[0][:, None] * np.exp(0.7j), True, False, 8, 8, U=U)
    assert r1.iters == r2.iters
    assert np.allclose(r2.X, r1.X * np.exp(0.7j), atol=1e-10)


# ---------------------------------------------------------------------------- TFOCS / PhaseLift
def test_tfocs_tracels_known_answer():
    """The TFOCS restatement reproduces TFOCS's own known answer for solver_TraceLS
    (examples/smallscale/test_TraceLS.m: tol 1e-12, restart 100; pass = relative error to
    the CVX solution below 1e-5)."""
    import tfocs_oracle as T
    g = np.load(GOLD / "tfocs_traceLS_problem1.npz")
    om, b, lam, Xr = g["omega"] - 1, g["b"], float(g["lam"]), g["X_reference"]
    N = Xr.shape[0]

    def Aop(X):
        return X.flatten(order="F")[om]

    def Aadj(y):
        Z = np.zeros(N * N)
        Z[om] = y
        return Z.reshape(N, N, order="F")

    r = T.tfocs_at_tracels(Aop, Aadj, b, lam, np.zeros((N, N)), tol=1e-12, restart=100)
    err = np.linalg.norm(r.x - Xr) / np.linalg.norm(Xr)
    obj = 0.5 * np.linalg.norm(Aop(r.x) - b) ** 2 + lam * np.trace(r.x)
    assert r.status.startswith("Step size") and err < 1e-5, (r.status, err)
    assert abs(obj - float(g["obj_reference"])) < 1e-8


def test_phaselift_reduction_is_exact():
    """The GPU's reduced coordinates: with X0 = 0 every TFOCS iterate lies in
    Q X Q^H, Q = range(Phi^H), so the d x d iteration with R = chol(Phi Phi^H) reproduces the
    dense n x n oracle (here both in numpy)."""
    import math
    import tfocs_oracle as T
    from ace_amd import synth
    n, m = 64, 24
    Phi = synth.codebook(5, m, n) * math.sqrt(n)
    h = synth.channel(5, 0, 8, 8)
    b = np.abs(Phi @ h) ** 2
    dense = T.tfocs_at_tracels(*T.phaselift_ops(Phi), b, 0.05, np.zeros((n, n), complex), maxIts=30, tol=1e-10,
                               restart=200)
    R = np.linalg.cholesky(Phi @ Phi.conj().T).conj().T          # Phi^H = Q R
    Q = Phi.conj().T @ np.linalg.inv(R)
    red = T.tfocs_at_tracels(lambda X: np.einsum("ji,jk,ki->i", R.conj(), X, R),
                             lambda g: (R * g[None, :]) @ R.conj().T, b, 0.05, np.zeros((m, m), complex),
                             maxIts=30, tol=1e-10, restart=200)
    assert np.linalg.norm(Q @ red.x @ Q.conj().T - dense.x) <= 1e-10 * np.linalg.norm(dense.x)
