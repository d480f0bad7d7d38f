"""Full-horizon parity (the benchmarked 200 iterations) for the two solvers whose iterations amplify rounding:
PhaseLift / TFOCS at config 4's geometry, A2nuclear at config 3's (32 antennas, m = 256, a 4096-realisation
batch, so the split path runs) and at config 5's (the 32-antenna multiresolution codebook).

Past ~60-100 iterations the reference is rounding-chaotic against ITSELF: a 1e-15 relative change of its input moves
its own 200-iteration result by ~2e-3 (PhaseLift) and by anything from 1e-15 to O(1) per realisation (A2nuclear;
measured here, and see test_oracle.py::test_nuclear_refinement_is_rounding_chaotic).  So the bound on the GPU's distance from the
oracle is the oracle's own envelope, as in test_gpu_parity.py::test_nuclear_mspace_matches_nspace:

    bound = max(1e-8, 100 * ||oracle(B) - oracle(B (1 + 1e-15))||)        (relative, phase aligned)

(A2nuclear: the largest such distance over four perturbations of that size, B (1 +- 1e-15), B (1 + 3e-15),
X0 (1 + 1e-15)) per sampled realisation: tight (1e-8) where the reference is stable, as loose as the reference itself where it is
not.  The TFOCS objective 0.5 ||A(X) - b||^2 + lambda tr X (tfocs_AT.m:20-88, smooth_quad + prox_trace) of the final
iterate is held to the same kind of bound: at 200 iterations it moves ~8e-4 relative under the 1e-15 perturbation
in the oracle itself, so a fixed 1e-8 bar would fail the reference against itself (measured, r06).
"""
import numpy as np
import pytest

import ace_oracle as O
import ace_oracle_c as OC
import tfocs_oracle as T

from test_gpu_phaselift import _problem as _pl_problem

pytestmark = pytest.mark.gpu


def _tfocs_objective(X, R, b, lam=5e-2):
    """0.5 ||A(X) - b||^2 + lam tr X in the reduced coordinates: A(X) = diag(R^H X R)."""
    Ax = np.real(np.sum(R.conj() * (X @ R), axis=0))
    return 0.5 * float(np.sum((Ax - b) ** 2)) + lam * float(np.real(np.trace(X)))


def test_phaselift_config4_full_horizon_envelope(gpu):
    """MyPhaseLift at config 4's geometry (32 antennas, n = 1024, m = 256) for the full 200 TFOCS iterations:
    the final iterate X (solver_TraceLS's recoveredMat, reduced coordinates), the recovered signal and the TFOCS
    objective of sampled realisations of a 24-realisation batch, each within the oracle's own envelope."""
    from ace_amd import phaselift_host
    Phi, b = _pl_problem(29, 32, 256, 24)
    res = phaselift_host(Phi, b, maxIts=200, with_x=True)
    assert (res.iters == 200).all() and np.isfinite(res.X).all()
    R = np.linalg.cholesky(Phi @ Phi.conj().T).conj().T
    for r in (0, 23):
        sig_o, ref = T.my_phaselift_reduced(b[r], Phi, maxIts=200)
        sig_p, per = T.my_phaselift_reduced(b[r] * (1 + 1e-15), Phi, maxIts=200)
        assert ref.niter == per.niter == 200
        nx = np.linalg.norm(ref.x - per.x) / np.linalg.norm(ref.x)
        ns = O.phase_aligned_rel_err(sig_p, sig_o)
        f_o, f_p = _tfocs_objective(ref.x, R, b[r]), _tfocs_objective(per.x, R, b[r])
        nf = abs(f_o - f_p) / abs(f_o)
        ex = np.linalg.norm(res.X[r] - ref.x) / np.linalg.norm(ref.x)
        es = O.phase_aligned_rel_err(res.sig[r], sig_o)
        ef = abs(_tfocs_objective(res.X[r], R, b[r]) - f_o) / abs(f_o)
        assert ex <= max(1e-8, 100 * nx), (r, ex, nx)
        assert es <= max(1e-8, 100 * ns), (r, es, ns)
        assert ef <= max(1e-8, 100 * nf), (r, ef, nf)


def test_nuclear_config3_full_horizon_envelope(gpu):
    """A2nuclear at config 3 (32/256, batch 4096: the concurrent sub-batch split path) for the full 200
    iterations: sampled realisations against the C oracle within its own envelope, which is 1e-8 wherever the
    reference is stable at 200 iterations and loose only where the reference itself is not."""
    import torch
    from ace_amd import infer_admm_batch, synth_problem
    A, B, X0, _ = synth_problem(83, 0, 4096, 256, 32, 32)
    r = infer_admm_batch(A, B, X0, 32, 32, variant="A2nuclear", maxiter=200, fixed_iters=True)
    torch.cuda.synchronize()
    idx = [0, 511, 1024, 2047, 3000, 4095]
    X = r.X.cpu().numpy()[idx]
    assert (r.iters.cpu().numpy() == 200).all() and np.isfinite(X).all()
    Ah, Bh, X0h = A.cpu().numpy(), B.cpu().numpy()[idx], X0.cpu().numpy()[idx]
    U = OC.make_U(Ah[0])[None]
    Xo, _, ito, _, _ = OC.infer_admm_r1_batch(Ah, U, Bh, X0h, 32, 32, variant=1, maxiter=200, fixed_iters=True)
    assert (ito == 200).all()
    # the envelope from several 1e-15-sized perturbations (one sample under-states it: on a chaotic realisation the
    # oracle's own distance ranges over 5e-4 .. 1.3 between perturbations of the same size, measured)
    noise = np.zeros(len(idx))
    for Bq, Xq in ((Bh * (1 + 1e-15), X0h), (Bh * (1 - 1e-15), X0h), (Bh, X0h * (1 + 1e-15)),
                   (Bh * (1 + 3e-15), X0h)):
        Xp, _, _, _, _ = OC.infer_admm_r1_batch(Ah, U, Bq, Xq, 32, 32, variant=1, maxiter=200, fixed_iters=True)
        noise = np.maximum(noise, [O.unit_phase_aligned_rel_err(Xp[k], Xo[k]) for k in range(len(idx))])
    tight = 0
    for k in range(len(idx)):
        bound = max(1e-8, 100 * noise[k])
        tight += bound == 1e-8
        assert O.unit_phase_aligned_rel_err(X[k], Xo[k]) <= bound, (idx[k], noise[k])
    print(f"A2nuclear 200 iterations: {tight} of {len(idx)} sampled realisations held to 1e-8")


def test_config5_full_horizon_envelope(gpu):
    """Config 5 (A2nuclear on the 32-antenna multiresolution codebook, a 4096-realisation shard) for the full
    200 iterations, against the C oracle within its own multi-perturbation envelope (the tier-0 rows make the
    refinement rounding-chaotic from ~40 iterations on: test_gpu_config5.py)."""
    import torch
    from ace_amd import infer_admm_batch
    from test_gpu_config5 import _workload
    A, B, X0, _ = _workload(4096)
    r = infer_admm_batch(A, B, X0, 32, 32, variant="A2nuclear", maxiter=200, fixed_iters=True)
    torch.cuda.synchronize()
    idx = [0, 1234, 2048, 4095]
    X = r.X.cpu().numpy()[idx]
    assert (r.iters.cpu().numpy() == 200).all() and np.isfinite(X).all()
    Ah, Bh, X0h = A.cpu().numpy(), B.cpu().numpy()[idx], X0.cpu().numpy()[idx]
    U = OC.make_U(Ah[0])[None]
    Xo, _, ito, _, _ = OC.infer_admm_r1_batch(Ah, U, Bh, X0h, 32, 32, variant=1, maxiter=200, fixed_iters=True)
    assert (ito == 200).all()
    noise = np.zeros(len(idx))
    for Bq, Xq in ((Bh * (1 + 1e-15), X0h), (Bh * (1 - 1e-15), X0h), (Bh, X0h * (1 + 1e-15)),
                   (Bh * (1 + 3e-15), X0h)):
        Xp, _, _, _, _ = OC.infer_admm_r1_batch(Ah, U, Bq, Xq, 32, 32, variant=1, maxiter=200, fixed_iters=True)
        noise = np.maximum(noise, [O.unit_phase_aligned_rel_err(Xp[k], Xo[k]) for k in range(len(idx))])
    for k in range(len(idx)):
        assert O.unit_phase_aligned_rel_err(X[k], Xo[k]) <= max(1e-8, 100 * noise[k]), (idx[k], noise[k])
