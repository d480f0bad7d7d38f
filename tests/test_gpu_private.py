"""GPU parity of the private phase-code path (regime P, ace_private.hip): one codebook per
realisation, 2-bit code images, G_b = (I + A_b A_b^H)^{-1} as Hermitian tiles, pgk_kernel + the
one-wave Z-step per iteration.

Checked against the C oracle (U = inv(A'A + I) per realisation, inferLowRankV4_multi.m:281-386)
and against the f64 private path (f64_applies=True: complex128 GEMVs over A_b and G_b).
Tolerance (north_star): 1e-5 relative Frobenius error after global-phase alignment
(Evaluation_H.m:81-82), iteration counts equal; the two GPU paths agree to 1e-9.
"""
import numpy as np
import pytest

import ace_oracle as O
import ace_oracle_c as OC

pytestmark = pytest.mark.gpu

TOL = 1e-5


def _problem(seed, count, m, tx):
    from ace_amd import synth
    return synth.problem(seed, 0, count, m, tx, tx, a_shared=False)


def _oracle(A, B, X0, tx, **kw):
    U = np.stack([OC.make_U(a) for a in A])
    return OC.infer_admm_r1_batch(A, U, B, X0, tx, tx, **kw)


def _errs(Xg, Xo):
    return np.array([O.unit_phase_aligned_rel_err(Xg[b], Xo[b]) for b in range(Xg.shape[0])])


def _launches(fn):
    import ctypes as C
    import torch
    from ace_amd._lib import LIB, KERNEL_CLASSES, check
    fn()
    torch.cuda.synchronize()
    check(LIB.ace_prof_sample(1, 0))
    check(LIB.ace_prof_start(8192))
    fn()
    torch.cuda.synchronize()
    kt = (C.c_double * len(KERNEL_CLASSES))()
    kn = (C.c_int32 * len(KERNEL_CLASSES))()
    check(LIB.ace_prof_stop(kt, kn))
    return dict(zip(KERNEL_CLASSES, kn))


@pytest.mark.parametrize("tx,m", [(16, 64), (16, 20), (16, 48), (16, 160), (32, 256)])
@pytest.mark.parametrize("fixed", [True, False])
def test_private_phase_code_matches_oracle(gpu, tx, m, fixed):
    from ace_amd import infer_admm_host
    A, B, X0, _ = _problem(41 + m, 4, m, tx)
    kw = dict(variant="A2only", maxiter=200 if fixed else 500, fixed_iters=fixed)
    res = infer_admm_host(A, B, X0, tx, tx, **kw)
    r64 = infer_admm_host(A, B, X0, tx, tx, f64_applies=True, **kw)
    assert _errs(res.X, r64.X).max() <= 1e-9
    assert np.array_equal(res.iters, r64.iters)
    Xo, Yo, ito, cvo, _ = _oracle(A, B, X0, tx, variant=0, maxiter=kw["maxiter"], fixed_iters=fixed)
    e = _errs(res.X, Xo)
    assert e.max() <= TOL, e
    assert np.array_equal(res.iters, ito), (res.iters, ito)
    assert np.array_equal(res.converged, cvo)
    assert _errs(res.Y, Yo).max() <= TOL


def test_private_nuclear_short_horizon(gpu):
    from ace_amd import infer_admm_host
    A, B, X0, _ = _problem(9, 4, 256, 32)
    res = infer_admm_host(A, B, X0, 32, 32, variant="A2nuclear", maxiter=60, fixed_iters=True)
    Xo, _, _, _, _ = _oracle(A, B, X0, 32, variant=1, maxiter=60, fixed_iters=True)
    # the nuclear refinement's own 1-ulp noise floor at 60 iterations is ~1e-9 (test_gpu_parity.py)
    assert _errs(res.X, Xo).max() <= 1e-8


def test_private_batch_position_invariance(gpu):
    """A realisation's result does not depend on its batch or position (one work-group each)."""
    import torch
    from ace_amd import infer_admm_batch, synth_problem
    A, B, X0, _ = synth_problem(43, 0, 96, 256, 32, 32, a_shared=False)
    big = infer_admm_batch(A, B, X0, 32, 32, maxiter=60, fixed_iters=True)
    torch.cuda.synchronize()
    for lo in (0, 37, 80):
        sub = infer_admm_batch(A[lo:lo + 16].contiguous(), B[lo:lo + 16].contiguous(), X0[lo:lo + 16].contiguous(),
                               32, 32, maxiter=60, fixed_iters=True)
        torch.cuda.synchronize()
        assert np.array_equal(sub.X.cpu().numpy(), big.X.cpu().numpy()[lo:lo + 16]), lo


def test_private_phase_code_launches_two_kernels_per_iteration(gpu):
    """pgk_kernel (class apply_G) + Z-step per iteration; no separate A, A^H, K or Y-step launch."""
    from ace_amd import infer_admm_batch, synth_problem
    A, B, X0, _ = synth_problem(47, 0, 64, 256, 32, 32, a_shared=False)
    iters = 20
    n = _launches(lambda: infer_admm_batch(A, B, X0, 32, 32, maxiter=iters, fixed_iters=True))
    for k in ("apply_A", "apply_AH", "pre", "ystep", "apply_K"):
        assert n[k] == 0, (k, n)
    for k in ("apply_G", "zstep"):
        assert n[k] == iters, (k, n)


def test_private_non_phase_code_falls_back(gpu):
    """One realisation's codebook is not a phase code: the batch takes the f64 private path and
    still matches the oracle."""
    from ace_amd import infer_admm_host
    A, B, X0, _ = _problem(53, 3, 64, 16)
    A = A.copy()
    A[1, 3, 7] *= 1.5
    res = infer_admm_host(A, B, X0, 16, 16, variant="A2only")
    Xo, _, ito, _, _ = _oracle(A, B, X0, 16, variant=0)
    assert _errs(res.X, Xo).max() <= TOL
    assert np.array_equal(res.iters, ito)


def test_private_unnormalised_codes(gpu):
    """Codebooks with a different scale per realisation (c_b) and the raw +-1 / +-j codes."""
    from ace_amd import infer_admm_host
    A, B, X0, _ = _problem(59, 3, 64, 16)
    A = A * np.array([1.0, 16.0, 0.25])[:, None, None]
    B = B * np.array([1.0, 16.0, 0.25])[:, None]
    kw = dict(variant="A2only", maxiter=200, fixed_iters=True)
    res = infer_admm_host(A, B, X0, 16, 16, **kw)
    Xo, _, ito, _, _ = _oracle(A, B, X0, 16, variant=0, maxiter=200, fixed_iters=True)
    assert _errs(res.X, Xo).max() <= TOL


_FOUR_WAVE_SCRIPT = r"""
import sys, numpy as np
sys.path[:0] = sys.argv[1:]
import ace_amd, ace_oracle as O, ace_oracle_c as OC
from ace_amd import synth
A, B, X0, _ = synth.problem(37, 0, 3, 64, 16, 16, a_shared=False)
res = ace_amd.infer_admm_host(A, B, X0, 16, 16, variant="A2only", maxiter=150, fixed_iters=True)
U = np.stack([OC.make_U(a) for a in A])
Xo, _, ito, _, _ = OC.infer_admm_r1_batch(A, U, B, X0, 16, 16, variant=0, maxiter=150, fixed_iters=True)
e = max(O.unit_phase_aligned_rel_err(res.X[b], Xo[b]) for b in range(3))
assert e <= 1e-5 and np.array_equal(res.iters, ito), (e, res.iters, ito)
print("ok", e)
"""


def test_private_codes_with_four_wave_zstep(gpu):
    """ACE_ZSTEP_4WAVE=1 (the four-wave A/B Z-step, read once per process, hence a child process)
    cannot run the code-image iteration, so the private phase-code setup must not be taken either:
    the solve runs the generic f64 private path on properly formed K and G and matches the oracle."""
    import os
    import subprocess
    import sys
    from conftest import ROOT, PKG_DIR
    env = dict(os.environ, ACE_ZSTEP_4WAVE="1")
    out = subprocess.run([sys.executable, "-c", _FOUR_WAVE_SCRIPT, str(PKG_DIR), str(ROOT / "oracle")], env=env,
                         capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.startswith("ok")
