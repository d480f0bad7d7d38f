"""GPU parity: the HIP path (through the C-ABI) against the CPU oracles.

Tolerance (north_star): recovered X within 1e-5 relative Frobenius error after
global-phase alignment (Evaluation_H.m:81-82), iteration counts equal.  For the
A2only variant the observed agreement is ~1e-13.  The nuclear variant's
refinement is rounding-chaotic on long horizons (tests/test_oracle.py::
test_nuclear_refinement_is_rounding_chaotic shows the ORACLE against itself with
a 1-ulp input perturbation), so its parity is asserted on horizons where the
oracle is stable against itself.
"""
import numpy as np
import pytest

import ace_oracle as O
import ace_oracle_c as OC

pytestmark = pytest.mark.gpu

TOL = 1e-5


def _problem(seed, count, m, tx, a_shared=True):
    from ace_amd import synth
    return synth.problem(seed, 0, count, m, tx, tx, a_shared=a_shared)


def _oracle(A, B, X0, tx, **kw):
    """C oracle over the batch (U-form, exactly the reference formula)."""
    if A.shape[0] == 1:
        U = OC.make_U(A[0])[None]
    else:
        U = np.stack([OC.make_U(a) for a in A])
    return OC.infer_admm_r1_batch(A, U, B, X0, tx, tx, **kw)


def _errs(Xg, Xo):
    return np.array([O.unit_phase_aligned_rel_err(Xg[b], Xo[b]) for b in range(Xg.shape[0])])


@pytest.mark.parametrize("tx,m", [(16, 64), (16, 256), (32, 256)])
@pytest.mark.parametrize("a_shared", [True, False])
def test_a2only_convergence_mode(gpu, tx, m, a_shared):
    from ace_amd import infer_admm_host
    A, B, X0, _ = _problem(3, 5, m, tx, a_shared)
    res = infer_admm_host(A, B, X0, tx, tx, variant="A2only")
    Xo, Yo, ito, cvo, _ = _oracle(A, B, X0, tx, variant=0)
    e = _errs(res.X, Xo)
    assert e.max() <= TOL, e
    assert np.array_equal(res.iters, ito), (res.iters, ito)
    assert np.array_equal(res.converged, cvo)
    ey = _errs(res.Y, Yo)
    assert ey.max() <= TOL


@pytest.mark.parametrize("tx,m", [(16, 64), (32, 256)])
def test_a2only_fixed_200(gpu, tx, m):
    """Throughput-mode unit: exactly 200 iterations, opt_X parity."""
    from ace_amd import infer_admm_host
    A, B, X0, _ = _problem(5, 4, m, tx)
    res = infer_admm_host(A, B, X0, tx, tx, variant="A2only", maxiter=200, fixed_iters=True)
    Xo, _, ito, _, _ = _oracle(A, B, X0, tx, variant=0, maxiter=200, fixed_iters=True)
    assert (res.iters == 200).all() and (ito == 200).all()
    assert _errs(res.X, Xo).max() <= TOL


@pytest.mark.parametrize("tx,m", [(16, 64), (32, 256)])
@pytest.mark.parametrize("a_shared", [True, False])
def test_nuclear_short_horizon(gpu, tx, m, a_shared):
    from ace_amd import infer_admm_host
    A, B, X0, _ = _problem(9, 4, m, tx, a_shared)
    res = infer_admm_host(A, B, X0, tx, tx, variant="A2nuclear", maxiter=60, fixed_iters=True)
    Xo, _, _, _, _ = _oracle(A, B, X0, tx, variant=1, maxiter=60, fixed_iters=True)
    # the oracle against ITSELF with B or X0 perturbed by 1e-15 moves by up to 9e-10 here
    # (16-ant, 60 iterations); the bar sits one decade above that noise floor
    assert _errs(res.X, Xo).max() <= 1e-8


def test_warm_and_cold_eig_agree(gpu):
    from ace_amd import infer_admm_host
    A, B, X0, _ = _problem(13, 6, 256, 32)
    r1 = infer_admm_host(A, B, X0, 32, 32, eig_warm=True)
    r0 = infer_admm_host(A, B, X0, 32, 32, eig_warm=False)
    assert _errs(r1.X, r0.X).max() <= 1e-10
    assert np.array_equal(r1.iters, r0.iters)


def test_use_rank_one_profile(gpu):
    from ace_amd import infer_admm_host
    A, B, X0, _ = _problem(17, 3, 64, 16)
    res = infer_admm_host(A, B, X0, 16, 16, use_rank_one=True)
    Xo, _, ito, _, _ = _oracle(A, B, X0, 16, variant=0, use_rank_one=True)
    assert _errs(res.X, Xo).max() <= TOL
    assert np.array_equal(res.iters, ito)


def test_many_measurements_profile(gpu):
    """m >= 3n selects the single [r3]/[0.995] profile (inferLowRankV4_multi.m:451-453)."""
    from ace_amd import infer_admm_host
    A, B, X0, _ = _problem(19, 2, 3 * 64, 8)
    res = infer_admm_host(A, B, X0, 8, 8)
    Xo, _, ito, _, _ = _oracle(A, B, X0, 8, variant=0)
    assert _errs(res.X, Xo).max() <= TOL
    assert np.array_equal(res.iters, ito)


@pytest.mark.parametrize("m", [121, 243, 1])
def test_ragged_sizes(gpu, m):
    """m not a multiple of the GEMM tile (the reference's M sweep: 4,121,400,...,
    and floor(0.95 m) train rows), batch not a multiple of 64."""
    from ace_amd import infer_admm_host
    A, B, X0, _ = _problem(23, 67, m, 16)
    res = infer_admm_host(A, B, X0, 16, 16, maxiter=100)
    Xo, _, ito, _, _ = _oracle(A, B, X0, 16, variant=0, maxiter=100)
    assert _errs(res.X, Xo).max() <= TOL
    assert np.array_equal(res.iters, ito)


def test_zero_measurement_rows(gpu):
    """ArgMinY/normalize_rows zero guards (inferLowRankV4_multi.m:516-528, :542-554)."""
    from ace_amd import infer_admm_host
    A, B, X0, _ = _problem(29, 3, 64, 16)
    B = B.copy()
    B[:, ::7] = 0.0
    A = A.copy()
    A[0, 5, :] = 0.0  # a zero codebook row makes AX_5 == 0 exactly
    res = infer_admm_host(A, B, X0, 16, 16, maxiter=120)
    Xo, _, ito, _, _ = _oracle(A, B, X0, 16, variant=0, maxiter=120)
    assert np.isfinite(res.X).all()
    assert _errs(res.X, Xo).max() <= TOL
    assert np.array_equal(res.iters, ito)


def test_batch_position_invariance(gpu):
    """A realisation's result is bit-identical whatever batch it is solved in
    (per-output summation order of every kernel is batch-independent)."""
    from ace_amd import infer_admm_host
    A, B, X0, _ = _problem(31, 130, 256, 32)
    full = infer_admm_host(A, B, X0, 32, 32, maxiter=50, fixed_iters=True)
    for b in (0, 64, 129):
        one = infer_admm_host(A, B[b:b + 1], X0[b:b + 1], 32, 32, maxiter=50, fixed_iters=True)
        assert np.array_equal(one.X[0], full.X[b])


def test_device_synth_matches_host(gpu):
    import torch
    from ace_amd import synth, synth_problem
    for a_shared in (True, False):
        A, B, X0, H = synth_problem(77, 5, 3, 64, 16, 16, a_shared=a_shared)
        torch.cuda.synchronize()
        Ah, Bh, X0h, Hh = synth.problem(77, 5, 3, 64, 16, 16, a_shared=a_shared)
        assert np.array_equal(A.cpu().numpy(), Ah)                 # integer stream: exact
        assert np.allclose(B.cpu().numpy(), Bh, rtol=1e-12, atol=1e-14)
        assert np.allclose(H.cpu().numpy(), Hh, rtol=1e-11, atol=1e-13)
        assert np.allclose(X0.cpu().numpy(), X0h, rtol=1e-11, atol=1e-13)


def test_device_batch_api_full_size(gpu):
    """The throughput entry point on HBM-resident tensors at BASELINE config 2
    shape (32-ant, 256 meas) on a 512-realisation batch, 200 fixed iterations;
    a sample is checked against the oracle."""
    import torch
    from ace_amd import infer_admm_batch, synth_problem
    A, B, X0, H = synth_problem(2024, 0, 512, 256, 32, 32)
    res = infer_admm_batch(A, B, X0, 32, 32, maxiter=200, fixed_iters=True)
    torch.cuda.synchronize()
    X = res.X.cpu().numpy()
    assert np.isfinite(X).all()
    assert (res.iters.cpu().numpy() == 200).all()
    idx = [0, 255, 511]
    Ah, Bh, X0h = A.cpu().numpy(), B.cpu().numpy()[idx], X0.cpu().numpy()[idx]
    Xo, _, _, _, _ = _oracle(Ah, Bh, X0h, 32, variant=0, maxiter=200, fixed_iters=True)
    assert _errs(X[idx], Xo).max() <= TOL


def test_error_paths(gpu):
    from ace_amd import infer_admm_host, AceError
    A, B, X0, _ = _problem(1, 1, 16, 4)
    with pytest.raises(AceError):
        infer_admm_host(A, B, X0, 4, 5)            # n != tx*rx
    with pytest.raises(AceError):                  # tx = 33: beyond the Z-prox's 32 rows (33 + 1 padded)
        infer_admm_host(np.ones((1, 16, 66), np.complex128), np.ones((1, 16)), np.zeros((1, 66), np.complex128),
                        33, 2)


def test_a2only_odd_tx_device_path(gpu):
    """The device entry (torch tensors, torch's stream, a caller workspace it does not need) at an odd tx:
    the same X as the host entry, bit for bit."""
    import torch
    from ace_amd import infer_admm_batch, infer_admm_host, synth
    A, B, X0, _ = synth.problem(77, 0, 64, 256, 15, 16)
    ref = infer_admm_host(A, B, X0, 15, 16, variant="A2only", maxiter=200, fixed_iters=True)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        dev = infer_admm_batch(torch.from_numpy(A).cuda(), torch.from_numpy(B).cuda(), torch.from_numpy(X0).cuda(),
                               15, 16, variant="A2only", maxiter=200, fixed_iters=True)
    s.synchronize()
    np.testing.assert_array_equal(dev.X.cpu().numpy(), ref.X)


@pytest.mark.parametrize("tx,rx,m", [(3, 3, 32), (5, 4, 64), (15, 16, 256), (31, 8, 256), (1, 8, 32)])
def test_a2only_odd_tx(gpu, tx, rx, m):
    """Odd tx (inferLowRankV4_multi.m:426 reshapes z to tx x rx for any tx): solved as the zero-padded
    (tx + 1) x rx problem (ace_api.cpp solve_odd_tx), against the C oracle on the tx x rx problem itself:
    convergence mode (X, Y, iteration counts, converged flags) and 200 fixed iterations, shared and
    per-realisation A.  Bound: TOL, or 100x the oracle's own move under a 1e-15 perturbation of B where
    the reference is ill-conditioned (measured: at tx = 1, per-realisation A, one realisation's Y moves 1e-4
    in the oracle itself -- Y's phase at an entry where AX + M/mu is nearly zero)."""
    from ace_amd import infer_admm_host, synth
    for a_shared in (True, False):
        A, B, X0, _ = synth.problem(31 + tx, 0, 4, m, tx, rx, a_shared=a_shared)
        U = np.stack([OC.make_U(a) for a in A])
        res = infer_admm_host(A, B, X0, tx, rx, variant="A2only")
        Xo, Yo, ito, cvo, _ = OC.infer_admm_r1_batch(A, U, B, X0, tx, rx, variant=0)
        Xp, Yp, _, _, _ = OC.infer_admm_r1_batch(A, U, B * (1 + 1e-15), X0, tx, rx, variant=0)
        bx = np.maximum(TOL, 100 * _errs(Xp, Xo))
        by = np.maximum(TOL, 100 * _errs(Yp, Yo))
        assert (_errs(res.X, Xo) <= bx).all(), (a_shared, _errs(res.X, Xo), bx)
        assert (_errs(res.Y, Yo) <= by).all(), (a_shared, _errs(res.Y, Yo), by)
        assert np.array_equal(res.iters, ito), (res.iters, ito)
        assert np.array_equal(res.converged, cvo)
    res = infer_admm_host(A, B, X0, tx, rx, variant="A2only", maxiter=200, fixed_iters=True)
    Xo, _, ito, _, _ = OC.infer_admm_r1_batch(A, U, B, X0, tx, rx, variant=0, maxiter=200, fixed_iters=True)
    assert (res.iters == 200).all() and (ito == 200).all()
    assert _errs(res.X, Xo).max() <= TOL


@pytest.mark.parametrize("fixed", [True, False])
def test_int8_applies_match_f64(gpu, fixed):
    """The exact int8 digit-plane applies (phase-code codebook, ace_i8gemm.hip) against the f64
    matrix-core applies and the C oracle at the unit's size (32 antennas, m = 256)."""
    from ace_amd import infer_admm_host
    A, B, X0, _ = _problem(17, 6, 256, 32)
    kw = dict(variant="A2only", maxiter=200, fixed_iters=fixed)
    r8 = infer_admm_host(A, B, X0, 32, 32, **kw)
    r64 = infer_admm_host(A, B, X0, 32, 32, f64_applies=True, **kw)
    e = _errs(r8.X, r64.X)
    assert e.max() <= 1e-9, e
    assert np.array_equal(r8.iters, r64.iters)
    Xo, _, ito, _, _ = _oracle(A, B, X0, 32, variant=0, maxiter=200, fixed_iters=fixed)
    assert _errs(r8.X, Xo).max() <= TOL
    assert np.array_equal(r8.iters, ito)


def test_generic_codebook_runs_f64_path(gpu):
    """A shared codebook that is not a phase code (complex Gaussian) takes the f64 applies."""
    from ace_amd import infer_admm_host
    rng = np.random.default_rng(5)
    A, B, X0, _ = _problem(19, 4, 64, 16)
    A = (rng.standard_normal(A.shape) + 1j * rng.standard_normal(A.shape)) / np.sqrt(2 * 256)
    H = (rng.standard_normal((4, 256)) + 1j * rng.standard_normal((4, 256)))
    B = np.abs(np.einsum("mn,bn->bm", A[0], H))
    res = infer_admm_host(A, B, X0, 16, 16, variant="A2only")
    Xo, _, ito, _, _ = _oracle(A, B, X0, 16, variant=0)
    assert _errs(res.X, Xo).max() <= TOL
    assert np.array_equal(res.iters, ito)


def test_phase_code_with_switched_off_antennas(gpu):
    """Multiresolution-style codebook: phase codes with switched-off antennas (0 entries) stay
    on the int8 path ({0, +-c} components) and match the oracle."""
    from ace_amd import infer_admm_host
    A, B, X0, _ = _problem(23, 4, 128, 16)
    A = A.copy()
    A[0, :, ::3] = 0.0          # every third antenna off on every probe
    A[0, ::5, 1::3] = 0.0       # and a second group off on every fifth probe
    rng = np.random.default_rng(2)
    H = (rng.standard_normal((4, 256)) + 1j * rng.standard_normal((4, 256)))
    B = np.abs(np.einsum("mn,bn->bm", A[0], H))
    res = infer_admm_host(A, B, X0, 16, 16, variant="A2only", maxiter=200, fixed_iters=True)
    r64 = infer_admm_host(A, B, X0, 16, 16, variant="A2only", maxiter=200, fixed_iters=True, f64_applies=True)
    assert _errs(res.X, r64.X).max() <= 1e-9
    Xo, _, ito, _, _ = _oracle(A, B, X0, 16, variant=0, maxiter=200, fixed_iters=True)
    assert _errs(res.X, Xo).max() <= TOL


def test_split_streams_match_single_batch(gpu):
    """A 1024-batch runs as concurrent sub-batches (ACE_SPLIT); every realisation's result must
    equal the one it gets in a small batch (no cross-realisation coupling, identical kernels)."""
    import torch
    from ace_amd import infer_admm_batch, synth_problem
    A, B, X0, _ = synth_problem(29, 0, 1024, 256, 32, 32)
    big = infer_admm_batch(A, B, X0, 32, 32, maxiter=60, fixed_iters=True)
    torch.cuda.synchronize()
    Xb = big.X.cpu().numpy()
    for lo in (0, 500, 960):
        sub = infer_admm_batch(A, B[lo:lo + 64].contiguous(), X0[lo:lo + 64].contiguous(), 32, 32, maxiter=60,
                               fixed_iters=True)
        torch.cuda.synchronize()
        assert np.array_equal(sub.X.cpu().numpy(), Xb[lo:lo + 64]), lo
        assert np.array_equal(sub.iters.cpu().numpy(), big.iters.cpu().numpy()[lo:lo + 64])


@pytest.mark.parametrize("msp", ["1", "0"])
@pytest.mark.parametrize("batch", [64, 1024])
def test_unit_path_launches_three_kernels_per_iteration(gpu, monkeypatch, batch, msp):
    """The phase-code r = 1 iteration is gyk_kernel + apply_AH + Z-step: no apply_A, pre, Y-step
    or K Y launch (with and without concurrent sub-batches), one launch of each per iteration and
    sub-batch.  With concurrent sub-batches gyk and the fused apply_AH are one launch (gyf_kernel,
    counted as apply_G) except at the last iteration.  With m-space steps (ACE_MSPACE, default on)
    every iteration, the last included and one batch too, is gyf_kernel + Z-step, and one
    apply_AH launch at the end forms the m-space best iterates (RealState::optsrc 3)."""
    import ctypes as C
    monkeypatch.setenv("ACE_MSPACE", msp)
    import torch
    from ace_amd import infer_admm_batch, synth_problem
    from ace_amd._lib import LIB, KERNEL_CLASSES, check
    A, B, X0, _ = synth_problem(31, 0, batch, 256, 32, 32)
    iters = 20
    infer_admm_batch(A, B, X0, 32, 32, maxiter=iters, fixed_iters=True)   # warm-up (setup caches)
    torch.cuda.synchronize()
    check(LIB.ace_prof_sample(1, 0))
    check(LIB.ace_prof_start(4096))
    infer_admm_batch(A, B, X0, 32, 32, maxiter=iters, fixed_iters=True)
    torch.cuda.synchronize()
    kt = (C.c_double * len(KERNEL_CLASSES))()
    kn = (C.c_int32 * len(KERNEL_CLASSES))()
    check(LIB.ace_prof_stop(kt, kn))
    n = dict(zip(KERNEL_CLASSES, kn))
    subs = 2 if batch >= 512 else 1
    for k in ("apply_A", "pre", "ystep", "apply_K"):
        assert n[k] == 0, (k, n)
    for k in ("apply_G", "zstep"):
        assert n[k] == iters * subs, (k, n)
    if msp == "1":
        assert n["apply_AH"] == 0, n   # (the final opt_X launch runs under the finalize scope)
    else:
        assert n["apply_AH"] == (subs if subs > 1 else iters), n


@pytest.mark.parametrize("a_shared,batch", [(True, 1024), (True, 64), (False, 64)])
def test_lean_zstep_bit_identical(gpu, monkeypatch, a_shared, batch):
    """The steady-state Z-step under the perturbation certificate (zlean_kernel) produces exactly
    what the full one-wave Z-step produces (same element order and sums at 32 antennas); it only
    replaces the Ky Fan certificate by a bound that implies it.  ACE_LEAN=0 runs the full kernel
    every iteration.  Shared (split sub-batches and one batch) and private phase-code codebooks.
    The same Z-step fused into apply_AH's epilogue (ACE_FUSE, shared codebooks) reduces its sums
    in another order: equal to rounding, same iteration counts."""
    import torch
    from ace_amd import infer_admm_batch, synth_problem
    A, B, X0, _ = synth_problem(41, 0, batch, 256, 32, 32, a_shared=a_shared)
    out = {}
    for lean, fuse in (("0", "0"), ("1", "0"), ("1", "1")):
        monkeypatch.setenv("ACE_LEAN", lean)
        monkeypatch.setenv("ACE_FUSE", fuse)
        r = infer_admm_batch(A, B, X0, 32, 32, maxiter=200, fixed_iters=True)
        torch.cuda.synchronize()
        out[lean + fuse] = (r.X.cpu().numpy(), r.Y.cpu().numpy(), r.iters.cpu().numpy())
    for a, b in zip(out["00"], out["10"]):
        assert np.array_equal(a, b)
    assert _errs(out["11"][0], out["00"][0]).max() <= 1e-12
    assert np.array_equal(out["11"][2], out["00"][2])


@pytest.mark.parametrize("batch", [64, 1024])
def test_fused_zstep_convergence_mode(gpu, monkeypatch, batch):
    """Convergence mode through the fused apply_AH Z-step and the lazy dual residual: iteration
    counts and the converged flags equal the oracle's (a sample of the batch)."""
    import torch
    from ace_amd import infer_admm_batch, synth_problem
    A, B, X0, _ = synth_problem(43, 0, batch, 256, 32, 32)
    monkeypatch.setenv("ACE_LEAN", "1")
    monkeypatch.setenv("ACE_FUSE", "1")
    r = infer_admm_batch(A, B, X0, 32, 32, maxiter=500)
    torch.cuda.synchronize()
    idx = [0, batch // 2, batch - 1]
    Ah, Bh, X0h = A.cpu().numpy(), B.cpu().numpy()[idx], X0.cpu().numpy()[idx]
    Xo, _, ito, cvo, _ = _oracle(Ah, Bh, X0h, 32, variant=0, maxiter=500)
    assert _errs(r.X.cpu().numpy()[idx], Xo).max() <= TOL
    assert np.array_equal(r.iters.cpu().numpy()[idx], ito)
    assert np.array_equal(r.converged.cpu().numpy()[idx], cvo)


@pytest.mark.parametrize("fixed", [True, False])
def test_compact_zstep_bit_identical(gpu, monkeypatch, fixed):
    """The compact Z-step (ACE_ZCOMPACT: one wave per 8 realisations, fallbacks in turn) runs the
    same per-realisation code as the one-wave-per-realisation launch: bit-identical results, in
    fixed-iteration and convergence mode (from iteration 3, so the cold start takes its fallback)."""
    import torch
    from ace_amd import infer_admm_batch, synth_problem
    A, B, X0, _ = synth_problem(47, 0, 1024, 256, 32, 32)
    out = {}
    for zc in ("0", "3"):
        monkeypatch.setenv("ACE_ZCOMPACT", zc)
        r = infer_admm_batch(A, B, X0, 32, 32, maxiter=200, fixed_iters=fixed)
        torch.cuda.synchronize()
        out[zc] = (r.X.cpu().numpy(), r.iters.cpu().numpy(), r.status.cpu().numpy())
    for a, b in zip(out["0"], out["3"]):
        assert np.array_equal(a, b)


@pytest.mark.parametrize("fail_it", [None, "40", "200"])
@pytest.mark.parametrize("fixed", [True, False])
@pytest.mark.parametrize("batch,m,tx", [(1024, 256, 32), (64, 256, 32), (600, 121, 16)])
def test_mspace_steps(gpu, monkeypatch, batch, m, tx, fixed, fail_it):
    """m-space steady state (RealState::msp, ACE_MSPACE): Z kept as Z0 + A^H S, the fused pass's
    sums from m-space, no apply_AH pass for settled realisations, the best iterate materialised at
    the end.  Against the memory form (ACE_MSPACE=0): equal to rounding (1e-10 relative), identical
    iteration counts and flags; a sample against the oracle.  ACE_MSP_FAIL_IT forces the bound of
    every m-space iterate to fail at one iteration (the Z-step then materialises Z, Z' and opt_X from
    the implicit form and runs the full step): 40 = mid-solve, 200 = the last iteration."""
    import torch
    from ace_amd import infer_admm_batch, synth_problem
    A, B, X0, _ = synth_problem(59, 0, batch, m, tx, tx)
    out = {}
    for msp in ("0", "1"):
        monkeypatch.setenv("ACE_MSPACE", msp)
        if fail_it and msp == "1":
            monkeypatch.setenv("ACE_MSP_FAIL_IT", fail_it)
        r = infer_admm_batch(A, B, X0, tx, tx, maxiter=200, fixed_iters=fixed)
        torch.cuda.synchronize()
        out[msp] = (r.X.cpu().numpy(), r.Y.cpu().numpy(), r.iters.cpu().numpy(), r.status.cpu().numpy())
        monkeypatch.delenv("ACE_MSP_FAIL_IT", raising=False)
    X0_, Y0_, it0, st0 = out["0"]
    X1, Y1, it1, st1 = out["1"]
    assert np.isfinite(X1).all() and np.isfinite(Y1).all()
    assert _errs(X1, X0_).max() <= 1e-10
    assert _errs(Y1, Y0_).max() <= 1e-10
    assert np.array_equal(it1, it0)
    assert np.array_equal(st1, st0)
    idx = [0, batch // 3, batch - 1]
    Ah, Bh, X0h = A.cpu().numpy(), B.cpu().numpy()[idx], X0.cpu().numpy()[idx]
    Xo, _, ito, _, _ = _oracle(Ah, Bh, X0h, tx, variant=0, maxiter=200, fixed_iters=fixed)
    assert _errs(X1[idx], Xo).max() <= TOL
    assert np.array_equal(it1[idx], ito)


@pytest.mark.parametrize("fixed", [True, False])
def test_mspace_frequent_fallbacks(gpu, monkeypatch, fixed):
    """m-space entry with almost no margin (ACE_MSP_ROOM=1): realisations enter the implicit form
    as soon as the bound holds and many fall back soon after, so the Z-step materialises Z, Z' and
    opt_X (from opt_S, or from an S ping-pong buffer) at many different iterations.  Against the
    memory form: equal to rounding, identical iteration counts and flags."""
    import torch
    from ace_amd import infer_admm_batch, synth_problem
    A, B, X0, _ = synth_problem(67, 0, 512, 256, 32, 32)
    out = {}
    for msp in ("0", "1"):
        monkeypatch.setenv("ACE_MSPACE", msp)
        monkeypatch.setenv("ACE_MSP_ROOM", "1")
        r = infer_admm_batch(A, B, X0, 32, 32, maxiter=200, fixed_iters=fixed)
        torch.cuda.synchronize()
        out[msp] = (r.X.cpu().numpy(), r.Y.cpu().numpy(), r.iters.cpu().numpy(), r.status.cpu().numpy())
    assert np.isfinite(out["1"][0]).all()
    assert _errs(out["1"][0], out["0"][0]).max() <= 1e-10
    assert _errs(out["1"][1], out["0"][1]).max() <= 1e-10
    assert np.array_equal(out["1"][2], out["0"][2])
    assert np.array_equal(out["1"][3], out["0"][3])


@pytest.mark.parametrize("fixed", [True, False])
def test_gyf_control_bit_identical(gpu, monkeypatch, fixed):
    """The certificate and iteration control of m-space iterates run inside gyf_kernel (default) or
    in the Z-step launch (ACE_GYF_CTL=0): the same code on the same state, bit-identical results."""
    import torch
    from ace_amd import infer_admm_batch, synth_problem
    A, B, X0, _ = synth_problem(61, 0, 1024, 256, 32, 32)
    out = {}
    for c in ("1", "0"):
        monkeypatch.setenv("ACE_GYF_CTL", c)
        r = infer_admm_batch(A, B, X0, 32, 32, maxiter=200, fixed_iters=fixed)
        torch.cuda.synchronize()
        out[c] = (r.X.cpu().numpy(), r.Y.cpu().numpy(), r.iters.cpu().numpy(), r.status.cpu().numpy())
    for a, b in zip(out["1"], out["0"]):
        assert np.array_equal(a, b)


@pytest.mark.parametrize("batch,m,tx", [(1000, 256, 32), (1024, 121, 16), (1040, 243, 32)])
def test_gyf_ragged_batches_and_sizes(gpu, batch, m, tx):
    """gyf_kernel (gyk + fused apply_AH, concurrent sub-batches) on ragged sub-batches (not a
    multiple of the 16-realisation work-group), m not a multiple of the tiles (the T rows then too
    small to hold the Z-step's partial sums), 16 antennas: a sample matches the oracle and its own
    result in a small batch (batch invariance)."""
    import torch
    from ace_amd import infer_admm_batch, synth_problem
    A, B, X0, _ = synth_problem(53, 0, batch, m, tx, tx)
    r = infer_admm_batch(A, B, X0, tx, tx, maxiter=200, fixed_iters=True)
    torch.cuda.synchronize()
    X = r.X.cpu().numpy()
    idx = [0, batch // 2 + 7, batch - 1]
    Ah, Bh, X0h = A.cpu().numpy(), B.cpu().numpy()[idx], X0.cpu().numpy()[idx]
    Xo, _, _, _, _ = _oracle(Ah, Bh, X0h, tx, variant=0, maxiter=200, fixed_iters=True)
    assert _errs(X[idx], Xo).max() <= TOL
    small = infer_admm_batch(A, B[batch - 16:].contiguous(), X0[batch - 16:].contiguous(), tx, tx, maxiter=200,
                             fixed_iters=True)
    torch.cuda.synchronize()
    assert _errs(small.X.cpu().numpy(), X[batch - 16:]).max() <= 1e-12


def test_nuclear_config3_split_path_vs_oracle(gpu):
    """Config 3's benchmarked path: A2nuclear at 32 antennas, m = 256, a 4096-realisation batch, so
    the solve runs as concurrent sub-batches (admm_iterate_split: gyk_kernel, apply_AH, one-wave
    Z-step with the soft threshold of inferLowRank_Nuclear.m:411-419).  A sample against the C oracle
    on the horizon where the oracle is stable against itself (60 iterations; see
    test_oracle.py::test_nuclear_refinement_is_rounding_chaotic)."""
    import torch
    from ace_amd import infer_admm_batch, synth_problem
    A, B, X0, _ = synth_problem(71, 0, 4096, 256, 32, 32)
    r = infer_admm_batch(A, B, X0, 32, 32, variant="A2nuclear", maxiter=60, fixed_iters=True)
    torch.cuda.synchronize()
    idx = [0, 1500, 2048, 4095]
    X = r.X.cpu().numpy()[idx]
    Ah, Bh, X0h = A.cpu().numpy(), B.cpu().numpy()[idx], X0.cpu().numpy()[idx]
    Xo, _, ito, _, _ = _oracle(Ah, Bh, X0h, 32, variant=1, maxiter=60, fixed_iters=True)
    assert (r.iters.cpu().numpy() == 60).all() and (ito == 60).all()
    assert _errs(X, Xo).max() <= 1e-8


def test_nuclear_config3_split_path_batch_invariance_200(gpu):
    """The same benchmarked path over the full 200-iteration horizon: every sampled realisation
    is bit-identical to its result in a small batch (no sub-batch split, the single-stream loop of
    admm_run), so the benchmarked output is the verified small-batch output."""
    import torch
    from ace_amd import infer_admm_batch, synth_problem
    A, B, X0, _ = synth_problem(73, 0, 4096, 256, 32, 32)
    big = infer_admm_batch(A, B, X0, 32, 32, variant="A2nuclear", maxiter=200, fixed_iters=True)
    torch.cuda.synchronize()
    Xb, Yb, itb = big.X.cpu().numpy(), big.Y.cpu().numpy(), big.iters.cpu().numpy()
    assert np.isfinite(Xb).all() and (itb == 200).all()
    for lo in (0, 2040, 4032):
        sub = infer_admm_batch(A, B[lo:lo + 64].contiguous(), X0[lo:lo + 64].contiguous(), 32, 32,
                               variant="A2nuclear", maxiter=200, fixed_iters=True)
        torch.cuda.synchronize()
        assert np.array_equal(sub.X.cpu().numpy(), Xb[lo:lo + 64]), lo
        assert np.array_equal(sub.Y.cpu().numpy(), Yb[lo:lo + 64]), lo
    # and the small batch against the oracle on its stable horizon
    one = infer_admm_batch(A, B[:4].contiguous(), X0[:4].contiguous(), 32, 32, variant="A2nuclear", maxiter=60,
                           fixed_iters=True)
    torch.cuda.synchronize()
    Xo, _, _, _, _ = _oracle(A.cpu().numpy(), B[:4].cpu().numpy(), X0[:4].cpu().numpy(), 32, variant=1,
                             maxiter=60, fixed_iters=True)
    assert _errs(one.X.cpu().numpy(), Xo).max() <= 1e-8


@pytest.mark.parametrize("tx,m,batch,fixed", [(32, 256, 1024, True), (16, 64, 67, True), (16, 121, 40, False)])
def test_nuclear_mspace_matches_nspace(gpu, monkeypatch, tx, m, batch, fixed):
    """A2nuclear r = 1 iterated in m-space (ace_nucmsp.hip: Z, N as (X_init coefficient, m-vector)
    pairs, one launch per iteration) against the n-space path (ACE_NUC_MSP=0: gyk_kernel, apply_AH,
    the one-wave Z-step) and the C oracle, on the horizon where the oracle is stable against itself
    (60 iterations); convergence mode with its iteration counts and flags too (ragged m, batch)."""
    import torch
    from ace_amd import infer_admm_batch, synth_problem
    A, B, X0, _ = synth_problem(79, 0, batch, m, tx, tx)
    out = {}
    for ms in ("1", "0"):
        monkeypatch.setenv("ACE_NUC_MSP", ms)
        r = infer_admm_batch(A, B, X0, tx, tx, variant="A2nuclear", maxiter=60, fixed_iters=fixed)
        torch.cuda.synchronize()
        out[ms] = (r.X.cpu().numpy(), r.Y.cpu().numpy(), r.iters.cpu().numpy(), r.status.cpu().numpy(),
                   r.mu.cpu().numpy())
    X1, Y1, it1, st1, mu1 = out["1"]
    X0_, Y0_, it0, st0, mu0 = out["0"]
    assert np.isfinite(X1).all() and np.isfinite(Y1).all()
    e = _errs(X1, X0_)
    # the two rounding sequences agree closely for most realisations ...
    assert np.median(e) <= 1e-9 and _errs(Y1, Y0_).max() <= 1e-6
    assert np.array_equal(it1, it0) and np.array_equal(st1, st0) and np.array_equal(mu1, mu0)
    # ... and where they differ most, the reference itself moves as much under a 1e-15 change of
    # its input (the nuclear refinement amplifies rounding ~1.2x per iteration): the
    # oracle's own divergence on those realisations bounds the disagreement
    idx = sorted(set([0, batch - 1] + list(np.argsort(e)[-3:])))
    Ah, Bh, X0h = A.cpu().numpy(), B.cpu().numpy()[idx], X0.cpu().numpy()[idx]
    Xo, _, ito, cvo, _ = _oracle(Ah, Bh, X0h, tx, variant=1, maxiter=60, fixed_iters=fixed)
    Xp, _, _, _, _ = _oracle(Ah, Bh * (1 + 1e-15), X0h, tx, variant=1, maxiter=60, fixed_iters=fixed)
    noise = _errs(Xo, Xp)
    for k in range(len(idx)):
        bound = max(1e-8, 100 * noise[k])
        assert O.unit_phase_aligned_rel_err(X1[idx[k]], Xo[k]) <= bound, (idx[k], noise[k])
        assert O.unit_phase_aligned_rel_err(X0_[idx[k]], Xo[k]) <= bound, (idx[k], noise[k])
    assert np.array_equal(it1[idx], ito)
