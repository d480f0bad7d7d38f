"""GPU parity of configs[4]'s workload: A2nuclear on the 32-antenna multiresolution codebook
(ace_amd.synth.multires_*: kron(tx, rx) rows with phases per antenna group, the layout the
reference's 16-antenna multiresolution codebook has -- tests/test_multires.py), M = 256 rows drawn
within the tier ..._multiresolution.m:137-144 selects, a batch large enough for the concurrent
sub-batch path bench.py --mode config5 runs.

The rows are phase codes, so the solve runs the exact int8 applies (ace_amd.path_counts).  Parity:
a sample against the C oracle (U = inv(A'A + I), inferLowRank_Nuclear.m:411-419 soft threshold) on
the horizon where the oracle is stable against itself, and every sampled realisation of the
200-iteration benchmark horizon bit-identical to its result in a small batch.  The tier-0 rows span
only 64 dimensions (8 tx x 8 rx antenna groups), and the nuclear refinement on them is
rounding-chaotic sooner than on the random codebook: the C oracle against ITSELF with B scaled by
1 + 1e-15 moves 4.6e-11 at 20 iterations, 3.2e-10 at 30, 1.4e-6 at 40 and 5.3e-5 at 60 (random
codebook: 4.7e-10 at 60), so parity is asserted at 30 iterations."""
import numpy as np
import pytest

import ace_oracle as O
import ace_oracle_c as OC

pytestmark = pytest.mark.gpu


def _workload(batch, seed=58659179):
    import torch
    from ace_amd import synth, synth_problem
    rows, tier = synth.multires_rows(seed, 32, 256)
    Ah = synth.multires_codebook(seed, 32, rows)
    A = torch.from_numpy(Ah[None]).cuda()
    A, B, X0, _ = synth_problem(seed, 0, batch, 256, 32, 32, A=A)
    return A, B, X0, tier


def _errs(Xg, Xo):
    return np.array([O.unit_phase_aligned_rel_err(Xg[b], Xo[b]) for b in range(Xg.shape[0])])


def test_config5_unit_vs_oracle(gpu):
    import torch
    from ace_amd import infer_admm_batch, path_counts
    A, B, X0, tier = _workload(2048)
    assert tier == 0
    path_counts(reset=True)
    r = infer_admm_batch(A, B, X0, 32, 32, variant="A2nuclear", maxiter=30, fixed_iters=True)
    torch.cuda.synchronize()
    assert path_counts(reset=True)["int8_shared"] == 1
    idx = [0, 777, 1024, 2047]
    Ah = A.cpu().numpy()
    U = OC.make_U(Ah[0])[None]
    Xo, _, ito, _, _ = OC.infer_admm_r1_batch(Ah, U, B.cpu().numpy()[idx], X0.cpu().numpy()[idx], 32, 32, variant=1,
                                              maxiter=30, fixed_iters=True)
    assert (ito == 30).all()
    assert _errs(r.X.cpu().numpy()[idx], Xo).max() <= 1e-8


def test_config5_batch_invariance_200(gpu):
    import torch
    from ace_amd import infer_admm_batch
    A, B, X0, _ = _workload(4096)
    big = infer_admm_batch(A, B, X0, 32, 32, variant="A2nuclear", maxiter=200, fixed_iters=True)
    torch.cuda.synchronize()
    Xb = big.X.cpu().numpy()
    assert np.isfinite(Xb).all() and (big.iters.cpu().numpy() == 200).all()
    for lo in (0, 3000, 4080):
        sub = infer_admm_batch(A, B[lo:lo + 16].contiguous(), X0[lo:lo + 16].contiguous(), 32, 32,
                               variant="A2nuclear", maxiter=200, fixed_iters=True)
        torch.cuda.synchronize()
        assert np.array_equal(sub.X.cpu().numpy(), Xb[lo:lo + 16]), lo
