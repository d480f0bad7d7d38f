"""GPU parity of the refinement the reference actually runs, at the benchmarked scale.

inferLowRankV4_multi refines X_max of its restarts with InferADMM at r = 1 (:92/:100), passing the
LAST restart's use_rank_one (:73-77): the [1]/[0.95] rank profile (:448-450) whenever that restart's
first quality was below 0.6.  A Monte-Carlo batch of calls therefore refines with mixed profiles.
These tests drive that through the C-ABI's per-realisation flags (ace_admm_cfg::rank_one) at 32-ant,
m = 256, batch >= 1024 -- the split sub-batches, the fused gyf kernel and the m-space runs -- and
check a sample against the C oracle (oracle/ace_oracle.c, the reference's U-form algorithm):
X within 1e-5 after global-phase alignment (Evaluation_H.m:81-82), iteration counts equal.  They
also run the whole pipeline at batch 256 (the int8 r-column stages) against the numpy oracle's
outputs for a sample (tests/golden/pipeline_32ant_m256_b256.npz, make_pipeline_scale_golden.py) with
one partition set for the batch and with every realisation's own partitions, and InferADMM at
r = 20 (the stages :258 / :270) through the public solver API.
"""
import hashlib
import math
import pathlib

import numpy as np
import pytest

import ace_oracle as O
import ace_oracle_c as OC

pytestmark = pytest.mark.gpu

TOL = 1e-5
GOLD = pathlib.Path(__file__).resolve().parent / "golden"


def _errs(Xg, Xo):
    return np.array([O.unit_phase_aligned_rel_err(Xg[b], Xo[b]) for b in range(Xg.shape[0])])


def _oracle_mixed(A, B, X0, flags, **kw):
    """C oracle per flag group (its use_rank_one is one flag per call)."""
    U = OC.make_U(A)[None]
    batch, n = X0.shape
    X = np.empty((batch, n), np.complex128)
    it = np.empty(batch, np.int32)
    for f in (False, True):
        idx = np.flatnonzero(flags == f)
        if idx.size:
            Xo, _, ito, _, _ = OC.infer_admm_r1_batch(A[None], U, B[idx], X0[idx], 32, 32, variant=0,
                                                      use_rank_one=f, **kw)
            X[idx], it[idx] = Xo, ito
    return X, it


def _sample(flags, k=4):
    """k realisations of each flag value (fewer if the batch has fewer)."""
    a = np.flatnonzero(flags)
    b = np.flatnonzero(~flags)
    pick = lambda v: v[np.linspace(0, len(v) - 1, min(k, len(v))).astype(int)] if len(v) else v  # noqa: E731
    return np.sort(np.concatenate([pick(a), pick(b)]))


def test_refinement_mixed_flags_fixed_1024(gpu):
    """Mixed per-realisation profiles at the unit's shape, 200 fixed iterations (the bench's mode):
    each realisation's result is bit-identical to a batch-wide run with its own flag (the flags
    select the profile per realisation inside every kernel), and a sample matches the C oracle."""
    import torch
    from ace_amd import infer_admm_batch, synth_problem
    A, B, X0, _ = synth_problem(4111, 0, 1024, 256, 32, 32)
    flags = (np.arange(1024) % 3) == 0
    kw = dict(maxiter=200, fixed_iters=True)
    mixed = infer_admm_batch(A, B, X0, 32, 32, use_rank_one=torch.from_numpy(flags).cuda(), **kw)
    Xm = mixed.X.cpu().numpy()
    its = mixed.iters.cpu().numpy()
    all0 = infer_admm_batch(A, B, X0, 32, 32, use_rank_one=False, **kw).X.cpu().numpy()
    all1 = infer_admm_batch(A, B, X0, 32, 32, use_rank_one=True, **kw).X.cpu().numpy()
    assert (its == 200).all()
    assert np.array_equal(Xm[flags], all1[flags])
    assert np.array_equal(Xm[~flags], all0[~flags])
    idx = _sample(flags)
    Xo, ito = _oracle_mixed(A[0].cpu().numpy(), B.cpu().numpy()[idx], X0.cpu().numpy()[idx], flags[idx], **kw)
    e = _errs(Xm[idx], Xo)
    assert e.max() <= TOL, e


def test_refinement_of_pipeline_xmax_convergence_1024(gpu):
    """The reference's refinement on its own input: X0 = X_max of the 3-restart pipeline and the
    last restart's use_rank_one (ACE_ST_RANK_ONE of ace_pipeline_solve_batch with
    stop_before_refine), 32-ant, m = 256, batch 1024, convergence mode (maxiter 500): a sample of
    both profiles against the C oracle, iteration counts equal."""
    import torch
    from ace_amd import infer_admm_batch, infer_low_rank_pipeline_batch, synth_problem, draw_partitions
    A, B, _, _ = synth_problem(4127, 0, 1024, 256, 32, 32)
    tr = draw_partitions(np.random.default_rng(4127), 256, 3)
    pr = infer_low_rank_pipeline_batch(A, B, 32, 32, tr, stop_before_refine=True)
    flags = pr.rank_one.cpu().numpy()
    # at m = n / 4 most first-pass qualities are below 0.6 (magnitude-only recovery is underdetermined
    # there), so most realisations refine with the rank-one profile
    assert flags.sum() > 0, flags.sum()
    X0 = pr.X.contiguous()
    res = infer_admm_batch(A, B, X0, 32, 32, use_rank_one=pr.rank_one, maxiter=500)
    torch.cuda.synchronize()
    idx = _sample(flags)
    Xo, ito = _oracle_mixed(A[0].cpu().numpy(), B.cpu().numpy()[idx], X0.cpu().numpy()[idx], flags[idx],
                            maxiter=500)
    its = res.iters.cpu().numpy()[idx]
    assert np.array_equal(its, ito), (its, ito)
    e = _errs(res.X.cpu().numpy()[idx], Xo)
    assert e.max() <= TOL, e


def _gold_inputs(g):
    import sys
    sys.path.insert(0, str(GOLD))
    import make_pipeline_scale_golden as MG
    A, B, shared, each = MG.inputs()
    sha = lambda a: hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()  # noqa: E731
    assert sha(B) == str(g["sha_B"]) and sha(shared) == str(g["sha_shared"]) and sha(each) == str(g["sha_each"]), \
        "the synthetic generator drifted from the golden vectors' inputs"
    return A, B, shared, each


@pytest.mark.parametrize("stop", [False, True])
def test_pipeline_batch256_shared_partition_golden(gpu, stop):
    """The whole pipeline at batch 256 (32-ant, m = 256: int8 r-column stages over 5120 vectors,
    the split / gyf / m-space refinement with per-realisation profiles) against the numpy oracle
    on a sample of 8: stage iteration counts, last-restart quality, rollback and the refinement's
    use_rank_one equal, X (and X_max with stop_before_refine) within 1e-5."""
    import torch
    from ace_amd import infer_low_rank_pipeline_batch
    g = np.load(GOLD / "pipeline_32ant_m256_b256.npz")
    A, B, shared, _ = _gold_inputs(g)
    s = g["sample"]
    pr = infer_low_rank_pipeline_batch(torch.from_numpy(A).cuda(), torch.from_numpy(B).cuda(), 32, 32, shared,
                                       stop_before_refine=stop)
    its = pr.stage_iters.cpu().numpy()[s]
    gi = g["shared_stage_iters"].copy()
    if stop:
        gi[:, -1] = 0
    assert np.array_equal(its, gi), (its, gi)
    np.testing.assert_allclose(pr.quality.cpu().numpy()[s], g["shared_quality"], rtol=0, atol=1e-9)
    assert np.array_equal(pr.rank_one.cpu().numpy()[s], g["shared_rank_one"])
    X = pr.X.cpu().numpy()[s]
    ref = g["shared_X_max"] if stop else g["shared_X"]
    e = np.array([O.phase_aligned_rel_err(X[k], ref[k]) for k in range(len(s))])
    assert e.max() <= TOL, e
    if not stop:
        assert np.array_equal(pr.rolled_back.cpu().numpy()[s], g["shared_rolled_back"])


@pytest.mark.parametrize("batch,row_mode", [(2, True), (2, False), (13, True), (13, False)])
def test_infer_admm_r20_public_api(gpu, batch, row_mode):
    """InferADMM at r = 20 through the solver C-ABI (ace_admm_cfg::r): the row-scaled stage (:258,
    scale_by_row, n x r output) and the per-column stage (:270, best column), on the f64 applies
    (batch 2 x 20 = 40 vectors) and the int8 digit-plane applies (13 x 20 = 260 >= 256), against the
    numpy oracle in convergence mode: X within 1e-5, iteration counts equal."""
    from ace_amd import infer_admm_host, synth
    tx, m, r = 16, 64, 20
    A, B, _, _ = synth.problem(4133, 0, batch, m, tx, tx)
    rng = np.random.default_rng(4133)
    X0 = (rng.standard_normal((batch, r, tx * tx)) + 1j * rng.standard_normal((batch, r, tx * tx))) / 16
    res = infer_admm_host(A, B, X0, tx, tx, scale_by_row=row_mode, maxiter=300)
    U = O.make_U(A[0])
    for b in range(batch):
        o = O.infer_admm(A[0], B[b], X0[b].T, row_mode, False, tx, tx, maxiter=300, U=U)
        assert res.iters[b] == o.iters, (b, res.iters[b], o.iters)
        Xg = res.X[b].T                       # [R][n] -> n x R
        assert Xg.shape == o.X.shape
        e = np.linalg.norm(Xg - o.X) / np.linalg.norm(o.X)
        assert e <= TOL, (b, e)


def test_infer_admm_matlab_signature_r20(gpu):
    """InferADMM(A, B, X0, scale_by_row, use_rank_one, tx, rx) with an n x 20 X0 (MATLAB shapes)."""
    from ace_amd import InferADMM, synth
    A, B, _, _ = synth.problem(4139, 0, 1, 64, 16, 16)
    rng = np.random.default_rng(4139)
    X0 = rng.standard_normal((256, 20)) + 1j * rng.standard_normal((256, 20))
    X, Y, _ = InferADMM(A[0], B[0], X0, True, True, 16, 16, maxiter=120)
    o = O.infer_admm(A[0], B[0], X0, True, True, 16, 16, maxiter=120)
    assert X.shape == (256, 20) and Y.shape == (64, 20)
    assert np.linalg.norm(X - o.X) / np.linalg.norm(o.X) <= TOL
    X1, Y1, _ = InferADMM(A[0], B[0], X0, False, False, 16, 16, maxiter=120)
    o1 = O.infer_admm(A[0], B[0], X0, False, False, 16, 16, maxiter=120)
    assert X1.shape == (256, 1) and Y1.shape == (64, 1)
    assert np.linalg.norm(X1 - o1.X) / np.linalg.norm(o1.X) <= TOL


def test_pipeline_batch256_per_realisation_partitions_golden(gpu):
    """SURVEY.md §8(b)'s train_idx [batch][restarts][m_t]: 256 realisations, each with its own three
    partitions (randsample inside every call, inferLowRankV4_multi.m:48), in ONE batch: the stages run
    on the full A in m-space with (I + K_t)^{-1} from the full G by the Schur identity
    (launch_part_gfix).  Against the numpy oracle run per realisation on its own partitions (sample of
    8): stage iteration counts, quality, rollback and the refinement's profile equal, X within 1e-5."""
    import torch
    from ace_amd import infer_low_rank_pipeline_batch
    g = np.load(GOLD / "pipeline_32ant_m256_b256.npz")
    A, B, _, each = _gold_inputs(g)
    s = g["sample"]
    pr = infer_low_rank_pipeline_batch(torch.from_numpy(A).cuda(), torch.from_numpy(B).cuda(), 32, 32, each)
    its = pr.stage_iters.cpu().numpy()[s]
    assert np.array_equal(its, g["each_stage_iters"]), (its, g["each_stage_iters"])
    np.testing.assert_allclose(pr.quality.cpu().numpy()[s], g["each_quality"], rtol=0, atol=1e-9)
    assert np.array_equal(pr.rank_one.cpu().numpy()[s], g["each_rank_one"])
    assert np.array_equal(pr.rolled_back.cpu().numpy()[s], g["each_rolled_back"])
    X = pr.X.cpu().numpy()[s]
    e = np.array([O.phase_aligned_rel_err(X[k], g["each_X"][k]) for k in range(len(s))])
    assert e.max() <= TOL, e


def test_per_realisation_partitions_match_one_by_one(gpu):
    """Per-realisation partitions in one batch (m-space stages, Schur-form G_t) against each realisation
    solved alone on its own partition (the shared-A_t path with K_t, G_t formed directly): 16-ant,
    m = 64 (f64 applies) and 32-ant, m = 256, batch 16 (int8 digit-plane applies, 320 vectors): equal
    stage iteration counts and rollback flags, X within 1e-8 (different summation orders only)."""
    from ace_amd import infer_low_rank_pipeline_host, synth, draw_partitions
    for ant, m, batch, maxiter in ((16, 64, 5, 500), (32, 256, 16, 150)):
        A, B, _, _ = synth.problem(4151 + ant, 0, batch, m, ant, ant)
        tr = draw_partitions(np.random.default_rng(4151 + ant), m, 3, batch=batch)
        full = infer_low_rank_pipeline_host(A[0], B, ant, ant, tr, maxiter=maxiter)
        for b in range(batch):
            one = infer_low_rank_pipeline_host(A[0], B[b:b + 1], ant, ant, tr[b], maxiter=maxiter)
            assert np.array_equal(one.stage_iters[0], full.stage_iters[b]), (ant, b, one.stage_iters, full.stage_iters[b])
            assert one.rolled_back[0] == full.rolled_back[b] and one.rank_one[0] == full.rank_one[b]
            assert O.phase_aligned_rel_err(full.X[b], one.X[0]) <= 1e-8, (ant, b)
            assert abs(one.quality[0] - full.quality[b]) <= 1e-10


def test_partitions_drawn_by_the_build(gpu):
    """train_idx = NULL: per-realisation partitions from the build's counter RNG (train_seed; stream
    b * restarts + restart), the same as passing those draws explicitly."""
    import ctypes as C
    from ace_amd import infer_low_rank_pipeline_host, synth, engine
    from ace_amd._lib import LIB, check, pipeline_cfg, ACE_TRAIN_PER_REALISATION
    A, B, _, _ = synth.problem(4157, 0, 3, 64, 16, 16)
    tr = np.stack([np.stack([engine.randperm(77, b * 3 + i, 64, 60) for i in range(3)]) for b in range(3)])
    ref = infer_low_rank_pipeline_host(A[0], B, 16, 16, tr)
    cfg = pipeline_cfg(0, train_layout=ACE_TRAIN_PER_REALISATION, train_seed=77)
    X = np.empty((3, 256), np.complex128)
    Y = np.empty((3, 64), np.complex128)
    its = np.empty((3, 13), np.int32)
    dp = lambda a: a.ctypes.data_as(C.POINTER(C.c_double))  # noqa: E731
    check(LIB.ace_pipeline_solve_host(C.byref(cfg), 3, 64, 256, 16, 16, dp(A[0].view(np.float64)),
                                      dp(np.ascontiguousarray(B)), None, dp(X.view(np.float64)), dp(Y.view(np.float64)),
                                      None, its.ctypes.data_as(C.POINTER(C.c_int32)), None))
    assert np.array_equal(X, ref.X) and np.array_equal(its, ref.stage_iters)


def test_null_partitions_need_the_per_realisation_layout(gpu):
    """train_idx = NULL with the default (shared) layout is an argument error, not a workspace error:
    ace_pipeline_workspace_size sizes the per-realisation form only for ACE_TRAIN_PER_REALISATION."""
    import ctypes as C
    from ace_amd import synth
    from ace_amd._lib import LIB, pipeline_cfg, ACE_ERR_ARG
    A, B, _, _ = synth.problem(4159, 0, 3, 64, 16, 16)
    cfg = pipeline_cfg(0, train_seed=77)
    X = np.empty((3, 256), np.complex128)
    Y = np.empty((3, 64), np.complex128)
    dp = lambda a: a.ctypes.data_as(C.POINTER(C.c_double))  # noqa: E731
    rc = LIB.ace_pipeline_solve_host(C.byref(cfg), 3, 64, 256, 16, 16, dp(A[0].view(np.float64)),
                                     dp(np.ascontiguousarray(B)), None, dp(X.view(np.float64)),
                                     dp(Y.view(np.float64)), None, None, None)
    assert rc == ACE_ERR_ARG and b"ACE_TRAIN_PER_REALISATION" in LIB.ace_last_error()


def test_partitions_beyond_the_schur_block_run_per_group(gpu):
    """Per-realisation partitions with m - m_t > 96 test rows (cc_frac 0.5 at m = 256: 128) are beyond the
    per-realisation form's LDS inverse; the Python mirror then solves each group of realisations that
    share their partitions as one shared-layout call.  Against one call per realisation (bit-identical:
    the same calls), with two realisations sharing a partition set (one group of 2)."""
    from ace_amd import infer_low_rank_pipeline_host, infer_low_rank_pipeline_batch, synth, draw_partitions
    import torch
    A, B, _, _ = synth.problem(4163, 0, 3, 256, 16, 16)
    tr = draw_partitions(np.random.default_rng(4163), 256, 3, cc_frac=0.5, batch=3)
    tr[2] = tr[0]
    kw = dict(cc_frac=0.5, maxiter=120)
    full = infer_low_rank_pipeline_host(A[0], B, 16, 16, tr, **kw)
    for b in range(3):
        one = infer_low_rank_pipeline_host(A[0], B[b:b + 1], 16, 16, tr[b], **kw)
        assert np.array_equal(one.stage_iters[0], full.stage_iters[b]), b
        assert O.phase_aligned_rel_err(full.X[b], one.X[0]) <= 1e-12, b
    dev = torch.device("cuda:0")
    bt = infer_low_rank_pipeline_batch(torch.as_tensor(A[0], device=dev), torch.as_tensor(B, device=dev), 16, 16,
                                       tr, **kw)
    assert np.array_equal(bt.stage_iters.cpu().numpy(), full.stage_iters)
    assert max(O.phase_aligned_rel_err(bt.X.cpu().numpy()[b], full.X[b]) for b in range(3)) <= 1e-12


@pytest.mark.parametrize("tx,m,fixed", [(32, 256, True), (32, 256, False), (16, 64, False)])
def test_rank_one_top_eigenpair_matches_jacobi(gpu, monkeypatch, tx, m, fixed):
    """The rank-one profile's Z-step needs only (lambda_1, u_1) (every other eigenvalue takes one scale,
    inferLowRankV4_multi.m:469-484): the one-wave Z-step finds them by Lanczos with a certified residual
    and top-ness (r1_top) instead of the full Jacobi eigensolver.  Against the Jacobi path
    (ACE_R1_LANCZOS=0) on the reference's refinement input (X_max of the pipeline, its own flags): equal
    iteration counts, X within 1e-10; a sample against the C oracle within 1e-5."""
    import torch
    from ace_amd import infer_admm_batch, infer_low_rank_pipeline_batch, synth_problem, draw_partitions
    batch = 512 if tx == 32 else 256
    A, B, _, _ = synth_problem(4211 + tx, 0, batch, m, tx, tx)
    tr = draw_partitions(np.random.default_rng(4211), m, 3, batch=batch)
    pr = infer_low_rank_pipeline_batch(A, B, tx, tx, tr, stop_before_refine=True)
    flags = torch.ones(batch, dtype=torch.uint8, device=A.device)
    X0 = pr.X.contiguous()
    kw = dict(maxiter=200 if fixed else 500, fixed_iters=fixed, use_rank_one=flags)
    lz = infer_admm_batch(A, B, X0, tx, tx, **kw)
    Xl, il = lz.X.cpu().numpy(), lz.iters.cpu().numpy()
    monkeypatch.setenv("ACE_R1_LANCZOS", "0")
    jc = infer_admm_batch(A, B, X0, tx, tx, **kw)
    Xj, ij = jc.X.cpu().numpy(), jc.iters.cpu().numpy()
    assert np.array_equal(il, ij), (il[il != ij][:8], ij[il != ij][:8])
    e = _errs(Xl, Xj)
    assert np.median(e) <= 1e-12 and e.max() <= 1e-10, (np.median(e), e.max())
    idx = np.arange(0, batch, batch // 4)
    U = OC.make_U(A[0].cpu().numpy())[None]
    Xo, _, ito, _, _ = OC.infer_admm_r1_batch(A[0].cpu().numpy()[None], U, B.cpu().numpy()[idx], X0.cpu().numpy()[idx],
                                              tx, tx, variant=0, use_rank_one=True, maxiter=kw["maxiter"],
                                              fixed_iters=fixed)
    assert np.array_equal(il[idx], ito), (il[idx], ito)
    assert _errs(Xl[idx], Xo).max() <= TOL
