#!/usr/bin/env python3
"""Throughput benchmark: channel recoveries/s of the 2ACE ADMM hot path on MI355X.

Workload (BASELINE.json configs[1]): 32-antenna (tx = rx = 32,
n = 1024) channels, m = 256 random-codebook RSS measurements, A2only ADMM.
One recovery = one InferADMM refinement solve (inferLowRankV4_multi.m:281-386
called at :92 -- r = 1, scale_by_row, mu0 = 1e-3, rho = 1.03) with exactly 200
iterations (the convergence test is evaluated every iteration; early exit off).
A step = one batch of 4096 recoveries per GPU sharing one codebook (regime S),
including the per-batch setup (K = A A^H, (I+K)^-1); inputs are synthetic
(Generate_Channel / Random_Phase_State / Generate_Measurement semantics) and
already resident in HBM when the timed region starts.  With N GPUs each rank
solves its own 4096 realisations (weak scaling) and the recovered channels are
gathered to rank 0 over RCCL inside the timed region.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]

``--mode pipeline`` measures a different, separately named metric: full
inferLowRankV4_multi recoveries/s (3 restarts of spectral init + two r = 20 ADMM stages
+ rank-one retries, then the r = 1 refinement; convergence mode, up to 500 iterations
per stage), one partition set per batch.  It is never reported as the unit metric.
"""
from __future__ import annotations

import argparse
import json
import os
import pathlib
import sys
import time

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "2ace-mmwave-channel-estimation_amd"))

METRIC = "channel recoveries/sec (32-ant, 256 RSS meas, 200 ADMM iters) @1/2/4/8 GPU"
PEAK_FP64_TFLOPS = 78.6   # MI355X FP64 matrix (= FP64 vector) dense peak, spec
PEAK_HBM_GBS = 8000.0     # MI355X HBM3E spec
PEAK_I8_TOPS = 5000.0     # MI355X int8 matrix dense peak, spec (2x the BF16 rate per clock)
PROF_STRIDE = 7           # unit mode: kernel events on every 7th launch of each class (about 86 samples per
                          # class and stream over 3 steps; 200 mod 7 != 0, so the sampled iteration indices
                          # drift over the steps; the event pairs cost < 1 % of the throughput)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=4096, help="recoveries per GPU per step")
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--variant", default="A2only", choices=["A2only", "A2nuclear"])
    ap.add_argument("--private", action="store_true", help="private codebook per realisation (regime P)")
    ap.add_argument("--tx", type=int, default=32)
    ap.add_argument("--m", type=int, default=256)
    ap.add_argument("--seed", type=int, default=58659179)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-regime-p", action="store_true", help="unit mode: skip the regime-P measurement")
    ap.add_argument("--cpu-recoveries", type=int, default=0, help="CPU sample size (0 = auto)")
    ap.add_argument("--no-prof", action="store_true", help="disable live per-kernel event timing")
    ap.add_argument("--mode", default="unit", choices=["unit", "pipeline", "phaselift", "beamformer"])
    return ap.parse_args()


PIPE_METRIC = "pipeline recoveries/sec (inferLowRankV4_multi, 32-ant, 256 RSS meas, convergence mode)"


def bench_pipeline(args, dev, rank, world):
    """Full-pipeline throughput (separate metric): one batch per step, shared partitions."""
    import torch
    import ace_amd
    from ace_amd import infer_low_rank_pipeline_batch, synth_problem, draw_partitions
    from ace_amd._lib import LIB, KERNEL_CLASSES, check
    import ctypes as C
    tx, m, bsz = args.tx, args.m, args.batch
    restarts = 3 if args.variant == "A2only" else 1
    A, B, _, H = synth_problem(args.seed, rank * bsz, bsz, m, tx, tx, device=dev)
    tr = draw_partitions(np.random.default_rng(args.seed), m, restarts)
    ws = ace_amd.solver.Workspace()
    res = None

    def step():
        nonlocal res
        res = infer_low_rank_pipeline_batch(A, B, tx, tx, tr, variant=args.variant, workspace=ws)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if not args.no_prof:
        check(LIB.ace_prof_start(200000))
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kt = (C.c_double * 10)()
    kn = (C.c_int32 * 10)()
    if not args.no_prof:
        check(LIB.ace_prof_stop(kt, kn))
    if world > 1:
        import torch.distributed as dist
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    if rank != 0:
        return
    its = res.stage_iters.cpu().numpy()
    Xh = res.X.cpu().numpy()
    Hh = H.cpu().numpy()
    den = np.einsum("bi,bi->b", Xh.conj(), Xh)
    a = np.einsum("bi,bi->b", Xh.conj(), Hh) / np.where(den == 0, 1, den)
    nmse = np.linalg.norm(Hh - a[:, None] * Xh, axis=1) / np.linalg.norm(Hh, axis=1)
    line = {
        "metric": PIPE_METRIC, "value": round(world * bsz * args.steps / elapsed, 3), "unit": "recoveries/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(1e3 * elapsed / args.steps, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f64", "data": "synthetic (30 dB SNR, L=3 paths)",
        "config": {"workload": f"{args.variant} pipeline, tx=rx={tx}, m={m}, {restarts} restarts, r=20",
                   "batch_per_gpu": bsz, "partitions": "one per restart, shared by the batch"},
        "stage_iters_mean": np.round(its.mean(axis=0), 2).tolist(),
        "stage_iters_max": its.max(axis=0).tolist(),
        "median_rel_err_vs_true_H": float(np.median(nmse)),
        "rel_err_note": ("phase-aligned error vs the synthetic channel; m < n magnitude measurements are "
                         "underdetermined and the reference algorithm (oracle) does not recover H there "
                         "either: see DESIGN.md §3 (recovery regime)") if m < tx * tx else None,
        "kernels_total_ms": {KERNEL_CLASSES[i]: round(kt[i], 2) for i in range(10) if kn[i]},
    }
    print(json.dumps(line), flush=True)


PL_METRIC = "PhaseLift recoveries/sec (MyPhaseLift/TFOCS, 32-ant, 256 meas, 200 TFOCS iters)"


def bench_phaselift(args, dev, rank, world):
    """Config 4 (separate metric): batched MyPhaseLift, 200 TFOCS iterations per recovery."""
    import torch
    import ace_amd
    from ace_amd import phaselift_batch, synth_problem
    from ace_amd._lib import LIB, KERNEL_CLASSES, check
    import ctypes as C
    tx, m, bsz = args.tx, args.m, args.batch
    A, B, _, _ = synth_problem(args.seed, rank * bsz, bsz, m, tx, tx, device=dev)
    Phi = A[0] * float(np.sqrt(tx * tx))                       # unit-modulus codebook rows
    b = (B * float(np.sqrt(tx * tx)) / 2e5) ** 2 * 1e10         # Recover_Channel.m:34 scaling
    ws = ace_amd.solver.Workspace()
    res = None

    def step():
        nonlocal res
        res = phaselift_batch(Phi, b, maxIts=args.iters, workspace=ws)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if not args.no_prof:
        check(LIB.ace_prof_start(400000))
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kt = (C.c_double * 10)()
    kn = (C.c_int32 * 10)()
    if not args.no_prof:
        check(LIB.ace_prof_stop(kt, kn))
    if world > 1:
        import torch.distributed as dist
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    if rank != 0:
        return
    its = res.iters.cpu().numpy()
    names = {"setup": "setup (reduction)", "pre": "y, A_y, gradient", "apply_AH": "A*(g) GEMM",
             "zstep": "prox eig (tridiag+bisect+invit+backxf)", "apply_G": "prox assembly GEMM",
             "apply_A": "A(z) GEMM", "ystep": "x update, backtracking", "final": "final eig + map"}
    line = {
        "metric": PL_METRIC, "value": round(world * bsz * args.steps / elapsed, 3), "unit": "recoveries/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(1e3 * elapsed / args.steps, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f64", "data": "synthetic (30 dB SNR, L=3 paths)",
        "config": {"workload": f"config 4: MyPhaseLift, tx=rx={tx} (n={tx * tx}), m={m}, {args.iters} TFOCS iters",
                   "batch_per_gpu": bsz, "reduced_dim": min(m, tx * tx)},
        "iters_all": bool((its == args.iters).all()),
        "kernels_total_ms": {names.get(KERNEL_CLASSES[i], KERNEL_CLASSES[i]): round(kt[i], 2)
                             for i in range(10) if kn[i]},
    }
    print(json.dumps(line), flush=True)


BF_METRIC = "beamformer codebooks/sec (svd_beamformer: 2 zgesdd + 2-bit quantise + all-pairs search, 16x16)"


def bench_beamformer(args, dev, rank, world):
    """SURVEY.md §8f row 4 (separate metric): batched svd_beamformer on recovered 16 x 16
    channels (main.py:32 num_ant = 16; codebook_library.py:57-96).  One unit = one H ->
    (wr, wt) code pair.  Inputs: noisy synthetic channels (L = 3 paths + CN noise), resident
    in HBM; --tx selects the array size (default 16 in this mode)."""
    import torch
    from ace_amd import svd_beamformer_batch, synth_problem
    tx = args.tx if args.tx != 32 else 16
    bsz = args.batch if args.batch != 4096 else 65536
    _, _, X0, _ = synth_problem(args.seed, rank * bsz, bsz, 8, tx, tx, x0_noise=0.3, device=dev)
    H = X0.reshape(bsz, tx, tx).contiguous()
    res = None

    def step():
        nonlocal res
        res = svd_beamformer_batch(H)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()
    for _ in range(args.steps):
        step()
    ev1.record()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kern_ms = ev0.elapsed_time(ev1) / args.steps
    if world > 1:
        import torch.distributed as dist
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    if rank != 0:
        return
    st = res.status.cpu().numpy()
    per_unit = 16.0 * tx * tx + 2 * tx + 8 + 8 + 4        # read H; write codes, idx, rss, status
    achieved = per_unit * bsz / (kern_ms * 1e-3) / 1e9
    line = {
        "metric": BF_METRIC, "value": round(world * bsz * args.steps / elapsed, 1), "unit": "codebooks/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(1e3 * elapsed / args.steps, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f64", "data": "synthetic (L=3 paths + 0.3 relative CN noise)",
        "config": {"workload": f"svd_beamformer on {tx}x{tx} recovered channels", "batch_per_gpu": bsz},
        "status_clean": bool((st == 0).all()),
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": round(achieved / PEAK_HBM_GBS, 5), "traffic": None,
                     "kernel": "beamformer_kernel", "kernel_ms": round(kern_ms, 4),
                     "note": "latency-bound scalar QR chains (dbdsqr); HBM bytes are the only algorithmic floor"},
    }
    if not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline_beamformer(tx, H[: 2000].cpu().numpy())
    print(json.dumps(line), flush=True)


def cpu_baseline_beamformer(tx, Hs):
    """The oracle (numpy.linalg.svd = the reference's own dependency, all-pairs search
    vectorised) on one host core, on a bounded sample of the same inputs."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import beamformer_oracle as BO
    t0 = time.perf_counter()
    k = 0
    while k < len(Hs) and time.perf_counter() - t0 < 15.0:
        BO.svd_beamformer(Hs[k])
        k += 1
    dt = time.perf_counter() - t0
    return {"value": round(k / dt, 1), "unit": "codebooks/s", "cores": 1, "kind": "port",
            "sample": f"{k} of the same {tx}x{tx} channels through oracle/beamformer_oracle.svd_beamformer "
                      f"(numpy zgesdd + vectorised search; the reference's per-pair Python loop is slower) "
                      f"on {_cpu_model()}"}


def unit_flops(m, n, tx, rx):
    """Algorithmic flops per kernel launch class per realisation per iteration (complex MAC = 8)."""
    return {
        "apply_A": 8.0 * m * n,
        "apply_G": 8.0 * m * m,
        "apply_K": 8.0 * m * m,
        "apply_AH": 8.0 * n * m,
    }


def unit_i8_ops(m, n):
    """int8 matrix-core ops executed per realisation per launch by the digit-plane applies
    (ace_i8gemm.hip): 8 digit planes x the 2x2 real expansion (2m x 2n) x 2 ops per MAC.
    gyk_kernel runs no K Y in the steady state (lazy dual residual, from r02): its int8 work is the
    rare pending-test resolution, not counted."""
    return {"apply_A": 2.0 * 8 * (2 * m) * (2 * n), "apply_AH": 2.0 * 8 * (2 * n) * (2 * m), "apply_G": 0.0}


def gyf_bytes(m, n):
    """Algorithmic HBM bytes per realisation per iteration of gyf_kernel (gyk + the fused apply_AH in
    one launch, g on chip): read Y, M, AX (c128), B (f64) and Z; write AX, M, Y_new and Z' = X."""
    return 16.0 * 6 * m + 8.0 * m + 16.0 * 2 * n


def msp_bytes(m):
    """Algorithmic HBM bytes per realisation per iteration of gyf_kernel for a realisation in m-space
    form (RealState::msp: Z implicit as Z0 + A^H S, no apply_AH pass): read Y, M, AX, S (c128) and
    B (f64); write AX, M, Y_new and S' = S + g.  (opt_S, copied when the iterate improves, is not
    counted: a bookkeeping copy like the deferred opt_X / opt_Y.)"""
    return 16.0 * 8 * m + 8.0 * m


def unit_bytes(m, n, tx, rx):
    """Algorithmic HBM bytes per realisation per iteration of the steady-state unit path
    (complex128 = 16 B, each array read or written once):
      apply_G (gyk):  read Y, M, AX (T = Y - M/mu - AX, the Y-step re-reads M and Y) and B (f64);
                      write g, AX, M, Y_new.  No K Y and no dual-term reads (lazy dual residual);
                      opt_Y is deferred to the Y ping-pong buffer (RealState::optysrc)
      apply_AH (fused i8ah_kernel<false, true>): read g and Z; write Z' = X = Z + A^H g (W stays
                      on chip); N is the exact zero vector and is neither read nor written
      zstep:          certificate and iteration control from RealState (no vector traffic in the
                      steady state; the full Z-step only for realisations the bound cannot certify)
      apply_A (i8):   read Z, Y, M; write T -- cold iterations only (A V = AX in the steady state)"""
    return {
        "zstep": 0.0,
        "apply_G": 16.0 * 7 * m + 8.0 * m,
        "apply_A": 16.0 * (n + 3 * m),
        "apply_AH": 16.0 * (m + 2 * n),
    }


def private_bytes(m, n):
    """Algorithmic HBM bytes per realisation per iteration of pgk_kernel (private phase-code
    codebooks, ace_private.hip) in the steady state (A V = AX):
      G_b = (I + A_b A_b^H)^{-1}: its Hermitian lower triangle, m (m + 1) / 2 complex128
      A_b^H: 2-bit codes, m n / 4 bytes
      read Y, M, AX (c128) and B (f64); write AX, M, Y_new; write W = A^H g (n c128)"""
    return 16.0 * m * (m + 1) / 2 + m * n / 4.0 + 16.0 * 6 * m + 8.0 * m + 16.0 * n


def private_ops(m, n):
    """pgk_kernel's matrix-core and vector work per realisation per iteration: int8 ops of the three
    digit-plane right-hand sides (g, Y, Y - Y0; 8 digits each) times the 2x2 real expansion of A^H,
    and f64 flops of g = G T (8 per complex MAC over the full Hermitian G)."""
    return {"int8": 2.0 * 3 * 8 * (2 * n) * (2 * m), "f64": 8.0 * m * m}


def cpu_baseline(args, n_samples, private):
    """C restatement oracle (oracle/ace_oracle.c, the reference's U-form algorithm)
    timed on the host cores on a bounded sample of the same workload.  Shared codebook: one
    U = inv(A'A + I) amortised over a GPU-sized batch, as on the GPU.  Private codebooks: one U
    per realisation, inside the timed sample (as on the GPU, whose setup is in the timed step)."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import ace_oracle_c as OC
    from ace_amd import synth
    tx = args.tx
    n = tx * tx
    cores = max(1, min(16, len(os.sched_getaffinity(0))))
    A, B, X0, _ = synth.problem(args.seed, 0, n_samples, args.m, tx, tx, a_shared=not private)
    var = 0 if args.variant == "A2only" else 1
    t0 = time.perf_counter()
    if private:
        U = np.stack([OC.make_U(a, nthreads=cores) for a in A])
    else:
        U = OC.make_U(A[0], nthreads=cores)[None]
    t_setup = time.perf_counter() - t0
    t0 = time.perf_counter()
    OC.infer_admm_r1_batch(A if private else A[:1], U, B, X0, tx, tx, variant=var, fixed_iters=True,
                           maxiter=args.iters, nthreads=cores)
    t_solve = time.perf_counter() - t0
    if private:
        t_total = t_solve + t_setup
        setup_note = f"U=inv(A'A+I) per realisation {t_setup:.2f}s"
    else:
        t_total = t_solve + t_setup * n_samples / args.batch
        setup_note = f"U=inv(A'A+I) setup {t_setup:.2f}s amortised over {args.batch}"
    return {"value": n_samples / t_total, "unit": "recoveries/s", "cores": cores, "kind": "port",
            "sample": (f"{n_samples} recoveries of the same workload ({args.iters} fixed iters, m={args.m}, "
                       f"n={n}, {'private' if private else 'shared'} codebook) on {cores} threads of "
                       f"{_cpu_model()}; {setup_note}; solve {t_solve:.2f}s")}


PMC_KERNEL = {"zstep": "zstep1w_kernel<false>", "apply_A": "i8a_kernel", "apply_AH": "i8ah_kernel<false, true>",
              "apply_G": "gyf_kernel"}


PMC_KERNEL_PRIVATE = {"zstep": "zstep1w_kernel<false>", "apply_G": "pgk_kernel"}


def _pmc_traffic(cls, private=False):
    """HBM bytes per launch (PMC FETCH_SIZE, gfx950-corrected, + WRITE_SIZE) of a kernel class from
    the newest committed profiles/*_pmc_hbm.json that has it (written by tools/pmc_summary.py from
    separate rocprofv3 --pmc passes of this benchmark; private-codebook profiles are named
    *_private_pmc_hbm.json), or None."""
    name = (PMC_KERNEL_PRIVATE if private else PMC_KERNEL).get(cls)
    def version(f):   # r<round>_v<version>_pmc_hbm.json
        parts = f.name.split("_")
        try:
            return int(parts[0][1:]), int(parts[1][1:])
        except (IndexError, ValueError):
            return -1, -1
    files = sorted((f for f in (ROOT / "profiles").glob("r*_pmc_hbm.json") if ("_private_" in f.name) == private),
                   key=version)
    if not name:
        return None
    for f in reversed(files):
        try:
            d = json.loads(f.read_text())
        except (OSError, ValueError):
            continue
        for k, v in d.items():
            if k.split(" grid=")[0].strip().startswith(name):
                return round(v["hbm_bytes"]), f"profiles/{f.name}"
    return None


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown CPU"


def main():
    args = parse()
    import torch
    import torch.distributed as dist
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and world > 1:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE {world}")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)

    if args.mode in ("pipeline", "phaselift", "beamformer"):
        {"pipeline": bench_pipeline, "phaselift": bench_phaselift,
         "beamformer": bench_beamformer}[args.mode](args, dev, rank, world)
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return

    line = unit_bench(args, args.private, dev, rank, world)
    if not args.private and not args.no_regime_p and args.variant == "A2only":
        # both codebook regimes, each against its own bound; the headline value is
        # regime S (one codebook for the batch, as in Vs_M.m:192-194 and main.py's one cb_train per call)
        lp = unit_bench(args, True, dev, rank, world)
        if rank == 0:
            line["regime_P"] = {k: lp[k] for k in ("value", "unit", "ms_per_step", "roofline", "cpu_baseline",
                                                   "kernels_ms", "checks")}
            line["regime_P"]["codebook"] = lp["config"]["codebook"]
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def unit_bench(args, private, dev, rank, world):
    """One unit-metric measurement (regime S or P); returns the JSON line dict on rank 0."""
    import torch
    import torch.distributed as dist
    import ace_amd
    from ace_amd import infer_admm_batch, synth_problem
    from ace_amd._lib import LIB, KERNEL_CLASSES, check
    import ctypes as C

    tx = args.tx
    n, m, bsz = tx * tx, args.m, args.batch
    A, B, X0, H = synth_problem(args.seed, rank * bsz, bsz, m, tx, tx, a_shared=not private, device=dev)
    ws = ace_amd.solver.Workspace()
    out = None
    from ace_amd.dist import gather_to_root
    counts = [bsz] * world

    def step():
        nonlocal out
        out = infer_admm_batch(A, B, X0, tx, tx, variant=args.variant, maxiter=args.iters, fixed_iters=True,
                               out=out, workspace=ws)
        if world > 1:   # the single result gather of recovered channels over RCCL/xGMI (north_star)
            gather_to_root(out.X, counts)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    prof = not args.no_prof
    if prof:   # HIP event pairs on every PROF_STRIDE-th launch of each kernel class
        check(LIB.ace_prof_sample(PROF_STRIDE, 0))
        check(LIB.ace_prof_start(args.steps * (args.iters * 8 + 16)))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kt = (C.c_double * 10)()
    kn = (C.c_int32 * 10)()
    msp_steps = C.c_longlong(0)
    if prof:
        check(LIB.ace_prof_stop(kt, kn))
        check(LIB.ace_prof_msp_steps(C.byref(msp_steps)))
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    it_ok = bool((out.iters == args.iters).all().item())
    finite = bool(torch.isfinite(torch.view_as_real(out.X)).all().item())

    if rank == 0:
        total = world * bsz * args.steps
        value = total / elapsed
        kernels = {}
        roof = roof_gemm = None
        if prof:
            uf, ub = unit_flops(m, n, tx, tx), unit_bytes(m, n, tx, tx)
            for i, name in enumerate(KERNEL_CLASSES):
                if kn[i]:
                    kernels[name] = {"launches": int(kn[i]), "avg_ms": kt[i] / kn[i], "total_ms": kt[i]}

            # the int8 digit-plane applies run for a phase-code codebook in the A2only r = 1 iteration
            i8 = (not private) and os.environ.get("ACE_NO_I8") != "1"
            io = unit_i8_ops(m, n)
            # the unit path runs as `nsplit` concurrent sub-batches (ace_admm.cpp::split_count, ACE_SPLIT):
            # every launch of an iteration kernel covers bsz / nsplit realisations
            nsplit = 1
            if i8 and m <= 256:
                nsplit = max(1, min(4, int(os.environ.get("ACE_SPLIT", "2"))))
                while nsplit > 1 and bsz // nsplit < 256:
                    nsplit -= 1
            per_launch = -(-bsz // nsplit)

            gyk = i8 and m <= 256   # apply_G is the fused gyk_kernel (ace_i8gemm.hip)
            # with concurrent sub-batches apply_G is gyf_kernel: gyk and the fused apply_AH in one launch
            env_on = lambda k: os.environ.get(k) != "0"
            # (and with m-space steps, ACE_MSPACE, on one batch too, A2only)
            msp_on = env_on("ACE_MSPACE") and args.variant == "A2only"
            gyf = gyk and (nsplit > 1 or msp_on) and all(env_on(k) for k in ("ACE_GYF", "ACE_FUSE", "ACE_LAZY_DUAL",
                                                                             "ACE_LEAN"))
            # share of the realisation-iterations gyf_kernel settled in m-space form (no apply_AH
            # pass, no Z traffic: ace_prof_msp_steps); the per-launch work below is averaged with it
            msp_frac = msp_steps.value / float(args.steps * bsz * args.iters) if msp_on else 0.0
            # private phase-code codebooks: apply_G is pgk_kernel (ace_private.hip), HBM-bound on G_b
            pc = private and os.environ.get("ACE_NO_I8") != "1" and m <= 256 and n <= 2048

            def roofline(k):
                avg_s = kernels[k]["avg_ms"] * 1e-3
                if k == "apply_G" and pc:
                    b, po = private_bytes(m, n) * per_launch, private_ops(m, n)
                    o, f = po["int8"] * per_launch, po["f64"] * per_launch
                    return {"bound": "hbm", "achieved": round(b / avg_s / 1e9, 1), "peak": PEAK_HBM_GBS,
                            "unit": "GB/s", "frac": round(b / avg_s / 1e9 / PEAK_HBM_GBS, 4), "traffic": None,
                            "kernel": k, "bytes_per_launch": b,
                            "other_resources": {
                                "int8": {"bound": "mfma", "achieved": round(o / avg_s / 1e12, 1), "peak": PEAK_I8_TOPS,
                                         "unit": "TOP/s", "frac": round(o / avg_s / 1e12 / PEAK_I8_TOPS, 4),
                                         "ops_per_launch": o},
                                "f64": {"bound": "valu", "achieved": round(f / avg_s / 1e12, 3),
                                        "peak": PEAK_FP64_TFLOPS, "unit": "TFLOP/s",
                                        "frac": round(f / avg_s / 1e12 / PEAK_FP64_TFLOPS, 4), "flops_per_launch": f}},
                            "bytes_note": "per realisation: G_b lower triangle (c128) + A_b^H as 2-bit codes + "
                                          "Y, M, AX, B in and AX, M, Y out + W = A^H g out (bench.private_bytes)"}
                if k == "apply_G" and gyf:   # f64 G T, int8 A^H g, HBM (T, Y-step, Z pass), phase after phase
                    f = uf[k] * per_launch
                    o = io["apply_AH"] * per_launch * (1.0 - msp_frac)
                    b = (msp_frac * msp_bytes(m) + (1.0 - msp_frac) * gyf_bytes(m, n)) * per_launch
                    tf, to, tb = f / (PEAK_FP64_TFLOPS * 1e12), o / (PEAK_I8_TOPS * 1e12), b / (PEAK_HBM_GBS * 1e9)
                    res = {
                        "f64": {"bound": "mfma", "achieved": round(f / avg_s / 1e12, 3), "peak": PEAK_FP64_TFLOPS,
                                "unit": "TFLOP/s", "frac": round(f / avg_s / 1e12 / PEAK_FP64_TFLOPS, 4),
                                "flops_per_launch": f},
                        "int8": {"bound": "mfma", "achieved": round(o / avg_s / 1e12, 1), "peak": PEAK_I8_TOPS,
                                 "unit": "TOP/s", "frac": round(o / avg_s / 1e12 / PEAK_I8_TOPS, 4),
                                 "ops_per_launch": o},
                        "hbm": {"bound": "hbm", "achieved": round(b / avg_s / 1e9, 1), "peak": PEAK_HBM_GBS,
                                "unit": "GB/s", "frac": round(b / avg_s / 1e9 / PEAK_HBM_GBS, 4), "bytes_per_launch": b},
                    }
                    main = max((("f64", tf), ("int8", to), ("hbm", tb)), key=lambda x: x[1])[0]
                    out = dict(res[main])
                    out.update({"traffic": None, "kernel": "apply_G (gyf_kernel)", "resource": main,
                                "other_resources": {r: v for r, v in res.items() if r != main},
                                "serial_frac": round((tf + to + tb) / avg_s, 4),
                                "msp_frac": round(msp_frac, 4),
                                "flop_note": "gyf_kernel runs T and g = G T (f64 3M; achieved counts 8 flops per "
                                             "complex MAC), the Y-step, then W = A^H g (int8 digit planes) with the "
                                             "certified Z-step pass (Z in, Z' out) in its epilogue, one phase after "
                                             "another in each work-group; a realisation in m-space form (msp_frac of "
                                             "the realisation-iterations) skips the int8 pass and the Z traffic and "
                                             "moves S in / S' out instead (bench.msp_bytes); int8 ops and bytes are "
                                             "averaged with msp_frac; bound = the resource with the largest time "
                                             "at peak; serial_frac = (t_f64 + t_int8 + t_hbm at peak) / launch time"})
                    return out
                if k == "apply_G" and gyk:   # f64 G T + the Y-step's HBM traffic, phase after phase
                    f, b = uf[k] * per_launch, ub[k] * per_launch
                    tf, tb = f / (PEAK_FP64_TFLOPS * 1e12), b / (PEAK_HBM_GBS * 1e9)
                    res = {
                        "f64": {"bound": "mfma", "achieved": round(f / avg_s / 1e12, 3), "peak": PEAK_FP64_TFLOPS,
                                "unit": "TFLOP/s", "frac": round(f / avg_s / 1e12 / PEAK_FP64_TFLOPS, 4),
                                "flops_per_launch": f},
                        "hbm": {"bound": "hbm", "achieved": round(b / avg_s / 1e9, 1), "peak": PEAK_HBM_GBS,
                                "unit": "GB/s", "frac": round(b / avg_s / 1e9 / PEAK_HBM_GBS, 4), "bytes_per_launch": b},
                    }
                    main = "f64" if tf >= tb else "hbm"   # the resource that needs the most time at its peak
                    out = dict(res[main])
                    out.update({"traffic": None, "kernel": k, "resource": main,
                                "other_resources": {r: v for r, v in res.items() if r != main},
                                "serial_frac": round((tf + tb) / avg_s, 4),
                                "flop_note": "gyk_kernel runs g = G T (f64 3M; achieved counts 8 flops per complex "
                                             "MAC) and the Y-step (HBM) one after the other in each work-group; "
                                             "bound = the resource with the largest time at peak; "
                                             "serial_frac = (t_f64 + t_hbm at peak) / launch time"})
                    return out
                if k in io and i8:   # exact int8 digit planes on the matrix cores (+ apply_AH: the fused Z-step pass)
                    per, pb = io[k] * per_launch, ub[k] * per_launch
                    to, tb = per / (PEAK_I8_TOPS * 1e12), pb / (PEAK_HBM_GBS * 1e9)
                    res = {
                        "int8": {"bound": "mfma", "achieved": round(per / avg_s / 1e12, 1), "peak": PEAK_I8_TOPS,
                                 "unit": "TOP/s", "frac": round(per / avg_s / 1e12 / PEAK_I8_TOPS, 4),
                                 "ops_per_launch": per},
                        "hbm": {"bound": "hbm", "achieved": round(pb / avg_s / 1e9, 1), "peak": PEAK_HBM_GBS,
                                "unit": "GB/s", "frac": round(pb / avg_s / 1e9 / PEAK_HBM_GBS, 4),
                                "bytes_per_launch": pb},
                    }
                    main = "int8" if to >= tb else "hbm"
                    out = dict(res[main])
                    out.update({"traffic": None, "kernel": k, "resource": main,
                                "other_resources": {r: v for r, v in res.items() if r != main},
                                "serial_frac": round((to + tb) / avg_s, 4),
                                "f64_equiv_tflops": round(uf[k] * per_launch / avg_s / 1e12, 1),
                                "op_note": "int8 x int8 -> int32 ops of the 8 digit planes x the 2x2 real expansion "
                                           "(exact: the codebook is a phase code); f64_equiv_tflops counts the same "
                                           "product as 8 flops per complex MAC; apply_AH also streams Z in and Z' out "
                                           "(the steady-state Z-step pass fused into its epilogue)"})
                    return out
                if k in uf:   # MFMA-bound complex f64 GEMM
                    per = uf[k] * per_launch
                    # algorithmic = conventional 8 flops per complex MAC; the 3M kernel executes 6
                    return {"bound": "mfma", "achieved": round(per / avg_s / 1e12, 3), "peak": PEAK_FP64_TFLOPS,
                            "unit": "TFLOP/s", "frac": round(per / avg_s / 1e12 / PEAK_FP64_TFLOPS, 4),
                            "traffic": None, "kernel": k, "flops_per_launch": per,
                            "executed_frac": round(0.75 * per / avg_s / 1e12 / PEAK_FP64_TFLOPS, 4),
                            "flop_note": "achieved counts 8 real flops per complex MAC; the 3M (Gauss) kernel "
                                         "executes 6, so the matrix cores run at executed_frac of peak"}
                per = ub[k] * per_launch
                return {"bound": "hbm", "achieved": round(per / avg_s / 1e9, 1), "peak": PEAK_HBM_GBS,
                        "unit": "GB/s", "frac": round(per / avg_s / 1e9 / PEAK_HBM_GBS, 4), "traffic": None,
                        "kernel": k, "bytes_per_launch": per}

            timed = [k for k in kernels if k in uf or k in ub]
            if pc:   # pgk_kernel and the Z-step are the only iteration launches
                timed = [k for k in kernels if k in ("apply_G", "zstep")]
            # every timed class launches once per iteration: dominant = largest average launch
            dom = max(timed, key=lambda k: kernels[k]["avg_ms"])
            roof = roofline(dom)
            roof["realisations_per_launch"] = per_launch
            # the nsplit sub-batch launches of a class run at the same time on disjoint CUs (rocprofv3
            # kernel trace, tools/timeline.py): the chip-level rate is nsplit x the per-launch rate
            roof["concurrent_launches"] = nsplit
            roof["chip_frac"] = round(roof["frac"] * nsplit, 4)
            roof["note"] = (f"dominant kernel by device time (HIP event pairs on the launch stream inside the timed "
                            f"region, on every {PROF_STRIDE}th launch of each kernel class); peaks: MI355X spec (FP64 78.6 TF, int8 5 POP/s dense, HBM3E 8 TB/s); "
                            "traffic: PMC FETCH_SIZE+WRITE_SIZE per launch from the profile named in traffic_source")
            tr = _pmc_traffic(dom, private=pc)
            if tr:
                roof["traffic"], roof["traffic_source"] = tr
            if not pc:
                gemm = max((k for k in kernels if k in uf), key=lambda k: kernels[k]["avg_ms"])
                roof_gemm = roofline(gemm)
                roof_gemm["concurrent_launches"] = nsplit
                roof_gemm["chip_frac"] = round(roof_gemm["frac"] * nsplit, 4)
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            ns = args.cpu_recoveries or (32 if private else 256)
            cpu = cpu_baseline(args, ns, private)
        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "recoveries/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * elapsed / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (Generate_Channel/Random_Phase_State/Generate_Measurement semantics, 30 dB SNR)",
            "config": {
                "workload": ("config 2: 32-ant URA (n=1024), 256 random-codebook RSS meas, A2only ADMM "
                             "refinement solve (r=1), 200 fixed iterations" if args.variant == "A2only" and tx == 32
                             else f"{args.variant}, tx=rx={tx}, m={m}, {args.iters} fixed iterations"),
                "variant": args.variant,
                "codebook": "private per realisation (regime P)" if private else "shared (regime S)",
                "batch_per_gpu": bsz,
                "global_batch": world * bsz,
                "m": m, "n": n, "iters": args.iters,
                "parallelism": f"dp{world} (realisation sharding, RCCL gather of X to rank 0)",
            },
            "roofline": roof,
            "roofline_gemm": roof_gemm if prof else None,
            "cpu_baseline": cpu,
            "kernels_ms": {k: round(v["avg_ms"], 4) for k, v in kernels.items()},
            "checks": {"all_iters_ran": it_ok, "finite": finite},
        }
        return line
    return None



if __name__ == "__main__":
    main()
