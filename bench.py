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

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--mode MODE]

Modes (each its own line; only ``unit`` is the headline metric):
  unit       configs[1] (default; ``--variant A2nuclear`` = configs[2]); also measures regime P
             (private codebooks) and the unit on the reference's own refinement input
             (X0 = the pipeline's X_max, inferLowRankV4_multi.m:90-92)
  config5    configs[4]: 32-ant multiresolution codebook, A2nuclear, 65 536 realisations in
             total sharded over the ranks (strong scaling), one RCCL gather
  pipeline   full inferLowRankV4_multi recoveries/s (a separately named metric)
  phaselift  configs[3]: MyPhaseLift/TFOCS, 200 iterations, batch 512
  beamformer downstream svd_beamformer codebooks/s
  driver     latency of one drop-in driver call (main.py:427) on the reference probe codebook
  refine     the unit line's refine_input object alone (X_max and the per-realisation rank-one flags)
"""
from __future__ import annotations

import argparse
import json
import math
import os
import pathlib
import sys
import time
import traceback

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "2ace-mmwave-channel-estimation_amd"))

METRIC = "channel recoveries/sec (32-ant, 256 RSS meas, 200 ADMM iters) @1/2/4/8 GPU"
PEAK_FP64_TFLOPS = 78.6   # MI355X FP64 matrix (= FP64 vector) dense peak, spec
PEAK_HBM_GBS = 8000.0     # MI355X HBM3E spec
PEAK_I8_TOPS = 5000.0     # MI355X int8 matrix dense peak, spec (2x the BF16 rate per clock)
PROF_STRIDE = 7           # unit mode: kernel events on every 7th launch of each kernel class (about 86 samples per
                          # class and stream over 3 steps; 200 mod 7 != 0, so the sampled iteration indices
                          # drift over the steps; the event pairs cost < 1 % of the throughput)
CONFIG5_GLOBAL = 65536    # configs[4]: realisations over all GPUs
ITER_CLASSES = ("pre", "apply_A", "apply_G", "ystep", "apply_K", "apply_AH", "zstep")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=0, help="recoveries per GPU per step (0 = the mode's default)")
    ap.add_argument("--global-batch", type=int, default=CONFIG5_GLOBAL, help="config5: realisations over all GPUs")
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--variant", default="A2only", choices=["A2only", "A2nuclear"])
    ap.add_argument("--private", action="store_true", help="private codebook per realisation (regime P)")
    ap.add_argument("--tx", type=int, default=0, help="antennas per side (0 = the mode's default)")
    ap.add_argument("--m", type=int, default=256)
    ap.add_argument("--seed", type=int, default=58659179)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-regime-p", action="store_true", help="unit mode: skip the regime-P measurement")
    ap.add_argument("--no-refine-input", action="store_true",
                    help="unit mode: skip the measurement on the pipeline's refinement input")
    ap.add_argument("--no-default-profile", action="store_true",
                    help="refine_input: skip the comparison run with the default rank profile for every realisation")
    ap.add_argument("--cpu-recoveries", type=int, default=0, help="CPU sample size (0 = auto)")
    ap.add_argument("--cpu-seconds", type=float, default=20.0, help="time budget of a sampled CPU baseline")
    ap.add_argument("--no-configs", action="store_true",
                    help="unit mode: skip the config 3 / 4 / 5 and pipeline objects of the default line")
    ap.add_argument("--no-prof", action="store_true", help="disable live per-kernel event timing")
    ap.add_argument("--mode", default="unit",
                    choices=["unit", "config5", "pipeline", "phaselift", "beamformer", "driver", "refine"])
    a = ap.parse_args()
    if not a.tx:
        a.tx = 16 if a.mode in ("beamformer", "driver") else 32
    if not a.batch:
        a.batch = {"phaselift": 512, "beamformer": 65536}.get(a.mode, 4096)
    return a


# ------------------------------------------------------------------ roofline accounting
# Algorithmic work per realisation per iteration of each kernel class: f64 flops
# (8 per complex MAC), int8 matrix-core ops, HBM bytes (complex128 = 16 B, each array once).

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
    """Algorithmic HBM bytes per realisation per iteration of the steady-state A2only unit path
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


def nuclear_bytes(m, n):
    """The A2nuclear unit path (configs[2], configs[4]): its soft threshold never leaves Z' = E, so N
    is nonzero and A V is formed every iteration:
      apply_G (gyk_kernel): read Y, M, AX, B and Z, N (the digit planes of V = Z - N/mu);
                            write g, AX, M, Y_new
      apply_AH (i8ah_kernel<false, false>): read g, write W = A^H g
      zstep (one-wave, soft threshold): read W, Z, N; write Z', N'"""
    return {"apply_G": 16.0 * 7 * m + 8.0 * m + 32.0 * n, "apply_AH": 16.0 * (m + n), "zstep": 80.0 * n}


def nms_bytes(m):
    """A2nuclear at r = 1 in m-space (ace_nucmsp.hip::nms_kernel, one launch per iteration).  Z and N
    are both multiples of E_prev = alpha X_init + A^H e, so the state is one m-vector e and the
    image A E_prev; no n-vector moves.  Per realisation and iteration: read Y, M, e, A E (c128) and
    B (f64); write Y_new, M, e_new, A E_new (opt_w / opt_Y on an improved objective are
    bookkeeping copies, not counted)."""
    return 16.0 * 8 * m + 8.0 * m


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


def unit_resources(k, m, n, *, variant, pc, gyf, gyk, i8, msp_frac, nms=False):
    """Per-realisation work of one launch of kernel class k on the unit path: {resource: amount}
    with resources f64 (flops), int8 (ops), hbm (bytes).  {} = latency-bound, no roofline."""
    uf, io, ub = unit_flops(m, n, 0, 0), unit_i8_ops(m, n), unit_bytes(m, n, 0, 0)
    if nms:   # A2nuclear m-space iteration: g = G T on the f64 matrix cores and m-vectors only
        return {"f64": uf["apply_G"], "hbm": nms_bytes(m)} if k == "apply_G" else {}
    if pc:
        po = private_ops(m, n)
        return {"hbm": private_bytes(m, n), "int8": po["int8"], "f64": po["f64"]} if k == "apply_G" else {}
    if variant == "A2nuclear" and i8:
        nb = nuclear_bytes(m, n)
        if k == "apply_G" and gyk:
            return {"f64": uf["apply_G"], "int8": io["apply_A"], "hbm": nb["apply_G"]}
        if k == "apply_AH":
            return {"int8": io["apply_AH"], "hbm": nb["apply_AH"]}
        if k == "zstep":
            return {"hbm": nb["zstep"]}
    if k == "apply_G" and gyf:   # gyk + the fused apply_AH; m-space realisations skip the int8 pass
        return {"f64": uf[k], "int8": io["apply_AH"] * (1.0 - msp_frac),
                "hbm": msp_frac * msp_bytes(m) + (1.0 - msp_frac) * gyf_bytes(m, n)}
    if k == "apply_G" and gyk:
        return {"f64": uf[k], "hbm": ub[k]}
    if k in io and i8 and k != "apply_G":
        return {"int8": io[k], "hbm": ub[k]}
    if k in uf:
        return {"f64": uf[k]}
    return {}


_RES = {  # resource -> (peak per second, unit label, unit scale, roofline bound name, amount key)
    "f64": (PEAK_FP64_TFLOPS * 1e12, "TFLOP/s", 1e12, "mfma", "flops_per_launch"),
    "int8": (PEAK_I8_TOPS * 1e12, "TOP/s", 1e12, "mfma", "ops_per_launch"),
    "hbm": (PEAK_HBM_GBS * 1e9, "GB/s", 1e9, "hbm", "bytes_per_launch"),
}


def roofline_from(kernel, avg_s, res, bounds=None, note=None):
    """Roofline entry of one launch of `kernel` (avg_s seconds) doing `res` = {resource: amount}:
    the resource with the largest time at peak is the bound; the others go to other_resources;
    serial_frac = (sum of the times at peak) / launch time (phases that run one after another)."""
    bounds = bounds or {}
    t = {r: a / _RES[r][0] for r, a in res.items() if a > 0}
    main = max(t, key=t.get)

    def ent(r):
        peak, unit, scale, bound, key = _RES[r]
        a = res[r]
        return {"bound": bounds.get(r, bound), "achieved": round(a / avg_s / scale, 3), "peak": peak / scale,
                "unit": unit, "frac": round(a / avg_s / peak, 4), key: a}

    out = ent(main)
    out.update({"traffic": None, "kernel": kernel, "resource": main,
                "other_resources": {r: ent(r) for r in t if r != main},
                "serial_frac": round(sum(t.values()) / avg_s, 4)})
    if note:
        out["flop_note"] = note
    return out


def _pmc_traffic(kernel_prefix, tag, batch=None):
    """HBM bytes per launch (PMC FETCH_SIZE, gfx950-corrected, + WRITE_SIZE) of the kernel whose name
    starts with `kernel_prefix`, from the newest committed profiles/r<R>_v<V>[_<tag>]_pmc_hbm.json
    measured on the same workload (tag: unit | private | nuclear | config5 | pipeline | phaselift;
    files without a tag are unit-mode passes), or None.  Written by tools/pmc_summary.py from separate
    rocprofv3 --pmc passes, with the profiled run's realisations per GPU in "_meta" (every launch of
    these workloads covers a fixed share of the batch: the split halves, the stage launches over
    batch x r vectors), so the bytes are rescaled to the line's `batch` -- per realisation, like
    the algorithmic bytes they are compared with.  Profiles without "_meta" are not used."""
    def parse_name(f):   # r<round>_v<version>[_<tag>]_pmc_hbm.json
        parts = f.name[: -len("_pmc_hbm.json")].split("_")
        try:
            return (int(parts[0][1:]), int("".join(c for c in parts[1][1:] if c.isdigit()))), "_".join(parts[2:]) or "unit"
        except (IndexError, ValueError):
            return None, None
    files = []
    for f in (ROOT / "profiles").glob("r*_pmc_hbm.json"):
        ver, ftag = parse_name(f)
        if ver is not None and ftag == tag:
            files.append((ver, f))
    for _, f in sorted(files, reverse=True):
        try:
            d = json.loads(f.read_text())
        except (OSError, ValueError):
            continue
        meta = d.get("_meta")
        if not meta or not meta.get("batch"):
            continue
        scale = (batch / meta["batch"]) if batch else 1.0
        for k, v in d.items():
            if k != "_meta" and k.split(" grid=")[0].strip().startswith(kernel_prefix):
                return round(v["hbm_bytes"] * scale), f"profiles/{f.name}" + (
                    f" (profiled at batch {meta['batch']}, x {scale:g})" if scale != 1.0 else "")
    return None


PMC_KERNEL = {  # kernel-class -> kernel name prefix in the PMC profiles, per workload tag
    "unit": {"zstep": "zstep1w_kernel<false>", "apply_A": "i8a_kernel", "apply_AH": "i8ah_kernel<false, true>",
             "apply_G": "gyf_kernel"},
    "private": {"zstep": "zstep1w_kernel<false>", "apply_G": "pgk_kernel"},
    "nuclear": {"zstep": "zstep1w_kernel<false>", "apply_AH": "i8ah_kernel<false, false>", "apply_G": "gyk_kernel"},
}
PMC_KERNEL["nuclear"] = {"apply_G": "nms_kernel<false>"}   # the m-space iteration (ace_nucmsp.hip)
PMC_KERNEL["config5"] = PMC_KERNEL["nuclear"]
PMC_KERNEL["refine"] = PMC_KERNEL["unit"]   # the unit on the pipeline's X_max (bench.py --mode refine)
# pipeline / PhaseLift: the dominant class's largest kernel (one launch per class launch)
PMC_KERNEL["pipeline"] = {"apply_AH": "i8ah_kernel<false, false>", "apply_A": "i8a_kernel",
                          "apply_K": "i8ah_kernel<true, false>", "apply_G": "zgemm3m_kernel<0, false",
                          "zstep": "zstep_kernel", "ystep": "ystep_r_kernel", "pre": "pre_kernel"}
PMC_KERNEL["phaselift"] = {"zstep": "he2hb_kernel"}   # the two-stage reduction's stage 1 (ace_heev2.hip)


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown CPU"


def _cores():
    return max(1, min(16, len(os.sched_getaffinity(0))))


def _blas_threads():
    for k in ("OPENBLAS_NUM_THREADS", "OMP_NUM_THREADS", "MKL_NUM_THREADS"):
        if os.environ.get(k, "").isdigit():
            return int(os.environ[k])
    return len(os.sched_getaffinity(0))


def _max_over_ranks(elapsed, dev, world):
    if world > 1:
        import torch
        import torch.distributed as dist
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed


def _barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def _prof_read(nclass=11):
    """(total ms, launches, algorithmic flops, HBM bytes, int8 ops) per kernel class since ace_prof_start."""
    import ctypes as C
    from ace_amd._lib import LIB, check
    kt, kn = (C.c_double * nclass)(), (C.c_int32 * nclass)()
    kw, kb, ko = (C.c_double * nclass)(), (C.c_double * nclass)(), (C.c_double * nclass)()
    check(LIB.ace_prof_stop(kt, kn))
    check(LIB.ace_prof_work_ex(kw, kb, ko))
    return list(kt), list(kn), list(kw), list(kb), list(ko)


def work_roofline(kt, kn, kw, kb, ko, note, tag=None, batch=None):
    """Roofline of the dominant kernel class BY DEVICE TIME, from the algorithmic work its launches carry
    (ace_prof_work_ex: f64 flops of the GEMM-shaped applies and prox steps, HBM bytes of every stage
    kernel, int8 ops of the digit-plane applies), plus every class's share of the device time.  With
    `tag`, `traffic` is the PMC HBM bytes per launch of the class's largest kernel (PMC_KERNEL[tag])
    from a profile of the same workload, rescaled to `batch` realisations."""
    from ace_amd._lib import KERNEL_CLASSES
    tot = sum(kt)
    shares = {KERNEL_CLASSES[i]: round(kt[i] / tot, 4) for i in range(len(kt)) if kn[i]}
    cand = [i for i in range(len(kt)) if kn[i]]
    if not cand:
        return None, shares
    i = max(cand, key=lambda c: kt[c])
    avg_s = kt[i] / kn[i] * 1e-3
    res = {k: v / kn[i] for k, v in (("f64", kw[i]), ("hbm", kb[i]), ("int8", ko[i])) if v > 0}
    if not res:
        return {"kernel": KERNEL_CLASSES[i], "bound": "latency", "launches": kn[i], "avg_ms": round(avg_s * 1e3, 4),
                "device_time_share": shares[KERNEL_CLASSES[i]], "traffic": None,
                "note": "the dominant class carries no algorithmic work count"}, shares
    r = roofline_from(KERNEL_CLASSES[i], avg_s, res, note=note)
    r["launches"] = kn[i]
    r["avg_ms"] = round(avg_s * 1e3, 4)
    r["device_time_share"] = shares[KERNEL_CLASSES[i]]
    pmc = PMC_KERNEL.get(tag, {}).get(KERNEL_CLASSES[i]) if tag else None
    tr = _pmc_traffic(pmc, tag, batch) if pmc else None
    if tr:
        r["traffic"], r["traffic_source"] = tr
        r["traffic_kernel"] = pmc
        if res.get("hbm"):
            r["traffic_per_algorithmic"] = round(tr[0] / res["hbm"], 3)
    return r, shares


# ------------------------------------------------------------------ CPU baselines

def cpu_baseline(args, n_samples, private, variant=None, A_host=None):
    """C restatement oracle (oracle/ace_oracle.c, the reference's U-form algorithm)
    timed on the host cores on a bounded sample of the same workload.  Shared codebook: one
    U = inv(A'A + I) amortised over a GPU-sized batch, as on the GPU.  Private codebooks: one U
    per realisation, inside the timed sample (as on the GPU, whose setup is in the timed step)."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import ace_oracle_c as OC
    from ace_amd import synth
    tx = args.tx
    n = tx * tx
    cores = _cores()
    variant = variant or args.variant
    if A_host is not None:   # a given shared codebook (config5): the same synthetic channels on it
        A = A_host[None]
        H = np.stack([synth.channel(args.seed, c, tx, tx) for c in range(n_samples)])
        B = np.stack([synth.measurements(args.seed, c, A[0], H[c]) for c in range(n_samples)])
        X0 = np.stack([synth.initial_iterate(args.seed, c, H[c]) for c in range(n_samples)])
        nb = np.sqrt(np.sum(B * B, axis=1))
        B, X0 = B / nb[:, None], X0 / nb[:, None]
    else:
        A, B, X0, _ = synth.problem(args.seed, 0, n_samples, args.m, tx, tx, a_shared=not private)
    var = 0 if variant == "A2only" else 1
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
            "sample": (f"{n_samples} recoveries of the same workload ({variant}, {args.iters} fixed iters, "
                       f"m={args.m}, n={n}, {'private' if private else 'shared'} codebook) on {cores} threads of "
                       f"{_cpu_model()}; {setup_note}; solve {t_solve:.2f}s")}


# ------------------------------------------------------------------ unit / config5

def _work_accounting(per_gpu, variant, m, n, tx, iters, msp_frac):
    """SURVEY.md §8(d) prices a recovery in the reference's U-form (X = U (A^H (Y - M/mu) + Z - N/mu) with
    U = inv(A^H A + I) n x n: 8 (3mn + n^2 + 3 tx^3) flops per iteration for A2only, 8 (3mn + n^2) for
    A2nuclear); the build executes the Woodbury / m-space form instead (g = G T with
    G = (I + K)^-1 m x m, 8 m^2 f64 flops per iteration, the Aᴴ / A applies on the int8 digit planes for the
    iterations outside the m-space form).  Both rates per GPU, so that a U-form rate above the FP64 peak
    reads as what it is: less work done, not a faster chip."""
    u = 8.0 * (3 * m * n + n * n + (3 * tx ** 3 if variant == "A2only" else 0)) * iters
    ex64 = 8.0 * m * m * iters
    ex8 = (1.0 - msp_frac) * iters * 2 * 2.0 * 8 * (2 * m) * (2 * n) if variant == "A2only" else None
    d = {"u_form_flops_per_recovery": u, "u_form_tflops_per_gpu": round(per_gpu * u / 1e12, 2),
         "u_form_frac_of_fp64_peak": round(per_gpu * u / 1e12 / PEAK_FP64_TFLOPS, 3),
         "executed_f64_flops_per_recovery": ex64, "executed_f64_tflops_per_gpu": round(per_gpu * ex64 / 1e12, 2),
         "executed_f64_frac_of_peak": round(per_gpu * ex64 / 1e12 / PEAK_FP64_TFLOPS, 3)}
    if ex8 is not None:
        d["executed_int8_ops_per_recovery"] = ex8
        d["executed_int8_tops_per_gpu"] = round(per_gpu * ex8 / 1e12, 1)
    d["note"] = _work_accounting.__doc__.split("\n\n")[0].replace("\n    ", " ")
    return d


def unit_bench(args, private, dev, rank, world, workload=None):
    """One unit-metric measurement (regime S or P, or a given workload); the JSON line dict on rank 0.
    workload: {"tag", "name", "variant", "A" (device codebook), "A_host", "bsz", "first", "counts",
    "scaling", "codebook", "X0" (device X0), "x0_note"} -- all optional."""
    import torch
    import ace_amd
    from ace_amd import infer_admm_batch, synth_problem
    from ace_amd._lib import LIB, KERNEL_CLASSES, check
    from ace_amd.dist import gather_results_async
    import ctypes as C

    wl = workload or {}
    tx = args.tx
    variant = wl.get("variant", args.variant)
    n, m = tx * tx, args.m
    bsz = wl.get("bsz", args.batch)
    first = wl.get("first", rank * bsz)
    counts = wl.get("counts", [bsz] * world)
    A, B, X0, H = synth_problem(args.seed, first, bsz, m, tx, tx, a_shared=not private, device=dev, A=wl.get("A"))
    if wl.get("X0") is not None:
        X0 = wl["X0"]
    # per-realisation use_rank_one (the refinement's profile, inferLowRankV4_multi.m:73-77, :92/:100)
    r1 = wl.get("rank_one", False)
    ws = ace_amd.solver.Workspace()
    outs, pend, nstep = [None, None], [None, None], [0]

    # The single result gather over RCCL/xGMI (north_star; SURVEY.md §8(e): X, iteration counts and
    # status per realisation -- the unit solve has no quality -- packed into one byte row each, one
    # collective), asynchronous: the gather of step k overlaps the solve of step k + 1 (outputs
    # double-buffered; a buffer is reused only after its gather has completed, and the timed region
    # waits for the last one).
    def step():
        i = nstep[0] & 1
        if pend[i] is not None:
            pend[i].wait()
            pend[i] = None
        outs[i] = infer_admm_batch(A, B, X0, tx, tx, variant=variant, maxiter=args.iters, fixed_iters=True,
                                   use_rank_one=r1, out=outs[i], workspace=ws)
        if world > 1:
            o = outs[i]
            pend[i] = gather_results_async({"X": o.X, "iters": o.iters, "status": o.status, "mu": o.mu}, counts)
        nstep[0] += 1

    def drain():
        for i in range(2):
            if pend[i] is not None:
                pend[i].wait()
                pend[i] = None

    for _ in range(args.warmup):
        step()
    drain()
    torch.cuda.synchronize()
    _barrier(world)
    prof = not args.no_prof
    if prof:   # HIP event pairs on every PROF_STRIDE-th launch of each kernel class
        check(LIB.ace_prof_sample(PROF_STRIDE, 1 << 10))   # every m-space run (msr) launch
        check(LIB.ace_prof_start(args.steps * (args.iters * 8 + 16)))
    torch.cuda.synchronize()
    _barrier(world)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    drain()
    torch.cuda.synchronize()
    _barrier(world)
    elapsed = time.perf_counter() - t0
    out = outs[(nstep[0] - 1) & 1]
    msp_steps = C.c_longlong(0)
    if prof:
        kt, kn, kw, _, _ = _prof_read()
        check(LIB.ace_prof_msp_steps(C.byref(msp_steps)))
    elapsed = _max_over_ranks(elapsed, dev, world)
    it_ok = bool((out.iters == args.iters).all().item())
    finite = bool(torch.isfinite(torch.view_as_real(out.X)).all().item())
    if rank != 0:
        return None

    total = sum(counts) * args.steps
    kernels, roof, roof_gemm, roof_msr = {}, None, None, None
    tag = wl.get("tag", "private" if private else ("nuclear" if variant == "A2nuclear" else "unit"))
    msp_frac = 0.0
    if prof:
        for i, name in enumerate(KERNEL_CLASSES):
            if kn[i]:
                kernels[name] = {"launches": int(kn[i]), "avg_ms": kt[i] / kn[i], "total_ms": kt[i]}
        # the int8 digit-plane applies run for a phase-code codebook in the r = 1 iteration
        i8 = (not private) and os.environ.get("ACE_NO_I8") != "1"
        # the unit path runs as `nsplit` concurrent sub-batches (ace_admm.cpp::split_count, ACE_SPLIT):
        # every launch of an iteration kernel covers bsz / nsplit realisations
        # A2nuclear r = 1 on a shared A runs the m-space iteration (ace_nucmsp.hip, one launch per
        # iteration over the whole batch) unless ACE_NUC_MSP=0
        nms = (not private) and variant == "A2nuclear" and m <= 256 and os.environ.get("ACE_NUC_MSP") != "0"
        nsplit = 1
        if i8 and m <= 256 and not nms:
            nsplit = max(1, min(4, int(os.environ.get("ACE_SPLIT", "2"))))
            while nsplit > 1 and bsz // nsplit < 256:
                nsplit -= 1
        per_launch = -(-bsz // nsplit)
        env_on = lambda k: os.environ.get(k) != "0"   # noqa: E731
        gyk = i8 and m <= 256   # apply_G is the fused gyk_kernel (ace_i8gemm.hip)
        # m-space steps (ACE_MSPACE) for A2only: every iteration is gyf_kernel + Z-step
        msp_on = env_on("ACE_MSPACE") and variant == "A2only"
        gyf = gyk and variant == "A2only" and (nsplit > 1 or msp_on) and all(
            env_on(k) for k in ("ACE_GYF", "ACE_FUSE", "ACE_LAZY_DUAL", "ACE_LEAN"))
        # share of the realisation-iterations gyf_kernel settled in m-space form (no apply_AH pass,
        # no Z traffic: ace_prof_msp_steps); the per-launch work below is averaged with it
        msp_frac = msp_steps.value / float(args.steps * bsz * args.iters) if msp_on else 0.0
        # the m-space runs (msr_kernel) take the steady iterations away from gyf_kernel: its launches see
        # the m-space share of the realisation-iterations the runs did not execute (ace_prof_work counts
        # 8 m^2 per realisation-iteration of every run launch)
        msr_i = KERNEL_CLASSES.index("msr") if "msr" in KERNEL_CLASSES else -1
        msr_steps = kw[msr_i] / (8.0 * m * m) if (msr_i >= 0 and kn[msr_i]) else 0.0
        rest = float(args.steps * bsz * args.iters) - msr_steps
        msp_frac_gyf = min(1.0, max(0.0, (msp_steps.value - msr_steps) / rest)) if (msp_on and rest > 0) else 0.0
        # private phase-code codebooks: apply_G is pgk_kernel (ace_private.hip), HBM-bound on G_b
        pc = private and os.environ.get("ACE_NO_I8") != "1" and m <= 256 and n <= 2048
        ctx = dict(variant=variant, pc=pc, gyf=gyf, gyk=gyk, i8=i8, msp_frac=msp_frac_gyf, nms=nms)
        timed = [k for k in kernels if k in ITER_CLASSES and unit_resources(k, m, n, **ctx)]
        # device time per class: the iteration classes are sampled on every PROF_STRIDE-th launch, the
        # m-space runs (msr, ace_i8gemm.hip::msr_kernel) on every launch; dominant = most device time
        dev_ms = {k: kernels[k]["total_ms"] * PROF_STRIDE for k in timed}
        roof_msr = None
        if msr_i >= 0 and kn[msr_i] and kw[msr_i] > 0:
            # flops: 8 m^2 per realisation-iteration the runs executed (ace_prof_work, counted on the device)
            roof_msr = roofline_from("msr_kernel (m-space run)", kernels["msr"]["avg_ms"] * 1e-3,
                                     {"f64": kw[msr_i] / kn[msr_i]}, note=(
                "the unit's steady m-space iterations (T, g = G T on the f64 matrix cores in 3M form, the "
                "Y-step, the certified control) of a 16-realisation block inside one launch, state on chip; "
                "achieved counts 8 flops per complex MAC of g = G T over the realisation-iterations the run "
                "executed (device counter)"))
            roof_msr["iterations_per_launch"] = round(kw[msr_i] / kn[msr_i] / (8.0 * m * m) / per_launch, 1)
            roof_msr["realisations_per_launch"] = per_launch
            roof_msr["concurrent_launches"] = nsplit
            roof_msr["chip_frac"] = round(roof_msr["frac"] * nsplit, 4)
            tr = _pmc_traffic("msr_kernel", tag, bsz)
            if tr:
                roof_msr["traffic"], roof_msr["traffic_source"] = tr
            dev_ms["msr"] = kernels["msr"]["total_ms"]
        dom = max(dev_ms, key=dev_ms.get)

        def roof_of(k):
            res = {r: a * per_launch for r, a in unit_resources(k, m, n, **ctx).items()}
            name = "apply_G (gyf_kernel)" if (k == "apply_G" and gyf) else k
            note = None
            if nms:
                name = "apply_G (nms_kernel)"
                note = ("A2nuclear m-space iteration (ace_nucmsp.hip): T, g = G T (f64 3M; achieved counts 8 "
                        "flops per complex MAC), K g = T - g, the Y-step and the m-space Z-step, one phase after "
                        "another in each work-group; bytes: bench.nms_bytes")
            elif k == "apply_G" and gyf:
                note = ("gyf_kernel runs T and g = G T (f64 3M; achieved counts 8 flops per complex MAC), the "
                        "Y-step, then W = A^H g (int8 digit planes) with the certified Z-step pass (Z in, Z' out) "
                        "in its epilogue, one phase after another in each work-group; a realisation in m-space "
                        "form (msp_frac of the realisation-iterations its launches ran: those outside the m-space "
                        "runs) skips the int8 pass and the Z traffic and "
                        "moves S in / S' out instead (bench.msp_bytes); bound = the resource with the largest "
                        "time at peak; serial_frac = (t_f64 + t_int8 + t_hbm at peak) / launch time")
            elif variant == "A2nuclear" and i8:
                note = ("A2nuclear n-space unit path (bench.nuclear_bytes): A V in gyk_kernel every iteration, plain "
                        "apply_AH, the soft-threshold Z-step streams W, Z, N")
            r = roofline_from(name, kernels[k]["avg_ms"] * 1e-3, res, bounds={"f64": "valu"} if pc else None,
                              note=note)
            if gyf:
                r["msp_frac"] = round(msp_frac_gyf, 4)
            r["realisations_per_launch"] = per_launch
            # the nsplit sub-batch launches of a class run at the same time on disjoint CUs (rocprofv3
            # kernel trace, tools/timeline.py): the chip-level rate is nsplit x the per-launch rate
            r["concurrent_launches"] = nsplit
            r["chip_frac"] = round(r["frac"] * nsplit, 4)
            pmc = PMC_KERNEL.get(tag, {}).get(k)
            tr = _pmc_traffic(pmc, tag, bsz) if pmc else None
            if tr:
                r["traffic"], r["traffic_source"] = tr
                if res.get("hbm"):
                    r["traffic_per_algorithmic"] = round(tr[0] / res["hbm"], 3)
            return r

        roof = roof_msr if dom == "msr" else roof_of(dom)
        roof["device_time_share"] = {k: round(v / sum(dev_ms.values()), 4) for k, v in dev_ms.items()}
        roof["note"] = (f"dominant kernel by device time (HIP event pairs on the launch stream inside the timed "
                        f"region, on every {PROF_STRIDE}th launch of each iteration class and every m-space run); "
                        "peaks: MI355X spec (FP64 78.6 TF, int8 5 POP/s dense, HBM3E 8 TB/s); traffic: PMC "
                        "FETCH_SIZE+WRITE_SIZE per launch from the profile named in traffic_source (same workload tag)")
        if not pc:
            fk = [k for k in timed if "f64" in unit_resources(k, m, n, **ctx)]
            if fk:
                roof_gemm = roof_of(max(fk, key=lambda k: kernels[k]["avg_ms"]))
    cpu = None
    if not args.no_cpu_baseline and world == 1:
        ns = args.cpu_recoveries or (32 if private else 256)
        cpu = cpu_baseline(args, ns, private, variant, wl.get("A_host"))
    if variant == "A2only" and tx == 32 and m == 256:
        default_name = ("config 2: 32-ant URA (n=1024), 256 random-codebook RSS meas, A2only ADMM refinement "
                        "solve (r=1), 200 fixed iterations")
    elif tx == 32 and m == 256:
        default_name = "config 3: 32-ant, 256 meas, A2nuclear ADMM refinement solve (r=1), 200 fixed iterations"
    else:
        default_name = f"{variant}, tx=rx={tx}, m={m}, {args.iters} fixed iterations"
    return {
        "metric": METRIC,
        "value": round(total / elapsed, 2),
        "unit": "recoveries/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * elapsed / args.steps, 3),
        "higher_is_better": True,
        "scaling": wl.get("scaling", "weak"),
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (Generate_Channel/Random_Phase_State/Generate_Measurement semantics, 30 dB SNR)",
        "config": {
            "workload": wl.get("name", default_name),
            "variant": variant,
            "codebook": wl.get("codebook", "private per realisation (regime P)" if private else "shared (regime S)"),
            "batch_per_gpu": bsz,
            "global_batch": sum(counts),
            "m": m, "n": n, "iters": args.iters,
            "x0": wl.get("x0_note", "H + 0.5 CN noise (synthetic warm start; refine_input measures the "
                                    "reference's own refinement input)"),
            "parallelism": f"dp{world} (realisation sharding, one RCCL gather of X, iters, status, mu to rank 0)",
        },
        "roofline": roof,
        "roofline_gemm": roof_gemm,
        "roofline_msr": roof_msr if prof else None,
        "cpu_baseline": cpu,
        "kernels_ms": {k: round(v["avg_ms"], 4) for k, v in kernels.items()},
        "msp_frac": round(msp_frac, 4),
        "work_accounting": _work_accounting(total / elapsed / world, variant, m, n, tx, args.iters, msp_frac),
        "checks": {"all_iters_ran": it_ok, "finite": finite},
    }


def refine_input_bench(args, dev, rank, world):
    """The unit on the reference's own refinement: X0 = X_max of the 3-restart pipeline
    (inferLowRankV4_multi.m:90-92: spectral init, the r = 20 stages, rank-one retries, best of
    restarts) on the same synthetic batch, and each realisation's own use_rank_one -- the last
    restart's (:73-77), which selects the [1]/[0.95] rank profile (:448-450) of the refinement
    (:92/:100); ACE_ST_RANK_ONE of the pipeline.  The synthetic A has ||A||_F = sqrt(m) and B is
    unit-norm, so X_max is already in the unit's coordinates (A_norm = B_norm = 1, :27-38).  Also
    reports the same X0 with the default profile for every realisation (the round-3 measurement)."""
    import torch
    from ace_amd import synth_problem, infer_low_rank_pipeline_batch, draw_partitions
    tx, m, bsz = args.tx, args.m, args.batch
    A, B, _, _ = synth_problem(args.seed, rank * bsz, bsz, m, tx, tx, device=dev)
    tr = draw_partitions(np.random.default_rng(args.seed + rank), m, 3, batch=bsz)   # per call (:48)
    t0 = time.perf_counter()
    pr = infer_low_rank_pipeline_batch(A, B, tx, tx, tr, stop_before_refine=True)
    torch.cuda.synchronize()
    t_pipe = time.perf_counter() - t0
    X0 = pr.X.contiguous()
    flags = pr.rank_one.to(torch.uint8).contiguous()
    saved = args.no_cpu_baseline
    args.no_cpu_baseline = True
    line = unit_bench(args, False, dev, rank, world, {"X0": X0, "rank_one": flags, "x0_note": "pipeline X_max",
                                                      "tag": "refine"})
    line0 = None if args.no_default_profile else unit_bench(
        args, False, dev, rank, world, {"X0": X0, "x0_note": "pipeline X_max, default profile", "tag": "refine"})
    args.no_cpu_baseline = saved
    if rank != 0:
        return None
    q = pr.quality.cpu().numpy()
    return {"value": line["value"], "unit": "recoveries/s", "ms_per_step": line["ms_per_step"],
            "msp_frac": line["msp_frac"],
            "x0": "X_max of inferLowRankV4_multi's 3 restarts (:90-92) on the same batch (ace_pipeline_solve_batch "
                  "with stop_before_refine)",
            "rank_one_frac": round(float(flags.float().mean().item()), 4),
            "profile": "per realisation: the last restart's use_rank_one (:73-77, :92/:100; ACE_ST_RANK_ONE)",
            "pipeline_s": round(t_pipe, 2), "quality_median": float(np.median(q)),
            "roofline": line["roofline"], "roofline_msr": line["roofline_msr"],
            "kernels_ms": line["kernels_ms"], "checks": line["checks"],
            "default_profile": None if line0 is None else {
                "value": line0["value"], "ms_per_step": line0["ms_per_step"], "msp_frac": line0["msp_frac"],
                "note": "the same X0 with use_rank_one = 0 for every realisation (not the reference's refinement "
                        "for rank_one_frac of them)"}}


def config5_workload(args, rank, world, dev):
    """configs[4]: the 32-antenna multiresolution codebook (ace_amd.synth.multires_codes, the
    builder-defined analogue of generate_tx_codebook_multires_16ant.py / processsing_codebook_
    multires.m), M = m rows drawn by randperm within the tier ..._multiresolution.m:137-144 selects
    (the same rows on every rank), A2nuclear, the global batch sharded contiguously over the ranks."""
    import torch
    from ace_amd import synth
    from ace_amd.dist import shard_range
    tx, m = args.tx, args.m
    lens, th = synth.multires_tiers(tx)
    rows, tier = synth.multires_rows(args.seed, tx, m)
    A_host = synth.multires_codebook(args.seed, tx, rows)
    A = torch.from_numpy(A_host[None]).to(dev)
    counts = [shard_range(args.global_batch, world, r)[1] for r in range(world)]
    first, bsz = shard_range(args.global_batch, world, rank)
    name = (f"config 5: 32-ant multiresolution codebook (tier {tier}: {['4', '2', '1'][tier]}-antenna groups, "
            f"{m} of {lens[tier]} rows), A2nuclear ADMM refinement solve (r=1), {args.iters} fixed iterations, "
            f"{args.global_batch} realisations over {world} GPU(s)")
    return {"tag": "config5", "name": name, "variant": "A2nuclear", "A": A, "A_host": A_host, "bsz": bsz,
            "first": first, "counts": counts, "scaling": "strong",
            "codebook": f"shared multiresolution rows (tier {tier}, thresholds {list(th)})"}


# ------------------------------------------------------------------ other modes

PIPE_METRIC = "pipeline recoveries/sec (inferLowRankV4_multi, 32-ant, 256 RSS meas, convergence mode)"


def bench_pipeline(args, dev, rank, world):
    """Full-pipeline throughput (separate metric): one batch per step, shared partitions."""
    import torch
    import ace_amd
    from ace_amd import infer_low_rank_pipeline_batch, synth_problem, draw_partitions
    from ace_amd._lib import LIB, KERNEL_CLASSES, check
    from ace_amd.dist import gather_results_async
    tx, m, bsz = args.tx, args.m, args.batch
    restarts = 3 if args.variant == "A2only" else 1
    A, B, _, H = synth_problem(args.seed, rank * bsz, bsz, m, tx, tx, device=dev)
    # every realisation its own partitions: randsample inside each inferLowRankV4_multi call (:48), as a
    # Monte-Carlo batch of calls draws them (ACE_TRAIN_PER_REALISATION)
    tr = draw_partitions(np.random.default_rng(args.seed + rank), m, restarts, batch=bsz)
    ws = ace_amd.solver.Workspace()
    res = None

    counts = [bsz] * world

    def step():
        nonlocal res
        res = infer_low_rank_pipeline_batch(A, B, tx, tx, tr, variant=args.variant, workspace=ws)
        if world > 1:   # X, quality, stage iteration counts, status in one collective
            gather_results_async({"X": res.X, "quality": res.quality, "stage_iters": res.stage_iters,
                                  "status": res.status}, counts).wait()

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    _barrier(world)
    if not args.no_prof:
        check(LIB.ace_prof_sample(1, 0))
        check(LIB.ace_prof_start(400000))
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    _barrier(world)
    elapsed = time.perf_counter() - t0
    roof, shares, kt = None, None, None
    if not args.no_prof:
        kt, kn, kw, kb, ko = _prof_read()
        roof, shares = work_roofline(kt, kn, kw, kb, ko, (
            "algorithmic work of the dominant class by device time (ace_prof_work_ex), over the vectors of the stage "
            "still iterating (batch*r scaled by the live share at the convergence polls): f64 flops (8 per complex "
            "MAC), HBM bytes (every per-vector array read or written once), int8 ops of the digit-plane applies; "
            "the r-column Z-step: E E^H (tx^2 rx r MACs) + the 32x32 eig (0.8 Mflop), X, N, Z in / Z, N out"),
            tag="pipeline", batch=bsz)
    elapsed = _max_over_ranks(elapsed, dev, world)
    if rank != 0:
        return None
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
                   "batch_per_gpu": bsz,
                   "partitions": "per realisation and restart (train_idx [batch][restarts][m_t], randsample per call)"},
        "stage_iters_mean": np.round(its.mean(axis=0), 2).tolist(),
        "stage_iters_max": its.max(axis=0).tolist(),
        "median_rel_err_vs_true_H": float(np.median(nmse)),
        "rel_err_note": ("phase-aligned error vs the synthetic channel; m < n magnitude measurements are "
                         "underdetermined and the reference algorithm (oracle) does not recover H there "
                         "either: see DESIGN.md §3 (recovery regime)") if m < tx * tx else None,
        "roofline": roof,
        "device_time_shares": shares,
        "kernels_total_ms": {KERNEL_CLASSES[i]: round(kt[i], 2) for i in range(10) if kt[i]} if kt else None,
    }
    if not args.no_cpu_baseline and world == 1:
        line["cpu_baseline"] = cpu_baseline_pipeline(args, A[0].cpu().numpy(), B.cpu().numpy(), tr)
    return line


def cpu_baseline_pipeline(args, A, B, tr):   # tr: [batch][restarts][m_t]
    """The numpy oracle pipeline (oracle/ace_oracle.py::infer_low_rank_pipeline, the reference's
    algorithm line by line; BLAS threads as the host provides) on a bounded sample of the batch."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import ace_oracle as O
    k, t0 = 0, time.perf_counter()
    while k < min(len(B), args.cpu_recoveries or 8) and (k == 0 or time.perf_counter() - t0 < args.cpu_seconds):
        O.infer_low_rank_pipeline(A, B[k], args.tx, args.tx, list(tr[k]),
                                  variant=O.VARIANT_A2ONLY if args.variant == "A2only" else O.VARIANT_NUCLEAR)
        k += 1
    dt = time.perf_counter() - t0
    return {"value": round(k / dt, 4), "unit": "recoveries/s", "cores": _blas_threads(), "kind": "port",
            "sample": f"{k} recoveries of the same batch through oracle/ace_oracle.py (numpy, BLAS threads as "
                      f"available) on {_cpu_model()}"}


PL_METRIC = "PhaseLift recoveries/sec (MyPhaseLift/TFOCS, 32-ant, 256 meas, 200 TFOCS iters)"


def bench_phaselift(args, dev, rank, world):
    """Config 4 (separate metric): batched MyPhaseLift, 200 TFOCS iterations per recovery."""
    import torch
    import ace_amd
    from ace_amd import phaselift_batch, synth_problem
    from ace_amd._lib import LIB, KERNEL_CLASSES, check
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
    _barrier(world)
    if not args.no_prof:
        check(LIB.ace_prof_sample(1, 0))
        check(LIB.ace_prof_start(400000))
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    _barrier(world)
    elapsed = time.perf_counter() - t0
    roof, shares, kt = None, None, None
    if not args.no_prof:
        kt, kn, kw, kb, ko = _prof_read()
        roof, shares = work_roofline(
            kt, kn, kw, kb, ko, "algorithmic f64 flops per realisation in the backtracking step (8 per complex MAC) in "
            "the d = min(m, n) reduced coordinates: prox eig 17.3 d^3 (SURVEY.md §8d's count for a dense Hermitian "
            "eig with vectors), A*(g) 8 d^2 m, assembly 8 d^3, A(z) 8 m d^2", tag="phaselift", batch=bsz)
    elapsed = _max_over_ranks(elapsed, dev, world)
    if rank != 0:
        return None
    its = res.iters.cpu().numpy()
    names = {"setup": "setup (reduction)", "pre": "y, A_y, gradient", "apply_AH": "A*(g) GEMM",
             "zstep": "prox eig (tridiag+bisect+invit+backxf)", "apply_G": "prox assembly GEMM",
             "apply_A": "A(z) GEMM", "ystep": "x update, backtracking", "final": "final eig + map"}
    if roof:
        roof["kernel"] = names.get(roof["kernel"], roof["kernel"])
        if roof.get("traffic") and roof.get("traffic_kernel") == "he2hb_kernel":
            # the traffic is stage 1 of the two-stage reduction (PMC per launch of bsz matrices of order d): against
            # its compulsory bytes (read C, write the band and the reflectors: 2 d^2 complex) and against the
            # blocked algorithm's own floor: per panel of 16, X = A V reads the trailing matrix (L^2 entries through
            # its lower triangle) and the update reads and writes that lower triangle (L^2), sum 2 L^2 ~ d^3 / 24
            d = min(m, tx * tx)
            comp = bsz * 2 * 16 * d * d
            blk = bsz * 16 * d ** 3 / 24
            roof["traffic_algorithmic"] = comp
            roof["traffic_per_algorithmic"] = round(roof["traffic"] / comp, 3)
            roof["traffic_blocked_floor"] = round(blk)
            roof["traffic_per_blocked_floor"] = round(roof["traffic"] / blk, 3)
    line = {
        "metric": PL_METRIC, "value": round(world * bsz * args.steps / elapsed, 3), "unit": "recoveries/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(1e3 * elapsed / args.steps, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f64", "data": "synthetic (30 dB SNR, L=3 paths)",
        "config": {"workload": f"config 4: MyPhaseLift, tx=rx={tx} (n={tx * tx}), m={m}, {args.iters} TFOCS iters",
                   "batch_per_gpu": bsz, "reduced_dim": min(m, tx * tx)},
        "iters_all": bool((its == args.iters).all()),
        "roofline": roof,
        "device_time_shares": {names.get(k, k): v for k, v in shares.items()} if shares else None,
        "kernels_total_ms": {names.get(KERNEL_CLASSES[i], KERNEL_CLASSES[i]): round(kt[i], 2)
                             for i in range(10) if kt[i]} if kt else None,
    }
    if not args.no_cpu_baseline and world == 1:
        line["cpu_baseline"] = cpu_baseline_phaselift(args, Phi.cpu().numpy(), b[:4].cpu().numpy())
    return line


def cpu_baseline_phaselift(args, Phi, b):
    """The TFOCS oracle (oracle/tfocs_oracle.py::my_phaselift_reduced: MyPhaseLift + solver_TraceLS in
    the coordinates of range(Phi^H), the dense iteration up to rounding; numpy BLAS / LAPACK threads as
    available), the same 200 iterations, on a bounded sample of the batch."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import tfocs_oracle as T
    k, t0 = 0, time.perf_counter()
    while k < len(b) and (k == 0 or time.perf_counter() - t0 < args.cpu_seconds):
        T.my_phaselift_reduced(b[k], Phi, maxIts=args.iters)
        k += 1
    dt = time.perf_counter() - t0
    return {"value": round(k / dt, 4), "unit": "recoveries/s", "cores": _blas_threads(), "kind": "port",
            "sample": f"{k} recoveries of the same batch, {args.iters} TFOCS iterations, through "
                      f"oracle/tfocs_oracle.my_phaselift_reduced (numpy) on {_cpu_model()}"}


BF_METRIC = "beamformer codebooks/sec (svd_beamformer: 2 zgesdd + 2-bit quantise + all-pairs search, 16x16)"


def bench_beamformer(args, dev, rank, world):
    """SURVEY.md §8f row 4 (separate metric): batched svd_beamformer on recovered 16 x 16
    channels (main.py:32 num_ant = 16; codebook_library.py:57-96).  One unit = one H ->
    (wr, wt) code pair.  Inputs: noisy synthetic channels (L = 3 paths + CN noise), resident
    in HBM; --tx selects the array size (default 16 in this mode)."""
    import torch
    from ace_amd import svd_beamformer_batch, synth_problem
    tx, bsz = args.tx, args.batch
    _, _, X0, _ = synth_problem(args.seed, rank * bsz, bsz, 8, tx, tx, x0_noise=0.3, device=dev)
    H = X0.reshape(bsz, tx, tx).contiguous()
    res = None

    def step():
        nonlocal res
        res = svd_beamformer_batch(H)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    _barrier(world)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()
    for _ in range(args.steps):
        step()
    ev1.record()
    torch.cuda.synchronize()
    _barrier(world)
    elapsed = time.perf_counter() - t0
    kern_ms = ev0.elapsed_time(ev1) / args.steps
    elapsed = _max_over_ranks(elapsed, dev, world)
    if rank != 0:
        return None
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
    return line


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


DRIVER_METRIC = ("drop-in driver call latency (channel_recovery_ADMM_v2_simulation_A2only, 16x16, "
                 "reference probe codebook, 8-point M sweep)")
DRIVER_SEED_ID = 3


def driver_trace(tx, seed):
    """main.py's inputs to the driver: the reference's probing codebook (tests/golden/
    ref_codebooks_16x16_packed.npz = codebook/codebook_mat/random_probe_cb_16x16.mat as 2-bit codes)
    as |cb| and angle(cb) (main.py:301-302), RSS in dBm (main.py:113) of a synthetic channel."""
    from ace_amd import synth
    p = np.load(ROOT / "tests" / "golden" / "ref_codebooks_16x16_packed.npz")["random"]
    k = np.stack([(p >> (2 * i)) & 3 for i in range(4)], axis=-1).reshape(p.shape[0], -1).astype(np.int64)
    cb = np.exp(1j * np.pi / 2 * k)
    h = synth.channel(seed, 0, tx, tx)
    rss = 10 * np.log10(1000 * (np.abs(cb @ h) * 1e-4) ** 2)
    return np.abs(cb), np.angle(cb), rss


def bench_driver(args, dev, rank, world):
    """Wall-clock latency of one drop-in driver call, as main.py:427 makes it (host arrays in, host
    arrays out: the 8 sweep points' row draws, uploads, pipelines and downloads).  The reference
    states "2ACE solve time ... normally within a second" for 16 x 16 CSI (README.md:87, MATLAB on a
    laptop): the only published timing of the path, a qualitative upper bound."""
    from ace_amd import engine
    if rank != 0:
        return None
    tx = 16
    amp, ang, rss = driver_trace(tx, 17)
    eng = engine.start_matlab()

    def call():
        return eng.channel_recovery_ADMM_v2_simulation_A2only(tx, tx, engine.double(amp), engine.double(ang),
                                                             engine.double(rss[:, None]),
                                                             eng.double(DRIVER_SEED_ID), nargout=2)

    for _ in range(max(1, args.warmup)):
        call()
    lat = {}
    for mode in ("0", "1"):   # concurrent sweep points (default) and ACE_DRIVER_SERIAL=1
        os.environ["ACE_DRIVER_SERIAL"] = mode
        ts = []
        for _ in range(args.steps):
            t0 = time.perf_counter()
            Ha, _ = call()
            ts.append(time.perf_counter() - t0)
        lat[mode] = ts
    os.environ.pop("ACE_DRIVER_SERIAL", None)
    med = float(np.median(lat["0"]))
    line = {
        "metric": DRIVER_METRIC, "value": round(med, 4), "unit": "s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(1e3 * med, 2), "higher_is_better": False, "scaling": "none",
        "vs_baseline": round(med / 1.0, 4), "dtype": "f64",
        "data": "reference probe codebook random_probe_cb_16x16.mat (3968 x 256), synthetic channel RSS",
        "config": {"workload": "one ace_recover_driver call: M in round(linspace(2, 32, 8)).^2, 3-restart pipeline "
                               "per point (M = 4 ill-posed, returned as 0)",
                   "sweep_points": "concurrent host threads / HIP streams"},
        "baseline": {"value": 1.0, "unit": "s", "source": "README.md:87 'normally within a second' (MATLAB, "
                                                          "testbed laptop): a qualitative upper bound"},
        "latency_s": {"concurrent_median": round(med, 4), "concurrent_all": [round(t, 4) for t in lat["0"]],
                      "serial_median": round(float(np.median(lat["1"])), 4)},
        "finite": bool(np.all(np.isfinite(Ha))),
        "nonzero_points": int(sum(bool(Ha[i].max() > 0) for i in range(Ha.shape[0]))),
        "roofline": None,
        "roofline_note": "latency-bound (one realisation per sweep point); see the unit and pipeline lines",
    }
    if not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline_driver(tx, amp, ang, rss)
    return line


def cpu_baseline_driver(tx, amp, ang, rss):
    """The same driver call composed on the CPU: the driver's rows (engine.randperm, the build's RNG),
    then the numpy oracle pipeline per sweep point (oracle/ace_oracle.py)."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import ace_oracle as O
    from ace_amd import engine
    seed, fct = 36326041, 1e5 / 3      # seeds(3) of ..._A2only.m:103, rss_fct :132
    cb = amp * np.exp(1j * ang)
    t0 = time.perf_counter()
    for i, M in enumerate(engine.m_sweep(tx, tx)):
        mt = math.floor(0.95 * M)
        if mt < min(20, M):
            continue
        idx = engine.randperm(seed, 0x100 + 2 * i, len(rss), int(M))
        B = np.sqrt(10.0 ** (rss[idx] / 10.0) / 1000.0) * fct
        tr = [engine.randperm(seed, 0x101 + 2 * i + 0x10000 * s, int(M), mt) for s in range(3)]
        O.infer_low_rank_pipeline(cb[idx], B, tx, tx, tr)
    dt = time.perf_counter() - t0
    return {"value": round(dt, 3), "unit": "s", "cores": _blas_threads(), "kind": "port",
            "sample": f"one full driver call (7 well-posed sweep points) through oracle/ace_oracle.py (numpy) on "
                      f"{_cpu_model()}"}


# ------------------------------------------------------------------ the other configs on the default line

def _sub(args, **kw):
    a = argparse.Namespace(**vars(args))
    for k, v in kw.items():
        setattr(a, k, v)
    return a


def _leg_summary(ln, keep=()):
    """A config's own line reduced to what the default line carries for it."""
    if ln is None:
        return None
    d = {k: ln[k] for k in ("metric", "value", "unit", "ms_per_step", "steps", "warmup", "scaling", "config",
                            "roofline", "cpu_baseline") if k in ln}
    for k in keep:
        if k in ln:
            d[k] = ln[k]
    return d


def config_legs(args, dev, rank, world):
    """BASELINE.json configs[2..4] and the pipeline, each measured with its own steps inside the default run
    (every config driver-observed): (key, thunk returning the object on rank 0).  Steps are
    fewer for the slow workloads so that the whole default line stays within a few minutes; each object
    carries its own ms_per_step x steps, roofline (live HIP events + the newest PMC traffic of its tag) and
    CPU baseline (a shorter sample budget than the modes' own lines)."""
    cpu_s = min(args.cpu_seconds, 8.0)

    def config3():
        a = _sub(args, variant="A2nuclear", cpu_seconds=cpu_s)
        ln = unit_bench(a, False, dev, rank, world)
        return _leg_summary(ln, ("kernels_ms", "checks", "roofline_msr")) if rank == 0 else None

    def config5():
        a = _sub(args, cpu_seconds=cpu_s, global_batch=CONFIG5_GLOBAL)
        ln = unit_bench(a, False, dev, rank, world, config5_workload(a, rank, world, dev))
        return _leg_summary(ln, ("kernels_ms", "checks")) if rank == 0 else None

    def config4():
        a = _sub(args, batch=512, steps=1, warmup=1, cpu_seconds=cpu_s)
        return _leg_summary(bench_phaselift(a, dev, rank, world), ("iters_all", "device_time_shares"))

    def pipeline():
        a = _sub(args, batch=4096, steps=1, warmup=1, cpu_seconds=cpu_s, cpu_recoveries=2)
        return _leg_summary(bench_pipeline(a, dev, rank, world), ("stage_iters_mean", "device_time_shares"))

    return [("config3", config3), ("config5_shard", config5), ("config4", config4), ("pipeline", pipeline)]


# ------------------------------------------------------------------ main

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

    if args.mode in ("pipeline", "phaselift", "beamformer", "driver"):
        line = {"pipeline": bench_pipeline, "phaselift": bench_phaselift, "beamformer": bench_beamformer,
                "driver": bench_driver}[args.mode](args, dev, rank, world)
        if rank == 0:
            print(json.dumps(line), flush=True)
    elif args.mode == "refine":   # the unit on the reference's own refinement alone (refine_input of the unit line)
        ri = refine_input_bench(args, dev, rank, world)
        if rank == 0:
            print(json.dumps({"metric": METRIC + " -- reference refinement input", "n_gpus": world,
                              "steps": args.steps, "warmup": args.warmup, "higher_is_better": True,
                              "dtype": "f64", **ri}), flush=True)
    elif args.mode == "config5":
        line = unit_bench(args, False, dev, rank, world, config5_workload(args, rank, world, dev))
        if rank == 0:
            print(json.dumps(line), flush=True)
    else:
        line = unit_bench(args, args.private, dev, rank, world)
        if not args.private and args.variant == "A2only":
            # The secondary measurements ride on the headline line; a failure in one of them is reported
            # in its own field ({"error": ...}, the traceback on stderr) instead of discarding the
            # headline measurement already taken (round 4 lost its line that way)
            def leg(fn):
                try:
                    return fn()
                except Exception as e:   # noqa: BLE001
                    traceback.print_exc()
                    return {"error": f"{type(e).__name__}: {e}"}
            if not args.no_regime_p:
                # both codebook regimes, each against its own bound; the headline value is
                # regime S (one codebook for the batch, as in Vs_M.m:192-194 and main.py's one cb_train per call)
                def regime_p():
                    lp = unit_bench(args, True, dev, rank, world)
                    if rank != 0:
                        return None
                    d = {k: lp[k] for k in ("value", "unit", "ms_per_step", "roofline", "cpu_baseline",
                                            "kernels_ms", "checks")}
                    d["codebook"] = lp["config"]["codebook"]
                    return d
                rp = leg(regime_p)
                if rank == 0:
                    line["regime_P"] = rp
            if not args.no_refine_input and world == 1 and args.tx == 32:
                ri = leg(lambda: refine_input_bench(args, dev, rank, world))
                if rank == 0:
                    line["refine_input"] = ri
            if not args.no_configs and args.tx == 32:
                for key, fn in config_legs(args, dev, rank, world):
                    r = leg(fn)
                    if rank == 0:
                        line[key] = r
        if rank == 0:
            print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
