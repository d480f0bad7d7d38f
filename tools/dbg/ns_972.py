"""Debug: Newton-Schulz setup (I + K)^-1 on the reference codebook's train rows at M = 1024."""
import os, sys, math, numpy as np
sys.path[:0] = ['oracle', '2ace-mmwave-channel-estimation_amd', 'tests']
import ace_amd
from ace_amd import synth, engine, infer_admm_host
from test_gpu_driver import _ref_codebook, _cb, SEEDS
tx = 16
k, amp, ang = _ref_codebook("random")
seed = SEEDS[2]
idx = engine.randperm(seed, 0x100 + 14, 3968, 1024)
A = _cb(amp, ang)[idx]
A = A / np.linalg.norm(A) * math.sqrt(A.shape[0])
mt = 972
tr = engine.randperm(seed, 0x101 + 14, 1024, mt)
At = A[tr]
K = At @ At.conj().T
w = np.linalg.eigvalsh(np.eye(mt) + K)
print("eig(I+K) min %g max %g  gersh %g" % (w[0], w[-1], np.abs(np.eye(mt) + K).sum(1).max()), flush=True)
h = synth.channel(3, 0, tx, tx)
rng = np.random.default_rng(0)
cases = {"ref_train_rows": At, "ref_all_rows": A, "synth_972": synth.codebook(3, mt, 256),
         "ref_train_rows_perturbed": At + 1e-13 * rng.standard_normal(At.shape)}
for name, Am in cases.items():
    B = np.abs(Am @ h)[None]
    X0 = (h + 0.1 * rng.standard_normal(256))[None]
    try:
        r = infer_admm_host(Am[None], B, X0, tx, tx, maxiter=5, fixed_iters=True, f64_applies=True)
        print(name, Am.shape, "ok finite", np.isfinite(r.X).all(), flush=True)
    except Exception as e:
        print(name, Am.shape, "ERR", e, flush=True)
