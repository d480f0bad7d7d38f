"""Diagnostic: m-space steady state (ACE_MSPACE) against the C oracle and against ACE_MSPACE=0."""
import os, sys, time
import numpy as np
sys.path.insert(0, "2ace-mmwave-channel-estimation_amd"); sys.path.insert(0, "oracle")
import torch
import ace_oracle as O, ace_oracle_c as OC
from ace_amd import infer_admm_batch, synth_problem
batch, m, tx, iters, fixed = (int(v) for v in sys.argv[1:6])
A, B, X0, _ = synth_problem(53, 0, batch, m, tx, tx)
idx = list(range(0, batch, max(1, batch // 24))) + [batch - 1]
Ah, Bh, X0h = A.cpu().numpy(), B.cpu().numpy()[idx], X0.cpu().numpy()[idx]
U = OC.make_U(Ah[0])[None]
Xo, _, it_o, _, _ = OC.infer_admm_r1_batch(Ah, U, Bh, X0h, tx, tx, variant=0, maxiter=iters, fixed_iters=bool(fixed))
def run(env):
    for k in ("ACE_MSPACE", "ACE_MSP_FAIL_IT"):
        os.environ.pop(k, None)
    os.environ.update(env)
    r = infer_admm_batch(A, B, X0, tx, tx, maxiter=iters, fixed_iters=bool(fixed))
    torch.cuda.synchronize()
    t0 = time.time()
    r = infer_admm_batch(A, B, X0, tx, tx, maxiter=iters, fixed_iters=bool(fixed))
    torch.cuda.synchronize()
    return r, time.time() - t0
for env in ({"ACE_MSPACE": "0"}, {}, {"ACE_MSP_FAIL_IT": "60"}, {"ACE_MSP_FAIL_IT": str(iters)}):
    r, dt = run(env)
    X = r.X.cpu().numpy()
    it = r.iters.cpu().numpy()
    e = [O.unit_phase_aligned_rel_err(X[j], Xo[i]) for i, j in enumerate(idx)]
    itok = int(np.sum(it[idx] == np.asarray(it_o)))
    print(env, f"{dt*1e3:.1f} ms", "max err %.2e" % max(e), "iters equal", itok, "of", len(idx), "finite", bool(np.isfinite(X).all()))
