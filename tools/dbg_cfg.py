"""Diagnostic: one configuration under the unit path's switches against the C oracle (sample)."""
import os, sys
import numpy as np
sys.path.insert(0, "2ace-mmwave-channel-estimation_amd"); sys.path.insert(0, "oracle")
import torch
import ace_oracle as O, ace_oracle_c as OC
from ace_amd import infer_admm_batch, synth_problem
batch, m, tx, iters = (int(v) for v in sys.argv[1:5])
A, B, X0, _ = synth_problem(53, 0, batch, m, tx, tx)
idx = [0, 519, 1023]
Ah, Bh, X0h = A.cpu().numpy(), B.cpu().numpy()[idx], X0.cpu().numpy()[idx]
U = OC.make_U(Ah[0])[None]
Xo, _, _, _, _ = OC.infer_admm_r1_batch(Ah, U, Bh, X0h, tx, tx, variant=0, maxiter=iters, fixed_iters=True)
for env in ({}, {"ACE_LEAN": "0"}, {"ACE_LAZY_DUAL": "0"}, {"ACE_SPLIT": "1"}, {"ACE_NO_I8": "1"}):
    for k in ("ACE_LEAN", "ACE_LAZY_DUAL", "ACE_SPLIT", "ACE_NO_I8"):
        os.environ.pop(k, None)
    os.environ.update(env)
    r = infer_admm_batch(A, B, X0, tx, tx, maxiter=iters, fixed_iters=True)
    torch.cuda.synchronize()
    X = r.X.cpu().numpy()[idx]
    print(env, [f"{O.unit_phase_aligned_rel_err(X[i], Xo[i]):.2e}" for i in range(3)])
sm = infer_admm_batch(A, B[512:576].contiguous(), X0[512:576].contiguous(), tx, tx, maxiter=iters, fixed_iters=True)
torch.cuda.synchronize()
print("small batch 512..575, realisation 519:", f"{O.unit_phase_aligned_rel_err(sm.X.cpu().numpy()[7], Xo[1]):.2e}")
