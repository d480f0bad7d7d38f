"""Diagnostic: which realisations of a batch disagree with the C oracle."""
import sys
import numpy as np
sys.path.insert(0, "2ace-mmwave-channel-estimation_amd"); sys.path.insert(0, "oracle")
import torch
import ace_oracle as O, ace_oracle_c as OC
from ace_amd import infer_admm_batch, synth_problem
batch, m, tx, iters = (int(v) for v in sys.argv[1:5])
A, B, X0, _ = synth_problem(53, 0, batch, m, tx, tx)
idx = list(range(0, batch, 37)) + [batch - 1]
Ah, Bh, X0h = A.cpu().numpy(), B.cpu().numpy()[idx], X0.cpu().numpy()[idx]
U = OC.make_U(Ah[0])[None]
Xo, _, _, _, _ = OC.infer_admm_r1_batch(Ah, U, Bh, X0h, tx, tx, variant=0, maxiter=iters, fixed_iters=True)
r = infer_admm_batch(A, B, X0, tx, tx, maxiter=iters, fixed_iters=True)
torch.cuda.synchronize()
X = r.X.cpu().numpy()[idx]
e = [O.unit_phase_aligned_rel_err(X[i], Xo[i]) for i in range(len(idx))]
print([(j, f"{v:.1e}") for j, v in zip(idx, e) if v > 1e-9])
print("ok", sum(v <= 1e-9 for v in e), "of", len(e))
