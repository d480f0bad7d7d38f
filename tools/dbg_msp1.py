"""One solve (for rocprofv3): batch m tx iters fixed."""
import sys
sys.path.insert(0, "2ace-mmwave-channel-estimation_amd")
import torch
from ace_amd import infer_admm_batch, synth_problem
batch, m, tx, iters, fixed = (int(v) for v in sys.argv[1:6])
A, B, X0, _ = synth_problem(53, 0, batch, m, tx, tx)
for _ in range(2):
    r = infer_admm_batch(A, B, X0, tx, tx, maxiter=iters, fixed_iters=bool(fixed))
torch.cuda.synchronize()
print("iters", r.iters.float().mean().item())
