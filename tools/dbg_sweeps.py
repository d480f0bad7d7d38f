"""Diagnostic: the unit solve with the ACE_DEBUG_SWEEPS build (per-phase cycle stamps of the
one-wave Z-step for realisations 0 and 2000), 40 iterations at batch 4096."""
import os
import sys
sys.path.insert(0, "2ace-mmwave-channel-estimation_amd")
import torch  # noqa: E402
import ace_amd  # noqa: E402
from ace_amd import infer_admm_batch, synth_problem  # noqa: E402
dev = torch.device("cuda", 0)
A, B, X0, _ = synth_problem(58659179, 0, 4096, 256, 32, 32, a_shared=True, device=dev)
out = infer_admm_batch(A, B, X0, 32, 32, maxiter=40, fixed_iters=True)
torch.cuda.synchronize()
print("done", os.environ.get("ACE_LIB"))
