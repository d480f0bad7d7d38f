"""Where m-space runs (msr_kernel) and the per-iteration launches part: X, Y, iters, status of
ACE_MSR=1 against ACE_MSR=0 for several run windows.  Diagnostic only."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "2ace-mmwave-channel-estimation_amd"))
import torch  # noqa: E402
from ace_amd import infer_admm_batch, synth_problem  # noqa: E402

A, B, X0, _ = synth_problem(71, 0, 1024, 256, 32, 32)


def run(env, maxiter):
    for k in ("ACE_MSR", "ACE_MSR_START"):
        os.environ.pop(k, None)
    os.environ.update(env)
    r = infer_admm_batch(A, B, X0, 32, 32, maxiter=maxiter, fixed_iters=True)
    torch.cuda.synchronize()
    return r.X.cpu().numpy(), r.Y.cpu().numpy(), r.iters.cpu().numpy(), r.status.cpu().numpy()


for maxiter, start in ((60, 59), (60, 58), (60, 56), (120, 56), (200, 199), (200, 56)):
    a = run({"ACE_MSR": "0"}, maxiter)
    b = run({"ACE_MSR_START": str(start)}, maxiter)
    dx = np.abs(a[0] - b[0]).max(axis=1)
    dy = np.abs(a[1] - b[1]).max(axis=1)
    print(f"maxiter {maxiter} start {start}: X differs in {int((dx > 0).sum())} (max {dx.max():.3g}), "
          f"Y in {int((dy > 0).sum())} (max {dy.max():.3g}), iters eq {np.array_equal(a[2], b[2])}, "
          f"status differs in {int((a[3] != b[3]).sum())}", flush=True)
