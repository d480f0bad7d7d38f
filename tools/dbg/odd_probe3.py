"""Probe: the tx = 1, m = 64 Newton-Schulz failure -- odd path vs the same zero-padded problem through the even path."""
import sys
import numpy as np
sys.path[:0] = ["oracle", "tests", "2ace-mmwave-channel-estimation_amd"]
from ace_amd import infer_admm_host, synth

tx, rx, m = 1, 8, 64
A, B, X0, _ = synth.problem(32, 0, 4, m, tx, rx, a_shared=True)
Ap = np.zeros((1, m, 2 * rx), complex); Ap[:, :, 0::2] = A
X0p = np.zeros((4, 2 * rx), complex); X0p[:, 0::2] = X0
K = A[0] @ A[0].conj().T
w = np.linalg.eigvalsh(np.eye(m) + K)
print("I+K eig range", w.min(), w.max(), "gersh", np.abs(np.eye(m) + K).sum(axis=1).max(), flush=True)
for name, args in (("manual pad, even path", (Ap, B, X0p, 2, rx)), ("odd path", (A, B, X0, tx, rx))):
    try:
        res = infer_admm_host(*args, variant="A2only")
        print(name, "ok", res.iters.tolist(), flush=True)
    except Exception as e:
        print(name, "error", e, flush=True)
