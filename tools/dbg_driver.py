"""Diagnostic: driver vs hand composition vs oracle on one trace (prints errors)."""
import math
import sys

import numpy as np

sys.path.insert(0, "oracle")
sys.path.insert(0, "2ace-mmwave-channel-estimation_amd")
sys.path.insert(0, "tests")
import ace_oracle as O  # noqa: E402
from ace_amd import engine, infer_low_rank_pipeline_host  # noqa: E402
from test_gpu_driver import _trace, RSS_FCT  # noqa: E402

tx = 16
amp, ang, rss = _trace(400, tx)
seed = 58659179
Ms = [121, 225]
Ha, Hp = engine.recover(engine.DRIVER_A2ONLY, tx, tx, amp, ang, rss, 1, M_list=Ms)
H = np.squeeze(Ha * np.exp(1j * Hp))
for i, M in enumerate(Ms):
    idx = engine.randperm(seed, 0x100 + 2 * i, 400, M)
    A = (amp * np.exp(1j * ang))[idx]
    B = np.array([math.sqrt(math.pow(10.0, x / 10.0) / 1000.0) * RSS_FCT for x in rss[idx]])
    mt = math.floor(0.95 * M)
    tr = np.stack([engine.randperm(seed, 0x101 + 2 * i + 0x10000 * s, M, mt) for s in range(3)])
    res = infer_low_rank_pipeline_host(A, B[None], tx, tx, tr)
    ref = O.infer_low_rank_pipeline(A, B, tx, tx, list(tr))
    print(M, "gpu iters", res.stage_iters[0].tolist(), "q", res.quality[0])
    print(M, "ora iters", ref.stage_iters, "q", ref.quality)
    print(M, "driver-vs-comp %.2e" % O.phase_aligned_rel_err(H[i], res.X[0] / RSS_FCT),
          "comp-vs-oracle %.2e" % O.phase_aligned_rel_err(res.X[0], ref.X),
          "bitwise", np.array_equal(H[i], res.X[0] / RSS_FCT))
