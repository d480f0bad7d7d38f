"""Debug: the driver's sweep points on the reference probe codebook, one by one through the
pipeline host API and through the driver in serial mode."""
import os, sys, math, numpy as np
sys.path[:0] = ['oracle', '2ace-mmwave-channel-estimation_amd', 'tests']
import ace_amd
from ace_amd import synth, engine, infer_low_rank_pipeline_host
from test_gpu_driver import _ref_codebook, _cb, SEEDS, RSS_FCT
tx = 16
k, amp, ang = _ref_codebook("random")
cb = (1j ** k).astype(complex)
h = synth.channel(17, 0, tx, tx)
rss = 10 * np.log10(1000 * (np.abs(cb @ h) * 1e-4) ** 2)
seed = SEEDS[2]
for i, M in enumerate(engine.m_sweep(tx, tx)):
    M = int(M); mt = math.floor(0.95 * M)
    if mt < min(20, M):
        continue
    idx = engine.randperm(seed, 0x100 + 2 * i, 3968, M)
    A = _cb(amp, ang)[idx]
    B = np.array([math.sqrt(math.pow(10.0, x / 10.0) / 1000.0) * RSS_FCT for x in rss[idx]])
    tr = np.stack([engine.randperm(seed, 0x101 + 2 * i + 0x10000 * s, M, mt) for s in range(3)])
    try:
        r = infer_low_rank_pipeline_host(A, B[None], tx, tx, tr)
        print("point", i, M, "finite", np.isfinite(r.X).all(), r.stage_iters[0].tolist(), flush=True)
    except Exception as e:
        print("point", i, M, "ERR", e, flush=True)
for ser in ("1", "0", "1"):
    os.environ["ACE_DRIVER_SERIAL"] = ser
    try:
        Ha, Hp = engine.recover(engine.DRIVER_A2ONLY, tx, tx, amp, ang, rss, 3)
        print("driver serial", ser, "zero rows", [i for i in range(8) if Ha[i].max() == 0], flush=True)
    except Exception as e:
        print("driver serial", ser, "ERR", e, flush=True)
