"""Phase timestamps of pgk_kernel (private phase-code path): run with ACE_LIB=tools/libace_stamps_pc.so
(built with EXTRA=-DACE_PHASE_STAMPS); prints per-phase durations (10 ns ticks) of work-group 5."""
import sys, pathlib
ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "2ace-mmwave-channel-estimation_amd"))
import torch
from ace_amd import infer_admm_batch, synth_problem
A, B, X0, _ = synth_problem(7, 0, 4096, 256, 32, 32, a_shared=False)
infer_admm_batch(A, B, X0, 32, 32, maxiter=12, fixed_iters=True)
torch.cuda.synchronize()
