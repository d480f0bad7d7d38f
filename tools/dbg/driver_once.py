"""One drop-in driver call on the reference probe codebook (for kernel traces of the latency path)."""
import os, sys, time
sys.path[:0] = ['.', '2ace-mmwave-channel-estimation_amd']
import numpy as np
import bench
from ace_amd import engine
amp, ang, rss = bench.driver_trace(16, 17)
eng = engine.start_matlab()
for k in range(3):
    t0 = time.perf_counter()
    Ha, Hp = eng.channel_recovery_ADMM_v2_simulation_A2only(16, 16, engine.double(amp), engine.double(ang),
                                                           engine.double(rss[:, None]), eng.double(3), nargout=2)
    print("call", k, round(time.perf_counter() - t0, 4), "s", flush=True)
