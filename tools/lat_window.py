"""Window-mode latency breakdown for one 10 s clip (6 x 5 s windows in one
launch): wall p50 and per-stage device times, both precisions.
    python tools/lat_window.py [reps]"""
import ctypes
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
import bench  # noqa: E402
import numpy as np  # noqa: E402
import torch  # noqa: E402
from sedx import _lib, inference, synth  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
dev = torch.device('cuda:0')
w = torch.from_numpy(synth.make_waveforms(1, seconds=10.0, sample_rate=16000, seed=11)).to(dev)
m = bench.build_model('Cnn_9layers_Gru_FrameAtt', dev)
nat, L = m.native(dev), _lib.lib()
for prec in ('exact', 'x3'):
    m.set_precision(prec)
    with torch.no_grad():
        for _ in range(5):
            inference.predict_windows(m, w, 5, 1)
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            a = time.perf_counter()
            inference.predict_windows(m, w, 5, 1)
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - a) * 1e3)
        _lib.check(L.sedx_set_profiling(nat.h, 1), nat.h, 'set_profiling')
        acc = np.zeros(len(_lib.STAGES))
        for _ in range(reps):
            inference.predict_windows(m, w, 5, 1)
            ms = (ctypes.c_float * len(_lib.STAGES))()
            n = ctypes.c_int32()
            _lib.check(L.sedx_stage_times(nat.h, ms, len(_lib.STAGES), ctypes.byref(n)), nat.h, 'stage_times')
            acc += np.array(ms[:])
        _lib.check(L.sedx_set_profiling(nat.h, 0), nat.h, 'set_profiling')
    st = {s: round(float(v), 4) for s, v in zip(_lib.STAGES, acc / reps)}
    print(prec, 'window p50 %.4f ms' % statistics.median(ts), 'stages sum %.4f' % sum(st.values()), st, flush=True)
