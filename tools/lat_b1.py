"""B=1 latency breakdown: per-stage device times (sedx_set_profiling mode 1)
and the wall-clock p50 of one 10 s clip, both precisions and both models.
    python tools/lat_b1.py [reps]"""
import os
import sys
import time
import statistics

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
import bench  # noqa: E402
import torch  # noqa: E402
from sedx import synth  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
dev = torch.device('cuda:0')
w = torch.from_numpy(synth.make_waveforms(1, seconds=10.0, sample_rate=16000, seed=11)).to(dev)
for name in ('Cnn_9layers_Gru_FrameAtt', 'Cnn_9layers_Transformer_FrameAtt'):
    m = bench.build_model(name, dev)
    for prec in ('exact', 'x3'):
        m.set_precision(prec)
        with torch.no_grad():
            for _ in range(5):
                m(w)
            torch.cuda.synchronize()
            ts = []
            for _ in range(reps):
                a = time.perf_counter()
                m(w)
                torch.cuda.synchronize()
                ts.append((time.perf_counter() - a) * 1e3)
        st = bench.stage_times_isolated(m, w, dev, reps)
        print(name, prec, 'p50 %.4f ms' % statistics.median(ts), 'stages sum %.4f' % sum(st.values()), st,
              flush=True)
