"""Frontend (log-mel) device time: per-stage HIP events of isolated B-clip
forwards (sedx_set_profiling mode 1), stage 0 averaged.
    python tools/fe_bench.py [B] [reps]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
import bench  # noqa: E402
import torch  # noqa: E402
from sedx import synth  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
dev = torch.device('cuda:0')
w = torch.from_numpy(synth.make_waveforms(B, seconds=10.0, sample_rate=16000, seed=3)).to(dev)
m = bench.build_model('Cnn_9layers_Gru_FrameAtt', dev)
for prec in ('exact',):
    m.set_precision(prec)
    with torch.no_grad():
        m(w)
    st = bench.stage_times_isolated(m, w, dev, reps)
    ms = st['frontend']
    gbps = B * bench.FRONTEND_BYTES_PER_CLIP / (ms * 1e-3) / 1e9
    print('B=%d frontend %.4f ms  %.1f GB/s  (%.3f of 8 TB/s)' % (B, ms, gbps, gbps / 8000), flush=True)
