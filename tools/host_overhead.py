"""Host-side cost of one forward: time to return from model(w) (launches
issued) vs to completion, and the C ABI call alone (sedx_forward via ctypes).
    python tools/host_overhead.py [batch]   (default 1 clip of 10 s)"""
import os
import sys
import time
import statistics

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
import bench  # noqa: E402
import torch  # noqa: E402
from sedx import synth  # noqa: E402

dev = torch.device('cuda:0')
B = int(sys.argv[1]) if len(sys.argv) > 1 else 1
w = torch.from_numpy(synth.make_waveforms(B, seconds=10.0, sample_rate=16000, seed=11)).to(dev)
m = bench.build_model('Cnn_9layers_Gru_FrameAtt', dev)
with torch.no_grad():
    for _ in range(10):
        m(w)
    torch.cuda.synchronize()
    ret, tot, gpu = [], [], []
    for _ in range(50):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        a = time.perf_counter()
        e0.record()
        m(w)
        e1.record()
        b = time.perf_counter()
        torch.cuda.synchronize()
        c = time.perf_counter()
        ret.append((b - a) * 1e3)
        tot.append((c - a) * 1e3)
        gpu.append(e0.elapsed_time(e1))
print('model(w) returns after %.3f ms (launches issued), done after %.3f ms; device events %.3f ms (p50)' %
      (statistics.median(ret), statistics.median(tot), statistics.median(gpu)))
