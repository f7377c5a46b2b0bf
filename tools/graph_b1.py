"""B=1 latency: eager forward vs the same forward captured in a HIP graph
(torch.cuda.graph around the libsedx launches) and replayed.
    python tools/graph_b1.py"""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
import bench  # noqa: E402
import torch  # noqa: E402
from sedx import synth  # noqa: E402

dev = torch.device('cuda:0')
w = torch.from_numpy(synth.make_waveforms(1, seconds=10.0, sample_rate=16000, seed=11)).to(dev)
for name in ('Cnn_9layers_Gru_FrameAtt', 'Cnn_9layers_Transformer_FrameAtt'):
    m = bench.build_model(name, dev)
    static_in = w.clone()
    s = torch.cuda.Stream(dev)
    with torch.no_grad(), torch.cuda.stream(s):
        for _ in range(3):
            ref = m(static_in)['framewise_output'].clone()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            out = m(static_in)
    torch.cuda.synchronize()

    def timeit(fn, reps=50):
        ts = []
        for _ in range(reps):
            torch.cuda.synchronize()
            a = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - a) * 1e3)
        return statistics.median(ts)
    with torch.no_grad():
        eager = timeit(lambda: m(static_in))
    g.replay()
    torch.cuda.synchronize()
    same = torch.equal(out['framewise_output'], ref)
    graph = timeit(g.replay)
    print('%s B=1: eager p50 %.4f ms, graph replay p50 %.4f ms, outputs identical: %s' % (name, eager, graph, same),
          flush=True)
