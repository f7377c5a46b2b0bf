"""Save a fixed forward's outputs (both models, both precisions, B=1 and B=32)
for bit-exactness checks between two builds of the package:
    python tools/ab_outputs.py out.npz --ab-package <pkg dir>
    python tools/ab_outputs.py --compare a.npz b.npz"""
import os
import sys

if sys.argv[1] == '--compare':
    import numpy as np
    a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
    bad = 0
    for k in a.files:
        eq = np.array_equal(a[k], b[k])
        d = float(np.max(np.abs(a[k].astype(np.float64) - b[k]))) if a[k].shape == b[k].shape else float('nan')
        print('%-40s %s  max|d| %.3g' % (k, 'IDENTICAL' if eq else 'DIFFERENT', d))
        bad += not eq
    sys.exit(1 if bad else 0)

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
import bench  # noqa: E402  (honours --ab-package in sys.argv)
import numpy as np  # noqa: E402
import torch  # noqa: E402
from sedx import synth  # noqa: E402

dev = torch.device('cuda:0')
out = {}
for name in ('Cnn_9layers_Gru_FrameAtt', 'Cnn_9layers_Transformer_FrameAtt'):
    m = bench.build_model(name, dev)
    for prec in ('exact', 'x3'):
        m.set_precision(prec)
        for B in (1, 32):
            w = torch.from_numpy(synth.make_waveforms(B, seconds=10.0, sample_rate=16000, seed=77)).to(dev)
            with torch.no_grad():
                o = m(w)
            out['%s_%s_B%d' % (name[:16], prec, B)] = o['framewise_output'].cpu().numpy()
np.savez(sys.argv[1], **out)
print('saved', sys.argv[1], len(out))
