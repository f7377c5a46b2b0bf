"""A/B of the n_fft 512 frontend's mel path (SEDX_TUNE_MEL_MFMA 1 / 0):
per-stage HIP-event time of the frontend stage, one batch at a time,
alternating rounds.  python tools/fe_ab.py [B]"""
import os
import sys

sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__)))]
import bench  # noqa: E402
import torch  # noqa: E402
from sedx import _lib, synth  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
dev = torch.device('cuda', 0)
m = bench.build_model(bench.MODEL_NAMES['gru'], dev)
wave = torch.from_numpy(synth.make_waveforms(B, 10.0, 16000, seed=1)).to(dev)
for r in range(3):
    for on in (1, 0):
        m.set_tuning(_lib.TUNE_MEL_MFMA, on)
        st = bench.stage_times_isolated(m, wave, dev, 20)
        print('round %d mel_mfma=%d B=%d frontend %.4f ms' % (r, on, B, st['frontend']), flush=True)
