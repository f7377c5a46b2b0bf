"""Diagnostic: sedx forwards on stream 0 while stream 1 runs unrelated torch
work (GEMMs + elementwise) — do stream-0 outputs stay bit-identical?
usage: python tools/diag_streams3.py gru|trf [x3|exact]
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, 'sound-event-detection_amd')]

import torch  # noqa: E402

from sedx import models, synth  # noqa: E402

NAMES = {'gru': 'Cnn_9layers_Gru_FrameAtt', 'trf': 'Cnn_9layers_Transformer_FrameAtt'}


def main():
    name = NAMES[sys.argv[1] if len(sys.argv) > 1 else 'gru']
    prec = sys.argv[2] if len(sys.argv) > 2 else 'x3'
    m = getattr(models, name)(16000, 512, 160, 64, 25, 7000, 25, 'logmel')
    sd = m.state_dict()
    for k, v in synth.make_state_dict(name, seed=0).items():
        sd[k] = torch.from_numpy(v)
    m.load_state_dict(sd)
    m = m.cuda().eval().set_precision(prec)
    waves = [torch.from_numpy(synth.make_waveforms(32, 10.0, 16000, seed=s)).cuda() for s in (5, 6, 7, 8)]
    a = torch.randn(4096, 4096, device='cuda')
    with torch.no_grad():
        refs = [m(w)['framewise_output'].clone() for w in waves]
        torch.cuda.synchronize()
        s0, s1 = torch.cuda.Stream(), torch.cuda.Stream()
        worst = 0.0
        nbad = 0
        for rep in range(8):
            outs = []
            with torch.cuda.stream(s1):
                x = a
                for _ in range(40):
                    x = torch.tanh(x @ a * 1e-3)
            with torch.cuda.stream(s0):
                for w in waves:
                    outs.append(m(w)['framewise_output'])
            torch.cuda.synchronize()
            for o, r in zip(outs, refs):
                d = float((o - r).abs().max())
                worst = max(worst, d)
                nbad += d > 0
    print('%s %s vs unrelated torch work on stream 1: %d of 32 forwards differ, worst %.3g'
          % (name, prec, nbad, worst), flush=True)


if __name__ == '__main__':
    main()
