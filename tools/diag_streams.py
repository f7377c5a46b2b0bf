"""Diagnostic: outputs of forwards issued on two streams vs one at a time.

usage (GPU box): python tools/diag_streams.py [gru|trf] [x3|exact]
Environment switches read by libsedx: SEDX_GRU_GLOBAL_ONLY=1 (GRU hand-off
through the global protocol only), SEDX_GRU_SIMPLE=1 (per-(clip, dir) GRU).
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.environ.get('SEDX_PKG', os.path.join(REPO, 'sound-event-detection_amd'))]

import torch  # noqa: E402

from sedx import models, synth  # noqa: E402

NAMES = {'gru': 'Cnn_9layers_Gru_FrameAtt', 'trf': 'Cnn_9layers_Transformer_FrameAtt'}


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else 'gru'
    prec = sys.argv[2] if len(sys.argv) > 2 else 'x3'
    name = NAMES[which]
    m = getattr(models, name)(16000, 512, 160, 64, 25, 7000, 25, 'logmel')
    sd = m.state_dict()
    for k, v in synth.make_state_dict(name, seed=0).items():
        sd[k] = torch.from_numpy(v)
    m.load_state_dict(sd)
    m = m.cuda().eval().set_precision(prec)
    waves = [torch.from_numpy(synth.make_waveforms(32, 10.0, 16000, seed=s)).cuda() for s in (5, 6, 7, 8)]
    keys = ('framewise_output', 'clipwise_output', 'embedding')
    with torch.no_grad():
        ref = [{k: v.clone() for k, v in m(w).items()} for w in waves]
        torch.cuda.synchronize()
        again = [{k: v.clone() for k, v in m(w).items()} for w in waves]
        torch.cuda.synchronize()
        d1 = max(float((a[k] - b[k]).abs().max()) for a, b in zip(again, ref) for k in keys)
        print('%s %s env=%s: serial repeat max|d| = %.3g' % (
            which, prec, {k: v for k, v in os.environ.items() if k.startswith('SEDX')}, d1))
        streams = [torch.cuda.Stream(), torch.cuda.Stream()]
        worst = 0.0
        for rep in range(5):
            outs = []
            for i, w in enumerate(waves):
                with torch.cuda.stream(streams[i % 2]):
                    outs.append(m(w))
            torch.cuda.synchronize()
            for i, (a, b) in enumerate(zip(outs, ref)):
                d = {k: float((a[k] - b[k]).abs().max()) for k in keys}
                worst = max(worst, max(d.values()))
                if max(d.values()) > 0:
                    bad = (a['framewise_output'] - b['framewise_output']).abs().amax(dim=2)  # [B, T]
                    clips = torch.nonzero(bad.amax(dim=1) > 0).flatten().tolist()
                    frames = torch.nonzero(bad.amax(dim=0) > 0).flatten().tolist()
                    print('  rep %d batch %d: %s clips %s frames %d..%d (%d)' % (
                        rep, i, {k: '%.3g' % v for k, v in d.items()}, clips[:8],
                        frames[0] if frames else -1, frames[-1] if frames else -1, len(frames)))
        print('%s %s two streams: worst max|d| = %.3g' % (which, prec, worst))


if __name__ == '__main__':
    main()
