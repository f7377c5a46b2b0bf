"""Diagnostic: which combination of concurrent forwards perturbs outputs.

Stream 0 runs model P (precision p0), stream 1 model Q (precision p1); P and
Q are the same handle or two instances.  Reports max|d| of every forward
against its own serial reference.
usage: python tools/diag_streams2.py gru|trf
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, 'sound-event-detection_amd')]

import torch  # noqa: E402

from sedx import models, synth  # noqa: E402

NAMES = {'gru': 'Cnn_9layers_Gru_FrameAtt', 'trf': 'Cnn_9layers_Transformer_FrameAtt'}


def build(name):
    m = getattr(models, name)(16000, 512, 160, 64, 25, 7000, 25, 'logmel')
    sd = m.state_dict()
    for k, v in synth.make_state_dict(name, seed=0).items():
        sd[k] = torch.from_numpy(v)
    m.load_state_dict(sd)
    return m.cuda().eval()


def trial(tag, mods, precs, waves, reps=6):
    for m, p in zip(mods, precs):
        m.set_precision(p)
    with torch.no_grad():
        refs = []
        for i, w in enumerate(waves):
            m = mods[i % 2]
            m.set_precision(precs[i % 2])
            refs.append(m(w)['framewise_output'].clone())
        torch.cuda.synchronize()
        streams = [torch.cuda.Stream(), torch.cuda.Stream()]
        worst = [0.0, 0.0]
        for _ in range(reps):
            outs = []
            for i, w in enumerate(waves):
                with torch.cuda.stream(streams[i % 2]):
                    outs.append(mods[i % 2](w)['framewise_output'])
            torch.cuda.synchronize()
            for i, (a, b) in enumerate(zip(outs, refs)):
                worst[i % 2] = max(worst[i % 2], float((a - b).abs().max()))
    print('%-40s stream0 (%s) worst %.3g | stream1 (%s) worst %.3g' % (tag, precs[0], worst[0], precs[1],
                                                                        worst[1]), flush=True)


def main():
    name = NAMES[sys.argv[1] if len(sys.argv) > 1 else 'gru']
    a = build(name)
    b = build(name)
    waves = [torch.from_numpy(synth.make_waveforms(32, 10.0, 16000, seed=s)).cuda() for s in (5, 6, 7, 8)]
    trial('same handle, x3 | x3', [a, a], ['x3', 'x3'], waves)
    trial('two handles, x3 | x3', [a, b], ['x3', 'x3'], waves)
    trial('two handles, x3 | exact', [a, b], ['x3', 'exact'], waves)
    trial('two handles, exact | exact', [a, b], ['exact', 'exact'], waves)


if __name__ == '__main__':
    main()
