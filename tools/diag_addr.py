"""Diagnostic: do outputs depend on where the workspace / outputs live?
Serial forwards on one stream with differently-sized live dummy tensors in
between, so the caching allocator hands out different addresses.
usage: python tools/diag_addr.py gru|trf [x3|exact]
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
    wave = torch.from_numpy(synth.make_waveforms(32, 10.0, 16000, seed=5)).cuda()
    keep = []
    with torch.no_grad():
        ref = {k: v.clone() for k, v in m(wave).items()}
        for i in range(12):
            keep.append(torch.empty(int(1 + 37 * i) * 4096 + 512 * i, dtype=torch.uint8, device='cuda'))
            if i % 3 == 2:                       # fragment: drop some, keep others
                keep.pop(0)
            o = m(wave)
            torch.cuda.synchronize()
            d = {k: float((o[k] - ref[k]).abs().max()) for k in ref}
            print('%s %s shift %2d: ws@%s max|d| %s' % (name, prec, i, hex(o['framewise_output'].data_ptr()),
                                                        {k: '%.3g' % v for k, v in d.items()}), flush=True)


if __name__ == '__main__':
    main()
