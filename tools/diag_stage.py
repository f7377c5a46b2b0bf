"""Diagnostic: localise a concurrency-dependent difference by reading the
intermediate buffers a forward leaves in its (caller-owned) workspace:
X0 (frontend + bn0 output), S (conv stack output = sequence input), H (GRU /
MHA-fc output) and the head logits, for forwards issued on two streams vs
serially.  Offsets follow ws_layout() in csrc/api.cpp (B=32, 10 s, 16 kHz).
usage: python tools/diag_stage.py gru|trf [x3|exact]
"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.environ.get('SEDX_PKG', os.path.join(REPO, 'sound-event-detection_amd'))]

import torch  # noqa: E402

from sedx import _lib, models, synth  # noqa: E402

NAMES = {'gru': 'Cnn_9layers_Gru_FrameAtt', 'trf': 'Cnn_9layers_Transformer_FrameAtt'}


def al(x):
    return (x + 63) & ~63


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
    B, L = 32, 160000
    T, T1, T2, T3 = 1001, 500, 250, 125
    M = B * T3
    nac = 64
    nat = m.native(torch.device('cuda', 0))
    two = os.environ.get('DIAG_TWO_HANDLES') == '1'
    if two:                                  # a second model instance = a second handle
        m2 = getattr(models, name)(16000, 512, 160, 64, 25, 7000, 25, 'logmel')
        m2.load_state_dict(sd)
        m2 = m2.cuda().eval().set_precision(prec)
        nat2 = m2.native(torch.device('cuda', 0))
    reps = int(os.environ.get('DIAG_REPS', '6'))
    quiet = os.environ.get('DIAG_QUIET') == '1'
    nbad = {'fw': 0, 'X0': 0}
    lib = _lib.lib()
    wsz = ctypes.c_size_t()
    lib.sedx_workspace_size(nat.h, B, L, ctypes.byref(wsz))
    x0 = 0
    bufA = x0 + al(B * T * 64)
    a = max(B * T * 64 * 64, B * T1 * 32 * 128, B * T2 * 16 * 256, B * T3 * 8 * 512)
    bufB = bufA + al(a + 0)  # a dominates the head term at this shape
    b = max(B * T1 * 32 * 64, B * T2 * 16 * 128, B * T3 * 8 * 256, B * T3 * 512)
    dbg = bufB + al(b) + al(7 * 256)
    regions = {'X0': (x0, B * T * 64), 'S': (bufB, M * 512),
               'H': (bufA + al(M * 1536), M * 512),
               'LG': (bufA + al(M * 1536) + 2 * al(M * 512), M * nac)}
    if os.environ.get('SEDX_DEBUG_X0'):
        regions['X0snap'] = (dbg, B * T * 64)

    def fwd(w, stream, h=None):
        fw = torch.empty((B, 1000, 25), device='cuda')
        clip = torch.empty((B, 25), device='cuda')
        emb = torch.empty((B, 25 if which == 'gru' else 512, T3), device='cuda')
        ws = torch.empty(wsz.value // 4, dtype=torch.float32, device='cuda')
        st = ctypes.c_void_p(stream.cuda_stream)
        p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
        hh = h if h is not None else nat.h
        _lib.check(lib.sedx_forward(hh, p(w), B, L, p(fw), p(clip), p(emb), p(ws), wsz.value, st),
                   hh, 'forward')
        return fw, ws

    waves = [torch.from_numpy(synth.make_waveforms(B, 10.0, 16000, seed=s)).cuda() for s in (5, 6, 7, 8)]
    dflt = torch.cuda.current_stream()
    refs = [fwd(w, dflt) for w in waves]
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    for rep in range(reps):
        outs = [fwd(w, streams[i % 2], nat2.h if (two and i % 2) else None) for i, w in enumerate(waves)]
        torch.cuda.synchronize()
        for i, ((fw, ws), (rfw, rws)) in enumerate(zip(outs, refs)):
            d = {'fw': float((fw - rfw).abs().max())}
            for k, (o, n) in regions.items():
                d[k] = float((ws[o:o + n] - rws[o:o + n]).abs().max())
            nbad['fw'] += d['fw'] > 0
            nbad['X0'] += d['X0'] > 0
            if d['X0'] > 0:
                # where do the corrupted X0 values come from?  compare with the
                # X0 of every batch (refs) at the same index
                o, n = regions['X0']
                cur = ws[o:o + n]
                bad = torch.nonzero(cur != rws[o:o + n]).flatten()
                src = {}
                for j, (_, rws2) in enumerate(refs):
                    src['batch%d' % j] = int((cur[bad] == rws2[o:o + n][bad]).sum())
                for j, (_, ws2) in enumerate(outs):
                    if j != i:
                        src['live%d' % j] = int((cur[bad] == ws2[o:o + n][bad]).sum())
                fr = sorted(set((bad // 64).tolist()))
                print('   rep %d batch %d: %d bad X0 elements in %d frames %s; equal-at-same-index counts %s'
                      % (rep, i, bad.numel(), len(fr), [(f // T, f % T) for f in fr[:6]], src), flush=True)
                # is a bad frame some other frame's row (misplaced), in any batch?
                for f in fr[:3]:
                    row = cur[f * 64:(f + 1) * 64]
                    hits = []
                    for j, (_, rws2) in enumerate(refs):
                        allx = rws2[o:o + n].view(-1, 64)
                        eq = (allx == row[None, :]).sum(dim=1)
                        best = int(eq.argmax())
                        if int(eq[best]) >= 8:
                            hits.append(('batch%d' % j, best // T, best % T, int(eq[best])))
                    nref = int((row == rws[o + f * 64:o + (f + 1) * 64]).sum())
                    print('     frame (%d, %d): %d/64 mels still equal; best matches elsewhere %s'
                          % (f // T, f % T, nref, hits), flush=True)
            if any(v > 0 for v in d.values()) and not quiet:
                s0, sn = regions['S']
                ds = (ws[s0:s0 + sn] - rws[s0:s0 + sn]).abs().view(B, T3, 512).amax(dim=(1, 2))
                print('%s %s rep %d batch %d: %s  S-clips %s' % (which, prec, rep, i,
                      {k: '%.3g' % v for k, v in d.items()}, torch.nonzero(ds > 0).flatten().tolist()[:10]),
                      flush=True)
                o, n = regions['X0']
                dx = (ws[o:o + n] - rws[o:o + n]).view(B, T, 64)
                idx = torch.nonzero(dx != 0)
                print('   X0: %d elements differ; (clip, frame, mel) first %s last %s; frames per clip %s' % (
                    idx.shape[0], idx[:4].tolist(), idx[-4:].tolist(),
                    {int(c): (int(idx[idx[:, 0] == c][:, 1].min()), int(idx[idx[:, 0] == c][:, 1].max()),
                              int((idx[:, 0] == c).sum())) for c in idx[:, 0].unique()[:8]}), flush=True)
                for e in idx[:3].tolist():
                    print('     at %s: got %.6g ref %.6g' % (e, float(ws[o + (e[0] * T + e[1]) * 64 + e[2]]),
                                                           float(rws[o + (e[0] * T + e[1]) * 64 + e[2]])))
    print('%s %s handles=%d reps=%d: forwards with fw diff %d, with X0 diff %d (of %d)' % (
        which, prec, 2 if two else 1, reps, nbad['fw'], nbad['X0'], 4 * reps), flush=True)


if __name__ == '__main__':
    main()
