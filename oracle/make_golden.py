"""Generate the golden fixtures in ``tests/golden/`` by running the REFERENCE
(``/root/reference``, Python) in this build container.

Test infrastructure only.  The reference is imported read-only with
``sys.dont_write_bytecode`` and the test-only stand-ins in ``oracle/refshim``
(librosa filter design / power_to_db restated; sed_eval / h5py / prettytable
empty) — SURVEY.md §8(c), Appendix B.  ``pytorch/predict.py`` and
``pytorch/main_strong.py`` are not importable (speech_recognition, dicttoxml,
h5py), so their driver loops are re-run here by calling the reference's own
``models``, ``utilities.merge / avg_merge`` and
``utilities.frame_prediction_to_event_prediction_v2``.

The threshold pickles under ``opt_thresholds/`` are NOT used: the safe loader
(``torch.load(weights_only=True)``) refuses them, so the events goldens use
the reference's default parameters plus a synthetic per-class threshold table.

Usage:  python oracle/make_golden.py   (writes tests/golden/*.npz, *.json)
"""
import json
import os
import sys

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
REF = os.environ.get('SEDX_REFERENCE', '/root/reference')
sys.path[:0] = [os.path.join(HERE, 'refshim'), os.path.join(REF, 'pytorch'), os.path.join(REF, 'utils')]
sys.path.append(os.path.join(REPO, 'sound-event-detection_amd'))

import numpy as np  # noqa: E402
import torch  # noqa: E402

torch.set_num_threads(8)
torch.manual_seed(0)

import models as ref_models  # noqa: E402  (reference)
import utilities as ref_util  # noqa: E402  (reference)
import vad as ref_vad  # noqa: E402  (reference)
import gammatone.fftweight as ref_gt  # noqa: E402  (reference)
import librosa  # noqa: E402  (refshim)

from sedx import synth  # noqa: E402

OUT = os.path.join(REPO, 'tests', 'golden')
GRU, TRF = 'Cnn_9layers_Gru_FrameAtt', 'Cnn_9layers_Transformer_FrameAtt'
SEEDS = {GRU: 0, TRF: 1}
P16 = (16000, 512, 160, 64, 25, 7000)
P32 = (32000, 1024, 320, 64, 50, 14000)


def build(model_type, preset=P16, feature_type='logmel'):
    m = getattr(ref_models, model_type)(*preset, 25, feature_type).eval()
    sd = m.state_dict()
    for k, v in synth.make_state_dict(model_type, seed=SEEDS[model_type]).items():
        assert k in sd and tuple(sd[k].shape) == v.shape, k
        sd[k] = torch.from_numpy(v)
    m.load_state_dict(sd, strict=True)
    return m


def stages(m, model_type, x=None, feats=None):
    """Run the reference submodules one by one (models.py:625-688 /
    :1029-1077) recording every intermediate."""
    out = {}
    with torch.no_grad():
        if feats is None:
            x = m.logmel_extractor(m.spectrogram_extractor(x))
        else:
            x = feats
        out['logmel'] = x
        x = m.bn0(x.transpose(1, 3)).transpose(1, 3)
        out['bn0'] = x
        for k, pool in ((1, (2, 2)), (2, (2, 2)), (3, (2, 2)), (4, (1, 1))):
            x = getattr(m, 'conv_block%d' % k)(x, pool_size=pool, pool_type='avg')
            out['block%d' % k] = x
        x = torch.mean(x, dim=3)
        out['cnn_out'] = x
        x = x.transpose(1, 2)
        x = m.gru(x)[0] if model_type == GRU else m.multihead(x, x, x)
        out['seq_out'] = x
        x = x.transpose(1, 2)
        clip, norm_att, cla = m.att_block(x)
        out['norm_att'] = norm_att
        fw = ref_models.interpolate(cla.transpose(1, 2), 8)
        if model_type == GRU and fw.size()[1] != 1000:
            fw = ref_models.pad_framewise_output(fw, ref_models.roundup(fw.size()[1]))
        out['framewise_output'] = fw
        out['clipwise_output'] = clip
        out['embedding'] = cla if model_type == GRU else x
    return {k: v.numpy().astype(np.float32) for k, v in out.items()}


def synthetic_params(seed=7):
    rng = np.random.default_rng(seed)
    hi = rng.uniform(0.25, 0.55, 25)
    lo = hi - rng.uniform(0.05, 0.35, 25)
    lo[3] = -0.12        # negative low threshold (GRU 16k pickle has one): edge extension
    return {'audio_tagging_threshold': [0.1] * 25, 'sed_high_threshold': hi.tolist(),
            'sed_low_threshold': lo.tolist(), 'n_smooth': 10, 'n_salt': 10}


DEFAULT_PREDICT = {'audio_tagging_threshold': 0.099, 'sed_high_threshold': 0.5,
                   'sed_low_threshold': 0.3, 'n_smooth': 10, 'n_salt': 10}   # predict.py:252-257


def windowed(m, audio, sr, sample_duration, overlap_value, driver='predict', overlap=True, audio_duration=None):
    """The reference drivers' window loops line for line, around the
    reference's own model, merge and avg_merge:
      driver='predict'      pytorch/predict.py:277-349 — every window
                            pad_truncate'd to sample_duration s (:263, :305);
                            ``start += 1`` with --overlap, else ``start +=
                            sample_duration`` (:334-337)
      driver='main_strong'  pytorch/main_strong.py:778-832 — the clip
                            pad_truncate'd to 10 s (:761, :790), windows
                            sliced without padding (:795-797), ``start +=
                            overlap_value`` (:829)
    audio_duration stands for librosa.get_duration(filename) (predict.py:277,
    main_strong.py:778): the file's own length."""
    if audio_duration is None:
        audio_duration = len(audio) / float(sr)
    audio_full = ref_util.pad_truncate_sequence(audio, sr * 10) if driver == 'main_strong' else audio
    audio_samples = sr * sample_duration
    num_segment, start, end, merged, prev = 1, 0, 0, None, None
    while end <= audio_duration:
        start_index = int(start * sr)
        end_index = int((sample_duration * sr) + start_index)
        seg = audio_full[start_index:end_index]
        if driver == 'predict':
            seg = ref_util.pad_truncate_sequence(seg, audio_samples)
        seg = torch.Tensor(seg)
        seg = torch.reshape(seg, (1, seg.size()[0]))
        with torch.no_grad():
            curr = m(seg)['framewise_output'].data.cpu().numpy()
        if num_segment == 2:
            merged = ref_util.merge(prev, curr, sample_duration, num_segment, overlap_value)
        elif num_segment > 2:
            merged = ref_util.merge(merged, curr, sample_duration, num_segment, overlap_value)
        else:
            merged = curr
        prev = curr
        if driver == 'predict':
            start += 1 if overlap else sample_duration
        else:
            start += overlap_value
        end = start + sample_duration
        num_segment += 1
    return ref_util.avg_merge(merged, sample_duration, overlap_value)


def events(merged, params):
    ev = ref_util.frame_prediction_to_event_prediction_v2(
        merged, 'test', {k: (list(v) if isinstance(v, list) else v) for k, v in params.items()}, 100)
    return sorted(ev, key=lambda k: k['onset'])


def main():
    os.makedirs(OUT, exist_ok=True)
    meta = {'generator': 'oracle/make_golden.py', 'reference': REF,
            'weights': 'sedx.synth.make_state_dict(model_type, seed={GRU:0, Transformer:1})',
            'waves': 'sedx.synth.make_waveforms(B, seconds, sr, seed)'}

    # --- frontend construction (stft.py:157-221, :688-692) ---
    fr = {}
    for q, p in (('8k', (8000, 256, 80, 64, 12, 3500)), ('16k', P16), ('32k', P32)):
        m = ref_models.Cnn_9layers_Gru_FrameAtt(*p, 25, 'logmel')
        fr['melW_' + q] = m.logmel_extractor.melW.detach().numpy()
        rows = np.array([0, 1, 2, 3, p[1] // 8, p[1] // 4, p[1] // 2 - 1, p[1] // 2])
        fr['conv_real_rows_' + q] = m.spectrogram_extractor.stft.conv_real.weight.detach().numpy()[rows, 0]
        fr['conv_imag_rows_' + q] = m.spectrogram_extractor.stft.conv_imag.weight.detach().numpy()[rows, 0]
        fr['rows_' + q] = rows
    np.savez_compressed(os.path.join(OUT, 'frontend.npz'), **fr)

    # --- per-stage goldens, short clip, both models ---
    short = synth.make_waveforms(2, seconds=5280 / 16000., sample_rate=16000, seed=11)
    for mt in (GRU, TRF):
        m = build(mt)
        st = stages(m, mt, x=torch.from_numpy(short))
        with torch.no_grad():
            o = m(torch.from_numpy(short))
        for k in ('framewise_output', 'clipwise_output', 'embedding'):
            assert np.array_equal(o[k].numpy(), st[k]), k
        np.savez_compressed(os.path.join(OUT, 'stages_%s.npz' % mt), wave=short, **st)

    # --- odd-length ragged clip (T odd at every pooling level) ---
    rag = synth.make_waveforms(1, seconds=7777 / 16000., sample_rate=16000, seed=12)
    for mt in (GRU, TRF):
        m = build(mt)
        with torch.no_grad():
            o = m(torch.from_numpy(rag))
        np.savez_compressed(os.path.join(OUT, 'ragged_%s.npz' % mt), wave=rag,
                            **{k: v.numpy() for k, v in o.items()})

    # --- full 10 s clips, B=2 (clip mode, main_strong inference_prob) ---
    full = synth.make_waveforms(2, seconds=10.0, sample_rate=16000, seed=1234)
    for mt in (GRU, TRF):
        m = build(mt)
        with torch.no_grad():
            o = m(torch.from_numpy(full))
        np.savez_compressed(os.path.join(OUT, 'clip10s_%s.npz' % mt),
                            **{k: v.numpy() for k, v in o.items()})

    # --- windowed 10 s (predict.py semantics) + events ---
    ev_out = {'params_default': DEFAULT_PREDICT, 'params_synthetic': synthetic_params()}
    for mt in (GRU, TRF):
        m = build(mt)
        audio = full[0].astype(np.float32)
        merged = windowed(m, audio, 16000, 5, 1, 'predict', overlap=True)       # run.sh's predict.py call
        merged_ms = windowed(m, audio, 16000, 6, 0.5, 'main_strong')           # main_strong sweep setting
        np.savez_compressed(os.path.join(OUT, 'windowed_%s.npz' % mt),
                            merged_5_1=merged, merged_6_05=merged_ms)
        ev_out[mt] = {'default': events(merged.copy(), DEFAULT_PREDICT),
                      'synthetic': events(merged.copy(), synthetic_params())}
    with open(os.path.join(OUT, 'events.json'), 'w') as f:
        json.dump(ev_out, f, indent=0)

    # --- merge / avg_merge known answers (all-ones windows; Appendix F) ---
    mk = {}
    for (dur, ov, n_frames) in ((5, 1, 500), (5, 1, 496), (6, 0.5, 600), (7, 0.5, 700),
                                (6, 1, 600), (7, 1, 700)):
        nwin = len(np.arange(0, 10 - dur + 1e-9, ov))
        merged = None
        prev = None
        for s in range(1, nwin + 1):
            curr = np.ones((1, n_frames, 2), np.float32)
            if s == 1:
                merged = curr
            elif s == 2:
                merged = ref_util.merge(prev, curr, dur, s, ov)
            else:
                merged = ref_util.merge(merged, curr, dur, s, ov)
            prev = curr
        mk['d%s_o%s_n%d' % (dur, ov, n_frames)] = ref_util.avg_merge(merged, dur, ov)[0, :, 0]
    np.savez_compressed(os.path.join(OUT, 'merge_kat.npz'), **mk)

    # --- vad known answers (utils/vad.py) ---
    rng = np.random.default_rng(5)
    kat = []
    x40 = np.zeros(40)
    x40[2:5] = 0.6
    x40[10:12] = 0.6
    x40[12:14] = 0.35
    x40[30] = 0.9
    cases = [(x40, 0.5, 0.3, 0, 0), (x40, 0.5, 0.3, 10, 10), (x40, 0.5, 0.7, 0, 0),
             (x40, 0.5, -0.1, 0, 0), (x40, 0.5, None, 1, 0), (np.zeros(10), 0.5, 0.3, 1, 0),
             (np.ones(10), 0.5, 0.3, 1, 0)]
    for _ in range(40):
        x = np.clip(np.convolve(rng.uniform(0, 1, 300), np.ones(7) / 7, mode='same')
                    + rng.normal(0, 0.08, 300), 0, 1)
        hi = float(rng.uniform(0.3, 0.7))
        lo = float(hi - rng.uniform(-0.05, 0.3))
        cases.append((x, hi, lo, int(rng.integers(0, 12)), int(rng.integers(0, 12))))
    for x, hi, lo, ns, nsalt in cases:
        pairs = ref_vad.activity_detection(x, hi, lo, ns, nsalt)
        kat.append({'x': np.asarray(x, np.float64).tolist(), 'thres': hi, 'low_thres': lo,
                    'n_smooth': ns, 'n_salt': nsalt,
                    'pairs': [[int(a), int(b)] for a, b in pairs]})
    kat.append({'find_bgn_fin_pairs': [2, 3, 4, 10, 11],
                'pairs': [[int(a), int(b)] for a, b in ref_vad.find_bgn_fin_pairs([2, 3, 4, 10, 11])]})
    with open(os.path.join(OUT, 'vad_kat.json'), 'w') as f:
        json.dump(kat, f)

    # --- gammatone frontend (32k) + gamma-branch forward ---
    g_audio = synth.make_waveforms(2, seconds=10.0, sample_rate=32000, seed=77)
    gt, g_feats = [], []
    for b in range(2):
        a = ref_util.pad_truncate_sequence(g_audio[b], 320000)
        g = ref_gt.fft_gtgram(a, 32000, 1024 / 32000, 320 / 32000, 64, 50)
        gt.append(g)
        db = librosa.core.power_to_db(g)
        g_feats.append(ref_util.int16_to_float32(ref_util.float32_to_int16(db)))
    g_feats = np.stack(g_feats)                      # [B, 64, 994]
    m = build(GRU, preset=P32, feature_type='gamma')
    x = torch.from_numpy(g_feats).unsqueeze(1).transpose(2, 3)   # models.py:637-639 (sans .to('cuda'))
    st = stages(m, GRU, feats=x)
    q = np.round(g_feats.astype(np.float64) * 32767.).astype(np.int16)      # exact int16 codes
    assert np.array_equal(ref_util.int16_to_float32(q), g_feats)
    np.savez_compressed(os.path.join(OUT, 'gamma_%s.npz' % GRU), gtgram=np.stack(gt).astype(np.float32),
                        features_int16=q, framewise_output=st['framewise_output'],
                        clipwise_output=st['clipwise_output'], embedding=st['embedding'])
    with open(os.path.join(OUT, 'meta.json'), 'w') as f:
        json.dump(meta, f, indent=1)
    print('golden written to', OUT)


if __name__ == '__main__':
    main()
