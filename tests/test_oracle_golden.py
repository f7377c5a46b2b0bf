"""Pin the CPU oracle (oracle/sed_oracle.py) against fixtures produced by the
reference itself (oracle/make_golden.py).  CPU only."""
import json
import os

import numpy as np
import pytest
import torch

from oracle import sed_oracle as O
from sedx import synth

GRU, TRF = 'Cnn_9layers_Gru_FrameAtt', 'Cnn_9layers_Transformer_FrameAtt'
SEEDS = {GRU: 0, TRF: 1}


def _sd(mt, preset='16k'):
    return O.full_state(synth.make_state_dict(mt, seed=SEEDS[mt]), preset)


def _close(a, b, tol, what=''):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    assert a.shape == b.shape, (what, a.shape, b.shape)
    err = np.max(np.abs(a - b)) / max(1.0, np.max(np.abs(b)))
    assert err <= tol, '%s: max rel err %.3g > %.3g' % (what, err, tol)


@pytest.mark.parametrize('q', ['8k', '16k', '32k'])
def test_frontend_construction(golden_dir, q):
    g = np.load(os.path.join(golden_dir, 'frontend.npz'))
    p = O.PRESETS[q]
    melW = O.mel_filterbank(p['sample_rate'], p['window_size'], p['mel_bins'], p['fmin'], p['fmax'])
    np.testing.assert_allclose(melW, g['melW_' + q], rtol=2e-6, atol=1e-9)
    wr, wi = O.stft_weights(p['window_size'])
    rows = g['rows_' + q]
    np.testing.assert_allclose(wr[rows, 0], g['conv_real_rows_' + q], atol=2e-7)
    np.testing.assert_allclose(wi[rows, 0], g['conv_imag_rows_' + q], atol=2e-7)


@pytest.mark.parametrize('mt', [GRU, TRF])
def test_stages(golden_dir, mt):
    g = np.load(os.path.join(golden_dir, 'stages_%s.npz' % mt))
    out, acts = O.forward(_sd(mt), mt, wave=g['wave'], return_acts=True)
    for k in ('logmel', 'bn0', 'block1', 'block2', 'block3', 'block4', 'cnn_out', 'seq_out',
              'norm_att'):
        _close(acts[k], g[k], 1e-5, k)
    for k in ('framewise_output', 'clipwise_output', 'embedding'):
        _close(out[k], g[k], 1e-5, k)


@pytest.mark.parametrize('mt', [GRU, TRF])
@pytest.mark.parametrize('kind', ['ragged', 'clip10s'])
def test_forward(golden_dir, mt, kind):
    g = np.load(os.path.join(golden_dir, '%s_%s.npz' % (kind, mt)))
    if kind == 'ragged':
        wave = synth.make_waveforms(1, seconds=7777 / 16000., sample_rate=16000, seed=12)
        np.testing.assert_array_equal(wave, g['wave'])
    else:
        wave = synth.make_waveforms(2, seconds=10.0, sample_rate=16000, seed=1234)
    out = O.forward(_sd(mt), mt, wave=wave)
    for k in ('framewise_output', 'clipwise_output', 'embedding'):
        _close(out[k], g[k], 1e-5, k)


@pytest.mark.parametrize('mt', [GRU, TRF])
def test_windowed_and_events(golden_dir, mt):
    g = np.load(os.path.join(golden_dir, 'windowed_%s.npz' % mt))
    ev = json.load(open(os.path.join(golden_dir, 'events.json')))
    audio = synth.make_waveforms(2, seconds=10.0, sample_rate=16000, seed=1234)[0]
    sd = _sd(mt)
    merged = O.predict_windows(sd, mt, audio, 16000, 5, 1, 'predict', overlap=True)
    _close(merged, g['merged_5_1'], 1e-5, 'merged_5_1')
    merged_ms = O.predict_windows(sd, mt, audio, 16000, 6, 0.5, 'main_strong')
    _close(merged_ms, g['merged_6_05'], 1e-5, 'merged_6_05')
    for which in ('default', 'synthetic'):
        got = O.events_from_framewise(g['merged_5_1'], ev['params_' + which])
        assert got == ev[mt][which]


@pytest.mark.parametrize('mt', [GRU, TRF])
def test_long_file_windowed(golden_dir, mt):
    """Long files (predict.py's unbounded loop, oracle/make_golden_long.py):
    the oracle's window count and merged length match the reference golden,
    the oracle reproduces the 66-window predict.py --sample_duration 6
    --overlap --overlap_value 0.5 merge (1 s stride, windows 50 frames apart
    in the merged output), and its events match the reference's on both long
    goldens."""
    ev = json.load(open(os.path.join(golden_dir, 'long_events.json')))
    for case, c in sorted(ev['cases'].items()):
        g = np.load(os.path.join(golden_dir, 'long_%s.npz' % case))[mt]
        secs = c['samples'] / 16000.
        starts = O.window_starts(secs, c['sample_duration'],
                                 O.driver_stride(c['driver'], c['sample_duration'], c['overlap_value'], c['overlap']))
        step = int(100 * c['overlap_value'])
        assert len(starts) > 64
        # N = Tw + (n_win - 1) * step, Tw = a window's framewise length
        # (models.py:678-681: 8 * T3, the GRU's padded to a multiple of 100)
        tw = 8 * ((((100 * c['sample_duration'] + 1) // 2) // 2) // 2)
        if mt == GRU:
            tw = O.roundup(tw)
        assert g.shape[1] == tw + (len(starts) - 1) * step
        if case == '6_05':   # 66 batch-1 forwards: a few s on the CPU
            audio = synth.make_waveforms(1, seconds=secs, sample_rate=16000, seed=c['seed'])[0]
            merged = O.predict_windows(_sd(mt), mt, audio, 16000, c['sample_duration'], c['overlap_value'],
                                       c['driver'], overlap=c['overlap'])
            _close(merged, g, 1e-5, 'long_' + case)
        for which in ('default', 'synthetic'):
            assert O.events_from_framewise(g, ev['params_' + which]) == c[mt][which], (case, which)


@pytest.mark.parametrize('mt', [GRU, TRF])
def test_driver_windows(golden_dir, mt):
    """Every window-driver case the reference produced (oracle/
    make_golden_drivers.py: predict.py with and without --overlap and with
    merge steps 50 / 70 / 100 / 130 / 1000, main_strong at 0.7 / 0.9 / 1.3,
    clips shorter and longer than 10 s): the oracle's loop gives the same
    merged output and events, and raises where the reference raised."""
    ev = json.load(open(os.path.join(golden_dir, 'drivers_events.json')))
    g = np.load(os.path.join(golden_dir, 'drivers_%s.npz' % mt))
    sd = _sd(mt)
    for case, c in sorted(ev['cases'].items()):
        audio = synth.make_waveforms(1, seconds=c['samples'] / 16000., sample_rate=16000, seed=c['seed'])[0]
        args = (sd, mt, audio, 16000, c['sample_duration'], c['overlap_value'], c['driver'])
        if 'raises' in c[mt]:
            with pytest.raises(ValueError):
                O.predict_windows(*args, overlap=c['overlap'])
            continue
        merged = O.predict_windows(*args, overlap=c['overlap'])
        _close(merged, g[case], 1e-5, case)
        for which in ('default', 'synthetic'):
            assert O.events_from_framewise(g[case], ev['params_' + which]) == c[mt][which], (case, which)


def test_merge_kat(golden_dir):
    g = np.load(os.path.join(golden_dir, 'merge_kat.npz'))
    for key in g.files:
        dur, ov, n = key.split('_')
        dur, ov, n = int(dur[1:]), float(ov[1:]), int(n[1:])
        ov = int(ov) if ov == int(ov) else ov
        nwin = len(O.window_starts(10.0, dur, ov))
        merged = None
        for s in range(1, nwin + 1):
            curr = np.ones((1, n, 2), np.float32)
            merged = curr if s == 1 else O.merge(merged, curr, dur, s, ov)
        np.testing.assert_array_equal(O.avg_merge(merged, dur, ov)[0, :, 0], g[key])


def test_vad_kat(golden_dir):
    kat = json.load(open(os.path.join(golden_dir, 'vad_kat.json')))
    for case in kat:
        if 'find_bgn_fin_pairs' in case:
            assert O.find_bgn_fin_pairs(case['find_bgn_fin_pairs']) == case['pairs']
            continue
        got = O.activity_detection(np.array(case['x']), case['thres'], case['low_thres'],
                                   case['n_smooth'], case['n_salt'])
        assert [[int(a), int(b)] for a, b in got] == case['pairs']


def test_gamma(golden_dir):
    g = np.load(os.path.join(golden_dir, 'gamma_%s.npz' % GRU))
    audio = synth.make_waveforms(2, seconds=10.0, sample_rate=32000, seed=77)
    for b in range(2):
        gt = O.fft_gtgram(O.pad_truncate_sequence(audio[b], 320000), 32000, 1024 / 32000,
                          320 / 32000, 64, 50)
        np.testing.assert_allclose(gt, g['gtgram'][b], rtol=1e-5, atol=1e-12)
        f = O.gamma_features(audio[b], '32k')
        q = np.round(f.astype(np.float64) * 32767).astype(np.int16)
        assert np.array_equal(q.astype(np.int32), g["features_int16"][b].astype(np.int32))   # bit-exact codes
    feats = torch.from_numpy(O.int16_to_float32(g['features_int16'])).unsqueeze(1).transpose(2, 3)
    out = O.forward(_sd(GRU, '32k'), GRU, features=feats)
    for k in ('framewise_output', 'clipwise_output', 'embedding'):
        _close(out[k], g[k], 1e-5, k)


def _vote_params(ev, which):
    return ev['params_' + which]


@pytest.mark.parametrize('mt', [GRU, TRF])
def test_vote_and_overlap_sweep(golden_dir, mt):
    """inference_prob_vote (binarize_pred + merge + activity_detection_binary)
    and the inference_prob_overlap merge, oracle vs reference fixtures."""
    g = np.load(os.path.join(golden_dir, 'vote_%s.npz' % mt))
    ev = json.load(open(os.path.join(golden_dir, 'vote_events.json')))
    for ov, sd in ev['settings'][mt]:
        tag = '%s_%s' % (ov, sd)
        wins = [g['windows_' + tag][i:i + 1] for i in range(g['windows_' + tag].shape[0])]
        merged = wins[0]
        for s in range(2, len(wins) + 1):
            merged = O.merge(merged if s > 2 else wins[0], wins[s - 1], sd, s, ov)
        np.testing.assert_array_equal(O.avg_merge(merged.copy(), sd, ov), g['avg_' + tag])
        got = O.events_from_framewise(g['avg_' + tag], ev['params_default'], 'clip', sort=False)
        assert got == ev[mt]['overlap_' + tag]
        for which in ('default', 'synthetic', 'mid'):
            p = _vote_params(ev, which)
            votes = None
            for s, w in enumerate(wins, start=1):
                b = O.binarize_pred(w, p['sed_low_threshold'])
                votes = b if s == 1 else O.merge(votes, b, sd, s, ov)
            np.testing.assert_array_equal(votes, g['votes_%s_%s' % (which, tag)])
            got = O.events_from_votes(votes, ov, sd, p, 'clip')
            assert got == ev[mt]['vote_%s_%s' % (which, tag)], (tag, which)
