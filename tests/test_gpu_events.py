"""GPU event extraction (events.hip) and the voting / overlap
sweep drivers of main_strong.py (§8 f3, f4) through the C ABI, against the
reference fixtures (oracle/make_golden_vote.py, oracle/make_golden.py), the
host C++ path and the CPU oracle.

Integer outputs (event frame indices, vote counts) must match bit for bit.
Where a vote or event depends on a model output within 1e-4 of a threshold
(the HIP forward is within ~1e-6 of the reference's), the comparison says so
and skips that cell instead of guessing.
"""
import json
import os
import time

import numpy as np
import pytest
import torch

from oracle import sed_oracle as O
from sedx import inference, synth

pytestmark = pytest.mark.gpu

GRU, TRF = 'Cnn_9layers_Gru_FrameAtt', 'Cnn_9layers_Transformer_FrameAtt'
SEEDS = {GRU: 0, TRF: 1}
MARGIN = 1e-4


def build(mt):
    from sedx import models
    m = getattr(models, mt)(16000, 512, 160, 64, 25, 7000, 25, 'logmel')
    sd = m.state_dict()
    for k, v in synth.make_state_dict(mt, seed=SEEDS[mt]).items():
        sd[k] = torch.from_numpy(v)
    m.load_state_dict(sd, strict=True)
    return m.to('cuda').eval()


def _series(rng, N, T, C):
    fw = rng.uniform(0, 1, (N, T, C)).astype(np.float32)
    return (np.cumsum(fw - 0.5, axis=1) / 8 + 0.5).astype(np.float32)


def test_device_events_match_host_and_oracle():
    rng = np.random.default_rng(11)
    for it in range(30):
        N, T, C = int(rng.integers(1, 5)), int(rng.integers(1, 400)), 25
        fw = _series(rng, N, T, C)
        params = {'sed_high_threshold': rng.uniform(0.4, 0.7, C).tolist(),
                  'sed_low_threshold': rng.uniform(-0.1, 0.4, C).tolist() if it % 5 else None,
                  'n_smooth': int(rng.integers(0, 12)), 'n_salt': int(rng.integers(0, 12))}
        try:
            host = inference.event_pairs(fw, params)
        except RuntimeError:
            with pytest.raises(RuntimeError):
                inference.event_pairs(torch.from_numpy(fw).cuda(), params)
            continue
        dev = inference.event_pairs(torch.from_numpy(fw).cuda(), params)
        np.testing.assert_array_equal(dev, host)
        if params['sed_low_threshold'] is not None:
            ref = O.events_from_framewise(fw, params, sort=False)
            got = inference.events_from_framewise(torch.from_numpy(fw).cuda(), params, sort=False)
            assert got == ref


def test_device_events_edge_lengths():
    """Word boundaries of the per-series bitmaps: runs that end exactly at a
    64-frame boundary or at T, all-on / all-off series, dense alternation,
    long series; device == host C++ path bit for bit."""
    rng = np.random.default_rng(5)
    for T in (1, 2, 63, 64, 65, 127, 128, 129, 1000, 4096, 5003):
        C = 7
        fw = _series(rng, 2, T, C)
        fw[0, :, 0] = 0.9                                   # one run over the whole series
        fw[0, :, 1] = 0.1                                   # no run
        fw[0, :, 2] = np.where(np.arange(T) % 2 == 0, 0.9, 0.1)      # alternating
        fw[0, :, 3] = np.where((np.arange(T) // 64) % 2 == 0, 0.9, 0.35)  # 64-frame blocks
        fw[0, :, 4] = np.where(np.arange(T) >= T - 1, 0.9, 0.1)  # last frame only
        for low in (None, 0.3, -0.1):
            params = {'sed_high_threshold': 0.5, 'sed_low_threshold': low,
                      'n_smooth': int(rng.integers(0, 4)), 'n_salt': int(rng.integers(0, 4))}
            try:
                host = inference.event_pairs(fw, params)
            except RuntimeError:
                with pytest.raises(RuntimeError):
                    inference.event_pairs(torch.from_numpy(fw).cuda(), params)
                continue
            dev = inference.event_pairs(torch.from_numpy(fw).cuda(), params)
            np.testing.assert_array_equal(dev, host, err_msg='T=%d low=%s' % (T, low))


def test_device_events_vad_kat(golden_dir):
    kat = json.load(open(os.path.join(golden_dir, 'vad_kat.json')))
    for case in kat:
        if 'x' not in case:
            continue
        x = torch.tensor(np.asarray(case['x'], np.float32)[None, :, None]).cuda()
        params = {'sed_high_threshold': case['thres'], 'sed_low_threshold': case['low_thres'],
                  'n_smooth': case['n_smooth'], 'n_salt': case['n_salt']}
        got = inference.event_pairs_device(x, params)[:, 2:].tolist()
        assert got == case['pairs'], case


def test_device_events_golden_windowed(golden_dir):
    ev = json.load(open(os.path.join(golden_dir, 'events.json')))
    for mt in (GRU, TRF):
        merged = np.load(os.path.join(golden_dir, 'windowed_%s.npz' % mt))['merged_5_1']
        for which in ('default', 'synthetic'):
            got = inference.events_from_framewise(torch.from_numpy(merged).cuda(), ev['params_' + which])
            assert got == ev[mt][which]


def test_device_vote_events_from_golden_votes(golden_dir):
    """activity_detection_binary on the reference's own vote counts: bit-exact."""
    ev = json.load(open(os.path.join(golden_dir, 'vote_events.json')))
    for mt in (GRU, TRF):
        g = np.load(os.path.join(golden_dir, 'vote_%s.npz' % mt))
        for ov, sd in ev['settings'][mt]:
            for which in ('default', 'synthetic', 'mid'):
                votes = torch.from_numpy(g['votes_%s_%s_%s' % (which, ov, sd)]).cuda()
                got = inference.events_from_votes(votes, ov, sd, ev['params_' + which], 'clip')
                assert got == ev[mt]['vote_%s_%s_%s' % (which, ov, sd)], (mt, ov, sd, which)


def _near(windows, thr, ov, Tw, N):
    """[N, C] mask of merged frames fed by a window value within MARGIN of thr."""
    thr = np.broadcast_to(np.asarray(thr, np.float64), (windows.shape[2],))
    near = np.abs(windows.astype(np.float64) - thr[None, None, :]) < MARGIN     # [n_win, Tw, C]
    step = int(100 * ov)
    out = np.zeros((N, windows.shape[2]), bool)
    for w in range(windows.shape[0]):
        out[w * step:w * step + Tw] |= near[w]
    return out


@pytest.mark.parametrize('mt', [GRU, TRF])
def test_vote_pipeline_end_to_end(golden_dir, mt):
    """predict_windows_vote (one native batch, GPU binarise + merge) and the
    GPU binary event extraction against the reference fixtures."""
    g = np.load(os.path.join(golden_dir, 'vote_%s.npz' % mt))
    ev = json.load(open(os.path.join(golden_dir, 'vote_events.json')))
    m = build(mt)
    audio = torch.from_numpy(synth.make_waveforms(2, seconds=10.0, sample_rate=16000, seed=1234)[1:2]).cuda()
    for ov, sd in ev['settings'][mt]:
        tag = '%s_%s' % (ov, sd)
        wins = g['windows_' + tag]
        avg = inference.predict_windows(m, audio, sd, ov, driver='main_strong').cpu().numpy()
        e = float(np.max(np.abs(avg - g['avg_' + tag])))
        print(mt, tag, 'overlap merge max|d| =', e)
        assert e <= 1e-3
        for which in ('default', 'synthetic', 'mid'):
            p = ev['params_' + which]
            votes = inference.predict_windows_vote(m, audio, sd, ov, p['sed_low_threshold'])
            exp = g['votes_%s_%s' % (which, tag)]
            near = _near(wins, p['sed_low_threshold'], ov, wins.shape[1], exp.shape[1])
            diff = votes.cpu().numpy()[0] != exp[0]
            assert not np.any(diff & ~near), (tag, which, int(np.sum(diff & ~near)))
            got = inference.events_from_votes(votes, ov, sd, p, 'clip')
            if not near.any():
                assert got == ev[mt]['vote_%s_%s' % (which, tag)], (tag, which)
            else:
                print(mt, tag, which, '%d cells within %g of the threshold: event check skipped'
                      % (int(near.sum()), MARGIN))


def test_sweep_overlap_matches_reference(golden_dir):
    ev = json.load(open(os.path.join(golden_dir, 'vote_events.json')))
    for mt in (GRU, TRF):
        g = np.load(os.path.join(golden_dir, 'vote_%s.npz' % mt))
        m = build(mt)
        audio = torch.from_numpy(synth.make_waveforms(2, seconds=10.0, sample_rate=16000, seed=1234)[1:2]).cuda()
        combos = ev['settings'][mt]
        res = inference.sweep_overlap(m, audio, ['clip'], ev['params_default'], combos)
        for ov, sd in combos:
            tag = '%s_%s' % (ov, sd)
            margin = float(np.min(np.abs(g['avg_' + tag].astype(np.float64) - 0.5)))
            if margin > MARGIN:
                assert res[(ov, sd)] == ev[mt]['overlap_' + tag], tag


def test_device_events_batch32_timing():
    """Events for a B=32 clip-mode batch on the GPU (reported, and checked
    against the host C++ path)."""
    m = build(GRU)
    wave = torch.from_numpy(synth.make_waveforms(32, seconds=10.0, sample_rate=16000, seed=4321)).cuda()
    with torch.no_grad():
        fw = m(wave)['framewise_output']
    params = {'sed_high_threshold': 0.5, 'sed_low_threshold': 0.3, 'n_smooth': 10, 'n_salt': 10}
    dev = inference.event_pairs(fw, params)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        inference.event_pairs(fw, params)
    t_dev = (time.perf_counter() - t0) / 10
    t0 = time.perf_counter()
    host = inference.event_pairs(fw.cpu().numpy(), params)
    t_host = time.perf_counter() - t0
    print('events B=32: %d events; device %.3f ms (incl. D2H + sync), host C++ %.3f ms' %
          (len(dev), t_dev * 1e3, t_host * 1e3))
    np.testing.assert_array_equal(dev, host)
