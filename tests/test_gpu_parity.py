"""HIP path (libsedx through the C ABI) vs the golden fixtures / CPU oracle.

Tolerance: north_star requires framewise_output within 1e-3 (fp32) of the
reference CPU path and identical event segments.  TOL below is that bound;
the fp32-MFMA path is expected to land near 1e-6, which the tests print.
"""
import json
import os

import numpy as np
import pytest
import torch

from oracle import sed_oracle as O
from sedx import synth

pytestmark = pytest.mark.gpu

GRU, TRF = 'Cnn_9layers_Gru_FrameAtt', 'Cnn_9layers_Transformer_FrameAtt'
SEEDS = {GRU: 0, TRF: 1}
TOL = 1e-3          # north_star: |framewise - reference| <= 1e-3 (fp32)
P16 = (16000, 512, 160, 64, 25, 7000)
P32 = (32000, 1024, 320, 64, 50, 14000)
P8 = (8000, 256, 80, 64, 12, 3500)
PRESET_ARGS = {'8k': P8, '16k': P16, '32k': P32}


def build(mt, preset=P16, feature_type='logmel'):
    from sedx import models
    m = getattr(models, mt)(*preset, 25, feature_type)
    sd = m.state_dict()
    for k, v in synth.make_state_dict(mt, seed=SEEDS[mt]).items():
        sd[k] = torch.from_numpy(v)
    m.load_state_dict(sd, strict=True)
    return m.to('cuda').eval()


def run(m, wave):
    with torch.no_grad():
        out = m(torch.as_tensor(np.asarray(wave), dtype=torch.float32).cuda())
    return {k: v.cpu().numpy() for k, v in out.items()}


def err(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    assert a.shape == b.shape, (a.shape, b.shape)
    return float(np.max(np.abs(a - b)))


@pytest.fixture(scope='module', params=[(GRU, 'exact'), (TRF, 'exact'), (GRU, 'x3'), (TRF, 'x3'),
                                        (GRU, 'winograd'), (TRF, 'winograd')],
                ids=['gru-exact', 'trf-exact', 'gru-x3', 'trf-x3', 'gru-wino', 'trf-wino'])
def model(request):
    mt, prec = request.param
    return mt, build(mt).set_precision(prec)


def test_short_clip_all_outputs(model, golden_dir):
    mt, m = model
    g = np.load(os.path.join(golden_dir, 'stages_%s.npz' % mt))
    out = run(m, g['wave'])
    for k in ('framewise_output', 'clipwise_output'):
        e = err(out[k], g[k])
        print(mt, k, 'max|d| =', e)
        assert e <= TOL
    emb_scale = max(1.0, float(np.abs(g['embedding']).max()))
    assert err(out['embedding'], g['embedding']) <= TOL * emb_scale


@pytest.mark.parametrize('kind', ['ragged', 'clip10s'])
def test_clip_goldens(model, golden_dir, kind):
    mt, m = model
    g = np.load(os.path.join(golden_dir, '%s_%s.npz' % (kind, mt)))
    if kind == 'ragged':
        wave = synth.make_waveforms(1, seconds=7777 / 16000., sample_rate=16000, seed=12)
    else:
        wave = synth.make_waveforms(2, seconds=10.0, sample_rate=16000, seed=1234)
    out = run(m, wave)
    for k in ('framewise_output', 'clipwise_output'):
        e = err(out[k], g[k])
        print(mt, kind, k, 'max|d| =', e)
        assert e <= TOL


def test_batch32_vs_oracle(model):
    """Headline config (B=32, 10 s @ 16 kHz) against the CPU oracle."""
    mt, m = model
    wave = synth.make_waveforms(32, seconds=10.0, sample_rate=16000, seed=4321)
    out = run(m, wave)
    ref = O.forward(O.full_state(synth.make_state_dict(mt, seed=SEEDS[mt])), mt, wave=wave)
    for k in ('framewise_output', 'clipwise_output', 'embedding'):
        assert np.isfinite(out[k]).all(), k      # a timed-out GRU hand-off poisons with NaN
        scale = max(1.0, float(ref[k].abs().max()))
        e = err(out[k], ref[k].numpy())
        print(mt, 'B=32', k, 'max|d| =', e)
        assert e <= TOL * scale


@pytest.mark.parametrize('f43', [0, 1, 2], ids=['f23', 'f43b24', 'f43'])
@pytest.mark.parametrize('mt', [GRU, TRF])
def test_batch32_vs_oracle_wino_forms(mt, f43):
    """test_batch32_vs_oracle for every Winograd form (SEDX_TUNE_WINO_F43):
    the headline batch against the CPU oracle at the Winograd bar (2e-5, far
    inside north_star's 1e-3), with the oracle's thresholded events, and a
    ragged 7.33 s batch (partial last tile rows, odd rows dropped by the
    pools) at the same bar."""
    from sedx import inference
    m = build_prec(mt, 'winograd', f43)
    st = O.full_state(synth.make_state_dict(mt, seed=SEEDS[mt]))
    params = {'sed_high_threshold': 0.5, 'sed_low_threshold': 0.3, 'n_smooth': 10, 'n_salt': 10}
    for n, sec, seed in ((32, 10.0, 4321), (3, 7.33, 5)):
        wave = synth.make_waveforms(n, seconds=sec, sample_rate=16000, seed=seed)
        out = run(m, wave)
        ref = O.forward(st, mt, wave=wave)
        for k in ('framewise_output', 'clipwise_output', 'embedding'):
            assert np.isfinite(out[k]).all(), k
            scale = max(1.0, float(ref[k].abs().max()))
            e = err(out[k], ref[k].numpy())
            print(mt, 'f43=%d' % f43, 'B=%d' % n, k, 'max|d| =', e)
            assert e <= 2e-5 * scale, (k, e)
        ev = inference.events_from_framewise(out['framewise_output'], params)
        assert ev == inference.events_from_framewise(ref['framewise_output'].numpy(), params)


@pytest.mark.parametrize('seconds', [61.3])
def test_long_clip_vs_oracle(model, seconds):
    """A long, ragged clip (6131 frames: many t-tiles per clip, the last one
    partial in every layer, odd frame counts before each pooling) against
    the CPU oracle: the epilogues' per-tile store ranges and the
    range-checked stores past a clip's end."""
    mt, m = model
    wave = synth.make_waveforms(2, seconds=seconds, sample_rate=16000, seed=77)
    out = run(m, wave)
    ref = O.forward(O.full_state(synth.make_state_dict(mt, seed=SEEDS[mt])), mt, wave=wave)
    for k in ('framewise_output', 'clipwise_output'):
        scale = max(1.0, float(ref[k].abs().max()))
        e = err(out[k], ref[k].numpy())
        print(mt, 'long', k, out[k].shape, 'max|d| =', e)
        assert out[k].shape == tuple(ref[k].shape)
        assert e <= TOL * scale


def test_batch_invariance(model):
    """A clip's output does not depend on the batch it runs in."""
    mt, m = model
    wave = synth.make_waveforms(5, seconds=3.0, sample_rate=16000, seed=99)
    full = run(m, wave)
    for i in (0, 3):
        one = run(m, wave[i:i + 1])
        assert np.array_equal(one['framewise_output'][0], full['framewise_output'][i])


@pytest.mark.parametrize('pipelined', [0, 1, 2])
def test_concurrent_streams_bit_identical(model, pipelined):
    """Batches in flight on two HIP streams (bench.py --streams 2: one batch's
    GRU / head overlapping the next batch's conv stack, whose workgroups then
    claim tiles dynamically) give bit-identical outputs to one batch at a time,
    with and without the conv stacks ordered across streams
    (sedx_set_pipelined 1; 2: block 1's conv1 issued ahead of that wait, so
    it runs beside the previous batch's conv tail).  Unpipelined, the default GRU kernel (AUTO) is the
    16-slice cooperative one, which needs 32 co-resident workgroups beside the
    other stream's work: no NaN, no reported failure."""
    mt, m = model
    waves = [torch.from_numpy(synth.make_waveforms(32, seconds=10.0, sample_rate=16000, seed=s)).cuda()
             for s in (5, 6, 7, 8)]
    with torch.no_grad():
        ref = [m(w)['framewise_output'].clone() for w in waves]
        torch.cuda.synchronize()
        streams = [torch.cuda.Stream(), torch.cuda.Stream()]
        m.set_pipelined(pipelined)
        try:
            for rep in range(3):
                outs = []
                for i, w in enumerate(waves):
                    with torch.cuda.stream(streams[i % 2]):
                        outs.append(m(w)['framewise_output'])
                torch.cuda.synchronize()
                m.check_error()
                for i, (a, b) in enumerate(zip(outs, ref)):
                    assert torch.equal(a, b), (mt, rep, i, float((a - b).abs().max()))
        finally:
            m.set_pipelined(False)


@pytest.mark.parametrize('n_clips,seconds', [(1, 1.0), (40, 1.0), (544, 0.5)])
def test_gru_clip_groups(n_clips, seconds):
    """Cooperative GRU: 1 group, 2 groups (ragged last), and more groups than
    resident slots (544 clips = 17 groups of 32 > 16 slots)."""
    m = build(GRU)
    wave = synth.make_waveforms(n_clips, seconds=seconds, sample_rate=16000, seed=n_clips)
    out = run(m, wave)
    ref = O.forward(O.full_state(synth.make_state_dict(GRU, seed=0)), GRU, wave=wave)
    e = err(out['framewise_output'], ref['framewise_output'].numpy())
    print('GRU groups', n_clips, 'max|d| =', e)
    assert e <= TOL


def _tune(m, knob, value):
    from sedx import _lib
    nat = m.native(torch.device('cuda', 0))
    _lib.check(_lib.lib().sedx_set_tuning(nat.h, knob, value), nat.h, 'set_tuning')


@pytest.mark.parametrize('prec', ['exact', 'x3'])
def test_gru_handoff_modes_bit_identical(prec):
    """XCD-local and global GRU hand-off protocols — the latter also with the
    slices dealt over every XCD (SPREAD), and LOCAL (one XCD per group and
    direction even on a pipelined handle) — move the same bytes: the outputs
    must be bit-identical (and the faster one is used by default)."""
    import time
    from sedx import _lib
    m = build(GRU).set_precision(prec)
    wave = synth.make_waveforms(32, seconds=10.0, sample_rate=16000, seed=8)
    outs, times = {}, {}
    for mode in (1, 2, 3, 0):     # SEDX_GRU_HANDOFF_GLOBAL, _SPREAD, _LOCAL, _AUTO
        _tune(m, _lib.TUNE_GRU_HANDOFF, mode)
        run(m, wave)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        outs[mode] = run(m, wave)['framewise_output']
        times[mode] = time.perf_counter() - t0
    print('GRU hand-off (%s): global %.3f ms, spread %.3f ms, local %.3f ms, auto %.3f ms (whole forward)' %
          (prec, times[1] * 1e3, times[2] * 1e3, times[3] * 1e3, times[0] * 1e3))
    assert np.isfinite(outs[0]).all()
    for mode in (1, 2, 3):
        assert np.array_equal(outs[mode], outs[0]), mode


@pytest.mark.parametrize('n_clips,seconds', [(40, 4.0), (160, 1.0)])
def test_gru_pipelined_placements_bit_identical(n_clips, seconds):
    """On a pipelined handle every recurrence kernel and placement gives the
    non-pipelined default's bits: AUTO (16 slices dealt over every XCD), the
    8-slice kernel (SEDX_GRU_KERNEL_COOP) under SPREAD and LOCAL, and the
    two-half PAIR kernel under SPREAD — at 40 clips (two groups, the second
    ragged) and 160 clips (5 groups of 32: more than GRU_MAX_SLOTS = 4, so
    workgroups run a second group)."""
    from sedx import _lib
    w = synth.make_waveforms(n_clips, seconds=seconds, sample_rate=16000, seed=9)
    ref = run(build(GRU), w)['framewise_output']
    assert np.isfinite(ref).all()
    for kern, ho in ((5, 0), (0, 2), (0, 3), (7, 2), (4, 3)):
        mp = build(GRU).set_pipelined(True)
        mp.set_tuning(_lib.TUNE_GRU_KERNEL, kern).set_tuning(_lib.TUNE_GRU_HANDOFF, ho)
        got = run(mp, w)['framewise_output']
        mp.check_error()
        assert np.array_equal(got, ref), (kern, ho)


@pytest.mark.parametrize('n_clips', [40, 80])
def test_gru_tag_kernels_bit_identical(n_clips):
    """The data-tagged recurrences (SEDX_GRU_KERNEL_TAG16 / TAG8: 16-clip
    groups, granules straight into v_mfma_f32_16x16x4_f32 operands) and the
    16-slice cooperative kernels (COOP16: 16 units per workgroup on 16x16x4
    MFMAs; KSPLIT: each K-eighth wave waits for and loads only its two
    slices) keep the exact kernels' arithmetic contract (eight in-order K
    partials, summed in order): bit-identical to the 8-slice 32-clip kernel,
    ragged last group and more groups than resident slots (80 clips) included;
    AUTO (the default: COOP16 on an unpipelined handle) and PAIR (a group's
    two 16-clip halves stepped alternately in one workgroup, with the
    SPREAD placement too) as well."""
    from sedx import _lib
    m = build(GRU).set_precision('exact')
    wave = synth.make_waveforms(n_clips, seconds=2.0, sample_rate=16000, seed=n_clips + 3)
    outs = {}
    for knob in (0, 2, 3, 4, 5, 6, 7):  # COOP, TAG16, TAG8, COOP16, AUTO, KSPLIT, PAIR
        _tune(m, _lib.TUNE_GRU_KERNEL, knob)
        outs[knob] = run(m, wave)['framewise_output']
    _tune(m, _lib.TUNE_GRU_HANDOFF, 2)
    outs['pair_spread'] = run(m, wave)['framewise_output']
    _tune(m, _lib.TUNE_GRU_HANDOFF, 0)
    _tune(m, _lib.TUNE_GRU_KERNEL, 5)
    assert np.isfinite(outs[0]).all()
    for knob in (2, 3, 4, 5, 6, 7, 'pair_spread'):
        assert np.array_equal(outs[knob], outs[0]), knob


@pytest.mark.parametrize('kernel,n_clips', [(0, 32), (4, 32), (0, 4), (2, 40), (6, 40), (7, 40)])
def test_gru_spin_timeout_surfaces(kernel, n_clips):
    """A GRU hand-off spin that runs out (forced with SEDX_TUNE_GRU_SPIN = 0
    polls: every step that would wait fails, deterministically) turns that forward's outputs into NaN and is reported by
    sedx_check_error / model.check_error() once the batch is complete — for
    the 8- and 16-slice cooperative kernels, the small-batch VALU kernel and
    the data-tagged one; with the default bound the same handle is clean and
    exact again."""
    from sedx import _lib
    m = build(GRU).set_precision('exact')
    _tune(m, _lib.TUNE_GRU_KERNEL, kernel)
    wave = torch.from_numpy(synth.make_waveforms(n_clips, seconds=2.0, sample_rate=16000, seed=31)).cuda()
    with torch.no_grad():
        ref = m(wave)['framewise_output'].clone()
        torch.cuda.synchronize()
        m.check_error()
        failed = 0
        _tune(m, _lib.TUNE_GRU_SPIN, 0)
        try:
            for _ in range(4):
                out = m(wave)['framewise_output']
                torch.cuda.synchronize()
                nan = bool(torch.isnan(out).any())
                try:
                    m.check_error()
                    reported = False
                except RuntimeError as e:
                    reported = 'GRU' in str(e)
                assert nan == reported, (nan, reported)
                failed += nan
        finally:
            _tune(m, _lib.TUNE_GRU_SPIN, 1 << 24)
            _tune(m, _lib.TUNE_GRU_KERNEL, 5)
        assert failed == 4
        _tune(m, _lib.TUNE_GRU_KERNEL, kernel)
        out = m(wave)['framewise_output']
        torch.cuda.synchronize()
        m.check_error()
        _tune(m, _lib.TUNE_GRU_KERNEL, 5)
    assert torch.equal(out, ref)


@pytest.mark.parametrize('vote', [False, True])
def test_windows_spin_timeout_raises(vote):
    """A GRU hand-off spin that runs out inside a windowed forward
    (SEDX_TUNE_GRU_SPIN = 0) raises from predict_windows / predict_windows_vote
    themselves (sedx.inference syncs and calls model.check_error() before
    returning), so sweep_overlap never extracts events from NaN merges; with
    the default bound the same handle is clean again."""
    from sedx import _lib, inference
    m = build(GRU).set_precision('exact')
    audio = torch.from_numpy(synth.make_waveforms(16, seconds=10.0, sample_rate=16000, seed=33)).cuda()
    call = ((lambda: inference.predict_windows_vote(m, audio, 5, 1.0, 0.3)) if vote
            else (lambda: inference.predict_windows(m, audio, 5, 1.0, driver='main_strong')))
    with torch.no_grad():
        ref = call().clone()
        _tune(m, _lib.TUNE_GRU_SPIN, 0)
        try:
            with pytest.raises(RuntimeError, match='GRU'):
                call()
        finally:
            _tune(m, _lib.TUNE_GRU_SPIN, 1 << 24)
        again = call()
    assert torch.equal(again, ref)


def test_gru_exact_recurrence_is_fp32():
    """Exact mode runs the recurrence on fp32 MFMA operands: it agrees with
    the per-(clip, direction) fp32-FMA kernel and the oracle far inside the
    x3 split's error, for a full and a partial 32-clip group."""
    from sedx import _lib
    m = build(GRU).set_precision('exact')
    wave = synth.make_waveforms(40, seconds=4.0, sample_rate=16000, seed=21)
    coop = run(m, wave)
    _tune(m, _lib.TUNE_GRU_KERNEL, 1)
    simple = run(m, wave)
    _tune(m, _lib.TUNE_GRU_KERNEL, 5)
    ref = O.forward(O.full_state(synth.make_state_dict(GRU, seed=0)), GRU, wave=wave)
    for k in ('framewise_output', 'embedding'):
        e_cs = err(coop[k], simple[k])
        e_ref = err(coop[k], ref[k].numpy())
        print('GRU exact', k, 'coop vs simple max|d| = %.3g, vs oracle %.3g' % (e_cs, e_ref))
        assert e_cs <= 2e-6 and e_ref <= 1e-5


@pytest.mark.parametrize('prec,seconds', [('exact', 10.0), ('x3', 10.0), ('exact', 7.33), ('winograd', 10.0),
                                          ('winograd', 7.33)])
def test_small_batch_shapes_bit_identical(prec, seconds):
    """Small batches run other kernel shapes — 32x32-wave-tile convs, the
    barrier-free small-M linear, (exact) the VALU fma-chain GRU product for
    groups of <= 8 clips instead of 32-clip MFMAs, and (winograd) the
    F(4x4,3x3) layers' 16-channel items with their own weight pack and, at
    one or two clips, 16-tile items.  Each keeps every output's operation
    sequence, so a clip's outputs are bit-identical whether it runs alone,
    in a pair, in four, or inside a full 32-clip group (40 clips: a full MFMA
    group + a ragged 8-clip group)."""
    m = build(GRU).set_precision(prec)
    # 7.33 s: odd frame counts after the pools (T 734 -> 367 -> 183 -> 91)
    wave = synth.make_waveforms(40, seconds=seconds, sample_rate=16000, seed=31)
    full = run(m, wave)
    for i in (0, 17, 39):
        one = run(m, wave[i:i + 1])
        for k in ('framewise_output', 'clipwise_output', 'embedding'):
            assert np.array_equal(one[k][0], full[k][i]), (prec, i, k, err(one[k][0], full[k][i]))
    four = run(m, wave[8:12])
    assert np.array_equal(four['framewise_output'], full['framewise_output'][8:12])
    two = run(m, wave[20:22])
    assert np.array_equal(two['framewise_output'], full['framewise_output'][20:22])


def test_graphed_forward_bit_identical(model):
    """The forward captured in a HIP graph and replayed (GraphedForward)
    gives the eager forward's outputs bit for bit, also on new input."""
    from sedx import inference
    mt, m = model
    w0 = torch.from_numpy(synth.make_waveforms(2, seconds=4.0, sample_rate=16000, seed=3)).cuda()
    w1 = torch.from_numpy(synth.make_waveforms(2, seconds=4.0, sample_rate=16000, seed=4)).cuda()
    g = inference.GraphedForward(m, w0)
    for w in (w1, w0):
        with torch.no_grad():
            ref = m(w)
        out = g(w)
        for k in ('framewise_output', 'clipwise_output'):
            assert torch.equal(out[k], ref[k]), (mt, k)
    # a pipelined handle waits on an event recorded outside any capture: refused
    m.set_pipelined(True)
    try:
        with pytest.raises(RuntimeError):
            inference.GraphedForward(m, w0)
    finally:
        m.set_pipelined(False)


def test_windowed_and_events(model, golden_dir):
    from sedx import inference
    mt, m = model
    g = np.load(os.path.join(golden_dir, 'windowed_%s.npz' % mt))
    ev = json.load(open(os.path.join(golden_dir, 'events.json')))
    audio = torch.from_numpy(synth.make_waveforms(2, seconds=10.0, sample_rate=16000, seed=1234)[:1]).cuda()
    merged = inference.predict_windows(m, audio, 5, 1.0, overlap=True, driver='predict').cpu().numpy()
    e = err(merged, g['merged_5_1'])
    print(mt, 'windowed 5/1 max|d| =', e)
    assert e <= TOL
    merged_ms = inference.predict_windows(m, audio, 6, 0.5, driver='main_strong').cpu().numpy()
    assert err(merged_ms, g['merged_6_05']) <= TOL
    for which in ('default', 'synthetic'):
        params = ev['params_' + which]
        got = inference.events_from_framewise(merged, params)
        exp = ev[mt][which]
        if got != exp:
            # report the threshold margin that explains a flip
            hi = np.broadcast_to(np.asarray(params['sed_high_threshold'], np.float64), (25,))
            margin = np.min(np.abs(g['merged_5_1'][0] - hi[None, :]))
            pytest.fail('event mismatch (%s), min |x - high| = %g' % (which, margin))


@pytest.mark.parametrize('case', ['5_1', '6_05'])
def test_long_file_windowed(model, golden_dir, case):
    """predict.py over a whole long file (183 windows of 5 s at 1 s stride over
    187.37 s; 66 windows of 6 s at 1 s stride merged 50 frames apart
    (--overlap_value 0.5) over 71.3 s): every window in one native batch, the
    merge + avg_merge of any window count, and the events, against goldens
    the reference produced (oracle/make_golden_long.py)."""
    from sedx import inference
    mt, m = model
    ev = json.load(open(os.path.join(golden_dir, 'long_events.json')))
    c = ev['cases'][case]
    g = np.load(os.path.join(golden_dir, 'long_%s.npz' % case))[mt]
    audio = synth.make_waveforms(1, seconds=c['samples'] / 16000., sample_rate=16000, seed=c['seed'])
    assert audio.shape[1] == c['samples']
    nw, _, nf = inference.window_geometry(m, c['samples'], c['sample_duration'], c['overlap_value'],
                                          c['driver'], c['overlap'])
    stride = O.driver_stride(c['driver'], c['sample_duration'], c['overlap_value'], c['overlap'])
    assert nw == len(O.window_starts(c['samples'] / 16000., c['sample_duration'], stride)) > 64
    assert nf == g.shape[1]
    merged = inference.predict_windows(m, torch.from_numpy(audio).cuda(), c['sample_duration'],
                                       c['overlap_value'], c['overlap'], c['driver'])
    got = merged.cpu().numpy()
    assert np.isfinite(got).all()
    e = err(got, g)
    print(mt, 'long', case, nw, 'windows, merged', got.shape, 'max|d| =', e)
    assert e <= TOL
    for which in ('default', 'synthetic'):
        params = ev['params_' + which]
        exp = c[mt][which]
        for ev_got in (inference.events_from_framewise(merged, params),          # GPU events
                       inference.events_from_framewise(got, params)):            # host C++ events
            if ev_got != exp:
                hi = np.broadcast_to(np.asarray(params['sed_high_threshold'], np.float64), (25,))
                margin = np.min(np.abs(g[0].astype(np.float64) - hi[None, :]))
                pytest.fail('%s %s event mismatch (%s): %d vs %d events, min |x - high| = %g'
                            % (mt, case, which, len(ev_got), len(exp), margin))


@pytest.mark.parametrize('case', ['p_ov05', 'p_noov', 'p_ov07', 'p_noov_ov13', 'p_short', 'p_ov10', 'p_ov6',
                                  'ms_07', 'ms_09_6', 'ms_13_7', 'ms_short', 'ms_long'])
def test_driver_windows(model, golden_dir, case):
    """The reference's two window drivers with their own arguments
    (oracle/make_golden_drivers.py, produced by the reference): predict.py
    strides 1 s with --overlap and sample_duration s without, and merges at
    int(100 * overlap_value) frames whatever the stride; main_strong strides
    overlap_value (float64 running start: 0.7, 0.9, 1.3) over the clip padded
    to 10 s and feeds windows past 10 s shorter (their own batch).  Merged
    framewise within TOL, the same shape, identical events; where the
    reference raised (numpy broadcast), sedx raises too.  Two clips per call
    (the same audio twice): the batched merge of both equals the golden."""
    from sedx import inference
    mt, m = model
    ev = json.load(open(os.path.join(golden_dir, 'drivers_events.json')))
    assert case in ev['cases']
    c = ev['cases'][case]
    audio = synth.make_waveforms(1, seconds=c['samples'] / 16000., sample_rate=16000, seed=c['seed'])
    audio = torch.from_numpy(np.concatenate([audio, audio])).cuda()
    args = (m, audio, c['sample_duration'], c['overlap_value'], c['overlap'], c['driver'])
    if 'raises' in c[mt]:
        with pytest.raises(RuntimeError):
            inference.predict_windows(*args)
        return
    g = np.load(os.path.join(golden_dir, 'drivers_%s.npz' % mt))[case]
    merged = inference.predict_windows(*args)
    got = merged.cpu().numpy()
    assert got.shape == (2,) + g.shape[1:], (got.shape, g.shape)
    e = max(err(got[:1], g), err(got[1:], g))
    print(mt, case, 'merged', got.shape, 'max|d| =', e)
    assert e <= TOL
    for which in ('default', 'synthetic'):
        params = ev['params_' + which]
        exp = c[mt][which]
        ev_got = inference.events_from_framewise(merged[:1], params)
        if ev_got != exp:
            hi = np.broadcast_to(np.asarray(params['sed_high_threshold'], np.float64), (25,))
            margin = np.min(np.abs(g[0].astype(np.float64) - hi[None, :]))
            pytest.fail('%s %s event mismatch (%s): %d vs %d events, min |x - high| = %g'
                        % (mt, case, which, len(ev_got), len(exp), margin))


def test_windowed_multi_clip_matches_single(model):
    from sedx import inference
    mt, m = model
    audio = torch.from_numpy(synth.make_waveforms(3, seconds=10.0, sample_rate=16000, seed=5)).cuda()
    allm = inference.predict_windows(m, audio, 5, 1).cpu().numpy()
    for i in range(3):
        one = inference.predict_windows(m, audio[i:i + 1], 5, 1).cpu().numpy()
        assert np.array_equal(one[0], allm[i])


def _codes(feats):
    """int16 codes of dequantised features (x = q / 32767 rounded to f32)."""
    return torch.round(feats.double() * 32767).to(torch.int32).cpu().numpy()


def test_gamma(golden_dir):
    """Gammatone features (float64 on the GPU) give exactly the reference's
    int16 codes (tests/golden/gamma_*.npz, made by the reference itself)."""
    from sedx import inference
    g = np.load(os.path.join(golden_dir, 'gamma_%s.npz' % GRU))
    m = build(GRU, P32, 'gamma')
    audio = torch.from_numpy(synth.make_waveforms(2, seconds=10.0, sample_rate=32000, seed=77)).cuda()
    feats = inference.gamma_features(m, audio)
    q = _codes(feats)
    d = np.abs(q - g['features_int16'].astype(np.int32))
    print('gamma int16 codes: max |d| =', d.max(), 'cells differing =', int((d > 0).sum()))
    assert d.max() == 0
    gold_feats = torch.from_numpy(g['features_int16'].astype(np.float64) / 32767.).float().cuda()
    assert torch.equal(feats, gold_feats)
    with torch.no_grad():
        out = m(gold_feats)
    for k in ('framewise_output', 'clipwise_output'):
        e = err(out[k].cpu().numpy(), g[k])
        print('gamma', k, 'max|d| =', e)
        assert e <= TOL


@pytest.mark.parametrize('spec', [0, 1])
@pytest.mark.parametrize('seconds,seed', [(10.0, 5), (10.0, 6), (3.3, 7)])
def test_gamma_codes_vs_oracle(seconds, seed, spec):
    """Bit-exact int16 codes against the oracle's numpy float64 restatement on
    other clips, incl. a clip whose last specgram column stays unfilled
    (the frame count divides exactly: range(0, s - n, h) stops one short) —
    with either spectrum kernel (SEDX_TUNE_GAMMA_SPEC 0: workgroup Stockham,
    1: one wave per frame)."""
    from sedx import inference, _lib
    m = build(GRU, P32, 'gamma')
    m.set_tuning(_lib.TUNE_GAMMA_SPEC, spec)
    audio = synth.make_waveforms(3, seconds=seconds, sample_rate=32000, seed=seed)
    if seconds != 10.0:
        L = 2048 + 320 * 300                      # (L - nfft) % hop == 0
        audio = audio[:, :L]
    feats = inference.gamma_features(m, torch.from_numpy(np.ascontiguousarray(audio)).cuda())
    q = _codes(feats)
    for b in range(audio.shape[0]):
        a = audio[b] if seconds != 10.0 else O.pad_truncate_sequence(audio[b], 320000)
        gt = O.fft_gtgram(a, 32000, 1024 / 32000, 320 / 32000, 64, 50)
        ref = O.float32_to_int16(O.power_to_db(gt)).astype(np.int32)
        assert np.array_equal(q[b], ref), (b, int((q[b] != ref).sum()))


@pytest.mark.parametrize('mt', [GRU, TRF])
@pytest.mark.parametrize('preset', ['8k', '32k'])
def test_logmel_presets_vs_oracle(mt, preset):
    """8 k / 32 k logmel presets (pytorch/predict.py:186-205): other FFT sizes
    through the same kernels, checked against the oracle on 3 ragged clips."""
    args = PRESET_ARGS[preset]
    m = build(mt, args)
    wave = synth.make_waveforms(3, seconds=2.7, sample_rate=args[0], seed=31)
    out = run(m, wave)
    ref = O.forward(O.full_state(synth.make_state_dict(mt, seed=SEEDS[mt]), preset), mt, wave=wave)
    for k in ('framewise_output', 'clipwise_output'):
        e = err(out[k], ref[k].numpy())
        print(mt, preset, k, 'max|d| =', e)
        assert e <= TOL


def test_errors_are_loud():
    m = build(GRU)
    with pytest.raises(RuntimeError):
        m(torch.zeros(1, 16000))                       # CPU tensor: no fallback
    with pytest.raises(RuntimeError):
        m(torch.zeros(1, 200, device='cuda'))          # too short for reflect pad
    m.train()
    with pytest.raises(RuntimeError):
        m(torch.zeros(1, 16000, device='cuda'))        # training mode out of scope


@pytest.mark.parametrize('mt', [GRU, TRF])
def test_int16_waveform_input(mt):
    """HDF5 int16 batches (utils/data_generator.py:39): the fused dequantise is
    bit-identical to feeding int16_to_float32(x) (utils/utilities.py:78-79)."""
    m = build(mt)
    q = (synth.make_waveforms(3, seconds=4.0, sample_rate=16000, seed=17) * 32767).astype(np.int16)
    q[0, :5] = [32767, -32768, 0, 1, -1]
    deq = O.int16_to_float32(q)
    assert deq.dtype == np.float32
    a = run(m, deq)
    with torch.no_grad():
        b = m(torch.from_numpy(q).cuda())
    for k in ('framewise_output', 'clipwise_output', 'embedding'):
        assert np.array_equal(a[k], b[k].cpu().numpy()), k


def test_stage_times_accumulate():
    """sedx_set_profiling(h, 2): one event set per forward, so forwards in
    flight on two streams time independently; sedx_stage_times averages them
    and resets.  Mode 1 still reports the last forward; bad modes fail."""
    import ctypes
    from sedx import _lib
    m = build(GRU)
    nat, L = m.native(torch.device('cuda', 0)), _lib.lib()
    w = torch.from_numpy(synth.make_waveforms(4, seconds=2.0, sample_rate=16000, seed=3)).cuda()
    ms = (ctypes.c_float * len(_lib.STAGES))()
    n = ctypes.c_int32()
    assert L.sedx_set_profiling(nat.h, 3) != 0
    assert L.sedx_set_profiling(nat.h, 2) == 0
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    with torch.no_grad():
        outs = []
        for i in range(6):
            with torch.cuda.stream(streams[i % 2]):
                outs.append(m(w)['framewise_output'])
    torch.cuda.synchronize()
    assert L.sedx_stage_times(nat.h, ms, len(_lib.STAGES), ctypes.byref(n)) == 0
    assert n.value == len(_lib.STAGES)
    acc = dict(zip(_lib.STAGES, ms[:]))
    wait = acc.pop('pipeline_wait')
    assert all(v > 0 for v in acc.values()), acc
    assert 0 <= wait < acc['frontend'] + 0.05, wait     # not pipelined: nothing to wait for
    # reset after the read: nothing recorded since
    assert L.sedx_stage_times(nat.h, ms, len(_lib.STAGES), ctypes.byref(n)) == 0
    assert all(v == 0 for v in ms[:])
    # pipelined over two streams: the wait for the previous forward's conv
    # stack is its own stage, so the frontend stage times the frontend only
    m.set_pipelined(True)
    try:
        with torch.no_grad():
            for i in range(8):
                with torch.cuda.stream(streams[i % 2]):
                    outs.append(m(w)['framewise_output'])
        torch.cuda.synchronize()
        assert L.sedx_stage_times(nat.h, ms, len(_lib.STAGES), ctypes.byref(n)) == 0
        pip = dict(zip(_lib.STAGES, ms[:]))
    finally:
        m.set_pipelined(False)
    print('frontend', acc['frontend'], 'pipelined frontend', pip['frontend'], 'wait', pip['pipeline_wait'])
    assert pip['pipeline_wait'] >= 0
    assert pip['frontend'] <= 3 * acc['frontend'] + 0.1, (pip['frontend'], acc['frontend'])
    assert L.sedx_set_profiling(nat.h, 1) == 0
    with torch.no_grad():
        m(w)
    assert L.sedx_stage_times(nat.h, ms, len(_lib.STAGES), ctypes.byref(n)) == 0
    one = dict(zip(_lib.STAGES, ms[:]))
    assert one.pop('pipeline_wait') >= 0
    assert all(v > 0 for v in one.values()), one
    assert L.sedx_set_profiling(nat.h, 0) == 0
    for o in outs[1:]:
        assert torch.equal(o, outs[0])


def _capture(m, stage, shape, wave):
    """Run one forward with stage `stage`'s output copied out (sedx_set_capture)."""
    from sedx import _lib
    nat = m.native(torch.device('cuda', 0))
    buf = torch.full(shape, float('nan'), dtype=torch.float32, device='cuda')
    L = _lib.lib()
    _lib.check(L.sedx_set_capture(nat.h, stage, ctypes_ptr(buf), buf.numel() * 4), nat.h, 'set_capture')
    try:
        run(m, wave)
        torch.cuda.synchronize()
    finally:
        _lib.check(L.sedx_set_capture(nat.h, -1, None, 0), nat.h, 'set_capture')
    return buf.cpu().numpy()


def ctypes_ptr(t):
    import ctypes
    return ctypes.c_void_p(t.data_ptr())


# Winograd forms (SEDX_TUNE_WINO_F43): 0 = F(2x2,3x3) in every layer (block 1
# the fused conv1 + F(2,3) launch, blocks 2-4 conv_wino.hip), 1 = block 1 on
# F(2,3) and blocks 2-4 on F(4x4,3x3), 2 = F(4x4,3x3) everywhere (default)
WINO_FORMS = [('exact', None), ('x3', None), ('winograd', 0), ('winograd', 1), ('winograd', 2)]
WINO_IDS = ['exact', 'x3', 'wino-f23', 'wino-f43b24', 'wino-f43']


def build_prec(mt, prec, f43=None):
    m = build(mt).set_precision(prec)
    if f43 is not None:
        from sedx import _lib
        m.set_tuning(_lib.TUNE_WINO_F43, f43)
    return m


@pytest.mark.parametrize('prec,f43', WINO_FORMS, ids=WINO_IDS)
@pytest.mark.parametrize('mt', [GRU, TRF])
def test_stage_goldens(mt, prec, f43, golden_dir):
    """Every stage of the HIP path against the reference's own per-stage
    activations (tests/golden/stages_*.npz): bn0 output, the pooled output of
    blocks 1-3, block 4 + freq mean and the GRU / MHA output, so a
    regression names its stage.  Every Winograd form is checked."""
    g = np.load(os.path.join(golden_dir, 'stages_%s.npz' % mt))
    m = build_prec(mt, prec, f43)
    wave = g['wave']
    B = wave.shape[0]
    T = g['bn0'].shape[2]
    checks = [(0, (B, T, 64), g['bn0'][:, 0]),
              (2, None, g['block1']), (4, None, g['block2']), (6, None, g['block3']),
              (8, (B, g['cnn_out'].shape[2], 512), np.transpose(g['cnn_out'], (0, 2, 1))),
              (9, (B, g['seq_out'].shape[1], 512), g['seq_out'])]
    for stage, shape, ref in checks:
        if shape is None:               # NCHW golden -> channels-last capture
            ref = np.transpose(ref, (0, 2, 3, 1))
            shape = ref.shape
        got = _capture(m, stage, shape, wave)
        scale = max(1.0, float(np.abs(ref).max()))
        e = err(got, ref)
        print(mt, prec, 'stage', stage, shape, 'max|d| = %.3g (scale %.3g)' % (e, scale))
        assert e <= 1e-4 * scale, (stage, e)


@pytest.mark.parametrize('n_clips,seconds', [(3, 10.0), (37, 2.0), (1, 0.08)])
def test_mel_mfma_bit_identical(n_clips, seconds):
    """The n_fft 512 frontend's opt-in mel projection on
    v_mfma_f32_16x16x4_f32 (SEDX_TUNE_MEL_MFMA 1: 16 frames x one 16-band tile
    per wave, over the tile's bin range) gives the default VALU band sums'
    bits: the X0 stage (bn0 output) is
    bit-identical, a ragged last 16-frame group and a 9-frame clip included,
    and matches the reference's per-stage golden."""
    from sedx import _lib
    m = build(GRU)
    wave = synth.make_waveforms(n_clips, seconds=seconds, sample_rate=16000, seed=n_clips)
    T = wave.shape[1] // 160 + 1
    x0 = {}
    for on in (1, 0):
        _tune(m, _lib.TUNE_MEL_MFMA, on)
        x0[on] = _capture(m, 0, (n_clips, T, 64), wave)
    _tune(m, _lib.TUNE_MEL_MFMA, 0)
    assert np.isfinite(x0[1]).all()
    assert np.array_equal(x0[1], x0[0])


@pytest.mark.parametrize('f43', [0, 1, 2], ids=['f23', 'f43b24', 'f43'])
@pytest.mark.parametrize('mt', [GRU, TRF])
def test_winograd_vs_exact(mt, f43):
    """Each fp32 Winograd form (SEDX_TUNE_WINO_F43 0: F(2x2,3x3) in every
    layer; 1: block 1 F(2x2,3x3), blocks 2-4 F(4x4,3x3); 2, the default:
    F(4x4,3x3) everywhere) against the direct fp32 conv and the CPU oracle on
    the headline batch (B = 32 x 10 s): same arithmetic type, different
    rounding — framewise within 2e-5 of both, and the thresholded events of
    the Winograd form, the direct conv and the oracle all identical."""
    from sedx import inference
    wave = synth.make_waveforms(32, seconds=10.0, sample_rate=16000, seed=4321)
    ex = run(build(mt).set_precision('exact'), wave)
    wg = run(build_prec(mt, 'winograd', f43), wave)
    ref = O.forward(O.full_state(synth.make_state_dict(mt, seed=SEEDS[mt])), mt, wave=wave)
    for k in ('framewise_output', 'clipwise_output', 'embedding'):
        assert np.isfinite(wg[k]).all(), k
    e_we = err(wg['framewise_output'], ex['framewise_output'])
    e_w = err(wg['framewise_output'], ref['framewise_output'].numpy())
    e_e = err(ex['framewise_output'], ref['framewise_output'].numpy())
    e_c = err(wg['clipwise_output'], ref['clipwise_output'].numpy())
    print(mt, 'f43=%d winograd vs exact %.3g, vs oracle %.3g (clipwise %.3g; exact vs oracle %.3g)'
          % (f43, e_we, e_w, e_c, e_e))
    assert e_we <= 2e-5 and e_w <= 2e-5 and e_c <= 2e-5
    params = {'sed_high_threshold': 0.5, 'sed_low_threshold': 0.3, 'n_smooth': 10, 'n_salt': 10}
    ev = inference.events_from_framewise(wg['framewise_output'], params)
    assert len(ev) > 0 and ev == inference.events_from_framewise(ex['framewise_output'], params)
    assert ev == inference.events_from_framewise(ref['framewise_output'].numpy(), params)


def test_config5_transformer_b256():
    """BASELINE config 5 (Transformer logmel 16k, 256 clips clip-sharded over 8
    GPUs) on one GPU: the B=256 forward equals the 8 contiguous 32-clip shards
    concatenated bit for bit (what the 8 ranks compute before the gather), and
    a clip subset matches the oracle."""
    m = build(TRF)
    wave = synth.make_waveforms(256, seconds=10.0, sample_rate=16000, seed=256)
    full = run(m, wave)
    for r in range(8):
        shard = run(m, wave[32 * r:32 * (r + 1)])
        for k in ('framewise_output', 'clipwise_output', 'embedding'):
            assert np.array_equal(shard[k], full[k][32 * r:32 * (r + 1)]), (r, k)
    idx = [0, 37, 101, 200, 255]
    ref = O.forward(O.full_state(synth.make_state_dict(TRF, seed=SEEDS[TRF])), TRF, wave=wave[idx])
    for k in ('framewise_output', 'clipwise_output'):
        e = err(full[k][idx], ref[k].numpy())
        print('config 5 B=256', k, 'max|d| =', e)
        assert e <= TOL


@pytest.mark.parametrize('wino_block1', [0, 1, 2])
def test_winograd_block1_knob(wino_block1):
    """SEDX_TUNE_WINO_BLOCK1: block 1 as the Winograd F = 64 launch with conv1
    computed inside it (2), fed by a separate conv1 launch (1), or as the
    direct fused kernel (0);
    both within the Winograd bar of the oracle at the headline batch, with
    identical thresholded events, and an odd-length clip (partial last tile
    row, pooled rows dropped by floor) as close."""
    from sedx import _lib, inference
    wave = synth.make_waveforms(32, seconds=10.0, sample_rate=16000, seed=99)
    m = build(GRU).set_precision('winograd').set_tuning(_lib.TUNE_WINO_BLOCK1, wino_block1)
    got = run(m, wave)
    ex = run(build(GRU).set_precision('exact'), wave)
    ref = O.forward(O.full_state(synth.make_state_dict(GRU, seed=SEEDS[GRU])), GRU, wave=wave)
    e = err(got['framewise_output'], ref['framewise_output'].numpy())
    print('wino_block1=%d vs oracle %.3g' % (wino_block1, e))
    assert e <= 2e-5
    params = {'sed_high_threshold': 0.5, 'sed_low_threshold': 0.3, 'n_smooth': 10, 'n_salt': 10}
    assert inference.events_from_framewise(got['framewise_output'], params) == \
        inference.events_from_framewise(ex['framewise_output'], params)
    odd = synth.make_waveforms(3, seconds=7.33, sample_rate=16000, seed=5)
    ref_o = O.forward(O.full_state(synth.make_state_dict(GRU, seed=SEEDS[GRU])), GRU, wave=odd)
    assert err(run(m, odd)['framewise_output'], ref_o['framewise_output'].numpy()) <= 2e-5


def test_wino_order_bit_identical():
    """SEDX_TUNE_WINO_ORDER 1 (4 tile blocks x 8 channel groups per round of
    32 items on the 512-channel layers) and 2 (also block 1's tile blocks in
    one contiguous range per XCD) run the same items with the same
    arithmetic: bit-identical to tile block major order (B = 32 x 10 s, where
    they apply, and B = 3, where the launcher keeps the default)."""
    from sedx import _lib
    m = build(GRU).set_precision('winograd')
    for n in (32, 3):
        wave = torch.from_numpy(synth.make_waveforms(n, seconds=10.0, sample_rate=16000, seed=40 + n)).cuda()
        outs = []
        for order in (0, 1, 2):
            _tune(m, _lib.TUNE_WINO_ORDER, order)
            with torch.no_grad():
                outs.append(m(wave)['framewise_output'].clone())
        _tune(m, _lib.TUNE_WINO_ORDER, 1)
        assert torch.isfinite(outs[0]).all()
        assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2]), n


def test_wino43_item_claims_dirty_workspace_and_regimes():
    """The F(4x4,3x3) launches of a B = 32 forward claim their items from
    counters in the caller's workspace (more than two items per CU); B = 4
    runs the static item order.  A workspace filled with 0xFF bytes, two
    forwards back to back on it, and the same clips inside the two batch
    sizes all give the same framewise output bit for bit (the forward zeroes
    its counters; the item order never changes an output)."""
    import ctypes
    from sedx import _lib
    from sedx.models import _ptr
    m = build(GRU).set_precision('winograd')
    wave = torch.from_numpy(synth.make_waveforms(32, seconds=10.0, sample_rate=16000, seed=77)).cuda()
    with torch.no_grad():
        ref = m(wave)['framewise_output'].clone()
        small = m(wave[:4].contiguous())['framewise_output'].clone()
    assert torch.isfinite(ref).all()
    assert torch.equal(ref[:4], small)
    nat = m.native(wave.device)
    L = _lib.lib()
    B, length = wave.shape
    wsz = ctypes.c_size_t()
    _lib.check(L.sedx_workspace_size(nat.h, B, length, ctypes.byref(wsz)), nat.h, 'workspace_size')
    ws = torch.full((wsz.value,), 255, dtype=torch.uint8, device=wave.device)
    fw = torch.empty_like(ref)
    clip = torch.empty((B, ref.shape[2]), dtype=torch.float32, device=wave.device)
    fr, sl = ctypes.c_int64(), ctypes.c_int64()
    _lib.check(L.sedx_output_geometry(nat.h, length, ctypes.byref(fr), ctypes.byref(sl)), nat.h, 'geometry')
    emb = torch.empty((B, ref.shape[2], sl.value), dtype=torch.float32, device=wave.device)
    stream = ctypes.c_void_p(torch.cuda.current_stream(wave.device).cuda_stream)
    for _ in range(2):
        fw.fill_(float('nan'))
        _lib.check(L.sedx_forward(nat.h, _ptr(wave), B, length, _ptr(fw), _ptr(clip), _ptr(emb), _ptr(ws),
                                  wsz.value, stream), nat.h, 'forward')
        torch.cuda.synchronize()
        assert torch.equal(fw, ref)


def test_wino_block1_knob_errors():
    """A bad value for the knob is a loud error, not a silent fallback."""
    from sedx import _lib
    m = build(GRU)
    nat = m.native(torch.device('cuda', 0))
    L = _lib.lib()
    assert L.sedx_set_tuning(nat.h, _lib.TUNE_WINO_BLOCK1, 3) != 0
    assert L.sedx_set_tuning(nat.h, _lib.TUNE_WINO_BLOCK1, -1) != 0
    assert L.sedx_set_tuning(nat.h, _lib.TUNE_WINO_BLOCK1, 1) == 0


@pytest.mark.parametrize('f43', [1, 2])
@pytest.mark.parametrize('B,seconds', [(32, 10.0), (3, 7.33), (1, 2.0), (5, 0.33)])
def test_wino_block1_conv1_fused_bit_identical(B, seconds, f43):
    """F(2x2,3x3) block 1 (SEDX_TUNE_WINO_F43 1): conv1 computed inside the
    Winograd launch (WINO_BLOCK1 2) against the separate conv1 launch (1) —
    the same fma chain per channel, the same conv2.  F(4x4,3x3) block 1 (2,
    the default): conv1's launch into the chunk-of-4 layout + the C4 conv2
    (2) against the NHWC pair (1).  Every block-1 output and the framewise
    output bit for bit equal, at the headline batch, an odd length (partial
    last tile block, odd last row dropped by the pool), one short clip and
    clips of a few frames."""
    from sedx import _lib
    wave = synth.make_waveforms(B, seconds=seconds, sample_rate=16000, seed=31 + B)
    T = wave.shape[1] // 160 + 1                  # frames (hop 160, centred STFT)
    outs = []
    for v in (1, 2):
        m = build(GRU).set_precision('winograd').set_tuning(_lib.TUNE_WINO_F43, f43)
        m.set_tuning(_lib.TUNE_WINO_BLOCK1, v)
        b1 = _capture(m, 2, (B, T // 2, 32, 64), wave)
        assert not np.isnan(b1).any()
        outs.append((b1, run(m, wave)['framewise_output']))
    assert np.array_equal(outs[0][0], outs[1][0]), 'block 1 outputs differ'
    assert np.array_equal(outs[0][1], outs[1][1]), 'framewise outputs differ'


def test_winograd_batch_past_32bit_offsets():
    """A batch whose block-1 activation passes 2^31 elements (530 x 10 s clips:
    530 x 1001 x 64 x 64) runs the Winograd layers as several launches over
    whole clips; every clip's outputs stay bit-identical to running it alone."""
    m = build(GRU).set_precision('winograd')
    wave = synth.make_waveforms(530, seconds=10.0, sample_rate=16000, seed=77)
    full = run(m, wave)
    for i in (0, 264, 529):
        one = run(m, wave[i:i + 1])
        assert np.array_equal(one['framewise_output'][0], full['framewise_output'][i]), i
    torch.cuda.empty_cache()


def _replicate(mod):
    """What torch.nn.parallel.replicate hands each device's thread: every
    module replicated, parameters / buffers broadcast copies (new storage)."""
    r = mod._replicate_for_data_parallel()
    r._parameters = {k: (p.detach().clone() if p is not None else None) for k, p in mod._parameters.items()}
    r._buffers = {k: (b.clone() if b is not None else None) for k, b in mod._buffers.items()}
    r._modules = {k: _replicate(c) for k, c in mod._modules.items()}
    return r


@pytest.mark.parametrize('mt', [GRU, TRF])
def test_dataparallel_call_site(mt, monkeypatch):
    """The reference's own call site wraps the model in DataParallel
    unconditionally (pytorch/predict.py:239-242, main_strong.py:541): the
    wrapped model gives the bare model's outputs bit for bit, and replicas
    with broadcast parameter copies (the >1-GPU case) reuse the packed
    per-device handle instead of re-packing the weights every call."""
    from sedx import models
    m = build(mt)
    wave = synth.make_waveforms(4, seconds=10.0, sample_rate=16000, seed=21)
    bare = run(m, wave)
    loads = []
    orig = models._Native.load

    def counting_load(self, sd):
        loads.append(1)
        return orig(self, sd)

    monkeypatch.setattr(models._Native, 'load', counting_load)
    dp = torch.nn.DataParallel(m, device_ids=[0])
    dp.to('cuda')
    dp.eval()
    for _ in range(2):
        out = run(dp, wave)
        for k in ('framewise_output', 'clipwise_output', 'embedding'):
            assert np.array_equal(out[k], bare[k]), k
    for _ in range(3):
        r = _replicate(m)
        out = run(r, wave)
        for k in ('framewise_output', 'clipwise_output', 'embedding'):
            assert np.array_equal(out[k], bare[k]), k
    assert loads == []
