"""CPU-only checks of the product's host side: the C-ABI library loads and
exports every symbol include/sedx.h declares, the native event extraction
(host C++) matches the reference's vad known answers, and the model classes
keep the reference state_dict contract.  No GPU compute is called."""
import json
import os
import re

import numpy as np
import pytest
import torch

from oracle import sed_oracle as O

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_symbols():
    src = open(os.path.join(REPO, 'include', 'sedx.h')).read()
    return sorted(set(re.findall(r'\b(sedx_[a-z0-9_]+)\s*\(', src)))


def test_library_exports_every_declared_symbol():
    from sedx import _lib
    L = _lib.lib()
    syms = _header_symbols()
    assert len(syms) >= 15
    for s in syms:
        assert hasattr(L, s), s
    assert sorted(_lib.EXPORTS) == syms
    assert b'gfx950' in L.sedx_version()


def test_state_dict_contract():
    from sedx import models
    exp = {'Cnn_9layers_Gru_FrameAtt': (73, 6178336), 'Cnn_9layers_Transformer_FrameAtt': (75, 6047264)}
    for mt, (nk, ne) in exp.items():
        m = getattr(models, mt)(16000, 512, 160, 64, 25, 7000, 25, 'logmel')
        sd = m.state_dict()
        assert len(sd) == nk and sum(v.numel() for v in sd.values()) == ne
        fr = O.frontend_state('16k')
        for k, v in fr.items():
            np.testing.assert_allclose(sd[k].numpy(), v, rtol=2e-6, atol=2e-7)


def test_frontend_construction_matches_reference(golden_dir):
    from sedx import stft
    g = np.load(os.path.join(golden_dir, 'frontend.npz'))
    for q, p in O.PRESETS.items():
        w = stft.mel_weights(p['sample_rate'], p['window_size'], 64, p['fmin'], p['fmax'])
        np.testing.assert_allclose(w, g['melW_' + q], rtol=2e-6, atol=1e-9)


def test_native_events_match_vad_kat(golden_dir):
    from sedx import inference
    kat = json.load(open(os.path.join(golden_dir, 'vad_kat.json')))
    for case in kat:
        if 'x' not in case:
            continue
        x = np.asarray(case['x'], np.float32)[None, :, None]
        params = {'sed_high_threshold': case['thres'], 'sed_low_threshold': case['low_thres'],
                  'n_smooth': case['n_smooth'], 'n_salt': case['n_salt']}
        try:
            got = inference.event_pairs(x, params)[:, 2:].tolist()
        except RuntimeError:
            got = 'raises'
        # the reference is run on float64 arrays here; float32 compare is identical
        # unless a value sits within float32 rounding of a threshold
        assert got == case['pairs'], case


def test_native_events_match_golden_events(golden_dir):
    from sedx import inference
    ev = json.load(open(os.path.join(golden_dir, 'events.json')))
    for mt in ('Cnn_9layers_Gru_FrameAtt', 'Cnn_9layers_Transformer_FrameAtt'):
        merged = np.load(os.path.join(golden_dir, 'windowed_%s.npz' % mt))['merged_5_1']
        for which in ('default', 'synthetic'):
            got = inference.events_from_framewise(merged, ev['params_' + which])
            assert got == ev[mt][which]


def test_native_events_match_long_file_goldens(golden_dir):
    """Host C++ events over the reference's long-file merges (183 / 131
    windows, 18,700 / 7,100 frames; oracle/make_golden_long.py)."""
    from sedx import inference
    ev = json.load(open(os.path.join(golden_dir, 'long_events.json')))
    for case, c in ev['cases'].items():
        g = np.load(os.path.join(golden_dir, 'long_%s.npz' % case))
        for mt in ('Cnn_9layers_Gru_FrameAtt', 'Cnn_9layers_Transformer_FrameAtt'):
            for which in ('default', 'synthetic'):
                got = inference.events_from_framewise(g[mt], ev['params_' + which])
                assert got == c[mt][which], (case, mt, which)


def test_events_random_vs_oracle():
    from sedx import inference
    rng = np.random.default_rng(3)
    for _ in range(20):
        fw = rng.uniform(0, 1, (2, 200, 25)).astype(np.float32)
        fw = np.cumsum(fw - 0.5, axis=1) / 8 + 0.5
        fw = fw.astype(np.float32)
        params = {'sed_high_threshold': rng.uniform(0.4, 0.7, 25).tolist(),
                  'sed_low_threshold': rng.uniform(0.1, 0.4, 25).tolist(),
                  'n_smooth': int(rng.integers(0, 12)), 'n_salt': int(rng.integers(0, 12))}
        try:
            got = inference.events_from_framewise(fw, params)
        except RuntimeError:
            with pytest.raises(IndexError):
                O.events_from_framewise(fw, params)
            continue
        assert got == O.events_from_framewise(fw, params)


def test_window_geometry_host_rules():
    # loop control of predict.py:297-338 on the oracle side
    assert O.window_starts(10.0, 5, 1) == [0, 1, 2, 3, 4, 5]
    assert len(O.window_starts(10.0, 6, 0.5)) == 9
    assert O.window_starts(3.0, 5, 1) == [0]


DRIVER_CASES = [  # (driver, overlap, sample_duration, overlap_value, seconds)
    ('predict', True, 5, 1.0, 10.0), ('predict', True, 5, 0.5, 23.0), ('predict', False, 5, 1.0, 23.0),
    ('predict', False, 5, 0.7, 17.3), ('predict', True, 6, 0.5, 71.3), ('predict', True, 5, 1.0, 187.37),
    ('predict', True, 5, 1.0, 3.2), ('main_strong', True, 5, 0.7, 10.0), ('main_strong', True, 6, 0.9, 10.0),
    ('main_strong', True, 7, 1.3, 10.0), ('main_strong', True, 5, 0.1, 10.0), ('main_strong', True, 5, 0.3, 9.9),
    ('main_strong', True, 5, 1.0, 12.3), ('main_strong', True, 6, 0.5, 8.7), ('main_strong', True, 7, 0.9, 14.1)]


@pytest.mark.parametrize('driver,overlap,sd,ov,secs', DRIVER_CASES)
def test_native_window_starts_match_reference_loops(driver, overlap, sd, ov, secs):
    """sedx_window_starts (host C++, no GPU) against the reference's loop
    control restated in the oracle: predict.py:297-338 strides 1 s with
    --overlap, else sample_duration; main_strong.py:790-832 strides
    overlap_value (float64 running start) over the clip padded to 10 s and
    feeds windows past 10 s shorter."""
    from sedx import inference
    L = int(round(secs * 16000))
    starts, lens = inference.window_starts(16000, L, sd, ov, driver, overlap)
    ref = O.window_starts(L / 16000., sd, O.driver_stride(driver, sd, ov, overlap))
    assert starts == [int(s * 16000) for s in ref]
    for s, n in zip(starts, lens):
        want = sd * 16000 if driver == 'predict' else max(0, min(s + sd * 16000, 160000) - s)
        assert n == want


def _ref_merge_all(wins, sd, ov, avg):
    merged = wins[0].copy()
    for k in range(2, len(wins) + 1):
        merged = O.merge(merged if k > 2 else wins[0], wins[k - 1], sd, k, ov)
    return O.avg_merge(merged, sd, ov) if avg else merged


@pytest.mark.parametrize('seed', range(40))
def test_native_merge_matches_numpy_merge(seed):
    """sedx_merge_host (the host plan the GPU merge runs by) against
    utilities.merge / avg_merge (restated in the oracle, numpy semantics) on
    random windows, bit for bit: random window counts and lengths (incl.
    ragged last windows), steps below / at / above the window length
    (numpy's clamped slicing concatenates; broadcasting of a 1-frame
    operand), float and zero steps; where numpy raises, sedx raises."""
    from sedx import inference
    rng = np.random.default_rng(seed)
    n = int(rng.integers(1, 12))
    tw = int(rng.choice([1, 2, 40, 96, 100, 296, 400, 496, 500]))
    frames = [tw] * n
    if rng.random() < 0.4:                     # shorter trailing windows (main_strong past 10 s)
        for j in range(int(rng.integers(1, 3))):
            frames[-1 - j % n] = int(rng.integers(1, tw + 1))
    sd = int(rng.integers(1, 8))
    ov = float(rng.choice([0.5, 0.7, 0.9, 1.0, 1.3, 1.4, 1.9, 2.0, 3.0, 4.99, 5.0, 6.0, 10.0, 0.004, -0.5]))
    avg = bool(rng.random() < 0.7)
    C = 3
    wins = [rng.uniform(0, 1, (1, f, C)).astype(np.float32) for f in frames]
    try:
        ref = _ref_merge_all(wins, sd, ov, avg)
    except ValueError:
        with pytest.raises(ValueError):
            inference.merge_host(wins, sd, ov, avg)
        return
    got = inference.merge_host(wins, sd, ov, avg)
    assert got.shape == ref.shape
    np.testing.assert_array_equal(got, ref.astype(np.float32))


def test_native_merge_float_overlap_steps():
    """int(100 * overlap_value) in float64: 70 / 90 / 130 / 140 / 190
    frames (a float32 overlap_value would give 69 / 89 / ...)."""
    from sedx import inference
    for ov, step in ((0.7, 70), (0.9, 90), (1.3, 130), (1.4, 140), (1.9, 190)):
        assert int(100 * ov) == step
        wins = [np.ones((1, 500, 1), np.float32)] * 3
        got = inference.merge_host(wins, 5, ov, avg=False)
        assert got.shape[1] == 500 + 2 * step


def test_no_packed_fp32_in_any_kernel():
    """Every kernel's gfx950 ISA is free of packed FP32 VALU (v_pk_add/mul/
    fma_f32): measured on MI355X, packed FP32 beside MFMA waves on the same
    SIMD returns wrong values (tools/fe_race.cpp; sedx_internal.h "packed
    FP32").  `make isa-check` compiles each .hip with the library's flags
    (-fno-slp-vectorize -fno-vectorize) and greps the assembly."""
    import shutil
    import subprocess
    if shutil.which('/opt/rocm/bin/hipcc') is None:
        pytest.skip('needs hipcc')
    pkg = os.path.join(REPO, 'sound-event-detection_amd')
    r = subprocess.run(['make', '-s', '-C', pkg, '-j8', 'isa-check'], capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert 'no packed FP32 VALU' in r.stdout


def test_dataparallel_replicas_reuse_the_source_handle(monkeypatch):
    """torch.nn.DataParallel (pytorch/predict.py:239) re-replicates the model on
    every forward, each replica holding freshly broadcast parameter copies
    (new data_ptrs).  The handle cache is shared with the replicas and keyed
    on the SOURCE module's parameters, so a replica does not re-pack the
    weights (no sedx_load_param); an in-place update of the source does."""
    import copy
    import io
    from sedx import models, synth

    loads = []

    class FakeNative(object):          # stands in for the libsedx handle (no GPU here)
        def __init__(self, cfg, idx):
            self.device_index, self.signature, self.precision, self.h = idx, None, 'winograd', None

        def load(self, sd):
            loads.append(len(sd))

    monkeypatch.setattr(models, '_Native', FakeNative)
    mt = 'Cnn_9layers_Gru_FrameAtt'
    m = getattr(models, mt)(16000, 512, 160, 64, 25, 7000, 25, 'logmel')
    sd = m.state_dict()
    for k, v in synth.make_state_dict(mt, seed=0).items():
        sd[k] = torch.from_numpy(v)
    m.load_state_dict(sd)
    m.eval()
    dev = torch.device('cuda', 0)
    m.native(dev)
    assert len(loads) == 1
    m.native(dev)
    assert len(loads) == 1
    def replicate(mod):
        """torch.nn.parallel.replicate for one device without a GPU: every
        module replicated, parameters and buffers broadcast copies (same
        values, new storage)"""
        r = mod._replicate_for_data_parallel()
        r._parameters = {k: (p.detach().clone() if p is not None else None) for k, p in mod._parameters.items()}
        r._buffers = {k: (b.clone() if b is not None else None) for k, b in mod._buffers.items()}
        r._modules = {k: replicate(c) for k, c in mod._modules.items()}
        return r

    for _ in range(3):                 # one replica per DataParallel call
        r = replicate(m)
        assert r._natives is m._natives and r._weights_source() is m
        assert r._signature() != m._signature()
        assert r.native(dev) is m._natives[0]
    assert len(loads) == 1
    with torch.no_grad():
        m.conv_block2.conv1.weight.mul_(1.0)   # in-place update of the source
    replicate(m).native(dev)
    assert len(loads) == 2
    # copies / pickles start with their own empty cache
    c = copy.deepcopy(m)
    assert isinstance(c._natives, models._HandleCache) and len(c._natives) == 0
    assert c._weights_source() is c
    buf = io.BytesIO()
    torch.save(m, buf)


def test_weights_signature_follows_every_change(monkeypatch):
    """The packed weights of a handle are re-made after any change the forward
    must see, and only then: the per-call check (models._SedModel._signature)
    re-walks the state_dict only after a parameter / buffer / submodule was
    registered anywhere, and otherwise re-reads the cached tensors' storage
    and version — so an in-place update, a `.data` swap, a replaced Parameter
    and a new buffer each re-pack once, and a plain repeat does not."""
    import torch
    from sedx import models

    loads = []

    class FakeNative(object):          # stands in for the libsedx handle (no GPU here)
        def __init__(self, cfg, idx):
            self.device_index, self.signature, self.precision, self.h = idx, None, 'winograd', None

        def load(self, sd):
            loads.append(sorted(sd))

    monkeypatch.setattr(models, '_Native', FakeNative)
    m = models.Cnn_9layers_Gru_FrameAtt(16000, 512, 160, 64, 25, 7000, 25, 'logmel').eval()
    dev = torch.device('cuda', 0)

    def packs():
        m.native(dev)
        return len(loads)

    assert packs() == 1 and packs() == 1
    with torch.no_grad():
        m.conv_block3.conv2.weight.mul_(0.5)               # in place: version counter
    assert packs() == 2 and packs() == 2
    m.bn0.weight.data = m.bn0.weight.data.clone()         # new storage, no registration
    assert packs() == 3
    m.att_block.cla.bias = torch.nn.Parameter(torch.zeros(25))   # replaced Parameter (registration hook)
    assert packs() == 4 and packs() == 4
    m.bn0.register_buffer('extra', torch.zeros(1))        # new state_dict key
    assert packs() == 5 and 'bn0.extra' in loads[-1]
    m.load_state_dict(m.state_dict())                      # copy_ into every tensor
    assert packs() == 6 and packs() == 6


def test_python_tuning_constants_match_the_header():
    """The ctypes mirror's knob numbers (sedx/_lib.py) and bench.py's GRU
    kernel table are the values include/sedx.h declares (a drifted number
    would silently A/B the wrong implementation)."""
    import re
    from sedx import _lib
    import bench
    hdr = open(os.path.join(REPO, 'include', 'sedx.h')).read()
    enum = {m.group(1): int(m.group(2)) for m in re.finditer(r'\b(SEDX_[A-Z0-9_]+)\s*=\s*(\d+)', hdr)}
    for name in ('GRU_KERNEL', 'GRU_HANDOFF', 'WINO_BLOCK1', 'MEL_MFMA', 'GRU_SPIN', 'WINO_ORDER', 'GAMMA_SPEC'):
        assert getattr(_lib, 'TUNE_' + name) == enum['SEDX_TUNE_' + name], name
    for key, name in (('coop', 'COOP'), ('simple', 'SIMPLE'), ('tag16', 'TAG16'), ('tag8', 'TAG8'),
                      ('coop16', 'COOP16'), ('auto', 'AUTO'), ('ksplit', 'KSPLIT')):
        assert bench.GRU_KERNELS[key] == enum['SEDX_GRU_KERNEL_' + name], key
