"""Golden fixtures for the voting post-processing and the
main_strong overlap sweep, produced by the REFERENCE in this build container.

Test infrastructure only (same import rules as oracle/make_golden.py).
``pytorch/main_strong.py`` is not importable (h5py, data files), so its
``binarize_pred`` (main_strong.py:870-883) is taken from the file's own AST and
executed as written; the window loops of ``inference_prob_vote``
(:1058-1097) and ``inference_prob_overlap`` (:791-835) are re-run around the
reference's ``models``, ``utilities.merge / avg_merge``,
``utilities.frame_binary_prediction_to_event_prediction`` (-> vad
.activity_detection_binary) and ``utilities.frame_prediction_to_event_prediction_v2``.

Thresholds are passed as numpy float64 (as the optimised-threshold pickles
hold them), so every binarisation compare is float64 under any numpy version.

Usage:  python oracle/make_golden_vote.py   (writes tests/golden/vote_*.npz, vote_events.json)
"""
import ast
import json
import os
import sys

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as G  # noqa: E402  (sets up the reference import paths)

import numpy as np  # noqa: E402
import torch  # noqa: E402

ref_util = G.ref_util


def _reference_function(path, name):
    tree = ast.parse(open(path).read(), path)
    node = next(n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name == name)
    ns = {'np': np}
    exec(compile(ast.Module(body=[node], type_ignores=[]), path, 'exec'), ns)
    return ns[name]


binarize_pred = _reference_function(os.path.join(G.REF, 'pytorch', 'main_strong.py'), 'binarize_pred')

VOTE_DEFAULT = {'audio_tagging_threshold': 0.099, 'sed_high_threshold': np.float64(0.5),
                'sed_low_threshold': np.float64(0.2), 'n_smooth': 10, 'n_salt': 10}   # main_strong.py:1004-1009


def vote_synthetic():
    p = G.synthetic_params(seed=9)
    p['sed_high_threshold'] = [np.float64(v) for v in p['sed_high_threshold']]
    p['sed_low_threshold'] = [np.float64(abs(v)) for v in p['sed_low_threshold']]
    return p


def windows(m, audio, sr, sample_duration, overlap_value):
    """Per-window framewise outputs of the main_strong loop (clip padded to 10 s)."""
    audio_duration = len(audio) / float(sr)
    audio = ref_util.pad_truncate_sequence(audio, sr * 10)
    out, start, end = [], 0, 0
    while end <= audio_duration:
        s = int(start * sr)
        seg = torch.reshape(torch.Tensor(audio[s:int(sample_duration * sr) + s]), (1, -1))
        with torch.no_grad():
            out.append(m(seg)['framewise_output'].data.cpu().numpy())
        start += overlap_value
        end = start + sample_duration
    return out


def merge_windows(wins, sample_duration, overlap_value, bin_thres=None, sed_thresholds=False):
    merged, prev = None, None
    for num_segment, curr in enumerate(wins, start=1):
        if bin_thres is not None:
            curr = binarize_pred(curr, bin_thres, sed_thresholds)
        if num_segment == 2:
            merged = ref_util.merge(prev, curr, sample_duration, num_segment, overlap_value)
        elif num_segment > 2:
            merged = ref_util.merge(merged, curr, sample_duration, num_segment, overlap_value)
        else:
            merged = curr
        prev = curr
    if bin_thres is None:
        merged = ref_util.avg_merge(merged, sample_duration, overlap_value)
    return merged


def _copy(p):
    return {k: (list(v) if isinstance(v, list) else v) for k, v in p.items()}


def _json_params(p):
    return {k: ([float(x) for x in v] if isinstance(v, list) else float(v) if isinstance(v, np.floating) else v)
            for k, v in p.items()}


def main():
    audio = G.synth.make_waveforms(2, seconds=10.0, sample_rate=16000, seed=1234)[1].astype(np.float32)
    settings = {G.GRU: [(1, 5), (0.5, 7)], G.TRF: [(0.5, 6), (1, 7)]}
    rng = np.random.default_rng(21)
    mid = {'audio_tagging_threshold': 0.1, 'sed_high_threshold': np.float64(0.5),
           'sed_low_threshold': [np.float64(v) for v in np.round(rng.uniform(0.3, 0.6, 25), 3)],
           'n_smooth': 3, 'n_salt': 2}
    params = {'default': VOTE_DEFAULT, 'synthetic': vote_synthetic(), 'mid': mid}
    ev = {'params_' + k: _json_params(v) for k, v in params.items()}
    for mt, combos in settings.items():
        m = G.build(mt)
        arrays = {}
        ev[mt] = {}
        for ov, sd in combos:
            tag = '%s_%s' % (ov, sd)
            wins = windows(m, audio, 16000, sd, ov)
            arrays['windows_' + tag] = np.concatenate(wins, axis=0)          # [n_win, Tw, C]
            arrays['avg_' + tag] = merge_windows(wins, sd, ov)                # inference_prob_overlap merge
            ev[mt]['overlap_' + tag] = ref_util.frame_prediction_to_event_prediction_v2(
                arrays['avg_' + tag].copy(), 'clip', _copy(VOTE_DEFAULT), 100)
            for which, p in params.items():
                scalar = not isinstance(p['sed_low_threshold'], list)
                votes = merge_windows(wins, sd, ov, p['sed_low_threshold'], sed_thresholds=not scalar)
                arrays['votes_%s_%s' % (which, tag)] = votes.astype(np.float32)
                assert np.array_equal(arrays['votes_%s_%s' % (which, tag)].astype(np.float64), votes)
                ev[mt]['vote_%s_%s' % (which, tag)] = ref_util.frame_binary_prediction_to_event_prediction(
                    votes, ov, sd, 'clip', _copy(p))
        np.savez_compressed(os.path.join(G.OUT, 'vote_%s.npz' % mt), **arrays)
    for mt in settings:
        for key, lst in ev[mt].items():
            ev[mt][key] = [{'filename': e['filename'], 'onset': float(e['onset']), 'offset': float(e['offset']),
                            'event_label': e['event_label']} for e in lst]
    with open(os.path.join(G.OUT, 'vote_events.json'), 'w') as f:
        json.dump({'settings': {mt: [list(c) for c in cs] for mt, cs in settings.items()}, **ev}, f, indent=0)
    print('vote golden written to', G.OUT)


if __name__ == '__main__':
    main()
