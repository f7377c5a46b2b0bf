"""ORACLE (test infrastructure only): CPU restatement of the reference SED
inference path.  See ``oracle/__init__.py`` for the usage rule.

Every function cites the reference file:line it restates.  Arithmetic is fp32
torch-eager on the CPU with the reference's own op sequence (Conv1d-DFT STFT,
matmul mel, conv2d/BN/ReLU/avg-pool, GRU recurrence, bmm attention), so its
rounding matches the reference to ~1e-6.  Post-processing (merge, avg_merge,
vad) is numpy / pure Python, quirk-exact.
"""
import math

import numpy as np
import torch
import torch.nn.functional as F

FRAMES_PER_SECOND = 100          # utils/config.py:13 (sample_rate // hop_size)
LABELS = ['Applause', 'Breathing', 'Chatter', 'Cheering', 'Child_speech_kid_speaking',
          'Clapping', 'Conversation', 'Cough', 'Crowd', 'Crying_sobbing',
          'Female_speech_woman_speaking', 'Laughter', 'Male_speech_man_speaking', 'Run',
          'Screaming', 'Shout', 'Sneeze', 'Walk_footsteps', 'Whispering',
          'Air_horn_truck_horn', 'Car_alarm', 'Emergency_vehicle', 'Explosion',
          'Gunshot_gunfire', 'Siren']   # utils/config.py:31

# quality presets: pytorch/predict.py:186-205, pytorch/main_strong.py:646-669
PRESETS = {
    '8k': dict(sample_rate=8000, window_size=256, hop_size=80, mel_bins=64, fmin=12, fmax=3500),
    '16k': dict(sample_rate=16000, window_size=512, hop_size=160, mel_bins=64, fmin=25, fmax=7000),
    '32k': dict(sample_rate=32000, window_size=1024, hop_size=320, mel_bins=64, fmin=50, fmax=14000),
}


# ---------------------------------------------------------------------------
# frontend construction (pytorch/stft.py:157-221, :674-692)
# ---------------------------------------------------------------------------
def stft_weights(n_fft):
    """conv_real / conv_imag weights [n_fft//2+1, 1, n_fft]: Re/Im of the DFT
    matrix columns 0..n_fft/2 times the periodic Hann window
    (pytorch/stft.py:192-217; DFT matrix pytorch/stft.py:20-24)."""
    n = np.arange(n_fft)
    win = 0.5 - 0.5 * np.cos(2.0 * np.pi * n / n_fft)          # scipy hann, fftbins=True
    k = np.arange(n_fft // 2 + 1)
    ang = -2.0 * np.pi * np.outer(n, k) / n_fft                 # W[n, k]
    wr = (np.cos(ang) * win[:, None]).T.astype(np.float32)[:, None, :]
    wi = (np.sin(ang) * win[:, None]).T.astype(np.float32)[:, None, :]
    return wr, wi


def _hz_to_mel(f):
    f = np.asarray(f, dtype=np.float64)
    f_sp = 200.0 / 3
    logstep = np.log(6.4) / 27.0
    return np.where(f >= 1000.0, 15.0 + np.log(np.maximum(f, 1e-30) / 1000.0) / logstep, f / f_sp)


def _mel_to_hz(m):
    m = np.asarray(m, dtype=np.float64)
    f_sp = 200.0 / 3
    logstep = np.log(6.4) / 27.0
    return np.where(m >= 15.0, 1000.0 * np.exp(logstep * (m - 15.0)), f_sp * m)


def mel_filterbank(sr, n_fft, n_mels, fmin, fmax):
    """melW [n_fft//2+1, n_mels] = librosa.filters.mel(...).T, librosa-0.8
    Slaney scale + Slaney area norm (pytorch/stft.py:688-689; third-party
    algorithm restated)."""
    n_bins = n_fft // 2 + 1
    fftfreqs = np.linspace(0, sr / 2.0, n_bins)
    mel_f = _mel_to_hz(np.linspace(_hz_to_mel(fmin), _hz_to_mel(fmax), n_mels + 2))
    fdiff = np.diff(mel_f)
    ramps = mel_f[:, None] - fftfreqs[None, :]
    w = np.zeros((n_mels, n_bins), np.float32)
    for i in range(n_mels):
        w[i] = np.maximum(0, np.minimum(-ramps[i] / fdiff[i], ramps[i + 2] / fdiff[i + 1]))
    w *= (2.0 / (mel_f[2:n_mels + 2] - mel_f[:n_mels]))[:, None]
    return np.ascontiguousarray(w.T)


def frontend_state(preset='16k'):
    p = PRESETS[preset]
    wr, wi = stft_weights(p['window_size'])
    return {
        'spectrogram_extractor.stft.conv_real.weight': wr,
        'spectrogram_extractor.stft.conv_imag.weight': wi,
        'logmel_extractor.melW': mel_filterbank(p['sample_rate'], p['window_size'],
                                                p['mel_bins'], p['fmin'], p['fmax']),
    }


# ---------------------------------------------------------------------------
# forward pieces
# ---------------------------------------------------------------------------
def _t(a):
    return a if isinstance(a, torch.Tensor) else torch.from_numpy(np.asarray(a))


def logmel(sd, wave):
    """Spectrogram + LogmelFilterBank (pytorch/stft.py:223-247, :651-670,
    :694-734; top_db=None, ref=1, amin=1e-10 per models.py:568-574).
    wave [B, L] -> [B, 1, T, n_mels]."""
    wr = _t(sd['spectrogram_extractor.stft.conv_real.weight'])
    wi = _t(sd['spectrogram_extractor.stft.conv_imag.weight'])
    n_fft = wr.shape[-1]
    hop = sd['_hop']
    x = F.pad(wave[:, None, :], (n_fft // 2, n_fft // 2), mode='reflect')
    re = F.conv1d(x, wr, stride=hop)[:, None].transpose(2, 3)
    im = F.conv1d(x, wi, stride=hop)[:, None].transpose(2, 3)
    power = re ** 2 + im ** 2
    mel = torch.matmul(power, _t(sd['logmel_extractor.melW']))
    out = 10.0 * torch.log10(torch.clamp(mel, min=1e-10, max=np.inf))
    out -= 10.0 * np.log10(np.maximum(1e-10, 1.0))
    return out


def _bn(sd, p, x):
    return F.batch_norm(x, _t(sd[p + '.running_mean']), _t(sd[p + '.running_var']),
                        _t(sd[p + '.weight']), _t(sd[p + '.bias']), False, 0.0, 1e-5)


def bn0(sd, x):
    """models.py:642-644: BatchNorm2d(64) over the mel axis via transpose."""
    return _bn(sd, 'bn0', x.transpose(1, 3)).transpose(1, 3)


def conv_block(sd, k, x, pool):
    """ConvBlock.forward (models.py:125-141) with avg pooling."""
    p = 'conv_block%d' % k
    x = F.relu(_bn(sd, p + '.bn1', F.conv2d(x, _t(sd[p + '.conv1.weight']), padding=1)))
    x = F.relu(_bn(sd, p + '.bn2', F.conv2d(x, _t(sd[p + '.conv2.weight']), padding=1)))
    return F.avg_pool2d(x, kernel_size=pool)


def cnn(sd, x):
    """bn0 -> 4 ConvBlocks -> freq mean (models.py:642-668). x [B,1,T,64]
    -> [B, 512, T/8]; also returns the per-block activations."""
    acts = {}
    x = bn0(sd, x)
    acts['bn0'] = x
    for k, pool in ((1, (2, 2)), (2, (2, 2)), (3, (2, 2)), (4, (1, 1))):
        x = conv_block(sd, k, x, pool)
        acts['block%d' % k] = x
    x = torch.mean(x, dim=3)
    acts['cnn_out'] = x
    return x, acts


def gru_bidirectional(sd, x):
    """torch nn.GRU(512, 256, bidirectional, batch_first) recurrence
    (models.py:614-615, :670), gate order (r, z, n):
      r = s(Wir x + bir + Whr h + bhr); z = s(Wiz x + biz + Whz h + bhz)
      n = tanh(Win x + bin + r * (Whn h + bhn)); h' = (1 - z) n + z h.
    x [B, T, 512] -> [B, T, 512] (fwd || bwd)."""
    B, T, _ = x.shape
    outs = []
    for sfx, order in (('', range(T)), ('_reverse', range(T - 1, -1, -1))):
        w_ih, w_hh = _t(sd['gru.weight_ih_l0' + sfx]), _t(sd['gru.weight_hh_l0' + sfx])
        b_ih, b_hh = _t(sd['gru.bias_ih_l0' + sfx]), _t(sd['gru.bias_hh_l0' + sfx])
        H = w_hh.shape[1]
        gi = torch.matmul(x, w_ih.t()) + b_ih
        h = torch.zeros(B, H, dtype=x.dtype)
        out = torch.empty(B, T, H, dtype=x.dtype)
        for t in order:
            gh = torch.matmul(h, w_hh.t()) + b_hh
            r = torch.sigmoid(gi[:, t, :H] + gh[:, :H])
            z = torch.sigmoid(gi[:, t, H:2 * H] + gh[:, H:2 * H])
            n = torch.tanh(gi[:, t, 2 * H:] + r * gh[:, 2 * H:])
            h = (1 - z) * n + z * h
            out[:, t] = h
        outs.append(out)
    return torch.cat(outs, dim=2)


def multihead(sd, x, n_head=8, d_k=64):
    """MultiHead.forward + ScaledDotProductAttention (models.py:853-877,
    :805-820): no residual, no LayerNorm, dropout inert in eval.
    x [B, T, 512] -> [B, T, 512]."""
    B, T, _ = x.shape

    def lin(nm, v):
        return F.linear(v, _t(sd['multihead.%s.weight' % nm]), _t(sd['multihead.%s.bias' % nm]))

    q = lin('w_qs', x).view(B, T, n_head, d_k).permute(2, 0, 1, 3).contiguous().view(-1, T, d_k)
    k = lin('w_ks', x).view(B, T, n_head, d_k).permute(2, 0, 1, 3).contiguous().view(-1, T, d_k)
    v = lin('w_vs', x).view(B, T, n_head, d_k).permute(2, 0, 1, 3).contiguous().view(-1, T, d_k)
    attn = torch.softmax(torch.bmm(q, k.transpose(1, 2)) / np.power(d_k, 0.5), dim=2)
    o = torch.bmm(attn, v).view(n_head, B, T, d_k).permute(1, 2, 0, 3).contiguous().view(B, T, -1)
    return F.relu(lin('fc', o))


def att_block(sd, x):
    """AttBlock.forward, activation='sigmoid' (models.py:161-175).
    x [B, 512, T] -> clipwise [B, C], norm_att [B, C, T], cla [B, C, T]."""
    tmp = F.conv1d(x, _t(sd['att_block.att.weight']), _t(sd['att_block.att.bias']))
    att = torch.exp(torch.clamp(tmp, -10, 10) / 1.0) + 1e-6
    norm_att = att / torch.sum(att, dim=2)[:, :, None]
    cla = torch.sigmoid(F.conv1d(x, _t(sd['att_block.cla.weight']), _t(sd['att_block.cla.bias'])))
    return torch.sum(norm_att * cla, dim=2), norm_att, cla


def roundup(x):
    """models.py:62-63"""
    return x if x % 100 == 0 else x + 100 - x % 100


def framewise_from_cla(cla, pad_to_100):
    """interpolate x8 (models.py:84-95) then, GRU model only, repeat the last
    frame up to roundup(T) when T != 1000 (models.py:65-81, :678-681)."""
    fw = cla.transpose(1, 2)
    B, T, C = fw.shape
    fw = fw[:, :, None, :].repeat(1, 1, 8, 1).reshape(B, T * 8, C)
    if pad_to_100 and fw.shape[1] != 1000:
        n = roundup(fw.shape[1])
        fw = torch.cat([fw, fw[:, -1:, :].repeat(1, n - fw.shape[1], 1)], dim=1)
    return fw


def forward(sd, model_type, wave=None, features=None, return_acts=False):
    """Cnn_9layers_{Gru,Transformer}_FrameAtt.forward in eval mode
    (models.py:625-688, :1029-1077).  ``wave`` [B, L] (logmel) or
    ``features`` [B, 1, T, 64] (gamma branch models.py:636-640, already
    transposed).  ``sd`` must hold '_hop'."""
    with torch.no_grad():
        if features is None:
            x = logmel(sd, _t(wave).float())
        else:
            x = _t(features).float()
        x_in = x
        x, acts = cnn(sd, x)
        acts['logmel'] = x_in
        x = x.transpose(1, 2)
        if model_type == 'Cnn_9layers_Gru_FrameAtt':
            x = gru_bidirectional(sd, x)
        else:
            x = multihead(sd, x)
        acts['seq_out'] = x
        x = x.transpose(1, 2)
        clipwise, norm_att, cla = att_block(sd, x)
        acts['norm_att'] = norm_att
        fw = framewise_from_cla(cla, model_type == 'Cnn_9layers_Gru_FrameAtt')
        emb = cla if model_type == 'Cnn_9layers_Gru_FrameAtt' else x
        out = {'framewise_output': fw, 'clipwise_output': clipwise, 'embedding': emb}
    if return_acts:
        return out, acts
    return out


def full_state(model_sd, preset='16k'):
    sd = dict(model_sd)
    sd.update(frontend_state(preset))
    sd['_hop'] = PRESETS[preset]['hop_size']
    return sd


# ---------------------------------------------------------------------------
# windowed drivers + merge (pytorch/predict.py:297-349, utils/utilities.py:405-446)
# ---------------------------------------------------------------------------
def pad_truncate_sequence(x, max_len):
    """utils/utilities.py:66-70"""
    if len(x) < max_len:
        return np.concatenate((x, np.zeros(max_len - len(x))))
    return x[0:max_len]


def merge(prev, curr, sample_duration, num_segment, overlap_value=1):
    """utils/utilities.py:405-423: overlap-add of the next window at frame
    offset (num_segment-1)*100*overlap."""
    ov = int(100 * overlap_value)
    front = (num_segment - 1) * ov
    back = prev.shape[1] - front
    mid = prev[:, front:] + curr[:, :back]
    return np.concatenate((np.concatenate((prev[:, :front], mid), axis=1), curr[:, back:]), axis=1)


def avg_merge(merged, sample_duration, overlap_value=1):
    """utils/utilities.py:425-446: divide 100*ov-frame blocks by the
    reference's fixed schedule (NOT the true coverage)."""
    ov = int(100 * overlap_value)
    interval = sample_duration * 100 - ov
    N = merged.shape[1]
    for i in range(ov, N - ov, ov):
        if i < interval:
            d = i // ov + 1
        elif i >= N - interval:
            d = (N - i) // ov + 1
        else:
            d = sample_duration
        merged[:, i:i + ov] /= d
    return merged


def window_starts(audio_duration, sample_duration, stride):
    """Loop control of pytorch/predict.py:297-338 and
    pytorch/main_strong.py:791-832 (``while end <= audio_duration``;
    ``start += stride``)."""
    starts = []
    start, end = 0, 0
    while end <= audio_duration:
        starts.append(start)
        start += stride
        end = start + sample_duration
    return starts


def driver_stride(driver, sample_duration, overlap_value, overlap=True):
    """predict.py:334-337 (``start += 1`` with --overlap, else ``start +=
    sample_duration``) / main_strong.py:829 (``start += overlap_value``)."""
    if driver == 'predict':
        return 1 if overlap else sample_duration
    if driver == 'main_strong':
        return overlap_value
    raise ValueError(driver)


def predict_windows(sd, model_type, audio, sample_rate, sample_duration=5, overlap_value=1.0,
                    driver='predict', overlap=True, audio_duration=None):
    """Per-clip windowed inference: predict.py:297-349 (driver='predict':
    every window pad_truncate'd, :305) or main_strong.py:786-835
    (driver='main_strong': the clip pad_truncate'd to 10 s, :790, windows
    sliced without padding, :795-797).  Runs the model batch-1 per window
    exactly like the reference; returns merged [1,N,C]."""
    if audio_duration is None:
        audio_duration = len(audio) / float(sample_rate)
    if driver == 'main_strong':
        audio = pad_truncate_sequence(audio, sample_rate * 10)
    n_win = int(sample_rate * sample_duration)
    merged, prev = None, None
    stride = driver_stride(driver, sample_duration, overlap_value, overlap)
    for num_segment, start in enumerate(window_starts(audio_duration, sample_duration, stride), start=1):
        s = int(start * sample_rate)
        seg = audio[s:int(sample_duration * sample_rate) + s]
        if driver == 'predict':
            seg = pad_truncate_sequence(seg, n_win)
        seg = torch.Tensor(np.asarray(seg))[None, :]
        curr = forward(sd, model_type, wave=seg)['framewise_output'].numpy()
        if num_segment == 1:
            merged = curr
        elif num_segment == 2:
            merged = merge(prev, curr, sample_duration, num_segment, overlap_value)
        else:
            merged = merge(merged, curr, sample_duration, num_segment, overlap_value)
        prev = curr
    return avg_merge(merged, sample_duration, overlap_value)


# ---------------------------------------------------------------------------
# thresholding (utils/vad.py:11-199, pytorch/predict.py:57-121)
# ---------------------------------------------------------------------------
def find_bgn_fin_pairs(locts):
    """utils/vad.py:108-130 incl. the +1 on every non-first bgn and the
    un-incremented final fin."""
    if len(locts) == 0:
        return []
    bgns, fins = [locts[0]], []
    for i in range(1, len(locts)):
        if locts[i] - locts[i - 1] > 1:
            fins.append(locts[i - 1] + 1)
            bgns.append(locts[i] + 1)
    fins.append(locts[-1])
    return [[b, f] for b, f in zip(bgns, fins)]


def smooth(pairs, n_smooth):
    """utils/vad.py:158-183"""
    if len(pairs) == 0:
        return []
    out = []
    mem_bgn, fin = pairs[0]
    for n in range(1, len(pairs)):
        pre_fin = pairs[n - 1][1]
        bgn, fin = pairs[n]
        if bgn - pre_fin > n_smooth:
            out.append([mem_bgn, pre_fin])
            mem_bgn = bgn
    out.append([mem_bgn, fin])
    return out


def second_threshold(x, pairs, thres):
    """utils/vad.py:133-155"""
    out = []
    for bgn, fin in pairs:
        while bgn != -1:
            if x[bgn] < thres:
                break
            bgn -= 1
        while fin != len(x):
            if x[fin] < thres:
                break
            fin += 1
        out.append([bgn + 1, fin])
    return smooth(out, 1)


def remove_salt_noise(pairs, n_salt):
    """utils/vad.py:186-199"""
    return [[b, f] for b, f in pairs if not (f - b <= n_salt)]


def activity_detection(x, thres, low_thres=None, n_smooth=1, n_salt=0):
    """utils/vad.py:11-45"""
    locts = np.where(x > thres)[0]
    pairs = find_bgn_fin_pairs(locts)
    if low_thres is not None:
        pairs = second_threshold(x, pairs, low_thres)
    pairs = smooth(pairs, n_smooth)
    return remove_salt_noise(pairs, n_salt)


def binarize_pred(pred, thres):
    """pytorch/main_strong.py:870-883 (float64 0/1; per-class list or scalar
    threshold).  The element compare is made in float64 (an np.float32 element
    against a float64 threshold)."""
    C = pred.shape[2]
    t = np.asarray(list(thres) if isinstance(thres, (list, tuple, np.ndarray)) else [thres] * C,
                   np.float64)
    return (pred.astype(np.float64) > t[None, None, :]).astype(np.float64)


def activity_detection_binary(x, overlap_value, sample_duration, thres, low_thres=None,
                              n_smooth=1, n_salt=0):
    """utils/vad.py:47-106: locts from 100*overlap-frame blocks with at least
    num_overlaps votes (avg_merge schedule; the last block is never scanned);
    ``thres`` is unused, as in the reference."""
    ov = int(100 * overlap_value)
    interval = sample_duration * 100 - ov
    locts = []
    for i in range(0, x.shape[0] - ov, ov):
        if i < interval:
            nov = i // ov + 1
        elif i >= x.shape[0] - interval:
            nov = ((x.shape[0] - i) // ov) + 1
        else:
            nov = sample_duration
        locts.extend(int(j) + i for j in np.where(x[i:i + ov] >= nov)[0])
    pairs = find_bgn_fin_pairs(locts)
    if low_thres is not None:
        pairs = second_threshold(x, pairs, low_thres)
    pairs = smooth(pairs, n_smooth)
    return remove_salt_noise(pairs, n_salt)


def predict_windows_vote(sd, model_type, audio, sample_rate, sample_duration, overlap_value,
                         bin_thres, audio_duration=None):
    """inference_prob_vote window loop (pytorch/main_strong.py:1052-1100): the
    clip pad_truncate'd to 10 s, stride overlap_value, binarised windows
    merged with utilities.merge, no avg_merge."""
    if audio_duration is None:
        audio_duration = len(audio) / float(sample_rate)
    audio = pad_truncate_sequence(audio, sample_rate * 10)
    merged, prev = None, None
    for num_segment, start in enumerate(window_starts(audio_duration, sample_duration, overlap_value), start=1):
        s = int(start * sample_rate)
        seg = audio[s:int(sample_duration * sample_rate) + s]
        seg = torch.Tensor(np.asarray(seg))[None, :]
        curr = binarize_pred(forward(sd, model_type, wave=seg)['framewise_output'].numpy(), bin_thres)
        if num_segment == 1:
            merged = curr
        elif num_segment == 2:
            merged = merge(prev, curr, sample_duration, num_segment, overlap_value)
        else:
            merged = merge(merged, curr, sample_duration, num_segment, overlap_value)
        prev = curr
    return merged


def events_from_votes(votes, overlap_value, sample_duration, params, audio_name='test',
                      frames_per_second=FRAMES_PER_SECOND):
    """frame_binary_prediction_to_event_prediction (utils/utilities.py:216-276)."""
    N, T, C = votes.shape

    def as_list(v):
        return list(v) if isinstance(v, (list, tuple, np.ndarray)) else [v] * C

    lo = as_list(params['sed_low_threshold'])
    ns, nsalt = as_list(params['n_smooth']), as_list(params['n_salt'])
    ev = []
    for n in range(N):
        for k in range(C):
            for b, f in activity_detection_binary(votes[n, :, k], overlap_value, sample_duration, None,
                                                  lo[k], ns[k], nsalt[k]):
                ev.append({'filename': audio_name, 'onset': b / float(frames_per_second),
                           'offset': f / float(frames_per_second), 'event_label': LABELS[k]})
    return ev


def events_from_framewise(framewise, params, audio_name='test',
                          frames_per_second=FRAMES_PER_SECOND, sort=True):
    """frame_prediction_to_event_prediction_v2 (pytorch/predict.py:57-121 ==
    utils/utilities.py:155-214) + the onset sort of predict.py:353."""
    N, T, C = framewise.shape

    def as_list(v):
        return list(v) if isinstance(v, (list, tuple, np.ndarray)) else [v] * C

    hi, lo = as_list(params['sed_high_threshold']), as_list(params['sed_low_threshold'])
    ns, nsalt = as_list(params['n_smooth']), as_list(params['n_salt'])
    ev = []
    for n in range(N):
        for k in range(C):
            for b, f in activity_detection(framewise[n, :, k], hi[k], lo[k], ns[k], nsalt[k]):
                ev.append({'filename': audio_name, 'onset': b / float(frames_per_second),
                           'offset': f / float(frames_per_second), 'event_label': LABELS[k]})
    if sort:
        ev = sorted(ev, key=lambda e: e['onset'])
    return ev


# ---------------------------------------------------------------------------
# gammatone frontend (utils/gammatone/*, utils/features.py:361-370)
# ---------------------------------------------------------------------------
def _erb_space(low, high, num):
    """utils/gammatone/filters.py:18-72 (Glasberg & Moore constants)."""
    ear_q, min_bw = 9.26449, 24.7
    frac = np.arange(1, num + 1) / num
    return -ear_q * min_bw + np.exp(frac * (-np.log(high + ear_q * min_bw)
                                            + np.log(low + ear_q * min_bw))) * (high + ear_q * min_bw)


def gammatone_weights(fs, nfft, nfilts, fmin, fmax):
    """fft_weights (utils/gammatone/fftweight.py:63-123) with
    make_erb_filters (utils/gammatone/filters.py:90-193), width=1.
    Returns [nfilts, nfft//2+1] float64."""
    T = 1.0 / fs
    cf = _erb_space(fmin, fmax, nfilts)[::-1]
    ear_q, min_bw = 9.26449, 24.7
    erb = (cf / ear_q + min_bw)
    B = 1.019 * 2 * np.pi * erb
    arg = 2 * cf * np.pi * T
    vec = np.exp(2j * arg)
    rt_pos, rt_neg = np.sqrt(3 + 2 ** 1.5), np.sqrt(3 - 2 ** 1.5)
    common = -T * np.exp(-(B * T))
    k11 = np.cos(arg) + rt_pos * np.sin(arg)
    k12 = np.cos(arg) - rt_pos * np.sin(arg)
    k13 = np.cos(arg) + rt_neg * np.sin(arg)
    k14 = np.cos(arg) - rt_neg * np.sin(arg)
    A11, A12, A13, A14 = common * k11, common * k12, common * k13, common * k14
    gain_arg = np.exp(1j * arg - B * T)
    gain = np.abs((vec - gain_arg * k11) * (vec - gain_arg * k12) * (vec - gain_arg * k13)
                  * (vec - gain_arg * k14)
                  * (T * np.exp(B * T) / (-1 / np.exp(B * T) + 1 + vec * (1 - np.exp(B * T)))) ** 4)
    B2 = np.exp(-2 * B * T)
    ucirc = np.exp(1j * 2 * np.pi * np.arange(0, nfft / 2 + 1) / nfft)[None, :]
    r = np.sqrt(B2)
    theta = 2 * np.pi * cf / fs
    pole = (r * np.exp(1j * theta))[:, None]
    w = (np.abs(ucirc + A11[:, None] * fs) * np.abs(ucirc + A12[:, None] * fs)
         * np.abs(ucirc + A13[:, None] * fs) * np.abs(ucirc + A14[:, None] * fs)
         * np.abs(fs * (pole - ucirc) * (pole.conj() - ucirc)) ** (-4) / gain[:, None])
    return w


def gammatone_window(nfft, nwin):
    """specgram_window (utils/gammatone/fftweight.py:15-30)."""
    halflen = nwin // 2
    halff = nfft // 2
    act = int(np.floor(min(halff, halflen)))
    halfwin = 0.5 * (1 + np.cos(np.pi * np.arange(0, halflen + 1) / halflen))
    win = np.zeros((nfft,))
    win[halff:halff + act] = halfwin[0:act]
    win[halff:halff - act:-1] = halfwin[0:act]
    return win


def fft_gtgram(wave, fs, window_time, hop_time, channels, f_min):
    """fft_gtgram (utils/gammatone/fftweight.py:126-168) incl. specgram
    (:33-60): frames b in range(0, s - n, h), un-centred."""
    nfft = int(2 ** (np.ceil(np.log2(2 * window_time * fs))))
    nwin = int(np.sign(window_time * fs) * np.floor(abs(window_time * fs) + 0.5))
    nhop = int(np.sign(hop_time * fs) * np.floor(abs(hop_time * fs) + 0.5))
    w = gammatone_weights(fs, nfft, channels, f_min, fs / 2)
    win = gammatone_window(nfft, nwin)
    s = wave.shape[0]
    ncols = 1 + int(np.floor((s - nfft) / nhop))
    d = np.zeros((nfft // 2 + 1, ncols), dtype=complex)
    for c, b in enumerate(range(0, s - nfft, nhop)):
        d[:, c] = np.fft.fft(win * wave[b:b + nfft])[0:nfft // 2 + 1]
    return w.dot(np.abs(d)) / nfft


def power_to_db(S, ref=1.0, amin=1e-10, top_db=80.0):
    """librosa.power_to_db (utils/features.py:363; librosa-0.8 algorithm)."""
    log_spec = 10.0 * np.log10(np.maximum(amin, S)) - 10.0 * np.log10(np.maximum(amin, ref))
    if top_db is not None:
        log_spec = np.maximum(log_spec, log_spec.max() - top_db)
    return log_spec


def float32_to_int16(x):
    """utils/utilities.py:73-76"""
    x = np.array(x, copy=True)
    if np.max(np.abs(x)) > 1.:
        x /= np.max(np.abs(x))
    return (x * 32767.).astype(np.int16)


def int16_to_float32(x):
    """utils/utilities.py:78-79"""
    return (x / 32767.).astype(np.float32)


def gamma_features(audio, preset='32k'):
    """HDF5 pack branch (utils/features.py:356-370) + loader
    (utils/data_generator.py:37): audio [L] -> model input [64, T] float32."""
    p = PRESETS[preset]
    sr = p['sample_rate']
    audio = pad_truncate_sequence(np.asarray(audio), sr * 10)
    g = fft_gtgram(audio, sr, p['window_size'] / sr, p['hop_size'] / sr, p['mel_bins'], p['fmin'])
    return int16_to_float32(float32_to_int16(power_to_db(g)))
