"""CPU restatement of ``librosa.core.load(path, sr, mono=True)`` (librosa 0.8,
as pytorch/predict.py:295 and pytorch/main_strong.py:787 call it).

TEST INFRASTRUCTURE ONLY: imported by tests/ as the checker of
sedx.audio.load / sedx_resample, never by the product path.

Third-party pieces (none of them is in /root/reference or installed here):
  * soundfile / libsndfile float32 reading: restated (int16 * 2^-15,
    int24 * 2^-23, float32(int32) * 2^-31, (u8 - 128) * 2^-7, float as is);
  * librosa 0.8 ``to_mono`` (np.mean over axis 0 of the float32 [C, N] array),
    ``resample`` (resampy for 'kaiser_best' / 'kaiser_fast', then
    ``util.fix_length`` to ceil(n * ratio)) - librosa/core/audio.py;
  * resampy 0.2 ``filters.sinc_window`` (Kaiser-tapered sinc: kaiser_best =
    64 zero crossings, 2^9 taps per crossing, rolloff 0.9475937167399596,
    beta 14.769656459379492; kaiser_fast = 16, 2^9, 0.85, 8.555504641634386)
    and ``interp.resample_f`` (two-wing band-limited interpolation, float64
    weights, float32 output accumulated in place).
Parity of the resampler is therefore UNPINNED by any reference output: the
tests check the HIP path against this restatement and the restatement
against band-limited reconstruction of known signals.
"""
import struct

import numpy as np

FILTERS = {'kaiser_best': (64, 9, 0.9475937167399596, 14.769656459379492),
           'kaiser_fast': (16, 9, 0.85, 8.555504641634386)}


def parse_wav(raw):
    """RIFF/WAVE image -> (fmt_tag, channels, sr, bits, data bytes)."""
    raw = bytes(raw)
    assert raw[:4] == b'RIFF' and raw[8:12] == b'WAVE'
    o, fmt, data = 12, None, None
    while o + 8 <= len(raw):
        cid, sz = raw[o:o + 4], struct.unpack('<I', raw[o + 4:o + 8])[0]
        body = raw[o + 8:o + 8 + sz]
        if cid == b'fmt ':
            tag, ch, sr, _, _, bits = struct.unpack('<HHIIHH', body[:16])
            if tag == 0xFFFE:
                tag = struct.unpack('<H', body[24:26])[0]
            fmt = (tag, ch, sr, bits)
        elif cid == b'data':
            data = body
            break
        o += 8 + sz + (sz & 1)
    return fmt + (data,)


def decode(raw):
    """soundfile.read(dtype='float32', always_2d) equivalent -> [C, N] float32, sr."""
    tag, ch, sr, bits, data = parse_wav(raw)
    if tag == 1 and bits == 8:
        x = (np.frombuffer(data, np.uint8).astype(np.int32) - 128).astype(np.float32) * np.float32(2 ** -7)
    elif tag == 1 and bits == 16:
        x = np.frombuffer(data, '<i2').astype(np.float32) * np.float32(2 ** -15)
    elif tag == 1 and bits == 24:
        b = np.frombuffer(data, np.uint8).reshape(-1, 3).astype(np.uint32)
        i = ((b[:, 0] << 8) | (b[:, 1] << 16) | (b[:, 2] << 24)).view(np.int32)
        x = i.astype(np.float32) * np.float32(2 ** -31)
    elif tag == 1 and bits == 32:
        x = np.frombuffer(data, '<i4').astype(np.float32) * np.float32(2 ** -31)
    elif tag == 3 and bits == 32:
        x = np.frombuffer(data, '<f4').astype(np.float32)
    elif tag == 3 and bits == 64:
        x = np.frombuffer(data, '<f8').astype(np.float32)
    else:
        raise ValueError('unsupported WAV format %d/%d' % (tag, bits))
    n = x.size // ch
    return x[:n * ch].reshape(n, ch).T, sr


def to_mono(y):
    """librosa.to_mono: np.mean(y, axis=0) of the float32 [C, N] array."""
    return np.mean(y, axis=0) if y.shape[0] > 1 else y[0]


def sinc_window(num_zeros, precision, rolloff, beta):
    """resampy.filters.sinc_window with window = np.kaiser(., beta)."""
    num_bits = 2 ** precision
    n = num_bits * num_zeros
    sinc_win = rolloff * np.sinc(rolloff * np.linspace(0, num_zeros, num=n + 1, endpoint=True))
    taper = np.kaiser(2 * n + 1, beta)[n:]
    return taper * sinc_win, num_bits


def resample(x, sr_orig, sr_new, res_type='kaiser_best'):
    """librosa.resample (0.8): resampy.resample then fix_length(ceil(n * ratio)).
    resample_f vectorised over output samples; per output the taps are added
    in resample_f's order (left wing i = 0.., then right wing k = 0..), each
    as float64 weight * sample added to the float32 accumulator."""
    x = np.asarray(x, np.float32)
    if sr_orig == sr_new:
        return x
    ratio = float(sr_new) / sr_orig
    n_fix = int(np.ceil(x.shape[-1] * ratio))
    win, num_table = sinc_window(*FILTERS[res_type])
    if ratio < 1:
        win = win * ratio
    delta = np.zeros_like(win)
    delta[:-1] = np.diff(win)
    n_res = int(x.shape[-1] * ratio)
    scale = min(1.0, ratio)
    inc = 1.0 / ratio
    index_step = int(scale * num_table)
    nwin = win.shape[0]
    treg = np.empty(n_res)
    tr = 0.0
    for t in range(n_res):          # resample_f's running float64 time register
        treg[t] = tr
        tr += inc
    n = treg.astype(np.int64)
    y = np.zeros(n_res, np.float32)
    xd = x.astype(np.float64)
    # left wing
    frac = scale * (treg - n)
    index_frac = frac * num_table
    offset = index_frac.astype(np.int64)
    eta = index_frac - offset
    i_max = np.minimum(n + 1, (nwin - offset) // index_step)
    for i in range(int(i_max.max()) if n_res else 0):
        m = i < i_max
        o = offset[m] + i * index_step
        w = win[o] + eta[m] * delta[o]
        y[m] = (y[m].astype(np.float64) + w * xd[n[m] - i]).astype(np.float32)
    # right wing
    frac = scale - frac
    index_frac = frac * num_table
    offset = index_frac.astype(np.int64)
    eta = index_frac - offset
    k_max = np.minimum(x.shape[-1] - n - 1, (nwin - offset) // index_step)
    for k in range(int(k_max.max()) if n_res else 0):
        m = k < k_max
        o = offset[m] + k * index_step
        w = win[o] + eta[m] * delta[o]
        y[m] = (y[m].astype(np.float64) + w * xd[n[m] + k + 1]).astype(np.float32)
    out = np.zeros(n_fix, np.float32)
    out[:min(n_fix, n_res)] = y[:n_fix]
    return out


def load(raw, sr=22050, res_type='kaiser_best'):
    """librosa.core.load(path, sr=sr, mono=True) on a WAV file image."""
    y, sr_native = decode(raw)
    y = to_mono(y)
    if sr is None or sr == sr_native:
        return y, sr_native
    return resample(y, sr_native, sr, res_type), sr


def write_wav(samples, sr, bits=16, fmt='pcm', extensible=False):
    """Test helper: a WAV file image from float samples [C, N] in [-1, 1)."""
    s = np.atleast_2d(np.asarray(samples, np.float64))
    ch, n = s.shape
    il = s.T.reshape(-1)
    if fmt == 'pcm' and bits == 8:
        data = np.clip(np.round(il * 128 + 128), 0, 255).astype(np.uint8).tobytes()
    elif fmt == 'pcm' and bits == 16:
        data = np.clip(np.round(il * 32768), -32768, 32767).astype('<i2').tobytes()
    elif fmt == 'pcm' and bits == 24:
        v = np.clip(np.round(il * 2 ** 23), -2 ** 23, 2 ** 23 - 1).astype(np.int32)
        b = v.view(np.uint32)
        data = np.stack([b & 0xFF, (b >> 8) & 0xFF, (b >> 16) & 0xFF], 1).astype(np.uint8).tobytes()
    elif fmt == 'pcm' and bits == 32:
        data = np.clip(np.round(il * 2 ** 31), -2 ** 31, 2 ** 31 - 1).astype('<i4').tobytes()
    elif fmt == 'float' and bits == 32:
        data = il.astype('<f4').tobytes()
    elif fmt == 'float' and bits == 64:
        data = il.astype('<f8').tobytes()
    else:
        raise ValueError(fmt, bits)
    tag = 1 if fmt == 'pcm' else 3
    ba = ch * bits // 8
    if extensible:
        guid = struct.pack('<H', tag) + b'\x00\x00\x00\x00\x10\x00\x80\x00\x00\xaa\x00\x38\x9b\x71'
        fmt_chunk = struct.pack('<HHIIHHHHI', 0xFFFE, ch, sr, sr * ba, ba, bits, 22, bits, 0) + guid
    else:
        fmt_chunk = struct.pack('<HHIIHH', tag, ch, sr, sr * ba, ba, bits)
    body = b'WAVE' + b'fmt ' + struct.pack('<I', len(fmt_chunk)) + fmt_chunk
    body += b'LIST' + struct.pack('<I', 3) + b'abc\x00'          # odd-sized chunk (word padding)
    body += b'data' + struct.pack('<I', len(data)) + data
    return b'RIFF' + struct.pack('<I', len(body)) + body
