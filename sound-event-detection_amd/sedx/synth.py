"""Seeded synthetic weights and waveforms for parity tests and the bench.

Pretrained checkpoints are absent from the reference (``.MISSING_LARGE_BLOBS``),
so every parity run uses random-init weights of the reference architecture.
The generator is plain numpy ``default_rng`` (bit-identical on every host), so
the golden fixtures under ``tests/golden/`` never need to store the 24.7 MB
state_dict: tests regenerate it from the seed.

Keys/shapes follow the reference state_dict (SURVEY.md Appendix A;
``pytorch/models.py:564-624`` GRU model, ``:981-1027`` Transformer model).
Only the learnable tensors and BN statistics are produced here; the frontend
buffers (``spectrogram_extractor.stft.conv_{real,imag}.weight``,
``logmel_extractor.melW``) come from the model constructors.
"""
import numpy as np

CONV_CHANNELS = [(1, 64), (64, 128), (128, 256), (256, 512)]


def _xavier_uniform(rng, shape, fan_in, fan_out, gain=1.0):
    a = gain * np.sqrt(6.0 / (fan_in + fan_out))
    return rng.uniform(-a, a, size=shape).astype(np.float32)


def _bn(rng, prefix, n, mean_range=(-1.0, 1.0), var_range=(0.5, 2.0)):
    return {
        prefix + '.weight': rng.uniform(0.5, 1.5, n).astype(np.float32),
        prefix + '.bias': rng.uniform(-0.2, 0.2, n).astype(np.float32),
        prefix + '.running_mean': rng.uniform(*mean_range, n).astype(np.float32),
        prefix + '.running_var': rng.uniform(*var_range, n).astype(np.float32),
        prefix + '.num_batches_tracked': np.array(1000, dtype=np.int64),
    }


def make_state_dict(model_type, classes_num=25, seed=0):
    """Return {key: np.ndarray} for the non-frontend parameters of
    ``Cnn_9layers_Gru_FrameAtt`` or ``Cnn_9layers_Transformer_FrameAtt``."""
    if model_type not in ('Cnn_9layers_Gru_FrameAtt', 'Cnn_9layers_Transformer_FrameAtt'):
        raise ValueError('unknown model_type %r' % model_type)
    rng = np.random.default_rng(seed)
    sd = {}
    # bn0 normalises log-mel dB values (models.py:607,642-644); realistic stats
    sd.update(_bn(rng, 'bn0', 64, mean_range=(-45.0, -35.0), var_range=(300.0, 500.0)))
    for k, (cin, cout) in enumerate(CONV_CHANNELS, start=1):
        p = 'conv_block%d' % k
        sd[p + '.conv1.weight'] = _xavier_uniform(rng, (cout, cin, 3, 3), cin * 9, cout * 9)
        sd[p + '.conv2.weight'] = _xavier_uniform(rng, (cout, cout, 3, 3), cout * 9, cout * 9)
        sd.update(_bn(rng, p + '.bn1', cout))
        sd.update(_bn(rng, p + '.bn2', cout))
    if model_type == 'Cnn_9layers_Gru_FrameAtt':
        # init_gru (models.py:35-60): U(+-sqrt(3/fan_in)) per gate block; small
        # random biases so the bias paths are exercised.
        for sfx in ('', '_reverse'):
            b_ih = np.sqrt(3.0 / 512)
            b_hh = np.sqrt(3.0 / 256)
            sd['gru.weight_ih_l0' + sfx] = rng.uniform(-b_ih, b_ih, (768, 512)).astype(np.float32)
            sd['gru.weight_hh_l0' + sfx] = rng.uniform(-b_hh, b_hh, (768, 256)).astype(np.float32)
            sd['gru.bias_ih_l0' + sfx] = rng.uniform(-0.1, 0.1, 768).astype(np.float32)
            sd['gru.bias_hh_l0' + sfx] = rng.uniform(-0.1, 0.1, 768).astype(np.float32)
    else:
        # MultiHead init (models.py:835-852): normal(0, sqrt(2/(d_model+d_k)))
        std_qkv = np.sqrt(2.0 / (512 + 64))
        for nm in ('w_qs', 'w_ks', 'w_vs'):
            sd['multihead.%s.weight' % nm] = rng.normal(0, std_qkv, (512, 512)).astype(np.float32)
            sd['multihead.%s.bias' % nm] = rng.uniform(-0.05, 0.05, 512).astype(np.float32)
        sd['multihead.layer_norm.weight'] = np.ones(512, np.float32)
        sd['multihead.layer_norm.bias'] = np.zeros(512, np.float32)
        std_fc = np.sqrt(2.0 / (512 + 512))
        sd['multihead.fc.weight'] = rng.normal(0, std_fc, (512, 512)).astype(np.float32)
        sd['multihead.fc.bias'] = rng.uniform(-0.05, 0.05, 512).astype(np.float32)
    sd['att_block.att.weight'] = _xavier_uniform(rng, (classes_num, 512, 1), 512, classes_num)
    sd['att_block.att.bias'] = rng.uniform(-0.1, 0.1, classes_num).astype(np.float32)
    sd['att_block.cla.weight'] = _xavier_uniform(rng, (classes_num, 512, 1), 512, classes_num)
    sd['att_block.cla.bias'] = rng.uniform(-0.5, 0.0, classes_num).astype(np.float32)
    sd.update(_bn(rng, 'att_block.bn_att', classes_num))
    return sd


def make_waveforms(batch, seconds=10.0, sample_rate=16000, seed=1234):
    """[batch, L] float32: 0.1*N(0,1) noise + gated tones (440/1000/3000 Hz,
    1 s on/off envelopes with a per-clip phase) so that events occur
    (SURVEY.md §8(d) "Synthetic inputs")."""
    rng = np.random.default_rng(seed)
    L = int(round(seconds * sample_rate))
    t = np.arange(L, dtype=np.float64) / sample_rate
    out = np.empty((batch, L), dtype=np.float32)
    for b in range(batch):
        x = 0.1 * rng.standard_normal(L)
        for j, f in enumerate((440.0, 1000.0, 3000.0)):
            period = 2.0 + j
            shift = rng.uniform(0, period)
            gate = (np.floor((t + shift) / (period / 2.0)) % 2 == 0).astype(np.float64)
            amp = rng.uniform(0.2, 0.6)
            x += amp * gate * np.sin(2 * np.pi * f * t + rng.uniform(0, 2 * np.pi))
        out[b] = x.astype(np.float32)
    return out
