"""Drop-in model classes for the reference's hot path (pytorch/models.py).

``Cnn_9layers_Gru_FrameAtt`` and ``Cnn_9layers_Transformer_FrameAtt`` keep the
reference constructor ``(sample_rate, window_size, hop_size, mel_bins, fmin,
fmax, classes_num, feature_type)``, ``forward(input, mixup_lambda=None,
timeshift=False, spec_augment=True)`` and the exact state_dict keys/shapes
(so ``model.load_state_dict(torch.load(path)['model'])`` works unchanged).
The submodules are parameter containers; the whole eval-mode forward runs in
libsedx (HIP kernels for gfx950) through the C ABI in include/sedx.h.  There
is no CPU or eager-PyTorch fallback: a non-HIP input raises.

Usage mirrors the reference call sites (pytorch/predict.py:229-242, 311-313):

    Model = getattr(sedx.models, model_type)
    model = Model(16000, 512, 160, 64, 25, 7000, 25, 'logmel')
    model.load_state_dict(checkpoint['model'])
    model.to('cuda').eval()
    with torch.no_grad():
        out = model(waveform_on_gpu)      # {'framewise_output', 'clipwise_output', 'embedding'}
"""
import ctypes
import math
import threading
import weakref

import numpy as np
import torch
import torch.nn as nn

from . import _lib
from .stft import Spectrogram, LogmelFilterBank

__all__ = ['Cnn_9layers_Gru_FrameAtt', 'Cnn_9layers_Transformer_FrameAtt', 'ConvBlock',
           'AttBlock', 'MultiHead', 'interpolate', 'pad_framewise_output', 'roundup',
           'init_layer', 'init_bn', 'init_gru']

MODEL_IDS = {'Cnn_9layers_Gru_FrameAtt': 0, 'Cnn_9layers_Transformer_FrameAtt': 1}
FEATURE_IDS = {'logmel': 0, 'gamma': 1}


# ---------------------------------------------------------------------------
# reference helpers (pytorch/models.py:20-95)
# ---------------------------------------------------------------------------
def init_layer(layer):
    """models.py:20-26"""
    nn.init.xavier_uniform_(layer.weight)
    if getattr(layer, 'bias', None) is not None:
        layer.bias.data.fill_(0.)


def init_bn(bn):
    """models.py:29-32"""
    bn.bias.data.fill_(0.)
    bn.weight.data.fill_(1.)


def init_gru(rnn):
    """models.py:35-60: U(+-sqrt(3/fan_in)) per gate block, orthogonal n-gate
    recurrent block, zero biases -- of the forward-direction tensors only
    (``weight_ih_l{i}`` etc.); the ``_reverse`` tensors keep nn.GRU's own
    initialisation, as in the reference."""
    def _concat_init(tensor, init_funcs):
        length, fan_out = tensor.shape
        fan_in = length // len(init_funcs)
        for i, fn in enumerate(init_funcs):
            fn(tensor[i * fan_in:(i + 1) * fan_in, :])

    def _inner_uniform(tensor):
        fan_in = nn.init._calculate_correct_fan(tensor, 'fan_in')
        nn.init.uniform_(tensor, -math.sqrt(3 / fan_in), math.sqrt(3 / fan_in))

    for i in range(rnn.num_layers):
        _concat_init(getattr(rnn, 'weight_ih_l%d' % i), [_inner_uniform] * 3)
        nn.init.constant_(getattr(rnn, 'bias_ih_l%d' % i), 0)
        _concat_init(getattr(rnn, 'weight_hh_l%d' % i),
                     [_inner_uniform, _inner_uniform, nn.init.orthogonal_])
        nn.init.constant_(getattr(rnn, 'bias_hh_l%d' % i), 0)


def roundup(x):
    """models.py:62-63"""
    return x if x % 100 == 0 else x + 100 - x % 100


def pad_framewise_output(framewise_output, frames_num):
    """models.py:65-81 (tensor helper; the model forward does this natively)."""
    pad = framewise_output[:, -1:, :].repeat(1, frames_num - framewise_output.shape[1], 1)
    return torch.cat((framewise_output, pad), dim=1)


def interpolate(x, ratio):
    """models.py:84-95 (tensor helper; the model forward does this natively)."""
    b, t, c = x.shape
    return x[:, :, None, :].repeat(1, 1, ratio, 1).reshape(b, t * ratio, c)


# ---------------------------------------------------------------------------
# parameter containers with the reference module names
# ---------------------------------------------------------------------------
class ConvBlock(nn.Module):
    """models.py:98-141 (weights only; conv+BN+ReLU+pool run in libsedx)."""

    def __init__(self, in_channels, out_channels):
        super().__init__()
        self.conv1 = nn.Conv2d(in_channels, out_channels, (3, 3), (1, 1), (1, 1), bias=False)
        self.conv2 = nn.Conv2d(out_channels, out_channels, (3, 3), (1, 1), (1, 1), bias=False)
        self.bn1 = nn.BatchNorm2d(out_channels)
        self.bn2 = nn.BatchNorm2d(out_channels)
        init_layer(self.conv1)
        init_layer(self.conv2)
        init_bn(self.bn1)
        init_bn(self.bn2)

    def forward(self, input, pool_size=(2, 2), pool_type='avg'):
        raise RuntimeError('ConvBlock is fused into the native model forward (libsedx)')


class AttBlock(nn.Module):
    """models.py:144-175 (weights only)."""

    def __init__(self, n_in, n_out, activation='linear', temperature=1.):
        super().__init__()
        self.activation = activation
        self.temperature = temperature
        self.att = nn.Conv1d(n_in, n_out, kernel_size=1, stride=1, padding=0, bias=True)
        self.cla = nn.Conv1d(n_in, n_out, kernel_size=1, stride=1, padding=0, bias=True)
        self.bn_att = nn.BatchNorm1d(n_out)
        init_layer(self.att)
        init_layer(self.cla)
        init_bn(self.bn_att)

    def forward(self, x):
        raise RuntimeError('AttBlock is fused into the native model forward (libsedx)')


class MultiHead(nn.Module):
    """models.py:823-877 (weights only)."""

    def __init__(self, n_head, d_model, d_k, d_v, dropout=0.1):
        super().__init__()
        if (n_head, d_model, d_k, d_v) != (8, 512, 64, 64):
            raise ValueError('the native MHA implements the reference shape (8 heads, 512, 64, 64)')
        self.n_head, self.d_k, self.d_v = n_head, d_k, d_v
        self.w_qs = nn.Linear(d_model, n_head * d_k)
        self.w_ks = nn.Linear(d_model, n_head * d_k)
        self.w_vs = nn.Linear(d_model, n_head * d_v)
        nn.init.normal_(self.w_qs.weight, mean=0, std=np.sqrt(2.0 / (d_model + d_k)))
        nn.init.normal_(self.w_ks.weight, mean=0, std=np.sqrt(2.0 / (d_model + d_k)))
        nn.init.normal_(self.w_vs.weight, mean=0, std=np.sqrt(2.0 / (d_model + d_v)))
        for m in (self.w_qs, self.w_ks, self.w_vs):
            m.bias.data.fill_(0)
        self.layer_norm = nn.LayerNorm(d_model)
        self.fc = nn.Linear(n_head * d_v, d_model)
        nn.init.xavier_normal_(self.fc.weight)
        self.fc.bias.data.fill_(0)

    def forward(self, q, k, v, mask=None):
        raise RuntimeError('MultiHead is fused into the native model forward (libsedx)')


# ---------------------------------------------------------------------------
# native handle management
# ---------------------------------------------------------------------------
class _Native(object):
    def __init__(self, cfg, device_index):
        L = _lib.lib()
        h = ctypes.c_void_p()
        _lib.check(L.sedx_create(ctypes.byref(cfg), device_index, ctypes.byref(h)), None,
                   'sedx_create(model=%d, feature=%d)' % (cfg.model_type, cfg.feature_type))
        self.h = h
        self.device_index = device_index
        self.signature = None
        self.precision = 'winograd'   # the library default (sedx_set_precision)

    def load(self, state_dict):
        L = _lib.lib()
        for k, v in state_dict.items():
            if k.endswith('num_batches_tracked'):
                continue
            a = np.ascontiguousarray(v.detach().to('cpu', torch.float32).numpy())
            shape = (ctypes.c_int64 * a.ndim)(*a.shape)
            _lib.check(L.sedx_load_param(self.h, k.encode(), a.ctypes.data_as(ctypes.c_void_p),
                                         shape, a.ndim), self.h, 'load_param(%s)' % k)
        _lib.check(L.sedx_finalize_weights(self.h), self.h, 'finalize_weights')

    def __del__(self):
        try:
            if self.h:
                _lib.lib().sedx_destroy(self.h)
        except Exception:
            pass


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


# generation of the module tree anywhere in the process: bumped whenever a
# parameter, buffer or submodule is registered (setattr of an nn.Parameter /
# register_buffer / add_module), so _SedModel._signature re-walks its
# state_dict only after such a change
_REG_GEN = [0]


def _bump_reg_gen(*_args):
    _REG_GEN[0] += 1


torch.nn.modules.module.register_module_parameter_registration_hook(_bump_reg_gen)
torch.nn.modules.module.register_module_buffer_registration_hook(_bump_reg_gen)
torch.nn.modules.module.register_module_module_registration_hook(_bump_reg_gen)


class _HandleCache(dict):
    """device index -> _Native, shared by a model and its DataParallel
    replicas.  ``torch.nn.DataParallel`` (pytorch/predict.py:239,
    pytorch/main_strong.py:541) re-replicates the module on every forward
    (``Module._replicate_for_data_parallel``: a shallow ``__dict__`` copy, so
    this object is shared) and hands each replica parameters freshly broadcast
    to its device, i.e. new ``data_ptr``s every call.  The replicas' weights
    are copies of the source module's, so a replica's handle is keyed on the
    SOURCE module's parameters (``source``) and the per-device handle is
    packed once, not once per call.  ``lock`` serialises handle creation and
    packing across DataParallel's per-device threads.  Copies and pickles of
    a model start with an empty cache (a handle owns device memory)."""

    def __init__(self, owner=None):
        super().__init__()
        self.lock = threading.Lock()
        self.source = weakref.ref(owner) if owner is not None else None

    def __reduce__(self):
        return (_HandleCache, ())


class _SedModel(nn.Module):
    """Shared construction + native forward for the two hot-path models."""

    _model_name = None

    def __init__(self, sample_rate, window_size, hop_size, mel_bins, fmin, fmax, classes_num,
                 feature_type='logmel'):
        super().__init__()
        if mel_bins != 64:
            raise ValueError('mel_bins must be 64 (bn0 = BatchNorm2d(64), models.py:607)')
        self.feature_type = feature_type
        self.sample_rate, self.window_size, self.hop_size = sample_rate, window_size, hop_size
        self.mel_bins, self.fmin, self.fmax, self.classes_num = mel_bins, fmin, fmax, classes_num
        self.spectrogram_extractor = Spectrogram(n_fft=window_size, hop_length=hop_size,
                                                 win_length=window_size, window='hann',
                                                 center=True, pad_mode='reflect',
                                                 freeze_parameters=True)
        self.logmel_extractor = LogmelFilterBank(sr=sample_rate, n_fft=window_size,
                                                 n_mels=mel_bins, fmin=fmin, fmax=fmax, ref=1.0,
                                                 amin=1e-10, top_db=None, freeze_parameters=True)
        self.bn0 = nn.BatchNorm2d(64)
        self.conv_block1 = ConvBlock(1, 64)
        self.conv_block2 = ConvBlock(64, 128)
        self.conv_block3 = ConvBlock(128, 256)
        self.conv_block4 = ConvBlock(256, 512)
        self._natives = _HandleCache(self)
        self.precision = 'winograd'
        self.pipelined = False
        self.tuning = {}           # sedx_set_tuning knob -> value, applied to every handle

    def _config(self):
        cfg = _lib.SedxConfig()
        cfg.model_type = MODEL_IDS[self._model_name]
        if self.feature_type not in FEATURE_IDS:
            raise ValueError('feature_type %r not supported (logmel | gamma)' % self.feature_type)
        cfg.feature_type = FEATURE_IDS[self.feature_type]
        cfg.sample_rate = int(self.sample_rate)
        cfg.window_size = int(self.window_size)
        cfg.hop_size = int(self.hop_size)
        cfg.mel_bins = int(self.mel_bins)
        cfg.fmin = float(self.fmin)
        cfg.fmax = float(self.fmax if self.fmax is not None else self.sample_rate // 2)
        cfg.classes_num = int(self.classes_num)
        return cfg

    def _signature(self):
        """What the packed weights of a handle were made from: every
        state_dict tensor's key, shape, storage and version counter (an
        in-place update — load_state_dict, optimizer-free edits — bumps the
        version).  The state_dict walk (~75 tensors, ~0.1-0.2 ms of Python per
        call) runs again only when a parameter, buffer or submodule was
        registered anywhere since (torch's global registration hooks bump
        _REG_GEN); otherwise the cached tensor list is re-read for storage and
        version only, so a one-clip forward does not wait on it."""
        # (keyed on the object too: a DataParallel replica is a shallow
        # __dict__ copy whose parameter dicts are replaced without
        # registration, so it must not reuse its source's cache)
        c = self.__dict__.get('_sig_cache')
        if c is None or c[0] != _REG_GEN[0] or c[1] != id(self):
            sd = self.state_dict(keep_vars=True)
            c = (_REG_GEN[0], id(self), tuple(sd.keys()), tuple(sd.values()),
                 tuple(tuple(v.shape) for v in sd.values()))
            self.__dict__['_sig_cache'] = c
        _, _, keys, tensors, shapes = c
        return keys, shapes, tuple([(t.data_ptr(), t._version) for t in tensors])

    def _weights_source(self):
        """The module whose parameters a handle is packed from: the source
        module for a DataParallel replica (its own parameters are broadcast
        copies of the source's, re-made every call), else the module itself."""
        if getattr(self, '_is_replica', False):
            ref = getattr(self._natives, 'source', None)
            src = ref() if ref is not None else None
            if src is not None:
                return src
        return self

    def native(self, device):
        """The libsedx handle for ``device`` with the current weights packed."""
        if device.type != 'cuda':
            raise RuntimeError('sedx runs on HIP devices only (got a %s tensor); there is no CPU '
                               'fallback' % device.type)
        idx = device.index if device.index is not None else torch.cuda.current_device()
        with self._natives.lock:
            return self._native_locked(idx)

    def _native_locked(self, idx):
        nat = self._natives.get(idx)
        if nat is None:
            nat = _Native(self._config(), idx)
            self._natives[idx] = nat
        src = self._weights_source()
        sig = src._signature()
        if nat.signature != sig:
            nat.load(src.state_dict())
            nat.signature = sig
        if nat.precision != self.precision:
            _lib.check(_lib.lib().sedx_set_precision(nat.h, _lib.PRECISION[self.precision]), nat.h,
                       'set_precision')
            nat.precision = self.precision
        for knob, value in self.tuning.items():
            if getattr(nat, 'tuning', {}).get(knob) != value:
                _lib.check(_lib.lib().sedx_set_tuning(nat.h, knob, value), nat.h, 'set_tuning')
                nat.tuning = dict(getattr(nat, 'tuning', {}))
                nat.tuning[knob] = value
        if getattr(nat, 'pipelined', False) != self.pipelined:
            _lib.check(_lib.lib().sedx_set_pipelined(nat.h, int(self.pipelined)), nat.h, 'set_pipelined')
            nat.pipelined = self.pipelined
        return nat

    def set_precision(self, mode):
        """GEMM arithmetic (conv stack, GRU / MHA projections and recurrence,
        AttBlock projection): 'winograd' (default; fp32 operands, transforms
        and accumulation, block 1's conv2 and blocks 2-4 as Winograd
        F(4x4,3x3) — _lib.TUNE_WINO_F43 0 / 1 select F(2x2,3x3) in every layer
        / in block 1 only; error vs float64 max <= 2.5e-5, rms <= 1.7e-6 per
        layer), 'exact'
        (fp32 direct convolution, the reference's operation order) or 'x3'
        (opt-in; 3xbf16-split MFMA, fp32 accumulate, ~1e-6 from fp32)."""
        if mode not in _lib.PRECISION:
            raise ValueError('precision must be one of %s' % sorted(_lib.PRECISION))
        self.precision = mode
        return self

    def set_tuning(self, knob, value):
        """An implementation choice of the library (sedx_set_tuning: _lib.TUNE_*)."""
        self.tuning[int(knob)] = int(value)
        return self

    def set_pipelined(self, on=True):
        """Several batches in flight on different streams: run the conv
        stacks in issue order so one batch's GRU / MHA + head overlap the next
        batch's conv stack (sedx_set_pipelined).  on = 2: also issue block 1's
        conv1 ahead of that wait."""
        self.pipelined = int(on) if on in (0, 1, 2) else bool(on)
        return self

    def check_error(self):
        """Raise if an earlier forward failed asynchronously (a GRU hand-off
        spin ran out: its outputs are NaN; sedx_check_error).  Call once the
        outputs in question are complete (after a sync or a copy to the
        host); the drivers in sedx.inference call it after every batch they
        copy back."""
        L = _lib.lib()
        for nat in list(self._natives.values()):
            _lib.check(L.sedx_check_error(nat.h), nat.h, 'asynchronous GRU failure')

    def _check_eval(self, mixup_lambda, timeshift):
        if self.training:
            raise RuntimeError('sedx models are inference-only: call model.eval() first '
                               '(training-mode SpecAugment/mixup/timeshift are out of scope)')
        if mixup_lambda is not None or timeshift:
            pass  # ignored in eval, as in the reference (models.py:647-661)

    def output_geometry(self, length):
        L = _lib.lib()
        with self._natives.lock:
            nat = self._natives.get(next(iter(self._natives))) if self._natives else None
            if nat is None:
                nat = _Native(self._config(), torch.cuda.current_device() if torch.cuda.is_available() else 0)
                self._natives[nat.device_index] = nat
        fr, sl = ctypes.c_int64(), ctypes.c_int64()
        _lib.check(L.sedx_output_geometry(nat.h, int(length), ctypes.byref(fr), ctypes.byref(sl)),
                   nat.h, 'output_geometry')
        return fr.value, sl.value

    def forward(self, input, mixup_lambda=None, timeshift=False, spec_augment=True):
        """Input: (batch_size, data_length) waveform [logmel] or
        (batch_size, 64, frames) features [gamma].  Eval mode only.  An int16
        waveform (the reference's HDF5 packing) is dequantised x / 32767 inside
        the frontend (int16_to_float32, utils/utilities.py:78-79)."""
        self._check_eval(mixup_lambda, timeshift)
        if not isinstance(input, torch.Tensor) or input.device.type != 'cuda':
            raise RuntimeError('sedx forward needs a tensor on a HIP device (no CPU fallback)')
        i16 = input.dtype == torch.int16 and self.feature_type != 'gamma'
        x = input.contiguous() if i16 else input.to(torch.float32).contiguous()
        nat = self.native(x.device)
        L = _lib.lib()
        if self.feature_type == 'gamma':
            if x.dim() != 3 or x.shape[1] != 64:
                raise ValueError('gamma input must be (batch, 64, frames)')
            B, length = x.shape[0], x.shape[2]
        else:
            if x.dim() != 2:
                raise ValueError('input must be (batch_size, data_length)')
            B, length = x.shape
        fr, sl = ctypes.c_int64(), ctypes.c_int64()
        _lib.check(L.sedx_output_geometry(nat.h, length, ctypes.byref(fr), ctypes.byref(sl)),
                   nat.h, 'output_geometry')
        C = self.classes_num
        dev = x.device
        fw = torch.empty((B, fr.value, C), dtype=torch.float32, device=dev)
        clip = torch.empty((B, C), dtype=torch.float32, device=dev)
        emb_shape = (B, C, sl.value) if self._model_name == 'Cnn_9layers_Gru_FrameAtt' else (B, 512, sl.value)
        emb = torch.empty(emb_shape, dtype=torch.float32, device=dev)
        wsz = ctypes.c_size_t()
        _lib.check(L.sedx_workspace_size(nat.h, B, length, ctypes.byref(wsz)), nat.h, 'workspace_size')
        ws = torch.empty(wsz.value, dtype=torch.uint8, device=dev)
        stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        fn = L.sedx_forward_features if self.feature_type == 'gamma' else (
            L.sedx_forward_i16 if i16 else L.sedx_forward)
        _lib.check(fn(nat.h, _ptr(x), B, length, _ptr(fw), _ptr(clip), _ptr(emb), _ptr(ws),
                      wsz.value, stream), nat.h, 'forward')
        return {'framewise_output': fw, 'clipwise_output': clip, 'embedding': emb}


class Cnn_9layers_Gru_FrameAtt(_SedModel):
    """pytorch/models.py:564-688."""
    _model_name = 'Cnn_9layers_Gru_FrameAtt'

    def __init__(self, sample_rate, window_size, hop_size, mel_bins, fmin, fmax, classes_num,
                 feature_type):
        super().__init__(sample_rate, window_size, hop_size, mel_bins, fmin, fmax, classes_num,
                         feature_type)
        self.gru = nn.GRU(input_size=512, hidden_size=256, num_layers=1, bias=True,
                          batch_first=True, bidirectional=True)
        self.att_block = AttBlock(n_in=512, n_out=classes_num, activation='sigmoid')
        init_bn(self.bn0)
        init_gru(self.gru)


class Cnn_9layers_Transformer_FrameAtt(_SedModel):
    """pytorch/models.py:981-1077 (always logmel: the reference has no
    feature-type branch)."""
    _model_name = 'Cnn_9layers_Transformer_FrameAtt'

    def __init__(self, sample_rate, window_size, hop_size, mel_bins, fmin, fmax, classes_num,
                 feature_type='logmel'):
        super().__init__(sample_rate, window_size, hop_size, mel_bins, fmin, fmax, classes_num,
                         'logmel')
        self.multihead = MultiHead(8, 512, 64, 64, 0.2)
        self.att_block = AttBlock(n_in=512, n_out=classes_num, activation='sigmoid')
        init_bn(self.bn0)
