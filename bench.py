"""Benchmark of the MI355X-native SED inference path (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--model gru|transformer]
                    [--mode clip|window] [--batch 32] [--precision winograd|exact|x3]
                    [--no-cpu-baseline] [--no-side]

With --gpus N > 1 and no WORLD_SIZE in the environment (a plain
``python bench.py --gpus 8``) the process launches N ranks itself before it
touches the GPU: N child processes of this script with RANK / LOCAL_RANK /
WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT set (the contract torchrun
gives them; under torch.distributed.run the script runs as that rank
directly), prints rank 0's JSON line and exits non-zero if any rank fails.

One step = one forward of the hot path over one batch of synthetic 10 s @
16 kHz clips per GPU (clip mode = main_strong inference_prob semantics, B=32
per GPU: BASELINE.json configs[1]), inputs already resident in HBM, weights
random-init with the reference architecture.  The headline computes in fp32
throughout (no operand narrower than fp32): every GEMM on fp32 operands with
fp32 accumulation (v_mfma_f32_32x32x2_f32, GRU recurrence on fp32 MFMA), block
1's conv2 and blocks 2-4's convs as Winograd F(2x2,3x3) with fp32 transforms
(--precision winograd, the library's default arithmetic).  For
N > 1 (one process per GPU) every rank runs its own shard of clips (weak
scaling) and the framewise outputs are gathered to rank 0 over RCCL inside
each step — the path's only collective.  Rank 0 prints ONE JSON line.

At N = 1 the line also carries, each with its own roofline:
  value_exact         the same workload with the direct fp32 conv everywhere
                      (the reference's operation order; sedx_set_precision EXACT)
  value_x3            the same workload with the opt-in 3xbf16-split MFMA
  configs.config3     Cnn_9layers_Transformer_FrameAtt logmel 16k, B=32
  configs.config4     Cnn_9layers_Gru_FrameAtt gammatone 32k, B=32 (float64
                      gammatone features from 32 kHz audio + the forward)
  configs.window_mode predict.py semantics, 6 x 5 s windows per clip
  cpu_baseline        the oracle (CPU restatement) at B=32 on the host cores,
                      clip mode and predict.py's batch-1 window loop, with the
                      parity of the same clips (framewise, event lists,
                      threshold margin)
"""
import argparse
import contextlib
import ctypes
import json
import os
import socket
import statistics
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.abspath(__file__))
T_START = time.perf_counter()


def _ab_package(argv):
    """--ab-package DIR (A/B runs of kernel variants, tools/ab_build.sh): an
    alternative build of the package, named on the command line and recorded
    in the JSON line ('library'); the default is the in-tree package."""
    for i, a in enumerate(argv):
        if a == '--ab-package' and i + 1 < len(argv):
            return os.path.abspath(argv[i + 1])
        if a.startswith('--ab-package='):
            return os.path.abspath(a.split('=', 1)[1])
    return None


for _p in (REPO, _ab_package(sys.argv[1:]) or os.path.join(REPO, 'sound-event-detection_amd')):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from sedx import _lib, distributed, inference, models, synth  # noqa: E402

MODEL_NAMES = {'gru': 'Cnn_9layers_Gru_FrameAtt', 'transformer': 'Cnn_9layers_Transformer_FrameAtt'}
METRICS = {'gru': '10s@16kHz clips/sec (whole node) + ms/clip p50, Cnn_9_Gru_FrameAtt logmel',
           'transformer': '10s@16kHz clips/sec (whole node) + ms/clip p50, Cnn_9_Transformer_FrameAtt logmel'}
# MI355X_MICROARCH.md: FP32 matrix peak 157.3 TF; BF16 dense MFMA ~2.5 PF.  The
# x3 scheme issues 3 bf16 MFMAs per useful MAC, so its arithmetic peak is 2.5/3 PF.
PEAK_TF = {'exact': 157.3, 'winograd': 157.3, 'x3': 2500.0 / 3}
PEAK_HBM_GBPS = 8000.0
PEAK_FP64_TF = 78.6        # MI355X datasheet FP64 vector (not in MI355X_MICROARCH.md)
DTYPE = {'exact': 'f32',
         'x3': 'bf16x3-split (3 bf16 MFMAs per f32 MAC: hi*hi + hi*lo + lo*hi, f32 accumulate)'}


def dtype_of(precision):
    """The arithmetic a precision computes in (winograd: which layers run which
    Winograd form, per WINO_F43 / WINO_BLOCK1)."""
    if precision != 'winograd':
        return DTYPE[precision]
    b1 = ('conv1 + conv2 of block 1 as the direct fused conv' if not WINO_BLOCK1 else
          'conv2 of block 1 as Winograd F(4x4,3x3)' if WINO_F43 == 2 else
          'conv2 of block 1 as Winograd F(2x2,3x3)')
    rest = 'blocks 2-4 as Winograd F(4x4,3x3)' if WINO_F43 else 'blocks 2-4 as Winograd F(2x2,3x3)'
    return 'f32 (%s, %s: f32 transforms, f32 MFMA, f32 accumulate)' % (b1, rest)
# Winograd F(2x2,3x3): 16 matrix-pipe multiplies per 2x2 output tile where the
# direct conv does 36 ('winograd' mode: blocks 2-4, and block 1's conv2 unless
# --wino-block1 0 keeps block 1 as the direct fused launch; 1 feeds it from a
# separate conv1 launch, 2 computes conv1 inside the Winograd launch)
WINO_BLOCK1 = 2
WINO_MUL = 16.0 / 36.0
# Winograd F(4x4,3x3) (SEDX_TUNE_WINO_F43): 36 multiplies per 4x4 output tile
# where the direct conv does 144 — 1: blocks 2-4; 2 (the library default):
# blocks 1-4, block 1 as a conv1 launch + the F(4x4,3x3) conv2
WINO_F43 = 2
WINO43_MUL = 36.0 / 144.0
# SEDX_TUNE_GRU_KERNEL values (include/sedx.h)
GRU_KERNELS = {'coop': 0, 'simple': 1, 'tag16': 2, 'tag8': 3, 'coop16': 4, 'auto': 5, 'ksplit': 6, 'pair': 7}


def wino_stages():
    return (('b1c2',) if WINO_BLOCK1 else ()) + ('b2c1', 'b2c2', 'b3c1', 'b3c2', 'b4c1', 'b4c2')


def wino_mul(stage):
    """Matrix-pipe multiplies of a winograd-mode stage per direct-conv multiply."""
    if stage not in wino_stages():
        return 1.0
    return WINO43_MUL if (WINO_F43 and (stage != 'b1c2' or WINO_F43 == 2)) else WINO_MUL
# conv stages of sedx_stage_times: (F, Cin, Cout, number of 2x poolings before it)
CONV_STAGES = {'b1c2': (64, 64, 64, 0), 'b2c1': (32, 64, 128, 1), 'b2c2': (32, 128, 128, 1),
               'b3c1': (16, 128, 256, 2), 'b3c2': (16, 256, 256, 2), 'b4c1': (8, 256, 512, 3),
               'b4c2': (8, 512, 512, 3)}
FRONTEND_BYTES_PER_CLIP = 160000 * 4 + 1001 * 64 * 4   # waveform in + X0 out
# per 512-sample frame: 256-point complex FFT (5 N log2 N), real unpack
# (~10 per bin), window, |X|^2 (3 per bin), mel (2 per band weight, 514 at
# 16 kHz), dB + bn0 (~4 per band)
FRONTEND_FLOPS_PER_FRAME = 5 * 256 * 8 + 10 * 257 + 512 + 3 * 257 + 2 * 514 + 4 * 64
PEAK_VALU_F32_TF = 78.6    # non-packed f32 VALU (packed FP32 is excluded beside MFMA)


# --backend gloo (a rehearsal of the N-rank path on one GPU: every rank on
# device 0, the gathers through host copies); nccl (= RCCL, the default at
# N > 1) gathers device tensors over xGMI
GATHER_CPU = False


def gather_outputs(out, world, rank):
    """The step's only collective: framewise + clipwise of every
    rank's shard to rank 0.  Returns (framewise, clipwise) on rank 0."""
    fw, cw = out['framewise_output'], out['clipwise_output']
    if world == 1:
        return fw, cw
    if GATHER_CPU:
        fw, cw = fw.cpu(), cw.cpu()
    return distributed.gather_to_rank0(fw, world, rank), distributed.gather_to_rank0(cw, world, rank)


def conv_flops(stage, B, T):
    F, cin, cout, npool = CONV_STAGES[stage]
    for _ in range(npool):
        T //= 2
    return 2.0 * B * T * F * cout * 9 * cin


def build_model(name, device, preset=(16000, 512, 160, 64, 25, 7000), feature='logmel'):
    m = getattr(models, name)(*preset, 25, feature)
    sd = m.state_dict()
    for k, v in synth.make_state_dict(name, seed=0).items():
        sd[k] = torch.from_numpy(v)
    m.load_state_dict(sd)
    m.set_tuning(_lib.TUNE_WINO_BLOCK1, int(WINO_BLOCK1))
    m.set_tuning(_lib.TUNE_WINO_F43, int(WINO_F43))
    return m.to(device).eval()


# ---------------------------------------------------------------------------
# CPU baseline: the oracle (test infrastructure) on the host cores
# ---------------------------------------------------------------------------
def cpu_info():
    model, logical, cores = None, os.cpu_count(), set()
    try:
        phys = core = None
        with open('/proc/cpuinfo') as f:
            for line in f:
                k, _, v = line.partition(':')
                k, v = k.strip(), v.strip()
                if k == 'model name' and model is None:
                    model = v
                elif k == 'physical id':
                    phys = v
                elif k == 'core id':
                    core = v
                elif not k and phys is not None:
                    cores.add((phys, core))
                    phys = core = None
    except OSError:
        pass
    return {'cpu_model': model, 'host_logical_cpus': logical,
            'host_physical_cores': len(cores) or None}


def cpu_quota():
    """CPUs granted by the cgroup CPU quota (cgroup v2 cpu.max or v1
    cfs_quota/period), None when unlimited or unreadable."""
    try:
        with open('/sys/fs/cgroup/cpu.max') as f:
            q, per = f.read().split()[:2]
        if q != 'max':
            return max(1, -(-int(q) // int(per)))
    except (OSError, ValueError):
        pass
    try:
        with open('/sys/fs/cgroup/cpu/cpu.cfs_quota_us') as f:
            q = int(f.read())
        with open('/sys/fs/cgroup/cpu/cpu.cfs_period_us') as f:
            per = int(f.read())
        if q > 0:
            return max(1, -(-q // per))
    except (OSError, ValueError):
        pass
    return None


def cpu_threads():
    """Host CPUs this process may use: its affinity set, capped by the cgroup
    CPU quota (the GPU box's lease grants a share of a large machine whose
    affinity set shows every CPU): the oracle runs one torch thread per CPU
    it may use."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    q = cpu_quota()
    return min(n, q) if q else n


def progress(msg):
    """One line on stderr per bench leg (the JSON record is the only stdout
    line): a long run shows it is alive."""
    print('[bench %.0fs] %s' % (time.perf_counter() - T_START, msg), file=sys.stderr, flush=True)


def cpu_baseline(name, model, dev, seconds, B=32):
    """Clip mode: the oracle forward on B=32 clips per iteration (1 warm-up,
    then timed iterations for ~``seconds``).  The same clips go through the
    GPU path; the oracle is the checker: max |d framewise|, event lists
    (frame_prediction_to_event_prediction_v2 on both sides) and the smallest
    distance of any oracle value to a threshold."""
    from oracle import sed_oracle as O
    torch.set_num_threads(cpu_threads())
    sd = O.full_state(synth.make_state_dict(name, seed=0), '16k')
    wave = synth.make_waveforms(B, seconds=10.0, sample_rate=16000, seed=7)
    O.forward(sd, name, wave=wave[:2])  # warm-up (allocator, threads)
    ts, ref = [], None
    t_all = time.perf_counter()
    while True:
        a = time.perf_counter()
        ref = O.forward(sd, name, wave=wave)
        ts.append(time.perf_counter() - a)
        if time.perf_counter() - t_all >= seconds and len(ts) >= 2:
            break
    rate = B * len(ts) / sum(ts)
    out = {'value': round(rate, 3), 'unit': 'clips/s', 'cores': torch.get_num_threads(), 'kind': 'port',
           'cpus_affinity': len(os.sched_getaffinity(0)) if hasattr(os, 'sched_getaffinity') else None,
           'cpu_quota': cpu_quota(),
           'ms_per_clip_p50': round(statistics.median(ts) / B * 1e3, 2),
           'sample': '%d iterations of B=%d x 10 s clips (clip mode, %.1f s) through oracle/sed_oracle.py '
                     'forward (torch fp32, the reference op sequence) on %d host threads'
                     % (len(ts), B, sum(ts), torch.get_num_threads())}
    out.update(cpu_info())
    with torch.no_grad():
        fw = model(torch.from_numpy(wave).to(dev))['framewise_output']
    gfw = fw.cpu().numpy()
    rfw = ref['framewise_output'].numpy()
    params = dict(inference.DEFAULT_PREDICT_PARAMS)
    ev_gpu = inference.events_from_framewise(fw, params)
    ev_ref = O.events_from_framewise(rfw, params)
    thr = np.array([params['sed_high_threshold'], params['sed_low_threshold']], np.float64)
    out['parity'] = {
        'max_abs_framewise': float(np.max(np.abs(gfw - rfw))), 'tolerance': 1e-3,
        'events_identical': ev_gpu == ev_ref, 'n_events': len(ev_ref),
        'min_threshold_margin': float(np.min(np.abs(rfw.astype(np.float64)[..., None] - thr))),
        'thresholds': {'high': params['sed_high_threshold'], 'low': params['sed_low_threshold']},
        'sample': '%d clips, GPU (this precision) vs oracle' % B}
    return out


def cpu_baseline_window(name, seconds, max_clips=64):
    """predict.py's loop (pytorch/predict.py:297-349): every 10 s clip as six
    batch-1 forwards of 5 s windows at 1 s stride, merged and averaged, then
    thresholded — the oracle restatement of that loop, timed per clip."""
    from oracle import sed_oracle as O
    sd = O.full_state(synth.make_state_dict(name, seed=0), '16k')
    audio = synth.make_waveforms(max_clips, seconds=10.0, sample_rate=16000, seed=9)
    O.predict_windows(sd, name, audio[0], 16000)   # warm-up
    ts = []
    t_all = time.perf_counter()
    for i in range(max_clips):
        a = time.perf_counter()
        merged = O.predict_windows(sd, name, audio[i], 16000, 5, 1)
        O.events_from_framewise(merged, inference.DEFAULT_PREDICT_PARAMS)
        ts.append(time.perf_counter() - a)
        if time.perf_counter() - t_all >= seconds and len(ts) >= 3:
            break
    return {'value': round(len(ts) / sum(ts), 3), 'unit': 'clips/s', 'cores': torch.get_num_threads(),
            'kind': 'port', 'ms_per_clip_p50': round(statistics.median(ts) * 1e3, 1),
            'sample': '%d x 10 s clips through oracle predict_windows (6 batch-1 5 s windows, '
                      'merge + avg_merge) + events, %.1f s' % (len(ts), sum(ts))}


# ---------------------------------------------------------------------------
# GPU measurement
# ---------------------------------------------------------------------------
def measure(step, args, world, dev, model=None, B=32):
    """Throughput over K steps with ``args.streams`` batches in flight: step i
    is issued on stream i % streams (a serving loop with that many concurrent
    requests), so one batch's GRU / MHA + head overlap the next batch's conv
    stack.  Every step is a complete forward of its own batch.  Returns
    (clips/s over all ranks, elapsed s, per-stage ms over the timed region)."""
    cuda = dev.type == 'cuda'
    streams = [torch.cuda.Stream(dev) if cuda else None for _ in range(max(1, args.streams))]

    def on(st):
        return torch.cuda.stream(st) if cuda else contextlib.nullcontext()

    if model is not None:
        # conv stacks in issue order (sedx_set_pipelined): without it the
        # batches in flight can fall into lockstep, two conv stacks splitting
        # the chip and the GRUs running side by side on 32 CUs
        model.set_pipelined(getattr(args, 'pipeline_mode', 1) if len(streams) > 1 and not args.no_pipeline else 0)
    sync(dev)
    for i in range(args.warmup):
        with on(streams[i % len(streams)]):
            step()
    sync(dev)
    if world > 1:
        dist.barrier()
    nat = L = None
    prof = model is not None and getattr(model, 'stage_profiling', True)
    if prof:
        # per-stage HIP events over the timed region: libsedx records them on
        # the stream each forward's kernels are launched on, one event set per
        # forward (accumulate mode), averaged by sedx_stage_times afterwards
        nat, L = model.native(dev), _lib.lib()
        _lib.check(L.sedx_set_profiling(nat.h, 2), nat.h, 'set_profiling')
    sync(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        with on(streams[i % len(streams)]):
            step()
    sync(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    stage_ms = None
    if prof:
        ms = (ctypes.c_float * len(_lib.STAGES))()
        n = ctypes.c_int32()
        _lib.check(L.sedx_stage_times(nat.h, ms, len(_lib.STAGES), ctypes.byref(n)), nat.h, 'stage_times')
        _lib.check(L.sedx_set_profiling(nat.h, 0), nat.h, 'set_profiling')
        stage_ms = {s_: round(float(v), 4) for s_, v in zip(_lib.STAGES, ms[:])}
    if model is not None:
        model.set_pipelined(False)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device='cpu' if GATHER_CPU else dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return world * B * args.steps / elapsed, elapsed, stage_ms


def sync(dev):
    if dev.type == 'cuda':
        torch.cuda.synchronize(dev)


def latency(step_fn, B, reps, dev=None):
    """p50 / p99 of (batch wall time / clips), one batch at a time."""
    dev = dev or torch.device('cuda', torch.cuda.current_device())
    lat = []
    for _ in range(reps):
        sync(dev)
        a = time.perf_counter()
        step_fn()
        sync(dev)
        lat.append((time.perf_counter() - a) * 1e3 / B)
    lat.sort()
    return statistics.median(lat), lat[min(len(lat) - 1, int(0.99 * len(lat)))]


def host_to_host_step(model, host_wave, host_out, dev, world, rank):
    """One batch from host-visible (pinned) input to the gathered framewise
    output back in pinned host memory on rank 0 (SURVEY §8(d) p50 definition):
    the H2D copy runs on a copy stream and the compute stream waits for it."""
    copy = torch.cuda.Stream(dev)

    def step():
        with torch.cuda.stream(copy):
            d = host_wave.to(dev, non_blocking=True)
        torch.cuda.current_stream(dev).wait_stream(copy)
        d.record_stream(torch.cuda.current_stream(dev))
        with torch.no_grad():
            fw, _ = gather_outputs(model(d), world, rank)
        if rank == 0:
            host_out.copy_(fw, non_blocking=True)
    return step


def latency_b1(model, dev, reps=20):
    """End-to-end latency of ONE 10 s clip: clip mode (eager,
    and replayed from a HIP graph: sedx.inference.GraphedForward), window mode
    (its 6 windows in one launch) with the input on the device, and clip mode
    from a host buffer to the framewise output back on the host
    (PCIe-inclusive)."""
    w1 = torch.from_numpy(synth.make_waveforms(1, seconds=10.0, sample_rate=16000, seed=11))
    wd = w1.to(dev)
    out = {}
    graphed = inference.GraphedForward(model, wd)
    for key, fn in (('clip', lambda: model(wd)['framewise_output']),
                    ('clip_graph', lambda: graphed(wd)['framewise_output']),
                    ('window', lambda: inference.predict_windows(model, wd, 5, 1)),
                    ('clip_host_to_host', lambda: model(w1.to(dev))['framewise_output'].cpu())):
        with torch.no_grad():
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            ts = []
            for _ in range(reps):
                a = time.perf_counter()
                fn()
                torch.cuda.synchronize()
                ts.append((time.perf_counter() - a) * 1e3)
        out[key] = round(statistics.median(ts), 4)
    out['unit'] = 'ms p50'
    # where the one clip's device time goes (per stage, HIP events, one
    # forward at a time)
    out['stage_ms'] = stage_times_isolated(model, wd, dev, reps)
    return out


def stage_times_isolated(model, wave, dev, reps):
    """Per-stage device time one batch at a time (sedx_set_profiling mode 1)."""
    nat, L = model.native(dev), _lib.lib()
    _lib.check(L.sedx_set_profiling(nat.h, 1), nat.h, 'set_profiling')
    acc = np.zeros(len(_lib.STAGES))
    for _ in range(reps):
        with torch.no_grad():
            model(wave)
        ms = (ctypes.c_float * len(_lib.STAGES))()
        n = ctypes.c_int32()
        _lib.check(L.sedx_stage_times(nat.h, ms, len(_lib.STAGES), ctypes.byref(n)), nat.h, 'stage_times')
        acc += np.array(ms[:])
    _lib.check(L.sedx_set_profiling(nat.h, 0), nat.h, 'set_profiling')
    return {s: round(float(v), 4) for s, v in zip(_lib.STAGES, acc / reps)}


# ---------------------------------------------------------------------------
# rooflines
# ---------------------------------------------------------------------------
# HBM traffic per launch, rocprof average duration, MFMA busy and clock come
# from the rocprofv3 passes of this bench command (tools/profile_round.sh ->
# tools/pmc_summary.py; FETCH_SIZE x2 per the gfx950 correction + WRITE_SIZE),
# committed under profiles/.
PROFILE_SUMMARY = os.path.join(REPO, 'profiles', 'r06zd_winograd_kernel_summary.json')
# the same passes over the config-4 leg (bench.py --mode gamma: B = 32 x 10 s
# @ 32 kHz, T = 994 frames)
GAMMA_PROFILE_SUMMARY = os.path.join(REPO, 'profiles', 'r06zd_config4_kernel_summary.json')
# the same passes over the window-mode leg (bench.py --mode window: B' = 192
# windows x 501 frames per call)
WINDOW_PROFILE_SUMMARY = os.path.join(REPO, 'profiles', 'r06zd_window_kernel_summary.json')
GAMMA_KERNELS = ('sedx::gamma_init_kernel', 'sedx::gamma_spec_kernel<2048>', 'sedx::gamma_erb_kernel',
                 'sedx::gamma_quant_kernel')


# block 1's conv1 (Cin 1 -> 64) computed inside the b1c2 launch (winograd
# mode with the Winograd block 1: its own launch, stage b1c1)
def fused_block1(precision):
    # matrix-pipe conv1 inside the b1c2 launch (exact / x3 / --wino-block1 0);
    # --wino-block1 2 computes it inside too, but on the VALU (not priced here)
    return precision != 'winograd' or not WINO_BLOCK1


def conv_kernel_name(stage, precision):
    """rocprof kernel name of a conv stage's launch."""
    F, cin, cout, _ = CONV_STAGES[stage]
    epi = {'b1c2': 1, 'b2c1': 0, 'b2c2': 1, 'b3c1': 0, 'b3c2': 1, 'b4c1': 0, 'b4c2': 2}[stage]
    bn = 64 if cout == 64 else 128
    if precision == 'x3':
        return 'sedx::conv3x3_x3_kernel<%d, %d, %d, %s>' % (F, bn, epi, 'true' if stage == 'b1c2' else 'false')
    # winograd with F(4x4,3x3) and block 1 in one launch: the chunk-of-4
    # activation layout between them (the kernels' last template argument)
    c4 = 'true' if (WINO_F43 and WINO_BLOCK1 == 2) else 'false'
    if precision == 'winograd' and stage == 'b1c2' and WINO_BLOCK1 == 2 and WINO_F43 != 2:
        return 'sedx::wino_block1_kernel<2, %s>' % c4
    if precision == 'winograd' and stage in wino_stages() and wino_mul(stage) == WINO43_MUL:
        # (the last two arguments: 4 channel tiles and 2 tile groups per item
        # at the bench's B = 32)
        return 'sedx::conv3x3_wino43_kernel<%d, %d, %s, 4, 2>' % (F, epi, c4)
    if precision == 'winograd' and stage in wino_stages():
        # 2 tile groups x 64 channels (8 row waves) at the bench shapes
        return 'sedx::conv3x3_wino_kernel<%d, %d, 2, 2>' % (F, epi)
    # exact: 8-wave 64x64 wave tiles at the bench shapes (4-wave / 32x32 only for small grids)
    return 'sedx::conv3x3_kernel<%d, %d, %d, %s, 8, 64>' % (F, bn, epi, 'true' if stage == 'b1c2' else 'false')


def profiled(kernel, summary=PROFILE_SUMMARY):
    """(HBM bytes per launch, rocprofv3 average ms, MFMA busy fraction,
    effective clock GHz) of ``kernel`` from the committed summary."""
    try:
        with open(summary) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None, None, None, None
    # summaries before round 6 name the F(4x4,3x3) kernels without the tile
    # group argument (<F, EPI, C4, 4>, the same launch as <..., 4, 2>)
    v = d.get(kernel) or d.get(kernel.replace(', 4, 2>', ', 4>'), {})
    ns = v.get('avg_ns')
    util, clk = v.get('mfma_util'), v.get('clock_ghz')
    return (v.get('hbm_bytes_corrected'), (round(ns * 1e-6, 4) if ns else None),
            round(util, 4) if util else None, round(clk, 3) if clk else None)


def roofline(stage_ms, B, precision, T=1001, iso_ms=None, summary=None):
    """MFMA roofline of the dominant conv launch.

    achieved = FLOPs the launch executes on the matrix pipe (direct conv:
    2 B T F Cout 9 Cin, + the fused block-1 conv1 2 B T 64 64 9 for b1c2;
    Winograd layers: 16/36 (F(2x2,3x3)) or 36/144 (F(4x4,3x3)) of the direct
    conv's, without the tile padding of a ragged last tile row) / its launch time, with the
    launch time from HIP events on the launch stream measured live in this
    run ONE BATCH AT A TIME (``iso_ms``: sedx_set_profiling mode 1; the
    rocprofv3 summary of the same single-stream work is committed under
    profiles/ and must agree).  The same launch's interval inside the
    two-stream timed region (it then shares the chip with the previous
    batch's GRU / head) is reported beside it (``*_timed_region``), and the
    direct-conv-equivalent rate (what a direct conv would need for this time;
    can exceed the peak for Winograd) as ``direct_conv_equiv_tflops``.
    Profile-derived fields (traffic, rocprof time, MFMA busy) come from the
    committed summary of the same shapes: ``summary`` (config 4's passes), or
    for the B=32, 10 s @ 16 kHz shapes PROFILE_SUMMARY."""
    conv = {s_: stage_ms[s_] for s_ in CONV_STAGES}
    dom = max(conv, key=conv.get)
    wino = precision == 'winograd'
    mul = {st: (wino_mul(st) if wino else 1.0) for st in CONV_STAGES}
    flops = conv_flops(dom, B, T) * mul[dom]
    if dom == 'b1c2' and fused_block1(precision):
        flops += 2.0 * B * T * 64 * 64 * 9      # conv1 (Cin 1 -> 64) computed inside the launch
    peak = PEAK_TF[precision]
    t_iso = iso_ms.get(dom) if iso_ms else None
    t = t_iso if t_iso else conv[dom]
    achieved = flops / (t * 1e-3) / 1e12
    conv1 = 2.0 * B * T * 64 * 64 * 9
    total = sum(conv_flops(st, B, T) * mul[st] for st in CONV_STAGES) + conv1
    total_direct = sum(conv_flops(st, B, T) for st in CONV_STAGES) + conv1
    conv_ms = sum(conv.values()) + stage_ms.get('b1c1', 0.0)
    kname = conv_kernel_name(dom, precision)
    if summary is None and (B, T) == (32, 1001):
        summary = PROFILE_SUMMARY
    traffic, rocprof_ms, mfma_util, clock = profiled(kname, summary) if summary else (None,) * 4
    direct = flops / mul[dom]
    out = {'bound': 'mfma', 'kernel': '%s (%s)' % (kname, dom),
           'arith': {'exact': 'fp32 MFMA v_mfma_f32_32x32x2_f32 (f32 in, f32 acc)',
                     'winograd': ('fp32 MFMA (f32 in, f32 acc); Winograd layers counted as executed FLOPs: '
                                  '%s' % ', '.join('%s %s' % (st, 'F(4x4,3x3) 36/144 of direct, v_mfma_f32_16x16x4_f32'
                                                             if wino_mul(st) == WINO43_MUL else
                                                             'F(2x2,3x3) 16/36 of direct, v_mfma_f32_32x32x2_f32')
                                                   for st in wino_stages())),
                     'x3': '3xbf16-split MFMA 32x32x16, f32 acc (peak = bf16 dense 2.5 PF / 3)'}[precision],
           'achieved': round(achieved, 2), 'peak': round(peak, 1), 'unit': 'TFLOP/s',
           'frac': round(achieved / peak, 4),
           'traffic': traffic, 'traffic_unit': 'bytes/launch (HBM, rocprofv3 PMC)',
           'traffic_source': os.path.relpath(summary, REPO) if traffic is not None else None,
           'flops_per_launch': flops, 'avg_launch_ms': round(t, 4),
           'timing': ('avg_launch_ms: HIP events on the launch stream, one batch at a time, measured live in this '
                      'run (sedx_set_profiling 1)' if t_iso else
                      'avg_launch_ms: HIP events on the launch stream over the timed region'),
           'avg_launch_ms_timed_region': conv[dom],
           'achieved_timed_region': round(flops / (conv[dom] * 1e-3) / 1e12, 2),
           'frac_timed_region': round(flops / (conv[dom] * 1e-3) / 1e12 / peak, 4),
           'timed_region_note': 'the launch interval inside the two-stream timed region (one event set per '
                                'forward, all steps averaged): it shares the chip with the previous batch\'s '
                                'GRU / head and the next batch\'s frontend',
           'avg_launch_ms_rocprof': rocprof_ms,
           'frac_rocprof': round(flops / (rocprof_ms * 1e-3) / 1e12 / peak, 4) if rocprof_ms else None,
           'mfma_busy_frac_pmc': mfma_util, 'clock_ghz_pmc': clock,
           'rocprof_source': ('rocprofv3 --kernel-trace --stats of bench.py --streams 1 --no-side, %s'
                              % os.path.relpath(summary, REPO)) if rocprof_ms else None,
           # the reference's algorithmic FLOPs (the direct conv's)
           # over the same time: a rate, not a roofline fraction (> peak for
           # Winograd, which executes 16/36 of the multiplies)
           'flops_per_launch_direct_conv': direct,
           'direct_conv_equiv_tflops': round(direct / (t * 1e-3) / 1e12, 2),
           'conv_stack_tflops': round(total / (conv_ms * 1e-3) / 1e12, 2),
           'conv_stack_frac': round(total / (conv_ms * 1e-3) / 1e12 / peak, 4),
           'conv_stack_direct_equiv_tflops': round(total_direct / (conv_ms * 1e-3) / 1e12, 2),
           'conv_stack_ms': round(conv_ms, 4)}
    return out


# ---------------------------------------------------------------------------
# legs
# ---------------------------------------------------------------------------
def clip_leg(model, wave, args, world, rank, dev, precision, isolated=False):
    """Throughput + per-stage timed-region times + device p50/p99; with
    ``isolated`` also the per-stage times one batch at a time (the roofline's
    launch time)."""
    model.set_precision(precision)
    B = wave.shape[0]

    def step():
        with torch.no_grad():
            gather_outputs(model(wave), world, rank)

    value, elapsed, stage_ms = measure(step, args, world, dev, model, B)
    p50, p99 = latency(step, B, max(5, min(args.steps, 20)), dev)
    iso = stage_times_isolated(model, wave, dev, max(3, min(args.steps, 10))) if isolated else None
    return value, elapsed, stage_ms, p50, p99, iso


def gamma_profile(B):
    """(HBM bytes, rocprofv3 ms) per batch of the gammatone frontend's launches
    from the config-4 PMC passes (B = 32 only; else (None, None))."""
    prof = [profiled(k, GAMMA_PROFILE_SUMMARY) for k in GAMMA_KERNELS] if B == 32 else []
    traffic = sum(p[0] for p in prof) if prof and all(p[0] is not None for p in prof) else None
    rocprof_ms = sum(p[1] for p in prof) if prof and all(p[1] is not None for p in prof) else None
    return traffic, rocprof_ms


def gamma_leg(args, dev, precision):
    """BASELINE config 4: Cnn_9layers_Gru_FrameAtt gammatone 32k, B=32.  A
    step = float64 gammatone features of 32 x 10 s @ 32 kHz clips (the
    reference computes them on the CPU at HDF5-pack time, utils/features.py:
    361-370) + the gamma-branch forward (models.py:636-688)."""
    name = MODEL_NAMES['gru']
    m = build_model(name, dev, (32000, 1024, 320, 64, 50, 14000), 'gamma').set_precision(precision)
    if getattr(args, 'gamma_spec', None) is not None:
        m.set_tuning(_lib.TUNE_GAMMA_SPEC, args.gamma_spec)
    B = args.batch
    audio = torch.from_numpy(synth.make_waveforms(B, 10.0, 32000, seed=4321)).to(dev)

    def step():
        with torch.no_grad():
            m(inference.gamma_features(m, audio))

    value, elapsed, stage_ms = measure(step, args, 1, dev, m, B)
    with torch.no_grad():
        feats = inference.gamma_features(m, audio)
    iso = stage_times_isolated(m, feats, dev, max(3, min(args.steps, 10)))
    # gamma frontend alone, timed with torch events on the current stream (its
    # kernels are launched on that stream)
    for _ in range(2):
        inference.gamma_features(m, audio)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 5
    e0.record()
    for _ in range(reps):
        inference.gamma_features(m, audio)
    e1.record()
    torch.cuda.synchronize()
    fe_ms = e0.elapsed_time(e1) / reps
    T = 994
    flops = B * (T * (5.0 * 1024 * 10 + 8.0 * 1025) + 2.0 * 64 * 1025 * T)   # FFT + unpack/|X| + ERB product
    bytes_ = B * (320000 * 4 + 64 * T * 4)
    traffic, rocprof_fe = gamma_profile(B)
    return {'workload': 'Cnn_9layers_Gru_FrameAtt gammatone 32k, %d x 10 s @ 32 kHz clips per step '
                        '(float64 gammatone features + forward)' % B,
            'value': round(value, 2), 'unit': 'clips/s', 'dtype': dtype_of(precision) + '; gammatone frontend f64',
            'ms_per_step': round(elapsed / args.steps * 1e3, 4),
            'roofline': roofline(stage_ms, B, precision, T=T, iso_ms=iso,
                                 summary=GAMMA_PROFILE_SUMMARY if B == 32 else None),
            'gamma_frontend': {'ms_per_batch': round(fe_ms, 4), 'bound': 'fp64',
                               'achieved': round(flops / (fe_ms * 1e-3) / 1e12, 3), 'peak': PEAK_FP64_TF,
                               'unit': 'TFLOP/s (f64)', 'frac': round(flops / (fe_ms * 1e-3) / 1e12 / PEAK_FP64_TF, 4),
                               'hbm_gbps_algorithmic': round(bytes_ / (fe_ms * 1e-3) / 1e9, 1),
                               'bytes_algorithmic': bytes_, 'traffic': traffic,
                               'traffic_unit': 'bytes/batch (HBM, rocprofv3 PMC, %s)' % ', '.join(GAMMA_KERNELS),
                               'ms_per_batch_rocprof': round(rocprof_fe, 4) if rocprof_fe else None,
                               'traffic_source': (os.path.relpath(GAMMA_PROFILE_SUMMARY, REPO)
                                                  if traffic is not None else None),
                               'note': 'algorithmic f64 FLOPs: 5 N log2 N complex FFT (N=1024) + unpack '
                                       '+ 64 x 1025 ERB product per frame; bytes: audio in + features out'}}


def window_leg(model, wave, args, dev, precision):
    model.set_precision(precision)
    B = wave.shape[0]

    def step():
        with torch.no_grad():
            inference.predict_windows(model, wave, 5, 1)

    value, elapsed, _ = measure(step, args, 1, dev, None, B)
    p50, p99 = latency(step, B, max(5, min(args.steps, 20)), dev)
    # the dominant launch of one windowed call: B' = 6 B windows of T = 501
    # frames (5 s at hop 160) through the model as one batch
    iso = window_stage_times(model, wave, dev, max(3, min(args.steps, 10)))
    nwin, Tw = 6 * B, 80000 // 160 + 1
    summary = WINDOW_PROFILE_SUMMARY if (B == 32 and os.path.exists(WINDOW_PROFILE_SUMMARY)) else None
    roof = roofline(iso, nwin, precision, T=Tw, iso_ms=iso, summary=summary)
    roof['workload_per_launch'] = '%d windows x %d frames (5 s windows of %d clips)' % (nwin, Tw, B)
    return {'value': round(value, 2), 'unit': 'clips/s', 'windows_per_clip': 6,
            'windows_per_s': round(6 * value, 1), 'ms_per_step': round(elapsed / args.steps * 1e3, 4),
            'ms_per_clip_p50': round(p50, 4), 'ms_per_clip_p99': round(p99, 4),
            'ms_per_clip_p50_note': 'device input, one batch of %d clips (its %d windows) at a time, per clip'
                                    % (B, nwin),
            'roofline': roof, 'stage_ms_isolated': iso,
            'dtype': dtype_of(precision),
            'note': '5 s windows, 1 s stride, all windows of the batch in one launch, merged + avg_merge '
                    'on the GPU (predict.py:297-349)'}


def config5_leg(model, wave, args, world, rank, dev, precision, isolated=True):
    """BASELINE config 5 (Cnn_9layers_Transformer_FrameAtt, B per GPU, N GPUs):
    the N > 1 run's second leg — the same clip-sharded step (every rank its
    own clips, framewise + clipwise gathered to rank 0 each step) on the
    Transformer model.  Whole-job clips/s from the max-over-ranks time."""
    B = wave.shape[0]
    v, e, st, p50, _, iso = clip_leg(model, wave, args, world, rank, dev, precision, isolated=isolated)
    out = {'workload': '%s logmel 16k, %d x 10 s clips per GPU per step (clip mode)' % (MODEL_NAMES['transformer'], B),
           'metric': METRICS['transformer'], 'value': round(v, 2), 'unit': 'clips/s', 'n_gpus': world,
           'global_batch': B * world, 'batch_per_gpu': B,
           'backend': dist.get_backend() if world > 1 else None,
           'ms_per_step': round(e / args.steps * 1e3, 4), 'ms_per_clip_p50_device': round(p50, 4),
           'scaling': 'weak', 'dtype': dtype_of(precision) if precision in PEAK_TF else precision,
           'gathered': 'framewise_output + clipwise_output to rank 0 every step'}
    if st is not None:
        out['roofline'] = roofline(st, B, precision, iso_ms=iso)
        out['stage_ms'] = st
    return out


def window_stage_times(model, wave, dev, reps):
    """Per-stage device time of one windowed call (all windows of the batch as
    one forward, sedx_set_profiling mode 1), averaged over reps."""
    nat, L = model.native(dev), _lib.lib()
    _lib.check(L.sedx_set_profiling(nat.h, 1), nat.h, 'set_profiling')
    acc = np.zeros(len(_lib.STAGES))
    for _ in range(reps):
        with torch.no_grad():
            inference.predict_windows(model, wave, 5, 1)
        ms = (ctypes.c_float * len(_lib.STAGES))()
        n = ctypes.c_int32()
        _lib.check(L.sedx_stage_times(nat.h, ms, len(_lib.STAGES), ctypes.byref(n)), nat.h, 'stage_times')
        acc += np.array(ms[:])
    _lib.check(L.sedx_set_profiling(nat.h, 0), nat.h, 'set_profiling')
    return {s: round(float(v), 4) for s, v in zip(_lib.STAGES, acc / reps)}


def events_side(model, wave):
    with torch.no_grad():
        fw = model(wave)['framewise_output']
    params = dict(inference.DEFAULT_PREDICT_PARAMS)
    inference.event_pairs(fw, params)
    torch.cuda.synchronize()
    reps = 10
    t0 = time.perf_counter()
    for _ in range(reps):
        n_ev = len(inference.event_pairs(fw, params))
    return {'events_ms_per_batch': round((time.perf_counter() - t0) / reps * 1e3, 4), 'events_per_batch': n_ev}


# ---------------------------------------------------------------------------
# N ranks from a plain `python bench.py --gpus N` (no torchrun around it)
# ---------------------------------------------------------------------------
def _free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(('127.0.0.1', 0))
        return so.getsockname()[1]


def launch_ranks(n, argv):
    """Start n ranks of this script (one process per GPU, the environment
    torch.distributed.run gives each: RANK, LOCAL_RANK, WORLD_SIZE,
    LOCAL_WORLD_SIZE, MASTER_ADDR=127.0.0.1, MASTER_PORT), wait for all of
    them, print rank 0's stdout (the JSON line) and return the exit code: the
    first failing rank's, after stopping the others (they would wait at the
    next collective).  Lines rank 0's libraries print to stdout (gloo's
    connection notes) go to stderr, so stdout holds the one JSON line.  The caller has not touched the GPU (no HIP call in this
    process); the ranks are child processes, never an exec of this one."""
    port = _free_port()
    out = tempfile.TemporaryFile(mode='w+')
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK='0', MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
        env.setdefault('HSA_ENABLE_IPC_MODE_LEGACY', '0')   # dmabuf IPC for RCCL on this host driver
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env,
                                      stdout=out if r == 0 else subprocess.DEVNULL))
    rc = 0
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                rc = bad[0]
                break
            if all(c == 0 for c in codes):
                break
            time.sleep(0.2)
    finally:
        for p in procs:                       # exactly the processes started here
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    out.seek(0)
    for line in out:          # the JSON record to stdout; library chatter on rank 0's stdout to stderr
        (sys.stdout if line.startswith('{"metric"') else sys.stderr).write(line)
    sys.stdout.flush()
    if rc:
        print('bench: a rank exited with %d' % rc, file=sys.stderr)
    return rc if rc > 0 else (1 if rc else 0)


class StubModel:
    """CPU stand-in for the model (tests/test_bench_cpu.py drives the N-rank
    launcher and the N > 1 measurement path with it over gloo): a fixed
    framewise-shaped output from a small CPU computation per call."""
    stage_profiling = False

    def __init__(self):
        self.w = torch.linspace(-1, 1, 25)

    def set_precision(self, p):
        return self

    def set_pipelined(self, on):
        pass

    def __call__(self, wave):
        x = wave[:, :1000].reshape(wave.shape[0], 1000, 1)
        fw = torch.sigmoid(x * self.w)
        return {'framewise_output': fw, 'clipwise_output': fw.max(dim=1).values}


def rank0_cpu_baseline(args, world, rank, run):
    """The CPU baseline on rank 0 only, after every timed leg, at any N: the
    other ranks go on to the closing barrier and wait there while rank 0
    times the oracle (so the N > 1 line carries cpu_baseline too; its sample
    is the same bounded B = 32 oracle run as at N = 1, on rank 0's host
    threads)."""
    if rank != 0 or args.no_cpu_baseline:
        return None
    return run()


def stub_cpu_baseline(B):
    """--stub: the StubModel forward timed on the host (the shape of the real
    record: value / unit / cores / kind / sample)."""
    m = StubModel()
    wave = torch.from_numpy(synth.make_waveforms(B, 0.1, 16000, seed=7))
    ts = []
    for _ in range(3):
        a = time.perf_counter()
        m(wave)
        ts.append(time.perf_counter() - a)
    return {'value': round(B * len(ts) / max(sum(ts), 1e-9), 3), 'unit': 'clips/s',
            'cores': torch.get_num_threads(), 'kind': 'port', 'stub': True,
            'sample': '3 iterations of the CPU stand-in model at B=%d' % B}


def stub_main(args, world, rank):
    """--stub: the launcher + clip_leg's N > 1 branch (gather to rank 0 in
    every step, barrier, all_reduce(MAX) of the elapsed time) on the CPU."""
    dev = torch.device('cpu')
    if rank == args.stub_fail_rank:
        sys.exit(3)
    B = args.batch
    wave = torch.from_numpy(synth.make_waveforms(B, 0.1, 16000, seed=1234 + rank))
    value, elapsed, _, p50, _, _ = clip_leg(StubModel(), wave, args, world, rank, dev, args.precision)
    # the config-5 leg of the N > 1 run (a second model, the same measurement path)
    c5 = config5_leg(StubModel(), wave, args, world, rank, dev, args.precision, isolated=False)
    env = {k: os.environ.get(k) for k in ('RANK', 'LOCAL_RANK', 'WORLD_SIZE', 'MASTER_ADDR')}
    envs = [None] * world if rank == 0 else None
    if world > 1:
        dist.gather_object(env, envs, dst=0)
    else:
        envs = [env]
    cpu = rank0_cpu_baseline(args, world, rank, lambda: stub_cpu_baseline(args.batch))
    if rank == 0:
        print(json.dumps({'metric': 'stub', 'value': round(value, 3), 'unit': 'clips/s', 'n_gpus': world,
                          'steps': args.steps, 'warmup': args.warmup,
                          'ms_per_step': round(elapsed / args.steps * 1e3, 4), 'stub': True,
                          'config': {'world_size': dist.get_world_size() if world > 1 else 1},
                          'cpu_baseline': cpu, 'rank_env': envs, 'configs': {'config5': c5}}))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--batch', type=int, default=32, help='clips per GPU per step')
    ap.add_argument('--streams', type=int, default=2,
                    help='batches in flight per GPU (HIP streams the steps rotate over)')
    ap.add_argument('--no-pipeline', action='store_true',
                    help='streams > 1 without ordering the conv stacks (A/B of sedx_set_pipelined)')
    ap.add_argument('--pipeline-mode', type=int, choices=[1, 2], default=1,
                    help='sedx_set_pipelined mode with streams > 1 (A/B runs): 1 = conv stacks in issue order, '
                         '2 = the same with block 1\'s conv1 issued before the wait')
    ap.add_argument('--model', choices=list(MODEL_NAMES), default='gru')
    ap.add_argument('--mode', choices=['clip', 'window', 'gamma'], default='clip',
                    help="gamma: BASELINE config 4 alone (profiling passes of the gammatone leg)")
    # headline: fp32 with the Winograd conv for blocks 2-4 (the exact direct
    # conv and the opt-in x3 arithmetic are reported beside it)
    ap.add_argument('--precision', choices=list(PEAK_TF), default='winograd')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-side', action='store_true',
                    help='headline only (no x3 / config 3 / config 4 / window legs, no latency_b1): '
                         'profiling passes use it so per-kernel rocprof averages cover only the headline')
    ap.add_argument('--cpu-seconds', type=float, default=15.0)
    ap.add_argument('--gru-kernel', choices=list(GRU_KERNELS), default='auto',
                    help='GRU recurrence kernel (SEDX_TUNE_GRU_KERNEL; A/B runs); auto: the library default '
                         '(16 slices; on a pipelined handle dealt over every XCD)')
    ap.add_argument('--wino-order', type=int, choices=[0, 1, 2], default=None,
                    help='SEDX_TUNE_WINO_ORDER (A/B runs): Winograd item order on the 512-channel layers')
    ap.add_argument('--gamma-spec', type=int, choices=[0, 1], default=None,
                    help='SEDX_TUNE_GAMMA_SPEC (A/B runs): gammatone spectrum kernel (config 4)')
    ap.add_argument('--ab-package', default=None,
                    help='A/B runs: load sedx from this package directory instead of the in-tree build '
                         '(recorded in the JSON line as "library")')
    ap.add_argument('--stub', action='store_true',
                    help='CPU stand-in model (tests of the N-rank launcher and the N > 1 measurement path)')
    ap.add_argument('--stub-fail-rank', type=int, default=-1,
                    help='with --stub: this rank exits with status 3 after the process group is up (launcher test)')
    ap.add_argument('--backend', choices=['nccl', 'gloo'], default=None,
                    help='N > 1 process-group backend: nccl (= RCCL, the default with GPUs; rank r on GPU r) or '
                         'gloo (every rank on GPU 0, gathers through host copies: a rehearsal of the N-rank path '
                         'with the real model on a one-GPU box)')
    ap.add_argument('--gru-handoff', choices=['auto', 'global', 'spread', 'local'], default=None,
                    help='SEDX_TUNE_GRU_HANDOFF (A/B runs): XCD-local when placed on one XCD (auto), always the '
                         'global protocol, or the global protocol with the slices dealt over every XCD (spread), '
                         'or one XCD per (group, direction) with the XCD-local hand-off also on a pipelined '
                         'handle (local)')
    ap.add_argument('--wino-f43', type=int, choices=[0, 1, 2], default=None,
                    help='SEDX_TUNE_WINO_F43 (A/B runs): blocks 1-4 (2, the default) or 2-4 (1) as Winograd '
                         'F(4x4,3x3), or all F(2x2,3x3) (0)')
    ap.add_argument('--wino-block1', type=int, choices=[0, 1, 2], default=None,
                    help='winograd precision: block 1 as Winograd with conv1 inside the launch (2), fed by a '
                         'separate conv1 launch (1), or as the direct fused kernel (0); default: WINO_BLOCK1')
    args = ap.parse_args()

    if args.gpus > 1 and 'WORLD_SIZE' not in os.environ:
        # a plain `python bench.py --gpus N`: start the N ranks here, before
        # anything in this process touches the GPU
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    global GATHER_CPU
    backend = 'gloo' if args.stub else args.backend
    GATHER_CPU = backend == 'gloo'
    world, rank, local = distributed.init(backend)
    if world != args.gpus:
        if rank == 0:
            print('bench: --gpus %d but WORLD_SIZE %d' % (args.gpus, world), file=sys.stderr)
        sys.exit(2)
    if args.stub:
        stub_main(args, world, rank)
        return
    # gloo rehearsal: every rank on GPU 0 (each with its own libsedx handle)
    dev = torch.device('cuda', 0 if GATHER_CPU else local)
    torch.cuda.set_device(dev)
    name = MODEL_NAMES[args.model]
    global WINO_BLOCK1, WINO_F43
    if args.wino_block1 is not None:
        WINO_BLOCK1 = args.wino_block1
    if args.wino_f43 is not None:
        WINO_F43 = args.wino_f43
    model = build_model(name, dev)
    model.set_tuning(_lib.TUNE_GRU_KERNEL, GRU_KERNELS[args.gru_kernel])
    if args.wino_order is not None:
        model.set_tuning(_lib.TUNE_WINO_ORDER, args.wino_order)
    if args.gru_handoff is not None:
        model.set_tuning(_lib.TUNE_GRU_HANDOFF, {'auto': 0, 'global': 1, 'spread': 2, 'local': 3}[args.gru_handoff])
    B = args.batch
    wave = torch.from_numpy(synth.make_waveforms(B, 10.0, 16000, seed=1234 + rank)).to(dev)

    side = world == 1 and rank == 0 and not args.no_side and args.mode == 'clip'
    iso_ms = None
    if rank == 0:
        progress('headline leg (%s, %s mode, B=%d, %d steps)' % (args.precision, args.mode, B, args.steps))
    if args.mode == 'gamma':
        res = gamma_leg(args, dev, args.precision)
        if rank == 0:
            print(json.dumps(res))
        return
    if args.mode == 'clip':
        # per-stage times one batch at a time (the roofline's launch time) on
        # every rank at N > 1 too (no collective inside; rank 0's are reported)
        value, elapsed, stage_ms, p50_dev, p99_dev, iso_ms = clip_leg(model, wave, args, world, rank, dev,
                                                                     args.precision, isolated=side or world > 1)
        roof = roofline(stage_ms, B, args.precision, iso_ms=iso_ms)
    else:
        model.set_precision(args.precision)
        wl = window_leg(model, wave, args, dev, args.precision)
        value, elapsed, stage_ms, roof = wl['value'], wl['ms_per_step'] * args.steps / 1e3, None, None
        p50_dev = p99_dev = None
    # p50 from host-visible input (pinned) to the framewise output on the host
    host_wave = wave.cpu().pin_memory()
    host_out = torch.empty((B * world, 1000, 25), dtype=torch.float32).pin_memory() if rank == 0 else None
    # BASELINE config 5 at N > 1: the Transformer model through the same
    # sharded step (the driver's `bench.py --gpus N` measures both models)
    c5 = None
    if world > 1 and args.mode == 'clip' and args.model == 'gru' and not args.no_side:
        if rank == 0:
            progress('config5 (Transformer, %d ranks) leg' % world)
        trf = build_model(MODEL_NAMES['transformer'], dev)
        c5 = config5_leg(trf, wave, args, world, rank, dev, args.precision)
        del trf
    h2h = host_to_host_step(model, host_wave, host_out, dev, world, rank)
    for _ in range(3):
        h2h()
    p50, p99 = latency(h2h, B, max(5, min(args.steps, 20))) if args.mode == 'clip' else (None, None)
    # the same from int16 host input: the reference's batched clip driver
    # reads HDF5 int16 waveforms (utils/data_generator.py:20-49); the model
    # takes them as they are and dequantises on the device (half the PCIe bytes)
    p50_i16 = None
    if args.mode == 'clip' and side:
        host_i16 = (torch.clamp(wave, -1.0, 1.0) * 32767.0).to(torch.int16).cpu().pin_memory()
        h2h16 = host_to_host_step(model, host_i16, host_out, dev, world, rank)
        for _ in range(3):
            h2h16()
        p50_i16, _ = latency(h2h16, B, max(5, min(args.steps, 20)))

    extra = {}
    if side:
        extra['stage_ms_isolated'] = iso_ms
        if extra['stage_ms_isolated'].get('frontend'):
            fe = extra['stage_ms_isolated']['frontend']
            extra['frontend_roofline'] = {
                'bound': 'hbm', 'kernel': 'sedx::logmel512_kernel<false>',
                'achieved': round(B * FRONTEND_BYTES_PER_CLIP / (fe * 1e-3) / 1e9, 1), 'peak': PEAK_HBM_GBPS,
                'unit': 'GB/s', 'frac': round(B * FRONTEND_BYTES_PER_CLIP / (fe * 1e-3) / 1e9 / PEAK_HBM_GBPS, 4),
                'ms_per_batch': fe, 'bytes_per_clip': FRONTEND_BYTES_PER_CLIP,
                # the FFT's arithmetic intensity (~16 FLOP/B) is past the
                # non-packed f32 VALU ridge (78.6 TF / 8 TB/s = 9.8): the
                # VALU side, with algorithmic FLOPs (radix-2 count) per frame
                'flops_per_frame': FRONTEND_FLOPS_PER_FRAME,
                'valu_tflops': round(B * 1001 * FRONTEND_FLOPS_PER_FRAME / (fe * 1e-3) / 1e12, 2),
                'valu_peak_tflops': PEAK_VALU_F32_TF,
                'valu_frac': round(B * 1001 * FRONTEND_FLOPS_PER_FRAME / (fe * 1e-3) / 1e12 / PEAK_VALU_F32_TF, 4)}
        progress('events + latency_b1')
        extra.update(events_side(model, wave))
        extra['latency_b1'] = latency_b1(model, dev)
        if args.precision == 'winograd' and WINO_F43:
            # a handle tuned for one-clip latency: every conv on F(2x2,3x3),
            # whose items are a quarter the size, so a 1-clip grid keeps more
            # CUs busy (profiles/r05q_small_batch.log); outputs of one handle
            # never depend on the batch, so the form is a per-handle choice
            model.set_tuning(_lib.TUNE_WINO_F43, 0)
            extra['latency_b1_wino_f23'] = latency_b1(model, dev)
            model.set_tuning(_lib.TUNE_WINO_F43, int(WINO_F43))
        notes = {'x3': 'opt-in arithmetic (operands narrowed to 16 significant bits), same workload',
                 'exact': 'fp32, direct 3x3 conv everywhere (bit-reproducible reference arithmetic), same workload',
                 'winograd': dtype_of('winograd') + ', same workload'}
        for other in [p for p in ('exact', 'winograd', 'x3') if p != args.precision]:
            progress('value_%s leg' % other)
            model.set_precision(other)
            extra['latency_b1_%s' % other] = latency_b1(model, dev)
            model.set_precision(args.precision)
            v2, e2, st2, p2, _, iso2 = clip_leg(model, wave, args, 1, 0, dev, other, isolated=True)
            extra['value_%s' % other] = {'value': round(v2, 2), 'unit': 'clips/s', 'dtype': dtype_of(other),
                                         'ms_per_step': round(e2 / args.steps * 1e3, 4),
                                         'ms_per_clip_p50_device': round(p2, 4),
                                         'roofline': roofline(st2, B, other, iso_ms=iso2), 'stage_ms': st2,
                                         'note': notes[other]}
        model.set_precision(args.precision)
        cfgs = {}
        if args.model == 'gru':
            progress('config3 (Transformer) leg')
            trf = build_model(MODEL_NAMES['transformer'], dev)
            v3, e3, st3, p3, _, iso3 = clip_leg(trf, wave, args, 1, 0, dev, args.precision, isolated=True)
            cfgs['config3'] = {'workload': 'Cnn_9layers_Transformer_FrameAtt logmel 16k, %d x 10 s clips '
                                           'per step (clip mode)' % B,
                               'metric': METRICS['transformer'],
                               'value': round(v3, 2), 'unit': 'clips/s', 'dtype': dtype_of(args.precision),
                               'ms_per_step': round(e3 / args.steps * 1e3, 4),
                               'ms_per_clip_p50_device': round(p3, 4),
                               'roofline': roofline(st3, B, args.precision, iso_ms=iso3), 'stage_ms': st3}
            del trf
        progress('config4 (gammatone 32k) leg')
        cfgs['config4'] = gamma_leg(args, dev, args.precision)
        progress('window-mode leg')
        cfgs['window_mode'] = window_leg(model, wave, args, dev, args.precision)
        model.set_precision(args.precision)
        extra['configs'] = cfgs

    def run_cpu():
        progress('cpu baseline (%d threads)' % cpu_threads())
        c = cpu_baseline(name, model, dev, args.cpu_seconds, B)
        if args.mode == 'clip' and not args.no_side and world == 1:
            progress('cpu baseline, window mode')
            c['window_mode'] = cpu_baseline_window(name, min(args.cpu_seconds, 10.0))
        return c

    cpu = rank0_cpu_baseline(args, world, rank, run_cpu)

    if rank == 0:
        line = {
            'metric': METRICS[args.model], 'value': round(value, 2), 'unit': 'clips/s', 'n_gpus': world,
            'steps': args.steps, 'warmup': args.warmup,
            'ms_per_step': round(elapsed / args.steps * 1e3, 4),
            'ms_per_clip_p50': round(p50, 4) if p50 is not None else None,
            'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None,
            'dtype': dtype_of(args.precision),
            'data': 'synthetic (seeded 0.1*N(0,1) + gated tones; random-init weights)',
            'config': {'workload': '%s logmel 16k, %d x 10 s clips per GPU per step (%s mode)'
                                   % (name, B, args.mode),
                       'batch_per_gpu': B, 'global_batch': B * world, 'clip_seconds': 10,
                       'sample_rate': 16000, 'mode': args.mode, 'precision': args.precision,
                       'parallelism': 'dp%d clip-sharded, %s gather of framewise + clipwise to rank 0'
                                      % (world, 'gloo (host copies, all ranks on GPU 0)' if GATHER_CPU else 'RCCL'),
                       'backend': dist.get_backend() if world > 1 else None,
                       'world_size': dist.get_world_size() if world > 1 else 1,
                       'streams': args.streams,
                       'pipelined': args.streams > 1 and not args.no_pipeline,
                       'pipeline_mode': args.pipeline_mode if args.streams > 1 and not args.no_pipeline else 0,
                       'gru_kernel': args.gru_kernel if args.model == 'gru' else None,
                       'gru_handoff': (args.gru_handoff or 'auto') if args.model == 'gru' else None},
            'ms_per_clip_p99': round(p99, 4) if p99 is not None else None,
            'ms_per_clip_p50_note': 'per batch, one at a time, from pinned host input (H2D on a copy '
                                    'stream) to framewise in pinned host memory on rank 0',
            'ms_per_clip_p50_device': round(p50_dev, 4) if p50_dev is not None else None,
            'ms_per_clip_p50_i16_input': round(p50_i16, 4) if p50_i16 is not None else None,
            'ms_per_clip_p99_device': round(p99_dev, 4) if p99_dev is not None else None,
            'roofline': roof, 'cpu_baseline': cpu, 'stage_ms': stage_ms,
            # the libsedx.so this run loaded (--ab-package selects another build for A/B runs)
            'library': os.path.relpath(_lib.LIB_PATH, REPO), 'library_version': _lib.lib().sedx_version().decode(),
        }
        line.update(extra)
        if c5 is not None:
            line.setdefault('configs', {})['config5'] = c5
        if cpu:
            line['speedup_vs_cpu'] = round(value / cpu['value'], 1)
        print(json.dumps(line))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
