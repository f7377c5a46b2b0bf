"""Benchmark of the MI355X-native SED inference path (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--model gru|transformer]
                    [--mode clip|window] [--batch 32] [--precision x3|exact]
                    [--no-cpu-baseline] [--no-exact]

One step = one forward of the hot path over one batch of synthetic 10 s @
16 kHz clips per GPU (clip mode = main_strong inference_prob semantics, B=32
per GPU: BASELINE.json configs[1]), inputs already resident in HBM, weights
random-init with the reference architecture.  For N > 1 (launched by
torch.distributed.run, one process per GPU) every rank runs its own shard of
clips (weak scaling) and the framewise outputs are gathered to rank 0 over
RCCL inside each step — the path's only collective.  Rank 0 prints ONE JSON
line.  The headline uses the default conv arithmetic (3xbf16-split MFMA, fp32
accumulate); the exact fp32-MFMA mode is timed beside it (value_exact_fp32).
"""
import argparse
import ctypes
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
# SEDX_PKG: an alternative build of the package (A/B runs of kernel variants)
for _p in (REPO, os.environ.get('SEDX_PKG') or os.path.join(REPO, 'sound-event-detection_amd')):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from sedx import _lib, distributed, inference, models, synth  # noqa: E402

METRIC = '10s@16kHz clips/sec (whole node) + ms/clip p50, Cnn_9_Gru_FrameAtt logmel'
# MI355X_MICROARCH.md: FP32 matrix peak 157.3 TF; BF16 dense MFMA ~2.5 PF.  The
# x3 scheme issues 3 bf16 MFMAs per useful MAC, so its arithmetic peak is 2.5/3 PF.
PEAK_TF = {'exact': 157.3, 'x3': 2500.0 / 3}
MODEL_NAMES = {'gru': 'Cnn_9layers_Gru_FrameAtt', 'transformer': 'Cnn_9layers_Transformer_FrameAtt'}
# conv stages of sedx_stage_times: (F, Cin, Cout, number of 2x poolings before it)
CONV_STAGES = {'b1c2': (64, 64, 64, 0), 'b2c1': (32, 64, 128, 1), 'b2c2': (32, 128, 128, 1),
               'b3c1': (16, 128, 256, 2), 'b3c2': (16, 256, 256, 2), 'b4c1': (8, 256, 512, 3),
               'b4c2': (8, 512, 512, 3)}


def conv_flops(stage, B, T):
    F, cin, cout, npool = CONV_STAGES[stage]
    for _ in range(npool):
        T //= 2
    return 2.0 * B * T * F * cout * 9 * cin


def build_model(name, device):
    m = getattr(models, name)(16000, 512, 160, 64, 25, 7000, 25, 'logmel')
    sd = m.state_dict()
    for k, v in synth.make_state_dict(name, seed=0).items():
        sd[k] = torch.from_numpy(v)
    m.load_state_dict(sd)
    return m.to(device).eval()


def cpu_baseline(name, seconds, model=None, dev=None):
    """Oracle (CPU restatement, torch fp32, reference op sequence) on a bounded
    sample: B=4 clips of 10 s per iteration, repeated for ~``seconds``.  With
    ``model`` the same 4 clips also go through the GPU path and the oracle's
    output is the checker: max |d framewise| is reported beside the rate."""
    from oracle import sed_oracle as O
    sd = O.full_state(synth.make_state_dict(name, seed=0), '16k')
    wave = synth.make_waveforms(4, seconds=10.0, sample_rate=16000, seed=7)
    O.forward(sd, name, wave=wave[:1])  # warm-up
    n, t0 = 0, time.perf_counter()
    while True:
        ref = O.forward(sd, name, wave=wave)
        n += 4
        el = time.perf_counter() - t0
        if el >= seconds or n >= 400:
            break
    out = {'value': n / el, 'unit': 'clips/s', 'cores': torch.get_num_threads(), 'kind': 'port',
           'sample': '%d x 10 s clips (B=4 per iteration, %.1f s) through oracle/sed_oracle.py '
                     'forward on the host CPU' % (n, el)}
    if model is not None:
        with torch.no_grad():
            fw = model(torch.from_numpy(wave).to(dev))['framewise_output'].cpu().numpy()
        out['parity_max_abs_framewise'] = float(np.max(np.abs(fw - ref['framewise_output'].numpy())))
        out['parity_tolerance'] = 1e-3
    return out


def latency_b1(model, dev, reps=20):
    """End-to-end latency of ONE 10 s clip: clip mode and
    window mode (its 6 windows in one launch), input already on the device;
    and clip mode from a host buffer to the framewise output back on the
    host (PCIe-inclusive)."""
    w1 = torch.from_numpy(synth.make_waveforms(1, seconds=10.0, sample_rate=16000, seed=11))
    wd = w1.to(dev)
    out = {}
    for key, fn in (('clip', lambda: model(wd)['framewise_output']),
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
    return out


def measure(model, wave, args, world, rank, dev):
    """Throughput over K steps with ``args.streams`` batches in flight: step i
    is issued on stream i % streams (a serving loop with that many concurrent
    requests), so one batch's GRU recurrence — 16 CUs for ~0.5 ms — overlaps
    the next batch's conv stack.  Every step is a complete forward of its own
    batch.  Latency (p50/p99 ms per clip) is then taken one step at a time on
    a single stream."""
    B = wave.shape[0]
    streams = [torch.cuda.Stream(dev) for _ in range(max(1, args.streams))]
    # conv stacks in issue order (sedx_set_pipelined): without it the batches
    # in flight can fall into lockstep, two conv stacks splitting the chip and
    # the GRUs running side by side on 32 CUs (measured: ~10 % slower runs)
    model.set_pipelined(len(streams) > 1 and not args.no_pipeline)

    def step(st=None):
        with torch.no_grad(), torch.cuda.stream(st or torch.cuda.current_stream(dev)):
            if args.mode == 'clip':
                fw = model(wave)['framewise_output']
            else:
                fw = inference.predict_windows(model, wave, 5, 1)
            if world > 1:
                distributed.gather_to_rank0(fw, world, rank)
        return fw

    torch.cuda.synchronize()
    for i in range(args.warmup):
        step(streams[i % len(streams)])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    # per-stage HIP events over the timed region: libsedx records them on the
    # stream each forward's kernels are launched on, one event set per
    # forward (accumulate mode), averaged by sedx_stage_times afterwards
    nat, L = model.native(dev), _lib.lib()
    _lib.check(L.sedx_set_profiling(nat.h, 2), nat.h, 'set_profiling')
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(streams[i % len(streams)])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ms = (ctypes.c_float * len(_lib.STAGES))()
    n = ctypes.c_int32()
    _lib.check(L.sedx_stage_times(nat.h, ms, len(_lib.STAGES), ctypes.byref(n)), nat.h, 'stage_times')
    _lib.check(L.sedx_set_profiling(nat.h, 0), nat.h, 'set_profiling')
    timed_stage_ms = {s_: round(float(v), 4) for s_, v in zip(_lib.STAGES, ms[:])}
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    value = world * B * args.steps / elapsed
    model.set_pipelined(False)
    lat = []
    for _ in range(max(5, min(args.steps, 20))):
        torch.cuda.synchronize()
        a = time.perf_counter()
        step()
        torch.cuda.synchronize()
        lat.append((time.perf_counter() - a) * 1e3 / B)
    lat.sort()
    return value, elapsed, statistics.median(lat), lat[min(len(lat) - 1, int(0.99 * len(lat)))], timed_stage_ms


def stage_times(model, wave, dev, reps):
    """Per-stage device time: HIP events recorded by libsedx on the stream the
    kernels are launched on (sedx_set_profiling / sedx_stage_times)."""
    nat = model.native(dev)
    L = _lib.lib()
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


# HBM traffic per launch comes from the rocprofv3 PMC passes of this bench
# command (tools/profile_round.sh -> tools/pmc_summary.py; FETCH_SIZE x2 per
# the gfx950 correction + WRITE_SIZE), committed under profiles/.
PROFILE_SUMMARY = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'profiles',
                               'r01j_kernel_summary.json')
STAGE_KERNEL = {'b1c2': '<64, 64, 1', 'b2c1': '<32, 128, 0', 'b2c2': '<32, 128, 1',
                'b3c1': '<16, 128, 0', 'b3c2': '<16, 128, 1', 'b4c1': '<8, 128, 0',
                'b4c2': '<8, 128, 2'}
# x3 kernels carry a 4th template argument (FUSE: block 1's conv1 fused into b1c2)
STAGE_FUSE = {'b1c2': 'true'}


def profiled(kernel):
    """(HBM bytes per launch, rocprofv3 average duration in ms, MFMA busy
    fraction, effective clock GHz) of ``kernel`` from the committed profile
    summary (None where absent)."""
    try:
        with open(PROFILE_SUMMARY) as f:
            v = json.load(f).get(kernel, {})
        ns = v.get('avg_ns')
        util, clk = v.get('mfma_util'), v.get('clock_ghz')
        return (v.get('hbm_bytes_corrected'), (round(ns * 1e-6, 4) if ns else None),
                round(util, 4) if util else None, round(clk, 3) if clk else None)
    except (OSError, ValueError):
        return None, None, None, None


def roofline(stage_ms, B, precision):
    T = 160000 // 160 + 1
    conv = {s: stage_ms[s] for s in CONV_STAGES}
    dom = max(conv, key=conv.get)
    flops = conv_flops(dom, B, T)
    if precision == 'x3' and dom == 'b1c2':
        # the fused block-1 launch also computes conv1 (Cin 1 -> 64, 9 taps) for
        # every conv2 input pixel it stages: 2 * B * T * 64 * 64 * 9 flops
        flops += 2.0 * B * T * 64 * 64 * 9
    achieved = flops / (conv[dom] * 1e-3) / 1e12
    peak = PEAK_TF[precision]
    total = sum(conv_flops(s, B, T) for s in CONV_STAGES)
    if precision == 'x3':
        kname = 'sedx::conv3x3_x3_kernel%s, %s>' % (STAGE_KERNEL[dom], STAGE_FUSE.get(dom, 'false'))
    else:
        kname = 'sedx::conv3x3_kernel%s>' % STAGE_KERNEL[dom]
    traffic, rocprof_ms, mfma_util, clock = profiled(kname) if B == 32 else (None, None, None, None)
    return {'bound': 'mfma',
            'kernel': 'conv3x3_%s (%s)' % ('x3_kernel' if precision == 'x3' else 'kernel', dom),
            'arith': '3xbf16-split MFMA 32x32x16, fp32 acc (peak = bf16 dense 2.5 PF / 3)'
                     if precision == 'x3' else 'fp32 MFMA 32x32x2',
            'achieved': round(achieved, 2), 'peak': round(peak, 1), 'unit': 'TFLOP/s',
            'frac': round(achieved / peak, 4),
            'traffic': traffic, 'traffic_unit': 'bytes/launch (HBM, rocprofv3 PMC)',
            'traffic_source': os.path.relpath(PROFILE_SUMMARY, os.path.dirname(os.path.abspath(__file__)))
            if traffic is not None else None,
            'flops_per_launch': flops, 'avg_launch_ms': conv[dom],
            'avg_launch_ms_rocprof': rocprof_ms,
            'mfma_busy_frac_pmc': mfma_util, 'clock_ghz_pmc': clock,
            'timing': 'avg_launch_ms: HIP events on the launch stream over the timed region '
                      '(one event set per forward, all steps averaged); '
                      'avg_launch_ms_rocprof: rocprofv3 --kernel-trace --stats of this bench '
                      '(--streams 1 --no-side), committed summary',
            'conv_stack_tflops': round(total / (sum(conv.values()) * 1e-3) / 1e12, 2)}


FRONTEND_BYTES_PER_CLIP = 160000 * 4 + 1001 * 64 * 4   # waveform in + X0 out


def side_measurements(model, wave, args, dev, stage_ms):
    """Secondary numbers on rank 0 (not the headline): the frontend's achieved
    HBM rate, GPU event extraction for the batch, and window mode (predict.py
    semantics: 6 x 5 s windows per 10 s clip, merged + averaged)."""
    B = wave.shape[0]
    out = {}
    if stage_ms and stage_ms.get('frontend'):
        out['frontend_gbps'] = round(B * FRONTEND_BYTES_PER_CLIP / (stage_ms['frontend'] * 1e-3) / 1e9, 1)
    with torch.no_grad():
        fw = model(wave)['framewise_output']
    params = dict(inference.DEFAULT_PREDICT_PARAMS)
    inference.event_pairs(fw, params)
    torch.cuda.synchronize()
    reps = 10
    t0 = time.perf_counter()
    for _ in range(reps):
        n_ev = len(inference.event_pairs(fw, params))
    out['events_ms_per_batch'] = round((time.perf_counter() - t0) / reps * 1e3, 4)
    out['events_per_batch'] = n_ev
    with torch.no_grad():
        for _ in range(2):
            inference.predict_windows(model, wave, 5, 1)
        torch.cuda.synchronize()
        reps = max(3, min(args.steps, 10))
        t0 = time.perf_counter()
        for _ in range(reps):
            inference.predict_windows(model, wave, 5, 1)
        torch.cuda.synchronize()
    el = time.perf_counter() - t0
    out['value_window_mode'] = {'value': round(B * reps / el, 2), 'unit': 'clips/s',
                                'windows_per_clip': 6, 'note': '5 s windows, 1 s stride, merged + '
                                                             'avg_merge on the GPU (predict.py:297-349)'}
    return out


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
    ap.add_argument('--model', choices=list(MODEL_NAMES), default='gru')
    ap.add_argument('--mode', choices=['clip', 'window'], default='clip')
    ap.add_argument('--precision', choices=list(PEAK_TF), default='x3')
    ap.add_argument('--no-exact', action='store_true', help='skip timing the exact fp32 mode')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-side', action='store_true',
                    help='skip the side measurements (events, window mode): profiling passes use it so '
                         'that per-kernel rocprof averages cover only the headline launches')
    ap.add_argument('--cpu-seconds', type=float, default=15.0)
    args = ap.parse_args()

    world, rank, local = distributed.init()
    if world != args.gpus and rank == 0:
        print('warning: --gpus %d but WORLD_SIZE %d' % (args.gpus, world), file=sys.stderr)
    dev = torch.device('cuda', local)
    torch.cuda.set_device(dev)
    name = MODEL_NAMES[args.model]
    model = build_model(name, dev).set_precision(args.precision)
    B = args.batch
    wave = torch.from_numpy(synth.make_waveforms(B, 10.0, 16000, seed=1234 + rank)).to(dev)

    value, elapsed, p50, p99, stage_ms = measure(model, wave, args, world, rank, dev)
    roof = stage_iso = None
    if args.mode == 'clip':
        roof = roofline(stage_ms, B, args.precision)
        stage_iso = stage_times(model, wave, dev, max(3, min(args.steps, 10)))
    exact = None
    if not args.no_exact and args.precision != 'exact':
        model.set_precision('exact')
        ev, _, ep50, _, est = measure(model, wave, args, world, rank, dev)
        exact = {'value': round(ev, 2), 'ms_per_clip_p50': round(ep50, 4)}
        if args.mode == 'clip':
            exact['roofline'] = roofline(est, B, 'exact')
        model.set_precision(args.precision)

    extra = {}
    if args.mode == 'clip' and rank == 0 and not args.no_side:
        extra = side_measurements(model, wave, args, dev, stage_iso)
        extra['latency_b1'] = latency_b1(model, dev)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(name, args.cpu_seconds, model, dev)

    if rank == 0:
        line = {
            'metric': METRIC, 'value': round(value, 2), 'unit': 'clips/s', 'n_gpus': world,
            'steps': args.steps, 'warmup': args.warmup,
            'ms_per_step': round(elapsed / args.steps * 1e3, 4), 'ms_per_clip_p50': round(p50, 4),
            'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None,
            'dtype': 'f32' if args.precision == 'exact' else 'f32 (conv: 3xbf16-split MFMA, f32 accumulate)',
            'data': 'synthetic (seeded 0.1*N(0,1) + gated tones; random-init weights)',
            'config': {'workload': '%s logmel 16k, %d x 10 s clips per GPU per step (%s mode)'
                                   % (name, B, args.mode),
                       'batch_per_gpu': B, 'global_batch': B * world, 'clip_seconds': 10,
                       'sample_rate': 16000, 'mode': args.mode, 'precision': args.precision,
                       'parallelism': 'dp%d clip-sharded, RCCL gather of framewise' % world,
                       'streams': args.streams,
                       'pipelined': args.streams > 1 and not args.no_pipeline},
            'ms_per_clip_p99': round(p99, 4),
            'roofline': roof, 'cpu_baseline': cpu, 'stage_ms': stage_ms,
            'stage_ms_isolated': stage_iso,
            'value_exact_fp32': exact,
        }
        line.update(extra)
        if cpu:
            line['speedup_vs_cpu'] = round(value / cpu['value'], 1)
        print(json.dumps(line))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
