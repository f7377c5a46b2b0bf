"""bench.py host logic (no GPU): the algorithmic FLOP counts behind
roofline.achieved (26.03 GFLOP of conv per 10 s clip) and
the roofline record built from per-stage times."""
import importlib.util
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope='module')
def bench():
    spec = importlib.util.spec_from_file_location('bench_mod', os.path.join(REPO, 'bench.py'))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_conv_flops_per_clip(bench):
    T = 160000 // 160 + 1
    per_clip = sum(bench.conv_flops(s, 1, T) for s in bench.CONV_STAGES)
    # the seven implicit-GEMM convs; SURVEY §8(a) a7's 26.03 GF also holds
    # block 1's conv1 (Cin 1, 0.07 GF), hence the 1 % band
    assert abs(bench.conv_flops('b2c2', 1, T) - 2 * 500 * 32 * 128 * 9 * 128) < 1
    assert abs(bench.conv_flops('b4c2', 1, T) - 2 * 125 * 8 * 512 * 9 * 512) < 1
    assert abs(per_clip - 26.03e9) / 26.03e9 < 0.01


def test_roofline_record(bench):
    stage = {s: 0.2 for s in bench.CONV_STAGES}
    stage['b1c2'] = 0.4
    r = bench.roofline(stage, 32, 'x3')
    assert r['bound'] == 'mfma' and r['unit'] == 'TFLOP/s'
    assert r['kernel'].endswith('(b1c2)')
    T = 1001
    flops = bench.conv_flops('b1c2', 32, T) + 2.0 * 32 * T * 64 * 64 * 9
    assert r['flops_per_launch'] == flops
    assert abs(r['achieved'] - flops / 0.4e-3 / 1e12) < 0.01
    assert abs(r['frac'] - r['achieved'] / r['peak']) < 1e-3
    assert r['peak'] == round(2500.0 / 3, 1)
    e = bench.roofline(stage, 32, 'exact')
    assert e['peak'] == 157.3 and 'fp32' in e['arith']


def test_roofline_exact_unfused_and_names(bench):
    stage = {s: 0.2 for s in bench.CONV_STAGES}
    stage['b1c2'] = 1.0
    e = bench.roofline(stage, 32, 'exact')
    fused = bench.fused_block1('exact')
    flops = bench.conv_flops('b1c2', 32, 1001) + (2.0 * 32 * 1001 * 64 * 64 * 9 if fused else 0.0)
    assert e['flops_per_launch'] == flops
    assert e['kernel'].startswith(bench.conv_kernel_name('b1c2', 'exact'))
    assert bench.conv_kernel_name('b4c2', 'x3') == 'sedx::conv3x3_x3_kernel<8, 128, 2, false>'


def test_cpu_info(bench):
    info = bench.cpu_info()
    assert info['host_logical_cpus'] >= 1
    assert 'cpu_model' in info


def test_roofline_winograd_block1(bench):
    """Winograd mode: b1c2 is a Winograd launch — by default (--wino-f43 2)
    the F(4x4,3x3) conv2 (36/144 of the direct conv2) fed by its own b1c1
    conv1 launch in the chunk-of-4 layout; with --wino-f43 1 the F(2x2,3x3)
    launch (16/36) with conv1 computed inside it on the VALU (--wino-block1
    2: not priced on the matrix pipe) or fed by its own launch (1); with
    --wino-block1 0 the direct fused launch."""
    stage = {s: 0.2 for s in bench.CONV_STAGES}
    stage['b1c2'] = 1.0
    stage['b1c1'] = 0.1
    assert bench.WINO_BLOCK1 == 2 and bench.WINO_F43 == 2
    w = bench.roofline(stage, 32, 'winograd')
    assert w['kernel'] == 'sedx::conv3x3_wino43_kernel<64, 1, true, 4, 2> (b1c2)'
    assert w['flops_per_launch'] == bench.conv_flops('b1c2', 32, 1001) * 36.0 / 144.0
    try:
        bench.WINO_F43 = 1
        w = bench.roofline(stage, 32, 'winograd')
        assert w['kernel'] == 'sedx::wino_block1_kernel<2, true> (b1c2)'
        assert w['flops_per_launch'] == bench.conv_flops('b1c2', 32, 1001) * 16.0 / 36.0
        bench.WINO_BLOCK1 = 1
        w = bench.roofline(stage, 32, 'winograd')
        assert w['kernel'] == 'sedx::conv3x3_wino_kernel<64, 1, 2, 2> (b1c2)'
        assert w['flops_per_launch'] == bench.conv_flops('b1c2', 32, 1001) * 16.0 / 36.0
        bench.WINO_BLOCK1 = 0
        d = bench.roofline(stage, 32, 'winograd')
        assert d['kernel'].startswith('sedx::conv3x3_kernel<64, 64, 1, true')
        assert d['flops_per_launch'] == bench.conv_flops('b1c2', 32, 1001) + 2.0 * 32 * 1001 * 64 * 64 * 9
        bench.WINO_F43 = 2
        bench.WINO_BLOCK1 = 1
        w = bench.roofline(stage, 32, 'winograd')
        assert w['kernel'] == 'sedx::conv3x3_wino43_kernel<64, 1, false, 4, 2> (b1c2)'
    finally:
        bench.WINO_BLOCK1 = 2
        bench.WINO_F43 = 2


def test_roofline_winograd_f43(bench):
    """Blocks 1-4 as Winograd F(4x4,3x3) (the default): their launches are
    conv3x3_wino43_kernel<F, EPI> and execute 36/144 of the direct conv's
    multiplies; --wino-f43 1 keeps block 1 on F(2x2,3x3); with --wino-f43 0
    every layer is an F(2x2,3x3) kernel (16/36)."""
    stage = {s: 0.1 for s in bench.CONV_STAGES}
    stage['b4c2'] = 1.0
    assert bench.WINO_F43 == 2
    w = bench.roofline(stage, 32, 'winograd')
    assert w['kernel'] == 'sedx::conv3x3_wino43_kernel<8, 2, true, 4, 2> (b4c2)'
    assert w['flops_per_launch'] == bench.conv_flops('b4c2', 32, 1001) * 36.0 / 144.0
    assert 'b1c2 F(4x4,3x3)' in w['arith'] and 'F(2x2,3x3)' not in w['arith']
    assert bench.conv_kernel_name('b2c2', 'winograd') == 'sedx::conv3x3_wino43_kernel<32, 1, true, 4, 2>'
    assert bench.conv_kernel_name('b1c2', 'winograd') == 'sedx::conv3x3_wino43_kernel<64, 1, true, 4, 2>'
    try:
        bench.WINO_F43 = 1
        w = bench.roofline(stage, 32, 'winograd')
        assert 'b1c2 F(2x2,3x3)' in w['arith']
        assert bench.conv_kernel_name('b1c2', 'winograd') == 'sedx::wino_block1_kernel<2, true>'
        bench.WINO_F43 = 0
        w = bench.roofline(stage, 32, 'winograd')
        assert w['kernel'] == 'sedx::conv3x3_wino_kernel<8, 2, 2, 2> (b4c2)'
        assert w['flops_per_launch'] == bench.conv_flops('b4c2', 32, 1001) * 16.0 / 36.0
    finally:
        bench.WINO_F43 = 2


def test_roofline_fracs_are_fractions(bench):
    """The launch time behind ``frac`` is the isolated HIP-event time when the
    run measured it; every ``frac*`` field is executed FLOPs over the matrix
    peak (<= 1 for any launch time the hardware can reach), and the Winograd
    layers' direct-conv equivalent is a rate, not a fraction."""
    T = 1001
    stage = {s: 0.3 for s in bench.CONV_STAGES}
    # fastest physically possible b1c2: executed FLOPs at exactly the peak
    ex = bench.conv_flops('b1c2', 32, T) * 16.0 / 36.0
    t_peak = ex / 157.3e12 * 1e3
    stage['b1c2'] = t_peak * 1.3
    iso = dict(stage, b1c2=t_peak * 1.05)
    w = bench.roofline(stage, 32, 'winograd', iso_ms=iso)
    assert w['avg_launch_ms'] == round(iso['b1c2'], 4) and 'one batch at a time' in w['timing']
    assert w['avg_launch_ms_timed_region'] == stage['b1c2']
    for k, v in w.items():
        if k.startswith('frac') and v is not None:
            assert 0 < v <= 1.0, (k, v)
    assert w['direct_conv_equiv_tflops'] > w['peak']      # Winograd: more than a direct conv could do
    assert not any(k.endswith('_algorithmic') for k in w)
    t = bench.roofline(stage, 32, 'winograd')              # no isolated pass: the timed region
    assert t['avg_launch_ms'] == round(stage['b1c2'], 4)


def _bench_env():
    env = dict(os.environ)
    for k in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'MASTER_ADDR', 'MASTER_PORT', 'LOCAL_WORLD_SIZE'):
        env.pop(k, None)
    env['OMP_NUM_THREADS'] = '1'
    return env


@pytest.mark.parametrize('n', [2, 8])
def test_bench_launches_n_ranks(n):
    """`python bench.py --gpus N` with no torchrun around it starts N ranks
    itself (the driver's BENCH form): each child gets RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_ADDR, the N > 1 measurement path runs (gather of the
    framewise output to rank 0 every step, barrier, all_reduce(MAX) of the
    elapsed time; gloo and a CPU stand-in model here), and exactly one JSON
    line comes back, with n_gpus = N."""
    B, steps = 4, 3
    r = subprocess.run([sys.executable, os.path.join(REPO, 'bench.py'), '--gpus', str(n), '--stub', '--steps',
                        str(steps), '--warmup', '1', '--batch', str(B), '--streams', '1'],
                       capture_output=True, text=True, timeout=600, cwd=REPO, env=_bench_env())
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d['n_gpus'] == n and d['stub'] and d['steps'] == steps
    assert sorted(int(e['RANK']) for e in d['rank_env']) == list(range(n))
    for e in d['rank_env']:
        assert e['WORLD_SIZE'] == str(n) and e['LOCAL_RANK'] == e['RANK'] and e['MASTER_ADDR'] == '127.0.0.1'
    # whole-job clips/s over all ranks from the max-over-ranks elapsed time
    assert abs(d['value'] - n * B * steps / (d['ms_per_step'] * steps / 1e3)) <= 0.01 * d['value'] + 1e-3
    # the config-5 leg (BASELINE configs[5]: the Transformer model at N GPUs)
    # runs through the same sharded step, framewise + clipwise gathered
    c5 = d['configs']['config5']
    assert c5['n_gpus'] == n and c5['global_batch'] == n * B and c5['batch_per_gpu'] == B
    assert c5['backend'] == 'gloo' and 'clipwise' in c5['gathered']
    assert 'Transformer' in c5['metric'] and c5['scaling'] == 'weak'
    assert abs(c5['value'] - n * B * steps / (c5['ms_per_step'] * steps / 1e3)) <= 0.01 * c5['value'] + 1e-3
    # the N > 1 line is complete: rank 0 times the CPU baseline after the
    # timed legs (the other ranks wait at the closing barrier), and the
    # process group's world size is recorded
    cpu = d['cpu_baseline']
    assert cpu is not None and cpu['value'] > 0 and cpu['unit'] == 'clips/s' and cpu['kind'] == 'port'
    assert cpu['cores'] >= 1 and cpu['sample']
    assert d['config']['world_size'] == n


def test_bench_launcher_fails_when_a_rank_fails():
    """A failing rank makes the launcher stop the other ranks (they would wait
    at the next collective) and exit non-zero, with no JSON line."""
    r = subprocess.run([sys.executable, os.path.join(REPO, 'bench.py'), '--gpus', '3', '--stub', '--steps', '2',
                        '--warmup', '1', '--batch', '2', '--streams', '1', '--stub-fail-rank', '1'],
                       capture_output=True, text=True, timeout=300, cwd=REPO, env=_bench_env())
    assert r.returncode != 0
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith('{')]


def test_config4_profile_fields(bench):
    """Config 4 (gammatone 32k, T = 994 frames) reads its own committed
    profile: the conv roofline's HBM traffic and the gamma frontend's bytes
    and rocprof time per batch are filled (round 3 left them null because
    only the (32, 1001) shapes were looked up)."""
    stage = {s: 0.2 for s in bench.CONV_STAGES}
    stage['b1c2'] = 1.0
    r = bench.roofline(stage, 32, 'winograd', T=994, summary=bench.GAMMA_PROFILE_SUMMARY)
    assert r['traffic'] is not None and r['traffic'] > 0
    assert r['traffic_source'].endswith('config4_kernel_summary.json')
    traffic, ms = bench.gamma_profile(32)
    assert traffic is not None and traffic > 49e6 and ms is not None and 0.0 < ms < 1.0
    assert bench.gamma_profile(8) == (None, None)


def test_dtype_strings(bench):
    """Every precision's dtype string: the arithmetic, and for winograd which
    layers run which Winograd form under the current knobs."""
    assert bench.dtype_of('exact') == 'f32'
    assert bench.dtype_of('x3').startswith('bf16x3')
    w = bench.dtype_of('winograd')
    assert 'block 1 as Winograd F(4x4,3x3)' in w and 'blocks 2-4 as Winograd F(4x4,3x3)' in w
    try:
        bench.WINO_F43 = 1
        assert 'block 1 as Winograd F(2x2,3x3)' in bench.dtype_of('winograd')
    finally:
        bench.WINO_F43 = 2
