"""Multi-rank logic on CPU with the gloo backend (world size 2, 3 and 8): clip
sharding covers every clip exactly once and the rank-0 gather of per-rank
framewise outputs reproduces the single-process result in clip order.
World 8 runs BASELINE config 5's geometry (256 clips, 32 per rank, framewise
[32, 1000, 25] + clipwise [32, 25] per rank).  The
per-rank compute here is the CPU oracle (no GPU in this container); on the
GPU box the same code path runs libsedx + RCCL (bench.py --gpus N)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import sed_oracle as O
from sedx import distributed, synth

MT = 'Cnn_9layers_Gru_FrameAtt'


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_clips, out_q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    w, r, _ = distributed.init(backend='gloo')
    assert (w, r) == (world, rank)
    lo, hi = distributed.shard_range(n_clips, rank, world)
    wave = synth.make_waveforms(n_clips, seconds=1.0, sample_rate=16000, seed=21)[lo:hi]
    sd = O.full_state(synth.make_state_dict(MT, seed=0), '16k')
    fw = O.forward(sd, MT, wave=wave)['framewise_output'].contiguous()
    full = distributed.gather_ragged_to_rank0(fw, world, rank)
    if rank == 0:
        out_q.put(full.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize('world,n_clips', [(2, 4), (3, 5)])
def test_gather_matches_single_process(world, n_clips):
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_clips, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    wave = synth.make_waveforms(n_clips, seconds=1.0, sample_rate=16000, seed=21)
    ref = O.forward(O.full_state(synth.make_state_dict(MT, seed=0), '16k'), MT, wave=wave)
    np.testing.assert_allclose(got, ref['framewise_output'].numpy(), rtol=0, atol=1e-6)


def test_shard_range_partitions():
    for n in range(0, 40):
        for world in (1, 2, 3, 8):
            spans = [distributed.shard_range(n, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            for (a, b), (c, d) in zip(spans, spans[1:]):
                assert b == c and b >= a
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1


def _expected(n_clips, frames=1000, classes=25):
    """Deterministic per-clip stand-ins for the model outputs (the compute is
    covered by the parity tests; this checks placement through the gather)."""
    c = np.arange(n_clips, dtype=np.float32)[:, None, None]
    t = np.arange(frames, dtype=np.float32)[None, :, None]
    k = np.arange(classes, dtype=np.float32)[None, None, :]
    fw = np.sin(0.37 * c + 0.011 * t + 0.7 * k).astype(np.float32)
    clip = fw.max(axis=1)
    return fw, clip


def _worker_geometry(rank, world, port, n_clips, out_q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    w, r, _ = distributed.init(backend='gloo')
    assert (w, r) == (world, rank)
    lo, hi = distributed.shard_range(n_clips, rank, world)
    fw, clip = _expected(n_clips)
    fw_r, clip_r = torch.from_numpy(fw[lo:hi].copy()), torch.from_numpy(clip[lo:hi].copy())
    full_fw = full_clip = None
    if n_clips % world == 0:
        full_fw = distributed.gather_to_rank0(fw_r, world, rank)
        full_clip = distributed.gather_to_rank0(clip_r, world, rank)
    ragged_fw = distributed.gather_ragged_to_rank0(fw_r, world, rank)
    if rank == 0:
        out_q.put((None if full_fw is None else full_fw.numpy(),
                   None if full_clip is None else full_clip.numpy(), ragged_fw.numpy()))
    else:
        assert full_fw is None and full_clip is None and ragged_fw is None
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize('world,n_clips', [(8, 256), (8, 250)])
def test_world8_config5_gather(world, n_clips):
    """8 ranks, 256 clips (32 per rank) and a ragged 250 (31-32 per rank):
    rank 0 receives every rank's framewise [32, 1000, 25] and clipwise
    [32, 25] in clip order, through the equal-shard gather (the bench's path)
    and the ragged one."""
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_geometry, args=(r, world, port, n_clips, q)) for r in range(world)]
    for p in procs:
        p.start()
    fw, clip, ragged = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    exp_fw, exp_clip = _expected(n_clips)
    assert np.array_equal(ragged, exp_fw)
    if n_clips % world == 0:
        assert np.array_equal(fw, exp_fw) and np.array_equal(clip, exp_clip)
