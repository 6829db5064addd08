"""libh2s under a real multi-rank launch on the GPU: two ranks (one process
each, gloo for the collectives because both share the box's one card) run
the frame-sharded flow of hdr2sdr/dist.py with the HIP library doing the
conversion, and the reduced result equals one process converting the whole
sequence, bit for bit.  The 8-GPU RCCL form is bench.py's;
tests/test_dist.py covers the same flow on CPU with the oracle."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
NF, W, H = 7, 256, 128


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


# case -> (params, frames, W, H, bits_in): the C2-shaped static case, the one
# exchange step (libplacebo peak_detect=1), and BASELINE's two 8-GPU configs at
# full frame size: C4 (4K Mobius, frame-sharded) and C5 (8K 12-bit HLG, Hable
# + 65^3, 12-bit out)
CASES = {
    'hable': (dict(tonemapper='hable', gamma=2.2), NF, W, H, 10),
    'bt2390-peak-detect': (dict(tonemapper='bt.2390', peak_detect=True, maxcll=4000.0), 6, W, H, 10),
    'C4-4k-mobius': (dict(tonemapper='mobius', gamma=1.0, bits_out=10), 4, 3840, 2160, 10),
    'C5-8k-hlg12-hable': (dict(tonemapper='hable', gamma=1.0, bits_in=12, bits_out=12, transfer='arib-std-b67'),
                          2, 7680, 4320, 12),
}


def _params(case):
    import hdr2sdr
    return hdr2sdr.TonemapParams(**CASES[case][0])


def _frames(case, a, b):
    """global frames [a, b) of the test sequence, on the host"""
    from hdr2sdr.synth import synth_frames
    from test_peak_detect import sequence
    _, _, w, h, bits = CASES[case]
    if case == 'bt2390-peak-detect':
        return np.ascontiguousarray(sequence(w, h)[a:b])
    return synth_frames('smooth', b - a, w, h, bits, device='cpu', seed=0x5EED + a).to_numpy().buf


def _worker(rank, world, port, out_dir, case):
    for p in (os.path.join(REPO, 'hdr-to-sdr_amd'), REPO, HERE):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch
    import torch.distributed as dist

    import hdr2sdr
    from hdr2sdr.dist import broadcast_setup, frame_checksum, reduce_run, shard_range, sync_peak_state

    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        params = _params(case) if rank == 0 else None
        lattice = hdr2sdr.generate_lattice(65) if rank == 0 else None
        params, lattice = broadcast_setup(params, lattice, 65)
        _, n, w, h, bits = CASES[case]
        a, b = shard_range(n, world, rank)
        tm = hdr2sdr.Tonemapper(0, params, lattice)
        shard = hdr2sdr.FrameBatch(_frames(case, a, b), w, h, bits).to_torch('cuda:0')
        if params.peak_detect:
            sync_peak_state(tm, shard, n)
        out = tm(shard)
        torch.cuda.synchronize()
        px, total, _ = reduce_run((b - a) * w * h, frame_checksum(out.buf, a), 0.0)
        np.save(os.path.join(out_dir, f'r{rank}.npy'), np.array([px, total], dtype=np.int64))
        tm.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize('case', sorted(CASES))
def test_two_ranks_on_libh2s_equal_one_process(tmp_path, case):
    import torch

    import hdr2sdr
    from hdr2sdr.dist import frame_checksum
    _, n, w, h, bits = CASES[case]
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path), case), nprocs=world, join=True,
                       start_method='spawn')
    res = [np.load(tmp_path / f'r{r}.npy') for r in range(world)]
    tm = hdr2sdr.Tonemapper(0, _params(case), hdr2sdr.generate_lattice(65))
    want = tm(hdr2sdr.FrameBatch(_frames(case, 0, n), w, h, bits).to_torch('cuda:0'))
    torch.cuda.synchronize()
    cks = frame_checksum(want.buf, 0)
    tm.close()
    for r in res:
        assert int(r[0]) == n * w * h       # SUM of pixels over ranks
        assert int(r[1]) == cks             # SUM of shard checksums == the one-process checksum


_RCCL_CHILD = r'''
import os, sys
sys.path[:0] = [os.path.join(REPO, 'hdr-to-sdr_amd'), REPO]
import numpy as np, torch, torch.distributed as dist
import hdr2sdr
from hdr2sdr.dist import broadcast_setup, reduce_run, gather_peak_stats
dev = torch.device('cuda', 0)
torch.cuda.set_device(dev)
dist.init_process_group('nccl', device_id=dev)
assert dist.get_backend() == 'nccl'
p = hdr2sdr.TonemapParams(tonemapper='mobius', gamma=1.0, bits_out=10)
lat = hdr2sdr.generate_lattice(17)
p2, lat2 = broadcast_setup(p, lat, 17, dev)
assert p2 == p and np.array_equal(lat2, lat)
px, cks, el = reduce_run(123, 456, 0.25, dev)
assert (px, cks, el) == (123, 456, 0.25)
st = gather_peak_stats(np.array([1.0, 2.0]), np.array([0.5, 0.25]), 2, dev)
assert np.array_equal(st, [[1.0, 0.5], [2.0, 0.25]])
dist.barrier()
dist.destroy_process_group()
print('RCCL OK')
'''


@pytest.mark.gpu
def test_rccl_collectives_world1():
    """The nccl (= RCCL) backend through hdr2sdr/dist.py's collectives with
    device tensors (bench.py's N > 1 path: params + lattice broadcast, the
    SUM / MAX reduction, the peak-statistics all-gather) in a world of one
    rank on the box's one card; only the driver's 8-GPU run has more ranks."""
    import subprocess
    env = dict(os.environ, MASTER_ADDR='127.0.0.1', MASTER_PORT=str(_free_port()), RANK='0', WORLD_SIZE='1',
               LOCAL_RANK='0')
    r = subprocess.run([sys.executable, '-c', 'REPO=%r\n' % REPO + _RCCL_CHILD], env=env, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0 and 'RCCL OK' in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])
