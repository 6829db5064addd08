"""Benchmark: Mpixel/s HDR10 -> SDR on 4K frames at N GPUs, % of HBM roofline.

BASELINE.json metric "Mpixel/s HDR10->SDR (4K frames) at 1/2/4/8 GPUs; % HBM
roofline", measured on its configs[1] (C2): 3840x2160 PQ HDR10
yuv420p10le, Hable + tetrahedral 65^3 LUT + eq gamma, 10-bit output.

One step = one h2s_process launch over a batch of --frames device-resident
synthetic frames per rank.  Ranks shard frames (frame-parallel, no data-path
collective: weak scaling); the only collectives are the RCCL broadcast of the
LUT lattice at start-up and a MAX all-reduce of the elapsed time.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--frames B]
For N > 1 the driver launches one process per GPU with torch.distributed.run.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, 'hdr-to-sdr_amd'))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)


def parse_args():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--frames', type=int, default=16, help='frames per rank per step')
    ap.add_argument('--width', type=int, default=3840)
    ap.add_argument('--height', type=int, default=2160)
    ap.add_argument('--kind', default='smooth', help='synthetic content (smooth|uniform|ramp|edges)')
    ap.add_argument('--tonemapper', default='hable')
    ap.add_argument('--gamma', type=float, default=2.2)
    ap.add_argument('--bits-in', type=int, default=10)
    ap.add_argument('--bits-out', type=int, default=10)
    ap.add_argument('--transfer', default='smpte2084')
    ap.add_argument('--lut', type=int, default=65)
    ap.add_argument('--mode', default='compat8')
    ap.add_argument('--cpu-seconds', type=float, default=12.0, help='CPU-baseline budget (0 = skip)')
    ap.add_argument('--no-alt', action='store_true', help='skip the uniform-content secondary run')
    return ap.parse_args()


def cpu_baseline(params, lattice, width, height, budget_s):
    """Oracle (C restatement of the reference chain, OpenMP) on the host
    cores, on a bounded sample: whole frames until ~budget_s elapse."""
    import numpy as np
    import oracle
    from hdr2sdr.synth import synth_frames
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count() or 1
    cores = max(1, min(cores, int(os.environ.get('OMP_NUM_THREADS', cores))))
    p = oracle.params_from(params.to_c())
    src = synth_frames('smooth', 1, width, height, params.bits_in, device='cpu', seed=0x5EED).to_numpy()
    buf = np.ascontiguousarray(src.buf)
    oracle.process(p, lattice, buf, width, height, nthreads=cores)  # warm
    n, t0 = 0, time.perf_counter()
    while True:
        oracle.process(p, lattice, buf, width, height, nthreads=cores)
        n += 1
        el = time.perf_counter() - t0
        if el >= budget_s or n >= 64:
            break
    mpx = n * width * height / el / 1e6
    return {'value': round(mpx, 3), 'unit': 'Mpixel/s', 'cores': cores, 'kind': 'port',
            'sample': f'{n} x {width}x{height} smooth frame(s), same chain/params, {el:.1f} s, '
                      f'oracle/h2s_oracle.c (C restatement of the ffmpeg chain, not ffmpeg) with {cores} OpenMP threads'}


def main():
    args = parse_args()
    import torch
    import torch.distributed as dist

    import hdr2sdr
    from hdr2sdr.synth import synth_frames

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group('nccl', device_id=torch.device('cuda', local))
    dev = torch.device('cuda', local)
    torch.cuda.set_device(dev)

    params = hdr2sdr.TonemapParams(tonemapper=args.tonemapper, gamma=args.gamma, bits_in=args.bits_in,
                                   bits_out=args.bits_out, transfer=args.transfer, mode=args.mode)
    # LUT lattice: generated on rank 0, broadcast over RCCL (frames never move)
    n = args.lut
    lat = torch.empty((n ** 3, 3), dtype=torch.float32, device=dev)
    if rank == 0:
        lat.copy_(torch.from_numpy(hdr2sdr.generate_lattice(n)))
    if world > 1:
        dist.broadcast(lat, src=0)
    lattice_host = lat.cpu().numpy()

    tm = hdr2sdr.Tonemapper(local, params, lattice_host)
    W, H, B = args.width, args.height, args.frames

    def run(kind):
        src = synth_frames(kind, B, W, H, args.bits_in, device=dev, seed=0x5EED + rank * B)
        dst = hdr2sdr.FrameBatch.empty_torch(B, W, H, args.bits_out, dev)
        stream = torch.cuda.current_stream(dev)
        for _ in range(args.warmup):
            tm.process(src, dst, stream)
        torch.cuda.synchronize(dev)
        tm.set_timing(True)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            tm.process(src, dst, stream)
        torch.cuda.synchronize(dev)
        el = time.perf_counter() - t0
        if world > 1:
            dist.barrier()
            t = torch.tensor([el], device=dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        kms = tm.kernel_ms(args.steps)
        tm.set_timing(False)
        del src, dst
        return el, kms

    el, kms = run(args.kind)
    alt = None
    if not args.no_alt:
        el_u, kms_u = run('uniform')
        alt = {'kind': 'uniform', 'value': round(world * args.steps * B * W * H / el_u / 1e6, 1),
               'kernel_ms': round(kms_u, 4)}

    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return
    px_per_launch = B * W * H
    sb_in = 1 if args.bits_in == 8 else 2
    sb_out = 1 if args.bits_out == 8 else 2
    bytes_per_px = 1.5 * sb_in + 1.5 * sb_out
    value = world * args.steps * px_per_launch / el / 1e6
    achieved = bytes_per_px * px_per_launch / (kms / 1e3) / 1e9
    lut_bytes = n ** 3 * 16
    rec = {
        'metric': 'Mpixel/s HDR10->SDR (4K frames) at 1/2/4/8 GPUs; % HBM roofline',
        'value': round(value, 1),
        'unit': 'Mpixel/s',
        'n_gpus': world,
        'steps': args.steps,
        'warmup': args.warmup,
        'ms_per_step': round(el / args.steps * 1e3, 4),
        'higher_is_better': True,
        'scaling': 'weak',
        'vs_baseline': None,
        'dtype': 'f32',
        'data': 'synthetic',
        'config': {
            'workload': (f'C2: {W}x{H} PQ HDR10 yuv420p{args.bits_in}le -> yuv420p{args.bits_out}le, '
                         f'{args.tonemapper} + {n}^3 tetrahedral LUT + eq gamma {args.gamma}, mode {args.mode}'),
            'frames_per_rank_per_step': B,
            'width': W, 'height': H,
            'content': args.kind,
            'parallelism': f'frame-sharded x{world} (RCCL LUT broadcast only)',
            'alt_content': alt,
        },
        'roofline': {
            'bound': 'hbm',
            'achieved': round(achieved, 1),
            'peak': HBM_PEAK_GBS,
            'unit': 'GB/s',
            'frac': round(achieved / HBM_PEAK_GBS, 4),
            'traffic': None,
            'kernel': 'k_process (h2s_kernels.hip)',
            'kernel_ms': round(kms, 4),
            'bytes_per_px': bytes_per_px,
            'algorithmic_bytes_per_launch': int(bytes_per_px * px_per_launch),
            'lut_bytes_not_counted': lut_bytes,
        },
        'cpu_baseline': None,
    }
    if world == 1 and args.cpu_seconds > 0:
        rec['cpu_baseline'] = cpu_baseline(params, lattice_host, W, H, args.cpu_seconds)
    print(json.dumps(rec), flush=True)
    tm.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
