"""Benchmark: Mpixel/s HDR10 -> SDR on 4K frames at N GPUs, % of HBM roofline.

BASELINE.json metric "Mpixel/s HDR10->SDR (4K frames) at 1/2/4/8 GPUs; % HBM
roofline", measured on its configs[1] (C2): 3840x2160 PQ HDR10
yuv420p10le, Hable + tetrahedral 65^3 LUT + eq gamma, 10-bit output.

One step = one h2s_process launch over a batch of --frames device-resident
synthetic frames per rank.  Ranks shard frames (frame-parallel, no data-path
collective: weak scaling); the only collectives are the RCCL broadcast of the
LUT lattice at start-up and a MAX all-reduce of the elapsed time.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--frames B]
For N > 1 the driver launches one process per GPU with torch.distributed.run;
a plain ``python bench.py --gpus N`` (no WORLD_SIZE in the environment)
starts that launcher itself, as a child process, before touching the GPU.
--dry-run exercises the launch and collectives only (no GPU; gloo on CPU).
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
    # 1000 launches of 64 4K frames: a ~2 s timed region, long enough for an
    # outside sampler (rocm-smi) to see the GPU busy; kernel_ms averages the
    # last 256 launches (the context's event ring)
    ap.add_argument('--steps', type=int, default=1000)
    ap.add_argument('--warmup', type=int, default=10)
    ap.add_argument('--frames', type=int, default=64,
                    help='frames per rank per step (C4: 512 frames / 8 GPUs = 64)')
    ap.add_argument('--width', type=int, default=3840)
    ap.add_argument('--height', type=int, default=2160)
    ap.add_argument('--kind', default='smooth', help='synthetic content (smooth|uniform|ramp|edges), or website (the reference frame)')
    ap.add_argument('--tonemapper', default='hable')
    ap.add_argument('--gamma', type=float, default=2.2)
    ap.add_argument('--bits-in', type=int, default=10)
    ap.add_argument('--bits-out', type=int, default=10)
    ap.add_argument('--transfer', default='smpte2084')
    ap.add_argument('--lut', type=int, default=65)
    ap.add_argument('--mode', default='compat8')
    ap.add_argument('--pipeline', default='auto', help='auto | cpu | libplacebo (profiling runs of one chain)')
    ap.add_argument('--lp-tone', default='ipt', help='libplacebo branch tone form: ipt | max-rgb')
    ap.add_argument('--peak-detect', action='store_true', help='dynamic peak (profiling runs of C3_dyn)')
    ap.add_argument('--cpu-seconds', type=float, default=12.0, help='CPU-baseline budget (0 = skip)')
    ap.add_argument('--no-alt', action='store_true', help='skip the uniform-content secondary run')
    ap.add_argument('--no-sharded', action='store_true',
                    help='skip the sharded C4 / C5 lines (profiling runs of the headline kernel alone)')
    ap.add_argument('--dry-run', action='store_true',
                    help='launch + collectives only, no GPU work (CPU test of the multi-rank flow)')
    return ap.parse_args()


# BASELINE.json's multi-GPU configurations, measured sharded at every N
# beside the C2 headline (frames per rank fixed: weak scaling):
# C4 = configs[3] (512 x 4K Mobius at 8 GPUs: 64 frames per rank),
# C5 = configs[4] (8K 12-bit HLG in, Hable + 65^3, 12-bit out).
SHARDED = (
    ('C4', 'C4: 3840x2160 PQ HDR10 yuv420p10le -> yuv420p10le, mobius + 65^3 tetrahedral LUT, mode compat8, '
           '64 frames per rank (512 at 8 GPUs)',
     dict(tonemapper='mobius', gamma=1.0, bits_in=10, bits_out=10), 3840, 2160, 64, 65),
    ('C5', 'C5: 7680x4320 HLG yuv420p12le -> yuv420p12le, hable + 65^3 tetrahedral LUT, mode compat8, '
           '16 frames per rank',
     dict(tonemapper='hable', gamma=1.0, bits_in=12, bits_out=12, transfer='arib-std-b67'), 7680, 4320, 16, 65),
)
SHARDED_STEPS = 100


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def launch_ranks(gpus: int) -> int:
    """--gpus N without a torch.distributed launcher around us: start one
    (torch.distributed.run, N local ranks, rendezvous on 127.0.0.1) as a child
    process and return its exit code.  Called before anything initialises the
    GPU; the parent never execs."""
    import subprocess
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes', '1', '--nproc-per-node', str(gpus),
           '--master-addr', '127.0.0.1', '--master-port', str(_free_port()), os.path.abspath(__file__)]
    cmd += sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get('HSA_ENABLE_IPC_MODE_LEGACY', '0'))
    return subprocess.run(cmd, env=env).returncode


def cpu_baseline(params, lattice, width, height, budget_s):
    """Oracle (C restatement of the reference chain, OpenMP) on the host
    cores, on a bounded sample: whole frames until ~budget_s elapse, on all
    allowed host threads and on 1 thread (BASELINE.md's CPU plan)."""
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

    def rate(nthreads, budget):
        oracle.process(p, lattice, buf, width, height, nthreads=nthreads)  # warm
        n, t0 = 0, time.perf_counter()
        while True:
            oracle.process(p, lattice, buf, width, height, nthreads=nthreads)
            n += 1
            el = time.perf_counter() - t0
            if el >= budget or n >= 1024:
                return n, el

    n, el = rate(cores, budget_s * 0.45)
    n1, el1 = rate(1, budget_s * 0.2)
    mpx = n * width * height / el / 1e6
    rec = {'value': round(mpx, 3), 'unit': 'Mpixel/s', 'cores': cores, 'kind': 'port',
           'value_1thread': round(n1 * width * height / el1 / 1e6, 3),
           'sample': f'{n} x {width}x{height} smooth frame(s) in {el:.1f} s on {cores} OpenMP threads, '
                     f'{n1} in {el1:.1f} s on 1 thread (value_1thread); same chain/params; '
                     f'oracle/h2s_oracle.c (C restatement of the ffmpeg chain, not ffmpeg)'}
    # BASELINE configs[0] (C1), the reference's own CPU case: 1920x1080 PQ,
    # Reinhard + 33^3 LUT, eq gamma 1.0, 10-bit in -> 8-bit out (the
    # reference's default bit_depth 8, src/conversion.py:42), chain
    # src/utils.py:38-42
    import hdr2sdr
    c1p = hdr2sdr.TonemapParams(tonemapper='reinhard', gamma=1.0, bits_in=10, bits_out=8)
    p, lattice = oracle.params_from(c1p.to_c()), hdr2sdr.generate_lattice(33)
    width, height = 1920, 1080
    src = synth_frames('smooth', 1, width, height, 10, device='cpu', seed=0x5EED).to_numpy()
    buf = np.ascontiguousarray(src.buf)
    n, el = rate(cores, budget_s * 0.25)
    n1, el1 = rate(1, budget_s * 0.1)
    rec['c1'] = {'value': round(n * width * height / el / 1e6, 3), 'unit': 'Mpixel/s', 'cores': cores,
                 'kind': 'port', 'value_1thread': round(n1 * width * height / el1 / 1e6, 3),
                 'frames_per_s': round(n / el, 2), 'frames_per_s_1thread': round(n1 / el1, 2),
                 'workload': 'C1: 1920x1080 PQ yuv420p10le -> yuv420p, reinhard + 33^3 tetrahedral LUT, eq gamma 1.0',
                 'sample': f'{n} x 1920x1080 smooth frame(s) in {el:.1f} s on {cores} OpenMP threads, '
                           f'{n1} in {el1:.1f} s on 1 thread'}
    return rec


def workload_label(args, W, H, n, B):
    """The line's workload string (roofline.traffic is keyed on it): BASELINE's
    C2 for the default arguments; a profiling run of another chain names its
    own config (C3: the libplacebo branch's BT.2390; otherwise the operator,
    pipeline and peak detection)."""
    c2 = (args.tonemapper == 'hable' and args.gamma == 2.2 and args.pipeline == 'auto' and not args.peak_detect
          and args.transfer == 'smpte2084')
    c3 = (args.tonemapper == 'bt.2390' and args.gamma == 1.0 and args.pipeline in ('auto', 'libplacebo')
          and args.transfer == 'smpte2084')
    tag = 'C2' if c2 else ('C3' if c3 else 'profiling run')
    extra = '' if c2 else (f', pipeline {args.pipeline}, lp_tone {args.lp_tone}'
                           + (', peak_detect=1' if args.peak_detect else ''))
    return (f'{tag}: {W}x{H} {"HLG" if args.transfer != "smpte2084" else "PQ HDR10"} yuv420p{args.bits_in}le -> '
            f'yuv420p{args.bits_out}le, {args.tonemapper} + {n}^3 tetrahedral LUT + eq gamma {args.gamma}, '
            f'mode {args.mode}{extra}, {B} frames per launch')


def pmc_traffic(workload):
    """HBM bytes per k_tile dispatch from the committed PMC passes
    (scripts/profile.sh -> prof_summary.py -> profiles/<round>/traffic.json),
    used only when they were measured on this exact workload."""
    import glob
    for f in sorted(glob.glob(os.path.join(REPO, 'profiles', '*', 'traffic.json')), reverse=True):
        try:
            rec = json.load(open(f))
        except (OSError, ValueError):
            continue
        if rec.get('workload') == workload:
            rec['source'] = os.path.relpath(f, REPO) + ' (' + rec.get('method', '') + ')'
            return rec
    return None


def dry_run(args, world, rank):
    """The multi-rank flow without the GPU: gloo process group, the
    params + lattice broadcast, the SUM / MAX reduction; rank 0 prints the
    JSON line shape with n_gpus / world_size as the collectives saw them."""
    import torch.distributed as dist

    import hdr2sdr
    from hdr2sdr.dist import broadcast_setup, reduce_run, shard_range
    if world > 1:
        dist.init_process_group('gloo')
    params = hdr2sdr.TonemapParams(tonemapper=args.tonemapper, gamma=args.gamma)
    n = 17
    lat = hdr2sdr.generate_lattice(n) if rank == 0 else None
    if world > 1:
        params, lat = broadcast_setup(params if rank == 0 else None, lat, n)
        seen = dist.get_world_size()
    else:
        seen = 1
    a, b = shard_range(world * args.frames, world, rank)
    px, cks, el = (b - a) * args.width * args.height, 0, 0.001 * (rank + 1)
    if world > 1:
        px, cks, el = reduce_run(px, cks, el)
    # the sharded C4 / C5 lines: same shard and reduction flow, no GPU work
    sharded = {}
    for tag, workload, kw, w_, h_, fpr, _ in SHARDED:
        a_, b_ = shard_range(world * fpr, world, rank)
        px_, _, el_ = (b_ - a_) * w_ * h_, 0, 0.001 * (rank + 1)
        if world > 1:
            px_, _, el_ = reduce_run(px_, 0, el_)
        sharded[tag] = {'workload': workload, 'pixels': px_, 'max_elapsed_s': el_, 'frames_total': world * fpr}
    if world > 1:
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps({'dry_run': True, 'n_gpus': args.gpus, 'world_size': seen, 'pixels': px,
                          'max_elapsed_s': el, 'gamma': params.gamma, 'lattice_sum': float(lat.sum()),
                          'config': {'workload': 'C2 (dry run)', 'sharded_configs': sharded}}), flush=True)


def main():
    args = parse_args()
    env_world = os.environ.get('WORLD_SIZE')
    if env_world is None and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    world = int(env_world or '1')
    rank = int(os.environ.get('RANK', '0'))
    if world != args.gpus:
        print(f'bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: one rank per GPU is required',
              file=sys.stderr)
        sys.exit(2)
    if args.dry_run:
        return dry_run(args, world, rank)

    import torch
    import torch.distributed as dist

    import hdr2sdr
    from hdr2sdr.dist import broadcast_setup, frame_checksum, reduce_run, shard_range
    from hdr2sdr.synth import synth_frames

    # one process per GPU; H2S_BENCH_DEVICE / H2S_DIST_BACKEND=gloo only let a
    # single-GPU box rehearse the multi-rank flow (ranks sharing one device)
    local = int(os.environ.get('H2S_BENCH_DEVICE', os.environ.get('LOCAL_RANK', '0')))
    backend = os.environ.get('H2S_DIST_BACKEND', 'nccl')
    if world > 1:
        torch.cuda.set_device(local)
        if backend == 'nccl':
            dist.init_process_group('nccl', device_id=torch.device('cuda', local))
        else:
            dist.init_process_group(backend)
    seen_world = dist.get_world_size() if world > 1 else 1
    dev = torch.device('cuda', local)
    torch.cuda.set_device(dev)

    params = hdr2sdr.TonemapParams(tonemapper=args.tonemapper, gamma=args.gamma, bits_in=args.bits_in,
                                   bits_out=args.bits_out, transfer=args.transfer, mode=args.mode,
                                   pipeline=args.pipeline, lp_tone=args.lp_tone,
                                   **(dict(peak_detect=True, maxcll=4000.0) if args.peak_detect else {}))
    # params + LUT lattice: built on rank 0, broadcast over RCCL (frames never move)
    n = args.lut
    lattice_host = hdr2sdr.generate_lattice(n) if rank == 0 else None
    if world > 1:
        params, lattice_host = broadcast_setup(params if rank == 0 else None, lattice_host, n, dev)

    tm = hdr2sdr.Tonemapper(local, params, lattice_host)
    W, H, B = args.width, args.height, args.frames

    def run(kind, make_src=None):
        # this rank's frames: global indices [rank*B, rank*B + B) of a
        # world*B-frame sequence (shard_range), synthesised in place
        a, b = shard_range(world * B, world, rank)
        src = make_src(b - a) if make_src else synth_frames(kind, b - a, W, H, args.bits_in, device=dev, seed=0x5EED + a)
        dst = hdr2sdr.FrameBatch.empty_torch(b - a, W, H, args.bits_out, dev)
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
        kms = tm.kernel_ms(args.steps)
        tm.set_timing(False)
        px = (b - a) * W * H * args.steps
        cks = frame_checksum(dst.buf, a)
        if world > 1:
            px, cks, el = reduce_run(px, cks, el, dev)
        del src, dst
        return el, kms, px, cks

    real_npz = os.path.join(REPO, 'tests', 'golden', 'website_hdr_full.npz')
    if args.kind == 'website':   # profiling runs on the reference's own frame (4K only)
        import numpy as np
        from hdr2sdr.synth import frames_from_rgb8
        rgb8w = np.load(real_npz)['hdr']
        el, kms, px_total, checksum = run('website', lambda n: frames_from_rgb8(rgb8w, n, args.bits_in, dev))
        del rgb8w
    else:
        el, kms, px_total, checksum = run(args.kind)
    alt = None
    if not args.no_alt:
        el_u, kms_u, px_u, _ = run('uniform')
        alt = {'kind': 'uniform', 'value': round(px_u / el_u / 1e6, 1), 'kernel_ms': round(kms_u, 4)}

    # real content: the reference's own website HDR frame (a 4K capture of PQ
    # BT.2020 R'G'B', tests/golden/website_hdr_full.npz), repeated per frame
    real = None
    if world == 1 and not args.no_alt and os.path.exists(real_npz) and (W, H) == (3840, 2160):
        import numpy as np
        from hdr2sdr.synth import frames_from_rgb8
        rgb8 = np.load(real_npz)['hdr']
        el_r, kms_r, px_r, _ = run('real', lambda n: frames_from_rgb8(rgb8, n, args.bits_in, dev))
        real = {'kind': 'website HDR frame (reference HDR to SDR Website/hdr-frame.png, PQ BT.2020 capture)',
                'value': round(px_r / el_r / 1e6, 1), 'kernel_ms': round(kms_r, 4)}
        del rgb8

    # PCIe-inclusive rate (host-resident, page-locked frames through the
    # h2s_process host path: H2D, kernel, D2H): what the drop-in planner's
    # pipes see.  Reported beside, never as, the headline value.
    host_path = None
    if world == 1 and not args.no_alt:
        hs = synth_frames('smooth' if args.kind == 'website' else args.kind, B, W, H, args.bits_in, device='cpu',
                          seed=0x5EED).to_numpy()
        hsrc = hdr2sdr.FrameBatch.empty_pinned(B, W, H, args.bits_in)
        hsrc.buf[...] = hs.buf
        hdst = hdr2sdr.FrameBatch.empty_pinned(B, W, H, args.bits_out)
        def host_rate(t_):
            t_.process(hsrc, hdst)
            n_it, t0 = 5, time.perf_counter()
            for _ in range(n_it):
                t_.process(hsrc, hdst)
            return (time.perf_counter() - t0) / n_it

        el_h = host_rate(tm)
        host_bytes = B * W * H * 1.5 * ((2 if args.bits_in > 8 else 1) + (2 if args.bits_out > 8 else 1))
        os.environ['H2S_HOST_SERIAL'] = '1'   # read at context creation
        try:
            tser = hdr2sdr.Tonemapper(local, params, lattice_host)
        finally:
            del os.environ['H2S_HOST_SERIAL']
        el_s = host_rate(tser)
        tser.close()
        host_path = {'mpx_s': round(B * W * H / el_h / 1e6, 1), 'ms_per_step': round(el_h * 1e3, 3),
                     'serial_mpx_s': round(B * W * H / el_s / 1e6, 1),
                     'pcie_gb_s': round(host_bytes / el_h / 1e9, 1),
                     'pinned': hsrc.buf.ctypes.data != 0 and hasattr(hsrc, '_pin'),
                     'note': 'host frames in, host frames out per h2s_process call; chunks of the batch '
                             'pipelined H2D | kernel | D2H on three streams (serial_mpx_s: one H2D, kernel, D2H)'}
        del hs, hsrc, hdst

    # the other BASELINE.json configurations, single-GPU, for reference
    # (not the headline value): kernel time on device-resident frames
    other = None
    if world == 1 and not args.no_alt:
        other = {}
        for tag, kw, w_, h_, nf, lut_n in (
                ('C1', dict(tonemapper='reinhard', gamma=1.0, bits_out=8), 1920, 1080, 16, 33),
                # C3 as the reference runs it: the libplacebo branch (rgba8 + lut3d 8-bit, src/utils.py:444-460)
                ('C3', dict(tonemapper='bt.2390', gamma=1.0, bits_out=10), 3840, 2160, 16, 65),
                ('C3_cpu_chain', dict(tonemapper='bt.2390', gamma=1.0, bits_out=10, pipeline='cpu'), 3840, 2160, 16, 65),
                ('C3_max_rgb', dict(tonemapper='bt.2390', gamma=1.0, bits_out=10, lp_tone='max-rgb'), 3840, 2160, 16, 65),
                ('C2_libplacebo', dict(tonemapper='hable', gamma=2.2, bits_out=10, pipeline='libplacebo'), 3840, 2160, 16, 65),
                ('C4', dict(tonemapper='mobius', gamma=1.0, bits_out=10), 3840, 2160, 16, 65),
                ('C5', dict(tonemapper='hable', gamma=1.0, bits_in=12, bits_out=12, transfer='arib-std-b67'),
                 7680, 4320, 4, 65),
                # the reference's other GPU-only operator (libplacebo spline), C3's shape
                ('C3_spline', dict(tonemapper='spline', gamma=1.0, bits_out=10), 3840, 2160, 16, 65),
                # C3 with libplacebo's peak_detect=1 (src/utils.py:448): statistics + finish (device IIR, curve records), one tile launch
                ('C3_dyn', dict(tonemapper='bt.2390', gamma=1.0, bits_out=10, peak_detect=True, maxcll=4000.0),
                 3840, 2160, 16, 65),
                # C3 on the reference's own website frame (real content: its colours
                # cluster, so the lut3d table's lines mostly stay in the L2)
                ('C3_website', dict(tonemapper='bt.2390', gamma=1.0, bits_out=10), 3840, 2160, 16, 65)):
            if tag.endswith('_website') and not os.path.exists(real_npz):
                continue
            p_ = hdr2sdr.TonemapParams(mode=args.mode, **kw)
            t_ = hdr2sdr.Tonemapper(local, p_, hdr2sdr.generate_lattice(lut_n))
            if tag.endswith('_website'):
                import numpy as np
                from hdr2sdr.synth import frames_from_rgb8
                src_ = frames_from_rgb8(np.load(real_npz)['hdr'], nf, p_.bits_in, dev)
            else:
                src_ = synth_frames('smooth', nf, w_, h_, p_.bits_in, device=dev, seed=0x5EED)
            dst_ = hdr2sdr.FrameBatch.empty_torch(nf, w_, h_, p_.bits_out, dev)
            st_ = torch.cuda.current_stream(dev)

            def timed_(t_):
                for _ in range(3):
                    t_.process(src_, dst_, st_)
                torch.cuda.synchronize(dev)
                t_.set_timing(True)
                for _ in range(20):
                    t_.process(src_, dst_, st_)
                torch.cuda.synchronize(dev)
                return t_.kernel_ms(20)

            kms_ = timed_(t_)
            b_ = 1.5 * (1 if p_.bits_in == 8 else 2) + 1.5 * (1 if p_.bits_out == 8 else 2)
            other[tag] = {'size': f'{w_}x{h_}', 'frames': nf, 'tonemapper': kw['tonemapper'], 'lut': lut_n,
                          'content': 'website frame' if tag.endswith('_website') else 'smooth',
                          'bits': f"{p_.bits_in}->{p_.bits_out}", 'kernel_ms': round(kms_, 4),
                          'mpx_s': round(nf * w_ * h_ / kms_ / 1e3, 1),
                          'hbm_frac': round(b_ * nf * w_ * h_ / (kms_ / 1e3) / 1e9 / HBM_PEAK_GBS, 4)}
            if p_.peak_detect:
                # the detection's own cost: the same call without peak_detect
                # (same static peak, so the tile kernel's curve work matches)
                t0_ = hdr2sdr.Tonemapper(local, p_.with_(peak_detect=False), hdr2sdr.generate_lattice(lut_n))
                sms_ = timed_(t0_)
                t0_.close()
                other[tag]['static_same_peak_ms'] = round(sms_, 4)
                other[tag]['peak_detect_overhead_ms'] = round(kms_ - sms_, 4)
            if p_.resolved_pipeline() == 'libplacebo':
                # the libplacebo stage is a restatement (no libplacebo in the image):
                # GPU = oracle is tested, the oracle itself is not pinned to libplacebo;
                # the detected peak (peak_detect=1) even less so
                other[tag]['parity'] = ('unpinned: dynamic peak (libplacebo peak_detect restated)'
                                        if p_.peak_detect else 'unpinned: libplacebo stage restated')
            t_.close()
            del src_, dst_

    # BASELINE's multi-GPU configurations C4 / C5, frame-sharded over every
    # rank exactly as the headline (barrier + synchronize around the timed
    # launches, MAX of the elapsed time over ranks, SUM of pixels)
    sharded = {}
    for tag, workload, kw, w_, h_, fpr, lut_n in (() if args.no_sharded else SHARDED):
        p_ = hdr2sdr.TonemapParams(mode=args.mode, **kw)
        lat_ = hdr2sdr.generate_lattice(lut_n) if rank == 0 else None
        if world > 1:
            p_, lat_ = broadcast_setup(p_ if rank == 0 else None, lat_, lut_n, dev)
        t_ = hdr2sdr.Tonemapper(local, p_, lat_)
        a_, b_ = shard_range(world * fpr, world, rank)
        src_ = synth_frames('smooth', b_ - a_, w_, h_, p_.bits_in, device=dev, seed=0x5EED + a_)
        dst_ = hdr2sdr.FrameBatch.empty_torch(b_ - a_, w_, h_, p_.bits_out, dev)
        st_ = torch.cuda.current_stream(dev)
        for _ in range(3):
            t_.process(src_, dst_, st_)
        torch.cuda.synchronize(dev)
        t_.set_timing(True)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0_ = time.perf_counter()
        for _ in range(SHARDED_STEPS):
            t_.process(src_, dst_, st_)
        torch.cuda.synchronize(dev)
        el_ = time.perf_counter() - t0_
        if world > 1:
            dist.barrier()
        kms_ = t_.kernel_ms(SHARDED_STEPS)
        t_.set_timing(False)
        px_ = (b_ - a_) * w_ * h_ * SHARDED_STEPS
        cks_ = frame_checksum(dst_.buf, a_)
        if world > 1:
            px_, cks_, el_ = reduce_run(px_, cks_, el_, dev)
        b_px = 1.5 * (1 if p_.bits_in == 8 else 2) + 1.5 * (1 if p_.bits_out == 8 else 2)
        sharded[tag] = {'workload': workload, 'value': round(px_ / el_ / 1e6, 1), 'unit': 'Mpixel/s',
                        'ms_per_step': round(el_ / SHARDED_STEPS * 1e3, 4), 'steps': SHARDED_STEPS,
                        'frames_total': world * fpr, 'frames_per_rank': fpr,
                        'rank0_kernel_ms': round(kms_, 4),
                        'rank0_hbm_frac': round(b_px * (b_ - a_) * w_ * h_ / (kms_ / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                        'output_checksum': cks_}
        t_.close()
        del src_, dst_

    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return
    px_per_launch = B * W * H
    sb_in = 1 if args.bits_in == 8 else 2
    sb_out = 1 if args.bits_out == 8 else 2
    bytes_per_px = 1.5 * sb_in + 1.5 * sb_out
    value = px_total / el / 1e6
    achieved = bytes_per_px * px_per_launch / (kms / 1e3) / 1e9
    lut_bytes = n ** 3 * 12     # YUV-premultiplied lattice records read by k_tile
    rec = {
        'metric': 'Mpixel/s HDR10->SDR (4K frames) at 1/2/4/8 GPUs; % HBM roofline',
        'value': round(value, 1),
        'unit': 'Mpixel/s',
        'n_gpus': world,
        'world_size': seen_world,
        'steps': args.steps,
        'warmup': args.warmup,
        'ms_per_step': round(el / args.steps * 1e3, 4),
        'higher_is_better': True,
        'scaling': 'weak',
        'vs_baseline': None,
        'dtype': 'f32',
        'data': 'synthetic',
        'config': {
            'workload': workload_label(args, W, H, n, B),
            'frames_per_rank_per_step': B,
            'width': W, 'height': H,
            'content': args.kind,
            'parallelism': f'frame-sharded x{world} ({backend if world > 1 else "single rank"}; '
                           f'params + LUT broadcast only)',
            'alt_content': alt,
            'real_content': real,
            'other_configs': other,
            'sharded_configs': sharded,
            'host_path': host_path,
        },
        'roofline': {
            'bound': 'hbm',
            'achieved': round(achieved, 1),
            'peak': HBM_PEAK_GBS,
            'unit': 'GB/s',
            'frac': round(achieved / HBM_PEAK_GBS, 4),
            # the read-only share (the input bytes alone)
            'read_only_frac': round(1.5 * sb_in * px_per_launch / (kms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
            'traffic': None,
            'kernel': 'k_tile (h2s_fast.hip)',
            'kernel_ms': round(kms, 4),
            'bytes_per_px': bytes_per_px,
            'algorithmic_bytes_per_launch': int(bytes_per_px * px_per_launch),
            'lut_bytes_not_counted': lut_bytes,
        },
        'cpu_baseline': None,
    }
    tr = pmc_traffic(rec['config']['workload'])
    if tr is not None:
        rec['roofline']['traffic'] = tr['bytes_per_dispatch']
        rec['roofline']['traffic_source'] = tr['source']
        # k_tile's instruction mix from the same PMC passes (per pixel)
        rec['roofline']['instructions_per_px'] = {k: tr[k] for k in ('valu_per_px', 'trans_per_px', 'cvt_per_px',
                                                                      'lds_per_px', 'vmem_rd_per_px') if k in tr}
        # the unit that binds, from the same PMC passes
        # (scripts/prof_summary.py unit_shares): VALU issue against the
        # gfx950 rate (2 cycles per wave64 full-rate op per SIMD-32, 4 per
        # transcendental), the texture data / address units' busy shares;
        # 'frac' stays the HBM fraction north_star's roofline asks for
        for k in ('valu_insts_per_cu_cycle', 'valu_issue_frac', 'valu_waves_per_simd', 'td_busy_frac',
                  'td_tc_stall_frac', 'ta_busy_frac'):
            if k in tr:
                rec['roofline'][k] = tr[k]
        units = {'hbm': rec['roofline']['frac'], 'valu-issue': tr.get('valu_issue_frac', 0.0),
                 'vmem-td': tr.get('td_busy_frac', 0.0)}
        top = max(units, key=units.get)
        if top != 'hbm':
            rec['roofline']['bound'] = top
            rec['roofline']['bound_note'] = (
                'busiest unit by PMC: texture data (L1 -> VGPR) %.2f busy, %.2f of it waiting for the L1; '
                'VALU issue %.2f of the gfx950 rate (%.2f wave-instructions per CU-cycle); HBM %.2f: the '
                'lattice gathers and the frame I/O share the vector-memory path (DESIGN.md 4.1)'
                % (tr.get('td_busy_frac', float('nan')), tr.get('td_tc_stall_frac', float('nan')),
                   tr.get('valu_issue_frac', float('nan')), tr.get('valu_insts_per_cu_cycle', float('nan')),
                   rec['roofline']['frac']))
    rec['config']['output_checksum'] = checksum
    if world == 1 and args.cpu_seconds > 0:
        rec['cpu_baseline'] = cpu_baseline(params, lattice_host, W, H, args.cpu_seconds)
    print(json.dumps(rec), flush=True)
    tm.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
