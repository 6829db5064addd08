"""Drop-in I/O planner and executor around libh2s.

The reference runs one ffmpeg child per conversion:
``build()`` (src/ffmpeg_command.py:455-514) emits
``ffmpeg … -i IN -filter_complex "[0:v:0]{chain}[vout]" -map [vout] …``.
``ConversionManager.start`` launches it (src/conversion.py:209-224), and
``monitor_progress`` (:225-272) reads ``time=`` lines from its stderr.
ffmpeg has no external-filter ABI, so here ffmpeg keeps demux, decode,
encode and mux. The tone-map chain moves onto the GPU between two pipes:

    decode:  ffmpeg -i IN -map 0:v:0 -f rawvideo -pix_fmt yuv420p1Xle -
    libh2s:  h2s_process() on batches of frames
    encode:  ffmpeg -f rawvideo … -i - -i IN <every non-filter option build() chose>

``plan_from_argv`` takes the argv the reference's own ``build()`` produced.
Streams, encoder, rate control, tags, ``-r``, ``-pix_fmt``, metadata and
faststart therefore stay exactly the reference's choice. Only the filter
graph leaves ffmpeg. ``H2SProcess`` is Popen-shaped (``stderr``, ``wait``,
``poll``, ``returncode``, ``terminate``, ``kill``), so ``monitor_progress``
and its ``time=`` parsing work on it unchanged.
"""
from __future__ import annotations

import io
import queue
import subprocess
import threading
from dataclasses import dataclass, field
from typing import Any, Callable, Optional, Tuple

import numpy as np

from .chain import DOVI_P5_ERROR, TonemapParams, is_dovi_profile5, parse_filter_chain

# planar 4:2:0 formats the pipe carries, by bit depth
PIPE_PIX_FMT = {8: 'yuv420p', 10: 'yuv420p10le', 12: 'yuv420p12le'}
# encoder -pix_fmt values build() emits (src/ffmpeg_command.py:355-368) -> bits
OUT_PIX_FMT_BITS = {'yuv420p': 8, 'yuv420p10le': 10, 'p010le': 10, 'yuv420p12le': 12}
# setparams=color_primaries=bt709:color_trc=bt709:colorspace=bt709 (src/utils.py:40)
# on frames that leave zscale r=tv: as output tags on the encode side
BT709_TAGS = ['-color_primaries', 'bt709', '-color_trc', 'bt709', '-colorspace', 'bt709', '-color_range', 'tv']
TRANSFERS = {'smpte2084': 'smpte2084', 'arib-std-b67': 'arib-std-b67', '': 'smpte2084'}


@dataclass
class PipePlan:
    decode: 'list[str]'
    encode: 'list[str]'
    params: TonemapParams
    lut_path: 'str | None'
    width: int
    height: int
    input_path: str
    output_path: str
    reference_argv: 'list[str]' = field(default_factory=list)

    @property
    def frame_bytes_in(self) -> int:
        return self.width * self.height * 3 // 2 * (1 if self.params.bits_in == 8 else 2)

    @property
    def frame_bytes_out(self) -> int:
        return self.width * self.height * 3 // 2 * (1 if self.params.bits_out == 8 else 2)


def _remap_input(spec: str) -> str:
    """'0:a?' -> '1:a?': the original file is input 1 of the encode side."""
    if spec.startswith('0:') or spec == '0':
        return '1' + spec[1:]
    return spec


def plan_from_argv(argv: 'list[str]', properties: 'dict[str, Any]', hdr: 'dict[str, Any] | None' = None,
                   mode: str = 'compat8') -> PipePlan:
    """Split a reference ``build()`` argv into decode/encode argvs + params.

    properties: the reference's ``get_video_properties`` dict
    (src/utils.py:1040-1058): width, height, bit_depth, color_transfer.
    hdr: ``_probe_hdr_metadata`` output (src/utils.py:329-372). Inside
    ffmpeg, vf_tonemap reads MaxCLL from frame side data. Raw pipes drop side
    data, so it is passed to libh2s explicitly here.
    Raises ValueError for an argv without a tone-map filter graph, and for a
    Dolby Vision profile 5 source (its RPU cannot cross the pipe)."""
    argv = list(argv)
    if is_dovi_profile5(properties):
        # src/ffmpeg_command.py:100-106: profile 5 needs the RPU libplacebo
        # applies; the rawvideo decode pipe drops it
        raise ValueError(DOVI_P5_ERROR)
    if '-i' not in argv or '-filter_complex' not in argv:
        raise ValueError('argv has no -i / -filter_complex: not a build() conversion command')
    exe = argv[0]
    i_in = argv.index('-i')
    input_path = argv[i_in + 1]
    i_fc = argv.index('-filter_complex')
    chain = argv[i_fc + 1]
    rest = argv[i_fc + 2:]
    # drop '-map [vout]' (the filter graph's output pad)
    out: 'list[str]' = []
    k = 0
    while k < len(rest):
        tok = rest[k]
        if tok == '-map' and k + 1 < len(rest) and rest[k + 1].startswith('['):
            k += 2
            continue
        if tok == '-map' and k + 1 < len(rest):
            out += [tok, _remap_input(rest[k + 1])]
            k += 2
            continue
        if tok == '-map_metadata' and k + 1 < len(rest):
            out += [tok, _remap_input(rest[k + 1])]
            k += 2
            continue
        out.append(tok)
        k += 1
    if '-pix_fmt' not in out:
        raise ValueError('argv has no -pix_fmt for the output')
    enc_pix_fmt = out[out.index('-pix_fmt') + 1]
    if enc_pix_fmt not in OUT_PIX_FMT_BITS:
        raise ValueError(f'unsupported output pix_fmt {enc_pix_fmt!r}')
    bits_out = OUT_PIX_FMT_BITS[enc_pix_fmt]
    bits_in = int(properties.get('bit_depth') or 10)
    if bits_in not in (10, 12):
        raise ValueError(f'{bits_in}-bit sources are not HDR10/HLG inputs')
    trc = properties.get('color_transfer', '') or ''
    if trc not in TRANSFERS:
        raise ValueError(f'unsupported source transfer {trc!r} (expected smpte2084 or arib-std-b67)')
    extra: 'dict[str, Any]' = {}
    if hdr:
        if hdr.get('maxcll'):
            extra['maxcll'] = float(hdr['maxcll'])
        if hdr.get('mastering_max'):
            extra['mastering_max'] = float(hdr['mastering_max'])
    params, lut_path = parse_filter_chain(chain, bits_in=bits_in, bits_out=bits_out,
                                          transfer=TRANSFERS[trc], mode=mode, **extra)
    W, H = int(properties['width']), int(properties['height'])
    fps = out[out.index('-r') + 1] if '-r' in out else str(properties.get('frame_rate', 24.0))
    # output path = last positional before the optional trailing -y
    o_idx = len(out) - 2 if out and out[-1] == '-y' else len(out) - 1
    output_path = out[o_idx]
    encode_opts = out[:o_idx] + BT709_TAGS + out[o_idx:]
    pipe_out = PIPE_PIX_FMT[bits_out]
    decode = [exe, '-loglevel', 'error', '-nostdin', '-i', input_path, '-map', '0:v:0',
              '-f', 'rawvideo', '-pix_fmt', PIPE_PIX_FMT[bits_in], '-']
    encode = [exe, '-loglevel', 'info', '-f', 'rawvideo', '-pix_fmt', pipe_out, '-s', f'{W}x{H}',
              '-r', fps, '-i', '-', '-i', input_path, '-map', '0:v:0'] + encode_opts
    return PipePlan(decode=decode, encode=encode, params=params, lut_path=lut_path, width=W, height=H,
                    input_path=input_path, output_path=output_path, reference_argv=argv)


def _read_full(stream: Any, buf: memoryview) -> int:
    """Fill buf from a pipe; returns bytes read (short only at EOF)."""
    got = 0
    while got < len(buf):
        n = stream.readinto(buf[got:])
        if not n:
            break
        got += n
    return got


class H2SProcess:
    """Popen-shaped handle of a decode -> libh2s -> encode conversion.

    ``stderr`` is the encoder's stderr as text lines. ffmpeg prints its
    ``time=`` progress there, as it does for the reference's single process
    (src/conversion.py:225-240). ``returncode`` is the encoder's, or the
    decoder's when that failed, or 1 when the GPU stage raised (``error``
    holds the exception)."""

    def __init__(self, plan: PipePlan, tonemapper: Any, batch: int = 8,
                 popen: Callable[..., Any] = subprocess.Popen, depth: int = 2):
        from .frames import FrameBatch
        self.plan = plan
        self.error: Optional[BaseException] = None
        self._tm = tonemapper
        self._batch = max(1, int(batch))
        self.dec = popen(plan.decode, stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, stdin=subprocess.DEVNULL)
        self.enc = popen(plan.encode, stdin=subprocess.PIPE, stderr=subprocess.PIPE, stdout=subprocess.DEVNULL)
        self.stderr = io.TextIOWrapper(self.enc.stderr, encoding='utf-8', errors='replace')
        p = plan.params
        # page-locked staging: the pipe bytes go straight to / from HBM by DMA.
        # `depth` input slots let the decoder run ahead while the GPU stage
        # and the encoder work on earlier batches.
        self._src = [FrameBatch.empty_pinned(self._batch, plan.width, plan.height, p.bits_in)
                     for _ in range(max(1, int(depth)))]
        self._dst = FrameBatch.empty_pinned(self._batch, plan.width, plan.height, p.bits_out)
        self._free: 'queue.Queue[Optional[int]]' = queue.Queue()
        self._filled: 'queue.Queue[Optional[Tuple[int, int]]]' = queue.Queue()
        for i in range(len(self._src)):
            self._free.put(i)
        self.frames = 0
        self._reader = threading.Thread(target=self._read, name='h2s-read', daemon=True)
        self._thread = threading.Thread(target=self._pump, name='h2s-pump', daemon=True)
        self._reader.start()
        self._thread.start()

    def _fail(self, e: BaseException) -> None:
        """GPU / pipe failure: record the first error and stop both ends."""
        if self.error is None:
            self.error = e
        for p in (self.dec, self.enc):
            try:
                p.kill()
            except Exception:
                pass

    def _read(self) -> None:
        """Decoder pipe -> free input slots, in order (one batch per slot)."""
        fin = self.plan.frame_bytes_in
        try:
            while True:
                slot = self._free.get()
                if slot is None:          # the pump stopped
                    return
                mv = memoryview(self._src[slot].buf).cast('B')
                got = _read_full(self.dec.stdout, mv)
                if got // fin:
                    self._filled.put((slot, got // fin))
                if got < len(mv):
                    return
        except BaseException as e:
            self._fail(e)
        finally:
            self._filled.put(None)

    def _pump(self) -> None:
        """Filled slots -> libh2s -> encoder pipe, in decode order."""
        fout = self.plan.frame_bytes_out
        dst_mv = memoryview(self._dst.buf).cast('B')
        try:
            while True:
                item = self._filled.get()
                if item is None:
                    break
                slot, n = item
                self._tm.process(self._src[slot], self._dst, nframes=n)   # synchronous for host frames
                self._free.put(slot)
                self.enc.stdin.write(dst_mv[:n * fout])
                self.frames += n
        except BaseException as e:
            self._fail(e)
        finally:
            self._free.put(None)          # release a reader waiting for a slot
            try:
                self.enc.stdin.close()
            except Exception:
                pass

    # ---- Popen surface -----------------------------------------------------
    @property
    def returncode(self) -> 'int | None':
        rc = self.enc.poll()
        if rc is None or self._thread.is_alive():
            return None
        if self.error is not None:
            return 1
        drc = self.dec.poll()
        if drc not in (None, 0):
            return drc
        return rc

    def poll(self) -> 'int | None':
        return self.returncode

    def wait(self, timeout: 'float | None' = None) -> int:
        self._thread.join(timeout)
        self._reader.join(timeout)
        self.enc.wait(timeout)
        self.dec.wait(timeout)
        rc = self.returncode
        assert rc is not None
        return rc

    def terminate(self) -> None:
        for p in (self.dec, self.enc):
            p.terminate()

    def kill(self) -> None:
        for p in (self.dec, self.enc):
            p.kill()


def start(plan: PipePlan, device: int = 0, batch: int = 8, lattice: 'np.ndarray | None' = None,
          popen: Callable[..., Any] = subprocess.Popen) -> H2SProcess:
    """Launch a planned conversion on ``device`` (the GPU replacement of
    ``start_ffmpeg_process(cmd)``, src/conversion.py:209-224)."""
    from . import lut as _lut
    from .engine import Tonemapper
    tm = Tonemapper(device, plan.params)
    if plan.params.lut_enabled:
        if lattice is not None:
            tm.set_lut(lattice)
        elif plan.lut_path and plan.lut_path != '<LUT>':
            tm.load_cube(_lut.unescape_filter_path(plan.lut_path))
        else:
            tm.set_lut(_lut.generate_lattice(_lut.LUT_SIZE))
    return H2SProcess(plan, tm, batch=batch, popen=popen)
