"""Regenerate the committed golden fixtures from the reference itself.

Runs ONLY in the build container, where /root/reference is mounted (the GPU
box has no reference).  It imports the reference's own Python — nothing of it
is copied into this repository; only its outputs (hashes, sampled numbers,
strings) are written as JSON data.

* lut_hashes.json   — tools/generate_lut.py generate_cube_lines(n) for
                      n in (2, 3, 17, 33, 65): sha256/md5/byte count of the
                      .cube text, plus sampled lattice rows.
* lut_convert.json  — tools/generate_lut.py _convert() on a seeded point set.
* filter_chains.json — src/ffmpeg_command._filter_args / build() for the
                      BASELINE.json configurations C1..C5 (Appendix A of
                      SURVEY.md: stub tkinter, dummy ffmpeg on PATH, the LUT
                      regenerated into a temporary copy of src/).
* request_rules.json — build() over a matrix of requests and probe results
                      (use_gpu x operator x bit depth x lut_enabled x gamma,
                      CUDA interop, Dolby Vision profile 5, libplacebo absent):
                      the chain string or the ValueError it raises, plus the
                      preview chains (FFMPEG_FILTER, build_libplacebo_filter
                      with PREVIEW_SIZE) — pins TonemapParams.from_request.

Usage:  python tests/golden/make_golden.py [lut] [chains] [rules]   (default: all)
"""
from __future__ import annotations

import hashlib
import importlib.util
import json
import os
import random
import shutil
import stat
import subprocess
import sys
import tempfile

REF = '/root/reference'
HERE = os.path.dirname(os.path.abspath(__file__))


def load_generator():
    spec = importlib.util.spec_from_file_location('ref_generate_lut', os.path.join(REF, 'tools', 'generate_lut.py'))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def lut_goldens(gen) -> None:
    out = {'source': 'tools/generate_lut.py generate_cube_lines (reference, imported)', 'sizes': {}}
    rnd = random.Random(1234)
    for n in (2, 3, 17, 33, 65):
        lines = gen.generate_cube_lines(n)
        text = ('\n'.join(lines) + '\n').encode('ascii')
        idx = sorted(set([0, 1, n - 1, n * n, n ** 3 - 1] + [rnd.randrange(n ** 3) for _ in range(40)]))
        out['sizes'][str(n)] = {
            'sha256': hashlib.sha256(text).hexdigest(),
            'md5': hashlib.md5(text).hexdigest(),
            'bytes': len(text),
            'header': lines[0],
            'rows': {str(i): lines[1 + i] for i in idx},
        }
    with open(os.path.join(HERE, 'lut_hashes.json'), 'w') as f:
        json.dump(out, f, indent=1, sort_keys=True)


def convert_goldens(gen) -> None:
    rnd = random.Random(42)
    pts = [(0.0, 0.0, 0.0), (1.0, 1.0, 1.0), (1.0, 0.0, 0.0), (0.0, 1.0, 0.0), (0.0, 0.0, 1.0),
           (0.490196, 0.2, 0.8), (0.05, 0.5, 0.95)]
    pts += [(rnd.random(), rnd.random(), rnd.random()) for _ in range(200)]
    rows = [{'in': list(p), 'out': list(gen._convert(*p))} for p in pts]
    with open(os.path.join(HERE, 'lut_convert.json'), 'w') as f:
        json.dump({'source': 'tools/generate_lut.py _convert (reference, imported)', 'points': rows}, f)


def chain_goldens() -> None:
    tmp = tempfile.mkdtemp(prefix='h2s_refcopy_')
    try:
        shutil.copytree(os.path.join(REF, 'src'), os.path.join(tmp, 'src'))
        shutil.copytree(os.path.join(REF, 'tools'), os.path.join(tmp, 'tools'))
        subprocess.run([sys.executable, os.path.join(tmp, 'tools', 'generate_lut.py')], check=True,
                       stdout=subprocess.DEVNULL)
        fakebin = os.path.join(tmp, 'fakebin')
        os.makedirs(fakebin)
        for name in ('ffmpeg', 'ffprobe'):
            p = os.path.join(fakebin, name)
            with open(p, 'w') as f:
                f.write('#!/bin/sh\nexit 1\n')
            os.chmod(p, os.stat(p).st_mode | stat.S_IEXEC)
        script = r'''
import json, sys, os
from dataclasses import dataclass
sys.path.insert(0, os.path.join(sys.argv[1], 'src'))
import utils, ffmpeg_command
from conversion_view import ConversionView

@dataclass(frozen=True)
class Req:
    input_path: str = 'in.mkv'
    output_path: str = 'out.mkv'
    gamma: float = 1.0
    use_gpu: bool = False
    tonemapper: str = 'reinhard'
    quality: int = 23
    quality_mode: str = 'cq'
    bit_depth: int = 10
    licensed: bool = False
    lut_enabled: bool = True

class View:
    def notify(self, n): pass
    def schedule(self, fn, *a): fn(*a)

lut = utils.get_lut_filter_path()
props = {'codec_name': 'hevc', 'frame_rate': 24.0, 'bit_rate': 8000000}
probes = ffmpeg_command.Probes(lambda: None, lambda: True, lambda: False)
cases = {
  'C1': dict(tonemapper='Reinhard', gamma=1.0, bit_depth=10),
  'C2': dict(tonemapper='Hable', gamma=2.2, bit_depth=10),
  'C3': dict(tonemapper='BT.2390', gamma=1.0, bit_depth=10, use_gpu=True),
  'C4': dict(tonemapper='Mobius', gamma=1.0, bit_depth=10),
  'C5': dict(tonemapper='Hable', gamma=1.0, bit_depth=12, licensed=True),
  'default8': dict(tonemapper='Mobius', gamma=1.0, bit_depth=8),
  'gamma05': dict(tonemapper='Hable', gamma=0.5, bit_depth=8),
}
out = {}
for name, kw in cases.items():
    r = Req(**{**kw, 'tonemapper': kw['tonemapper'].lower()})
    argv = ffmpeg_command.build(r, props, probes, View())
    argv = [a.replace(lut, '<LUT>') if isinstance(a, str) else a for a in argv]
    argv[0] = 'ffmpeg'
    fc = argv[argv.index('-filter_complex') + 1]
    out[name] = {'request': kw, 'filter_complex': fc, 'pix_fmt': argv[argv.index('-pix_fmt') + 1],
                 'argv': argv}
try:
    ffmpeg_command._filter_args(Req(tonemapper='bt.2390'), ffmpeg_command._tonemap_plan(Req(), props, lambda: False),
                                ffmpeg_command._gpu_device_args(ffmpeg_command._tonemap_plan(Req(), props, lambda: False), lambda: None, lambda: False))
    out['cpu_bt2390_error'] = None
except ValueError as e:
    out['cpu_bt2390_error'] = str(e)
out['FFMPEG_CONVERT_FILTER'] = utils.FFMPEG_CONVERT_FILTER
out['FFMPEG_FILTER_LEGACY_NO_LUT'] = utils.FFMPEG_FILTER_LEGACY_NO_LUT
out['TONEMAP'] = utils.TONEMAP
out['GPU_ONLY_TONEMAPPERS'] = sorted(utils.GPU_ONLY_TONEMAPPERS)
print(json.dumps(out))
'''
        env = dict(os.environ, PATH=fakebin + os.pathsep + os.environ.get('PATH', ''))
        res = subprocess.run([sys.executable, '-c', script, tmp], env=env, check=True,
                             stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
        data = json.loads(res.stdout.strip().splitlines()[-1])
        data['source'] = 'src/ffmpeg_command.py build()/_filter_args (reference, imported; SURVEY.md App. A)'
        with open(os.path.join(HERE, 'filter_chains.json'), 'w') as f:
            json.dump(data, f, indent=1, sort_keys=True)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


RULES_SCRIPT = r'''
import json, sys, os
from dataclasses import dataclass
sys.path.insert(0, os.path.join(sys.argv[1], 'src'))
import utils, ffmpeg_command

@dataclass(frozen=True)
class Req:
    input_path: str = 'in.mkv'
    output_path: str = 'out.mkv'
    gamma: float = 1.0
    use_gpu: bool = False
    tonemapper: str = 'reinhard'
    quality: int = 23
    quality_mode: str = 'cq'
    bit_depth: int = 10
    licensed: bool = False
    lut_enabled: bool = True

class View:
    def notify(self, n): pass
    def schedule(self, fn, *a): fn(*a)

lut = utils.get_lut_filter_path()
base_props = {'codec_name': 'hevc', 'frame_rate': 24.0, 'bit_rate': 8000000}
cases = []
for tm in ('reinhard', 'mobius', 'hable', 'bt.2390', 'spline'):
    for use_gpu in (False, True):
        for bd in (8, 10, 12):
            cases.append(dict(req=dict(tonemapper=tm, use_gpu=use_gpu, bit_depth=bd, licensed=bd == 12)))
for tm in ('hable', 'bt.2390'):
    for lut_on in (True, False):
        for g in (1.0, 2.2):
            cases.append(dict(req=dict(tonemapper=tm, use_gpu=True, bit_depth=10, lut_enabled=lut_on, gamma=g)))
            cases.append(dict(req=dict(tonemapper=tm, use_gpu=True, bit_depth=10, lut_enabled=lut_on, gamma=g),
                              encoder='h264_nvenc', interop=True))
    cases.append(dict(req=dict(tonemapper=tm, use_gpu=False, bit_depth=10, lut_enabled=False)))
    cases.append(dict(req=dict(tonemapper=tm, use_gpu=True, bit_depth=10), libplacebo=False))
    for bd in (10, 12):
        cases.append(dict(req=dict(tonemapper=tm, use_gpu=False, bit_depth=bd, licensed=bd == 12),
                          props=dict(is_dolby_vision=True, dovi_profile=5)))
        cases.append(dict(req=dict(tonemapper=tm, use_gpu=False, bit_depth=bd, licensed=bd == 12),
                          props=dict(is_dolby_vision=True, dovi_profile=8)))
out = {'cases': []}
for c in cases:
    props = dict(base_props, **c.get('props', {}))
    probes = ffmpeg_command.Probes(lambda c=c: c.get('encoder'), lambda c=c: c.get('libplacebo', True),
                                   lambda c=c: c.get('interop', False))
    r = Req(**c['req'])
    rec = dict(c)
    try:
        argv = ffmpeg_command.build(r, props, probes, View())
        fc = argv[argv.index('-filter_complex') + 1]
        rec['filter_complex'] = fc.replace(lut, '<LUT>')
        rec['pix_fmt'] = argv[argv.index('-pix_fmt') + 1]
    except ValueError as e:
        rec['error'] = str(e)
    out['cases'].append(rec)
prev = {}
for tm in ('reinhard', 'mobius', 'hable'):
    prev['cpu_' + tm] = utils.FFMPEG_FILTER.format(gamma=1.0, width=3840, height=2160, tonemapper=tm,
                                                     lut_path='<LUT>')
for tm in ('bt.2390', 'spline', 'hable'):
    for lut_on in (True, False):
        prev[f'gpu_{tm}_lut{int(lut_on)}'] = utils.build_libplacebo_filter(
            1.0, tm, width=3840, height=2160, lut_enabled=lut_on).replace(lut, '<LUT>')
out['preview'] = prev
print(json.dumps(out))
'''


def rules_goldens() -> None:
    tmp = tempfile.mkdtemp(prefix='h2s_refcopy_')
    try:
        shutil.copytree(os.path.join(REF, 'src'), os.path.join(tmp, 'src'))
        shutil.copytree(os.path.join(REF, 'tools'), os.path.join(tmp, 'tools'))
        subprocess.run([sys.executable, os.path.join(tmp, 'tools', 'generate_lut.py')], check=True,
                       stdout=subprocess.DEVNULL)
        fakebin = os.path.join(tmp, 'fakebin')
        os.makedirs(fakebin)
        for name in ('ffmpeg', 'ffprobe'):
            p = os.path.join(fakebin, name)
            with open(p, 'w') as f:
                f.write('#!/bin/sh\nexit 1\n')
            os.chmod(p, os.stat(p).st_mode | stat.S_IEXEC)
        env = dict(os.environ, PATH=fakebin + os.pathsep + os.environ.get('PATH', ''))
        res = subprocess.run([sys.executable, '-c', RULES_SCRIPT, tmp], env=env, check=True,
                             stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
        data = json.loads(res.stdout.strip().splitlines()[-1])
        data['source'] = ('src/ffmpeg_command.py build() over a request/probe matrix and src/utils.py '
                          'FFMPEG_FILTER / build_libplacebo_filter preview chains (reference, imported)')
        with open(os.path.join(HERE, 'request_rules.json'), 'w') as f:
            json.dump(data, f, indent=1, sort_keys=True)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def main() -> None:
    only = sys.argv[1:]
    gen = load_generator()
    if not only or 'lut' in only:
        lut_goldens(gen)
        convert_goldens(gen)
    if not only or 'chains' in only:
        chain_goldens()
    if not only or 'rules' in only:
        rules_goldens()
    print('golden fixtures written to', HERE)


if __name__ == '__main__':
    main()
