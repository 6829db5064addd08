"""The float gate has teeth, on the CPU.

tests/float_gate.py states what check_float_stage allows beyond north_star's
1e-3 relative on the float path (the EOTF's conditioning, desaturation's
kink, Hable's cancellation, the IPT rows, the lattice slope, the download's
rounding boundary).  Those allowances must not swallow real errors: for every
(kernel, config, content, stage) of the GPU float suite, the gate applied to
the oracle's own planes

* accepts them unchanged;
* rejects them with ONE value off by 2e-3 relative -- the kept value of median
  magnitude among those the gate does not excuse for a stated reason (its
  allowance there is below 2e-3 relative; on the libplacebo branch after the
  download, a pixel away from the rounding boundary);
* rejects them with 1 % of the kept values (seeded) off by 1.2e-3 relative;

and the share of values it does excuse beyond 2e-3 relative ('loose') is
bounded per content and reported.  No GPU: the kernels' planes are replaced by
mutated copies of the oracle's."""
import functools

import numpy as np
import pytest

import hdr2sdr
from hdr2sdr.synth import synth_frames
from float_gate import FLOAT_CFGS, Planes, float_tolerance, judge_float

W, H = 128, 64


def loose_max(params, kernel, stage):
    """The share of the values with a relative scale (float_gate.judge_float)
    that the gate may excuse beyond 2e-3 relative, measured on these frames
     with margin: <= 10 % at stages 1-4; the tile kernel's IPT
    form on the libplacebo branch carries its tables' LMS error (EPS_IPT)
    through rows that cancel on saturated colours, up to 25 % at stages 2-5
    (measured <= 17 % with round 5's EPS_IPT 2e-5; 50 % before, at 1e-4);
    stage 5's chroma of nearly neutral colours carries the lattice's slope
    next to black (up to 9.5 per unit) at the quantiser's scale, up to 35 %."""
    if kernel == 'k_tile' and params.resolved_pipeline() == 'libplacebo' and params.lp_tone == 'ipt' and stage >= 2:
        return 0.25
    if stage == 5:
        return 0.35
    return 0.10


@functools.lru_cache(maxsize=None)
def _planes(cfg, kind):
    params = hdr2sdr.TonemapParams(**FLOAT_CFGS[cfg])
    src = synth_frames(kind, 1, W, H, params.bits_in, device='cpu', seed=3).to_numpy()
    return params, Planes(params, src.buf, W, H)


def _judge(params, kernel, kind, stage, T, got):
    return judge_float(params, kernel, kind, stage, got, T)


@pytest.mark.parametrize('stage', [1, 2, 3, 4, 5])
@pytest.mark.parametrize('kind', ['uniform', 'edges', 'ramp'])
@pytest.mark.parametrize('cfg', sorted(FLOAT_CFGS))
@pytest.mark.parametrize('kernel', ['k_tile', 'k_debug'])
def test_gate_accepts_the_oracle_and_rejects_mutations(kernel, cfg, kind, stage):
    params, P = _planes(cfg, kind)
    T = float_tolerance(params, kernel, stage, kind, P)
    want = T.want
    rep, fails = _judge(params, kernel, kind, stage, T, want.copy())
    assert not fails, fails
    assert rep['loose_frac'] <= loose_max(params, kernel, stage), f"{rep['loose_frac']:.2%} of values excused beyond 2e-3"

    aw = np.abs(want)
    with np.errstate(invalid='ignore'):
        tight = T.scaled & np.isfinite(want) & (T.tol < 2e-3 * aw)
    if T.near_tie is not None:
        tight &= ~T.near_tie[None]
    assert tight.any()
    # one value off by 2e-3 relative: the median-magnitude tight value
    idx = np.flatnonzero(tight.ravel())
    pick = idx[np.argsort(aw.ravel()[idx])[len(idx) // 2]]
    got = want.copy().ravel()
    got[pick] *= 1.0 + 2e-3
    _, fails = _judge(params, kernel, kind, stage, T, got.reshape(want.shape))
    assert fails, f'a 2e-3 error on one value (|want| {aw.ravel()[pick]:.4g}) passed the gate'

    # 1 % of the kept values off by 1.2e-3 relative
    rng = np.random.default_rng(1234 + stage)
    kept = np.flatnonzero((T.keep & np.isfinite(want)).ravel())
    sel = rng.choice(kept, size=max(1, len(kept) // 100), replace=False)
    got = want.copy().ravel()
    got[sel] *= 1.0 + 1.2e-3
    _, fails = _judge(params, kernel, kind, stage, T, got.reshape(want.shape))
    assert fails, 'a 1.2e-3 error on 1 % of the values passed the gate'
