"""bench.py's multi-rank launch on CPU: a plain
``python bench.py --gpus 2`` with no WORLD_SIZE starts torch.distributed.run
itself (one rank per GPU, rendezvous on 127.0.0.1); --dry-run runs the
params / lattice broadcast and the SUM / MAX reduction under gloo with no GPU
work, so rank 0's line shows the world size the collectives saw."""
import json
import os
import subprocess
import sys

from conftest import REPO

BENCH = os.path.join(REPO, 'bench.py')


def _run(args, **env):
    e = dict(os.environ)
    e.pop('WORLD_SIZE', None)
    e.update(env)
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True, timeout=300, env=e)


def test_plain_gpus2_spawns_two_ranks_under_gloo():
    out = _run(['--gpus', '2', '--dry-run', '--frames', '3'])
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [json.loads(l) for l in out.stdout.splitlines() if l.startswith('{')]
    assert len(lines) == 1                              # rank 0 prints the one line
    rec = lines[0]
    assert rec['n_gpus'] == 2 and rec['world_size'] == 2
    assert rec['pixels'] == 2 * 3 * 3840 * 2160         # SUM over ranks: each rank's 3-frame shard
    assert rec['max_elapsed_s'] == 0.002                # MAX over ranks (rank r reports 0.001 (r + 1))
    assert rec['gamma'] == 2.2 and rec['lattice_sum'] > 0   # rank 0's params / lattice reached rank 1
    # the line carries BASELINE's multi-GPU configurations beside C2, each
    # sharded over both ranks
    assert rec['config']['workload'].startswith('C2')
    sh = rec['config']['sharded_configs']
    assert sh['C4']['workload'].startswith('C4') and 'mobius' in sh['C4']['workload']
    assert sh['C5']['workload'].startswith('C5') and '7680x4320' in sh['C5']['workload']
    assert sh['C4']['pixels'] == 2 * 64 * 3840 * 2160 and sh['C4']['frames_total'] == 128
    assert sh['C5']['pixels'] == 2 * 16 * 7680 * 4320
    assert sh['C4']['max_elapsed_s'] == 0.002


def test_gpus_must_equal_world_size():
    out = _run(['--gpus', '2', '--dry-run'], WORLD_SIZE='1')
    assert out.returncode == 2 and 'WORLD_SIZE' in out.stderr
