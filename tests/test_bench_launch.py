"""bench.py --gpus N starts N ranks itself when no launcher env is set (the
driver's `python bench.py --gpus N` form), and the all-gather of the
per-(partition, bin) counts -- the exchange replacing
lddl/dask/load_balance.py:222-233 -- sees every rank.  CPU only: --launch-check
runs the world-dependent part over gloo, no GPU kernels."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args, env_extra=None):
  env = {k: v for k, v in os.environ.items() if k not in ('RANK', 'WORLD_SIZE', 'LOCAL_RANK', 'MASTER_ADDR',
                                                          'MASTER_PORT')}
  env.update(env_extra or {})
  p = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py')] + list(args), env=env, capture_output=True,
                     text=True, timeout=240)
  return p


@pytest.mark.parametrize('n', [1, 2, 3])
def test_launch_n_ranks(n):
  p = _run('--gpus', str(n), '--launch-check')
  assert p.returncode == 0, p.stderr[-2000:]
  lines = [l for l in p.stdout.splitlines() if l.startswith('{')]
  assert len(lines) == 1, p.stdout  # rank 0 only
  d = json.loads(lines[0])
  assert d['n_gpus'] == n
  assert d['gathered_partitions'] == n * d['partitions_per_rank']
  assert d['parallelism'] == 'shard%d' % n


def test_gpus_world_mismatch_fails():
  p = _run('--gpus', '2', '--launch-check', env_extra={'WORLD_SIZE': '1', 'RANK': '0'})
  assert p.returncode != 0
  assert 'WORLD_SIZE' in p.stderr


def test_check_gather_detects_missing_rank():
  import numpy as np
  sys.path.insert(0, ROOT)
  import bench
  own = np.arange(6).reshape(3, 2)
  assert bench.check_gather(np.concatenate([own, own + 10]), own, 0, 2) == 6
  with pytest.raises(RuntimeError):
    bench.check_gather(own, own, 0, 2)
