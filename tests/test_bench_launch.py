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


STUB = r'''#!/usr/bin/env python3
# stub hipcc (tests/test_bench_launch.py): logs each call; -c writes a dummy
# object, the link a real (empty) shared library, slowly, to widen any race
import os, subprocess, sys, time
a = sys.argv[1:]
with open(os.environ['STUB_LOG'], 'a') as f:
  f.write(('compile ' if '-c' in a else 'link ') + a[a.index('-o') + 1] + '\n')
out = a[a.index('-o') + 1]
time.sleep(0.3)
if '-c' in a:
  open(out, 'w').write('obj')
else:
  src = out + '.c'
  open(src, 'w').write('int lddl_stub_lib(void) { return 7; }\n')
  subprocess.run(['gcc', '-shared', '-fPIC', '-o', out, src], check=True)
  os.remove(src)
'''


def _stub_env(tmp_path):
  stub = tmp_path / 'hipcc'
  stub.write_text(STUB)
  stub.chmod(0o755)
  log = tmp_path / 'calls.log'
  return {'LDDL_HIPCC': str(stub), 'LDDL_BUILD_LIB': str(tmp_path / 'lib' / 'liblddl_stub.so'), 'STUB_LOG': str(log)}, log


def test_one_build_for_n_ranks(tmp_path):
  """bench.py --gpus 3 against a stale (absent) library: the launching process
  builds once before the ranks start; every rank's build is then a no-op and
  all of them load the same library"""
  import glob
  (tmp_path / 'lib').mkdir()
  env, log = _stub_env(tmp_path)
  p = _run('--gpus', '3', '--launch-check', '--build-check', env_extra=env)
  assert p.returncode == 0, p.stderr[-2000:]
  d = json.loads([l for l in p.stdout.splitlines() if l.startswith('{')][0])
  calls = log.read_text().splitlines()
  n_src = len(glob.glob(os.path.join(ROOT, 'lddl_amd', 'csrc', '*.hip')))
  assert sum(c.startswith('compile') for c in calls) == n_src, calls
  assert sum(c.startswith('link') for c in calls) == 1, calls
  assert len(d['libs']) == 3 and len({tuple(x) for x in d['libs']}) == 1, d['libs']
  assert d['libs'][0][0] == env['LDDL_BUILD_LIB']


def test_concurrent_builds_serialise(tmp_path):
  """three processes calling build_hip at once on a stale library (ranks
  started by torchrun, no parent build): one compiles, the others wait for
  the lock and find it built; no torn temporaries"""
  import glob
  (tmp_path / 'lib').mkdir()
  env, log = _stub_env(tmp_path)
  full = dict(os.environ, **env)
  code = 'import sys; sys.path.insert(0, %r); from lddl_amd import build; print(build.build_hip())' % ROOT
  ps = [subprocess.Popen([sys.executable, '-c', code], env=full, stdout=subprocess.PIPE, text=True) for _ in range(3)]
  outs = [p.communicate(timeout=240)[0].strip() for p in ps]
  assert all(p.returncode == 0 for p in ps)
  assert outs == [env['LDDL_BUILD_LIB']] * 3
  calls = log.read_text().splitlines()
  n_src = len(glob.glob(os.path.join(ROOT, 'lddl_amd', 'csrc', '*.hip')))
  assert sum(c.startswith('compile') for c in calls) == n_src and sum(c.startswith('link') for c in calls) == 1, calls
  assert not [f for f in os.listdir(tmp_path / 'lib') if '.tmp' in f]
