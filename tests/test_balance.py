"""Load balancer (lddl_amd.balance) vs the reference's own load_balance.py
outputs (tests/golden/balance.json.gz, tools/gen_golden_balance.py), and the
multi-rank count gather / shard ownership over gloo (world size 2)."""
import gzip
import json
import sys
import os

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq
import pytest
import torch.multiprocessing as mp

from lddl_amd import balance

GOLD = json.load(gzip.open(os.path.join(os.path.dirname(__file__), 'golden', 'balance.json.gz'), 'rt'))
CASES = GOLD['cases']


@pytest.mark.parametrize('k', range(len(CASES)))
@pytest.mark.parametrize('strict', [False, True])
def test_plan_matches_reference(k, strict):
  c = CASES[k]
  if c['error'] == 'TypeError':  # more shards than files
    with pytest.raises(ValueError):
      balance.plan_files(c['files'], c['counts'], c['num_shards'], c['bin_ids'], strict)
    return
  if c['error'] == 'TimeoutError':  # the reference never finishes
    if strict:
      with pytest.raises(RuntimeError, match='load balance cannot finish'):
        balance.plan_files(c['files'], c['counts'], c['num_shards'], c['bin_ids'], strict)
      return
    shards, ns = balance.plan_files(c['files'], c['counts'], c['num_shards'], c['bin_ids'], strict)
    for b in sorted({n.split('.parquet')[1] for n in ns}):
      v = [n for name, n in ns.items() if name.split('.parquet')[1] == b]
      assert len(v) == c['num_shards'] and max(v) - min(v) <= 1
    assert sum(ns.values()) == sum(c['counts'])
    return
  shards, ns = balance.plan_files(c['files'], c['counts'], c['num_shards'], c['bin_ids'], strict)
  idx = {n: i for i, n in enumerate(c['files'])}
  got = {name: [[idx[p], r0, n] for p, r0, n in runs] for name, runs, _ in shards}
  assert got == c['shards']
  assert list(ns.items()) == list(c['num_samples'].items())  # .num_samples.json incl. key order
  if len(shards):
    assert max(ns.values()) - min(ns.values()) <= 1 or c['bin_ids'] is not None or any(
        '_' in os.path.splitext(f)[1] for f in c['files'])


def _write_inputs(d, c):
  for i, (nm, n) in enumerate(zip(c['files'], c['counts'])):
    pq.write_table(pa.table({'rid': (np.int64(i) << 32) + np.arange(n, dtype=np.int64)}), os.path.join(d, nm))


def _runs_of(path):
  out = []
  for v in pq.read_table(path).column('rid').to_numpy():
    f, r = int(v) >> 32, int(v) & 0xFFFFFFFF
    if out and out[-1][0] == f and out[-1][1] + out[-1][2] == r:
      out[-1][2] += 1
    else:
      out.append([f, r, 1])
  return out


@pytest.mark.parametrize('k', [i for i, c in enumerate(CASES) if not c['error']][:12])
def test_cli_writes_reference_shards(tmp_path, k):
  c = CASES[k]
  ind, outd = tmp_path / 'in', tmp_path / 'out'
  ind.mkdir()
  _write_inputs(str(ind), c)
  args = balance.attach_args().parse_args(['--indir', str(ind), '--outdir', str(outd), '--num-shards',
                                           str(c['num_shards']), '--keep-orig'])
  balance.main(args)
  for name, runs in c['shards'].items():
    assert _runs_of(str(outd / name)) == runs
  with open(str(outd / '.num_samples.json')) as f:
    assert list(json.load(f).items()) == list(c['num_samples'].items())


def test_balance_counts_names():
  counts = np.array([[3, 1], [0, 5], [7, 2]])
  shards, ns = balance.balance_counts(counts, 2, binned=True)
  assert sorted(ns) == ['shard-0.parquet_0', 'shard-0.parquet_1', 'shard-1.parquet_0', 'shard-1.parquet_1']
  assert ns['shard-0.parquet_0'] + ns['shard-1.parquet_0'] == 10
  shards, ns = balance.balance_counts(counts, 3, binned=False)
  assert sorted(ns.values()) == [6, 6, 6]


def _rank(rank, world, port, d, counts, parts, q):
  import torch
  import torch.distributed as dist
  os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
  dist.init_process_group('gloo', rank=rank, world_size=world)
  lo, hi = parts[rank]
  got = balance.gather_bin_counts(torch.from_numpy(counts[lo:hi]), lo)
  shards, ns = balance.balance_counts(got, 3, binned=True, outdir=d)
  written = balance.write_shards(shards, os.path.join(d, 'out'), rank, world)
  q.put((rank, got.tolist(), sorted(os.path.basename(w) for w in written)))
  dist.barrier()
  dist.destroy_process_group()


def test_gather_and_ownership_gloo(tmp_path):
  """world size 2: counts of unequal partition ranges gathered, every rank
  computes the same plan, shard k written by rank k % 2, union = 1-rank run"""
  rng = np.random.default_rng(5)
  counts = rng.integers(0, 30, (7, 4)).astype(np.int64)
  d = str(tmp_path)
  names = ['part.%d.parquet_%d' % (p, b) for p in range(7) for b in range(4)]
  _write_inputs(d, {'files': names, 'counts': counts.ravel().tolist()})
  ctx = mp.get_context('spawn')
  q = ctx.Queue()
  port = 29500 + os.getpid() % 1000
  procs = [ctx.Process(target=_rank, args=(r, 2, port, d, counts, [(0, 3), (3, 7)], q)) for r in range(2)]
  for p in procs:
    p.start()
  res = sorted(q.get(timeout=120) for _ in range(2))
  for p in procs:
    p.join(60)
    assert p.exitcode == 0
  assert res[0][1] == counts.tolist() and res[1][1] == counts.tolist()
  assert all(int(n.split('-')[1].split('.')[0]) % 2 == r for r, _, ws in res for n in ws)
  shards, ns = balance.balance_counts(counts, 3, binned=True, outdir=d)
  assert sorted(res[0][2] + res[1][2]) == sorted(ns)
  for name, runs, n in shards:
    t = pq.read_table(os.path.join(d, 'out', name))
    assert t.num_rows == n


def _clean_env(**kw):
  env = {k: v for k, v in os.environ.items()
         if k not in ('RANK', 'WORLD_SIZE', 'LOCAL_RANK', 'MASTER_ADDR', 'MASTER_PORT') and not k.startswith(
             ('OMPI_', 'PMI', 'SLURM_'))}
  env.update(kw)
  return env


def test_cli_under_mpirun_env_only(tmp_path):
  """under mpirun the ranks have OMPI_COMM_WORLD_RANK / _SIZE and
  a job id, no MASTER_ADDR: the balancer meets through the shared-file
  barrier (or mpi4py when importable), rank 0 removes the inputs and writes
  .num_samples.json once both ranks have written their shards -- the same
  outputs as one rank"""
  import subprocess
  import sys
  c = next(c for c in CASES if not c['error'])
  ref_in, ref_out = tmp_path / 'ref_in', tmp_path / 'ref_out'
  ref_in.mkdir()
  _write_inputs(str(ref_in), c)
  balance.main(balance.attach_args().parse_args(['--indir', str(ref_in), '--outdir', str(ref_out), '--num-shards',
                                                 str(c['num_shards'])]), 0, 1)
  ind, outd = tmp_path / 'in', tmp_path / 'out'
  ind.mkdir()
  _write_inputs(str(ind), c)
  root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
  cmd = [sys.executable, '-m', 'lddl_amd.balance', '--indir', str(ind), '--outdir', str(outd), '--num-shards',
         str(c['num_shards'])]
  procs = [subprocess.Popen(cmd, cwd=root, env=_clean_env(OMPI_COMM_WORLD_RANK=str(r), OMPI_COMM_WORLD_SIZE='2',
                                                          OMPI_MCA_ess_base_jobid='4242'),
                            stdout=subprocess.PIPE, stderr=subprocess.PIPE) for r in range(2)]
  outs = [p.communicate(timeout=240) for p in procs]
  assert [p.returncode for p in procs] == [0, 0], outs
  want = sorted(n for n in os.listdir(str(ref_out)))
  assert sorted(os.listdir(str(outd))) == want  # no barrier markers left, inputs gone, .num_samples.json
  for n in want:
    if n.startswith('shard-'):
      assert _runs_of(str(outd / n)) == _runs_of(str(ref_out / n))
  with open(str(outd / '.num_samples.json')) as f, open(str(ref_out / '.num_samples.json')) as g:
    assert json.load(f) == json.load(g)
  assert not [n for n in os.listdir(str(ind)) if n.startswith('part.')]


def test_ranks_without_a_meeting_point_fail_before_writing(tmp_path):
  import subprocess
  import sys
  c = next(c for c in CASES if not c['error'])
  ind, outd = tmp_path / 'in', tmp_path / 'out'
  ind.mkdir()
  _write_inputs(str(ind), c)
  root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
  p = subprocess.run([sys.executable, '-m', 'lddl_amd.balance', '--indir', str(ind), '--outdir', str(outd),
                      '--num-shards', str(c['num_shards'])], cwd=root, capture_output=True, text=True, timeout=120,
                     env=_clean_env(OMPI_COMM_WORLD_RANK='1', OMPI_COMM_WORLD_SIZE='2'))
  try:
    import mpi4py  # noqa: F401
    pytest.skip('mpi4py importable: the ranks meet through it')
  except ImportError:
    pass
  assert p.returncode != 0 and 'no way to meet' in p.stderr
  assert not outd.exists() or not os.listdir(str(outd))


def test_mpi4py_singleton_world_is_not_a_barrier(monkeypatch):
  """an mpi4py whose COMM_WORLD is a singleton (srun without PMI,
  another MPI) must not be taken as the launch's barrier"""
  import sys
  import types

  class _W:
    def __init__(self, size, rank):
      self.s, self.r = size, rank

    def Get_size(self):
      return self.s

    def Get_rank(self):
      return self.r

  for k in ('MASTER_ADDR', 'MASTER_PORT') + balance._JOB_ENV:
    monkeypatch.delenv(k, raising=False)
  mod, mpi = types.ModuleType('mpi4py'), types.ModuleType('mpi4py.MPI')
  mod.MPI = mpi
  monkeypatch.setitem(sys.modules, 'mpi4py', mod)
  monkeypatch.setitem(sys.modules, 'mpi4py.MPI', mpi)
  mpi.COMM_WORLD = _W(1, 0)
  with pytest.raises(ValueError):
    balance.barrier_kind(2, 1)
  monkeypatch.setenv('PMIX_NAMESPACE', 'ns7')
  assert balance.barrier_kind(2, 1) == 'file'
  mpi.COMM_WORLD = _W(2, 1)
  assert balance.barrier_kind(2, 1) == 'mpi4py'


def test_file_barrier_ignores_markers_of_an_earlier_launch(tmp_path, monkeypatch):
  """a crashed earlier launch with the same job id left rank 1's
  marker; rank 0 must not pass the barrier on it"""
  for k in balance._JOB_ENV:
    monkeypatch.delenv(k, raising=False)
  monkeypatch.setenv('SLURM_JOB_ID', '77')
  monkeypatch.setenv('PMIX_NAMESPACE', 'launch-b')
  assert balance.job_id() == 'launch-b'  # the per-launch id wins over the allocation's
  stale = tmp_path / '.lddl_barrier.launch-b.1'
  stale.write_text('done\n')
  os.utime(str(stale), (1e9, 1e9))
  with pytest.raises(RuntimeError):
    balance._file_barrier(str(tmp_path), 0, 2, timeout=0.3)
  stale.write_text('done\n')  # a marker of this launch
  balance._file_barrier(str(tmp_path), 0, 2, timeout=5)
  assert not [n for n in os.listdir(str(tmp_path)) if n.startswith('.lddl_barrier')]


def test_mpi4py_not_initialised_without_an_mpi_launcher(monkeypatch):
  """outside mpirun / srun (no launcher environment) barrier_kind
  never imports mpi4py.MPI (its MPI_Init can abort the process)"""
  import types
  for k in ('MASTER_ADDR', 'MASTER_PORT') + balance._JOB_ENV + balance._MPI_ENV:
    monkeypatch.delenv(k, raising=False)
  mod = types.ModuleType('mpi4py')

  class _Boom(types.ModuleType):
    def __getattr__(self, name):
      raise AssertionError('mpi4py.MPI touched')
  monkeypatch.setitem(sys.modules, 'mpi4py', mod)
  monkeypatch.setitem(sys.modules, 'mpi4py.MPI', _Boom('mpi4py.MPI'))
  mod.MPI = sys.modules['mpi4py.MPI']
  monkeypatch.setenv('SLURM_JOB_ID', '5')
  assert balance.barrier_kind(2, 0) == 'file'


def test_file_barrier_markers_carry_the_launch_nonce(tmp_path, monkeypatch):
  """with rank 0's reference file a marker counts when it holds
  the file's nonce: a marker of an earlier launch with the same job tag is
  refused however fresh its mtime (a fast requeue), one of this launch is
  taken however old (another node's clock behind)"""
  for k in balance._JOB_ENV:
    monkeypatch.delenv(k, raising=False)
  monkeypatch.setenv('PMIX_NAMESPACE', 'launch-c')
  monkeypatch.setattr(balance, '_launch_start', lambda: 2e9)  # a local clock far ahead of the file server's
  d = str(tmp_path)
  balance.file_barrier_ref(d, 0)
  old_nonce = (tmp_path / '.lddl_barrier.launch-c.ref').read_text()
  balance._file_barrier(d, 1, 2)  # an earlier launch's rank 1 ...
  balance.file_barrier_ref(d, 0)  # ... then this launch's rank 0
  ref = tmp_path / '.lddl_barrier.launch-c.ref'
  assert ref.read_text() != old_nonce
  m1 = tmp_path / '.lddl_barrier.launch-c.1'
  assert m1.read_text() == old_nonce
  with pytest.raises(RuntimeError):
    balance._file_barrier(d, 0, 2, timeout=0.3)
  balance._file_barrier(d, 1, 2)  # this launch's rank 1
  os.utime(str(m1), (1e9, 1e9))
  balance._file_barrier(d, 0, 2, timeout=5)
  assert not [n for n in os.listdir(d) if n.startswith('.lddl_barrier')]


NSC = json.load(open(os.path.join(os.path.dirname(__file__), 'golden', 'num_samples_cache.json')))


def _nsc_tree(d):
  for rel, n in NSC['files']:
    p = os.path.join(d, rel)
    os.makedirs(os.path.dirname(p), exist_ok=True)
    pq.write_table(pa.table({'A': pa.array(['a %d' % i for i in range(n)], pa.string()),
                             'num_tokens': pa.array(np.arange(n, dtype=np.uint16))}), p)
  for rel in NSC['other']:
    with open(os.path.join(d, rel), 'w') as f:
      f.write('x\n')


def test_num_samples_cache_matches_reference(tmp_path):
  """generate_num_samples_cache (load_balance.py:428-455): the same bytes as
  the reference's .num_samples.json over the same tree (golden written by
  tools/gen_golden_num_samples.py from the reference with a one-rank MPI stub)"""
  _nsc_tree(str(tmp_path))
  ns = balance.num_samples_cache(str(tmp_path), 0, 1)
  with open(str(tmp_path / '.num_samples.json')) as f:
    assert f.read() == NSC['num_samples_json']
  assert list(ns.items()) == list(json.loads(NSC['num_samples_json']).items())


def test_num_samples_cache_console(tmp_path):
  import subprocess
  _nsc_tree(str(tmp_path))
  root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
  p = subprocess.run([sys.executable, '-m', 'lddl_amd.balance', '--num-samples-cache', '--indir', str(tmp_path)],
                     cwd=root, capture_output=True, text=True, timeout=120, env=_clean_env())
  assert p.returncode == 0, p.stderr
  with open(str(tmp_path / '.num_samples.json')) as f:
    assert f.read() == NSC['num_samples_json']


def _nsc_rank(rank, world, port, d, q):
  os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
  import torch.distributed as dist
  dist.init_process_group('gloo', rank=rank, world_size=world)
  try:
    q.put((rank, balance.num_samples_cache(d, rank, world)))
  finally:
    dist.destroy_process_group()


@pytest.mark.parametrize('world', [2, 3])
def test_num_samples_cache_gloo(tmp_path, world):
  """ranks read the footers of one block of the files each and all-gather the
  counts (gather_bin_counts): every rank gets the whole dict, rank 0 writes
  the reference's bytes"""
  import socket
  _nsc_tree(str(tmp_path))
  with socket.socket() as s:
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
  ctx = mp.get_context('spawn')
  q = ctx.Queue()
  ps = [ctx.Process(target=_nsc_rank, args=(r, world, port, str(tmp_path), q)) for r in range(world)]
  for p in ps:
    p.start()
  got = dict(q.get(timeout=120) for _ in range(world))
  for p in ps:
    p.join(60)
  assert all(p.exitcode == 0 for p in ps)
  want = json.loads(NSC['num_samples_json'])
  assert all(list(got[r].items()) == list(want.items()) for r in range(world))
  with open(str(tmp_path / '.num_samples.json')) as f:
    assert f.read() == NSC['num_samples_json']
