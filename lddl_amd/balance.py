"""Load balancer for the parquet shards (reference: lddl/dask/load_balance.py).

The reference balances the preprocessor's files ``part.{i}.parquet[_b]`` into
``--num-shards`` files ``shard-{k}.parquet[_b]`` whose sample counts differ
by at most one, per bin, and writes ``.num_samples.json``
(load_balance.py:372-378).  It counts rows by reading every file under MPI
(``_build_files`` + Allreduce, :222-233), then moves rows in pairwise steps
(``Shard.balance`` :129-140, ``Progress.report`` :190-203) that re-read and
re-write intermediate shard files on every step.

Here the same pairwise procedure runs on *row runs* instead of tables:
``plan()`` replays it exactly -- same file order (lexicographic paths, then a
stable sort by count), same pops from the back, same split of partially
consumed files, same pairing order -- and yields, per output shard, the list
of (file, first row, row count) runs it ends up holding.  Each shard is then
written once, by rank ``k % world``, from slices of the source files.  The
row counts need no file reads: on the GPU path they are the packer's
per-(partition, bin) counts, gathered over ranks with one all-gather
(RCCL on the GPUs, ``gather_bin_counts``) in place of the MPI Allreduce.

Where the reference cannot finish, this raises instead:
  * more shards than files: Shard._input_files is None (:240-242) and
    flush()/_load() raise TypeError -> ValueError here;
  * a total divisible by --num-shards keeps a zero-count target (:163-167);
    a shard passing through exactly base+1 samples is then taken as ready and
    the loop never ends (or ends with a shard never flushed).  By default the
    zero-count target is dropped, which changes nothing in any run the
    reference finishes correctly (the key only matters once a shard reaches
    it, which is exactly the failure) and finishes the others balanced;
    strict=True keeps it and raises RuntimeError at the first iteration that
    can pair no shards.
"""
import argparse
import json
import os
import re
import time

import numpy as np

__all__ = ['plan', 'plan_files', 'write_shards', 'gather_bin_counts', 'balance_counts', 'main', 'num_samples_cache',
           'generate_num_samples_cache']


class _Shard:
  """load_balance.py:42-157 Shard, holding runs [file, first_row, n] instead of tables."""

  def __init__(self, idx, inputs, counts, postfix):
    self.idx = idx
    self.inputs = inputs  # list of file indices (popped from the back) or None
    self.counts = counts
    self.postfix = postfix
    self.out = None       # runs of the output file, or None (no file yet)
    self.out_n = 0

  @property
  def num_samples(self):
    n = sum(self.counts[f] for f in self.inputs) if self.inputs is not None else 0
    return n + (self.out_n if self.out is not None else 0)

  @property
  def name(self):
    return 'shard-{}.parquet{}'.format(self.idx, self.postfix)

  def _store(self, n, runs):
    if self.out is None:
      self.out, self.out_n = [], 0
    self.out.extend(r for r in runs if r[2] > 0)
    self.out_n += n

  def _load(self, n):
    if self.inputs is None:
      raise ValueError('more shards than files (the reference fails here: load_balance.py:240-242)')
    taken = []
    while n > 0:
      if self.inputs:
        f = self.inputs.pop()
        runs, fn = [[f, 0, self.counts[f]]], self.counts[f]
      else:
        runs, fn = self.out, self.out_n
        self.out, self.out_n = None, 0
      k = min(fn, n)
      head, tail = _split(runs, k)
      taken.extend(head)
      if k < fn:
        self._store(fn - k, tail)
      n -= k
    return taken

  def balance(self, smaller):
    n = self.num_samples - (self.num_samples + smaller.num_samples) // 2
    smaller._store(n, self._load(n))

  def flush(self):
    if self.inputs is None:
      raise ValueError('more shards than files (the reference fails here: load_balance.py:143-148)')
    runs, n = [], 0
    while self.inputs:
      f = self.inputs.pop()
      n += self.counts[f]
      runs.append([f, 0, self.counts[f]])
    if n > 0:
      self._store(n, runs)


def _split(runs, k):
  head, tail = [], []
  for f, r0, n in runs:
    if k >= n:
      head.append([f, r0, n])
      k -= n
    elif k > 0:
      head.append([f, r0, k])
      tail.append([f, r0 + k, n - k])
      k = 0
    else:
      tail.append([f, r0, n])
  return head, tail


class _Progress:
  """load_balance.py:160-207 Progress (targets dict kept verbatim)."""

  def __init__(self, shards, strict):
    n = len(shards)
    total = sum(s.num_samples for s in shards)
    base = total // n
    self.targets = {base: n - total % n, base + 1: total % n}
    if not strict:
      self.targets = {k: v for k, v in self.targets.items() if v > 0}
    self.ready = []

  def completed(self):
    return sum(self.targets.values()) == 0

  def report(self, shards):
    smaller, larger = [], []
    for s in shards:
      ns = s.num_samples
      if ns in self.targets:
        self.targets[ns] -= 1
        self.ready.append(s)
        if self.targets[ns] == 0:
          del self.targets[ns]
      elif ns < min(self.targets.keys()):
        smaller.append(s)
      else:
        larger.append(s)
    return smaller, larger


def plan(counts, num_shards, postfix='', strict=False):
  """Replay load_balance.py:_balance (:281-322) over files with the given row
  counts (in the reference's path order).  Returns the ready shards in the
  reference's order as (shard file name, runs, num_samples); runs are
  [file index, first row, n] in row order."""
  counts = [int(c) for c in counts]
  if num_shards < 1:
    raise ValueError('--num-shards must be >= 1')
  order = sorted(range(len(counts)), key=lambda i: counts[i])  # _build_files: stable sort by count
  shards = [_Shard(k, order[k::num_shards] if k < len(order) else None, counts, postfix)
            for k in range(num_shards)]
  progress = _Progress(shards, strict)
  while not progress.completed():
    smaller, larger = progress.report(shards)
    smaller = sorted(smaller, key=lambda s: s.num_samples)
    larger = sorted(larger, key=lambda s: s.num_samples, reverse=True)
    npairs = min(len(smaller), len(larger))
    for s, l in zip(smaller[:npairs], larger[:npairs]):
      l.balance(s)
    if npairs == 0 and not progress.completed():
      raise RuntimeError('load balance cannot finish: %d samples over %d shards leaves shards it can no longer '
                         'pair (the reference loops forever here, load_balance.py:163-167,302-322)'
                         % (sum(counts), num_shards))
    shards = smaller + larger
  for s in progress.ready:
    s.flush()
  out = []
  for s in progress.ready:
    if s.out is None:
      raise ValueError('shard %d ends with no samples (the reference fails here: load_balance.py:327-330)' % s.idx)
    out.append((s.name, _merge(s.out), s.out_n))
  return out


def _merge(runs):
  """adjacent runs of the same file back to back -> one run"""
  out = []
  for f, r0, n in runs:
    if out and out[-1][0] == f and out[-1][1] + out[-1][2] == r0:
      out[-1][2] += n
    else:
      out.append([f, r0, n])
  return out


def _bin_of(name):
  ext = os.path.splitext(name)[1]
  return int(ext.split('_')[-1]) if '_' in ext else None


def plan_files(names, counts, num_shards, bin_ids=None, strict=False):
  """load_balance.py:main (:333-369) over (file path, row count) pairs:
  per bin (or unbinned) the files in sorted path order, then plan().
  Returns (list of (shard name, [(path, first_row, n)], num_samples),
  num_samples dict in the reference's .num_samples.json order)."""
  by_name = dict(zip(names, counts))
  paths = sorted(p for p in names if '.parquet' in os.path.splitext(p)[1])  # get_all_parquets_under
  if bin_ids is None:
    found = sorted({_bin_of(p) for p in paths if _bin_of(p) is not None})
    if found != list(range(len(found))):
      raise ValueError('bin id must be contiguous integers starting from 0!')
    bin_ids = found or None
  groups = [(paths, '')] if bin_ids is None else [
      ([p for p in paths if os.path.splitext(p)[1] == '.parquet_{}'.format(b)], '_{}'.format(b)) for b in bin_ids]
  shards = []
  for gp, postfix in groups:
    for name, runs, n in plan([by_name[p] for p in gp], num_shards, postfix, strict):
      shards.append((name, [(gp[f], r0, k) for f, r0, k in runs], n))
  return shards, {name: n for name, _, n in shards}


def write_shards(shards, outdir, rank=0, world=1, compression='snappy'):
  """Write every planned shard owned by this rank (shard k -> rank k % world,
  the reference's idx % world ownership) from slices of its source files.
  Returns the written paths."""
  import pyarrow as pa
  import pyarrow.parquet as pq
  os.makedirs(outdir, exist_ok=True)
  written = []
  cache = {}
  for name, runs, n in shards:
    k = int(name.split('-')[1].split('.')[0])
    if k % world != rank:
      continue
    parts = []
    for path, r0, cnt in runs:
      if path not in cache:
        cache.clear()  # runs of a shard mostly come from few files: keep the last one
        cache[path] = pq.read_table(path)
      parts.append(cache[path].slice(r0, cnt))
    t = pa.concat_tables(parts) if parts else None
    if t is None:
      raise ValueError('shard %s has no rows' % name)
    assert t.num_rows == n, (name, t.num_rows, n)
    path = os.path.join(outdir, name)
    from .hostinfo import DENSE_COLS
    pq.write_table(t, path, compression=compression,
                   use_dictionary=[c for c in t.schema.names if c not in DENSE_COLS])
    written.append(path)
  return written


def gather_bin_counts(bin_count, part_base, group=None):
  """All-gather every rank's per-(partition, bin) row counts.

  bin_count: int64 tensor [n_part_local, nbins] (PackResult.bin_count, on
  the GPU under the nccl=RCCL backend, on the CPU under gloo); part_base: the
  global index of this rank's first partition.  One all_gather_into_tensor of
  a padded [max_parts, nbins + 1] block per rank (row 0 carries part_base and
  n_part) replaces the MPI Allreduce of _build_files (load_balance.py:222-233).
  Returns a numpy int64 [n_part_total, nbins] array in global partition order."""
  import torch
  import torch.distributed as dist
  world = dist.get_world_size(group)
  n_part, nbins = bin_count.shape
  n = torch.tensor([n_part], dtype=torch.int64, device=bin_count.device)
  ns = torch.empty(world, dtype=torch.int64, device=bin_count.device)
  dist.all_gather_into_tensor(ns, n, group=group)
  mx = int(ns.max().item())
  blk = torch.zeros(mx + 1, nbins + 1, dtype=torch.int64, device=bin_count.device)
  blk[0, 0], blk[0, 1] = part_base, n_part
  blk[1:n_part + 1, :nbins] = bin_count.to(torch.int64)
  allb = torch.empty(world * (mx + 1), nbins + 1, dtype=torch.int64, device=bin_count.device)
  dist.all_gather_into_tensor(allb, blk, group=group)
  allb = allb.cpu().numpy().reshape(world, mx + 1, nbins + 1)
  total = max([int(allb[r, 0, 0] + allb[r, 0, 1]) for r in range(world)] + [0])
  out = np.zeros((total, nbins), dtype=np.int64)
  for r in range(world):
    b, k = int(allb[r, 0, 0]), int(allb[r, 0, 1])
    out[b:b + k] = allb[r, 1:k + 1, :nbins]
  return out


def balance_counts(counts, num_shards, binned, outdir=None, strict=False):
  """Plan from a [n_part, nbins] count array (no file reads): the files are
  part.{p}.parquet (unbinned, nbins == 1) or part.{p}.parquet_{b}."""
  counts = np.asarray(counts)
  base = outdir or ''
  if binned:
    names = [os.path.join(base, 'part.%d.parquet_%d' % (p, b)) for p in range(counts.shape[0])
             for b in range(counts.shape[1])]
  else:
    names = [os.path.join(base, 'part.%d.parquet' % p) for p in range(counts.shape[0])]
    counts = counts.sum(axis=1)
  return plan_files(names, counts.ravel().tolist(), num_shards, strict=strict)


def store_num_samples(num_samples, outdir):
  """load_balance.py:372-378 .num_samples.json"""
  with open(os.path.join(outdir, '.num_samples.json'), 'w') as f:
    json.dump(num_samples, f)


def attach_args(parser=None):
  """The reference's balance_dask_output flags (load_balance.py:265-306)."""
  parser = parser or argparse.ArgumentParser('lddl_amd load balancer for the preprocessor\'s parquet shards')
  parser.add_argument('--indir', type=str, required=True)
  parser.add_argument('--outdir', type=str, default=None)
  parser.add_argument('--num-shards', type=int, required=True)
  parser.add_argument('--bin-ids', type=int, nargs='*', default=None)
  parser.add_argument('--keep-orig', dest='keep_orig', action='store_true')
  parser.add_argument('--no-keep-orig', dest='keep_orig', action='store_false')
  parser.set_defaults(keep_orig=False)
  return parser


def rank_world():
  """(rank, world) of this process: torch.distributed.run (RANK / WORLD_SIZE)
  or mpirun / srun (OMPI_COMM_WORLD_*, PMI_*, SLURM_*), as the reference
  balancer runs under MPI (load_balance.py:381-445)."""
  for r, w in (('RANK', 'WORLD_SIZE'), ('OMPI_COMM_WORLD_RANK', 'OMPI_COMM_WORLD_SIZE'), ('PMI_RANK', 'PMI_SIZE'),
               ('SLURM_PROCID', 'SLURM_NTASKS')):
    if r in os.environ and w in os.environ:
      return int(os.environ[r]), int(os.environ[w])
  return 0, 1


# per-launch ids first: SLURM_JOB_ID is shared by every launch inside one
# allocation (mpirun under salloc often leaves SLURM_STEP_ID unset)
_JOB_ENV = ('PMIX_NAMESPACE', 'OMPI_MCA_ess_base_jobid', 'OMPI_MCA_orte_ess_jobid', 'PMI_JOBID', 'SLURM_JOB_ID')


_MPI_ENV = ('OMPI_COMM_WORLD_SIZE', 'PMI_SIZE', 'PMIX_RANK', 'PMIX_NAMESPACE', 'MV2_COMM_WORLD_SIZE', 'PMI_RANK')


def _mpi_joins(rank, world):
  """mpi4py is usable only when its COMM_WORLD is this launch's world: under
  srun without PMI wiring, or with an mpi4py built against another MPI, every
  process is a singleton and Barrier() would return at once.  mpi4py.MPI is
  imported (MPI_Init) only when an MPI launcher's environment is present:
  elsewhere MPI_Init can abort the process instead of raising."""
  if not any(k in os.environ for k in _MPI_ENV):
    return False
  try:
    from mpi4py import MPI
    c = MPI.COMM_WORLD
    return c.Get_size() == world and (rank is None or c.Get_rank() == rank)
  except Exception:  # ImportError, or an MPI that fails to initialise
    return False


def barrier_kind(world, rank=None):
  """How the ranks of this launch meet (checked BEFORE any shard is written):
  'dist' (torch.distributed already up, or MASTER_ADDR / MASTER_PORT set, as
  torch.distributed.run sets them), 'mpi4py' (importable under mpirun / srun
  AND its COMM_WORLD has this world's size and rank),
  'file' (a shared-file barrier in the output directory keyed by the
  launcher's job id), or a ValueError: without any of them the reference's
  MPI barrier (load_balance.py:442) has no counterpart here."""
  if world <= 1:
    return 'none'
  try:
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
      return 'dist'
  except ImportError:
    pass
  if os.environ.get('MASTER_ADDR') and os.environ.get('MASTER_PORT'):
    return 'dist'
  if _mpi_joins(rank, world):
    return 'mpi4py'
  if job_id():
    return 'file'
  raise ValueError('%d ranks but no way to meet: set MASTER_ADDR / MASTER_PORT (torch.distributed.run), make mpi4py '
                   'importable, or launch under mpirun / srun (a job id in %s)' % (world, '/'.join(_JOB_ENV)))


def job_id():
  for k in _JOB_ENV:
    v = os.environ.get(k)
    if v:
      return '%s-%s' % (v, os.environ.get('SLURM_STEP_ID', '')) if k == 'SLURM_JOB_ID' else v
  return None


def _launch_start():
  """This process' start time: barrier markers older than it belong to an
  earlier launch with the same job id (e.g. one that crashed)."""
  try:
    import psutil
    return psutil.Process().create_time()
  except Exception:
    return _T_IMPORT


_T_IMPORT = time.time()


def _barrier_tag():
  return re.sub(r'[^A-Za-z0-9_.-]', '_', job_id() or 'nojob')


def file_barrier_ref(outdir, rank):
  """Rank 0, before any shard is written: a reference file on the shared
  filesystem holding a nonce of this launch.  Every rank's marker carries
  the nonce it read there, so a marker left by an earlier launch with the
  same job tag (one that crashed, or a fast requeue in the same allocation)
  never counts, whatever the clocks say."""
  if rank == 0:
    ref = os.path.join(outdir, '.lddl_barrier.%s.ref' % _barrier_tag())
    tmp = ref + '.%d' % os.getpid()
    with open(tmp, 'w') as f:
      f.write('%d.%.6f.%s\n' % (os.getpid(), time.time(), os.urandom(8).hex()))
    os.replace(tmp, ref)  # (readers see the whole nonce or none)


def _read_nonce(ref):
  try:
    with open(ref) as f:
      v = f.read()
    return v if v.endswith('\n') else None
  except OSError:
    return None


def _file_barrier(outdir, rank, world, timeout=24 * 3600.0, poll=0.05, margin=60.0, ref_wait=600.0):
  """Every rank drops a marker file named by the job tag; rank 0 waits for
  all of them and removes them.  Only rank 0 acts after the barrier (it
  removes the inputs and writes .num_samples.json), so the other ranks need
  not wait.  With rank 0's reference file (file_barrier_ref) a marker counts
  when it holds that file's nonce (the other ranks wait up to ref_wait
  seconds for it to appear); without one, when it is no older than rank 0's
  start minus `margin` seconds."""
  tag = _barrier_tag()
  mk = lambda r: os.path.join(outdir, '.lddl_barrier.%s.%d' % (tag, r))
  ref = os.path.join(outdir, '.lddl_barrier.%s.ref' % tag)
  nonce = _read_nonce(ref)
  if rank != 0:
    t0 = time.time()
    while nonce is None and time.time() - t0 < ref_wait and os.path.exists(os.path.dirname(ref)):
      time.sleep(poll)
      nonce = _read_nonce(ref)
  with open(mk(rank) + '.tmp', 'w') as f:
    f.write(nonce or 'done\n')
  os.replace(mk(rank) + '.tmp', mk(rank))
  if rank != 0:
    return
  t0 = time.time()
  start = _launch_start() - margin

  def fresh(p):
    try:
      if nonce is not None:
        with open(p) as f:
          return f.read() == nonce
      return os.stat(p).st_mtime >= start
    except OSError:
      return False
  while not all(fresh(mk(r)) for r in range(world)):
    if time.time() - t0 > timeout:
      raise RuntimeError('file barrier: ranks missing after %.0f s' % timeout)
    time.sleep(poll)
  for r in range(world):
    os.remove(mk(r))
  if os.path.exists(ref):
    os.remove(ref)


def _barrier(world, kind='dist', outdir=None, rank=0):
  """host barrier between the ranks (barrier_kind)"""
  if world <= 1 or kind == 'none':
    return
  if kind == 'mpi4py':
    from mpi4py import MPI
    MPI.COMM_WORLD.Barrier()
  elif kind == 'file':
    _file_barrier(outdir, rank, world)
  else:
    import torch.distributed as dist
    if not dist.is_initialized():
      r, w = rank_world()
      dist.init_process_group('gloo', rank=r, world_size=w)
    dist.barrier()


def main(args, rank=None, world=None):
  """Counts from the parquet footers (no table reads), plan, write, and
  .num_samples.json (rank 0).  Every rank plans the same shards and writes
  shard k when k % world == rank (load_balance.py:129-140 ownership); once
  every rank is done, rank 0 removes the input files (unless --keep-orig)."""
  import pyarrow.parquet as pq
  if rank is None or world is None:
    rank, world = rank_world()
  outdir = args.indir if args.outdir is None else os.path.abspath(os.path.expanduser(args.outdir))
  kind = barrier_kind(world, rank)  # fail before writing when the ranks cannot meet
  os.makedirs(outdir, exist_ok=True)
  if kind == 'file':
    file_barrier_ref(outdir, rank)
  paths = sorted(os.path.join(r, f) for r, _, fs in os.walk(args.indir) for f in fs
                 if '.parquet' in os.path.splitext(f)[1])
  counts = [pq.ParquetFile(p).metadata.num_rows for p in paths]
  shards, ns = plan_files(paths, counts, args.num_shards, args.bin_ids)
  written = write_shards(shards, outdir, rank, world)
  _barrier(world, kind, outdir, rank)
  if rank == 0:
    if not args.keep_orig:
      keep = set(os.path.abspath(p) for p in written) | {os.path.abspath(os.path.join(outdir, n)) for n, _, _ in shards}
      for p in paths:
        if os.path.abspath(p) not in keep:
          os.remove(p)
    store_num_samples(ns, outdir)
  return written, ns


def _parquets_under(indir):
  """lddl/utils.py get_all_parquets_under: every file under indir whose
  extension holds '.parquet' (shards and their _<bin> forms), sorted by path"""
  return sorted(os.path.join(r, f) for r, _, fs in os.walk(indir) for f in fs
                if '.parquet' in os.path.splitext(f)[1])


def num_samples_cache(indir, rank=None, world=None):
  """load_balance.py:generate_num_samples_cache (:428-455): .num_samples.json
  for already balanced shards, {basename: rows} in sorted path order, written
  into indir.  The reference reads every table (get_num_samples_of_parquet,
  utils.py:77-78) strided over its MPI ranks and Allreduces the counts; here
  each rank reads the parquet footers (num_rows, no table reads) of one
  contiguous block of the files and one all-gather (gather_bin_counts, the
  RCCL / gloo path of the balancer) gives every rank all counts.  Under the
  file barrier (no collective) rank 0 reads every footer.  Rank 0 writes the
  file (the reference has every rank write the same bytes).  Returns the
  dict."""
  import pyarrow.parquet as pq
  if rank is None or world is None:
    rank, world = rank_world()
  paths = _parquets_under(indir)
  n = len(paths)
  kind = barrier_kind(world, rank)
  counts = np.zeros(n, dtype=np.int64)
  if kind in ('none', 'file'):
    if kind == 'file' and rank != 0:
      return None
    for i, p in enumerate(paths):
      counts[i] = pq.ParquetFile(p).metadata.num_rows
  else:
    lo, hi = n * rank // world, n * (rank + 1) // world
    mine = np.array([pq.ParquetFile(p).metadata.num_rows for p in paths[lo:hi]], dtype=np.int64).reshape(-1, 1)
    if kind == 'mpi4py':
      from mpi4py import MPI
      full = np.zeros(n, dtype=np.int64)
      full[lo:hi] = mine[:, 0]
      MPI.COMM_WORLD.Allreduce(MPI.IN_PLACE, full, op=MPI.SUM)
      counts = full
    else:
      import torch
      import torch.distributed as dist
      if not dist.is_initialized():
        dist.init_process_group('gloo', rank=rank, world_size=world)
      dev = torch.device('cuda', torch.cuda.current_device()) if dist.get_backend() == 'nccl' else torch.device('cpu')
      counts = gather_bin_counts(torch.from_numpy(mine).to(dev), lo)[:, 0]
  ns = {os.path.basename(p): int(c) for p, c in zip(paths, counts)}
  if rank == 0:
    store_num_samples(ns, indir)
  return ns


def generate_num_samples_cache(argv=None):
  """The reference's `generate_num_samples_cache` console script (setup.py:72)."""
  parser = argparse.ArgumentParser('Generate .num_samples.json for the balanced parquets.')
  parser.add_argument('--indir', type=str, default=None, help='path to the dir that contains the balanced shards')
  parser.add_argument('--num-samples-cache', action='store_true', help=argparse.SUPPRESS)
  args = parser.parse_args(argv)
  num_samples_cache(args.indir)


def console_script():
  tic = time.perf_counter()
  main(attach_args().parse_args())
  print('Load balancing took {} s!'.format(time.perf_counter() - tic))


if __name__ == '__main__':
  import sys
  if '--num-samples-cache' in sys.argv[1:]:  # python -m lddl_amd.balance --num-samples-cache --indir DIR
    generate_num_samples_cache()
  else:
    console_script()
