"""Host facts shared by the torch-free modules (balance, preprocess) and the
GPU ones (writer, bench): the parquet columns written without dictionary
pages, and the host CPU share worker pools are sized to."""
import os

# string / binary columns unique per row: the parquet encoder would build and
# then discard a dictionary for them (writer.write_shards, balance.write_shards)
DENSE_COLS = ('A', 'B', 'doc', 'code', 'masked_lm_positions', 'masked_lm_labels')

CPU_SHARE = 16  # host cores per GPU a GPU box of this harness allots one command's worker pools


def affinity():
  try:
    return len(os.sched_getaffinity(0))
  except (AttributeError, OSError):
    return None


def cgroup_cpu_max():
  """the cgroup v2 CPU quota as 'quota period' (or 'max period'), None if absent"""
  for p in ('/sys/fs/cgroup/cpu.max',):
    try:
      with open(p) as f:
        return f.read().strip()
    except OSError:
      pass
  return None


def cpu_share():
  """worker processes / threads for host pools: the affinity count, capped at
  LDDL_CPU_SHARE (default 16, one GPU's share of a GPU box: os.cpu_count()
  and the affinity show the whole machine there)"""
  aff = affinity() or os.cpu_count() or 1
  return max(1, min(aff, int(os.environ.get('LDDL_CPU_SHARE', CPU_SHARE))))


def cpu_evidence():
  """what the host shows about its CPUs (reported beside the CPU legs)"""
  q = cgroup_cpu_max()
  quota = None
  if q:
    a, b = (q.split() + ['100000'])[:2]
    quota = None if a == 'max' else float(a) / float(b)
  return {'os_cpu_count': os.cpu_count(), 'affinity': affinity(), 'cgroup_cpu_max': q, 'cgroup_cpus': quota,
          'env': {k: os.environ.get(k) for k in ('OMP_NUM_THREADS', 'MAX_JOBS', 'CMAKE_BUILD_PARALLEL_LEVEL',
                                                 'LDDL_CPU_SHARE')}}
