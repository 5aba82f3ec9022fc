"""Build liblddl_amd.so (gfx950), the host splitter libsplit.so and the
oracle's liboracle.so in-tree.

    python -m lddl_amd.build          # all
The HIP library and libsplit.so are the product; the oracle build is test
infrastructure.
"""
import glob
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, 'csrc')
LIB = os.path.join(PKG, 'liblddl_amd.so')
ARCH = os.environ.get('LDDL_OFFLOAD_ARCH', 'gfx950')


def _newer(target, deps):
  if not os.path.exists(target):
    return True
  t = os.path.getmtime(target)
  return any(os.path.getmtime(d) > t for d in deps)


SPLIT_LIB = os.path.join(PKG, 'libsplit.so')


def build_split(force=False, verbose=False):
  """lddl_amd/host/split_rules.c -> libsplit.so (plain C, gcc: the CLI's
  split workers load it without the HIP runtime)"""
  src = os.path.join(PKG, 'host', 'split_rules.c')
  if not force and not _newer(SPLIT_LIB, [src]):
    return SPLIT_LIB
  tmp = SPLIT_LIB + '.tmp%d' % os.getpid()
  cmd = [os.environ.get('CC', 'gcc'), '-O2', '-shared', '-fPIC', '-std=c99', '-Wall', '-o', tmp, src]
  if verbose:
    print(' '.join(cmd))
  subprocess.run(cmd, check=True)
  os.replace(tmp, SPLIT_LIB)
  from lddl_amd import splitnative  # its code point table, cached next to the library
  splitnative.props_table()
  return SPLIT_LIB


def build_hip(force=False, verbose=False, lib=None, defines=(), extra=()):
  """Each .hip compiled to its own object in parallel (device code is per
  translation unit: the kernels share headers only), then linked.
  lib / defines: A/B builds of variants (tools/ab_build.py).

  Safe to call from several processes at once (the ranks of a multi-GPU
  bench): one holds an exclusive lock on the build directory while it
  compiles, into temporaries named by its pid, and the others, once they get
  the lock, find the library up to date and return it.  LDDL_BUILD_LIB
  redirects the default output, LDDL_HIPCC the compiler (tests)."""
  import fcntl
  lib = lib or os.environ.get('LDDL_BUILD_LIB') or LIB
  srcs = sorted(glob.glob(os.path.join(CSRC, '*.hip')))
  hdrs = glob.glob(os.path.join(CSRC, '*.h')) + [os.path.join(ROOT, 'include', 'lddl_amd.h')]
  if not force and not _newer(lib, srcs + hdrs):
    return lib
  from concurrent.futures import ThreadPoolExecutor
  odir = os.path.join(CSRC, 'build') if lib == LIB else os.path.splitext(lib)[0] + '_obj'
  os.makedirs(odir, exist_ok=True)
  hipcc = os.environ.get('LDDL_HIPCC', 'hipcc')
  flags = ['--offload-arch=%s' % ARCH, '-O3', '-std=c++17', '-fPIC', '-Wno-unused-result'] + ['-D' + d for d in defines] + \
      list(extra)
  tag = '.tmp%d' % os.getpid()
  with open(os.path.join(odir, '.build.lock'), 'w') as lk:
    fcntl.flock(lk, fcntl.LOCK_EX)  # (released when the file closes)
    if not force and not _newer(lib, srcs + hdrs):  # another process built it meanwhile
      return lib

    def obj(src):
      o = os.path.join(odir, os.path.basename(src)[:-4] + '.o')
      if force or _newer(o, [src] + hdrs):
        cmd = [hipcc] + flags + ['-c', '-o', o + tag, src]
        if verbose:
          print(' '.join(cmd))
        subprocess.run(cmd, check=True, cwd=CSRC)
        os.replace(o + tag, o)
      return o

    with ThreadPoolExecutor(max_workers=min(len(srcs), max(1, min(8, os.cpu_count() or 1)))) as ex:
      objs = list(ex.map(obj, srcs))
    cmd = [hipcc, '--offload-arch=%s' % ARCH, '-shared', '-fPIC', '-o', lib + tag] + objs
    if verbose:
      print(' '.join(cmd))
    subprocess.run(cmd, check=True, cwd=CSRC)
    os.replace(lib + tag, lib)
  return lib


def build_oracle(force=False):
  odir = os.path.join(ROOT, 'oracle')
  subprocess.run(['make', '-s'] + (['-B'] if force else []), check=True, cwd=odir)
  return os.path.join(odir, 'liboracle.so')


if __name__ == '__main__':
  force = '--force' in sys.argv
  print(build_hip(force, verbose=True))
  print(build_split(force, verbose=True))
  print(build_oracle(force))
