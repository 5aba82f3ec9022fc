"""The scan's whole-word table (tok_tables.h: two 32-B candidate slots per
key, cuckoo placement) built on the host with ASan/UBSan for both vocabs:
every whole-word key of <= 24 bytes is found where the scan looks for it,
with the vocab dictionary's id (the last duplicate line), no slot holds
anything else, and the table stays L2-sized (<= 4 MB).  CPU only; the GPU
tokenizer tests check the device probe against the goldens and the oracle."""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT

VOCABS = {'bert': os.path.join(ROOT, 'lddl_amd', 'data', 'bert_vocab.txt'),
          'codebert': os.path.join(ROOT, 'lddl_amd', 'data', 'codebert_52000_vocab.txt')}


@pytest.fixture(scope='module')
def driver(tmp_path_factory):
  if shutil.which('g++') is None:
    pytest.skip('g++ not available')
  out = str(tmp_path_factory.mktemp('stab') / 'host_scan_table')
  subprocess.run(['g++', '-O1', '-g', '-std=c++17', '-fno-omit-frame-pointer', '-fsanitize=address,undefined',
                  '-fno-sanitize-recover=undefined', '-D__HIP_PLATFORM_AMD__', '-I/opt/rocm/include',
                  '-I' + os.path.join(ROOT, 'lddl_amd', 'csrc'), '-o', out,
                  os.path.join(ROOT, 'tests', 'host_scan_table.cpp')], check=True)
  return out


@pytest.mark.parametrize('name', ['bert', 'codebert'])
def test_scan_table_finds_every_whole_word(driver, name):
  env = dict(os.environ, ASAN_OPTIONS='detect_leaks=1:abort_on_error=0:exitcode=23',
             UBSAN_OPTIONS='print_stacktrace=1:halt_on_error=1:exitcode=24')
  env.pop('LD_PRELOAD', None)
  r = subprocess.run([driver, VOCABS[name]], env=env, capture_output=True, text=True, timeout=300)
  assert r.returncode == 0, r.stderr[-3000:]
  f = r.stdout.split()
  got = dict(zip(f[0::2], map(int, f[1::2])))
  assert got['misses'] == 0 and got['wrong'] == 0 and got['extra'] == 0, r.stdout
  assert got['used'] == got['keys'], r.stdout
  assert got['slots'] * 32 <= 4 << 20, r.stdout
