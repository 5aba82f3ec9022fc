"""The product's serial tokenizer path (lddl_amd/csrc/tokenize_serial.h: the
split tokenizer's exact fallback, tokenize_fallback_kernel) compiled for the
host by g++ with AddressSanitizer + UndefinedBehaviorSanitizer over the same
tables the device gets (lddl_amd/csrc/tok_tables.h), run over the golden
inputs of both vocabularies at max_tok 512 and 7: no sanitizer report and the
golden ids (HF tokenizers, the call at lddl/dask/bert/pretrain.py:79-80).
CPU only; the HIP build of the same header is checked on the GPU by
tests/test_tokenize_gpu.py."""
import os
import shutil
import subprocess

import numpy as np
import pytest

from conftest import ROOT
from oracle.oracle import TABLE, compact

VOCABS = {'bert': os.path.join(ROOT, 'lddl_amd', 'data', 'bert_vocab.txt'),
          'codebert': os.path.join(ROOT, 'lddl_amd', 'data', 'codebert_52000_vocab.txt')}


@pytest.fixture(scope='module')
def host_serial(tmp_path_factory):
  if shutil.which('g++') is None:
    pytest.skip('g++ not available')
  out = str(tmp_path_factory.mktemp('hsan') / 'host_serial')
  subprocess.run(['g++', '-O1', '-g', '-std=c++17', '-fno-omit-frame-pointer', '-fsanitize=address,undefined',
                  '-fno-sanitize-recover=undefined', '-D__HIP_PLATFORM_AMD__', '-I/opt/rocm/include',
                  '-I' + os.path.join(ROOT, 'lddl_amd', 'csrc'), '-o', out, os.path.join(ROOT, 'tests', 'host_serial.cpp')],
                 check=True)
  return out


@pytest.mark.parametrize('name,max_tok', [('bert', 512), ('codebert', 512), ('bert', 7)])
def test_serial_path_under_asan(host_serial, golden, tmp_path, name, max_tok):
  g = golden('tok_%s.npz' % name)
  n = len(g['sent_off']) - 1
  fb, fo = tmp_path / 'bytes.bin', tmp_path / 'off.bin'
  g['data'].astype(np.uint8).tofile(fb)
  g['sent_off'].astype(np.int64).tofile(fo)
  fi, fn = tmp_path / 'ids.bin', tmp_path / 'ntok.bin'
  env = dict(os.environ, ASAN_OPTIONS='detect_leaks=1:abort_on_error=0:exitcode=23',
             UBSAN_OPTIONS='print_stacktrace=1:halt_on_error=1:exitcode=24')
  env.pop('LD_PRELOAD', None)
  r = subprocess.run([host_serial, VOCABS[name], TABLE, str(fb), str(fo), str(n), str(max_tok), str(fi), str(fn)],
                     env=env, capture_output=True, text=True, timeout=300)
  assert r.returncode == 0, r.stderr[-3000:]
  assert 'runtime error' not in r.stderr and 'ERROR: AddressSanitizer' not in r.stderr, r.stderr[-3000:]
  ids = np.fromfile(fi, dtype=np.int32)
  ntok = np.fromfile(fn, dtype=np.int32)
  assert np.array_equal(ntok, np.minimum(g['ntok'], max_tok))
  exp = [x[:max_tok] for x in np.split(g['ids'], np.cumsum(g['ntok'])[:-1])]
  got = compact(ids, ntok, g['sent_off'])
  bad = [i for i, (a, b) in enumerate(zip(exp, got)) if not np.array_equal(a, b)]
  assert not bad, bad[:10]
