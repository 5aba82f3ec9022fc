"""The product's lane tokenizer logic (lddl_amd/csrc/tokenize_lane.h: the
per-lane trie walk that tokenize_lane.hip runs as waves on the GPU) compiled
for the host by g++ with AddressSanitizer + UndefinedBehaviorSanitizer, a
wave of 64 lanes emulated with the device's wave-level steps
(tests/host_lane.cpp), over the tables the device gets
(lddl_amd/csrc/tok_tables.h).  Checked against the golden ids (HF tokenizers
0.22.2, the call at lddl/dask/bert/pretrain.py:79-80) and against the C
oracle on adversarial and synthetic corpora.  CPU only; the HIP build of the
same header is checked on the GPU by tests/test_tokenize_gpu.py."""
import os
import shutil
import subprocess

import numpy as np
import pytest

from conftest import ROOT
from oracle.oracle import TABLE, OracleTokenizer, compact
from test_tokenize_gpu import adversarial_sentences

VOCABS = {'bert': os.path.join(ROOT, 'lddl_amd', 'data', 'bert_vocab.txt'),
          'codebert': os.path.join(ROOT, 'lddl_amd', 'data', 'codebert_52000_vocab.txt')}


@pytest.fixture(scope='module')
def host_lane(tmp_path_factory):
  if shutil.which('g++') is None:
    pytest.skip('g++ not available')
  out = str(tmp_path_factory.mktemp('hlane') / 'host_lane')
  subprocess.run(['g++', '-O1', '-g', '-std=c++17', '-fno-omit-frame-pointer', '-fsanitize=address,undefined',
                  '-fno-sanitize-recover=undefined', '-D__HIP_PLATFORM_AMD__', '-I/opt/rocm/include',
                  '-I' + os.path.join(ROOT, 'lddl_amd', 'csrc'), '-o', out, os.path.join(ROOT, 'tests', 'host_lane.cpp')],
                 check=True)
  return out


def run_lane(exe, tmp_path, name, data, sent_off, max_tok, seg=None):
  n = len(sent_off) - 1
  fb, fo = tmp_path / 'bytes.bin', tmp_path / 'off.bin'
  np.asarray(data, dtype=np.uint8).tofile(fb)
  np.asarray(sent_off, dtype=np.int64).tofile(fo)
  fi, fn = tmp_path / 'ids.bin', tmp_path / 'ntok.bin'
  env = dict(os.environ, ASAN_OPTIONS='detect_leaks=1:abort_on_error=0:exitcode=23',
             UBSAN_OPTIONS='print_stacktrace=1:halt_on_error=1:exitcode=24')
  env.pop('LD_PRELOAD', None)
  cmd = [exe, VOCABS[name], TABLE, str(fb), str(fo), str(n), str(max_tok), str(fi), str(fn)]
  if seg:
    cmd.append(str(seg))
  r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
  assert r.returncode == 0, r.stderr[-3000:]
  assert 'runtime error' not in r.stderr and 'ERROR: AddressSanitizer' not in r.stderr, r.stderr[-3000:]
  return np.fromfile(fi, dtype=np.int32), np.fromfile(fn, dtype=np.int32), r.stderr


@pytest.mark.parametrize('name,max_tok', [('bert', 512), ('codebert', 512), ('bert', 7), ('codebert', 3)])
def test_lane_golden_under_asan(host_lane, golden, tmp_path, name, max_tok):
  g = golden('tok_%s.npz' % name)
  ids, ntok, _ = run_lane(host_lane, tmp_path, name, g['data'], g['sent_off'], max_tok)
  assert np.array_equal(ntok, np.minimum(g['ntok'], max_tok))
  exp = [x[:max_tok] for x in np.split(g['ids'], np.cumsum(g['ntok'])[:-1])]
  got = compact(ids, ntok, g['sent_off'])
  bad = [i for i, (a, b) in enumerate(zip(exp, got)) if not np.array_equal(a, b)]
  assert not bad, bad[:10]


def check_vs_oracle(exe, tmp_path, name, c, max_tok, seg=None):
  ids, ntok, log = run_lane(exe, tmp_path, name, c.data, c.sent_off, max_tok, seg)
  oids, ontok = OracleTokenizer(VOCABS[name]).run(c.data, c.sent_off, max_tok, nthreads=8)
  bad = np.flatnonzero(ntok != ontok)
  assert not len(bad), [(int(i), c.sentence(int(i))[:80], int(ntok[i]), int(ontok[i])) for i in bad[:5]]
  for i, (a, b) in enumerate(zip(compact(ids, ntok, c.sent_off), compact(oids, ontok, c.sent_off))):
    assert np.array_equal(a.astype(np.int64), b.astype(np.int64)), (i, c.sentence(i)[:80])
  return log


@pytest.mark.parametrize('name', ['bert', 'codebert'])
def test_lane_adversarial_vs_oracle(host_lane, tmp_path, name):
  """empty / 1-byte sentences, specials at every offset, multi-byte chars at
  ring edges, words of 90-110 chars and > 300 bytes (ring overflow: slow path
  or the serial fallback), ccc>0 survivors, CJK, controls"""
  from lddl_amd.synth import corpus_from_sentences
  rng = np.random.default_rng(11 + len(name))
  sents = adversarial_sentences(rng, 3000)
  c = corpus_from_sentences(sents, [0, len(sents)])
  for max_tok in (512, 3):
    check_vs_oracle(host_lane, tmp_path, name, c, max_tok)


def test_lane_synthetic_wiki_and_code(host_lane, tmp_path):
  from lddl_amd import synth
  log = check_vs_oracle(host_lane, tmp_path, 'bert', synth.make_wiki(1_500_000, seed=41), 512)
  assert 'tiles to the serial path 0' in log, log
  check_vs_oracle(host_lane, tmp_path, 'codebert', synth.make_code(800, seed=43), 512)
  check_vs_oracle(host_lane, tmp_path, 'bert', synth.make_wiki(300_000, seed=47), 512, seg=7)
