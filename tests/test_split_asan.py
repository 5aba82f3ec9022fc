"""The C sentence splitter and line index (lddl_amd/host/split_rules.c)
built with AddressSanitizer + UndefinedBehaviorSanitizer (gcc, host only)
around a driver that sizes every buffer exactly (tests/split_asan_driver.c)
and first calls it at too small a sentence capacity: no sanitizer report,
leak included, and the same sentences, offsets, ids and line spans as the
library the CLI loads (lddl_amd/splitnative.py).  CPU only."""
import os
import shutil
import subprocess

import numpy as np
import pytest

from conftest import ROOT
from lddl_amd import build, splitnative, synth
from test_split_native import _adversarial


@pytest.fixture(scope='module')
def driver(tmp_path_factory):
  if shutil.which('gcc') is None:
    pytest.skip('gcc not available')
  build.build_split()
  out = str(tmp_path_factory.mktemp('split_asan') / 'split_asan_driver')
  subprocess.run(['gcc', '-O1', '-g', '-std=c99', '-fno-omit-frame-pointer', '-fsanitize=address,undefined',
                  '-fno-sanitize-recover=undefined', '-o', out, os.path.join(ROOT, 'tests', 'split_asan_driver.c'),
                  os.path.join(ROOT, 'lddl_amd', 'host', 'split_rules.c')], check=True)
  return out


def _run(driver, tmp_path, raws):
  n = len(raws)
  rec_off = np.zeros(n + 1, dtype=np.int64)
  np.cumsum([len(r) for r in raws], out=rec_off[1:])
  (tmp_path / 'tab.bin').write_bytes(splitnative.props_table().tobytes())
  (tmp_path / 'buf.bin').write_bytes(b''.join(raws))
  rec_off.tofile(tmp_path / 'off.bin')
  env = dict(os.environ, ASAN_OPTIONS='detect_leaks=1:abort_on_error=0:exitcode=23',
             UBSAN_OPTIONS='print_stacktrace=1:halt_on_error=1:exitcode=24')
  env.pop('LD_PRELOAD', None)
  out = str(tmp_path / 'out')
  r = subprocess.run([driver, str(tmp_path / 'tab.bin'), str(tmp_path / 'buf.bin'), str(tmp_path / 'off.bin'), str(n),
                      out], env=env, capture_output=True, text=True, timeout=300)
  assert r.returncode == 0, r.stderr[-3000:]
  assert 'runtime error' not in r.stderr and 'ERROR: AddressSanitizer' not in r.stderr, r.stderr[-3000:]
  return np.fromfile(out + '.split', dtype=np.uint8).tobytes(), np.fromfile(out + '.lines', dtype=np.int64)


def _check(driver, tmp_path, raws):
  split, lines = _run(driver, tmp_path, raws)
  rc, bad = np.frombuffer(split[:16], dtype=np.int64)
  exp = splitnative.split_raw(raws)
  if exp is None:  # invalid UTF-8: handed back to the Python path
    assert rc == -2 and 0 <= bad < len(raws)
  else:
    corpus, ids = exp
    n = len(raws)
    nb = int(corpus.sent_off[-1])
    assert rc == len(corpus.sent_off) - 1
    p = 16
    assert split[p:p + nb] == bytes(corpus.data)
    p += nb
    got = np.frombuffer(split[p:], dtype=np.int64)
    assert np.array_equal(got[:rc + 1], corpus.sent_off)
    assert np.array_equal(got[rc + 1:rc + 2 + n], corpus.doc_sent_off)
    joined = b''.join(raws)
    rng = got[rc + 2 + n:]
    assert [joined[rng[2 * r]:rng[2 * r + 1]].decode('utf-8') for r in range(n)] == ids
  buf = np.frombuffer(b''.join(raws) or b'\0', dtype=np.uint8)[:len(b''.join(raws))]
  at = 0
  for crlf_only in (False, True):
    m = int(lines[at])
    s, e = lines[at + 1:at + 1 + m], lines[at + 1 + m:at + 1 + 2 * m]
    at += 1 + 2 * m
    es, ee = splitnative.line_spans(buf, crlf_only)
    assert np.array_equal(s, es) and np.array_equal(e, ee)


def test_synthetic_wiki_under_asan(driver, tmp_path):
  docs = synth.make_wiki(400_000, seed=9).documents()
  _check(driver, tmp_path, [('wiki-%d %s\n' % (i, ' '.join(d))).encode() for i, d in enumerate(docs)])


@pytest.mark.parametrize('seed', [0, 1, 2])
def test_adversarial_records_under_asan(driver, tmp_path, seed):
  recs = _adversarial(np.random.default_rng(seed), 400)
  _check(driver, tmp_path, [r.encode('utf-8') for r in recs])


def test_invalid_utf8_and_edges_under_asan(driver, tmp_path):
  # truncated / overlong / surrogate sequences, at a record's end and in its id
  for raws in ([b'doc1 Fine.', b'doc2 bad \xe2\x82'], [b'doc\xc0\xaf body.'], [b'x \xed\xa0\x80.'],
               [b''], [b'id-only'], [b' '], [b'\xf4\x90\x80\x80']):
    _check(driver, tmp_path, raws)


def test_line_spans_cr_lf_dense_under_asan(driver, tmp_path):
  rng = np.random.default_rng(5)
  blob = rng.choice(np.frombuffer(b'\r\n\r\nab. ', dtype=np.uint8), 20_000).tobytes()
  _check(driver, tmp_path, [blob[:7000], blob[7000:7001], blob[7001:]])
