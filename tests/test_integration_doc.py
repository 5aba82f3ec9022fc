"""INTEGRATION.md §1 is the binding a maintainer pastes into the reference
(the ctypes stub next to lddl/dask/bert/pretrain.py:584-587 / :386-402).
Exec it against a recording stand-in for ctypes.CDLL and check every entry it
binds against lddl_amd/_lib.py:SIGNATURES and against the parameter lists
include/lddl_amd.h declares (count and C type class per argument)."""
import ctypes
import os
import re

from conftest import ROOT


def _binding_block():
  s = open(os.path.join(ROOT, 'INTEGRATION.md')).read()
  sec = s[s.index('## 1. Minimal ctypes binding'):s.index('## 2.')]
  blocks = re.findall(r'```python\n(.*?)```', sec, flags=re.S)
  assert len(blocks) == 1
  return blocks[0]


class _Fn:
  restype = 'unset'
  argtypes = 'unset'


class _FakeLib:
  def __init__(self, path):
    self.fns = {}

  def __getattr__(self, name):
    if name.startswith('__'):
      raise AttributeError(name)
    return self.fns.setdefault(name, _Fn())


def _exec_binding(monkeypatch):
  made = []

  def cdll(path):
    made.append(_FakeLib(path))
    return made[-1]

  monkeypatch.setattr(ctypes, 'CDLL', cdll)
  ns = {}
  exec(compile(_binding_block(), 'INTEGRATION.md#1', 'exec'), ns)
  assert len(made) == 1
  return made[0].fns


def _header_decls():
  src = open(os.path.join(ROOT, 'include', 'lddl_amd.h')).read()
  src = re.sub(r'/\*.*?\*/', '', src, flags=re.S)
  out = {}
  for m in re.finditer(r'^\s*([A-Za-z_][\w \*]*?)\b(lddl_\w+)\s*\(([^;{]*?)\)\s*;', src, flags=re.M | re.S):
    params = [p.strip() for p in ' '.join(m.group(3).split()).split(',')]
    if params == ['void']:
      params = []
    out[m.group(2)] = (m.group(1).strip(), params)
  return out


def _cls(ctype):
  """C parameter -> the ctypes class family it must be bound with."""
  if '*' in ctype or '[' in ctype:
    return 'ptr'
  base = ctype.rsplit(' ', 1)[0].replace('const ', '').strip()
  return {'int64_t': 'i64', 'int32_t': 'i32', 'int': 'i32', 'double': 'f64', 'uint64_t': 'u64'}[base]


def _ctypes_cls(t):
  if t in (ctypes.c_void_p, ctypes.c_char_p) or (isinstance(t, type) and issubclass(t, ctypes._Pointer)):
    return 'ptr'
  return {ctypes.c_int64: 'i64', ctypes.c_int32: 'i32', ctypes.c_double: 'f64', ctypes.c_uint64: 'u64'}[t]


def test_integration_binding_matches_lib_signatures(monkeypatch):
  from lddl_amd import _lib
  bound = _exec_binding(monkeypatch)
  assert set(bound) == set(_lib.SIGNATURES), set(bound) ^ set(_lib.SIGNATURES)
  for name, fn in bound.items():
    res, args = _lib.SIGNATURES[name]
    assert fn.argtypes != 'unset' and fn.restype != 'unset', name
    assert len(fn.argtypes) == len(args), (name, len(fn.argtypes), len(args))
    for i, (a, b) in enumerate(zip(fn.argtypes, args)):
      assert a is b, (name, i, a, b)
    assert fn.restype is res or (res is ctypes.c_int and fn.restype is ctypes.c_int32), (name, fn.restype, res)


def test_integration_binding_matches_header(monkeypatch):
  bound = _exec_binding(monkeypatch)
  decls = _header_decls()
  assert set(decls) == set(bound), set(decls) ^ set(bound)
  for name, (ret, params) in decls.items():
    fn = bound[name]
    assert len(fn.argtypes) == len(params), (name, len(fn.argtypes), params)
    for i, (t, p) in enumerate(zip(fn.argtypes, params)):
      assert _ctypes_cls(t) == _cls(p), (name, i, p, t)
    if ret == 'void':
      assert fn.restype is None, name


def test_lib_signatures_match_header():
  from lddl_amd import _lib
  decls = _header_decls()
  assert set(decls) == set(_lib.SIGNATURES)
  for name, (ret, params) in decls.items():
    _, args = _lib.SIGNATURES[name]
    assert [_ctypes_cls(a) for a in args] == [_cls(p) for p in params], name


def test_integration_binding_binds_the_built_library(monkeypatch):
  """§1 pasted into a scratch module binds every entry of the real .so."""
  from lddl_amd import build, _lib
  build.build_hip()
  monkeypatch.setenv('LDDL_AMD_LIB', _lib.LIB_PATH)
  ns = {}
  exec(compile(_binding_block(), 'INTEGRATION.md#1', 'exec'), ns)
  for name, (res, args) in ns['_SIG'].items():
    f = getattr(ns['_L'], name)
    assert list(f.argtypes or []) == list(args), name
