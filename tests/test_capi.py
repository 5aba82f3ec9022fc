"""The C-ABI library loads and exports every symbol include/lddl_amd.h
declares (no compute without a GPU)."""
import ctypes
import os
import re

from conftest import ROOT


def declared_symbols():
  src = open(os.path.join(ROOT, 'include', 'lddl_amd.h')).read()
  src = re.sub(r'/\*.*?\*/', '', src, flags=re.S)
  return sorted(set(re.findall(r'\b(lddl_[a-z_0-9]+)\s*\(', src)))


def test_library_exports_declared_symbols():
  from lddl_amd import build, _lib
  build.build_hip()
  L = ctypes.CDLL(_lib.LIB_PATH)
  syms = declared_symbols()
  assert len(syms) >= 7
  missing = [s for s in syms if not hasattr(L, s)]
  assert not missing, missing
  assert set(syms) <= set(_lib.SIGNATURES), set(syms) - set(_lib.SIGNATURES)


def test_create_without_gpu_fails_cleanly():
  import torch
  from lddl_amd import _lib
  if torch.cuda.is_available():
    return
  L = _lib.lib()
  h = ctypes.c_void_p()
  rc = L.lddl_create(_lib.VOCAB_BERT.encode(), _lib.TABLE_PATH.encode(), 0, ctypes.byref(h))
  assert rc < 0 and L.lddl_last_error()
