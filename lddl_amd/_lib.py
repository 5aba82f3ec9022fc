"""ctypes binding of liblddl_amd.so (the C-ABI in include/lddl_amd.h).

The product path has no CPU fallback: if the HIP library is missing or a call
fails, a RuntimeError is raised.
"""
import ctypes
import os

_PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('LDDL_LIB') or os.path.join(_PKG, 'liblddl_amd.so')  # LDDL_LIB: A/B tools
TABLE_PATH = os.path.join(_PKG, 'data', 'unicode_table.bin')
VOCAB_BERT = os.path.join(_PKG, 'data', 'bert_vocab.txt')
VOCAB_CODEBERT = os.path.join(_PKG, 'data', 'codebert_52000_vocab.txt')

c_void_p, c_int, c_int32, c_int64, c_double, c_uint64, c_char_p = (
    ctypes.c_void_p, ctypes.c_int, ctypes.c_int32, ctypes.c_int64, ctypes.c_double,
    ctypes.c_uint64, ctypes.c_char_p)

# name -> (restype, argtypes); every symbol include/lddl_amd.h declares
SIGNATURES = {
    'lddl_last_error': (c_char_p, []),
    'lddl_create': (c_int, [c_char_p, c_char_p, c_int, ctypes.POINTER(c_void_p)]),
    'lddl_destroy': (None, [c_void_p]),
    'lddl_vocab_size': (c_int, [c_void_p]),
    'lddl_special_ids': (c_int, [c_void_p, ctypes.POINTER(c_int32)]),
    'lddl_vocab_token': (c_int, [c_void_p, c_int32, c_char_p, c_int64]),
    'lddl_tokenize': (c_int, [c_void_p, c_void_p, c_int64, c_void_p, c_int64, c_int32, c_void_p, c_int64,
                              c_void_p, c_void_p, c_void_p]),
    'lddl_set_timing': (c_int, [c_void_p, c_int]),
    'lddl_set_special_flags': (c_int, [c_void_p, c_int]),
    'lddl_set_tokenize_algo': (c_int, [c_void_p, c_int, ctypes.POINTER(c_int)]),
    'lddl_tokenize_stats': (c_int, [c_void_p, ctypes.POINTER(c_double), c_int]),
    'lddl_pack_new': (c_int, [c_void_p, ctypes.POINTER(c_void_p)]),
    'lddl_pack_free': (None, [c_void_p]),
    'lddl_pack_rows': (c_int, [c_void_p, ctypes.POINTER(c_int64)]),
    'lddl_bin': (c_int, [c_void_p, c_void_p, c_int64, c_int32, c_int32, c_void_p, c_void_p, c_void_p]),
    'lddl_pack_bert': (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_int64,
                               c_void_p, c_int64, c_int32, c_double, c_int32, c_int32, c_double, c_uint64, c_int32,
                               ctypes.POINTER(c_int64), c_void_p]),
    'lddl_pack_codebert': (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_int64,
                                   c_void_p,
                                   c_int64, c_int32, c_double, c_int32, c_uint64, c_int32,
                                   ctypes.POINTER(c_int64), c_void_p]),
    'lddl_materialize': (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                 c_void_p, c_void_p, c_void_p, c_void_p]),
    'lddl_row_spans': (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                               c_void_p, c_void_p, c_void_p]),
    'lddl_masked_lm': (c_int, [c_void_p] * 6),
    'lddl_masked_lm_spans': (c_int, [c_void_p] * 12),
    'lddl_render_masked': (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int32, c_void_p, c_void_p,
                                   c_void_p, c_int64, c_int64, c_void_p, c_void_p, c_int64, ctypes.POINTER(c_int64),
                                   c_void_p]),
    'lddl_render_strings': (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int64,
                                    c_int32, c_int32, c_void_p, c_void_p, c_int64, ctypes.POINTER(c_int64),
                                    c_void_p]),
    'lddl_render_npy': (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_int64, c_void_p, c_int32, c_int32, c_void_p,
                                c_void_p, c_int64, ctypes.POINTER(c_int64), c_void_p]),
    'lddl_row_docs': (c_int, [c_void_p, c_void_p, c_void_p, c_void_p]),
    'lddl_collate_seq_len': (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int32,
                                     ctypes.POINTER(c_int64), c_void_p]),
    'lddl_collate_bert': (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                  c_void_p, c_void_p, c_int64, c_int64, c_int32, c_int64, c_double, c_uint64,
                                  c_uint64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    'lddl_mask_tokens': (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int64, c_double, c_int64,
                                 c_uint64, c_uint64, c_void_p]),
}

_lib = None


def lib():
  global _lib
  if _lib is None:
    if not os.path.exists(LIB_PATH):
      raise RuntimeError('liblddl_amd.so not built (%s); run python -m lddl_amd.build' % LIB_PATH)
    L = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
      if os.environ.get('LDDL_LIB') and not hasattr(L, name):
        continue  # an A/B build of an older revision (tools/ab_head.sh) lacks the newer entry points
      f = getattr(L, name)
      f.restype = res
      f.argtypes = args
    _lib = L
  return _lib


def check(rc):
  if rc < 0:
    raise RuntimeError('lddl_amd error %d: %s' % (rc, lib().lddl_last_error().decode(errors='replace')))
  return rc
