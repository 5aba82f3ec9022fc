"""lddl_amd: MI355X-native hot path of LDDL's BERT/CodeBERT preprocessor.

tokenize -> NSP pair / CodeBERT segment pack -> sequence binning, as HIP
kernels for gfx950 behind the C-ABI in include/lddl_amd.h.
"""
__version__ = '0.1.0'
