"""A/B variant libraries: python tools/ab_build.py NAME [DEFINE ...] builds
ab/lib_NAME.so with -DDEFINE for each define and, for an argument starting
with '-', that compiler flag as given (objects under ab/lib_NAME_obj,
which .gpurunignore keeps off the GPU box); tools/r5_*.sh load it with
LDDL_LIB.  The working tree's sources, so a variant differs only by its
defines."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lddl_amd import build  # noqa: E402

name = sys.argv[1]
defines = [d for d in sys.argv[2:] if not d.startswith('-')]
extra = [d for d in sys.argv[2:] if d.startswith('-')]
os.makedirs(os.path.join(build.ROOT, 'ab'), exist_ok=True)
print(build.build_hip(force=True, lib=os.path.join(build.ROOT, 'ab', 'lib_%s.so' % name), defines=defines, extra=extra))
