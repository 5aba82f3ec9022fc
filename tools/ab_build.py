"""Build A/B variants of liblddl_amd.so with extra -D defines into ab/:

    python tools/ab_build.py NAME DEF[=V] ...   -> ab/lib_NAME.so (load with LDDL_LIB=ab/lib_NAME.so)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from lddl_amd import build  # noqa: E402

if __name__ == '__main__':
  os.makedirs(os.path.join(ROOT, 'ab'), exist_ok=True)
  print(build.build_hip(force=True, lib=os.path.join(ROOT, 'ab', 'lib_%s.so' % sys.argv[1]), defines=sys.argv[2:]))
