"""Line index of a 2.3 GB file through a memory map (splitnative.line_spans)
at 1 / 8 / 16 threads, alternating (host-only; run on the GPU box's host
share).  python tools/line_index_probe.py [PATH]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
from lddl_amd import splitnative  # noqa: E402


def main():
  p = sys.argv[1] if len(sys.argv) > 1 else '/tmp/lddl_line_probe.txt'
  if not os.path.exists(p):
    line = (b'wiki-1 ' + b'lorem ipsum dolor sit amet. ' * 180)[:5000] + b'\n'
    with open(p, 'wb') as f:
      for _ in range(23):
        f.write(line * 20000)
  for th in (1, 8, 16, 1, 8, 16):
    t0 = time.perf_counter()
    buf = np.memmap(p, dtype=np.uint8, mode='r')
    s, _ = splitnative.line_spans(buf, False, threads=th)
    print('threads %2d: %.3f s, %d lines' % (th, time.perf_counter() - t0, len(s)), flush=True)
    del buf


if __name__ == '__main__':
  main()
