#!/usr/bin/env python3
"""End-to-end timing of the preprocessor CLI (GPU box tool).

    python tools/frontend_bench.py [MB] [chunk_mb] [--codebert]

Writes MB of synthetic raw input (Wikipedia-style lines ``wiki-<id> <text>``,
or CodeSearchNet-style ``id<CODESPLIT>doc<CODESPLIT>code`` records) to a temp
dir, runs lddl_amd.preprocess.main on it (seq 512, bin 64) and prints one
JSON line: host read / sentence split / GPU / parquet write seconds, how much
of the split the pipeline hid behind the GPU and the writer, and the
end-to-end raw MB/s.  The reference's Punkt split is absent in this image; the
rule-based stand-in takes its place (a Python regex pass, like Punkt a
host-core cost).
"""
import json
import os
import shutil
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
  argv = [a for a in sys.argv[1:] if not a.startswith('--')]
  codebert = '--codebert' in sys.argv
  mb = float(argv[0]) if argv else 64.0
  chunk = float(argv[1]) if len(argv) > 1 else 16.0
  from lddl_amd import synth, preprocess
  d = tempfile.mkdtemp(prefix='lddl_fe_')
  try:
    t0 = time.time()
    if codebert:
      lines = synth.make_code_lines(max(1, int(mb * (1 << 20) / 1700)), seed=11)
      os.makedirs(os.path.join(d, 'code'))
      with open(os.path.join(d, 'code', 'a.txt'), 'wb') as f:
        f.write('\r\n'.join(lines).encode('utf-8'))
      argl = ['--code', os.path.join(d, 'code')]
    else:
      c = synth.make_wiki(int(mb * (1 << 20)), seed=11)
      os.makedirs(os.path.join(d, 'wiki', 'en'))
      docs = c.documents()
      with open(os.path.join(d, 'wiki', 'en', 'a.txt'), 'w', encoding='utf-8') as f:
        for i, doc in enumerate(docs):
          f.write('wiki-%d %s\n' % (i, ' '.join(doc)))
      argl = ['--wikipedia', os.path.join(d, 'wiki'), '--sentence-splitter', 'rules']
    gen_s = time.time() - t0
    raw = sum(os.path.getsize(os.path.join(r, f)) for r, _, fs in os.walk(d) for f in fs)
    args = preprocess.attach_args(codebert=codebert).parse_args(
        argl + ['--sink', os.path.join(d, 'out'), '--target-seq-length', '512', '--bin-size', '64',
                '--block-size', str(1 << 20), '--chunk-mb', str(chunk), '--seed', '7'])
    t0 = time.perf_counter()
    files, t = preprocess.main(args, codebert=codebert)
    el = time.perf_counter() - t0
    t.pop('partitions', None)
    print(json.dumps({'what': 'preprocess CLI end to end (%s)' % ('codebert' if codebert else 'bert'),
                      'raw_mb': raw / 1e6, 'files': len(files), 'seconds': el, 'raw_mb_per_s': raw / 1e6 / el,
                      'gen_s': gen_s, 'chunk_mb': chunk, **t}), flush=True)
  finally:
    shutil.rmtree(d, ignore_errors=True)


if __name__ == '__main__':
  main()
