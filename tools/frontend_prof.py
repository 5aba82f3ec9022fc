"""cProfile of the preprocessor CLI on MB of synthetic Wikipedia-style input
(GPU box tool): the bench front-end leg's flags, then the top functions by
cumulative and own time.
    python tools/frontend_prof.py [MB]
"""
import cProfile
import os
import pstats
import shutil
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
  mb = float(sys.argv[1]) if len(sys.argv) > 1 else 100.0
  from lddl_amd import preprocess, synth
  d = tempfile.mkdtemp(prefix='lddl_fep_')
  try:
    c = synth.make_wiki(int(mb * (1 << 20)), seed=11)
    os.makedirs(os.path.join(d, 'wiki', 'en'))
    with open(os.path.join(d, 'wiki', 'en', 'a.txt'), 'w', encoding='utf-8') as f:
      for i, doc in enumerate(c.documents()):
        f.write('wiki-%d %s\n' % (i, ' '.join(doc)))
    argv = ['--wikipedia', os.path.join(d, 'wiki'), '--sentence-splitter', 'rules', '--sink', os.path.join(d, 'out'),
            '--target-seq-length', '128', '--block-size', '1M', '--chunk-mb', '4', '--seed', '7', '--split-workers', '16']
    preprocess.main(preprocess.attach_args().parse_args(argv + ['--sink', os.path.join(d, 'warm')]))  # warm-up
    pr = cProfile.Profile()
    t = time.perf_counter()
    pr.enable()
    files, tm = preprocess.main(preprocess.attach_args().parse_args(argv))
    pr.disable()
    print('wall %.3f s, %d files' % (time.perf_counter() - t, len(files)), {k: round(v, 3) for k, v in tm.items()
                                                                            if isinstance(v, float)})
    st = pstats.Stats(pr)
    st.sort_stats('cumulative').print_stats(35)
    st.sort_stats('tottime').print_stats(25)
  finally:
    shutil.rmtree(d, ignore_errors=True)


if __name__ == '__main__':
  main()
