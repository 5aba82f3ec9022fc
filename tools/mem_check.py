"""Device memory headroom after one bench step (GPU box tool):
    python tools/mem_check.py [bench.py flags]"""
import os
import runpy
import sys

sys.argv = ['bench.py', '--steps', '1', '--warmup', '0', '--no-cpu-baseline', '--parquet-parts', '0'] + sys.argv[1:]
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
runpy.run_path(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'bench.py'), run_name='__main__')
import torch  # noqa: E402
free, total = torch.cuda.mem_get_info()
print('device memory: %.1f GB free of %.1f GB (torch allocated %.1f GB)' % (
    free / 1e9, total / 1e9, torch.cuda.memory_allocated() / 1e9), flush=True)
