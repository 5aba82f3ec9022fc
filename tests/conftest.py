import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
  sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, 'tests', 'golden')


def pytest_configure(config):
  config.addinivalue_line('markers', 'gpu: needs a ROCm GPU (MI355X) and liblddl_amd.so')


@pytest.fixture(scope='session')
def golden():
  def load(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)
  return load


@pytest.fixture(scope='session')
def gpu():
  import torch
  if not torch.cuda.is_available():
    pytest.skip('no GPU')
  from lddl_amd import build
  build.build_hip()
  return torch.device('cuda', 0)
