"""pytest setup: markers and import paths (repo root for `oracle`, the package dir for `encx`)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, 'encodec-pytorch_amd')
for p in (ROOT, PKG, os.path.join(ROOT, 'tests', 'golden')):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (runs through the HIP C-ABI library)')
    config.addinivalue_line('markers', 'slow: long-running CPU test')
