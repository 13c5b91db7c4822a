"""The driver's round-end smoke step (`__graft_entry__.smoke()`: one small RLC encode + decode and an
XOR round trip on cuda:0, compared with the oracle) run as a GPU test, so a tree whose smoke would
fail is caught by `pytest -m gpu` first."""
import os
import sys

import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))


@pytest.mark.gpu
def test_graft_entry_smoke():
    sys.path.insert(0, ROOT)
    import __graft_entry__
    __graft_entry__.smoke()
