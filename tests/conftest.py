"""Test configuration: registers the ``gpu`` marker and puts the product
package directory (flat modules, as the reference's ``code/`` dir) and the
repo root (for ``oracle``) on sys.path."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "deep-multimodal-fusion-of-dce-mri-and-dwi-for-automated-breast-tumor-classification-w.-foundation_amd")
TOOLS = os.path.join(ROOT, "tools")  # make_golden's seeded recipes
for p in (ROOT, PKG, TOOLS):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")


def pytest_collection_modifyitems(config, items):
    import torch

    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no HIP device")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)
