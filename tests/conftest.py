import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the native HIP kernels)")


@pytest.fixture(autouse=True)
def _reset_context():
    from flink_ml_amd.parallel import context

    yield
    if not (context._CTX is not None and context._CTX.is_distributed):
        context.reset_context()
