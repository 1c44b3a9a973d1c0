import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (HERE, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: longer CPU-side checks")


@pytest.fixture(params=["service", "batch"])
def priority_path(request, monkeypatch):
    """PriorityConsensusDWFA through the submission service (the per-locus API,
    wc_service_priority_consensus) and through the batch path
    (wc_priority_consensus_batch, the streamed launch): hip_runner reads it."""
    monkeypatch.setenv("WC_TEST_PRIORITY_PATH", request.param)
    return request.param
