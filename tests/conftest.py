import os
import sys

import pytest

# The GPU tests run with bench.py's hardware-queue count (HIP reads it once, at its first call; the
# GPU boxes export 4): proof slots of the batch prover then really overlap, so the tests exercise the
# benchmarked concurrency (tests/test_gpu_metric.py).
os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("ZKFL_HW_QUEUES", "28")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(ROOT, "verifiable-federated-training-with-zero-knowledge-proofs-zk-fl-_amd")
for p in (ROOT, PKG_DIR):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through the C ABI)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def gpu_ctx():
    from zkfl import native
    ctx = native.Context(0)
    yield ctx
    ctx.close()
