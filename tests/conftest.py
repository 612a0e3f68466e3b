import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("oracle", "neptune-core_amd", ""):
    p = os.path.join(ROOT, sub)
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs via gpurun)")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


@pytest.fixture(scope="session")
def ctx():
    import neptune_hip as nh
    c = nh.Context(int(os.environ.get("LOCAL_RANK", "0")))
    yield c
    c.close()


@pytest.hookimpl(trylast=True)  # after -m / -k deselection
def pytest_collection_modifyitems(session, config, items):
    """The config-4 GPU tests draw from oracle/pool4.py's 256 distinct proofs, built once per machine
    in a child process: build it here, after collection and before any test creates a GPU context,
    so the child is never forked from a process that has initialised HIP."""
    users = ("test_gpu_config4", "test_gpu_fs_forms", "test_gpu_input_forms", "test_gpu_group_stream")
    if any(it.get_closest_marker("gpu") and any(u in it.nodeid for u in users) for it in items):
        import pool4  # oracle/: test-data generator
        pool4.load()
