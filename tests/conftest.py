import importlib
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "oracle"), os.path.join(REPO, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


@pytest.fixture(scope="session")
def pkg():
    return importlib.import_module("minion-plasmid-consensus_amd")


# experiments only: MPC_TEST_LIB=exp/v/<variant>.so runs the suite against a
# variant build of libmpc.so (engine.set_library, before anything loads it)
if os.environ.get("MPC_TEST_LIB"):
    importlib.import_module("minion-plasmid-consensus_amd").engine.set_library(os.path.abspath(os.environ["MPC_TEST_LIB"]))
