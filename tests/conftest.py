import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
TESTS = os.path.dirname(os.path.abspath(__file__))
if TESTS not in sys.path:
    sys.path.insert(0, TESTS)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: larger CPU cases")


GOLDEN = os.path.join(TESTS, "golden")
FIXTURES = os.path.join(GOLDEN, "fixtures")
SYNTH = os.path.join(GOLDEN, "synthetic")


@pytest.fixture(scope="session")
def python_ref():
    import json
    with open(os.path.join(GOLDEN, "python_ref.json")) as f:
        return json.load(f)["cases"]


@pytest.fixture(scope="session")
def librs_ka():
    import json
    with open(os.path.join(GOLDEN, "librs_known_answers.json")) as f:
        return json.load(f)
