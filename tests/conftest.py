import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
TESTS = os.path.dirname(os.path.abspath(__file__))
if TESTS not in sys.path:
    sys.path.insert(0, TESTS)

# The library and CLI under test.  `make sanitize` points WLD_TEST_BUILD at
# build/asan (host code under ASan + UBSan); the product's own loader has no
# such redirection.
CLI = os.path.join(REPO, "weightedld_amd", "bin", "weighted_ld")
_TEST_BUILD = os.environ.get("WLD_TEST_BUILD")
if _TEST_BUILD:
    import weightedld_amd
    from weightedld_amd import _lib
    _lib.LIB_PATH = weightedld_amd.LIB_PATH = os.path.join(os.path.abspath(_TEST_BUILD), "libweightedld.so")
    CLI = os.path.join(os.path.abspath(_TEST_BUILD), "weighted_ld")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: larger CPU cases")


class ParityReport:
    """Per-field tallies of the GPU-vs-oracle comparisons (test_gpu_parity.agree):
    values compared, max |GPU - reference| among strictly agreeing values, and
    the count and max |GPU - reference| of D' values accepted only because they
    are at least as close to the exact f64 value as the f32 reference."""

    def __init__(self):
        self.f = {}

    def record(self, field, n, max_strict, n_esc, max_esc):
        t = self.f.setdefault(field, [0, 0.0, 0, 0.0])
        t[0] += n
        t[1] = max(t[1], max_strict)
        t[2] += n_esc
        t[3] = max(t[3], max_esc)


PARITY = ParityReport()
# free-form lines for the session summary (tests/test_gpu_refsums.py: how far
# the default path's rows and TSV lines are from lib.rs's on each input, and
# the reference-order path's distance under either horizontal-sum order)
REF_REPORT = []


def pytest_terminal_summary(terminalreporter):
    if REF_REPORT:
        terminalreporter.write_line("reference-parity report (rows and %.3f TSV lines against the oracle):")
        for line in REF_REPORT:
            terminalreporter.write_line("  " + line)
    if not PARITY.f:
        return
    terminalreporter.write_line("parity report (GPU vs oracle, tolerance 1e-5):")
    for field, (n, ms, ne, me) in sorted(PARITY.f.items()):
        terminalreporter.write_line("  %-8s %12d values  max|diff| strict %.3g  escaped via f64 truth: %d (max|diff| %.3g)"
                                    % (field, n, ms, ne, me))


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
