import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# the library's routing test hook (bls_test_force_h2c_fallback) refuses to run without this opt-in
os.environ.setdefault("BLSMI355X_TEST_HOOKS", "1")
for p in (ROOT, os.path.join(ROOT, "eth-consensus-specs_amd"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libblsmi355x.so on the device)")
    config.addinivalue_line("markers", "slow: long-running oracle cases")
