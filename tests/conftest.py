import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    # scripts/sanitize.sh: the product's host C++ built with ASan + UBSan (the
    # same sources and build id; bound before any test loads the library)
    san = os.environ.get("SLIO_SANITIZE_LIB")
    if san:
        sys.path.insert(0, os.path.join(ROOT, "scripts"))
        from variant import use
        use(san)


@pytest.fixture(scope="session")
def oracle_mod():
    from oracle import oracle as O
    O.build()
    return O
