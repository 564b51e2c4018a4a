"""pytest configuration: the `gpu` marker, repository import paths, and the
package loader for the hyphenated package directory `repair-pipelining_amd/`."""
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
for p in (ROOT, ROOT / "oracle"):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device); run with -m gpu")


@pytest.fixture(scope="session")
def kats():
    import json
    return json.loads((ROOT / "tests" / "golden" / "reference_kats.json").read_text())
