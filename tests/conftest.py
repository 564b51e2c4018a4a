"""pytest configuration: the `gpu` marker, repository import paths, and the
package loader for the hyphenated package directory `repair-pipelining_amd/`."""
import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
# The tests force launch shapes (every shape must give the same bytes), so this process opts in
# to libecx's shape knobs (include/ecx_tune.h); test_abi checks a process without the opt-in.
os.environ["ECX_SHAPE_KNOBS"] = "1"
for p in (ROOT, ROOT / "oracle"):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "diag: needs the diagnostic library (make DIAG=1; ECX_LIB_PATH=.../libecx_diag.so)")
    config.addinivalue_line("markers", "host_exec: exercises the per-call host executor (ecx_tune host_exec_kib); "
                                       "every other test runs its per-call calls on the device")


def pytest_runtest_setup(item):
    """Tests of the measured-and-rejected kernels (marked `diag`) run only against the
    diagnostic library; the product library does not contain those kernels."""
    if item.get_closest_marker("diag"):
        import rpamd
        if not rpamd.load().is_diag():
            pytest.skip("diagnostic-library kernel (make DIAG=1, ECX_LIB_PATH=.../libecx_diag.so)")


@pytest.fixture(autouse=True)
def _per_call_on_device(request):
    """Per-call entry points below the crossover run on the host executor by default
    (ecx_tune "host_exec_kib"); the parity tests exercise the HIP kernels, so every test not
    marked `host_exec` runs with the threshold at 0 (every call on the device)."""
    import rpamd
    ecx = rpamd.load(shape_knobs=True)
    if request.node.get_closest_marker("host_exec") is None:
        ecx.tune("host_exec_kib", 0)
    yield


def diag_build() -> bool:
    import rpamd
    return rpamd.load().is_diag()


@pytest.fixture(scope="session")
def kats():
    import json
    return json.loads((ROOT / "tests" / "golden" / "reference_kats.json").read_text())


@pytest.fixture(scope="session")
def ecx():
    """The product package (repair-pipelining_amd/), loaded via rpamd."""
    import rpamd
    return rpamd.load(shape_knobs=True)


def shortened_clay_oracle(k, m, v, erased_real, inputs_real, B):
    """Oracle of a shortened Clay code: oracle.shortened_clay_perform_coding (the
    reference Clay(k+v, m) with the virtual data nodes zero-filled)."""
    import oracle as O
    return O.shortened_clay_perform_coding(k, m, v, erased_real, inputs_real, B)


def gf_apply_numpy(matrix, inputs):
    """Test-side reference application of a dense GF(256) map with the oracle's
    multiplication table: out[o] = XOR_j M[o][j] * in[j]."""
    import numpy as np
    import oracle as O
    mt = O.mul_table()
    outs = []
    for row in matrix:
        acc = np.zeros(len(inputs[0]), np.uint8)
        for c, x in zip(row, inputs):
            if c:
                acc ^= mt[c][x]
        outs.append(acc)
    return outs
