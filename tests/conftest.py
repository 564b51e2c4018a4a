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


@pytest.fixture(scope="session")
def ecx():
    """The product package (repair-pipelining_amd/), loaded via rpamd."""
    import rpamd
    return rpamd.load()


def shortened_clay_oracle(k, m, v, erased_real, inputs_real, B):
    """Oracle of a shortened Clay code: the reference Clay(k+v, m)
    (ClayCodeErasureDecodingStep.java:53-107, restated in oracle/ecx_oracle.c) run with
    the v virtual data nodes zero-filled.  inputs_real / the result use the REAL node
    numbering of the shortened code (slot z*(k+m) + node; output z*|E| + j)."""
    import numpy as np
    import oracle as O
    n_r, n_u = k + m, k + v + m
    und = lambda r: r if r < k else r + v  # noqa: E731
    c = O.Clay(k + v, m, [und(e) for e in erased_real])
    a = c.alpha
    inputs = [None] * (n_u * a)
    for z in range(a):
        for r in range(n_r):
            inputs[z * n_u + und(r)] = inputs_real[z * n_r + r]
        for u in range(k, k + v):
            inputs[z * n_u + u] = np.zeros(B, np.uint8)
    outs = [np.zeros(B, np.uint8) for _ in range(len(erased_real) * a)]
    c.perform_coding(inputs, outs, B)
    return outs


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
