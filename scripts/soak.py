"""Repeat the concurrency tests of tests/test_gpu_parity.py N times in one process (races in the
stream leases, host pipes, layout-selection probes or the codec registry would show as a wrong
byte, an error or a hang): test_every_entry_kind_at_once and test_per_call_concurrent_threads.
Usage: python scripts/soak.py [N]  (prints one line per round)."""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for p in (ROOT, ROOT / "oracle", ROOT / "tests"):
    sys.path.insert(0, str(p))

import conftest  # noqa: E402,F401 -- sets ECX_SHAPE_KNOBS before the library loads
import rpamd  # noqa: E402
import torch  # noqa: E402
import test_gpu_parity as T  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    ecx = rpamd.load(shape_knobs=True)
    for i in range(n):
        t0 = time.perf_counter()
        T.test_every_entry_kind_at_once(ecx, torch)
        ecx.tune("host_exec_kib", 0)
        for contexts in (1, 0):
            T.test_per_call_concurrent_threads(ecx, contexts)
        print("soak round %d ok (%.1f s)" % (i, time.perf_counter() - t0), flush=True)


if __name__ == "__main__":
    main()
