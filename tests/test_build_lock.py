"""The in-process build of libecx.so (_lib.build, run by lib() on a checkout without a
build) is serialised across processes: under `bench.py --gpus 8` every rank may find the
library missing at once, and eight concurrent `make` runs in one directory would race
on the same objects.  Here four processes call build(only_if_missing=True) on a fresh
copy of the loader whose Makefile records its runs: exactly one runs make."""
import importlib.util
import multiprocessing as mp
import shutil
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]

FAKE_MAKEFILE = """\
all:
\t@echo start >> runs.log
\t@sleep 1
\t@echo built > libecx.so
\t@echo end >> runs.log
"""


def _build_in(pkg):
    spec = importlib.util.spec_from_file_location("ecx_lib_copy", str(Path(pkg) / "_lib.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    assert mod.LIB_PATH == Path(pkg) / "libecx.so"
    mod.build(only_if_missing=True)


def test_concurrent_builds_run_make_once(tmp_path, monkeypatch):
    monkeypatch.delenv("ECX_LIB_PATH", raising=False)
    pkg = tmp_path / "pkg"
    pkg.mkdir()
    shutil.copy(ROOT / "repair-pipelining_amd" / "_lib.py", pkg / "_lib.py")
    (pkg / "Makefile").write_text(FAKE_MAKEFILE)
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_build_in, args=(str(pkg),)) for _ in range(4)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(60)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert (pkg / "runs.log").read_text().split() == ["start", "end"]
    assert (pkg / "libecx.so").read_text().strip() == "built"
