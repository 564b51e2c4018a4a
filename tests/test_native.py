"""Host-only native checks under AddressSanitizer + UndefinedBehaviorSanitizer:
the planner (gf.cpp, codes.cpp) compiled with g++ together with
tests/native/planner_check.cpp, which round-trips codewords through the
composed RS / Clay / shortened-Clay / LRC maps with a dense host application.
(GPU sanitizers are not available; the sanitizers cover host code only.)"""
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


@pytest.mark.timeout(300)
def test_planner_round_trips_under_asan_ubsan(tmp_path):
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("g++ not available")
    exe = tmp_path / "planner_check"
    srcs = [ROOT / "tests" / "native" / "planner_check.cpp", ROOT / "repair-pipelining_amd" / "csrc" / "gf.cpp",
            ROOT / "repair-pipelining_amd" / "csrc" / "codes.cpp"]
    subprocess.run([gxx, "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-omit-frame-pointer",
                    "-fno-sanitize-recover=all", "-o", str(exe)] + [str(s) for s in srcs], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "planner_check: ok" in r.stdout


@pytest.mark.timeout(300)
def test_host_executor_under_asan_ubsan(tmp_path):
    """The per-call host executor (host_exec.cpp, ecx_tune "host_exec_kib") at every
    instruction-set level this CPU has -- AVX-512BW + GFNI affine multiplies, AVX2 nibble
    tables, scalar product rows -- against Field::mul and a dense application: every product,
    random maps at every vector / block boundary, aliasing outputs, the all-zero check."""
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("g++ not available")
    exe = tmp_path / "host_exec_check"
    srcs = [ROOT / "tests" / "native" / "host_exec_check.cpp", ROOT / "repair-pipelining_amd" / "csrc" / "host_exec.cpp",
            ROOT / "repair-pipelining_amd" / "csrc" / "gf.cpp", ROOT / "repair-pipelining_amd" / "csrc" / "codes.cpp"]
    subprocess.run([gxx, "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-omit-frame-pointer",
                    "-fno-sanitize-recover=all", "-o", str(exe)] + [str(s) for s in srcs], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "host_exec_check: ok" in r.stdout
    assert "isa 2: not on this CPU" not in r.stdout or "isa 1: not on this CPU" not in r.stdout
