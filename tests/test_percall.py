"""The per-call CPU/GPU crossover (SURVEY.md 8(b) group 1; ecx_tune "host_exec_kib").

GPU (tests/native/percall_threshold.cpp on the box): at each drop-in site's call shape --
RS(3,1) encodeParitySingle words (NodeHelper.kt:89), RS(2,2) pair decodes (ClayCodeNode.kt:
125-132), RS(4,2) encodeParity (SampleEncoder.java:83), Clay(4,2) performCoding -- the device
path, the host executor and the library default all give the oracle's bytes, and the default
is within 2x of the restated reference loop at the fine-grained sizes (34 B, 2,174 B).  The
measured table is written to gpurun_out/percall_threshold.jsonl (profiles/r05_percall_threshold.jsonl).
CPU: the executor's arithmetic is checked in tests/test_native.py (every ISA level, under
ASan/UBSan); here, that without a HIP device even a tiny per-call request fails loudly."""
import json
import os
import subprocess
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
EXE = ROOT / "tests" / "native" / "_build" / "percall_threshold"


def default_host_exec_kib() -> int:
    """The library's compiled-in per-call threshold, read in a fresh process (ecx_tune_value:
    no device needed), since the GPU suite sets host_exec_kib 0 in this one."""
    code = ("import sys; sys.path.insert(0, %r); import rpamd; print(rpamd.load().tune_value('host_exec_kib'))"
            % str(ROOT))
    r = subprocess.run([os.environ.get("PYTHON", "python3"), "-c", code], capture_output=True, text=True,
                       timeout=300, env={k: v for k, v in os.environ.items() if k != "ECX_SHAPE_KNOBS"})
    assert r.returncode == 0, r.stderr[-2000:]
    return int(r.stdout.strip().splitlines()[-1])


def measured_crossover_bytes() -> int:
    """The per-call crossover in the committed concurrency sweep (profiles/r06_percall_threshold
    .jsonl, tests/native/percall_threshold.cpp --threads 1 / 16): the smallest size at which the
    device path's aggregate rate beats the host executor's, over every site and thread count."""
    rows = [json.loads(ln) for ln in (ROOT / "profiles" / "r06_percall_threshold.jsonl").read_text().splitlines()]
    cross = [x["crossover_bytes"] for x in rows if "crossover_bytes" in x and x["crossover_bytes"] > 0]
    sizes = [x for x in rows if "bytes" in x]
    assert {x["threads"] for x in sizes} == {1, 16} and {x["case"] for x in sizes} == {"rs22_pair", "clay42"}
    assert all(x["outputs_agree"] for x in sizes)
    return min(cross) if cross else max(x["bytes"] for x in sizes) * 2


def test_default_threshold_is_the_measured_crossover(ecx):
    """the default host_exec_kib is the measured crossover -- the largest size
    below the smallest one at which the device beats the host executor under the reference's
    concurrency (1 and 16 caller threads: 2 MiB, Clay(4,2) at one thread), i.e. 1 MiB; the
    reference's 32 KiB sub-chunk calls run on the calling thread.  The getter refuses shape keys."""
    cross = measured_crossover_bytes()
    assert cross == 2 << 20
    assert default_host_exec_kib() * 1024 == cross // 2
    with pytest.raises(ecx.EcxError):
        ecx.tune_value("depth")


def _has_device(ecx):
    try:
        return ecx.device_count() > 0
    except ecx.EcxError:
        return False


@pytest.mark.host_exec
def test_small_calls_without_a_device_fail_loudly(ecx):
    """A 34-byte encodeParitySingle is below the crossover, but with no HIP device it still
    returns ECX_E_DEVICE: the host executor is a latency path of the GPU library, never a
    fallback for a missing device."""
    if _has_device(ecx):
        pytest.skip("a device is present")
    rs = ecx.ReedSolomon.create(3, 1)
    with pytest.raises(ecx.EcxError) as e:
        rs.encodeParitySingle(np.ones(34, np.uint8), np.zeros(34, np.uint8), 0, 0, 0, 34)
    assert e.value.code == -10


@pytest.mark.gpu
@pytest.mark.host_exec
def test_percall_crossover_vs_oracle(ecx):
    subprocess.run(["make", "-s", "-C", str(ROOT / "tests" / "native")], check=True)
    r = subprocess.run([str(EXE)], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    rows = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    out = ROOT / "gpurun_out"
    if out.is_dir():
        (out / "percall_threshold.jsonl").write_text("".join(json.dumps(x) + "\n" for x in rows))
    assert len(rows) >= 28
    for x in rows:
        assert x["outputs_agree"], x
        assert min(x["device_us"], x["host_exec_us"], x["default_us"], x["oracle_us"]) > 0, x
    by = {(x["case"], x["bytes"]): x for x in rows}
    for key in (("rs31_single", 34), ("rs22_pair", 2174)):  # round-4 verdict item 4's bar
        x = by[key]
        assert x["default_us"] <= 2 * x["oracle_us"] + 0.5, x
    # the library's default threshold (a fresh process: this suite sets 0) is the measured crossover
    # (1 MiB; test_default_threshold_is_the_measured_crossover ties it to the committed profile,
    # which does not travel to the GPU box)
    assert default_host_exec_kib() == 1024


@pytest.mark.gpu
@pytest.mark.host_exec
def test_percall_concurrent_callers_agree(ecx):
    """The concurrent-caller mode of the threshold measurement (the full
    1- and 16-thread sweep to 4 MiB is profiles/r06_percall_threshold.jsonl): 4 threads on the
    RS(2,2) pair and Clay(4,2) performCoding sites up to 64 KiB, both paths byte-identical and
    every call successful under concurrency."""
    subprocess.run(["make", "-s", "-C", str(ROOT / "tests" / "native")], check=True)
    r = subprocess.run([str(EXE), "--threads", "4", "65536"], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    rows = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    sizes = [x for x in rows if "bytes" in x]
    assert len(sizes) == 2 * 6 and {x["case"] for x in sizes} == {"rs22_pair", "clay42"}
    for x in sizes:
        assert x["outputs_agree"] and x["device_calls_per_s"] > 0 and x["host_exec_calls_per_s"] > 0, x
    assert len([x for x in rows if "crossover_bytes" in x]) == 2


@pytest.mark.gpu
@pytest.mark.host_exec
@pytest.mark.parametrize("kib", [0, 8, 1024])
def test_per_call_paths_agree_with_oracle(ecx, kib):
    """codeSomeShards / isParityCorrect / decodeMissingSingle / Clay performCoding at the drop-in
    sizes equal the oracle on the device path (0), the default (8 KiB) and the host path forced up
    to 1 MiB -- including the aliasing rows of code_single (output ^= c * input)."""
    import oracle as O
    ecx.tune("host_exec_kib", kib)
    try:
        rng = np.random.default_rng(kib + 1)
        for L in (34, 2174, 8192 + 7, 40000):
            rows = rng.integers(0, 256, (3, 5), dtype=np.uint8)
            ins = [rng.integers(0, 256, L + 3, dtype=np.uint8) for _ in range(5)]
            outs = [rng.integers(0, 256, L + 3, dtype=np.uint8) for _ in range(3)]
            ref = [o.copy() for o in outs]
            O.code_some_shards(list(rows), ins, ref, 3, L)
            ecx.CodingLoop().codeSomeShards(rows, ins, 5, outs, 3, 3, L)
            assert all((a == b).all() for a, b in zip(outs, ref)), L
            assert ecx.CodingLoop().checkSomeShards(rows, ins, 5, outs, 3, 3, L)
            outs[1][3 + L - 1] ^= 1
            assert not ecx.CodingLoop().checkSomeShards(rows, ins, 5, outs, 3, 3, L)
            x, acc = ins[0][:L].copy(), outs[0][:L].copy()
            want = acc ^ O.mul_table()[rows[2][1]][x]
            ecx.InputOutputByteTableCodingLoopSingle().codeSomeShards(rows, x, 1, acc, 2, 0, L, False)
            assert (acc == want).all(), L
            rs = ecx.ReedSolomon.create(4, 2)
            shards = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(4)] + [np.zeros(L, np.uint8)] * 2
            shards = [s.copy() for s in shards]
            rs.encodeParity(shards, 0, L)
            assert rs.isParityCorrect(shards, 0, L)
            lost = [s.copy() for s in shards]
            lost[0][:] = 0
            lost[5][:] = 0
            rs.decodeMissing(lost, [False, True, True, True, True, False], 0, L)
            assert all((a == b).all() for a, b in zip(lost, shards)), L
        B = 2174
        step = ecx.ClayCodeErasureDecodingStep([1], 4, 2)
        data = [None if i % 6 == 1 else rng.integers(0, 256, B, dtype=np.uint8) for i in range(48)]
        got = [np.zeros(B, np.uint8) for _ in range(8)]
        step.performCoding(data, got, B)
        ref = [np.zeros(B, np.uint8) for _ in range(8)]
        O.Clay(4, 2, [1]).perform_coding([None if d is None else d.copy() for d in data], ref, B)
        assert all((a == b).all() for a, b in zip(got, ref))
    finally:
        ecx.tune("host_exec_kib", 0)
