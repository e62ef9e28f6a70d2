"""SURVEY.md §5 (race detection / sanitizers): the host C++ of the library under AddressSanitizer +
LeakSanitizer.  `make asan` compiles the library's sources with -fsanitize=address on the host side
(device code unoptimised, never launched) and links tests/asan/abi_asan.cpp, which drives the C ABI's
config validation, the launch-handle lifecycle (prepare / run / free; double free, use after free and
foreign handles refused; failing prepares must not leak) and the other entry points' argument checks
on this GPU-less machine.  A clean run prints "ASAN ABI OK" and exits 0 with no sanitizer report."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "rllib-warehouse_amd", "csrc")


@pytest.mark.timeout(900)
def test_host_abi_under_address_sanitizer():
    b = subprocess.run(["make", "-s", "-C", CSRC, "-j2", "asan"], capture_output=True, text=True, timeout=850)
    assert b.returncode == 0, b.stderr[-3000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1")
    r = subprocess.run([os.path.join(ROOT, "build", "asan", "abi_asan")], capture_output=True, text=True,
                       timeout=120, env=env)
    assert "AddressSanitizer" not in r.stderr and "LeakSanitizer" not in r.stderr, r.stderr[-3000:]
    assert r.returncode == 0 and "ASAN ABI OK" in r.stdout, (r.stdout + r.stderr)[-3000:]


@pytest.mark.timeout(600)
def test_host_engine_under_address_and_undefined_sanitizers():
    """The host engine (csrc/host_engine.cpp, BASELINE config 1's GPU-less path) compiled with
    -fsanitize=address,undefined and driven by tests/asan/host_engine_asan.cpp: resets (philox and
    injected), steps with dict orders of every length up to 4*NA and split-phase injected
    regeneration, rollouts across episode ends with metrics, masked vector steps, sampler steps and
    fragments, pack/unpack -- Small/Medium/Large, Train agent counts, ragged batches, every buffer
    exactly the size the header states.  No report, "ASAN HOST ENGINE OK"."""
    out = os.path.join(ROOT, "build", "asan", "host_engine_asan")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    cmd = ["g++", "-O1", "-g", "-std=c++17", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
           "-fno-omit-frame-pointer", "-DWH_HOST_ENGINE", '-DWH_SOURCE_SHA="asan"', '-DWH_VARIANT=""',
           "-I" + os.path.join(ROOT, "include"), os.path.join(CSRC, "host_engine.cpp"),
           os.path.join(CSRC, "version.cpp"), os.path.join(ROOT, "tests", "asan", "host_engine_asan.cpp"), "-o", out]
    b = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert b.returncode == 0, b.stderr[-3000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([out], capture_output=True, text=True, timeout=300, env=env)
    assert "Sanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-3000:]
    assert r.returncode == 0 and "ASAN HOST ENGINE OK" in r.stdout, (r.stdout + r.stderr)[-3000:]
