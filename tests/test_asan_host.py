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
