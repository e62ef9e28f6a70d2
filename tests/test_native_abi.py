"""CPU-side checks of the C ABI: the library loads, exports exactly what include/warehouse_amd.h
declares, and validates configurations host-side (no device calls)."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "warehouse_amd.h")


def declared_symbols():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|void|const char\*)\s+(wh_[a-z_]+)\s*\(", text, flags=re.M)))


def test_header_symbols_match_binding():
    from warehouse import _native

    assert declared_symbols() == sorted(_native.SYMBOLS)


def test_library_exports_every_declared_symbol():
    from warehouse import _native

    lib = _native.lib()
    for s in declared_symbols():
        assert hasattr(lib, s), s
    out = subprocess.run(["nm", "-D", "--defined-only", _native.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r" T (wh_[a-z_]+)$", out, flags=re.M))
    assert exported == set(declared_symbols())
    assert _native.lib().wh_version().startswith(b"warehouse_amd gfx950")


def test_library_built_from_this_tree():
    """Provenance: wh_version() carries the sha of every file the code depends on (kernel sources,
    version.cpp, the Makefile with its flags, include/warehouse_amd.h) equal to the tree's, and no
    variant; the assert-mode build carries the same sha and only the WH_CHECK variant."""
    from warehouse import _native

    sha = _native.tree_source_sha()
    assert _native.version_sha(_native.lib().wh_version()) == sha
    assert _native.verify_provenance(extra_libs=[os.path.join(ROOT, "build_ab", "check.so")]) == sha
    assert _native.file_version(_native.LIB_PATH) == (sha, "")
    assert _native.file_version(os.path.join(ROOT, "build_ab", "check.so")) == (sha, _native.CHECK_VARIANT)
    names = [os.path.basename(p) for p in _native.hashed_files()]
    assert {"Makefile", "version.cpp", "warehouse_amd.hip", "policy_mlp.hip", "philox.h", "warehouse_amd.h"} <= set(names)


def _probe_version(tmp_path, *make_args):
    """wh_version() of a build with these make settings (the Makefile's version_probe target: g++ on
    version.cpp only, no kernels compiled)."""
    import ctypes

    csrc = os.path.join(ROOT, "rllib-warehouse_amd", "csrc")
    subprocess.run(["make", "-s", "-C", csrc, "version_probe", f"OBJDIR={tmp_path}", *make_args], check=True)
    L = ctypes.CDLL(os.path.join(str(tmp_path), "version_probe.so"))
    L.wh_version.restype = ctypes.c_char_p
    return L.wh_version()


def test_variant_build_fails_provenance(tmp_path):
    """A library built from the same sources but with another -D flag, scheduler or flag set carries
    a variant tag, and verify_provenance's check refuses it as the production library (the assert-mode
    tag is accepted only for the extra check.so)."""
    from warehouse import _native

    sha = _native.tree_source_sha()
    plain = _probe_version(tmp_path / "plain")
    assert _native.parse_version(plain) == (sha, "")
    _native.check_provenance(plain, sha)
    for k, args in enumerate((["EXTRA=-DWH_ABLATION"], ["EXTRA=-DWH_FORCE_NOREV"], ["SCHED_warehouse_amd=-mllvm -amdgpu-sched-strategy=max-ilp"],
                 ["FLAGS=--offload-arch=gfx950 -O1"])):
        v = _probe_version(tmp_path / f"v{k}", *args)   # (a distinct path each: dlopen caches by path)
        got_sha, variant = _native.parse_version(v)
        assert got_sha == sha and variant == args[0], v
        with pytest.raises(_native.WarehouseNativeError, match="variant"):
            _native.check_provenance(v, sha)
    chk = _probe_version(tmp_path / "check", "EXTRA=-DWH_CHECK")
    assert b"assert mode" in chk
    _native.check_provenance(chk, sha, ("", _native.CHECK_VARIANT))
    with pytest.raises(_native.WarehouseNativeError, match="variant"):
        _native.check_provenance(chk, sha)
    with pytest.raises(_native.WarehouseNativeError, match="stale"):
        _native.check_provenance(plain, "0" * 16)


@pytest.mark.parametrize("variant", ["small", "medium", "large"])
def test_query_layouts(variant):
    from warehouse import _native
    from warehouse._geometry import GEOMETRY

    g = GEOMETRY[variant]
    for na in range(1, g["max_agents"] + 1):
        cfg = _native.make_config(g["D"], g["R"], g["racks"], na, g["T"], g["W"])
        lo = _native.query(cfg)
        P = 4 * len(g["racks"]) ** 2
        assert lo.num_pickups == P and lo.num_deliveries == 4 * (g["D"] - 4)
        assert lo.words_per_env == 2 + na + 2 * (P // 4)
        assert lo.obs_len == 9 * g["R"] + 1
        assert lo.kernel_agents >= na


def test_query_rejects_bad_configs():
    from warehouse import _native

    bad = [
        (12, 4, (4, 8), 5, 200, 200),      # more agents than requests (core.py:89)
        (12, 4, (4, 8), 0, 200, 200),      # no agents
        (12, 4, (4, 8), 2, 200, 0),        # zero wait
        (12, 4, (4, 8), 2, 200, 256),      # W does not fit the 8-bit timer plane
    ]
    for c in bad:
        with pytest.raises(ValueError):
            _native.query(_native.make_config(*c))
    with pytest.raises(_native.WarehouseNativeError):   # racks on the border: no kernel for it
        _native.query(_native.make_config(12, 4, (1, 8), 2, 200, 200))
    with pytest.raises(_native.WarehouseNativeError):   # geometry with no compiled kernel
        _native.query(_native.make_config(14, 4, (4, 8), 2, 200, 200))


def test_no_silent_fallback_between_engines():
    """Without a HIP device the classes run on the host engine (libwarehouse_host.so, product C++),
    never on the oracle; naming a HIP device on such a host raises instead of moving to the host,
    and the device-only policy network refuses the host.  With a HIP device the default is the
    gfx950 library."""
    import torch
    import warehouse
    import warehouse.policy  # noqa: F401
    from warehouse import _native

    if torch.cuda.is_available():
        env = warehouse.BatchedWarehouse("small", 4, 2)
        assert not env.host and env._lib is _native.lib()
        return
    env = warehouse.BatchedWarehouse("small", 4, 2)
    assert env.host and env._lib is _native.host_lib() and env.device.type == "cpu"
    assert warehouse.WarehouseSmall(2)._engine.host
    with pytest.raises(RuntimeError, match="no HIP device"):
        warehouse.BatchedWarehouse("small", 4, 2, device="cuda")
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        warehouse.policy.MLPPolicy("small")


def test_mlp_query_shapes():
    """wh_mlp_query: the three SAC policy_model shapes (scripts/experiments/warehouse-*-sac) and
    nothing else; host only."""
    import ctypes

    from warehouse import _native

    lib = _native.lib()
    n = ctypes.c_int64()
    for (i, h0, h1) in ((37, 256, 256), (82, 512, 512), (145, 1024, 256)):
        d = _native.WhMlpDesc(i, h0, h1, 9, _native.WH_MLP_BF16)
        assert lib.wh_mlp_query(ctypes.byref(d), ctypes.byref(n)) == _native.WH_OK
        # bf16 weights (padded into MFMA operand order) + f32 biases
        assert n.value >= 2 * (i * h0 + h0 * h1 + 9 * h1) + 4 * (h0 + h1 + 9)
        assert n.value % 16 == 0 and n.value < 8 * (2 * (i * h0 + h0 * h1 + 32 * h1))
        d = _native.WhMlpDesc(i, h0, h1, 9, _native.WH_MLP_F32)
        assert lib.wh_mlp_query(ctypes.byref(d), ctypes.byref(n)) == _native.WH_OK
        # f32 weights in operand-stream order (layer 0 padded, recomputed per pass) + f32 biases
        assert n.value >= 4 * (i * h0 + h0 * h1 + 9 * h1) + 4 * (h0 + h1 + 9)
        assert n.value % 16 == 0 and n.value < 4 * (4 * (i + 32) * h0 + h0 * h1 + 32 * h1) + 4 * (h0 + h1 + 32) + 4096
    for bad in ((82, 512, 256, 9, 0), (82, 512, 512, 4, 0), (40, 256, 256, 9, 0), (82, 512, 512, 9, 2)):
        d = _native.WhMlpDesc(*bad)
        assert lib.wh_mlp_query(ctypes.byref(d), ctypes.byref(n)) == _native.WH_ENOTSUP
    assert lib.wh_mlp_query(None, ctypes.byref(n)) == _native.WH_EINVAL
