"""ctypes binding of the C ABI in include/warehouse_amd.h, built in-tree for two engines:

  lib()       libwarehouse_amd.so   the gfx950 kernels (device memory, HIP streams)
  host_lib()  libwarehouse_host.so  the same entry points on host cores (csrc/host_engine.cpp, g++):
                                    BASELINE config 1 on a host without a GPU

Neither falls back to the other: a missing library raises, and a GPU run never touches the host
engine (batched.py picks the engine from the device a BatchedWarehouse lives on).  torch is imported
first so the HIP library resolves `libamdhip64.so.7` to the HIP runtime torch has already loaded
(one runtime per process; torch owns device memory and streams).
"""
from __future__ import annotations

import ctypes
import os
import re
from typing import Optional

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib", "libwarehouse_amd.so")
# kernel A/B experiments (tools/ab.sh) point this at an alternative build of the same library
LIB_PATH = os.environ.get("WAREHOUSE_AMD_LIB", LIB_PATH)
HOST_LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib", "libwarehouse_host.so")

WH_OK = 0
WH_EINVAL = 22
WH_ENOTSUP = 95
WH_EHIP = 1000
WH_MAX_RACKS = 8

WH_PHASE_ALL = 0
WH_PHASE_PRE_REGEN = 1
WH_PHASE_REGEN = 2

WH_POLICY_GREEDY = 1
WH_POLICY_RANDOM = 2

# every symbol include/warehouse_amd.h declares
SYMBOLS = ("wh_query", "wh_pack", "wh_unpack", "wh_reset", "wh_step", "wh_observe", "wh_policy",
           "wh_rollout", "wh_vector_step", "wh_mlp_query", "wh_mlp_pack", "wh_mlp_forward", "wh_version",
           "wh_observe_x", "wh_mlp_forward_x",
           "wh_check_read", "wh_rollout_prepare", "wh_launch_run", "wh_launch_run_timed", "wh_launch_free",
           "wh_sampler_step", "wh_sampler_step_to", "wh_sampler_rollout", "wh_vector_step_x")


class WhConfig(ctypes.Structure):
    _fields_ = [
        ("area_dimension", ctypes.c_int32),
        ("num_requests", ctypes.c_int32),
        ("num_racks", ctypes.c_int32),
        ("racks", ctypes.c_int32 * WH_MAX_RACKS),
        ("agent_slots", ctypes.c_int32),
        ("episode_duration", ctypes.c_int32),
        ("pickup_wait_duration", ctypes.c_int32),
    ]


class WhLayout(ctypes.Structure):
    _fields_ = [
        ("words_per_env", ctypes.c_int32),
        ("num_pickups", ctypes.c_int32),
        ("num_deliveries", ctypes.c_int32),
        ("obs_len", ctypes.c_int32),
        ("kernel_agents", ctypes.c_int32),
    ]


class WhResetDraws(ctypes.Structure):
    _fields_ = [
        ("spawn", ctypes.c_void_p),
        ("pickups", ctypes.c_void_p),
        ("targets", ctypes.c_void_p),
        ("n", ctypes.c_void_p),
    ]


class WhEpisodeStats(ctypes.Structure):
    _fields_ = [
        ("episode_return", ctypes.c_void_p),
        ("return_sum", ctypes.c_void_p),
        ("episodes", ctypes.c_void_p),
        ("return_min", ctypes.c_void_p),
        ("return_max", ctypes.c_void_p),
    ]


WH_MLP_BF16 = 0
WH_MLP_F32 = 1


class WhMlpDesc(ctypes.Structure):
    _fields_ = [("in_dim", ctypes.c_int32), ("hidden0", ctypes.c_int32), ("hidden1", ctypes.c_int32),
                ("out_dim", ctypes.c_int32), ("precision", ctypes.c_int32)]


class WarehouseNativeError(RuntimeError):
    pass


_lib: Optional[ctypes.CDLL] = None
_host_lib: Optional[ctypes.CDLL] = None

_P = ctypes.c_void_p
_I32, _I64, _U64, _F32 = ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64, ctypes.c_float
_CFG = ctypes.POINTER(WhConfig)


def lib() -> ctypes.CDLL:
    """Load the HIP library (once).  Raises loudly if it has not been built."""
    global _lib
    if _lib is None:
        _lib = _load(LIB_PATH, os.environ.get("WAREHOUSE_AMD_AB") == "1")
    return _lib


def host_lib() -> ctypes.CDLL:
    """Load the host engine (once).  Raises loudly if it has not been built."""
    global _host_lib
    if _host_lib is None:
        _host_lib = _load(HOST_LIB_PATH, False)
    return _host_lib


def _load(path: str, ab: bool) -> ctypes.CDLL:
    if not os.path.exists(path):
        raise WarehouseNativeError(
            f"{path} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "or `make -C rllib-warehouse_amd/csrc`")
    L = ctypes.CDLL(path)
    # Every entry point of include/warehouse_amd.h must be there: argtypes applied to an older build
    # whose signatures differ would turn a missing argument into out-of-bounds device writes.  Only
    # explicit A/B experiments (WAREHOUSE_AMD_AB=1, tools/ab.sh) may load a library lacking some.
    missing = [s for s in SYMBOLS if not hasattr(L, s)]
    if missing and not ab:
        raise WarehouseNativeError(f"{path} lacks entry points {missing}: built from other sources "
                                   "-- rebuild (__graft_entry__.build())")

    class _Sigs:   # (A/B builds only) argtypes of a symbol the library lacks go nowhere
        def __setattr__(self, name, val):
            pass

    class _Lib:
        def __getattr__(self, name):
            try:
                return getattr(L, name)
            except AttributeError:
                return _Sigs()
    S = _Lib()
    S.wh_version.restype = ctypes.c_char_p
    S.wh_version.argtypes = []
    S.wh_query.argtypes = [_CFG, ctypes.POINTER(WhLayout)]
    S.wh_pack.argtypes = [_CFG, _I64] + [_P] * 9 + [_P]
    S.wh_unpack.argtypes = [_CFG, _I64] + [_P] * 9 + [_P]
    S.wh_reset.argtypes = [_CFG, _I64, _P, _P, ctypes.POINTER(WhResetDraws), _I32, _U64, _I64, _P]
    S.wh_step.argtypes = [_CFG, _I64, _P, _P, _P, _I32, _P, _P, _P, _P, _I32, _U64, _I64, _P]
    S.wh_observe.argtypes = [_CFG, _I64, _P, _P, _P]
    S.wh_observe_x.argtypes = [_CFG, _I64, _P, _P, _P, _P]
    S.wh_policy.argtypes = [_CFG, _I64, _P, _I32, _F32, _P, _U64, _I64, _P]
    _ST = ctypes.POINTER(WhEpisodeStats)
    S.wh_rollout.argtypes = [_CFG, _I64, _P, _I32, _I32, _F32, _P, _P, _P, _ST, _I32, _I32, _U64, _I64, _P]
    S.wh_vector_step.argtypes = [_CFG, _I64, _P, _P, _P, _I32, _P, _P, _P, _P, _ST, _I32, _I32, _U64, _I64, _P]
    S.wh_vector_step_x.argtypes = [_CFG, _I64, _P, _P, _P, _I32, _P, _P, _P, _P, _ST, _I32, _I32, _U64, _I64, _P]
    S.wh_sampler_step.argtypes = [_CFG, _I64, _P, _I32, _F32, _P, _P, _P, _ST, _I32, _U64, _I64, _P]
    S.wh_sampler_step_to.argtypes = [_CFG, _I64, _P, _P, _I32, _F32, _P, _P, _ST, _I32, _U64, _I64, _P]
    S.wh_sampler_rollout.argtypes = [_CFG, _I64, _P, _I32, _I32, _F32, _P, _P, _P, _ST, _I32, _U64, _I64, _P]
    _MD = ctypes.POINTER(WhMlpDesc)
    S.wh_mlp_query.argtypes = [_MD, ctypes.POINTER(ctypes.c_int64)]
    S.wh_mlp_pack.argtypes = [_MD] + [_P] * 7
    S.wh_mlp_forward.argtypes = [_MD, _P, _I64, _P, _P, _P, _I32, _U64, ctypes.c_uint32, _P]
    S.wh_mlp_forward_x.argtypes = [_MD, _P, _I64, _P, _P, _P, _I32, _U64, ctypes.c_uint32, _P]
    S.wh_check_read.argtypes = [ctypes.POINTER(ctypes.c_uint64), _I32]
    S.wh_rollout_prepare.argtypes = [_CFG, _I64, _P, _I32, _I32, _F32, _P, _P, _P, _ST, _I32, _I32, _U64, _I64, _P,
                                     ctypes.POINTER(ctypes.c_void_p)]
    S.wh_launch_run.argtypes = [_P]
    S.wh_launch_run_timed.argtypes = [_P, _P, _P]
    S.wh_launch_free.argtypes = [_P]
    S.wh_launch_free.restype = ctypes.c_int
    for name in SYMBOLS:
        if name not in ("wh_version", "wh_launch_free") and hasattr(L, name):
            getattr(L, name).restype = ctypes.c_int
    return L


CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "csrc")
HEADER = os.path.join(os.path.dirname(os.path.dirname(CSRC)), "include", "warehouse_amd.h")
# the one variant an extra library may carry (build_ab/check.so: the assert-mode kernels)
CHECK_VARIANT = "EXTRA=-DWH_CHECK"


def hashed_files(csrc: str = CSRC, header: str = HEADER):
    """The files the library's code depends on, in the order the Makefile hashes them (HASHED):
    csrc/*.hip, *.h, *.cpp and the Makefile in sorted name order, then include/warehouse_amd.h."""
    names = sorted(f for f in os.listdir(csrc) if f.endswith((".hip", ".h", ".cpp")) or f == "Makefile")
    return [os.path.join(csrc, f) for f in names] + [header]


def tree_source_sha(csrc: str = CSRC, header: str = HEADER) -> str:
    """sha256 (16 hex digits) of hashed_files(): the hash the Makefile bakes into wh_version() and
    bench.py:source_sha() ties the committed profiles to."""
    import hashlib

    h = hashlib.sha256()
    for p in hashed_files(csrc, header):
        with open(p, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


_VERSION_RE = re.compile(r"(?:lane-per-env v3|host-engine v1) (?:\(assert mode\) )?sha=([0-9a-f]{16}|unknown)(?: variant=([^\x00]*))?")


def parse_version(version) -> tuple:
    """(sha, variant) of a wh_version() string ("... sha=<16 hex>[ variant=<settings>]"); variant is
    "" for a build with the Makefile's own settings, (None, None) if the string carries no sha."""
    v = version.decode(errors="replace") if isinstance(version, bytes) else version
    m = _VERSION_RE.search(v)
    return (m.group(1), (m.group(2) or "").strip()) if m else (None, None)


def version_sha(version: bytes) -> Optional[str]:
    """The source sha a wh_version() string carries, or None."""
    return parse_version(version)[0]


def file_version(path: str) -> tuple:
    """(sha, variant) baked into a built library file, read from its bytes (no load)."""
    with open(path, "rb") as fh:
        m = re.search(rb"(?:lane-per-env v3|host-engine v1) (?:\(assert mode\) )?sha=(?:[0-9a-f]{16}|unknown)(?: variant=[^\x00]*)?",
                      fh.read())
    return parse_version(m.group(0)) if m else (None, None)


def file_source_sha(path: str) -> Optional[str]:
    """The source sha baked into a built library file, read from its bytes (no load)."""
    return file_version(path)[0]


def check_provenance(version, want: str, allowed_variants=("",), what: str = "library") -> None:
    """Raise WarehouseNativeError unless wh_version() text `version` carries sha `want` and one of
    `allowed_variants` (the production library: none)."""
    sha, variant = parse_version(version)
    if sha != want:
        raise WarehouseNativeError(f"{what} was built from sources sha={sha}, the tree has sha={want}: "
                                   "stale library -- rebuild (__graft_entry__.build())")
    if variant not in allowed_variants:
        raise WarehouseNativeError(f"{what} is a variant build ({variant!r}), not the Makefile's own "
                                   "settings -- rebuild (__graft_entry__.build())")


def verify_provenance(extra_libs=()) -> str:
    """Raise WarehouseNativeError unless the loaded library was built from the sources in this tree
    with the Makefile's own settings (no variant), and every file in `extra_libs` (e.g. the
    assert-mode build_ab/check.so) from the same sources with no variant or the assert-mode one.
    Returns the sha."""
    want = tree_source_sha()
    check_provenance(lib().wh_version(), want, ("",), LIB_PATH)
    for p in extra_libs:
        if not os.path.exists(p):
            raise WarehouseNativeError(f"{p}: missing")
        sha, variant = file_version(p)
        check_provenance(f"lane-per-env v3 sha={sha}" + (f" variant={variant}" if variant else ""), want,
                         ("", CHECK_VARIANT), p)
    return want


def verify_host_provenance() -> str:
    """verify_provenance for the host engine: built from this tree's sources, no variant."""
    want = tree_source_sha()
    check_provenance(host_lib().wh_version(), want, ("",), HOST_LIB_PATH)
    return want


def check(rc: int, what: str) -> None:
    if rc == WH_OK:
        return
    if rc == WH_EINVAL:
        raise ValueError(f"{what}: invalid argument (WH_EINVAL)")
    if rc == WH_ENOTSUP:
        raise WarehouseNativeError(f"{what}: layout not supported by this build (WH_ENOTSUP)")
    if rc >= WH_EHIP:
        raise WarehouseNativeError(f"{what}: HIP error {rc - WH_EHIP}")
    raise WarehouseNativeError(f"{what}: error {rc}")


def make_config(area_dimension, num_requests, racks, agent_slots, episode_duration,
                pickup_wait_duration) -> WhConfig:
    racks = list(racks)
    if len(racks) > WH_MAX_RACKS:
        raise ValueError("at most %d racks" % WH_MAX_RACKS)
    arr = (ctypes.c_int32 * WH_MAX_RACKS)(*(racks + [0] * (WH_MAX_RACKS - len(racks))))
    return WhConfig(int(area_dimension), int(num_requests), len(racks), arr, int(agent_slots),
                    int(episode_duration), int(pickup_wait_duration))


def query(cfg: WhConfig, L=None) -> WhLayout:
    """wh_query of the HIP library (or of the engine L)."""
    out = WhLayout()
    check((L or lib()).wh_query(ctypes.byref(cfg), ctypes.byref(out)), "wh_query")
    return out


def ptr(t, host: bool = False) -> Optional[int]:
    """data pointer of a device tensor -- a host tensor for the host engine (None -> NULL)."""
    if t is None:
        return None
    if t.is_cuda == host:
        raise ValueError("the host engine takes host tensors" if host else "warehouse kernels take device tensors")
    if not t.is_contiguous():
        raise ValueError("warehouse kernels take contiguous tensors")
    return t.data_ptr()


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def stream_of(device) -> int:
    """The current HIP stream of `device` as a raw handle: every launch resolves it, so the
    single-env drop-in pays it several times per step -- the raw accessor skips building a
    torch Stream object (~5 us each).  A host device has none (0)."""
    if isinstance(device, torch.device) and device.type == "cpu":
        return 0
    if _raw_stream is not None:
        idx = device.index if isinstance(device, torch.device) and device.index is not None \
            else torch.cuda.current_device()
        return _raw_stream(idx)
    return torch.cuda.current_stream(device).cuda_stream
