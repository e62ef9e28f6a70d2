"""ctypes binding of the C ABI in include/warehouse_amd.h (libwarehouse_amd.so, built in-tree).

There is no CPU fallback: if the library or a HIP device is missing, every entry point raises.
torch is imported first so the library resolves `libamdhip64.so.7` to the HIP runtime torch has
already loaded (one runtime per process; torch owns device memory and streams).
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib", "libwarehouse_amd.so")
# kernel A/B experiments (tools/ab.sh) point this at an alternative build of the same library
LIB_PATH = os.environ.get("WAREHOUSE_AMD_LIB", LIB_PATH)

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
           "wh_check_read", "wh_rollout_prepare", "wh_launch_run", "wh_launch_run_timed", "wh_launch_free")


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

_P = ctypes.c_void_p
_I32, _I64, _U64, _F32 = ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64, ctypes.c_float
_CFG = ctypes.POINTER(WhConfig)


def lib() -> ctypes.CDLL:
    """Load the HIP library (once).  Raises loudly if it has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise WarehouseNativeError(
            f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "or `make -C rllib-warehouse_amd/csrc` (there is no CPU fallback)")
    L = ctypes.CDLL(LIB_PATH)
    L.wh_version.restype = ctypes.c_char_p
    L.wh_version.argtypes = []
    L.wh_query.argtypes = [_CFG, ctypes.POINTER(WhLayout)]
    L.wh_pack.argtypes = [_CFG, _I64] + [_P] * 9 + [_P]
    L.wh_unpack.argtypes = [_CFG, _I64] + [_P] * 9 + [_P]
    L.wh_reset.argtypes = [_CFG, _I64, _P, _P, ctypes.POINTER(WhResetDraws), _I32, _U64, _I64, _P]
    L.wh_step.argtypes = [_CFG, _I64, _P, _P, _P, _P, _P, _P, _P, _I32, _U64, _I64, _P]
    L.wh_observe.argtypes = [_CFG, _I64, _P, _P, _P]
    L.wh_observe_x.argtypes = [_CFG, _I64, _P, _P, _P, _P]
    L.wh_policy.argtypes = [_CFG, _I64, _P, _I32, _F32, _P, _U64, _I64, _P]
    _ST = ctypes.POINTER(WhEpisodeStats)
    L.wh_rollout.argtypes = [_CFG, _I64, _P, _I32, _I32, _F32, _P, _P, _P, _ST, _I32, _I32, _U64, _I64, _P]
    L.wh_vector_step.argtypes = [_CFG, _I64, _P, _P, _P, _P, _P, _P, _ST, _I32, _I32, _U64, _I64, _P]
    _MD = ctypes.POINTER(WhMlpDesc)
    L.wh_mlp_query.argtypes = [_MD, ctypes.POINTER(ctypes.c_int64)]
    L.wh_mlp_pack.argtypes = [_MD] + [_P] * 7
    L.wh_mlp_forward.argtypes = [_MD, _P, _I64, _P, _P, _P, _I32, _U64, ctypes.c_uint32, _P]
    L.wh_mlp_forward_x.argtypes = [_MD, _P, _I64, _P, _P, _P, _I32, _U64, ctypes.c_uint32, _P]
    L.wh_check_read.argtypes = [ctypes.POINTER(ctypes.c_uint64), _I32]
    L.wh_rollout_prepare.argtypes = [_CFG, _I64, _P, _I32, _I32, _F32, _P, _P, _P, _ST, _I32, _I32, _U64, _I64, _P,
                                     ctypes.POINTER(ctypes.c_void_p)]
    L.wh_launch_run.argtypes = [_P]
    L.wh_launch_run_timed.argtypes = [_P, _P, _P]
    L.wh_launch_free.argtypes = [_P]
    L.wh_launch_free.restype = None
    for name in SYMBOLS:
        if name != "wh_version":
            getattr(L, name).restype = ctypes.c_int
    _lib = L
    return L


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


def query(cfg: WhConfig) -> WhLayout:
    out = WhLayout()
    check(lib().wh_query(ctypes.byref(cfg), ctypes.byref(out)), "wh_query")
    return out


def ptr(t) -> Optional[int]:
    """data pointer of a device tensor (None -> NULL)."""
    if t is None:
        return None
    if not t.is_cuda:
        raise ValueError("warehouse kernels take device tensors")
    if not t.is_contiguous():
        raise ValueError("warehouse kernels take contiguous tensors")
    return t.data_ptr()


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def stream_of(device) -> int:
    """The current HIP stream of `device` as a raw handle: every launch resolves it, so the
    single-env drop-in pays it several times per step -- the raw accessor skips building a
    torch Stream object (~5 us each)."""
    if _raw_stream is not None:
        idx = device.index if isinstance(device, torch.device) and device.index is not None \
            else torch.cuda.current_device()
        return _raw_stream(idx)
    return torch.cuda.current_stream(device).cuda_stream
