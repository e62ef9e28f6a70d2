"""MI355X-native drop-in for the `warehouse` package of ffahleraz/rllib-warehouse.

Same public names as the reference package (warehouse/__init__.py:1-11): `Warehouse` and the six
variants.  `BatchedWarehouse` is the batched device API (B episodes per GPU); `WarehouseVectorEnv` /
`WarehouseBaseEnv` present a batch to an RLlib-style sampler (warehouse/vector.py).
"""
from . import core
from .core import *  # noqa: F401,F403

from . import variants
from .variants import *  # noqa: F401,F403

from .batched import BatchedWarehouse, EpisodeStats  # noqa: F401
from .vector import WarehouseBaseEnv, WarehouseVectorEnv  # noqa: F401

__all__ = []
__all__.extend(core.__all__)
__all__.extend(variants.__all__)
__all__ += ["BatchedWarehouse", "EpisodeStats", "WarehouseVectorEnv", "WarehouseBaseEnv"]

name = "warehouse"
