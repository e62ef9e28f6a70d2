"""MI355X-native drop-in for the `warehouse` package of ffahleraz/rllib-warehouse.

Same public names as the reference package (warehouse/__init__.py:1-11): `Warehouse` and the six
variants.  `BatchedWarehouse` is the batched device API (B episodes per GPU).
"""
from . import core
from .core import *  # noqa: F401,F403

from . import variants
from .variants import *  # noqa: F401,F403

from .batched import BatchedWarehouse  # noqa: F401

__all__ = []
__all__.extend(core.__all__)
__all__.extend(variants.__all__)
__all__.append("BatchedWarehouse")

name = "warehouse"
