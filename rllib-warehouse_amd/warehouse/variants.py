"""The six named environments of the reference (warehouse/variants.py:19-98), same signatures."""
from typing import Dict

import numpy as np

from ._geometry import GEOMETRY
from .core import Warehouse

__all__ = [
    "WarehouseSmall",
    "WarehouseMedium",
    "WarehouseLarge",
    "WarehouseSmallTrain",
    "WarehouseMediumTrain",
    "WarehouseLargeTrain",
]


def _init(env: Warehouse, size: str, num_agents: int) -> None:
    g = GEOMETRY[size]
    Warehouse.__init__(env, num_agents=num_agents, num_requests=g["R"], area_dimension=g["D"],
                       pickup_racks_arrangement=list(g["racks"]), episode_duration=g["T"],
                       pickup_wait_duration=g["W"])


class WarehouseSmall(Warehouse):
    max_num_agents = GEOMETRY["small"]["max_agents"]

    def __init__(self, num_agents: int) -> None:
        assert 1 <= num_agents <= self.max_num_agents
        _init(self, "small", num_agents)


class WarehouseMedium(Warehouse):
    max_num_agents = GEOMETRY["medium"]["max_agents"]

    def __init__(self, num_agents: int) -> None:
        assert 1 <= num_agents <= self.max_num_agents
        _init(self, "medium", num_agents)


class WarehouseLarge(Warehouse):
    max_num_agents = GEOMETRY["large"]["max_agents"]

    def __init__(self, num_agents: int) -> None:
        assert 1 <= num_agents <= self.max_num_agents
        _init(self, "large", num_agents)


class _TrainMixin:
    """Re-draws the agent count at construction and at every reset (variants.py:65-98), taking
    np.random.randint(1, max + 1) from the global stream exactly where the reference does."""

    def _draw_num_agents(self) -> int:
        return int(np.random.randint(1, self.max_num_agents + 1))

    def reset(self) -> Dict[str, dict]:
        self._base.__init__(self, num_agents=self._draw_num_agents())
        return Warehouse.reset(self)


class WarehouseSmallTrain(_TrainMixin, WarehouseSmall):
    _base = WarehouseSmall

    def __init__(self) -> None:
        WarehouseSmall.__init__(self, num_agents=self._draw_num_agents())


class WarehouseMediumTrain(_TrainMixin, WarehouseMedium):
    _base = WarehouseMedium

    def __init__(self) -> None:
        WarehouseMedium.__init__(self, num_agents=self._draw_num_agents())


class WarehouseLargeTrain(_TrainMixin, WarehouseLarge):
    _base = WarehouseLarge

    def __init__(self) -> None:
        WarehouseLarge.__init__(self, num_agents=self._draw_num_agents())
