"""mobheat: MI355X-native drop-in for the per-micro-batch hot path of the reference's streaming job.

Import path: add ``real-time-mobility-heatmap_amd/`` to ``sys.path`` (see ``real-time-mobility-heatmap_amd/__init__.py``).
"""
from ._lib import HM_MEM_DEVICE, HM_MEM_HOST, LIB_PATH, load  # noqa: F401
from .engine import BatchResult, HeatmapEngine, TileRows, latlng_to_cell  # noqa: F401

__all__ = ["HeatmapEngine", "BatchResult", "TileRows", "latlng_to_cell", "load", "LIB_PATH"]
