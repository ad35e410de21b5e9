"""Hardware models (GPU parts, partition layouts) used to check discovery,
size the fabric model and generate fixtures."""
from .gpu import MI210, MI300X, MI308X, MI355X, REGISTRY, GpuModel, check_inventory, model_for

__all__ = ["GpuModel", "MI355X", "MI300X", "MI308X", "MI210", "REGISTRY", "model_for", "check_inventory"]
