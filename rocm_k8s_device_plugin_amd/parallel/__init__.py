"""Data-plane view of a placement: the xGMI fabric an allocated device set
spans (``fabric``) and the RCCL collective bandwidth measured on it
(``collectives``)."""
from .fabric import Fabric, FabricReport

__all__ = ["Fabric", "FabricReport"]
