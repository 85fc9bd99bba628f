"""Node-local service orchestration (reference rafiki.container)."""
from .container_manager import (ContainerManager, ContainerService, GpuLedger, InProcessManager,  # noqa: F401
                                LocalProcessManager)
