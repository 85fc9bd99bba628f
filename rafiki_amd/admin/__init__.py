"""Admin service (reference rafiki.admin)."""
from .admin import Admin  # noqa: F401
from .services_manager import ServicesManager  # noqa: F401
