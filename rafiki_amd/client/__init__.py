"""Python SDK (reference rafiki.client)."""
from .client import Client, RafikiConnectionError  # noqa: F401
