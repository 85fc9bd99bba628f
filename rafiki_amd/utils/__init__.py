"""Cross-cutting utilities: auth, logging, service runner."""
