"""SQLite metadata store (reference rafiki.db)."""
from .database import (Database, DuplicateModelNameError, InvalidModelAccessRightError, InvalidUserTypeError,  # noqa
                       ModelUsedError)
