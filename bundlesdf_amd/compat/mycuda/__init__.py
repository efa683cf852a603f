"""`mycuda` package shim: `from mycuda import common` (Utils.py:29)."""
from . import common  # noqa: F401
