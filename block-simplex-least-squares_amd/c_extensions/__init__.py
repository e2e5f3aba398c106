"""MI355X drop-in for the reference package python/c_extensions (see c_extensions.py)."""
