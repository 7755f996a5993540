"""Utilities: diagnostics / pretty printers, profiling helpers, metrics logging."""
