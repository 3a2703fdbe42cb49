"""Standalone experiment entry points (compat with the reference fedml_experiments tree)."""
