"""Utilities: FLOP counting, logging, failure context managers, timers, checkpoint/resume."""
