"""Utilities: checkpoints, logging / metrics, profiling timers, seeding."""
