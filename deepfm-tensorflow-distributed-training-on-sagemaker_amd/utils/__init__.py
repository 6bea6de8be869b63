"""Utilities: counter RNG, logging/metrics, timers, profiling hooks."""
