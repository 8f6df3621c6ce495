"""Checkpoint format, training statistics, logging helpers."""
