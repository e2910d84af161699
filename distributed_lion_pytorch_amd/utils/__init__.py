"""Metrics, timers, checkpoint helpers and synthetic data."""
