"""Utilities: synthetic workloads, quantities, logging helpers."""
