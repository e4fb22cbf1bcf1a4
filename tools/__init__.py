"""Synthetic data tools."""
