"""Offline stand-in for autorootcwd (no-op)."""
