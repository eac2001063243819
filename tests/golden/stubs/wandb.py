"""Offline stand-in for wandb (never initialised by the fixture capture)."""


def init(*args, **kwargs):
    raise RuntimeError("wandb is not available offline")


def log(*args, **kwargs):
    raise RuntimeError("wandb is not available offline")
