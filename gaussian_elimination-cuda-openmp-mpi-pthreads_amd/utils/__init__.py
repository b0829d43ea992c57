"""Utilities: tensor plumbing, timers, IO, result reporting."""
from . import checkpoint, io, report, tensors, timing  # noqa: F401
