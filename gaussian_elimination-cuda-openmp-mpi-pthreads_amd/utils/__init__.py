"""Utilities: tensor plumbing, timers, IO, result reporting."""
from . import io, report, tensors, timing  # noqa: F401
