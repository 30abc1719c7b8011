"""Statistic keys of section / kernel summaries (reference: straggler/statistics.py:19-35)."""
import enum


class Statistic(enum.Enum):
    """Statistical measures carried by every section / kernel summary."""

    MIN = enum.auto()
    MAX = enum.auto()
    MED = enum.auto()
    AVG = enum.auto()
    STD = enum.auto()
    NUM = enum.auto()

    def __str__(self):
        return f"{self.name}"

    def __repr__(self):
        return f"{self.__class__.__name__}.{self.name}"
