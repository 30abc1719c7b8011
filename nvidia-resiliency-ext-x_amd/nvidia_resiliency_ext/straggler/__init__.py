"""Straggler detection, MI355X-native (drop-in for nvidia_resiliency_ext.straggler).

Exports the reference's public names (reference straggler/__init__.py:16-18) plus
``StragglerReport`` (alias of ``Report``) and ``ReportGenerator``.
"""
from .reporting import Report, ReportGenerator, StragglerId, StragglerReport  # noqa: F401
from .statistics import Statistic  # noqa: F401
from .straggler import CallableId, Detector  # noqa: F401
from . import reporting  # noqa: F401
