"""Lightning integration of the straggler detector (reference: ptl_resiliency/__init__.py).

Only the straggler callback is provided; the fault-tolerance and local-checkpoint
callbacks of the reference package are out of scope for this build.
"""
from .straggler_det_callback import StragglerDetectionCallback  # noqa: F401
