"""MI355X-native re-implementation of NVRx's straggler-detection scoring path.

Only the ``straggler`` subpackage (and the ``common.device_utils`` helper it uses) is
provided: the rest of the reference package (fault tolerance, in-process restart,
checkpointing, health checks) is out of scope for this build.
"""
