"""Device selection for collectives (reference: common/device_utils.py:23-39, 68-76)."""
import os
from typing import Optional

import torch

__all__ = ["get_current_device", "get_current_device_type", "get_local_device_count",
           "get_distributed_backend", "get_distributed_init_method"]

_current_device: Optional[torch.device] = None


def get_current_device() -> torch.device:
    """``cuda:LOCAL_RANK`` when a GPU is visible (set as current), else DEFAULT_DEVICE/cpu."""
    global _current_device
    if _current_device is None:
        if torch.cuda.is_available():
            _current_device = torch.device(f"cuda:{int(os.getenv('LOCAL_RANK', 0))}")
            torch.cuda.set_device(_current_device)
        else:
            _current_device = torch.device(os.getenv("DEFAULT_DEVICE", "cpu"))
    return _current_device


def get_current_device_type() -> str:
    return "cuda" if torch.cuda.is_available() else os.getenv("DEFAULT_DEVICE_TYPE", "cpu")


def get_local_device_count() -> int:
    return torch.cuda.device_count() if torch.cuda.is_available() else 1


def get_distributed_backend(backend=None) -> str:
    if backend is not None:
        return backend
    return "nccl" if torch.cuda.is_available() else "gloo"


def get_distributed_init_method(backend: Optional[str] = None) -> str:
    return "env://"
