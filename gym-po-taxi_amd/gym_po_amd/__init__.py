"""gym_po_amd — MI355X-native vectorised env engine for gym_po's POMDP gridworlds.

Drop-in replacements for the reference's vector envs (same constructors / reset / step
semantics), with the batched step/reset running as hand-written HIP kernels (libgympo_amd.so,
C ABI in include/gym_po_amd.h) and outputs returned as torch-ROCm tensors.
"""
from .envs import *  # noqa: F401,F403
from .envs import __all__ as _envs_all

__all__ = list(_envs_all)
__version__ = "0.1.0"
