"""gym_po_amd — MI355X-native vectorised env engine for gym_po's POMDP gridworlds.

Drop-in replacements for the reference's vector envs (same constructors / reset / step
semantics), with the batched step/reset running as hand-written HIP kernels (libgympo_amd.so,
C ABI in include/gym_po_amd.h) and outputs returned as torch-ROCm tensors.

Kernel arguments: set HIP_FORCE_DEV_KERNARG=1 in the environment before the HIP runtime starts (before the first
torch.cuda call) to have the runtime keep kernel arguments in device memory. The package does not change it on
import (that would change kernel-argument placement for every HIP user in the process, and only when imported
early enough); bench.py and the tools set it. The C-ROOMS exact mode's draw-call kernels take ~200-B call
descriptors by value and read them on their critical path: measured 10-12% faster per step with the arguments in
device memory.
"""
from .envs import *  # noqa: E402,F401,F403
from .envs import __all__ as _envs_all  # noqa: E402

__all__ = list(_envs_all)
__version__ = "0.1.0"
