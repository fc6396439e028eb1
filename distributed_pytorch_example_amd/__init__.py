"""MI355X-native distributed data-parallel training framework.

Same capabilities and CLI/env/checkpoint contract as
northflank-examples/distributed-pytorch-example, rebuilt for AMD Instinct
MI355X (gfx950): hand-written CDNA4 HIP kernels for the model ops, a C++
RCCL communicator + bucketed reducer overlapped with backward on a side HIP
stream, and a device-resident data path.
"""
__version__ = "0.1.0"

import os as _os

# RCCL and cross-process GPU tensor sharing fail on dmabuf-only host drivers
# (hipIpcGetMemHandle: invalid argument) unless legacy IPC is off; must be set
# before the HIP runtime initialises.
_os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
