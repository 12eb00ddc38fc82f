"""fantoch_amd — MI355X-native batched GraphExecutor for fantoch's leaderless protocols.

The product is `libfantoch_amd.so` (HIP kernels for gfx950 behind the C-ABI
declared in include/fantoch_amd.h).  This package is the Python host glue:
  * _lib      — ctypes binding of every C-ABI symbol
  * streams   — host-side packing of commit streams into the tiled plane layout
  * device    — device buffers and the batched executor / metrics / synthesis calls
  * executor  — `GraphExecutor`, the reference's Executor trait over the C-ABI
"""
from ._lib import (FX_OK, FX_ERR_CAPACITY, FX_ERR_NO_DEVICE, FxError, LIB_PATH, check, index,
                   load, make_hdr, pack_dot, plane_words, unpack_dot)

__version__ = "0.1.0"
