"""MI355X-native distributed DCGAN training framework.

Same capabilities as ``tiantengfei/Distributed-tensorflow-for-DCGAN`` (TF parameter-server
DCGAN), re-designed for AMD Instinct MI355X (gfx950): hand-written HIP/MFMA kernels for
the compute path, synchronous data parallelism over RCCL/xGMI, a native C++ TFRecord
loader, TF-compatible checkpoints/summaries and the ``image_train.py`` flag surface.
"""
__version__ = "0.1.0"

from .models.config import DCGANConfig  # noqa: F401
from .models.dcgan import DCGAN  # noqa: F401
