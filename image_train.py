#!/usr/bin/env python3
"""Drop-in entry point with the reference's CLI (``image_train.py`` of
tiantengfei/Distributed-tensorflow-for-DCGAN): same 22 flags, same defaults, same syntax.

    python image_train.py --data_dir=train --checkpoint_dir=checkpoint
    torchrun --nproc-per-node 8 image_train.py --batch_size=128        # 8 x MI355X, RCCL DDP
    python image_train.py --job_name=worker --task_index=0 --worker_hosts=h0:2222,h1:2222

``--job_name=ps`` is accepted and exits (there is no parameter server in synchronous DDP).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from distributed_tensorflow_for_dcgan_amd.train.trainer import run  # noqa: E402
from distributed_tensorflow_for_dcgan_amd.utils.flags import parse_flags  # noqa: E402


def main(argv=None) -> int:
    return run(parse_flags(sys.argv[1:] if argv is None else argv))


if __name__ == "__main__":
    sys.exit(main())
