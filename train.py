"""Distributed image-classification training CLI (reference: train.py).

Launch exactly like the reference (README.md:5-7, with the flag typo fixed):

    python -m torch.distributed.launch --nproc-per-node=8 train.py --datadir DATA
    torchrun --nproc-per-node=8 --master-addr 127.0.0.1 train.py --datadir DATA
    python train.py --synthetic --model resnet18 --image-size 32 --device cpu   # no GPU

Reference flags ``--local_rank/--local-rank``, ``--datadir``, ``--batchsize`` keep
their names and defaults; every constant the reference hard-codes is a flag
with the reference value as default (see ``engine/config.py``).
"""
from __future__ import annotations

import sys

from pytorch_imageclassification_distributed_amd.engine import Trainer, build_parser
from pytorch_imageclassification_distributed_amd.parallel import destroy, init_distributed


def main(argv=None):
    args = build_parser().parse_args(argv)
    if not args.synthetic and not args.datadir:
        build_parser().error("--datadir is required unless --synthetic is given")
    ctx = init_distributed(device=args.device, backend=args.backend, local_rank=args.local_rank,
                           timeout_min=args.timeout_min)
    try:
        trainer = Trainer(args, ctx)
        return trainer.fit()
    finally:
        destroy()


if __name__ == "__main__":
    main(sys.argv[1:])
