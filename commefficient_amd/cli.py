"""Federated training command line (``fed_train.py``, ``cv_train.py``,
``gpt2_train.py`` and the ``commeff-train`` console script).  Same flags as
the reference (commefficient_amd/utils/args.py); dispatches to the CV or
GPT-2 driver.

Multi-GPU: launch with torchrun (one process per GPU), e.g.
  torchrun --nproc-per-node 8 --master-addr 127.0.0.1 fed_train.py --dataset_name CIFAR10 ...
or pass --num_devices N and the ranks are spawned here (127.0.0.1 rendezvous).
"""
import os
import sys

from .utils.args import parse_args


def _run(args):
    if args.model == "GPT2DoubleHeads" or args.dataset_name == "PERSONA":
        from .train import gpt2
        return gpt2.main(args)
    from .train import cv
    return cv.main(args)


def _spawned(rank, args):
    _run(args)


def main(argv=None, default_lr=None):
    args = parse_args(default_lr=default_lr, argv=sys.argv[1:] if argv is None else argv)
    if args.num_devices > 1 and "WORLD_SIZE" not in os.environ:
        from .parallel import dist
        dist.spawn(_spawned, args.num_devices, args=(args,), port=args.port)
        return None
    return _run(args)
