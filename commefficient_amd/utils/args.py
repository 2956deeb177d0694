"""Command-line flags: every flag of the reference (same names, dests and
defaults; /root/reference/CommEfficient/utils.py:102-230)
plus MI355X-build extensions (marked NEW below).

The returned ``argparse.Namespace`` is the single config object passed through
the framework, like the reference's.  Validity checks mirror the reference's
asserts (utils.py:225-228, fed_worker.py:221-228, fed_aggregator.py:484-486,
512,545,573-576) but raise ``ValueError`` with a readable message up-front
instead of asserting deep inside a worker process.
"""
from __future__ import annotations

import argparse
import os
import socket
from typing import Optional, Sequence

import numpy as np

FED_DATASETS = {"CIFAR10": 10, "CIFAR100": 100, "EMNIST": 62, "ImageNet": 1000, "PERSONA": -1}
MODES = ["sketch", "true_topk", "local_topk", "fedavg", "uncompressed"]
ERROR_TYPES = ["none", "local", "virtual"]


def num_classes_of_dataset(name: str) -> int:
    return FED_DATASETS[name]


def is_port_in_use(port: int) -> bool:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        return s.connect_ex(("127.0.0.1", port)) == 0


def _model_names():
    from .. import models
    return models.model_names()


def build_parser(default_lr: Optional[float] = None) -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="commefficient_amd federated / DP training")

    # meta-args
    p.add_argument("--test", action="store_true", dest="do_test")
    p.add_argument("--mode", choices=MODES, default="sketch")
    p.add_argument("--tensorboard", dest="use_tensorboard", action="store_true")
    p.add_argument("--seed", type=int, default=21)

    # data/model args
    p.add_argument("--model", default="ResNet9", help="Name of the model.", choices=_model_names())
    p.add_argument("--finetune", action="store_true", dest="do_finetune")
    p.add_argument("--checkpoint", action="store_true", dest="do_checkpoint")
    p.add_argument("--checkpoint_path", type=str, default="./checkpoint",
                   help="Path or url to cache the model")
    p.add_argument("--finetune_path", type=str, default="./finetune",
                   help="Path or url of the model cache")
    p.add_argument("--finetuned_from", type=str, choices=list(FED_DATASETS.keys()),
                   help="Name of the dataset you pretrained on.")
    p.add_argument("--num_results_train", type=int, default=2)
    p.add_argument("--num_results_val", type=int, default=2)
    p.add_argument("--dataset_name", type=str, default="", choices=list(FED_DATASETS.keys()),
                   help="Name of the dataset.")
    p.add_argument("--dataset_dir", type=str, default="./dataset",
                   help="Path or url of the dataset cache")
    p.add_argument("--batchnorm", action="store_true", dest="do_batchnorm")
    p.add_argument("--nan_threshold", type=float, default=999)

    # compression args
    p.add_argument("--k", type=int, default=50000)
    p.add_argument("--num_cols", type=int, default=500000)
    p.add_argument("--num_rows", type=int, default=5)
    p.add_argument("--num_blocks", type=int, default=20)
    p.add_argument("--topk_down", action="store_true", dest="do_topk_down")

    # optimization args
    p.add_argument("--local_momentum", type=float, default=0.9)
    p.add_argument("--virtual_momentum", type=float, default=0)
    p.add_argument("--weight_decay", type=float, default=5e-4)
    p.add_argument("--num_epochs", type=float, default=24, help="Number of training epochs")
    p.add_argument("--num_fedavg_epochs", type=int, default=1)
    p.add_argument("--fedavg_batch_size", type=int, default=-1)
    p.add_argument("--fedavg_lr_decay", type=float, default=1)
    p.add_argument("--fedavg_batched", choices=["auto", "on", "off"], default="auto",
                   help="multi-step FedAvg local SGD of a rank's clients at once (torch.func.vmap "
                        "over per-client weight copies, parallel/fed_model.py) instead of one "
                        "client after another; auto: when the clients have equal sizes and no "
                        "worker-side DP is on")
    p.add_argument("--fedavg_engine", choices=["auto", "native", "vmap"], default="auto",
                   help="batched FedAvg program: native = the explicit G-client ResNet-18 of "
                        "parallel/fedavg_native.py (grouped MFMA convs, channel-stacked batch "
                        "norm, per-row SGD kernels); vmap = torch.func.vmap over the model's "
                        "stock ops; auto: native where supported (GPU, ResNet18 + BatchNorm)")
    p.add_argument("--error_type", choices=ERROR_TYPES, default="none")
    p.add_argument("--lr_scale", type=float, default=default_lr)
    p.add_argument("--pivot_epoch", type=float, default=5)

    # parallelization args
    p.add_argument("--port", type=int, default=5315)
    p.add_argument("--num_clients", type=int)
    p.add_argument("--num_workers", type=int, default=1)
    p.add_argument("--device", type=str, choices=["cpu", "cuda"], default=None,
                   help="Device (cuda or cpu)")
    p.add_argument("--num_devices", type=int, default=1, help="Number of gpus")
    p.add_argument("--share_ps_gpu", action="store_true")
    p.add_argument("--iid", action="store_true", dest="do_iid")
    p.add_argument("--train_dataloader_workers", type=int, default=0)
    p.add_argument("--val_dataloader_workers", type=int, default=0)

    # GPT2 args
    p.add_argument("--model_checkpoint", type=str, default="gpt2",
                   help="Path, url or short name of the model")
    p.add_argument("--num_candidates", type=int, default=2, help="Number of candidates for training")
    p.add_argument("--max_history", type=int, default=2,
                   help="Number of previous exchanges to keep in history")
    p.add_argument("--local_batch_size", type=int, default=8,
                   help="Batch size for training (-1 uses all data the client has)")
    p.add_argument("--valid_batch_size", type=int, default=8, help="Batch size for validation")
    p.add_argument("--microbatch_size", type=int, default=-1,
                   help="Size of each batch shard to be processed to save memory (-1 uses all data)")
    p.add_argument("--lm_coef", type=float, default=1.0, help="LM loss coefficient")
    p.add_argument("--mc_coef", type=float, default=1.0, help="Multiple-choice loss coefficient")
    p.add_argument("--max_grad_norm", type=float, help="Clipping gradient norm, is per-worker")
    p.add_argument("--personality_permutations", type=int, default=1,
                   help="Number of permutations of personality sentences")
    p.add_argument("--eval_before_start", action="store_true",
                   help="If true start with a first evaluation before training")

    # Differential Privacy args
    p.add_argument("--dp", action="store_true", dest="do_dp",
                   help="Whether to do differentially private training)")
    p.add_argument("--dp_mode", choices=["worker", "server"], default="worker")
    p.add_argument("--l2_norm_clip", type=float, default=1.0, help="What value to clip the l2 norm to")
    p.add_argument("--noise_multiplier", type=float, default=0.0,
                   help="Sigma, i.e. standard dev of noise")

    # ---------------------------------------------------------------- NEW
    g = p.add_argument_group("commefficient_amd (MI355X) extensions")
    g.add_argument("--synthetic", action="store_true",
                   help="use synthetic data shaped like --dataset_name (no files needed)")
    g.add_argument("--synthetic_size", type=int, default=None,
                   help="number of synthetic training examples (default: real dataset size)")
    g.add_argument("--synthetic_difficulty", choices=["easy", "hard"], default="easy",
                   help="synthetic images: 'easy' = class pattern + small noise; 'hard' = "
                        "weaker class pattern + a distractor class pattern + strong noise "
                        "(not separable by eye; convergence runs)")
    g.add_argument("--dtype", choices=["bf16", "fp32"], default="bf16",
                   help="compute dtype of forward/backward (master weights stay fp32)")
    g.add_argument("--merge_clients", choices=["auto", "on", "off"], default="auto",
                   help="merge the clients of a rank into one forward/backward when the "
                        "mode is linear per client (exact; see parallel/fed_model.py)")
    g.add_argument("--grouped_grads", choices=["auto", "on", "off"], default="auto",
                   help="for per-client (nonlinear) modes at shared weights: one merged "
                        "forward/backward that writes every client's weight gradient "
                        "separately (ops/grouped.py) instead of one pass per client")
    g.add_argument("--grouped_gb", type=float, default=16.0,
                   help="HBM budget (GB) of the [clients, d] grouped gradient buffer; more "
                        "clients than fit run in several grouped passes")
    g.add_argument("--sparse_allgather", choices=["auto", "on", "off"], default="auto",
                   help="local_topk: all-gather every client's k (index, value) pairs "
                        "instead of all-reducing the dense d-vector (auto: when that moves "
                        "fewer bytes over xGMI)")
    g.add_argument("--weight_cast", choices=["auto", "once", "autocast"], default="auto",
                   help="bf16 compute weights: 'once' = one cast of the flat fp32 master "
                        "weights into a bf16 model replica per forward and one gradient "
                        "gather back (parallel/flat.py); 'autocast' = torch.autocast per-op "
                        "casts; auto = once for GPT-2 on a GPU, else autocast")
    g.add_argument("--overlap_allreduce", choices=["auto", "on", "off"], default="auto",
                   help="dense merged modes on >1 rank: all-reduce gradient buckets as the "
                        "backward completes them (parallel/overlap.py)")
    g.add_argument("--allreduce_bucket_mb", type=float, default=32.0,
                   help="bucket size of the overlapped gradient all-reduce")
    g.add_argument("--client_dropout", type=float, default=0.0,
                   help="simulated client failures: each client selected for a round drops out "
                        "with this probability (same draw on every rank) and neither downloads "
                        "nor uploads; the round averages over the surviving examples")
    g.add_argument("--skip_nonfinite", type=int, default=0,
                   help="1: a round whose aggregated upload holds a NaN/Inf is dropped at the "
                        "server (weights and server state untouched) instead of poisoning them")
    g.add_argument("--inject_nonfinite_round", type=int, default=-1,
                   help="fault injection: corrupt the aggregated upload of this round with a NaN")
    g.add_argument("--sketch_seed", type=int, default=42, help="Count-Sketch hash seed")
    g.add_argument("--encode", choices=["region", "planned", "binned", "direct"], default="region",
                   help="Count-Sketch hash family + GPU kernels: region (region-permutation "
                        "family, ops/sketch_region.py: LDS-local encode and query, no plan) or "
                        "the csvec-layout multiply-shift family (numBlocks) with planned "
                        "(precomputed permutation, atomic free), binned (LDS atomics) or "
                        "direct (global atomics) kernels")
    g.add_argument("--client_state_device", choices=["auto", "gpu", "cpu"], default="auto",
                   help="where per-client momentum/error/weights live")
    g.add_argument("--client_prefetch", type=int, default=4,
                   help="host-tier client state: rows of the next N clients of the round copied "
                        "to the GPU ahead on a side stream (parallel/state.py)")
    g.add_argument("--resume", type=str, default=None,
                   help="resume from a *.fedstate.pt sidecar written with --checkpoint")
    g.add_argument("--checkpoint_every", type=int, default=0,
                   help="also write the checkpoint + resume sidecar every N rounds")
    g.add_argument("--log_every", type=int, default=0,
                   help="print a progress line every N rounds (0: per epoch only)")
    g.add_argument("--max_rounds", type=int, default=0,
                   help="stop after this many training rounds (0: no limit)")
    g.add_argument("--profile_dir", type=str, default=None,
                   help="write per-phase HIP-event timings + torch.profiler traces here")
    g.add_argument("--profile_rounds", type=int, default=5,
                   help="rounds captured by torch.profiler (after 1 wait + 1 warmup round)")
    g.add_argument("--channels_last", type=int, default=1, help="NHWC activations for convs")
    g.add_argument("--miopen_find", type=int, default=0,
                   help="1: MIOpen exhaustive kernel search per conv shape (cudnn.benchmark; "
                        "algorithm choice may differ run to run).  Default 0 = the reference's "
                        "benchmark=False (cv_train.py:325-326); only convs outside the native "
                        "kernels reach MIOpen")
    g.add_argument("--miopen_deterministic", type=int, default=0,
                   help="1: cudnn.deterministic=True as the reference sets it "
                        "(cv_train.py:325).  Off by default: MIOpen serves it with its naive "
                        "direct-convolution kernels (measured 60x slower on the ImageNet round); "
                        "the native conv paths are deterministic either way")
    g.add_argument("--conv", choices=["native", "miopen"], default="native",
                   help="3x3 conv(+relu+pool) units: native MFMA kernels (csrc/conv.hip) "
                        "where shapes fit, or MIOpen everywhere")
    g.add_argument("--transformer", choices=["native", "hf"], default="native",
                   help="GPT-2 blocks: native junction kernels (csrc/transformer.hip: fused "
                        "residual+dropout+LayerNorm, bias+GELU, bias gradients) around "
                        "hipBLASLt GEMMs and SDPA, or the HF module forward")
    g.add_argument("--shard_unsketch", choices=["on", "query", "off"], default="on",
                   help="sketch mode on >1 rank.  on: the sharded server -- region family: the "
                        "tables are reduce-scattered by region group and each rank keeps V/E, "
                        "runs the momentum, median query and top-k for its 1/N of the groups "
                        "(csvec layout: as 'query'); query: all-reduce of the whole table, each "
                        "rank queries 1/N of the coordinates; in both the k-lists are "
                        "all-gathered and merged (bitwise the replicated result); off: every "
                        "rank runs the whole server step")
    g.add_argument("--round_tape", choices=["auto", "off"], default="auto",
                   help="record a merged round of fixed geometry once and replay its native "
                        "kernel launches from C++ afterwards (parallel/tape.py); off: every "
                        "round is enqueued from Python")
    g.add_argument("--wgrad_stream", choices=["on", "off"], default="on",
                   help="native GPT-2 path: weight-gradient GEMMs on a side HIP stream, "
                        "overlapping the rest of the backward")
    g.add_argument("--unpad", choices=["on", "off"], default="on",
                   help="native GPT-2 path: token-wise ops (embeddings, GEMMs, LayerNorm/"
                        "GELU junctions) on the real tokens only, attention on the padded "
                        "layout (exact: right padding never reaches a real token)")
    g.add_argument("--synthetic_text", choices=["uniform", "bigram"], default="uniform",
                   help="--synthetic PersonaChat tokens: uniform i.i.d. (throughput benches) or a "
                        "learnable bigram language over 1,024 tokens (learning tests)")
    g.add_argument("--gpt2_size", choices=["small", "mini", "tiny"], default="small",
                   help="GPT-2 architecture: 'small' = 124M GPT-2 (reference); 'mini' (2 x 256, "
                        "4 heads: native kernels) and 'tiny' (2 x 64) for tests")
    return p


def validate_args(args) -> None:
    """Mode-validity constraints (reference asserts)."""
    def bad(msg):
        raise ValueError(msg)

    if args.mode == "fedavg":
        if args.local_batch_size != -1:
            bad("--mode fedavg requires --local_batch_size -1 (utils.py:225-228)")
        if args.local_momentum != 0:
            bad("--mode fedavg requires --local_momentum 0")
        if args.error_type != "none":
            bad("--mode fedavg requires --error_type none")
    if args.mode == "sketch":
        if args.local_momentum != 0:
            bad("--mode sketch requires --local_momentum 0: momentum lives in sketch space "
                "on the server (fed_worker.py:227-228); use --virtual_momentum")
        if args.error_type == "local":
            bad("--mode sketch requires --error_type none or virtual (fed_worker.py:221-222)")
    if args.mode == "true_topk" and args.error_type != "virtual":
        bad("--mode true_topk requires --error_type virtual (fed_aggregator.py:512)")
    if args.mode == "local_topk" and args.error_type not in ("local", "none"):
        bad("--mode local_topk requires --error_type local or none (fed_aggregator.py:545)")
    if args.mode == "uncompressed" and args.error_type == "local":
        bad("--mode uncompressed does not support --error_type local (fed_worker.py:221-222)")
    if args.error_type == "local" and args.virtual_momentum != 0 and args.mode == "sketch":
        bad("local error requires virtual_momentum 0")
    if args.num_rows > 16:
        bad("--num_rows must be <= 16")


def parse_args(default_lr: Optional[float] = None, argv: Optional[Sequence[str]] = None,
               probe_port: bool = True):
    parser = build_parser(default_lr)
    args = parser.parse_args(argv)
    finalize_args(args, probe_port=probe_port)
    return args


def finalize_args(args, probe_port: bool = True):
    if args.device is None:
        import torch
        # device_count() does not initialise the HIP runtime (is_available()
        # may), so a parent that later spawns ranks stays GPU-clean
        args.device = "cuda" if torch.cuda.device_count() > 0 else "cpu"
    # torchrun-provided rendezvous wins; otherwise probe for a free port like
    # the reference (utils.py:216-223)
    if "MASTER_PORT" in os.environ:
        args.port = int(os.environ["MASTER_PORT"])
    elif probe_port:
        rng = np.random.RandomState()
        while is_port_in_use(args.port):
            args.port += int(rng.randint(1, 1000))
    validate_args(args)
    return args
