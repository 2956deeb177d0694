#!/bin/bash
# ImageNet FixupResNet50, uncompressed, 7 clients per round (the reference's
# imagenet.sh, /root/reference/CommEfficient/imagenet.sh:1-21), one process
# per MI355X.  The reference's undefined --mixup/--mixup_alpha/--supervised
# flags are dropped; its 7 workers + 1 PS become 8 SPMD ranks (every rank
# computes its share of the round's clients and applies the same update).
# DATASET_DIR: torchvision ImageNet layout; SYNTHETIC=1 uses ImageNet-shaped
# synthetic data instead.
set -e
cd "$(dirname "$0")/.."
NGPU=${NGPU:-8}
DATA=${DATASET_DIR:-./dataset/imagenet}
EXTRA=()
[ "${SYNTHETIC:-0}" = "1" ] && EXTRA+=(--synthetic)
python -m torch.distributed.run --nnodes=1 --nproc-per-node "$NGPU" --master-addr 127.0.0.1 \
  fed_train.py \
    --dataset_dir "$DATA" \
    --dataset_name ImageNet \
    --model FixupResNet50 \
    --local_batch_size 64 \
    --local_momentum 0.0 \
    --virtual_momentum 0.9 \
    --weight_decay 1e-4 \
    --error_type virtual \
    --mode uncompressed \
    --iid \
    --num_clients 7 \
    --num_workers 7 \
    --k 1000000 \
    --num_rows 1 \
    --num_cols 10000000 \
    "${EXTRA[@]}" "$@"
