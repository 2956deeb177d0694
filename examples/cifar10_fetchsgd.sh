#!/bin/bash
# The FetchSGD CIFAR-10 setup of BASELINE.json on N MI355X: ResNet-9, 10,000
# non-iid clients of 5 images, 100 clients per round per GPU, Count Sketch
# 5 x 500,000, k = 50,000, virtual momentum 0.9 + virtual error feedback.
set -e
cd "$(dirname "$0")/.."
NGPU=${NGPU:-1}
python -m torch.distributed.run --nnodes=1 --nproc-per-node "$NGPU" --master-addr 127.0.0.1 \
  fed_train.py --dataset_name CIFAR10 ${SYNTHETIC:+--synthetic} --dataset_dir ${DATASET_DIR:-./dataset} \
    --mode sketch --error_type virtual --local_momentum 0 --virtual_momentum 0.9 \
    --k 50000 --num_rows 5 --num_cols 500000 --num_blocks 20 \
    --num_clients 10000 --num_workers $((100 * NGPU)) --local_batch_size -1 \
    --num_epochs 24 --lr_scale 0.4 --pivot_epoch 5 "$@"
