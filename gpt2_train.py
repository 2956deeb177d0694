"""Reference-compatible GPT-2 entry point (gpt2_train.py): PersonaChat double-heads
federated training, default --lr_scale 4e-2.  Same flags as fed_train.py."""
import sys

import fed_train

if __name__ == "__main__":
    argv = sys.argv[1:]
    if "--dataset_name" not in argv:
        argv = ["--dataset_name", "PERSONA"] + argv
    if "--model" not in argv:
        argv = ["--model", "GPT2DoubleHeads"] + argv
    fed_train.main(argv, default_lr=4e-2)
