"""Federated training entry point (the name referenced by the reference's
imagenet.sh:1 and BASELINE.json); see commefficient_amd/cli.py."""
import sys

from commefficient_amd.cli import main

if __name__ == "__main__":
    main(sys.argv[1:])
