"""Reference-compatible CV entry point (cv_train.py): same flags as fed_train.py."""
import sys

import fed_train

if __name__ == "__main__":
    fed_train.main(sys.argv[1:])
