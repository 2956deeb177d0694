from .args import (FED_DATASETS, MODES, build_parser, finalize_args, num_classes_of_dataset,
                   parse_args, validate_args)
from .logging import (Logger, PhaseTimer, ScalarWriter, TableLogger, Timer, TSVLogger,
                      make_logdir, union)
from .schedules import (Exp, PiecewiseLinear, linear_decay_lambda, steps_per_epoch,
                        triangular_lambda)
