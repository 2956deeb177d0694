"""Round-level tracing: torch.profiler with ROCm (HIP)
activity over a window of federated rounds.

The reference has no structured tracing (dead cProfile / line_profiler hooks,
/root/reference/CommEfficient/fed_aggregator.py:32-52, cv_train.py:292-305).
Here ``--profile_dir DIR`` turns on, per rank:

* ``DIR/rank{R}/*.pt.trace.json``  -- Chrome/Perfetto traces (CPU ops + HIP
  kernels + memcpys) of ``--profile_rounds`` rounds after 1 wait + 1 warmup round;
* ``DIR/rank{R}/kernels.txt``      -- the key_averages table sorted by device time;
* ``DIR/rank{R}/phases.json``      -- HIP-event per-phase timings (fwd/bwd,
  encode, all-reduce, server) from :class:`~commefficient_amd.utils.logging.PhaseTimer`.

Kernel-level counters come from ``rocprofv3`` instead (scripts/pmc_*.sh).
"""
from __future__ import annotations

import json
import os
from typing import Optional

import torch


class RoundProfiler:
    def __init__(self, profile_dir: Optional[str], rank: int = 0, rounds: int = 5,
                 wait: int = 1, warmup: int = 1):
        self.dir = os.path.join(profile_dir, f"rank{rank}") if profile_dir else None
        self.prof = None
        self.total = wait + warmup + rounds
        self.n = 0
        if self.dir is None:
            return
        os.makedirs(self.dir, exist_ok=True)
        acts = [torch.profiler.ProfilerActivity.CPU]
        if torch.cuda.is_available():
            acts.append(torch.profiler.ProfilerActivity.CUDA)  # HIP on ROCm builds
        self.prof = torch.profiler.profile(
            activities=acts,
            schedule=torch.profiler.schedule(wait=wait, warmup=warmup, active=rounds, repeat=1),
            on_trace_ready=torch.profiler.tensorboard_trace_handler(self.dir),
            record_shapes=False, with_stack=False)
        self.prof.__enter__()

    @property
    def enabled(self) -> bool:
        return self.prof is not None

    def step(self):
        if self.prof is None:
            return
        self.prof.step()
        self.n += 1
        if self.n >= self.total:
            self.close()

    def close(self, phase_timer=None):
        if self.prof is not None:
            prof, self.prof = self.prof, None
            prof.__exit__(None, None, None)
            if self.n < self.total:
                table = (f"profiler window not reached: {self.n} of {self.total} rounds ran\n")
            else:
                try:
                    table = prof.key_averages().table(sort_by="self_device_time_total",
                                                      row_limit=60)
                except Exception:  # older/newer profiler column names
                    table = prof.key_averages().table(row_limit=60)
            with open(os.path.join(self.dir, "kernels.txt"), "w") as f:
                f.write(table)
        if phase_timer is not None and self.dir is not None and phase_timer.enabled:
            with open(os.path.join(self.dir, "phases.json"), "w") as f:
                json.dump(phase_timer.summary(), f, indent=1)
