"""Python entry points over the native core: the object store and the
scheduler (``scheduler.New`` + ``Run`` of SURVEY.md §3.1)."""
from __future__ import annotations

import json
from pathlib import Path
from typing import Any

from . import _lifecycle
from ._native import native
from .config import SchedulerConfiguration, load_config


def Store():
    """A fresh in-process API object store (LIST/WATCH, binding, merge-patch)."""
    return native().Store()


def FakeClock(start_us: int = 1_000_000_000):
    return native().FakeClock(start_us)


def new_scheduler(store, config: SchedulerConfiguration | dict | str | Path | None = None, *, clock=None,
                  client=None, start: bool = False, **options: Any):
    """Build a native Scheduler for `store` from a KubeSchedulerConfiguration.

    ``options`` override scheduler options (parallelism, bindWorkers,
    statusUpdates, trace, seed, podInitialBackoffSeconds, ...).
    """
    cfg = config if isinstance(config, SchedulerConfiguration) else load_config(config)
    s = native().Scheduler(store, json.dumps(cfg.to_native(**options)), clock, client)
    _lifecycle.register(s, _lifecycle.LATE, "stop")
    if start:
        s.start()
    return s
