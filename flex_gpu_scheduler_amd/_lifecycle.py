"""Orderly shutdown of native resources at interpreter exit.

Daemon Python threads may be blocked inside a native wait (a store watch)
with the GIL released, and native scheduler threads may call back into Python
(API client trampolines). If either re-acquires the GIL while CPython is
finalizing, CPython terminates that thread from inside a C++ noexcept frame
and the process aborts. At exit we therefore stop every registered component
(informers first, then watches, then schedulers) and wait until no thread is
inside a native wait.
"""
from __future__ import annotations

import atexit
import time
import weakref

EARLY, WATCH, LATE = 0, 1, 2
_groups: dict[int, dict[str, "weakref.WeakSet"]] = {EARLY: {}, WATCH: {}, LATE: {}}


def register(obj, stage: int = EARLY, method: str = "shutdown_for_exit") -> None:
    """`getattr(obj, method)()` is called at exit (stages EARLY, WATCH, LATE);
    only a weak reference is kept."""
    _groups[stage].setdefault(method, weakref.WeakSet()).add(obj)


def shutdown(wait_s: float = 3.0) -> None:
    for stage in (EARLY, WATCH, LATE):
        for method, objs in _groups[stage].items():
            for obj in list(objs):
                try:
                    getattr(obj, method)()
                except Exception:  # noqa: BLE001 - best effort at exit
                    pass
    try:
        from ._native import native
        n = native()
    except Exception:  # noqa: BLE001
        return
    deadline = time.monotonic() + wait_s
    while n.native_waiters() > 0 and time.monotonic() < deadline:
        time.sleep(0.005)


atexit.register(shutdown)
