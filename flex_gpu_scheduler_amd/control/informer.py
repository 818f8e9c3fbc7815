"""Informers and a rate-limited work queue for the Python control plane.

`Informer` is the client-go SharedIndexInformer analog (list → watch from the
list's resourceVersion → local cache + add/update/delete handlers, relist on
410/stream loss) used by the controllers (pkg/controller/podgroup.go:75-82,
elasticquota.go:93-107 register handlers on informers built from the generated
factory, pkg/generated/informers/externalversions/factory.go:79-180).

`WorkQueue` follows client-go's rate-limiting workqueue: a key is queued at
most once, never handed to two workers at the same time (a key re-added while
being processed is re-queued on `done`), and `add_rate_limited` backs off per
item exponentially (5 ms · 2^n, capped at 1000 s — DefaultControllerRateLimiter)
until `forget`.
"""
from __future__ import annotations

import heapq
import logging
import threading
import time
import weakref
from typing import Callable

from .. import _lifecycle
from .client import Client
from .selectors import label_matcher

# Informers started in this process (weak): the test suite stops any that a
# test left running, so none retries against a server that is gone.
STARTED: "weakref.WeakSet[Informer]" = weakref.WeakSet()

log = logging.getLogger(__name__)


def meta_key(obj: dict) -> str:
    md = obj.get("metadata") or {}
    ns = md.get("namespace") or ""
    return f"{ns}/{md.get('name', '')}" if ns else md.get("name", "")


def split_key(key: str) -> tuple[str, str]:
    ns, _, name = key.rpartition("/")
    return ns, name


class Informer:
    def __init__(self, client: Client, kind: str, ns: str = "", label_selector: str | None = None,
                 resync_period: float = 0.0):
        self.client, self.kind, self.ns = client, kind, ns
        self.label_selector = label_selector
        self._match = label_matcher(label_selector)
        self.resync_period = resync_period
        self._cache: dict[str, dict] = {}
        self._lock = threading.RLock()
        self._handlers: list[tuple[Callable | None, Callable | None, Callable | None]] = []
        self._synced = threading.Event()
        self._stop = threading.Event()
        self._thread: threading.Thread | None = None
        self.relists = 0
        _lifecycle.register(self)

    def shutdown_for_exit(self) -> None:
        self._stop.set()

    # -------------------------------------------------------------- handlers
    def add_event_handler(self, on_add: Callable[[dict], None] | None = None,
                          on_update: Callable[[dict, dict], None] | None = None,
                          on_delete: Callable[[dict], None] | None = None) -> None:
        self._handlers.append((on_add, on_update, on_delete))
        if self._synced.is_set() and on_add:
            for o in self.list():
                on_add(o)

    def _fire(self, idx: int, *args) -> None:
        for h in self._handlers:
            fn = h[idx]
            if fn is None:
                continue
            try:
                fn(*args)
            except Exception:  # noqa: BLE001 - a handler must not kill the informer
                log.exception("informer %s handler failed", self.kind)

    # ---------------------------------------------------------------- lister
    def get(self, ns: str, name: str) -> dict | None:
        with self._lock:
            return self._cache.get(f"{ns}/{name}" if ns else name)

    def get_by_key(self, key: str) -> dict | None:
        with self._lock:
            return self._cache.get(key)

    def list(self, ns: str | None = None, selector: Callable[[dict], bool] | None = None) -> list[dict]:
        with self._lock:
            vals = list(self._cache.values())
        if ns:
            vals = [o for o in vals if (o.get("metadata") or {}).get("namespace") == ns]
        if selector:
            vals = [o for o in vals if selector(o)]
        return vals

    def has_synced(self) -> bool:
        return self._synced.is_set()

    def wait_for_sync(self, timeout: float = 30.0) -> bool:
        return self._synced.wait(timeout)

    # ------------------------------------------------------------------ run
    def start(self) -> "Informer":
        self._thread = threading.Thread(target=self._run, name=f"informer-{self.kind}", daemon=True)
        self._thread.start()
        STARTED.add(self)
        return self

    def running(self) -> bool:
        return self._thread is not None and self._thread.is_alive() and not self._stop.is_set()

    def stop(self) -> None:
        self._stop.set()
        if self._thread:
            self._thread.join(timeout=5)

    def _replace(self, items: list[dict]) -> None:
        fresh = {meta_key(o): o for o in items if self._match is None or self._match(o)}
        with self._lock:
            old = self._cache
            self._cache = fresh
        for k, o in fresh.items():
            prev = old.get(k)
            if prev is None:
                self._fire(0, o)
            elif prev.get("metadata", {}).get("resourceVersion") != o.get("metadata", {}).get("resourceVersion"):
                self._fire(1, prev, o)
        for k, o in old.items():
            if k not in fresh:
                self._fire(2, o)

    def _apply(self, etype: str, obj: dict) -> None:
        key = meta_key(obj)
        matches = self._match is None or self._match(obj)
        with self._lock:
            prev = self._cache.get(key)
            if etype == "DELETED" or not matches:
                if prev is None:
                    return
                del self._cache[key]
            else:
                self._cache[key] = obj
        if etype == "DELETED" or not matches:
            self._fire(2, prev if etype != "DELETED" else obj)
        elif prev is None:
            self._fire(0, obj)
        else:
            self._fire(1, prev, obj)

    def _run(self) -> None:
        backoff = 0.05
        while not self._stop.is_set():
            w = None
            try:
                items, rv = self.client.list(self.kind, self.ns, self.label_selector)
                w = self.client.watch([self.kind], self.ns, rv)
                if rv == 0:
                    # Nothing had happened when we listed; relist after the watch
                    # is open and drop replayed events the list already covers.
                    items, rv = self.client.list(self.kind, self.ns, self.label_selector)
                self._replace(items)
                self.relists += 1
                self._synced.set()
                backoff = 0.05
                last_resync = time.monotonic()
                while not self._stop.is_set():
                    evs = w.next(200, 4096)
                    broken = False
                    for etype, _kind, obj, erv in evs:
                        if etype == "ERROR":
                            broken = True
                            break
                        if erv and erv <= rv:
                            continue
                        self._apply(etype, obj)
                    if broken:
                        break
                    if self.resync_period and time.monotonic() - last_resync >= self.resync_period:
                        last_resync = time.monotonic()
                        for o in self.list():
                            self._fire(1, o, o)
            except Exception as e:  # noqa: BLE001
                if getattr(e, "code", 0) == 404 and not self._synced.is_set():
                    # The API does not serve this kind (a CRD that is not
                    # installed): sync as empty, retry the list now and then.
                    log.warning("informer %s: kind not served (%s); treating it as empty", self.kind, e)
                    self._synced.set()
                    self._stop.wait(30.0)
                    continue
                if self._stop.is_set():
                    break
                if isinstance(e, OSError):
                    # The API server is unreachable (restarting, or gone at
                    # shutdown): one line per attempt, no traceback.
                    log.warning("informer %s list/watch failed (%s); retrying in %.2fs", self.kind, e, backoff)
                else:
                    log.exception("informer %s list/watch failed; retrying", self.kind)
                self._stop.wait(backoff)
                backoff = min(backoff * 2, 5.0)
            finally:
                if w is not None:
                    w.stop()


class InformerFactory:
    """One informer per (kind, namespace, selector), started together."""

    def __init__(self, client: Client):
        self.client = client
        self._informers: dict[tuple, Informer] = {}

    def informer(self, kind: str, ns: str = "", label_selector: str | None = None) -> Informer:
        key = (kind, ns, label_selector)
        if key not in self._informers:
            self._informers[key] = Informer(self.client, kind, ns, label_selector)
        return self._informers[key]

    def start(self) -> None:
        for inf in self._informers.values():
            if inf._thread is None:
                inf.start()

    def wait_for_sync(self, timeout: float = 30.0) -> bool:
        deadline = time.monotonic() + timeout
        return all(inf.wait_for_sync(max(0.0, deadline - time.monotonic())) for inf in self._informers.values())

    def stop(self) -> None:
        for inf in self._informers.values():
            inf.stop()


class WorkQueue:
    def __init__(self, name: str = "", base_delay: float = 0.005, max_delay: float = 1000.0):
        self.name = name
        self.base_delay, self.max_delay = base_delay, max_delay
        self._cv = threading.Condition()
        self._queue: list[str] = []
        self._dirty: set[str] = set()
        self._processing: set[str] = set()
        self._failures: dict[str, int] = {}
        self._delayed: list[tuple[float, int, str]] = []
        self._seq = 0
        self._shutdown = False
        self.adds = 0

    def __len__(self) -> int:
        with self._cv:
            return len(self._queue)

    def add(self, key: str) -> None:
        with self._cv:
            if self._shutdown or key in self._dirty:
                return
            self.adds += 1
            self._dirty.add(key)
            if key not in self._processing:
                self._queue.append(key)
                self._cv.notify()

    def add_after(self, key: str, delay: float) -> None:
        if delay <= 0:
            return self.add(key)
        with self._cv:
            if self._shutdown:
                return
            self._seq += 1
            heapq.heappush(self._delayed, (time.monotonic() + delay, self._seq, key))
            self._cv.notify()

    def when(self, key: str) -> float:
        with self._cv:
            n = self._failures.get(key, 0)
            self._failures[key] = n + 1
        return min(self.base_delay * (2 ** n), self.max_delay)

    def add_rate_limited(self, key: str) -> None:
        self.add_after(key, self.when(key))

    def forget(self, key: str) -> None:
        with self._cv:
            self._failures.pop(key, None)

    def num_requeues(self, key: str) -> int:
        with self._cv:
            return self._failures.get(key, 0)

    def _promote_locked(self) -> float | None:
        now = time.monotonic()
        while self._delayed and self._delayed[0][0] <= now:
            _, _, key = heapq.heappop(self._delayed)
            if key not in self._dirty:
                self._dirty.add(key)
                self.adds += 1
                if key not in self._processing:
                    self._queue.append(key)
        return self._delayed[0][0] - now if self._delayed else None

    def get(self, timeout: float | None = None) -> str | None:
        """Next key, or None on shutdown/timeout."""
        deadline = None if timeout is None else time.monotonic() + timeout
        with self._cv:
            while True:
                wait = self._promote_locked()
                if self._queue:
                    key = self._queue.pop(0)
                    self._processing.add(key)
                    self._dirty.discard(key)
                    return key
                if self._shutdown:
                    return None
                if deadline is not None:
                    left = deadline - time.monotonic()
                    if left <= 0:
                        return None
                    wait = left if wait is None else min(wait, left)
                self._cv.wait(wait)

    def done(self, key: str) -> None:
        with self._cv:
            self._processing.discard(key)
            if key in self._dirty:
                self._queue.append(key)
                self._cv.notify()

    def shutdown(self) -> None:
        with self._cv:
            self._shutdown = True
            self._cv.notify_all()

    @property
    def shutting_down(self) -> bool:
        return self._shutdown
