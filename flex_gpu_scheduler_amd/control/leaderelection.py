"""Lease-based leader election (client-go tools/leaderelection semantics).

The reference controller optionally runs under leader election and exits when
the lease is lost (cmd/controller/app/server.go:94-117, lock
`kube-system/sched-plugins-controller`, Endpoints lock). We use a
coordination.k8s.io/v1 Lease with optimistic concurrency (update with the
observed resourceVersion). Expiry is judged from the local monotonic time at
which the current record was first observed — not from the holder's clock —
exactly like client-go's `observedTime`, so clock skew between replicas cannot
make two holders.
"""
from __future__ import annotations

import logging
import threading
import time
from datetime import datetime, timezone
from typing import Callable

from .client import Client, is_conflict, is_not_found

log = logging.getLogger(__name__)


def _micro_now() -> str:
    return datetime.now(timezone.utc).strftime("%Y-%m-%dT%H:%M:%S.%fZ")


class LeaderElector:
    def __init__(self, client: Client, name: str, namespace: str, identity: str, *,
                 lease_duration: float = 15.0, renew_deadline: float = 10.0, retry_period: float = 2.0,
                 on_started_leading: Callable[[], None] | None = None,
                 on_stopped_leading: Callable[[], None] | None = None,
                 on_new_leader: Callable[[str], None] | None = None):
        if not (lease_duration > renew_deadline > retry_period > 0):
            raise ValueError("need lease_duration > renew_deadline > retry_period > 0")
        self.client, self.name, self.ns, self.identity = client, name, namespace, identity
        self.lease_duration, self.renew_deadline, self.retry_period = lease_duration, renew_deadline, retry_period
        self.on_started, self.on_stopped, self.on_new_leader = on_started_leading, on_stopped_leading, on_new_leader
        self._observed: tuple | None = None   # (holder, renewTime)
        self._observed_at = 0.0
        self._leader = ""
        self._stop = threading.Event()
        self.is_leader = threading.Event()
        self.transitions_seen = 0
        self.renewed_at = 0.0  # monotonic time of the last successful acquire/renew

    @property
    def leader(self) -> str:
        return self._leader

    def _observe(self, spec: dict) -> None:
        rec = (spec.get("holderIdentity") or "", spec.get("renewTime") or "")
        if rec != self._observed:
            self._observed, self._observed_at = rec, time.monotonic()
            if rec[0] != self._leader:
                self._leader = rec[0]
                if self.on_new_leader and rec[0]:
                    self.on_new_leader(rec[0])

    def try_acquire_or_renew(self) -> bool:
        now = _micro_now()
        lease = self.client.get("leases", self.ns, self.name)
        if lease is None:
            spec = {"holderIdentity": self.identity, "leaseDurationSeconds": int(self.lease_duration),
                    "acquireTime": now, "renewTime": now, "leaseTransitions": 0}
            try:
                self.client.create("leases", {"metadata": {"name": self.name, "namespace": self.ns}, "spec": spec})
            except Exception as e:  # noqa: BLE001
                if is_conflict(e):
                    return False
                raise
            self._observe(spec)
            return True
        spec = dict(lease.get("spec") or {})
        self._observe(spec)
        holder = spec.get("holderIdentity") or ""
        duration = float(spec.get("leaseDurationSeconds") or self.lease_duration)
        if holder and holder != self.identity and time.monotonic() < self._observed_at + duration:
            return False
        if holder != self.identity:
            spec["acquireTime"] = now
            spec["leaseTransitions"] = int(spec.get("leaseTransitions") or 0) + 1
        spec.update(holderIdentity=self.identity, renewTime=now, leaseDurationSeconds=int(self.lease_duration))
        lease = dict(lease)
        lease["spec"] = spec
        try:
            self.client.update("leases", lease)
        except Exception as e:  # noqa: BLE001
            if is_conflict(e) or is_not_found(e):
                return False
            raise
        self._observe(spec)
        self.renewed_at = time.monotonic()
        return True

    def healthz(self, timeout: float = 20.0) -> tuple[bool, str]:
        """HealthzAdaptor (client-go leaderelection/healthzadaptor.go): a
        leader that has not renewed its lease within lease_duration +
        `timeout` is unhealthy (kube-scheduler installs this check,
        vendor/k8s.io/kubernetes/cmd/kube-scheduler/app/server.go:151-154).
        Followers are healthy."""
        if not self.is_leader.is_set():
            return True, "not leading"
        age = time.monotonic() - self.renewed_at
        if age > self.lease_duration + timeout:
            return False, f"failed election to renew leadership on lease {self.ns}/{self.name} ({age:.1f}s)"
        return True, "leading"

    def release(self) -> None:
        """Give the lease up on clean shutdown (ReleaseOnCancel)."""
        lease = self.client.get("leases", self.ns, self.name)
        if not lease or (lease.get("spec") or {}).get("holderIdentity") != self.identity:
            return
        lease = dict(lease)
        lease["spec"] = dict(lease["spec"], holderIdentity="", leaseDurationSeconds=1, renewTime=_micro_now())
        try:
            self.client.update("leases", lease)
        except Exception:  # noqa: BLE001
            pass

    def run(self) -> None:
        """Block: acquire, lead (callback on a thread), renew; return when the
        lease is lost or `stop()` is called."""
        while not self._stop.is_set():
            try:
                if self.try_acquire_or_renew():
                    break
            except Exception:  # noqa: BLE001
                log.exception("leader election: acquire failed")
            self._stop.wait(self.retry_period)
        if self._stop.is_set():
            return
        self.is_leader.set()
        log.info("leader election: %s became leader of %s/%s", self.identity, self.ns, self.name)
        if self.on_started:
            threading.Thread(target=self.on_started, name="leader-work", daemon=True).start()
        last_ok = time.monotonic()
        while not self._stop.is_set():
            self._stop.wait(self.retry_period)
            if self._stop.is_set():
                break
            try:
                ok = self.try_acquire_or_renew()
            except Exception:  # noqa: BLE001
                ok = False
            if ok:
                last_ok = time.monotonic()
            elif time.monotonic() - last_ok >= self.renew_deadline:
                break
        self.is_leader.clear()
        if self._stop.is_set():
            self.release()
        log.info("leader election: %s stopped leading", self.identity)
        if self.on_stopped:
            self.on_stopped()

    def stop(self) -> None:
        self._stop.set()
