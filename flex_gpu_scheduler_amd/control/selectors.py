"""Label and field selectors (k8s.io/apimachinery/pkg/labels, fields string
syntax): `a=b`, `a==b`, `a!=b`, `a in (x,y)`, `a notin (x)`, `a`, `!a`, joined
by commas. Used by the API server's list/watch filtering and by controllers
(the PodGroup controller lists pods by the `pod-group.scheduling.sigs.k8s.io`
label, pkg/controller/podgroup.go:209-210).
"""
from __future__ import annotations

import re
from dataclasses import dataclass
from typing import Callable, Mapping

_SET_RE = re.compile(r"^\s*(!?)\s*([A-Za-z0-9_./-]+)\s*(?:(notin|in)\s*\(([^)]*)\))?\s*$")


@dataclass(frozen=True)
class Requirement:
    key: str
    op: str                 # "=", "!=", "in", "notin", "exists", "!exists"
    values: tuple[str, ...] = ()

    def matches(self, labels: Mapping[str, str]) -> bool:
        has = self.key in labels
        if self.op == "exists":
            return has
        if self.op == "!exists":
            return not has
        if self.op in ("=", "in"):
            return has and labels[self.key] in self.values
        # "!=" / "notin": true when the key is absent (apimachinery semantics)
        return not has or labels[self.key] not in self.values


def _split_top(s: str) -> list[str]:
    out, depth, cur = [], 0, []
    for ch in s:
        if ch == "(":
            depth += 1
        elif ch == ")":
            depth -= 1
        if ch == "," and depth == 0:
            out.append("".join(cur))
            cur = []
        else:
            cur.append(ch)
    if cur:
        out.append("".join(cur))
    return [p.strip() for p in out if p.strip()]


def parse_selector(s: str | None) -> list[Requirement]:
    if not s:
        return []
    reqs = []
    for term in _split_top(s):
        if "!=" in term:
            k, v = term.split("!=", 1)
            reqs.append(Requirement(k.strip(), "!=", (v.strip(),)))
            continue
        if "==" in term or ("=" in term and "(" not in term):
            k, v = term.split("==", 1) if "==" in term else term.split("=", 1)
            reqs.append(Requirement(k.strip(), "=", (v.strip(),)))
            continue
        m = _SET_RE.match(term)
        if not m:
            raise ValueError(f"invalid selector term {term!r}")
        neg, key, op, vals = m.groups()
        if op:
            if neg:
                raise ValueError(f"invalid selector term {term!r}")
            reqs.append(Requirement(key, op, tuple(v.strip() for v in vals.split(",") if v.strip())))
        else:
            reqs.append(Requirement(key, "!exists" if neg else "exists"))
    return reqs


def label_matcher(s: str | None) -> Callable[[dict], bool] | None:
    reqs = parse_selector(s)
    if not reqs:
        return None

    def match(obj: dict) -> bool:
        labels = (obj.get("metadata") or {}).get("labels") or {}
        return all(r.matches(labels) for r in reqs)
    return match


def _field(obj: dict, path: str):
    cur = obj
    for part in path.split("."):
        if not isinstance(cur, dict):
            return ""
        cur = cur.get(part)
    return "" if cur is None else str(cur)


def field_matcher(s: str | None) -> Callable[[dict], bool] | None:
    """Field selectors support = / == / != on any dotted path (the API server
    restricts keys per kind; we accept any path, e.g. spec.nodeName)."""
    reqs = [r for r in parse_selector(s)]
    if not reqs:
        return None
    for r in reqs:
        if r.op not in ("=", "!="):
            raise ValueError(f"field selector supports only = and !=, got {r.op}")

    def match(obj: dict) -> bool:
        for r in reqs:
            v = _field(obj, r.key)
            if (v == r.values[0]) != (r.op == "="):
                return False
        return True
    return match


def combine(*ms: Callable[[dict], bool] | None) -> Callable[[dict], bool] | None:
    live = [m for m in ms if m is not None]
    if not live:
        return None
    if len(live) == 1:
        return live[0]
    return lambda o: all(m(o) for m in live)
