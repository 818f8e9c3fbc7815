"""A small renderer for the subset of Helm/Go templates our charts use.

Helm is not available in the build image, so charts under deploy/charts are
rendered and validated in tests with this renderer (the manifests it
produces are what `helm template` would produce for the same subset):

  {{ .Values.a.b }} {{ .Release.Name }} {{ .Release.Namespace }} {{ .Chart.Name }}
  {{ $ }} (root) · pipelines: quote, default, toYaml, toJson, indent, nindent,
  trunc, trimSuffix, upper, lower, printf "%s-%s" a b, include "tpl" .
  {{- if X }} / {{- else if Y }} / {{- else }} / {{- end }}, {{- with X }},
  {{- range X }} (dot = item), {{- define "name" }} in _helpers.tpl,
  {{/* comments */}} and `{{-` / `-}}` whitespace trimming.
"""
from __future__ import annotations

import json
import os
import re
import shlex
from typing import Any

import yaml

_TOKEN = re.compile(r"\{\{(-?)(.*?)(-?)\}\}", re.S)


class TemplateError(Exception):
    pass


def _lex(src: str) -> list[tuple[str, str]]:
    out: list[tuple[str, str]] = []
    pos = 0
    for m in _TOKEN.finditer(src):
        text = src[pos:m.start()]
        if m.group(1):
            text = text.rstrip()
        out.append(("text", text))
        body = m.group(2).strip()
        out.append(("action", body))
        pos = m.end()
        if m.group(3):
            rest = src[pos:]
            pos += len(rest) - len(rest.lstrip())
    out.append(("text", src[pos:]))
    return [t for t in out if not (t[0] == "action" and t[1].startswith("/*"))]


def _parse(tokens: list[tuple[str, str]], i: int = 0, stop=("end",)) -> tuple[list, int, str]:
    nodes: list = []
    while i < len(tokens):
        kind, val = tokens[i]
        if kind == "text":
            if val:
                nodes.append(("text", val))
            i += 1
            continue
        word = val.split(None, 1)[0] if val else ""
        if word in stop or (word == "else" and "else" in stop):
            return nodes, i, val
        if word in ("if", "with", "range"):
            cond = val[len(word):].strip()
            body, i, term = _parse(tokens, i + 1, ("end", "else"))
            branches = [(cond, body)]
            while term.startswith("else"):
                rest = term[4:].strip()
                if rest.startswith("if "):
                    body, i, term = _parse(tokens, i + 1, ("end", "else"))
                    branches.append((rest[3:].strip(), body))
                else:
                    body, i, term = _parse(tokens, i + 1, ("end",))
                    branches.append((None, body))
            nodes.append((word, branches))
            i += 1
            continue
        if word == "define":
            name = shlex.split(val[6:].strip())[0]
            body, i, _ = _parse(tokens, i + 1, ("end",))
            nodes.append(("define", name, body))
            i += 1
            continue
        nodes.append(("expr", val))
        i += 1
    if stop != ("end",) or True:
        return nodes, i, ""


def _truthy(v: Any) -> bool:
    return bool(v) and v != 0


class Renderer:
    def __init__(self, chart_dir: str, values: dict | None = None, release: str = "release",
                 namespace: str = "default"):
        self.dir = chart_dir
        with open(os.path.join(chart_dir, "Chart.yaml")) as f:
            self.chart = yaml.safe_load(f)
        vals_path = os.path.join(chart_dir, "values.yaml")
        base = {}
        if os.path.exists(vals_path):
            with open(vals_path) as f:
                base = yaml.safe_load(f) or {}
        self.values = _deep_merge(base, values or {})
        self.root = {"Values": self.values, "Release": {"Name": release, "Namespace": namespace, "Service": "Helm"},
                     "Chart": {"Name": self.chart.get("name"), "Version": self.chart.get("version"),
                               "AppVersion": self.chart.get("appVersion")}}
        self.defines: dict[str, list] = {}
        tdir = os.path.join(chart_dir, "templates")
        for fn in sorted(os.listdir(tdir)):
            if fn.endswith(".tpl"):
                with open(os.path.join(tdir, fn)) as f:
                    self._collect(_parse(_lex(f.read()))[0])

    def _collect(self, nodes: list) -> None:
        for n in nodes:
            if n[0] == "define":
                self.defines[n[1]] = n[2]

    # ------------------------------------------------------------- evaluation
    def _lookup(self, path: str, dot: Any) -> Any:
        if path == ".":
            return dot
        if path == "$":
            return self.root
        base = dot
        if path.startswith("$."):
            base, path = self.root, path[1:]
        cur = base
        for part in path.lstrip(".").split("."):
            if isinstance(cur, dict):
                cur = cur.get(part)
            else:
                return None
        return cur

    def _atom(self, tok: str, dot: Any) -> Any:
        if tok.startswith('"') and tok.endswith('"'):
            return json.loads(tok)
        if re.fullmatch(r"-?\d+", tok):
            return int(tok)
        if tok in ("true", "false"):
            return tok == "true"
        if tok.startswith(".") or tok.startswith("$"):
            return self._lookup(tok, dot)
        raise TemplateError(f"cannot evaluate {tok!r}")

    def _call(self, fn: str, args: list, dot: Any, piped: Any = None, has_pipe: bool = False) -> Any:
        vals = [self._atom(a, dot) for a in args] + ([piped] if has_pipe else [])
        if fn == "include":
            name, ctx = vals[0], vals[1]
            return self._render(self.defines[name], ctx)
        if fn == "quote":
            return json.dumps("" if vals[0] is None else str(vals[0]))
        if fn == "default":
            return vals[1] if _truthy(vals[1]) else vals[0]
        if fn == "toYaml":
            v = vals[0]
            return "" if v in (None, {}, []) else yaml.safe_dump(v, default_flow_style=False, sort_keys=False).rstrip()
        if fn == "toJson":
            return json.dumps(vals[0])
        if fn in ("indent", "nindent"):
            pad = " " * vals[0]
            s = "\n".join(pad + line if line else line for line in str(vals[1]).split("\n"))
            return ("\n" + s) if fn == "nindent" else s
        if fn == "trunc":
            return str(vals[1])[:vals[0]]
        if fn == "trimSuffix":
            s = str(vals[1])
            return s[:-len(vals[0])] if vals[0] and s.endswith(vals[0]) else s
        if fn == "upper":
            return str(vals[0]).upper()
        if fn == "lower":
            return str(vals[0]).lower()
        if fn == "printf":
            return vals[0] % tuple(vals[1:])
        if fn == "not":
            return not _truthy(vals[0])
        if fn == "eq":
            return vals[0] == vals[1]
        if fn == "and":
            return all(_truthy(v) for v in vals)
        if fn == "or":
            return next((v for v in vals if _truthy(v)), vals[-1])
        raise TemplateError(f"unknown function {fn!r}")

    def _eval(self, expr: str, dot: Any) -> Any:
        stages = [s.strip() for s in _split_pipes(expr)]
        val, has = None, False
        for st in stages:
            toks = shlex.split(st, posix=False)
            head = toks[0]
            if head.startswith((".", "$", '"')) or re.fullmatch(r"-?\d+", head) or head in ("true", "false"):
                if len(toks) != 1:
                    raise TemplateError(f"bad expression {st!r}")
                val, has = self._atom(head, dot), True
            else:
                val, has = self._call(head, toks[1:], dot, val, has), True
        return val

    def _render(self, nodes: list, dot: Any) -> str:
        out = []
        for n in nodes:
            kind = n[0]
            if kind == "text":
                out.append(n[1])
            elif kind == "expr":
                v = self._eval(n[1], dot)
                out.append("" if v is None else (str(v).lower() if isinstance(v, bool) else str(v)))
            elif kind == "define":
                continue
            elif kind in ("if", "with"):
                for cond, body in n[1]:
                    if cond is None:
                        out.append(self._render(body, dot))
                        break
                    v = self._eval(cond, dot)
                    if _truthy(v):
                        out.append(self._render(body, v if kind == "with" else dot))
                        break
            elif kind == "range":
                cond, body = n[1][0]
                seq = self._eval(cond, dot) or []
                items = seq.values() if isinstance(seq, dict) else seq
                for item in items:
                    out.append(self._render(body, item))
        return "".join(out)

    def render(self) -> dict[str, str]:
        tdir = os.path.join(self.dir, "templates")
        out = {}
        for fn in sorted(os.listdir(tdir)):
            if not fn.endswith((".yaml", ".yml")):
                continue
            with open(os.path.join(tdir, fn)) as f:
                out[fn] = self._render(_parse(_lex(f.read()))[0], self.root)
        return out

    def objects(self) -> list[dict]:
        objs = []
        for text in self.render().values():
            objs.extend(d for d in yaml.safe_load_all(text) if d)
        return objs


def _split_pipes(expr: str) -> list[str]:
    parts, cur, q = [], [], False
    for ch in expr:
        if ch == '"':
            q = not q
        if ch == "|" and not q:
            parts.append("".join(cur))
            cur = []
        else:
            cur.append(ch)
    parts.append("".join(cur))
    return parts


def _deep_merge(a: dict, b: dict) -> dict:
    out = dict(a)
    for k, v in b.items():
        out[k] = _deep_merge(out[k], v) if isinstance(v, dict) and isinstance(out.get(k), dict) else v
    return out


def render_chart(chart_dir: str, values: dict | None = None, **kw) -> list[dict]:
    return Renderer(chart_dir, values, **kw).objects()
