"""`make verify`: the repository's static checks (the reference's
hack/verify-*.sh + golangci-lint, Makefile:43-129), with tools this image has.

  python     every module compiles; no unused imports (AST); no tabs,
             trailing whitespace or lines over 130 columns
  native     C++/HIP sources: no tabs, trailing whitespace or lines over 130
             columns; headers use #pragma once and no `using namespace`
  crds       deploy/crds equals a fresh `deploy.crds` generation
  charts     both Helm charts render (deploy/helm.py) and every image they
             reference is the one the Makefile builds
  configs    every example KubeSchedulerConfiguration decodes strictly
  docker     every Dockerfile COPY source exists and the entrypoint module imports

    python -m flex_gpu_scheduler_amd.tools.verify [--only python,crds,...]
"""
from __future__ import annotations

import argparse
import ast
import filecmp
import re
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
MAX_COLS = 130
PY_DIRS = ["flex_gpu_scheduler_amd", "tests", "bench.py", "__graft_entry__.py"]
NATIVE_DIRS = ["csrc"]
NATIVE_EXT = {".cc", ".h", ".hip", ".cpp"}


def _files(dirs: list[str], exts: set[str]) -> list[Path]:
    out = []
    for d in dirs:
        p = ROOT / d
        if p.is_file():
            out.append(p)
            continue
        out += [f for f in p.rglob("*") if f.suffix in exts and "__pycache__" not in f.parts]
    return sorted(out)


def _text_checks(path: Path, text: str) -> list[str]:
    errs = []
    for i, line in enumerate(text.splitlines(), 1):
        if "\t" in line:
            errs.append(f"{path}:{i}: tab")
        if line != line.rstrip():
            errs.append(f"{path}:{i}: trailing whitespace")
        if len(line) > MAX_COLS:
            errs.append(f"{path}:{i}: {len(line)} columns (max {MAX_COLS})")
    return errs


class _Names(ast.NodeVisitor):
    def __init__(self):
        self.used: set[str] = set()

    def visit_Name(self, node):
        self.used.add(node.id)

    def visit_Attribute(self, node):
        root = node
        while isinstance(root, ast.Attribute):
            root = root.value
        if isinstance(root, ast.Name):
            self.used.add(root.id)
        self.generic_visit(node)


def unused_imports(path: Path, tree: ast.Module, text: str) -> list[str]:
    if path.name == "__init__.py":
        return []  # re-exports
    imported: dict[str, int] = {}
    for node in ast.walk(tree):
        if isinstance(node, ast.Import):
            for a in node.names:
                imported[(a.asname or a.name).split(".")[0]] = node.lineno
        elif isinstance(node, ast.ImportFrom):
            if node.module == "__future__":
                continue
            for a in node.names:
                if a.name != "*":
                    imported[a.asname or a.name] = node.lineno
    v = _Names()
    v.visit(tree)
    # Names referenced only in string annotations or __all__ count as used.
    strings = " ".join(n.value for n in ast.walk(tree) if isinstance(n, ast.Constant) and isinstance(n.value, str))
    errs = []
    lines = text.splitlines()
    for name, ln in sorted(imported.items(), key=lambda kv: kv[1]):
        if name in v.used or re.search(rf"\b{re.escape(name)}\b", strings):
            continue
        if "noqa" in lines[ln - 1]:
            continue
        errs.append(f"{path}:{ln}: unused import {name}")
    return errs


def check_python() -> list[str]:
    errs = []
    for f in _files(PY_DIRS, {".py"}):
        text = f.read_text()
        try:
            tree = ast.parse(text, str(f))
        except SyntaxError as e:
            errs.append(f"{f}:{e.lineno}: {e.msg}")
            continue
        errs += _text_checks(f, text) + unused_imports(f, tree, text)
    return errs


def check_native() -> list[str]:
    errs = []
    for f in _files(NATIVE_DIRS, NATIVE_EXT):
        text = f.read_text()
        errs += _text_checks(f, text)
        if f.suffix == ".h":
            if "#pragma once" not in text:
                errs.append(f"{f}: header without #pragma once")
            if re.search(r"^\s*using namespace\s", text, re.M):
                errs.append(f"{f}: `using namespace` in a header")
    return errs


_LOG_CALL = re.compile(r"\bXS_(LOGV|INFO|WARN|ERROR)\(")


def check_logging() -> list[str]:
    """Structured logging (the reference's hack/verify-structured-logging.sh):
    native log calls take a constant message and put every variable in
    key/values (`XS_LOGV(6, "fit indexes").kv("pod", ...)`), never a message
    built at run time."""
    errs = []
    for f in _files(NATIVE_DIRS, NATIVE_EXT):
        if f.name not in ("log.h", "log.cc"):
            errs += log_call_errors(f, f.read_text())
    return errs


def log_call_errors(f, text: str) -> list[str]:
    errs = []
    for m in _LOG_CALL.finditer(text):
        rest = text[m.end():]
        if m.group(1) == "LOGV":
            rest = rest.split(",", 1)[1] if "," in rest else ""
        if not re.match(r'\s*"(?:[^"\\]|\\.)*"\s*\)', rest):
            line = text.count("\n", 0, m.start()) + 1
            errs.append(f"{f}:{line}: log message is not a constant string (use .kv() for values)")
    return errs


def check_crds() -> list[str]:
    from ..deploy.crds import write_all

    with tempfile.TemporaryDirectory() as d:
        write_all(d)
        ours = ROOT / "deploy" / "crds"
        cmp = filecmp.dircmp(d, ours)
        errs = [f"deploy/crds/{n}: differs from the generator (run `make crds`)" for n in cmp.diff_files]
        errs += [f"deploy/crds/{n}: missing (run `make crds`)" for n in cmp.left_only]
        errs += [f"deploy/crds/{n}: not produced by the generator" for n in cmp.right_only]
        # dircmp compares shallowly (size+mtime); compare contents explicitly.
        for n in cmp.same_files:
            if (Path(d) / n).read_bytes() != (ours / n).read_bytes():
                errs.append(f"deploy/crds/{n}: differs from the generator (run `make crds`)")
        return errs


def makefile_image() -> str:
    mk = (ROOT / "Makefile").read_text()
    vals = dict(re.findall(r"^(\w+)\s*\?=\s*(\S+)", mk, re.M))
    return f"{vals['IMAGE_REPO']}:{vals['IMAGE_TAG']}"


def _images(obj, out: set[str]) -> None:
    if isinstance(obj, dict):
        for k, v in obj.items():
            if k == "image" and isinstance(v, str):
                out.add(v)
            else:
                _images(v, out)
    elif isinstance(obj, list):
        for v in obj:
            _images(v, out)


def check_charts() -> list[str]:
    import yaml

    from ..deploy.helm import Renderer

    want = makefile_image()
    errs = []
    for chart in sorted((ROOT / "deploy" / "charts").iterdir()):
        for vf in [None] + sorted(chart.glob("values.*.yaml")):
            vals = yaml.safe_load(vf.read_text()) if vf else None
            try:
                objs = Renderer(str(chart), vals).objects()
            except Exception as e:  # noqa: BLE001
                errs.append(f"{chart.name} ({vf.name if vf else 'values.yaml'}): render failed: {e}")
                continue
            imgs: set[str] = set()
            _images(objs, imgs)
            for img in sorted(imgs - {want}):
                errs.append(f"{chart.name} ({vf.name if vf else 'values.yaml'}): image {img} is not the "
                            f"Makefile's {want}")
            if not imgs:
                errs.append(f"{chart.name}: renders no container image")
    return errs


def check_configs() -> list[str]:
    import yaml

    from ..config import load_config

    errs = []
    for f in sorted((ROOT / "deploy" / "examples").glob("*-config.yaml")):
        try:
            load_config(yaml.safe_load(f.read_text()))
        except Exception as e:  # noqa: BLE001
            errs.append(f"{f}: {e}")
    return errs


def check_docker() -> list[str]:
    import importlib

    errs = []
    files = sorted((ROOT / "deploy" / "docker").glob("Dockerfile*"))
    if not files:
        return ["deploy/docker: no Dockerfile"]
    for f in files:
        text = f.read_text()
        for m in re.finditer(r"^COPY\s+(?!--from)(.+)$", text, re.M):
            parts = [p for p in m.group(1).split() if not p.startswith("--")]
            for src in parts[:-1]:
                if not list(ROOT.glob(src)):
                    errs.append(f"{f.name}: COPY source {src} does not exist")
        ep = re.search(r'^ENTRYPOINT\s+\[(.*)\]', text, re.M)
        if not ep:
            errs.append(f"{f.name}: no exec-form ENTRYPOINT")
            continue
        args = [a.strip().strip('"') for a in ep.group(1).split(",")]
        if "-m" in args:
            mod = args[args.index("-m") + 1]
            try:
                importlib.import_module(mod)
            except Exception as e:  # noqa: BLE001
                errs.append(f"{f.name}: entrypoint module {mod} does not import: {e}")
    return errs


CHECKS = {"python": check_python, "native": check_native, "logging": check_logging, "crds": check_crds,
          "charts": check_charts, "configs": check_configs, "docker": check_docker}


def main(argv: list[str] | None = None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--only", default="", help="comma-separated subset of " + ",".join(CHECKS))
    a = ap.parse_args(argv)
    names = [n for n in a.only.split(",") if n] or list(CHECKS)
    total = 0
    for n in names:
        errs = CHECKS[n]()
        total += len(errs)
        print(f"verify {n}: {'ok' if not errs else f'{len(errs)} problem(s)'}")
        for e in errs[:200]:
            print("  " + str(e).replace(str(ROOT) + "/", ""))
    return 1 if total else 0


if __name__ == "__main__":
    sys.exit(main())
