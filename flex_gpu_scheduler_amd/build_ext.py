"""In-tree native build: the C++ scheduler core (`_xsched`) and the HIP/CDNA4
probe kernels (`ops/_hipprobe`).

Both land next to the Python sources (not site-packages) so the built `.so`
files travel with the repo snapshot to the MI355X box and show up as loaded
native code. Compilation is parallel and incremental (object files are
rebuilt when their source or any header is newer).

Usage:
    python -m flex_gpu_scheduler_amd.build_ext            # core + hip
    python -m flex_gpu_scheduler_amd.build_ext --core     # C++ core only
    python -m flex_gpu_scheduler_amd.build_ext --tsan     # ThreadSanitizer stress driver
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "csrc"
PKG = ROOT / "flex_gpu_scheduler_amd"
BUILD = ROOT / "build"
HIP_ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))

CORE_DIRS = ["common", "api", "store", "framework", "scheduler", "plugins", "rest", "apiserver"]
# OpenSSL for the native REST client's TLS (rest/http.cc).
LINK_LIBS = ["-lssl", "-lcrypto"]
CXXFLAGS = ["-std=c++20", "-O3", "-fPIC", "-Wall", "-Wno-unused-variable", "-Wno-unused-parameter",
            "-Wno-sign-compare", "-fvisibility=hidden", "-pthread",
            *os.environ.get("XSCHED_CXXFLAGS_EXTRA", "").split()]


def _ext_suffix() -> str:
    return sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def core_sources() -> list[Path]:
    out = []
    for d in CORE_DIRS:
        out.extend(sorted((CSRC / d).glob("*.cc")))
    return out


def _headers_mtime() -> float:
    hs = list(CSRC.rglob("*.h"))
    return max((h.stat().st_mtime for h in hs), default=0.0)


def _jobs() -> int:
    env = os.environ.get("MAX_JOBS")
    if env and env.isdigit():
        return max(1, int(env))
    return max(1, min(16, os.cpu_count() or 4))


def _compile(cmd: list[str], src: Path) -> None:
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed for {src}:\n{' '.join(cmd)}\n{r.stderr[-8000:]}")


def build_objects(srcs: list[Path], objdir: Path, extra: list[str], includes: list[str]) -> list[Path]:
    objdir.mkdir(parents=True, exist_ok=True)
    hmt = _headers_mtime()
    todo = []
    objs = []
    for s in srcs:
        o = objdir / (s.relative_to(CSRC).as_posix().replace("/", "__") + ".o")
        objs.append(o)
        if o.exists() and o.stat().st_mtime >= max(s.stat().st_mtime, hmt):
            continue
        cmd = ["g++", *CXXFLAGS, *extra, *[f"-I{i}" for i in includes], "-c", str(s), "-o", str(o)]
        todo.append((cmd, s))
    if todo:
        with cf.ThreadPoolExecutor(_jobs()) as ex:
            futs = [ex.submit(_compile, c, s) for c, s in todo]
            for f in futs:
                f.result()
    return objs


def build_core(verbose: bool = True) -> Path:
    import pybind11

    py_inc = sysconfig.get_paths()["include"]
    # The amd-smi telemetry sampler compiles against the ROCm header and loads
    # libamd_smi with dlopen at first use (no link-time dependency).
    includes = [str(CSRC), pybind11.get_include(), py_inc, str(ROCM / "include")]
    srcs = core_sources() + sorted((CSRC / "telemetry").glob("*.cc")) + [CSRC / "python" / "bindings.cc"]
    objs = build_objects(srcs, BUILD / "core", [], includes)
    out = PKG / f"_xsched{_ext_suffix()}"
    newest = max(o.stat().st_mtime for o in objs)
    if not out.exists() or out.stat().st_mtime < newest:
        cmd = ["g++", "-shared", "-pthread", *[str(o) for o in objs], *LINK_LIBS, "-o", str(out)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr[-8000:]}")
        if verbose:
            print(f"[build_ext] linked {out.relative_to(ROOT)}")
    return out


def build_core_debuginfo(verbose: bool = True) -> Path:
    """The extension with -g (same optimisation: identical code, line
    tables for tools/sample_report --lines) in dbg/, for sampling runs that
    copy it over the package's extension on a scratch tree."""
    import pybind11

    py_inc = sysconfig.get_paths()["include"]
    includes = [str(CSRC), pybind11.get_include(), py_inc, str(ROCM / "include")]
    srcs = core_sources() + sorted((CSRC / "telemetry").glob("*.cc")) + [CSRC / "python" / "bindings.cc"]
    objs = build_objects(srcs, BUILD / "core_g", ["-g1", "-gz"], includes)
    out = ROOT / "dbg" / f"_xsched{_ext_suffix()}"
    out.parent.mkdir(exist_ok=True)
    cmd = ["g++", "-shared", "-pthread", *[str(o) for o in objs], *LINK_LIBS, "-o", str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr[-8000:]}")
    if verbose:
        print(f"[build_ext] linked {out.relative_to(ROOT)}")
    return out


def build_hip(verbose: bool = True) -> Path | None:
    hipcc = shutil.which("hipcc") or str(ROCM / "bin" / "hipcc")
    if not Path(hipcc).exists():
        raise RuntimeError("hipcc not found; the HIP probes require ROCm")
    srcs = sorted((CSRC / "hip").glob("*.hip"))
    if not srcs:
        return None
    out = PKG / "ops" / "_hipprobe.so"
    newest = max([s.stat().st_mtime for s in srcs] + [_headers_mtime()])
    if out.exists() and out.stat().st_mtime >= newest:
        return out
    cmd = [hipcc, f"--offload-arch={HIP_ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           f"-I{CSRC}", *[str(s) for s in srcs], "-o", str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed:\n{' '.join(cmd)}\n{r.stderr[-8000:]}")
    if verbose:
        print(f"[build_ext] built {out.relative_to(ROOT)} for {HIP_ARCH}")
    return out


def build_stream_sweep(verbose: bool = True) -> Path:
    """The HBM streaming design sweep (csrc/tools/stream_sweep.hip), a
    standalone gfx950 executable next to the probes: ops/stream_sweep."""
    hipcc = shutil.which("hipcc") or str(ROCM / "bin" / "hipcc")
    src = CSRC / "tools" / "stream_sweep.hip"
    out = PKG / "ops" / "stream_sweep"
    if out.exists() and out.stat().st_mtime >= src.stat().st_mtime:
        return out
    cmd = [hipcc, f"--offload-arch={HIP_ARCH}", "-O3", "-std=c++17", str(src), "-o", str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed:\n{' '.join(cmd)}\n{r.stderr[-8000:]}")
    if verbose:
        print(f"[build_ext] built {out.relative_to(ROOT)} for {HIP_ARCH}")
    return out


def build_tsan(verbose: bool = True) -> Path:
    """Native concurrency stress driver built with -fsanitize=thread (host only)."""
    includes = [str(CSRC)]
    extra = ["-fsanitize=thread", "-g", "-O1", "-include", str(CSRC / "tools" / "tsan_compat.h")]
    objs = build_objects(core_sources() + [CSRC / "tools" / "stress_main.cc"], BUILD / "tsan", extra, includes)
    out = BUILD / "xsched_stress_tsan"
    cmd = ["g++", "-fsanitize=thread", "-pthread", *[str(o) for o in objs], *LINK_LIBS, "-o", str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"tsan link failed:\n{r.stderr[-8000:]}")
    if verbose:
        print(f"[build_ext] built {out.relative_to(ROOT)}")
    return out


def build_asan(verbose: bool = True) -> Path:
    """Native stress driver built with -fsanitize=address,undefined (host only)."""
    includes = [str(CSRC)]
    flags = ["-fsanitize=address,undefined", "-fno-omit-frame-pointer"]
    objs = build_objects(core_sources() + [CSRC / "tools" / "stress_main.cc"], BUILD / "asan", [*flags, "-g", "-O1"],
                         includes)
    out = BUILD / "xsched_stress_asan"
    cmd = ["g++", *flags, "-pthread", *[str(o) for o in objs], *LINK_LIBS, "-o", str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"asan link failed:\n{r.stderr[-8000:]}")
    if verbose:
        print(f"[build_ext] built {out.relative_to(ROOT)}")
    return out


def build_prof(verbose: bool = True, gprof: bool = True, debuginfo: bool = False) -> Path:
    """Native stress driver (no Python in the loop). With `gprof` it is built
    with -pg for a per-function CPU profile of the scheduling hot path;
    without, at the core's optimisation level for timing (`debuginfo` adds
    -g, same code, for sample_report --lines)."""
    includes = [str(CSRC)]
    extra = ["-pg", "-g", "-O2", "-fno-omit-frame-pointer", "-fno-inline-functions-called-once"] if gprof else []
    if debuginfo and not gprof:
        extra = ["-g"]
    sub = "prof" if gprof else ("stress_g" if debuginfo else "stress")
    objs = build_objects(core_sources() + [CSRC / "tools" / "stress_main.cc"], BUILD / sub, extra, includes)
    out = BUILD / ("xsched_stress_prof" if gprof else ("xsched_stress_g" if debuginfo else "xsched_stress"))
    cmd = ["g++", *(["-pg"] if gprof else []), "-pthread", *[str(o) for o in objs], *LINK_LIBS, "-o", str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"prof link failed:\n{r.stderr[-8000:]}")
    if verbose:
        print(f"[build_ext] built {out.relative_to(ROOT)}")
    return out


def build_tests(verbose: bool = True) -> Path:
    """Native unit-test binary (csrc/tests/native_tests.cc)."""
    # Same flags as the extension's objects, so the core objects are shared
    # with build/core (no second compile of the core).
    includes = [str(CSRC)]
    objs = build_objects(core_sources() + [CSRC / "tests" / "native_tests.cc"], BUILD / "core", [], includes)
    out = BUILD / "xsched_native_tests"
    newest = max(o.stat().st_mtime for o in objs)
    if out.exists() and out.stat().st_mtime >= newest:
        return out
    cmd = ["g++", "-pthread", *[str(o) for o in objs], *LINK_LIBS, "-o", str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"native tests link failed:\n{r.stderr[-8000:]}")
    if verbose:
        print(f"[build_ext] built {out.relative_to(ROOT)}")
    return out


def main(argv: list[str] | None = None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--core", action="store_true")
    ap.add_argument("--hip", action="store_true")
    ap.add_argument("--tsan", action="store_true")
    ap.add_argument("--asan", action="store_true")
    ap.add_argument("--prof", action="store_true")
    ap.add_argument("--stress", action="store_true")
    ap.add_argument("--stress-g", action="store_true", help="stress driver with -g (sample_report --lines)")
    ap.add_argument("--tests", action="store_true")
    ap.add_argument("--core-g", action="store_true", help="the extension with -g into dbg/ (sampling runs)")
    a = ap.parse_args(argv)
    if a.core_g:
        build_core_debuginfo()
        return 0
    if a.tests:
        build_tests()
        return 0
    if a.prof or a.stress or a.stress_g:
        build_prof(gprof=a.prof, debuginfo=a.stress_g)
        return 0
    everything = not (a.core or a.hip or a.tsan or a.asan)
    if a.core or everything:
        build_core()
    if a.hip or everything:
        build_hip()
    if a.tsan:
        build_tsan()
    if a.asan:
        build_asan()
    return 0


if __name__ == "__main__":
    sys.exit(main())
