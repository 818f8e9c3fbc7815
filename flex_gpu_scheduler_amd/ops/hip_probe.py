"""ctypes front-end for the HIP/CDNA4 device probes (csrc/hip/hbm_probe.hip,
csrc/hip/mfma_probe.hip).

The probes are what the node agent runs before advertising an MI355X as
schedulable: device properties, HBM streaming bandwidth (optionally with a
partition-sized CU budget), an XCD census that verifies the compute-partition
mode, a checksum health test, an exact-integer MFMA tile check of the matrix
cores and the dense bf16 MFMA throughput of the whole GPU or of one
partition's XCDs.
"""
from __future__ import annotations

import ctypes
import json
from dataclasses import dataclass
from pathlib import Path

_LIB = Path(__file__).resolve().parent / "_hipprobe.so"
MODES = {"read": 0, "write": 1, "copy": 2, "triad": 3}


class ProbeError(RuntimeError):
    pass


@dataclass
class Bandwidth:
    """`gbps` / `ms_per_iter`: the median launch, each timed by its own event
    pair (what rocprofv3 reports as the dispatch time). `best_gbps`: the
    fastest launch. `batch_gbps`: back-to-back launches including the gaps
    between them."""
    mode: str
    bytes: int
    gbps: float
    ms_per_iter: float
    cu_limit: int
    best_gbps: float = 0.0
    batch_gbps: float = 0.0


# Working sets default to 1 GiB per array: 4x the MI355X's 256 MB Infinity
# Cache, so a streaming rate is HBM's, not the cache's.
DEFAULT_BYTES = 1 << 30


class HipProbe:
    def __init__(self, path: str | Path = _LIB):
        if not Path(path).exists():
            raise ProbeError(f"{path} not built; run `python -m flex_gpu_scheduler_amd.build_ext --hip`")
        try:
            # torch's bundled libamdhip64.so.7 first, whatever the import order
            # of the caller: the probe library then resolves the same soname to
            # that copy, so one HIP runtime owns every device pointer and
            # stream in the process (tensors handed to the kernels included).
            import torch  # noqa: F401
        except ImportError:
            pass
        self.lib = ctypes.CDLL(str(path))
        L = self.lib
        L.xs_last_error.restype = ctypes.c_char_p
        L.xs_device_count.restype = ctypes.c_int
        L.xs_device_props.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_int]
        L.xs_hbm_bandwidth.argtypes = [ctypes.c_int, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                       ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]
        L.xs_hbm_bandwidth_v.argtypes = [ctypes.c_int, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_int, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]
        L.xs_hbm_bandwidth_xcd.argtypes = [ctypes.c_int, ctypes.c_size_t, ctypes.c_int, ctypes.c_uint32, ctypes.c_int,
                                           ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]
        L.xs_hbm_bandwidth_d.argtypes = [ctypes.c_int, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_int, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                         ctypes.POINTER(ctypes.c_double)]
        L.xs_hbm_bandwidth_xcd_d.argtypes = [ctypes.c_int, ctypes.c_size_t, ctypes.c_int, ctypes.c_uint32,
                                             ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                                             ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]
        L.xs_xcd_census.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                                    ctypes.POINTER(ctypes.c_int)]
        L.xs_health_check.argtypes = [ctypes.c_int, ctypes.c_size_t, ctypes.POINTER(ctypes.c_ulonglong),
                                      ctypes.POINTER(ctypes.c_ulonglong)]
        L.xs_stream_op.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                   ctypes.c_size_t, ctypes.c_uint32, ctypes.c_float, ctypes.c_int]
        L.xs_pinned_op.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                   ctypes.c_uint32]
        L.xs_segment_access.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_size_t,
                                        ctypes.c_size_t, ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
        L.xs_mfma_last_error.restype = ctypes.c_char_p
        L.xs_mfma_check.argtypes = [ctypes.c_int, ctypes.c_int]
        L.xs_mfma_peak.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_uint32, ctypes.c_int,
                                   ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                   ctypes.POINTER(ctypes.c_int)]

    def _err(self, rc: int, what: str) -> ProbeError:
        return ProbeError(f"{what} failed ({rc}): {self.lib.xs_last_error().decode(errors='replace')}")

    def device_count(self) -> int:
        return int(self.lib.xs_device_count())

    def props(self, dev: int = 0) -> dict:
        buf = ctypes.create_string_buffer(4096)
        rc = self.lib.xs_device_props(dev, buf, len(buf))
        if rc < 0:
            raise self._err(rc, "device_props")
        return json.loads(buf.value.decode())

    def hbm_bandwidth(self, dev: int = 0, nbytes: int = DEFAULT_BYTES, iters: int = 20, cu_limit: int = 0,
                      mode: str = "copy", variant: int = 0) -> Bandwidth:
        g, ms = ctypes.c_double(), ctypes.c_double()
        d = (ctypes.c_double * 3)()
        rc = self.lib.xs_hbm_bandwidth_d(dev, nbytes, iters, cu_limit, MODES[mode], variant, ctypes.byref(g),
                                         ctypes.byref(ms), d)
        if rc != 0:
            raise self._err(rc, "hbm_bandwidth")
        return Bandwidth(mode, nbytes, g.value, ms.value, cu_limit, d[0], d[1])

    @staticmethod
    def variant(unroll: int = 4, nontemporal: bool = True, blocks_per_cu: int = 8) -> int:
        """blocks_per_cu 0: the one-shot grid (one workgroup per 4 KiB x
        unroll, no loop) instead of a persistent one."""
        if blocks_per_cu == 0:
            return unroll | (0x100 if nontemporal else 0) | 0x200
        return unroll | (0x100 if nontemporal else 0) | (blocks_per_cu << 16)

    def hbm_bandwidth_variant(self, dev: int, nbytes: int, iters: int, mode: str, unroll: int, nontemporal: bool,
                              blocks_per_cu: int, cu_limit: int = 0) -> Bandwidth:
        return self.hbm_bandwidth(dev, nbytes, iters, cu_limit, mode,
                                  variant=self.variant(unroll, nontemporal, blocks_per_cu))

    def tune(self, dev: int = 0, mode: str = "copy", nbytes: int = DEFAULT_BYTES, iters: int = 10) -> dict:
        """Sweep unroll x cache policy x workgroups/CU; return the fastest."""
        results = []
        for unroll in (1, 4, 8):
            for nt in (True, False):
                for bpc in (0, 4, 8, 16):
                    bw = self.hbm_bandwidth_variant(dev, nbytes, iters, mode, unroll, nt, bpc)
                    results.append({"unroll": unroll, "nontemporal": nt, "blocks_per_cu": bpc,
                                    "GBps": round(bw.gbps, 1)})
        best = max(results, key=lambda r: r["GBps"])
        return {"mode": mode, "best": best, "all": results}

    # ------------------------------------------------ kernels on torch tensors
    # The streaming kernels run on caller-owned device buffers so the GPU tier
    # can check their output against a plain PyTorch fp32 reference. torch
    # must be imported before this library is loaded (one HIP runtime: both
    # resolve the soname libamdhip64.so.7 to the same copy).
    @staticmethod
    def _dev_buf(t, what: str) -> tuple[int, int]:
        if not t.is_cuda or not t.is_contiguous():
            raise ValueError(f"{what} must be a contiguous device tensor")
        nbytes = t.numel() * t.element_size()
        if nbytes % 16 or t.data_ptr() % 16:
            raise ValueError(f"{what}: {nbytes} bytes at {t.data_ptr():#x} is not 16-byte granular")
        return t.data_ptr(), nbytes

    def _stream(self, dev: int, mode: int, a, b, c, nbytes: int, seed: int = 7, scale: float = 3.0,
                variant: int = 0) -> None:
        rc = self.lib.xs_stream_op(dev, mode, a, b, c, nbytes, seed, scale, variant)
        if rc != 0:
            raise self._err(rc, "stream_op")

    def write_pattern(self, dst, seed: int = 7, variant: int = 0) -> None:
        """k_write: every 16-B lane of `dst` <- (seed, seed^0x55555555, seed+1, ~seed) as uint32."""
        p, n = self._dev_buf(dst, "dst")
        self._stream(dst.device.index or 0, MODES["write"], p, None, None, n, seed=seed, variant=variant)

    def copy(self, dst, src, variant: int = 0) -> None:
        """k_copy: dst <- src (byte copy; equal sizes)."""
        pd, n = self._dev_buf(dst, "dst")
        ps, ns = self._dev_buf(src, "src")
        if n != ns:
            raise ValueError("copy: size mismatch")
        self._stream(dst.device.index or 0, MODES["copy"], ps, pd, None, n, variant=variant)

    def triad(self, a, b, c, scale: float = 3.0, variant: int = 0) -> None:
        """k_triad (STREAM): a <- b + scale*c on fp32 tensors."""
        import torch

        if not (a.dtype == b.dtype == c.dtype == torch.float32):
            raise ValueError("triad: fp32 tensors only")
        pa, n = self._dev_buf(a, "a")
        pb_, nb = self._dev_buf(b, "b")
        pc, nc = self._dev_buf(c, "c")
        if not n == nb == nc:
            raise ValueError("triad: size mismatch")
        self._stream(a.device.index or 0, MODES["triad"], pa, pb_, pc, n, scale=scale, variant=variant)

    def pinned(self, dst, src=None, xcd_mask: int = 0x1) -> None:
        """k_pinned on the XCDs of `xcd_mask`: copy src -> dst, or write the
        fill pattern (1, 2, 3, 4) into dst when src is None."""
        pd, n = self._dev_buf(dst, "dst")
        ps = 0
        if src is not None:
            ps, ns = self._dev_buf(src, "src")
            if ns != n:
                raise ValueError("pinned: size mismatch")
        rc = self.lib.xs_pinned_op(dst.device.index or 0, 2 if src is not None else 1, ps or None, pd, n, xcd_mask)
        if rc != 0:
            raise self._err(rc, "pinned_op")

    def hbm_bandwidth_xcd(self, dev: int = 0, xcd_mask: int = 0x1, nbytes: int = DEFAULT_BYTES, iters: int = 10,
                          mode: str = "read") -> Bandwidth:
        g, ms = ctypes.c_double(), ctypes.c_double()
        d = (ctypes.c_double * 3)()
        rc = self.lib.xs_hbm_bandwidth_xcd_d(dev, nbytes, iters, xcd_mask, MODES[mode], ctypes.byref(g),
                                             ctypes.byref(ms), d)
        if rc != 0:
            raise self._err(rc, "hbm_bandwidth_xcd")
        return Bandwidth(mode, nbytes, g.value, ms.value, bin(xcd_mask).count("1") * 32, d[0], d[1])

    def partition_table(self, dev: int = 0, nbytes: int = DEFAULT_BYTES, iters: int = 10) -> dict:
        """HBM read/copy GB/s that the CUs of one compute partition pull, for
        each partition size of an MI355X (CPX = 1 XCD, QPX = 2, DPX = 4,
        SPX = 8), measured on the XCDs a partition of that size would own.
        The node agent publishes it with the GPU's health (gpu/telemetry)."""
        rows = {}
        for mode_name, xcds in (("CPX", 1), ("QPX", 2), ("DPX", 4), ("SPX", 8)):
            if xcds == 8:
                # An SPX partition is the whole GPU, dispatched as any kernel
                # is: measured with the full-device streaming kernels, not the
                # XCD-pinned one (whose per-XCD work queues cost ~16% at 8 XCDs).
                r = self.hbm_bandwidth(dev, nbytes, iters, mode="read")
                c = self.hbm_bandwidth(dev, nbytes, iters, mode="copy")
                kernel = "k_read / k_copy (full device)"
            else:
                mask = (1 << xcds) - 1
                r = self.hbm_bandwidth_xcd(dev, mask, nbytes, iters, "read")
                c = self.hbm_bandwidth_xcd(dev, mask, nbytes, iters, "copy")
                kernel = "k_pinned (workgroups on the partition's XCDs)"
            rows[mode_name] = {"xcds": xcds, "cus": xcds * 32, "read_GBps": round(r.gbps, 1),
                               "copy_GBps": round(c.gbps, 1), "read_ms": round(r.ms_per_iter, 4), "kernel": kernel}
        return {"bytes": nbytes, "timing": "median of per-launch event pairs", "partitions": rows}

    def segment_access(self, dev: int = 0, mode: str = "read", seg_bytes: int = 128, stride_bytes: int = 4096,
                       touches: int = 1 << 18, iters: int = 5, nontemporal: bool = False) -> dict:
        """k_segments: `touches` segments of `seg_bytes`, one per
        `stride_bytes` slot -- a dispatch of known bytes and 128-B lines, for
        calibrating rocprofv3's L2 request counters (scripts/pmc_calibrate.sh)."""
        out = (ctypes.c_double * 3)()
        rc = self.lib.xs_segment_access(dev, MODES[mode], int(nontemporal), seg_bytes, stride_bytes, touches, iters,
                                        out)
        if rc != 0:
            raise self._err(rc, "segment_access")
        return {"kernel": "k_segments", "mode": mode, "nontemporal": nontemporal, "seg_bytes": seg_bytes,
                "stride_bytes": stride_bytes, "touches": touches, "ms": round(out[0], 4),
                "bytes_per_dispatch": int(out[1]), "lines128_per_dispatch": int(out[2])}

    def xcd_census(self, dev: int = 0, blocks: int = 4096) -> dict:
        hist = (ctypes.c_int * 8)()
        cus = ctypes.c_int()
        rc = self.lib.xs_xcd_census(dev, blocks, hist, ctypes.byref(cus))
        if rc < 0:
            raise self._err(rc, "xcd_census")
        return {"distinct_xcds": rc, "blocks_per_xcd": list(hist), "distinct_cu_slots": cus.value}

    def health(self, dev: int = 0, nbytes: int = 64 << 20) -> dict:
        d, h = ctypes.c_ulonglong(), ctypes.c_ulonglong()
        rc = self.lib.xs_health_check(dev, nbytes, ctypes.byref(d), ctypes.byref(h))
        if rc < 0:
            raise self._err(rc, "health_check")
        return {"healthy": rc == 0, "device_sum": d.value, "host_sum": h.value}


    def mfma_check(self, dev: int = 0, k: int = 64) -> dict:
        """C[32x32] = A·B through v_mfma_f32_32x32x16_bf16 on exact integers."""
        rc = self.lib.xs_mfma_check(dev, k)
        if rc < 0:
            raise ProbeError(f"mfma_check failed: {self.lib.xs_mfma_last_error().decode(errors='replace')}")
        return {"healthy": rc == 0, "mismatches": int(rc), "k": k}

    def mfma_peak(self, dev: int = 0, xcd_mask: int = 0xFF, iters: int = 4096, blocks: int = 0) -> dict:
        """Dense bf16 MFMA TFLOP/s on the XCDs of `xcd_mask`."""
        tf, ms, act = ctypes.c_double(), ctypes.c_double(), ctypes.c_int()
        rc = self.lib.xs_mfma_peak(dev, iters, xcd_mask, blocks, ctypes.byref(tf), ctypes.byref(ms), ctypes.byref(act))
        if rc != 0:
            raise ProbeError(f"mfma_peak failed: {self.lib.xs_mfma_last_error().decode(errors='replace')}")
        return {"tflops": tf.value, "ms": ms.value, "active_blocks": act.value, "xcd_mask": xcd_mask}


_probe: HipProbe | None = None


def probe() -> HipProbe:
    global _probe
    if _probe is None:
        _probe = HipProbe()
    return _probe
