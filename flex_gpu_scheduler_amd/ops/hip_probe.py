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
    mode: str
    bytes: int
    gbps: float
    ms_per_iter: float
    cu_limit: int


class HipProbe:
    def __init__(self, path: str | Path = _LIB):
        if not Path(path).exists():
            raise ProbeError(f"{path} not built; run `python -m flex_gpu_scheduler_amd.build_ext --hip`")
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
        L.xs_xcd_census.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                                    ctypes.POINTER(ctypes.c_int)]
        L.xs_health_check.argtypes = [ctypes.c_int, ctypes.c_size_t, ctypes.POINTER(ctypes.c_ulonglong),
                                      ctypes.POINTER(ctypes.c_ulonglong)]
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

    def hbm_bandwidth(self, dev: int = 0, nbytes: int = 1 << 30, iters: int = 20, cu_limit: int = 0,
                      mode: str = "copy") -> Bandwidth:
        g, ms = ctypes.c_double(), ctypes.c_double()
        rc = self.lib.xs_hbm_bandwidth(dev, nbytes, iters, cu_limit, MODES[mode], ctypes.byref(g), ctypes.byref(ms))
        if rc != 0:
            raise self._err(rc, "hbm_bandwidth")
        return Bandwidth(mode, nbytes, g.value, ms.value, cu_limit)

    @staticmethod
    def variant(unroll: int = 4, nontemporal: bool = True, blocks_per_cu: int = 8) -> int:
        return unroll | (0x100 if nontemporal else 0) | (blocks_per_cu << 16)

    def hbm_bandwidth_variant(self, dev: int, nbytes: int, iters: int, mode: str, unroll: int, nontemporal: bool,
                              blocks_per_cu: int, cu_limit: int = 0) -> Bandwidth:
        g, ms = ctypes.c_double(), ctypes.c_double()
        v = self.variant(unroll, nontemporal, blocks_per_cu)
        rc = self.lib.xs_hbm_bandwidth_v(dev, nbytes, iters, cu_limit, MODES[mode], v, ctypes.byref(g), ctypes.byref(ms))
        if rc != 0:
            raise self._err(rc, "hbm_bandwidth_v")
        return Bandwidth(mode, nbytes, g.value, ms.value, cu_limit)

    def tune(self, dev: int = 0, mode: str = "copy", nbytes: int = 1 << 30, iters: int = 10) -> dict:
        """Sweep unroll x cache policy x workgroups/CU; return the fastest."""
        results = []
        for unroll in (1, 4, 8):
            for nt in (True, False):
                for bpc in (4, 8, 16):
                    bw = self.hbm_bandwidth_variant(dev, nbytes, iters, mode, unroll, nt, bpc)
                    results.append({"unroll": unroll, "nontemporal": nt, "blocks_per_cu": bpc,
                                    "GBps": round(bw.gbps, 1)})
        best = max(results, key=lambda r: r["GBps"])
        return {"mode": mode, "best": best, "all": results}

    def hbm_bandwidth_xcd(self, dev: int = 0, xcd_mask: int = 0x1, nbytes: int = 1 << 30, iters: int = 10,
                          mode: str = "read") -> Bandwidth:
        """HBM bandwidth pulled by the workgroups on the XCDs of `xcd_mask`
        only — what one CPX (1 XCD) / QPX (2) / DPX (4) partition can stream."""
        g, ms = ctypes.c_double(), ctypes.c_double()
        rc = self.lib.xs_hbm_bandwidth_xcd(dev, nbytes, iters, xcd_mask, MODES[mode], ctypes.byref(g), ctypes.byref(ms))
        if rc != 0:
            raise self._err(rc, "hbm_bandwidth_xcd")
        return Bandwidth(mode, nbytes, g.value, ms.value, bin(xcd_mask).count("1") * 32)

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
