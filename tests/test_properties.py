"""Hypothesis property tests (SURVEY.md §4 test plan): exact Quantity
arithmetic against a rational-number oracle, and FlexGPU bin-packing
invariants over random pod mixes on random MI355X nodes."""
import json
import time
from fractions import Fraction

from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from flex_gpu_scheduler_amd import Store, load_config, new_scheduler
from flex_gpu_scheduler_amd._native import native
from flex_gpu_scheduler_amd.models import GPU, GPU_MEMORY, GPU_XCD, GpuInfo, make_pod, mi355x_node

from helpers import FLEXGPU_PLUGINS, coscheduling_config

X = native()

DEC = {"n": Fraction(1, 10**9), "u": Fraction(1, 10**6), "m": Fraction(1, 1000), "": Fraction(1), "k": Fraction(10**3),
       "M": Fraction(10**6), "G": Fraction(10**9), "T": Fraction(10**12)}
BIN = {"Ki": 2**10, "Mi": 2**20, "Gi": 2**30, "Ti": 2**40}


@st.composite
def quantity(draw):
    whole = draw(st.integers(0, 99999))
    frac = draw(st.sampled_from(["", ".5", ".25", ".125", ".001"]))
    suffix = draw(st.sampled_from(list(DEC) + list(BIN)))
    if (suffix in BIN or suffix == "n") and frac:
        frac = ""  # (sub-nano amounts round up to 1n, like apimachinery)
    return f"{whole}{frac}{suffix}"


def exact(q: str) -> Fraction:
    for s in sorted(BIN, key=len, reverse=True):
        if q.endswith(s):
            return Fraction(q[: -len(s)]) * BIN[s]
    for s in sorted(DEC, key=len, reverse=True):
        if s and q.endswith(s):
            return Fraction(q[: -len(s)]) * DEC[s]
    return Fraction(q)


def ceil(f: Fraction) -> int:
    return -((-f.numerator) // f.denominator)


@settings(max_examples=300, deadline=None)
@given(quantity())
def test_quantity_value_and_milli_round_up(q):
    milli, value, canon = X.parse_quantity(q)
    v = exact(q)
    sat = 2**63 - 1  # Value()/MilliValue() saturate instead of wrapping
    assert value == min(ceil(v), sat)
    assert milli == min(ceil(v * 1000), sat)
    # The canonical form denotes the same amount.
    assert X.quantity_cmp(canon, q) == 0


@settings(max_examples=200, deadline=None)
@given(quantity(), quantity())
def test_quantity_compare_and_sum_exact(a, b):
    va, vb = exact(a), exact(b)
    assert X.quantity_cmp(a, b) == (va > vb) - (va < vb)
    s = X.resource_list_op({"r": a}, {"r": b}, "add")["r"]
    assert exact_canonical(s) == va + vb
    d = X.resource_list_op({"r": s}, {"r": b}, "sub")["r"]
    assert exact_canonical(d) == va
    m = X.resource_list_op({"r": a}, {"r": b}, "max")["r"]
    assert exact_canonical(m) == max(va, vb)


def exact_canonical(q: str) -> Fraction:
    if "e" in q and not q.endswith(("Ki", "Mi", "Gi", "Ti", "Pi", "Ei")):
        base, exp = q.split("e")
        return Fraction(base) * Fraction(10) ** int(exp)
    return exact(q) if not q.endswith(("P", "E", "Pi", "Ei")) else Fraction(X.parse_quantity(q)[1])


# ------------------------------------------------------------ bin packing --
MODES = ["spx", "dpx", "qpx", "cpx"]


@st.composite
def cluster(draw):
    nodes = []
    for n in range(draw(st.integers(1, 3))):
        modes = draw(st.lists(st.sampled_from(MODES), min_size=8, max_size=8))
        nodes.append([GpuInfo(g, modes[g], numa=g // 4) for g in range(8)])
    pods = draw(st.lists(st.one_of(
        st.tuples(st.just(GPU), st.integers(1, 4)),
        st.tuples(st.just(GPU_XCD), st.sampled_from([1, 2, 4, 8])),
        st.tuples(st.just(GPU_MEMORY), st.sampled_from([16, 36, 72, 144]))), min_size=1, max_size=40))
    return nodes, pods


@settings(max_examples=40, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(cluster())
def test_flexgpu_never_overcommits(c):
    nodes, pods = c
    store = Store()
    for i, gpus in enumerate(nodes):
        store.create("nodes", mi355x_node(f"n{i}", gpus=gpus))
    s = new_scheduler(store, load_config(coscheduling_config(FLEXGPU_PLUGINS)), start=True)
    try:
        store.create_many("pods", json.dumps([make_pod(f"p{k}", limits={r: str(v)}, requests={r: str(v)})
                                              for k, (r, v) in enumerate(pods)]))
        s.sync_informers(50)
        # Let every pod get at least one attempt; stop once nothing is active.
        deadline = time.time() + 10
        while time.time() < deadline:
            q = s.queue_counts()
            if q["active"] == 0:
                time.sleep(0.05)
                if s.queue_counts()["active"] == 0:
                    break
            time.sleep(0.01)
        placed = [p for p in store.list("pods", "default")[0] if p["spec"].get("nodeName")]
        per_node: dict = {}
        for p in placed:
            per_node.setdefault(p["spec"]["nodeName"], []).append(p)
        for name, ps in per_node.items():
            gpus = nodes[int(name[1:])]
            whole, parts, mem = {}, {}, {}
            for p in ps:
                ann = p["metadata"]["annotations"]
                lim = p["spec"]["containers"][0]["resources"]["limits"]
                (res, amount), = lim.items()
                idx = [int(x) for x in ann["amd.com/gpu-index"].split(",")]
                if res == GPU:
                    assert len(idx) == int(amount)
                    for g in idx:
                        assert gpus[g].partition_mode == "spx", "whole-GPU pod on a partitioned GPU"
                        whole[g] = whole.get(g, 0) + 1
                elif res == GPU_XCD:
                    assert len(idx) == 1
                    g = idx[0]
                    ps_ = [tuple(map(int, x.split(":"))) for x in ann["amd.com/gpu-partitions"].split(",")]
                    xpp = 8 // gpus[g].partitions
                    assert len(ps_) * xpp >= int(amount)
                    for gp in ps_:
                        assert gp[0] == g
                        parts[gp] = parts.get(gp, 0) + 1
                else:
                    g, part = map(int, ann["amd.com/gpu-partitions"].split(":"))
                    mem[(g, part)] = mem.get((g, part), 0) + int(amount)
            for g, n in whole.items():
                assert n == 1, f"GPU {g} on {name} given to {n} whole-GPU pods"
                assert not any(k[0] == g for k in parts) and not any(k[0] == g for k in mem)
            for gp, n in parts.items():
                assert n == 1, f"partition {gp} on {name} double-booked"
                assert gp not in mem
            for (g, part), used in mem.items():
                assert used <= gpus[g].hbm_gib // gpus[g].partitions, f"partition {(g, part)} memory overcommitted"
    finally:
        s.stop()
