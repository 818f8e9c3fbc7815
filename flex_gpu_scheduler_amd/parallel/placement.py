"""End-to-end xGMI placement validation.

The scheduler's promise for a distributed-training gang on one 8x MI355X node
is that every rank gets its own physical GPU on the node's xGMI mesh, so the
job's RCCL ring never leaves the fabric. This module checks that promise with
the real components, in the order a cluster runs them:

  1. discovery   the node is built from live sysfs/KFD discovery
                 (gpu/discovery.py) by the node agent's own Node/NRT builders;
                 GPUs this job does not hold are occupied by bound "tenant"
                 pods, so the scheduler has to pick around them;
  2. scheduling  PodGroups of 1/2/4/8 ranks go through Coscheduling + FlexGPU
                 + NodeResourceTopologyMatch(XGMIGangAffinity) (the bench's
                 flagship profile, reference gang semantics
                 pkg/coscheduling/coscheduling.go:184-216);
  3. allocation  each bound rank is resolved by the kubelet device-plugin gRPC
                 `Allocate` (control/device_plugin.py) served on a unix
                 socket; its DeviceSpecs (render nodes) name the GPUs;
  4. data plane  the render nodes are mapped back to host GPUs and, by PCI
                 address, to HIP ordinals; the torch.distributed ranks that own
                 exactly those ordinals form a sub-communicator and run an
                 all-reduce sweep (RCCL when on GPUs), checked numerically.

Each gang is measured next to deliberately bad placements of the same size:
  * `cross_socket`: the same number of GPUs straddling both CPU sockets (on a
    full xGMI mesh this should NOT lose bandwidth: the check that socket
    affinity only matters for host traffic, docs/ARCHITECTURE.md §3);
  * `host_staged`: the placed ranks reduced through host memory over TCP
    (gloo), the path a gang split across nodes without GPU-direct RDMA gets.

Each multi-rank row is judged against an expected-bandwidth model built from
the discovered KFD io_links (`busbw_model`): a ring all-reduce on a full mesh
drives, per rank, the direct xGMI links to the other members of its gang, so
the model is  min over ranks of (sum of those links' one-way bandwidth) x
RING_EFFICIENCY (one-way link bandwidth: KFD reports it per direction). `verdict` is "pass" when the placed gang reaches at least
PASS_FRACTION of the model and beats the host-staged path, "fail" otherwise,
and "n/a" where no xGMI model applies (one GPU, or a gloo/CPU rehearsal).

Everything runs outside the bench's timed region. On a CPU-only host (tests)
the node comes from `fake_host` and the collectives run on gloo.
"""
from __future__ import annotations

import datetime
import json
import os
import tempfile
import time
from dataclasses import asdict, dataclass, field

GANG_SIZES = (1, 2, 4, 8)
NODE = "mi355x-live"
NAMESPACE = "placement"

# MI355X Infinity Fabric: 7 xGMI links per GPU, 153.6 GB/s per link counting
# both directions (1,075 GB/s aggregate), i.e. 76.8 GB/s each way. KFD's
# io_links `max_bandwidth` (MB/s) is the one-way figure: the MI355X box reads
# 76,000 MB/s per xGMI link (profiles/r5bf_bench_store_shrink.json,
# rccl_placement.node), next to the 153.6 GB/s bidirectional spec. The spec
# value is used when KFD reports no plausible per-link bandwidth.
XGMI_LINK_GBPS_BIDIR = 153.6
XGMI_LINK_GBPS_ONEWAY = XGMI_LINK_GBPS_BIDIR / 2
# Fraction of the links' one-way bandwidth a large ring all-reduce turns into
# bus bandwidth (protocol, reduction and channel scheduling overheads). An
# assumption, not a measurement: no run of this code has had more than one
# GPU, so the 8-rank parity is unpinned until the driver's 8-GPU run.
RING_EFFICIENCY = 0.75
PASS_FRACTION = 0.7


def busbw_model(host, gpu_index: list[int]) -> dict:
    """Expected all-reduce bus bandwidth (GB/s) for a gang on these host GPUs,
    from the KFD xGMI io_links: each rank can drive its direct links to the
    other members, the slowest rank bounds the ring."""
    if len(gpu_index) < 2:
        return {"model_busbw_GBps": None, "why": "single rank"}
    by_index = {g.index: g for g in host.gpus}
    kfd_to_index = {g.kfd_node: g.index for g in host.gpus if g.kfd_node is not None}
    members = set(gpu_index)
    per_rank = []
    source = "kfd io_links"
    for i in gpu_index:
        g = by_index.get(i)
        if g is None:
            return {"model_busbw_GBps": None, "why": f"GPU {i} not discovered"}
        oneway = 0.0
        links = 0
        for lk in g.xgmi_links:
            peer = kfd_to_index.get(lk.peer_node, lk.peer_node if not kfd_to_index else None)
            if peer is None or peer == i or peer not in members:
                continue
            links += 1
            gbps = lk.bandwidth_mbps / 1000.0  # one way (see XGMI_LINK_GBPS_ONEWAY)
            if not 10.0 <= gbps <= 200.0:  # no usable per-link figure: the part's spec
                gbps = XGMI_LINK_GBPS_ONEWAY
                source = "kfd io_links (topology) + MI355X link spec (bandwidth)"
            oneway += gbps
        per_rank.append((links, oneway))
    min_links = min(n for n, _ in per_rank)
    if min_links == 0:
        return {"model_busbw_GBps": None, "why": "some rank has no direct xGMI link to the gang", "direct_links": 0}
    oneway = min(b for _, b in per_rank)
    return {"model_busbw_GBps": round(RING_EFFICIENCY * oneway, 1), "direct_links_min": min_links,
            "links_oneway_GBps": round(oneway, 1), "ring_efficiency": RING_EFFICIENCY, "source": source}


def judge_row(row: dict, model: dict, backend: str) -> dict:
    """Verdict fields for one gang row (see the module docstring)."""
    out = {"model": model}
    largest = lambda k: (row[k]["results"][-1]["busbw_GBps"]  # noqa: E731
                         if k in row and "results" in row[k] and row[k]["results"] else None)
    placed, staged, cross = largest("placed"), largest("host_staged"), largest("cross_socket")
    out["placed_busbw_GBps"] = placed
    out["host_staged_busbw_GBps"] = staged
    out["cross_socket_over_placed"] = round(cross / placed, 3) if cross and placed else None
    m = model.get("model_busbw_GBps")
    if backend != "nccl" or m is None or placed is None:
        out["verdict"] = "n/a"
        out["why"] = ("no xGMI data plane (gloo/CPU run)" if backend != "nccl" else
                      model.get("why") or "no placed measurement")
        return out
    out["placed_over_model"] = round(placed / m, 3)
    checks = {"placed_ge_%.0f%%_of_model" % (PASS_FRACTION * 100): placed >= PASS_FRACTION * m,
              "placed_ge_host_staged": staged is None or placed >= staged,
              "all_correct": all(x["correct"] for k in ("placed", "cross_socket", "host_staged")
                                 if k in row and "results" in row[k] for x in row[k]["results"])}
    out["checks"] = checks
    out["verdict"] = "pass" if all(checks.values()) else "fail"
    return out


@dataclass
class GangPlan:
    size: int
    pods: list[str]
    gpu_index: list[int]                      # host GPU index per rank (scheduler annotation)
    allocate_env: list[dict]                  # kubelet Allocate envs per rank
    render_nodes: list[str]                   # Allocate DeviceSpecs (one per rank)
    ordinals: list[int]                       # HIP ordinals of the allocated GPUs
    sockets: list[int]
    cross_socket: list[int] = field(default_factory=list)  # deliberately bad placement (ordinals)
    schedule_ms: float = 0.0


# --------------------------------------------------------------- discovery
def local_ordinals(host, world: int, cuda: bool) -> dict[int, int]:
    """Host GPU index -> HIP ordinal, for the GPUs of `host` this job's ranks
    own (ordinal < world). Matched by PCI address against what HIP reports, so
    a HIP enumeration order that differs from sysfs order cannot misroute a
    rank."""
    if not cuda:
        return {g.index: g.index for g in host.gpus if g.index < world}
    import torch

    by_bdf = {g.bdf.lower(): g.index for g in host.gpus}
    out: dict[int, int] = {}
    for o in range(min(world, torch.cuda.device_count())):
        p = torch.cuda.get_device_properties(o)
        bdf = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
        if bdf in by_bdf:
            out[by_bdf[bdf]] = o
    if not out:
        # No sysfs match (hidden PCI info): fall back to KFD enumeration order,
        # the order the ROCr runtime uses for the agents it can open.
        vis = sorted((g for g in host.gpus if g.kfd_node is not None), key=lambda g: g.kfd_node)
        out = {g.index: o for o, g in enumerate(vis) if o < world}
    return out


# -------------------------------------------------------------- scheduling
def _allocate_rpc(plugin, sock: str, n: int):
    import grpc

    from ..control.deviceplugin_api import method_path, pb

    with grpc.insecure_channel(f"unix://{sock}") as ch:
        call = ch.unary_unary(method_path("DevicePlugin", "Allocate"),
                              request_serializer=pb.AllocateRequest.SerializeToString,
                              response_deserializer=pb.AllocateResponse.FromString)
        req = pb.AllocateRequest()
        req.container_requests.add(devicesIDs=[f"gpu-{i}" for i in range(n)])
        return call(req, timeout=10)


def plan_gangs(host, ordinal_of: dict[int, int], sizes=GANG_SIZES, timeout: float = 30.0,
               bandwidth_tables: dict[int, dict] | None = None) -> dict:
    """Schedule one PodGroup per size on the live node and resolve each rank
    through the device plugin. `bandwidth_tables` (HIP ordinal -> the rank's
    partition table) are published on the Node by the node agent, one per
    GPU. Returns {"plans": [...], "node": {...}}."""
    from ..config import load_config
    from ..control.client import LocalClient
    from ..control.device_plugin import ASSIGNED_ANNOTATION, GpuDevicePlugin
    from ..control.node_agent import NodeAgent
    from ..models.mi355x import GPU, INDEX_ANNOTATION
    from ..models.objects import make_container, make_pod, make_pod_group
    from ..scheduler import Store, new_scheduler
    from ..utils.workload import flagship_config

    store = Store()
    client = LocalClient(store)
    agent = NodeAgent(client, NODE, host_fn=lambda: host, publish_metrics=False)
    for idx, o in ordinal_of.items():
        if bandwidth_tables and o in bandwidth_tables:
            agent.bandwidth[idx] = bandwidth_tables[o]
    agent.sync()
    held = sorted(ordinal_of)
    by_card = {}
    for g in host.gpus:
        minor = int(g.card[4:]) if g.card.startswith("card") and g.card[4:].isdigit() else 0
        by_card[f"/dev/dri/renderD{128 + minor}"] = g.index
    socket_of = {g.index: g.numa for g in host.gpus}

    # Other tenants hold every GPU this job does not own: bound, running pods
    # with a GPU index, exactly what the scheduler's cache sees on a shared node.
    for g in host.gpus:
        if g.index in ordinal_of:
            continue
        name = f"tenant-gpu{g.index}"
        store.create("pods", make_pod(name, NAMESPACE, containers=[make_container("t", limits={GPU: "1"},
                                                                                   requests={GPU: "1"})]))
        store.bind(NAMESPACE, name, "", NODE, {INDEX_ANNOTATION: str(g.index), ASSIGNED_ANNOTATION: "true"})

    sched = new_scheduler(store, load_config(flagship_config()), start=True)
    sockdir = tempfile.mkdtemp(prefix="xsp", dir="/tmp")  # unix socket paths must stay short
    plugin = GpuDevicePlugin(GPU, host, client, NODE, socket_dir=sockdir).serve()
    plans: list[GangPlan] = []
    try:
        for k in sizes:
            if k > len(held):
                continue
            pg = f"gang{k}"
            pods = [f"{pg}-r{r}" for r in range(k)]
            t0 = time.perf_counter()
            store.create("podgroups", make_pod_group(pg, NAMESPACE, k))
            store.create_many("pods", json.dumps([
                make_pod(p, NAMESPACE, pod_group=pg, containers=[make_container(
                    "trainer", requests={"cpu": "4", "memory": "16Gi", GPU: "1"}, limits={GPU: "1"})])
                for p in pods]))
            deadline = time.perf_counter() + timeout
            while True:
                bound = {p["metadata"]["name"]: p for p in store.list("pods", NAMESPACE)[0]
                         if p["metadata"]["name"] in pods and p["spec"].get("nodeName")}
                if len(bound) == k:
                    break
                if time.perf_counter() > deadline:
                    raise RuntimeError(f"gang of {k} not bound within {timeout}s: {sched.stats()}")
                time.sleep(0.001)
            t_sched = (time.perf_counter() - t0) * 1e3
            # kubelet side: one Allocate per rank container; the plugin
            # resolves which pod it is for and marks it assigned.
            envs, devs, gidx, owners = [], [], [], []
            for _ in range(k):
                resp = _allocate_rpc(plugin, plugin.socket_path, 1).container_responses[0]
                paths = [d.host_path for d in resp.devices if "renderD" in d.host_path]
                if len(paths) != 1 or paths[0] not in by_card:
                    raise RuntimeError(f"Allocate returned unexpected devices {paths}")
                envs.append(dict(resp.envs))
                devs.append(paths[0])
                gidx.append(by_card[paths[0]])
                owners.append(resp.annotations.get("xsched.amd.com/pod", ""))
            ann = [int(bound[p]["metadata"]["annotations"][INDEX_ANNOTATION]) for p in pods]
            if sorted(ann) != sorted(gidx):
                raise RuntimeError(f"Allocate devices {gidx} disagree with the scheduler's indexes {ann}")
            if len(set(gidx)) != k or any(i not in ordinal_of for i in gidx):
                raise RuntimeError(f"gang of {k} placed on {gidx}, not {k} distinct GPUs held by this job")
            order = sorted(range(k), key=lambda i: owners[i])
            plan = GangPlan(k, [owners[i] for i in order], [gidx[i] for i in order], [envs[i] for i in order],
                            [devs[i] for i in order], [ordinal_of[gidx[i]] for i in order],
                            [socket_of[gidx[i]] for i in order], schedule_ms=round(t_sched, 3))
            plan.cross_socket = _cross_socket(plan, ordinal_of, socket_of)
            plans.append(plan)
            for p in pods:
                store.delete("pods", NAMESPACE, p)
            store.delete("podgroups", NAMESPACE, pg)
            sched.sync_informers(int(timeout * 1000))  # the cache has dropped the gang before the next one
    finally:
        plugin.stop_server()
        sched.stop()
    return {"plans": plans, "node": {"gpus": len(host.gpus), "held": len(held),
                                     "sockets": sorted({g.numa for g in host.gpus}),
                                     "xgmi_links": [len(g.xgmi_links) for g in host.gpus],
                                     "xgmi_link_max_bandwidth_mbps": sorted({lk.bandwidth_mbps for g in host.gpus
                                                                             for lk in g.xgmi_links}),
                                     "bandwidth_tables_published": len(agent.bandwidth)}}


def _cross_socket(plan: GangPlan, ordinal_of: dict[int, int], socket_of: dict[int, int]) -> list[int]:
    """A same-size set of held GPUs that straddles both sockets, if the
    scheduler's choice did not (empty when no such set exists)."""
    if len(set(plan.sockets)) > 1 or plan.size < 2:
        return []
    by_socket: dict[int, list[int]] = {}
    for idx in sorted(ordinal_of):
        by_socket.setdefault(socket_of[idx], []).append(idx)
    if len(by_socket) < 2:
        return []
    lists = list(by_socket.values())
    pick: list[int] = []
    i = 0
    while len(pick) < plan.size and any(lists):
        lst = lists[i % len(lists)]
        if lst:
            pick.append(lst.pop(0))
        i += 1
    return [ordinal_of[x] for x in pick] if len(pick) == plan.size else []


# -------------------------------------------------------------- data plane
def _reduce_bw(group, members: list[int], rank: int, nbytes: int, cuda: bool, iters: int, warmup: int,
               host_staged: bool = False) -> dict:
    """All-reduce sweep on `group` (called by members only). Returns busBW and
    a numeric check: every rank contributes (rank+1), so each element must be
    sum(members)+len(members)."""
    import torch
    import torch.distributed as dist

    dev = torch.device("cuda", torch.cuda.current_device()) if cuda else torch.device("cpu")
    n = len(members)
    x = torch.full((nbytes // 4,), float(rank + 1), dtype=torch.float32, device=dev)
    host = torch.empty(x.shape, dtype=x.dtype, pin_memory=cuda) if host_staged else None

    def once():
        if host_staged:
            host.copy_(x)
            dist.all_reduce(host, group=group)
            x.copy_(host)
        else:
            dist.all_reduce(x, group=group)

    for _ in range(warmup):
        once()
    # After warmup every element has been summed `warmup` times: re-fill, run
    # one reduction and check it exactly.
    x.fill_(float(rank + 1))
    once()
    expect = float(sum(m + 1 for m in members))
    ok = bool(torch.all(x == expect).item())
    if cuda:
        torch.cuda.synchronize()
    dist.barrier(group=group)
    t0 = time.perf_counter()
    for _ in range(iters):
        once()
    if cuda:
        torch.cuda.synchronize()
    t = (time.perf_counter() - t0) / iters
    alg = nbytes / t / 1e9
    return {"MiB": nbytes >> 20, "ms": round(t * 1e3, 3), "algbw_GBps": round(alg, 2),
            "busbw_GBps": round(alg * 2 * (n - 1) / n, 2), "correct": ok}


def validate_placement(ctx, sizes=GANG_SIZES, rccl_mib=(16, 256), staged_mib=(16,), iters: int = 10,
                       warmup: int = 3, root: str = "/", group_timeout_s: float = 120.0,
                       bandwidth_tables: dict[int, dict] | None = None) -> dict:
    """Collective over all ranks of `ctx` (parallel/dist.py DistContext).
    Rank 0 plans (discovery -> scheduler -> Allocate), every rank joins the
    sub-communicators; rank 0 returns the table, other ranks return {}."""
    import torch.distributed as dist

    from ..gpu.discovery import discover_host, fake_host

    plan_doc = None
    if ctx.rank == 0:
        try:
            host = discover_host(root) if ctx.cuda else fake_host(max(ctx.world_size, 1))
            if ctx.cuda and not host.gpus:
                host = fake_host(ctx.world_size)
                source = "fake (no amdgpu sysfs visible)"
            else:
                source = "live sysfs/KFD" if ctx.cuda else "fake_host (CPU run)"
            ordinal_of = local_ordinals(host, ctx.world_size, ctx.cuda)
            res = plan_gangs(host, ordinal_of, sizes, bandwidth_tables=bandwidth_tables)
            plan_doc = {"source": source, "node": res["node"], "plans": [asdict(p) for p in res["plans"]],
                        "ordinal_of": {str(k): v for k, v in ordinal_of.items()},
                        "models": {str(p.size): busbw_model(host, p.gpu_index) for p in res["plans"]}}
        except Exception as e:  # noqa: BLE001 - reported, and every rank skips the data plane
            plan_doc = {"error": f"{type(e).__name__}: {e}"}
    if ctx.distributed:
        box = [plan_doc]
        dist.broadcast_object_list(box, src=0)
        plan_doc = box[0]
    if "error" in plan_doc:
        return plan_doc if ctx.rank == 0 else {}

    backend = "nccl" if ctx.cuda else "gloo"
    if not ctx.cuda:  # CPU rehearsal: the same path with loopback-sized messages
        rccl_mib, staged_mib = (1, 4), (1,)
    rows = []
    for p in plan_doc["plans"]:
        row = {"gang": p["size"], "gpus": p["gpu_index"], "ordinals": p["ordinals"], "sockets": p["sockets"],
               "hip_visible_devices_in_container": [e.get("HIP_VISIBLE_DEVICES") for e in p["allocate_env"]],
               "xsched_gpu_index": [e.get("XSCHED_GPU_INDEX") for e in p["allocate_env"]],
               "schedule_ms": p["schedule_ms"]}
        if p["size"] >= 2 and ctx.distributed:
            specs = [("placed", p["ordinals"], backend, False, rccl_mib)]
            if p["cross_socket"]:
                specs.append(("cross_socket", p["cross_socket"], backend, False, rccl_mib))
            specs.append(("host_staged", p["ordinals"], "gloo", True, staged_mib))
            for label, ranks, be, staged, mibs in specs:
                ranks = sorted(ranks)
                # new_group is collective over the whole world, members or not;
                # every rank walks the same specs even after a failure, so the
                # world stays in step and the error is reported per row.
                out = None
                g = None
                try:
                    g = dist.new_group(ranks=ranks, backend=be, timeout=datetime.timedelta(seconds=group_timeout_s))
                    if ctx.rank in ranks:
                        out = [_reduce_bw(g, ranks, ctx.rank, m << 20, ctx.cuda,
                                          iters if not staged else max(2, iters // 3), warmup if not staged else 1,
                                          host_staged=staged and ctx.cuda) for m in mibs]
                except Exception as e:  # noqa: BLE001
                    out = {"error": f"rank {ctx.rank}: {type(e).__name__}: {e}"}
                got = ctx.gather(out)
                if ctx.rank == 0:
                    errs = [r["error"] for r in got if isinstance(r, dict)]
                    res = [r for r in got if isinstance(r, list)]
                    if errs or not res:
                        row[label] = {"ranks": ranks, "backend": be, "error": "; ".join(errs) or "no results"}
                    else:
                        # The slowest member defines the collective's bandwidth.
                        per = []
                        for i in range(len(mibs)):
                            worst = min((r[i] for r in res), key=lambda d: d["busbw_GBps"])
                            per.append({**worst, "correct": all(r[i]["correct"] for r in res)})
                        row[label] = {"ranks": ranks, "backend": be, "results": per}
                if g is not None:
                    try:
                        dist.destroy_process_group(g)
                    except Exception:  # noqa: BLE001
                        pass
        rows.append(row)
    if ctx.rank != 0:
        return {}
    summary = {}
    for r in rows:
        model = plan_doc.get("models", {}).get(str(r["gang"]), {"model_busbw_GBps": None, "why": "no model"})
        r.update(judge_row(r, model, backend))
        if "placed" not in r:
            summary[str(r["gang"])] = {"verdict": r["verdict"], "why": r.get("why")}
            continue
        kinds = [k for k in ("placed", "cross_socket", "host_staged") if k in r]
        s = {k: ({str(x["MiB"]): x["busbw_GBps"] for x in r[k]["results"]} if "results" in r[k]
                 else {"error": r[k]["error"]}) for k in kinds}
        s["all_correct"] = all("results" in r[k] and all(x["correct"] for x in r[k]["results"]) for k in kinds)
        s["model_busbw_GBps"] = model.get("model_busbw_GBps")
        s["verdict"] = r["verdict"]
        summary[str(r["gang"])] = s
    return {"source": plan_doc["source"], "backend": backend, "node": plan_doc["node"], "gangs": rows,
            "summary": summary, "env": {"HSA_ENABLE_IPC_MODE_LEGACY": os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY")}}
