"""xGMI gang co-location (NodeResourceTopologyMatch PreFilter, gangColocation).

The reference aligns a pod to one NUMA zone in Filter: a pod that cannot be
aligned does not fit (pkg/noderesourcetopology/filter.go:84-150, 190-216).
SURVEY.md §2.1 C15 / §2.7 lift the zone to the 8-GPU xGMI mesh of one MI355X
node, for the gang rather than the pod (scheduler/gang_placement.h): a gang
goes to a node that can host all of its ranks whenever one exists (Preferred),
or waits parked until one does (Required). The gang records carry the node set
(`nodes`) and whether a hosting node existed at the first rank (`hostable`).
"""
import time

from flex_gpu_scheduler_amd import load_config, new_scheduler
from flex_gpu_scheduler_amd.models import GPU, make_pod, make_pod_group, mi355x_node
from flex_gpu_scheduler_amd.models.mi355x import GPU_XCD, INDEX_ANNOTATION, mi355x_nrt
from flex_gpu_scheduler_amd.utils.workload import flagship_config


def wait_for(pred, timeout=10.0):
    t0 = time.time()
    while not pred():
        if time.time() - t0 > timeout:
            return False
        time.sleep(0.002)
    return True


def scheduler(store, colocation="Preferred", start=True):
    cfg = flagship_config(permit_wait_s=10, denied_s=20, gang_colocation=colocation)
    s = new_scheduler(store, load_config(cfg), podInitialBackoffSeconds=1, podMaxBackoffSeconds=10)
    if start:
        s.start()
    return s


def add_node(store, name, mode="spx"):
    store.create("nodes", mi355x_node(name, mode=mode))
    store.create("noderesourcetopologies", mi355x_nrt(name))


def occupy(store, node, gpus, prefix="busy"):
    """`gpus` whole GPUs of `node` held by pods already bound there."""
    for i in range(gpus):
        store.create("pods", make_pod(f"{prefix}-{node}-{i}", limits={GPU: "1"}, node_name=node,
                                      annotations={INDEX_ANNOTATION: str(i)}))


def submit(store, name, size, limits=None):
    store.create("podgroups", make_pod_group(name, "default", size))
    names = [f"{name}-r{r}" for r in range(size)]
    for n in names:
        store.create("pods", make_pod(n, limits=limits or {GPU: "1"}, pod_group=name))
    return names


def node_of(store, names):
    return [store.get("pods", "default", n)["spec"].get("nodeName", "") for n in names]


def test_gang_of_four_goes_to_the_node_that_hosts_it_all(store):
    """The round-5 reproduction: mi-0 has 8 free GPUs, mi-1 has 3. Bin-packing
    alone prefers mi-1 for the first rank; co-location keeps all four on mi-0."""
    add_node(store, "mi-0")
    add_node(store, "mi-1")
    occupy(store, "mi-1", 5)
    s = scheduler(store)
    try:
        g = submit(store, "g4", 4)
        assert wait_for(lambda: all(node_of(store, g)))
        assert set(node_of(store, g)) == {"mi-0"}
        recs = [r for r in s.gang_records() if r["pod_group"] == "default/g4"]
        assert recs and recs[0]["nodes"] == 1 and recs[0]["hostable"] == 1
    finally:
        s.stop()


def test_none_mode_scores_only_and_can_split(store):
    """gangColocation None keeps round 5's soft score: the same setup splits
    (this is the behaviour the PreFilter plan removes)."""
    add_node(store, "mi-0")
    add_node(store, "mi-1")
    occupy(store, "mi-1", 5)
    s = scheduler(store, colocation="None")
    try:
        g = submit(store, "g4", 4)
        assert wait_for(lambda: all(node_of(store, g)))
        assert len(set(node_of(store, g))) == 2
        recs = [r for r in s.gang_records() if r["pod_group"] == "default/g4"]
        assert recs and recs[0]["nodes"] == 2 and recs[0]["hostable"] == -1
    finally:
        s.stop()


def test_split_only_when_no_node_can_host(store):
    """Preferred: 3 + 3 free GPUs and a gang of 4 -> it splits (no node could
    host it), and the record says so."""
    add_node(store, "mi-0")
    add_node(store, "mi-1")
    occupy(store, "mi-0", 5)
    occupy(store, "mi-1", 5)
    s = scheduler(store)
    try:
        g = submit(store, "g4", 4)
        assert wait_for(lambda: all(node_of(store, g)))
        recs = [r for r in s.gang_records() if r["pod_group"] == "default/g4"]
        assert recs and recs[0]["nodes"] == 2 and recs[0]["hostable"] == 0
    finally:
        s.stop()


def test_required_mode_parks_until_one_node_can_host(store):
    """Required: the same 3 + 3 cluster parks the gang instead of splitting
    it; freeing GPUs on one node lets it in, all ranks on that node."""
    add_node(store, "mi-0")
    add_node(store, "mi-1")
    occupy(store, "mi-0", 5)
    occupy(store, "mi-1", 5)
    s = scheduler(store, colocation="Required")
    try:
        g = submit(store, "g4", 4)
        assert wait_for(lambda: s.gang_parks() >= 1)
        time.sleep(0.2)
        assert not any(node_of(store, g))
        assert s.gang_denials()[0] == 0
        store.delete("pods", "default", "busy-mi-1-0")
        assert wait_for(lambda: all(node_of(store, g)), timeout=5.0)
        assert set(node_of(store, g)) == {"mi-1"}
    finally:
        s.stop()


def test_required_gang_larger_than_a_node_still_spans_nodes(store):
    """A 12-rank gang cannot fit one 8-GPU node: Required does not block it."""
    add_node(store, "mi-0")
    add_node(store, "mi-1")
    s = scheduler(store, colocation="Required")
    try:
        g = submit(store, "g12", 12)
        assert wait_for(lambda: all(node_of(store, g)))
        assert len(set(node_of(store, g))) == 2
    finally:
        s.stop()


def test_ranks_follow_the_first_rank(store):
    """Two idle nodes: every rank of an 8-gang and of a 4-gang lands on one
    node (later ranks are planned onto the node hosting their siblings)."""
    for i in range(4):
        add_node(store, f"mi-{i}")
    s = scheduler(store)
    try:
        gangs = {f"g{i}": submit(store, f"g{i}", size) for i, size in enumerate((8, 4, 2, 4, 8, 2))}
        assert wait_for(lambda: all(all(node_of(store, g)) for g in gangs.values()))
        for name, g in gangs.items():
            assert len(set(node_of(store, g))) == 1, (name, node_of(store, g))
    finally:
        s.stop()


def test_gang_plan_counts_ranks_owed_to_an_anchored_gang(store):
    """Gang x has 1 of 6 ranks on mi-0 (7 free): its 5 remaining ranks are
    owed to mi-0, so a new gang of 4 may only start on mi-1 — without the
    reservation the tighter mi-0 would win and one of the two would split."""
    add_node(store, "mi-0")
    add_node(store, "mi-1")
    store.create("podgroups", make_pod_group("x", "default", 6))
    store.create("pods", make_pod("x-r0", limits={GPU: "1"}, pod_group="x", node_name="mi-0",
                                  annotations={INDEX_ANNOTATION: "0"}))
    for r in range(1, 6):
        store.create("pods", make_pod(f"x-r{r}", limits={GPU: "1"}, pod_group="x"))
    store.create("podgroups", make_pod_group("y", "default", 4))
    for r in range(4):
        store.create("pods", make_pod(f"y-r{r}", limits={GPU: "1"}, pod_group="y"))
    s = scheduler(store, start=False)
    s.sync_informers()
    px = s.plugin_call("NodeResourceTopologyMatch", "gangPlan", {"pod": store.get("pods", "default", "x-r1")})
    assert px["gang"] and px["started"] and px["remaining"] == 5
    assert px["nodes"] == ["mi-0"] and px["hostable"]
    py = s.plugin_call("NodeResourceTopologyMatch", "gangPlan", {"pod": store.get("pods", "default", "y-r0")})
    assert py["gang"] and not py["started"] and py["remaining"] == 4 and py["hostable"]
    assert py["nodes"] == ["mi-1"] and py["fallback"]


def test_xcd_gang_stays_on_one_cpx_node(store):
    """CPX quarter gangs (4 x 2 XCDs) on two CPX nodes, one partly used."""
    add_node(store, "cpx-0", mode="cpx")
    add_node(store, "cpx-1", mode="cpx")
    s = scheduler(store)
    try:
        names = []
        for i in range(6):
            names.append(submit(store, f"q{i}", 4, limits={GPU_XCD: "2"}))
        assert wait_for(lambda: all(all(node_of(store, g)) for g in names))
        for g in names:
            assert len(set(node_of(store, g))) == 1
    finally:
        s.stop()


def test_random_clusters_keep_a_hostable_gang_on_one_node():
    """Randomised: 4 nodes with 0-8 GPUs already held each and one gang of
    2/4/8 that at least one node can host. Under Preferred every rank lands on
    one node, and that node had room for the whole gang."""
    import random

    from flex_gpu_scheduler_amd import Store

    rng = random.Random(20261019)
    trials = 0
    while trials < 12:
        held = [rng.randint(0, 8) for _ in range(4)]
        k = rng.choice((2, 4, 8))
        if max(8 - h for h in held) < k:
            continue
        trials += 1
        store = Store()
        for i, h in enumerate(held):
            add_node(store, f"mi-{i}")
            occupy(store, f"mi-{i}", h)
        s = scheduler(store)
        try:
            g = submit(store, f"g{trials}", k)
            assert wait_for(lambda: all(node_of(store, g))), (held, k)
            nodes = set(node_of(store, g))
            assert len(nodes) == 1, (held, k, node_of(store, g))
            host = int(next(iter(nodes)).split("-")[1])
            assert 8 - held[host] >= k, (held, k, nodes)
        finally:
            s.stop()


def test_concurrent_gangs_split_only_when_no_node_could_host_them():
    """Randomised, many gangs in flight at once: 6 empty nodes and gangs of
    1/2/4/8 submitted together (up to 40 of the 48 GPUs). A gang may span
    nodes only if, when its first rank was placed, no node could host it
    (`hostable` 0): an avoidable split never happens."""
    import random

    from flex_gpu_scheduler_amd import Store

    rng = random.Random(6)
    for trial in range(4):
        store = Store()
        for i in range(6):
            add_node(store, f"mi-{i}")
        s = scheduler(store)
        try:
            sizes, total = [], 0
            while True:
                k = rng.choice((1, 2, 4, 8))
                if total + k > 40:
                    break
                sizes.append(k)
                total += k
            groups = [submit(store, f"t{trial}-g{i}", k) for i, k in enumerate(sizes)]
            assert wait_for(lambda: all(all(node_of(store, g)) for g in groups), timeout=20.0), sizes
            recs = {r["pod_group"]: r for r in s.gang_records()}
            for i, g in enumerate(groups):
                r = recs.get(f"default/t{trial}-g{i}")
                assert r is not None
                if len(set(node_of(store, g))) > 1:
                    assert r["hostable"] == 0, (sizes, i, node_of(store, g), r)
        finally:
            s.stop()
