"""Informer windows parsed on the helper pool (XSCHED_PARSE_POOL=1,
Scheduler::informer_loop): a burst wave binds completely and the cache
debugger finds the accounting clean, as with inline parsing."""
import json
import time

import pytest

from flex_gpu_scheduler_amd import Store, load_config, new_scheduler
from flex_gpu_scheduler_amd.utils.workload import ClusterSpec, flagship_config, make_wave


@pytest.mark.parametrize("pool", ["0", "1"])
def test_wave_binds_and_cache_is_clean(monkeypatch, pool):
    monkeypatch.setenv("XSCHED_PARSE_POOL", pool)
    spec = ClusterSpec(nodes=48)
    store = Store()
    store.create_many("nodes", json.dumps(spec.node_objects()))
    store.create_many("noderesourcetopologies", json.dumps(spec.nrt_objects()))
    s = new_scheduler(store, load_config(flagship_config()), seed=5)
    s.start()
    try:
        w = make_wave(spec, 1, namespace="w", fill=0.6)
        for groups_js, pods_js in w.chunks_json():
            if groups_js != "[]":
                store.create_many("podgroups", groups_js)
            if pods_js != "[]":
                store.create_many("pods", pods_js)
        assert s.wait_bound(len(w.pods), 30.0), s.stats()
        # Bound counts at the Bind call; the informer confirms the assumed
        # pods when their Modified events arrive (a loaded host lags). The
        # debugger reads the listers and then the cache, two snapshots: an
        # event landing between them reads as a transient difference, so
        # only a difference that persists fails.
        deadline = time.time() + 10.0
        check = s.check_cache()
        while not check["clean"] and time.time() < deadline:
            time.sleep(0.01)
            check = s.check_cache()
        assert check["clean"], {k: v for k, v in check.items() if v}
        store.delete_all("pods", "w")
        assert s.wait_cache_empty(30.0)
    finally:
        s.stop()
