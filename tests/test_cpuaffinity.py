"""Shard CPU placement (utils/cpuaffinity.py): list parsing, domain ranking
and disjoint per-rank picks."""
import os

from flex_gpu_scheduler_amd.utils import cpuaffinity as ca


def test_parse_list():
    assert ca._parse_list("0-3,8,10-11\n") == {0, 1, 2, 3, 8, 10, 11}


def test_pick_none_and_explicit():
    assert ca.pick("none") is None
    assert ca.pick("") is None
    assert ca.pick("2,0-1") == [0, 1, 2]


def test_ranks_take_disjoint_domains():
    order = [[0, 1], [2, 3], [4, 5], [6, 7]]
    picks = [ca.pick("l3", r, order=order) for r in range(4)]
    assert picks == order
    assert ca.pick("l3x2", 1, order=order) == [4, 5, 6, 7]
    assert ca.pick("l3", 5, order=order) == [2, 3]  # wraps


def test_single_domain_is_left_alone():
    assert ca.pick("l3", 0, order=[[0, 1, 2]]) is None


def test_domains_cover_affinity():
    doms = ca.l3_domains()
    allowed = set(os.sched_getaffinity(0))
    assert set().union(*map(set, doms)) <= allowed
    assert all(doms)
