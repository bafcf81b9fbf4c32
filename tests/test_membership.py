"""Native membership registry (csrc/core/membership.cpp)."""
from serverless_learn_amd._core import core


def test_register_is_idempotent_and_bumps_epoch_once():
    r = core().Registry()
    assert r.register_birth("a:1", "h", 1, 11, 0.0) == (1, True)
    assert r.register_birth("a:1", "h", 1, 11, 1.0) == (1, False)   # duplicate announcement
    assert r.members() == ["a:1"]
    assert r.register_birth("a:1", "h", 1, 12, 2.0) == (2, True)    # restarted process
    assert len(r) == 1


def test_ranks_follow_join_order_and_compact():
    r = core().Registry()
    for i, a in enumerate(["c:1", "a:1", "b:1"]):
        r.register_birth(a, "h", 1, i, 0.0)
    assert r.members() == ["c:1", "a:1", "b:1"]
    assert r.rank_of("b:1") == 2
    assert r.deregister("a:1")
    assert r.members() == ["c:1", "b:1"] and r.rank_of("b:1") == 1
    assert not r.deregister("zz:1")


def test_miss_counting_and_eviction():
    r = core().Registry()
    r.register_birth("a:1", "h", 0, 1, 0.0)
    e0 = r.epoch()
    assert not r.heartbeat_fail("a:1", 3)
    assert not r.heartbeat_fail("a:1", 3)
    r.heartbeat_ok("a:1", 1.0)                      # resets the miss counter
    assert not r.heartbeat_fail("a:1", 3)
    assert not r.heartbeat_fail("a:1", 3)
    assert r.heartbeat_fail("a:1", 3)
    assert r.members() == [] and r.epoch() == e0 + 1


def test_evict_stale_and_assignment():
    r = core().Registry()
    r.register_birth("a:1", "h", 0, 1, 0.0)
    r.register_birth("b:1", "h", 0, 2, 5.0)
    assert r.evict_stale(10.0, 7.0) == ["a:1"]
    r.register_birth("c:1", "h", 0, 3, 10.0)
    assert r.assignment(2) == [("b:1", 0), ("c:1", 1)]
    assert r.assignment(2, 1) == [("b:1", 1), ("c:1", 0)]


def test_deregister_checks_incarnation():
    r = core().Registry()
    r.register_birth("a:1", incarnation=7)
    r.register_birth("a:1", incarnation=8)  # the process restarted at the same address
    e = r.epoch()
    assert not r.deregister("a:1", 7)  # a late leave from the dead process
    assert r.members() == ["a:1"] and r.epoch() == e
    assert r.deregister("a:1", 8)
    assert r.members() == []
