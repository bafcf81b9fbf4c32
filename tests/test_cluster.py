"""End-to-end plumbing on CPU (BASELINE config 1) plus elastic behaviour."""
import numpy as np
import pytest
import torch

from serverless_learn_amd.runtime.local_cluster import LocalCluster, fast_config

pytestmark = pytest.mark.slow


@pytest.fixture
def cluster(request):
    kw = getattr(request, "param", {})
    c = LocalCluster(fast_config(**kw))
    yield c
    c.stop()


def test_single_worker_registers_ingests_and_trains(cluster):
    w = cluster.add_worker(sync="none")
    assert cluster.wait_for(lambda: w.registered.is_set(), 10)
    assert cluster.wait_for(lambda: w.step >= 40, 60), w.step
    assert 0 in w.files_received and w.bytes_ingested > 0
    assert cluster.wait_for(lambda: w.addr in cluster.master.feedback and cluster.master.feedback[w.addr]["step"] > 0, 10)
    st = w.trainer.stats()
    assert st.accuracy > 0.5, st


def test_allreduce_workers_stay_identical(cluster):
    a = cluster.add_worker(sync="allreduce", batch=512, max_steps=150)
    b = cluster.add_worker(sync="allreduce", batch=512, max_steps=150)
    assert cluster.wait_for(lambda: a.state == "done" and b.state == "done", 120), (a.step, b.step, a.state, b.state)
    assert a.step == b.step == 150
    assert a.group.world == 2 and b.group.world == 2
    assert torch.equal(a.trainer.params, b.trainer.params)
    # distinct shards per rank
    assert set(a.files_received) != set(b.files_received) or len(a.files_received) > 1


def test_eviction_bumps_epoch_and_survivors_regroup(cluster):
    ws = [cluster.add_worker(sync="allreduce", batch=256) for _ in range(3)]
    assert cluster.wait_for(lambda: all(w.group.world == 3 and w.step > 20 for w in ws), 120), \
        [(w.group.world, w.step) for w in ws]
    victim = ws[2]
    epoch_before = cluster.master.registry.epoch()
    victim.fault.kill_step = None
    victim._stop.set()
    victim.server.stop(grace=0)  # crash: no Deregister
    survivors = ws[:2]
    assert cluster.wait_for(lambda: cluster.master.registry.epoch() > epoch_before, 40)
    assert victim.addr not in cluster.master.registry.members()
    steps = [w.step for w in survivors]
    assert cluster.wait_for(lambda: all(w.group.world == 2 for w in survivors), 120), \
        [(w.group.world, w.group.epoch, w.state) for w in survivors]
    assert cluster.wait_for(lambda: all(w.step > s + 20 for w, s in zip(survivors, steps)), 120)


def test_rpc_latency_histograms_and_step_phase_feedback(cluster):
    """every role times the RPCs it serves and makes
    (method, side, status code) into sl_rpc_seconds; the workers report a step-time breakdown
    (wall step, loop waits, one probed step's compute / exchange / update and the exchange's
    GB/s) through the additive FlowFeedback fields, and the master aggregates it per job."""
    a = cluster.add_worker(sync="allreduce", batch=256, log_every=10)
    b = cluster.add_worker(sync="allreduce", batch=256, log_every=10)
    m = cluster.master
    assert cluster.wait_for(lambda: all(m.feedback.get(w.addr, {}).get("exchange_ms", 0) > 0
                                        and m.feedback[w.addr].get("step_ms", 0) > 0 for w in (a, b)), 120), \
        m.feedback
    fb = m.feedback[a.addr]
    assert fb["compute_ms"] > 0 and fb["update_ms"] > 0 and fb["exchange_gbps"] > 0
    job = m.job_metrics()
    assert job["phases"]["max_step_ms"] >= job["phases"]["step_ms"] > 0
    assert job["phases"]["exchange_ms"] > 0
    # server and client sides of the same RPCs, with their status codes
    assert m.metrics.rpc_count("client", "Worker/CheckUp") > 0
    assert a.metrics.rpc_count("server", "Worker/CheckUp") > 0
    assert a.metrics.rpc_count("server", "Worker/ReceiveFile") > 0
    assert m.metrics.rpc_count("server", "Master/RegisterBirth") > 0
    assert cluster.file_server.metrics.rpc_count("client", "Worker/ReceiveFile") > 0
    assert cluster.file_server.metrics.rpc_count("server", "FileServer/DoPush") > 0
    text = m.metrics.text()
    assert 'sl_rpc_seconds_bucket{code="OK",le="0.001",method="Worker/CheckUp",role="master",side="client"}' in text
    assert "sl_step_phase_ms" in a.metrics.text() and "sl_exchange_gbps" in a.metrics.text()
    # a failing call is recorded with its code: CheckUp of an address nobody serves
    from serverless_learn_amd.runtime.transport import RpcFailure
    from serverless_learn_amd.proto import messages as pb

    with pytest.raises(RpcFailure):
        m.channels.unary("127.0.0.1:1", "Worker", "CheckUp", pb.PeerList().SerializeToString(), timeout=0.3)
    assert m.metrics.rpc_count("client", "Worker/CheckUp", "UNAVAILABLE") + \
        m.metrics.rpc_count("client", "Worker/CheckUp", "DEADLINE_EXCEEDED") >= 1


def test_gossip_workers_exchange(cluster):
    a = cluster.add_worker(sync="gossip")
    b = cluster.add_worker(sync="gossip")
    assert cluster.wait_for(lambda: a.gossip is not None and b.gossip is not None
                            and a.gossip.exchanges + b.gossip.exchanges >= 6, 60)
    assert a.step > 0 and b.step > 0


def test_checkpoint_then_new_worker_resumes(cluster):
    a = cluster.add_worker(sync="none", checkpoint_every=25)
    assert cluster.wait_for(lambda: cluster.master.latest_ckpt != 0 and a.step >= 50, 60)
    b = cluster.add_worker(sync="none")
    assert cluster.wait_for(lambda: b.step >= 25, 60)
    from serverless_learn_amd.ckpt.format import CKPT_BASE

    assert any(f >= CKPT_BASE for f in b.files_received)


def test_resnet_worker_trains_on_cifar_shards():
    """BASELINE config 4 plumbing on CPU: the CNN trains from pushed CIFAR-shaped shards."""
    c = LocalCluster(fast_config(dataset="synthetic-cifar", shard_records=64))
    try:
        w = c.add_worker(sync="none", model="resnet18", batch=8, max_steps=3, lr=0.01)
        assert c.wait_for(lambda: w.state == "done", 120), (w.state, w.step)
        assert w.trainer.model_name == "resnet18-cifar"
        assert w.trainer.x.shape[1:] == (32, 32, 3)
        assert np.isfinite(w.trainer.stats().loss)
        fn = w.save_checkpoint()
        from serverless_learn_amd.ckpt.format import decode

        meta, params, _ = decode(c.file_server.get_file(fn))
        assert meta["model"] == "resnet18-cifar" and params.size == w.trainer.n_params
    finally:
        c.stop()


def test_elastic_kill_two_respawn_two_resume_from_checkpoint():
    """BASELINE config 5 (in-process, CPU): 4 all-reduce workers; 2 crash mid-run
    (no Deregister); the survivors regroup; 2 fresh workers join, receive the
    file server's checkpoint, get rank 0's state on regroup and train in lock-step."""
    from serverless_learn_amd.ckpt.format import CKPT_BASE

    c = LocalCluster(fast_config(checkpoint_every=15))
    try:
        ws = [c.add_worker(sync="allreduce", batch=128) for _ in range(4)]
        assert c.wait_for(lambda: all(w.group.world == 4 and w.step > 30 for w in ws), 90), \
            [(w.group.world, w.step) for w in ws]
        assert c.wait_for(lambda: c.master.latest_ckpt >= CKPT_BASE, 30)
        epoch0 = c.master.registry.epoch()
        for v in ws[2:]:  # crash: stop training and serving, never deregister
            v._stop.set()
            v.server.stop(grace=0)
        survivors = ws[:2]
        assert c.wait_for(lambda: c.master.registry.epoch() > epoch0 and
                          all(w.group.world == 2 for w in survivors), 60), \
            [(w.group.world, w.group.epoch) for w in survivors]
        s0 = [w.step for w in survivors]
        assert c.wait_for(lambda: all(w.step > s + 10 for w, s in zip(survivors, s0)), 60)
        fresh = [c.add_worker(sync="allreduce", batch=128) for _ in range(2)]
        group = survivors + fresh
        assert c.wait_for(lambda: all(w.group.world == 4 for w in group) and
                          all(w.step > 10 for w in fresh), 90), \
            [(w.group.world, w.step, w.state) for w in group]
        assert all(any(f >= CKPT_BASE for f in w.files_received) for w in fresh), \
            [w.files_received for w in fresh]
        # lock-step replicas: stop all four at the same step and compare
        target = max(w.step for w in group) + 15
        for w in group:
            w.cfg.max_steps = target
        assert c.wait_for(lambda: all(w.state == "done" for w in group), 90), [(w.step, w.state) for w in group]
        steps = {w.step for w in group}
        assert steps == {target}, steps
        params = [w.trainer.params for w in group]
        assert all(torch.equal(params[0], p) for p in params[1:])
        assert min(steps) > max(s0), (steps, s0)  # resumed, not restarted from 0
    finally:
        c.stop()


def test_ps_workers_exchange_through_master(cluster):
    a = cluster.add_worker(sync="ps")
    b = cluster.add_worker(sync="ps")
    assert cluster.wait_for(lambda: cluster.master.ps.exchanges >= 6 and a.step > 0 and b.step > 0, 60)
    # the PS tracks each worker's exchanges separately (named by metadata, not the TCP peer)
    assert {a.addr, b.addr} <= set(cluster.master.ps.olds)
    assert cluster.master.ps.model.size == a.trainer.n_params


def test_evicted_worker_registers_again(cluster, monkeypatch):
    monkeypatch.setenv("SL_FAULT", "drop:CheckUp:p=0")
    w = cluster.add_worker(sync="none")
    assert cluster.wait_for(lambda: w.addr in cluster.master.registry.members() and w.step > 0, 30)
    epoch = cluster.master.registry.epoch()
    w.fault.drop["CheckUp"] = 1.0  # heartbeats fail (a network blip): the master evicts it
    assert cluster.wait_for(lambda: w.addr not in cluster.master.registry.members(), 30)
    w.fault.drop["CheckUp"] = 0.0
    assert cluster.wait_for(lambda: w.addr in cluster.master.registry.members(), 30)
    assert cluster.master.registry.epoch() > epoch + 1


def test_allreduce_member_whose_shard_arrives_late_stays_in_lockstep(cluster, monkeypatch):
    """The group forms before one member has any data: its trainer is built for the
    state broadcast, the gradient hook is installed, and both replicas stay identical."""
    a = cluster.add_worker(sync="allreduce", batch=512, max_steps=60)
    monkeypatch.setenv("SL_FAULT", "delay:ReceiveFile:ms=1500")
    b = cluster.add_worker(sync="allreduce", batch=512, max_steps=60)
    monkeypatch.delenv("SL_FAULT")
    assert cluster.wait_for(lambda: a.state == "done" and b.state == "done", 120), (a.step, b.step, a.state, b.state)
    assert a.trainer.allreduce is not None and b.trainer.allreduce is not None
    assert torch.equal(a.trainer.params, b.trainer.params)


def test_master_ps_broadcast_loop():
    """The reference's never-started periodically_send_updates (master.cc:268-293), enabled."""
    c = LocalCluster(fast_config(ps_broadcast_interval_ms=150))
    try:
        a = c.add_worker(sync="ps")
        b = c.add_worker(sync="ps")
        assert c.wait_for(lambda: c.master.ps_broadcasts >= 3 and a.gossip is not None and b.gossip is not None
                          and a.gossip.serves + b.gossip.serves >= 3, 60), \
            (c.master.ps_broadcasts, a.gossip and a.gossip.serves, b.gossip and b.gossip.serves)
        assert {a.addr, b.addr} & set(c.master.ps.olds)
    finally:
        c.stop()


def test_group_metrics_are_allreduced_and_master_reports_job_rate(cluster):
    """N3: every member of an all-reduce group reports the SAME group samples/s / loss (an
    all-reduce over the group every log_every steps) in FlowFeedback; the master counts each
    group once in its whole-job rate and exports it as a Prometheus gauge."""
    a = cluster.add_worker(sync="allreduce", batch=256)
    b = cluster.add_worker(sync="allreduce", batch=256)
    assert cluster.wait_for(lambda: a.group_metrics["world"] == 2 and b.group_metrics["world"] == 2
                            and a.step >= 60, 120), (a.group_metrics, b.group_metrics)

    def agree():
        f = cluster.master.feedback
        if a.addr not in f or b.addr not in f:
            return False
        x, y = f[a.addr], f[b.addr]
        return (x["group_world"] == 2 and y["group_world"] == 2
                and x["group_samples_per_sec"] == y["group_samples_per_sec"] > 0)
    assert cluster.wait_for(agree, 30), cluster.master.feedback
    job = cluster.master.job_metrics()
    f = cluster.master.feedback
    assert job["groups"] == 1
    assert job["samples_per_sec"] == pytest.approx(f[a.addr]["group_samples_per_sec"], rel=1e-3)
    assert cluster.wait_for(lambda: "sl_job_samples_per_second" in cluster.master.metrics.text(), 15)


def test_join_switches_epoch_at_an_agreed_step_without_failed_collectives(cluster):
    """A worker joining a training all-reduce group: the members see the new epoch from their
    CheckUps at different times, but switch together at a step boundary the whole group agreed
    on (Worker._agree), so no member runs a collective on the old group alone -- no
    collective_failed -- and all three then train in lock-step with identical weights."""
    a = cluster.add_worker(sync="allreduce", batch=256)
    b = cluster.add_worker(sync="allreduce", batch=256)
    assert cluster.wait_for(lambda: a.group.world == 2 and b.group.world == 2 and a.step > 30, 60)
    fails = []
    for w in (a, b):
        orig = w.log.warn

        def spy(event, _orig=orig, **f):
            if event == "collective_failed":
                fails.append(f)
            return _orig(event, **f)
        w.log.warn = spy
    c = cluster.add_worker(sync="allreduce", batch=256)
    ws = (a, b, c)
    assert cluster.wait_for(lambda: all(w.group.world == 3 for w in ws) and min(w.step for w in ws) > 0
                            and len({w.group.epoch for w in ws}) == 1, 60), \
        [(w.group.world, w.group.epoch, w.step, w.state) for w in ws]
    s0 = max(w.step for w in ws)
    assert cluster.wait_for(lambda: min(w.step for w in ws) > s0 + 20, 60)
    assert not fails, fails
    # lock-step replicas: stop the group at a boundary and compare
    for w in ws:
        w.cfg.max_steps = max(x.step for x in ws) + 40
    assert cluster.wait_for(lambda: all(w.state == "done" for w in ws), 60), [(w.step, w.state) for w in ws]
    assert a.step == b.step == c.step
    assert torch.equal(a.trainer.params, b.trainer.params) and torch.equal(a.trainer.params, c.trainer.params)
