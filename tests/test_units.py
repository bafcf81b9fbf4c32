"""CPU unit tests of the pure-Python pieces: gossip math,
checkpoint format (§5.4), fault-injection rules and tracing (§5.1/§5.3), and
config defaults (§5.6 -- every default equals the reference constant)."""
import json

import numpy as np
import pytest
import torch

from serverless_learn_amd.ckpt import format as ckpt
from serverless_learn_amd.config import Config
from serverless_learn_amd.parallel.gossip import GossipState, exact_exchange
from serverless_learn_amd.utils.fault import FaultInjector


def _pair(rng, n):
    mA, oA, mB, oB = (rng.standard_normal(n) for _ in range(4))
    return mA, oA, mB, oB


@pytest.mark.parametrize("compat", [True, False])
def test_gossip_exchange_matches_closed_form(compat):
    rng = np.random.default_rng(0)
    mA, oA, mB, oB = _pair(rng, 37)
    A = GossipState(torch.from_numpy(mA.copy()), alpha=0.5, compat=compat)
    A.old = torch.from_numpy(oA.copy())
    B = GossipState(torch.from_numpy(mB.copy()), alpha=0.5, compat=compat)
    B.old = torch.from_numpy(oB.copy())
    d = A.make_delta()
    r = B.serve(d)
    A.absorb(r, d)
    mA2, oA2, mB2, oB2, r_ref = exact_exchange(mA, oA, mB, oB, 0.5, compat=compat)
    np.testing.assert_allclose(r, r_ref, rtol=0, atol=1e-12)
    np.testing.assert_allclose(B.model.numpy(), mB2, atol=1e-12)
    np.testing.assert_allclose(B.old.numpy(), oB2, atol=1e-12)
    np.testing.assert_allclose(A.model.numpy(), mA2, atol=1e-12)
    np.testing.assert_allclose(A.old.numpy(), oA2, atol=1e-12)


def test_gossip_compat_has_alpha_squared_echo():
    # only A made progress: dA = 1, dB = 0 -> compat A ends at mA + a^2 dA, echo-free at mA
    mA, oA = np.ones(4), np.zeros(4)
    mB, oB = np.zeros(4), np.zeros(4)
    c = exact_exchange(mA, oA, mB, oB, 0.5, compat=True)[0]
    e = exact_exchange(mA, oA, mB, oB, 0.5, compat=False)[0]
    np.testing.assert_allclose(c, 1.25)
    np.testing.assert_allclose(e, 1.0)


def test_gossip_growable_vector_grows_with_zeros():
    # reference worker.cc:85-89: a shorter model grows to the incoming length
    B = GossipState(torch.zeros(2, dtype=torch.float64), growable=True)
    r = B.serve(np.array([2.0, 2.0, 2.0, 2.0]))
    np.testing.assert_allclose(r, [1.0, 1.0, 1.0, 1.0])
    assert B.model.numel() == 4
    fixed = GossipState(torch.zeros(2, dtype=torch.float64))
    with pytest.raises(ValueError):
        fixed.serve(np.ones(3))


def test_checkpoint_roundtrip_and_update_compat():
    from serverless_learn_amd.wire.codec import decode_update

    rng = np.random.default_rng(1)
    p = rng.standard_normal(1000).astype(np.float32)
    m = rng.standard_normal(1000).astype(np.float32)
    buf = ckpt.encode(p, {"model": "mlp", "step": 7, "epoch": 3}, momentum=m)
    assert ckpt.looks_like_checkpoint(buf)
    meta, p2, m2 = ckpt.decode(buf)
    assert meta["step"] == 7 and meta["epoch"] == 3 and meta["n_params"] == 1000
    np.testing.assert_array_equal(p2, p)
    np.testing.assert_array_equal(m2, m)
    # the parameter section is a plain serialized Update{repeated double delta}
    mlen = int.from_bytes(buf[12:16], "little")
    pos = 16 + mlen
    n = int.from_bytes(buf[pos:pos + 8], "little")
    np.testing.assert_array_equal(decode_update(bytes(buf[pos + 8:pos + 8 + n]), "float32"), p)
    meta, p3, m3 = ckpt.decode(ckpt.encode(p, {"model": "mlp"}))
    assert m3 is None
    with pytest.raises(ValueError):
        ckpt.decode(b"NOTACKPT" + bytes(8))
    assert ckpt.is_checkpoint_file(ckpt.CKPT_BASE) and not ckpt.is_checkpoint_file(0)


def test_fault_rules_parse_and_wrap():
    fi = FaultInjector("kill:step=5; drop:CheckUp:p=1; delay:ExchangeUpdates:ms=1; hang:ReceiveFile")
    assert fi.kill_step == 5 and fi.active
    assert fi.drop == {"CheckUp": 1.0} and fi.delay == {"ExchangeUpdates": 0.001}
    assert fi.hang == {"ReceiveFile"}
    f = lambda req, ctx: "ok"  # noqa: E731
    assert fi.wrap("RegisterBirth", f) is f

    class Ctx:
        def abort(self, code, msg):
            raise RuntimeError(msg)

    with pytest.raises(RuntimeError):
        fi.wrap("CheckUp", f)(None, Ctx())
    assert fi.wrap("ExchangeUpdates", f)(None, Ctx()) == "ok"
    with pytest.raises(ValueError):
        FaultInjector("explode:now")
    assert not FaultInjector("").active


def test_trace_spans_to_chrome_json(tmp_path, monkeypatch):
    from serverless_learn_amd.utils import trace

    monkeypatch.setattr(trace, "_path", str(tmp_path / "t.json"))
    monkeypatch.setattr(trace, "_events", [])
    with trace.span("step", step=1):
        pass
    trace.counter("samples_per_s", v=1.0)
    trace.flush()
    ev = json.load(open(tmp_path / "t.json"))["traceEvents"]
    assert [e["ph"] for e in ev] == ["X", "C"] and ev[0]["name"] == "step" and ev[0]["args"] == {"step": 1}


def test_config_defaults_equal_reference_constants(monkeypatch):
    for k in list(__import__("os").environ):
        if k.startswith("SL_"):
            monkeypatch.delenv(k)
    c = Config.from_env()
    assert c.master_addr == "localhost:50052"            # serverless_learn.h:5
    assert c.file_server_addr == "localhost:50053"       # serverless_learn.h:8
    assert c.gossip_interval_ms == 5000                  # serverless_learn.h:10
    assert c.simulated_train_interval_ms == 2000         # serverless_learn.h:12
    assert c.push_interval_ms == 5000 and c.checkup_interval_ms == 5000  # master.cc:43,46
    assert c.learn_rate == 0.5                           # master.cc:60
    assert c.chunk_size == 1_000_000 and c.dummy_file_length == 100_000_000  # file_server.cc:40,46
    monkeypatch.setenv("SL_GOSSIP_INTERVAL_MS", "250")
    monkeypatch.setenv("SL_GOSSIP_COMPAT", "true")
    c = Config.from_env()
    assert c.gossip_interval == 0.25 and c.gossip_compat is True


def test_metrics_from_log_events_and_http_exposition():
    import urllib.request

    from serverless_learn_amd.utils.log import Logger
    from serverless_learn_amd.utils.metrics import Metrics

    m = Metrics("worker")
    log = Logger("worker", "127.0.0.1:1", m)
    log.info("train", step=50, loss=0.25, acc=0.9, samples_per_sec=1.5e6, epoch=3)
    log.info("received_file", file_num=0, kind="shard", bytes=1000, s=0.01)
    log.warn("collective_failed", error="x")
    log.debug("below_level")  # filtered from the log, still counted
    txt = m.text()
    assert 'sl_step{role="worker"} 50.0' in txt
    assert 'sl_loss{role="worker"} 0.25' in txt
    assert 'sl_membership_epoch{role="worker"} 3.0' in txt
    assert 'sl_ingested_bytes_total{role="worker"} 1000.0' in txt
    assert 'sl_events_total{event="collective_failed",level="warn",role="worker"} 1.0' in txt
    assert 'event="below_level"' in txt
    port = m.serve(0, addr="127.0.0.1")
    try:
        body = urllib.request.urlopen(f"http://127.0.0.1:{port}/metrics", timeout=5).read().decode()
        assert 'sl_samples_per_second{role="worker"} 1.5e+06' in body
    finally:
        m.close()


def test_gossip_absorb_keeps_progress_made_during_the_rpc():
    """Steps taken while the exchange is in flight stay unshared (sent next time), not lost."""
    A = GossipState(torch.zeros(6, dtype=torch.float64), alpha=0.5)
    B = GossipState(torch.zeros(6, dtype=torch.float64), alpha=0.5)
    A.model += 1.0                    # progress before the exchange
    d = A.make_delta()
    A.model += 10.0                   # a training step lands while the RPC is in flight
    r = B.serve(d)
    A.absorb(r, d)
    # the in-flight step is still pending in A's next delta
    np.testing.assert_allclose(A.make_delta(), 10.0)
    # the classic o = m rule would have dropped it: A.model - A.old would be 0
    np.testing.assert_allclose(A.model.numpy(), 11.0)


def test_gossip_absorb_after_an_intervening_serve():
    """A serve that lands during the client's RPC resets o = m; absorb must not re-add `sent`."""
    A = GossipState(torch.zeros(3, dtype=torch.float64), alpha=0.5)
    B = GossipState(torch.zeros(3, dtype=torch.float64), alpha=0.5)
    C = GossipState(torch.zeros(3, dtype=torch.float64), alpha=0.5)
    A.model += 2.0
    d = A.make_delta()
    rC = A.serve(C.make_delta())      # C exchanges with A while A's own RPC to B is in flight
    np.testing.assert_allclose(rC, 2.0)  # A's progress went to C in that reply
    r = B.serve(d)
    A.absorb(r, d)
    np.testing.assert_allclose(A.make_delta(), 0.0)   # nothing double-counted, nothing pending
    np.testing.assert_allclose(A.old.numpy(), A.model.numpy())


def test_ps_per_client_mixes_models_between_workers():
    """sync=ps: two workers learn each other's progress through the master's PS."""
    from serverless_learn_amd.parallel.ps import ParameterServer

    for alpha, share in ((1.0, 1.0), (0.5, 0.25)):
        ps = ParameterServer(alpha)
        A = GossipState(torch.zeros(4, dtype=torch.float64), alpha=alpha)
        B = GossipState(torch.zeros(4, dtype=torch.float64), alpha=alpha)
        A.model += 3.0
        B.model -= 5.0
        for _ in range(2):
            for name, w in (("A", A), ("B", B)):
                d = w.make_delta()
                w.absorb(ps.exchange(d, name), d)
        # each keeps its own progress and gains alpha^2 (PS alpha, client alpha) of the other's
        np.testing.assert_allclose(A.model.numpy(), 3.0 + share * -5.0)
        np.testing.assert_allclose(B.model.numpy(), -5.0 + share * 3.0)
        np.testing.assert_allclose(ps.model, alpha * (3.0 - 5.0))


def test_ps_reference_single_old_echoes_the_callers_delta():
    """The reference rule (one old_state, master.cc:95-114): every reply is alpha*d."""
    from serverless_learn_amd.parallel.ps import ParameterServer

    ps = ParameterServer(0.5, per_client=False)
    np.testing.assert_allclose(ps.exchange(np.full(3, 4.0), "A"), 2.0)
    np.testing.assert_allclose(ps.exchange(np.full(3, -2.0), "B"), -1.0)


@pytest.mark.parametrize("world", [2, 3, 5, 8, 16])
def test_xgmi_two_shot_chunks_cover_payload_and_sum_like_one_shot(world):
    """Two-shot partition (csrc/kernels/xgmi.h): wave-aligned chunks that cover the slot, one
    owner per float4, and per-chunk rank-order sums equal to the one-shot rank-order sum."""
    from serverless_learn_amd.models.mlp import N_PARAMS
    from serverless_learn_amd.parallel.xgmi import two_shot_chunk4

    n = (N_PARAMS + 3) // 4 * 4
    slot_bytes = (n * 4 + 255) // 256 * 256
    c4 = two_shot_chunk4(slot_bytes, world)
    assert c4 % 64 == 0 and c4 * world * 16 >= slot_bytes
    owners = np.arange(slot_bytes // 16) // c4
    assert owners.max() < world
    # the kernel's wave-uniform owner: every aligned group of 64 float4 has one owner
    waves = np.arange(-(-owners.size // 64) * 64) // c4
    assert (waves.reshape(-1, 64).min(1) == waves.reshape(-1, 64).max(1)).all()
    rng = np.random.default_rng(world)
    parts = [rng.standard_normal(n).astype(np.float32) for _ in range(world)]
    one = parts[0].copy()
    for q in range(1, world):
        one += parts[q]
    two = np.empty(n, dtype=np.float32)
    for r in range(world):  # rank r reduces its chunk, in rank order
        lo, hi = r * c4 * 4, min(n, (r + 1) * c4 * 4)
        if lo >= hi:
            continue
        acc = parts[0][lo:hi].copy()
        for q in range(1, world):
            acc += parts[q][lo:hi]
        two[lo:hi] = acc
    assert np.array_equal(one, two)


def test_mlp_dw1_fp16_coefficients_reproduce_normalised_gradient():
    """The fp16 dW1 GEMM multiplies scale * dH1 by 1024 + u; the SGD coefficients must give
    back xa dH1^T X + xb db1 for the normalised input xa X + xb."""
    from serverless_learn_amd.models.mlp import dh1_scale, dw1_coeffs, norm_coeffs

    rng = np.random.default_rng(0)
    rows, feats, k = 512, 16, 24
    gs = 1.0 / (65536 * 8)
    dh = (rng.standard_normal((rows, feats)) * gs).astype(np.float64)
    x = rng.integers(0, 256, (rows, k)).astype(np.float64)
    xa, xb = norm_coeffs()
    s = dh1_scale(gs)
    assert s == 2.0 ** 19 and 0.25 < np.abs(dh * s).max() < 16  # O(1) in fp16
    slab = (dh * s).T @ (x + 1024.0)
    db1 = dh.sum(0)
    a, b = dw1_coeffs(xa, xb, s)
    got = a * slab + b * db1[:, None]
    want = xa * dh.T @ x + xb * db1[:, None]
    np.testing.assert_allclose(got, want, rtol=1e-9, atol=1e-18)
    ref = dh.T @ (xa * x + xb)  # the gradient w.r.t. W1 of the normalised input
    np.testing.assert_allclose(got, ref, rtol=1e-9, atol=1e-18)


def test_runtime_bench_times_exactly_k_worker_steps():
    """bench.py --runtime: the worker pauses exactly at W (hold_at), then at W + K once its
    device work drained; the roles ran end-to-end (shard over gRPC, master registration)."""
    import bench

    args = bench.parse(["--runtime", "--batch", "64", "--steps", "24", "--warmup", "5"])
    elapsed, info, tr = bench.runtime_bench(args, torch.device("cpu"))
    assert elapsed > 0
    assert info["roles"] == ["file_server", "master", "worker"]
    assert info["bytes_ingested"] > 64 * 784
    assert tr.cursor == 5 + 24  # CPU trainer: one batch per step, none skipped or repeated
    assert bench.main(["--runtime", "--gpus", "2"]) == 2


def test_bench_refuses_more_gpus_than_visible():
    """``bench.py --gpus 8`` on a machine with fewer devices exits non-zero and prints no
    JSON line: it never reports an N-GPU number measured on fewer GPUs (here: 0 visible)."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "8", "--steps", "2"],
                       cwd=root, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=120, env=env)
    assert p.returncode != 0
    assert '"metric"' not in p.stdout
    assert "refusing" in p.stderr
    # a torchrun-style rank whose WORLD_SIZE disagrees with --gpus is refused too
    env2 = dict(env, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "8"], cwd=root,
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=120, env=env2)
    assert p.returncode == 2 and '"metric"' not in p.stdout


def test_bench_replica_check_covers_every_path_and_refuses_persistent_divergence():
    """the N>1 replica check runs for every exchange path -- here the
    process group's (no xGMI exchange) -- and a divergence re-times with the uncaptured process
    group; replicas that still differ afterwards raise ReplicaDivergence, which bench.main turns
    into exit 2 with no JSON line.  Also: capturing multi-rank RCCL is opt-in."""
    import bench

    calls = []

    def retime():
        calls.append("retime")
        return 1.25

    # healthy: no re-time
    assert bench.verify_replicas(lambda: True, retime) == (True, None, None) and calls == []
    # process-group path, replicas diverged once: re-timed, the new time is reported
    seq = iter([False, True])
    assert bench.verify_replicas(lambda: next(seq), retime) == (True, "replicas diverged", 1.25)
    assert calls == ["retime"]
    # an xGMI barrier timeout with identical replicas still re-times
    assert bench.verify_replicas(lambda: True, retime, lambda: True)[1] == "barrier timeout"
    # persistent divergence: no number
    calls.clear()
    with pytest.raises(bench.ReplicaDivergence):
        bench.verify_replicas(lambda: False, retime)
    assert calls == ["retime"]
    # multi-rank RCCL capture is opt-in (flag or SL_GRAPH_COLLECTIVES=1)
    assert bench.parse([]).graph_collectives is False
    assert bench.parse(["--graph-collectives"]).graph_collectives is True


def test_ps_new_incarnation_restarts_old_and_anonymous_entries_are_bounded():
    from serverless_learn_amd.parallel.ps import ParameterServer

    ps = ParameterServer(alpha=0.5)
    ps.client_joined("w1", 1)
    ps.exchange(np.ones(4), "w1")
    ps.exchange(2 * np.ones(4), "w2")
    # w1 restarts at the same address: the new process has seen nothing of the PS model
    ps.client_joined("w1", 2)
    r = ps.exchange(np.zeros(4), "w1")
    np.testing.assert_allclose(r, ps.model)  # everything the PS holds is news to it
    # the same incarnation re-registering (eviction + re-join) keeps its history
    ps.client_joined("w1", 2)
    assert "w1" in ps.olds
    ps.max_anonymous = 4
    for i in range(20):
        ps.exchange(np.zeros(4), f"ipv4:127.0.0.1:{1000 + i}")
    assert sum(1 for k in ps.olds if k.startswith("ipv4")) <= 4
    ps.client_left("w1")
    assert "w1" not in ps.olds


def test_ps_broadcast_keeps_exchanges_that_land_in_flight():
    """absorb_reply advances o[target] by what was shared, so another client's exchange that
    lands while the broadcast RPC is in flight stays pending for the broadcast's target."""
    from serverless_learn_amd.parallel.ps import ParameterServer

    ps = ParameterServer(alpha=0.5)
    ps.set_model(np.zeros(3))
    ps.exchange(np.array([1.0, 0, 0]), "a")
    sent = ps.pending_delta("b")               # broadcast to b starts
    ps.exchange(np.array([0, 4.0, 0]), "c")     # lands while the RPC is in flight
    reply = 0.5 * sent                          # b had no progress of its own: pure echo
    ps.absorb_reply(reply, sent, "b")
    pending = ps.pending_delta("b")
    np.testing.assert_allclose(pending, [0, 2.0, 0])  # c's contribution is still news to b


def test_gossip_compat_absorb_sets_old_to_model():
    """compat mode keeps the reference's o = m after the client absorbs (worker.cc:215), even
    when training stepped while the exchange was in flight."""
    A = GossipState(torch.zeros(3, dtype=torch.float64), alpha=0.5, compat=True)
    A.model += 1.0
    d = A.make_delta()
    A.model += 1.0  # a step lands while the RPC is in flight
    A.absorb(np.full(3, 0.25), d)
    torch.testing.assert_close(A.old, A.model)
    B = GossipState(torch.zeros(3, dtype=torch.float64), alpha=0.5, compat=False)
    B.model += 1.0
    d = B.make_delta()
    B.model += 1.0
    B.absorb(np.full(3, 0.5), d)
    # echo-free: the in-flight step stays unshared
    torch.testing.assert_close(B.model - B.old, torch.ones(3, dtype=torch.float64))


def test_checkpoint_v2_extra_state_roundtrip_and_v1_compat():
    p = np.arange(10, dtype=np.float32)
    extra = {"cursor": np.array([7.0]), "bn/stem_bn/mean": np.linspace(0, 1, 5)}
    buf = ckpt.encode(p, {"model": "mlp", "step": 3}, momentum=p * 2, extra=extra)
    meta, p2, m2, ex = ckpt.decode_full(buf)
    assert meta["extra"] == sorted(extra) and int(ex["cursor"][0]) == 7
    np.testing.assert_array_equal(ex["bn/stem_bn/mean"], extra["bn/stem_bn/mean"])
    np.testing.assert_array_equal(p2, p) and np.testing.assert_array_equal(m2, p * 2)
    # every section is still a plain proto3 Update: the parameters parse with the reference message
    from serverless_learn_amd.proto import messages as pb
    import struct
    mlen = struct.unpack("<I", buf[12:16])[0]
    (n,) = struct.unpack("<Q", buf[16 + mlen:24 + mlen])
    assert list(pb.Update.FromString(buf[24 + mlen:24 + mlen + n]).delta) == list(map(float, p))
    # version-1 files (no extra sections) still decode
    v1 = bytearray(ckpt.encode(p, {"model": "mlp"}))
    v1[8:12] = struct.pack("<I", 1)
    v1 = bytes(v1[:-4])  # a v1 file ends after the momentum section
    meta, p3, m3, ex3 = ckpt.decode_full(v1)
    assert ex3 == {} and m3 is None


@pytest.mark.parametrize("model", ["mlp", "resnet18"])
def test_cpu_trainer_resume_is_exact(model):
    """CPU trainers: save after k steps (params, momentum, cursor, BN running stats), resume into a
    differently initialised trainer, run m steps -> identical to k + m uninterrupted steps."""
    from serverless_learn_amd.data.synthetic import make_cifar_like, make_mnist_like
    from serverless_learn_amd.models import make_trainer

    batch = 64 if model == "mlp" else 8
    x, y = (make_mnist_like if model == "mlp" else make_cifar_like)(3 * batch, seed=2)
    x, y = torch.from_numpy(x), torch.from_numpy(y)
    kw = dict(batch=batch, lr=0.05, momentum=0.9)
    a = make_trainer(model, torch.device("cpu"), seed=0, **kw)
    a.load_shard(x, y)
    for _ in range(2):
        a.step()
    buf = ckpt.encode(a.get_flat().numpy(), {"model": a.model_name}, a.mom.numpy(), a.state_extra())
    for _ in range(2):
        a.step()
    b = make_trainer(model, torch.device("cpu"), seed=5, **kw)
    b.load_shard(x, y)
    meta, params, mom, extra = ckpt.decode_full(buf)
    b.set_flat(torch.from_numpy(params))
    b.mom.copy_(torch.from_numpy(mom))
    b.load_state_extra(extra)
    for _ in range(2):
        b.step()
    assert torch.equal(a.get_flat(), b.get_flat()) and torch.equal(a.mom, b.mom)
    if model == "resnet18":
        for name, (rm, rv) in a.running.items():
            assert torch.allclose(rm, b.running[name][0], atol=1e-6) and torch.allclose(rv, b.running[name][1], atol=1e-6)
        st = b.evaluate(x[:batch], y[:batch])
        assert st.samples == batch and st.loss > 0


class _FakeGraphTrainer:
    """Counts steps; ``graph`` is dropped by ``load_shard`` like the fused engines'."""

    allreduce = None

    def __init__(self):
        self.graph = None
        self.ran = 0

    def step(self):
        self.ran += 1

    def steps(self, n):
        self.ran += n

    def capture(self, warmup=0, unroll=1):
        self.graph = object()

    def load_shard(self):
        self.graph = None


def test_worker_chunk_length_does_not_depend_on_graph_state(monkeypatch):
    """every chunk posts one group collective, so two lock-step members
    must cut chunks at the same steps.  A rank whose graph was just dropped (a shard landed
    on it mid-run) used to run a 1-step capture chunk while its peers ran 16."""
    from serverless_learn_amd.runtime.local_cluster import fast_config
    from serverless_learn_amd.runtime.worker import Worker

    cfg = fast_config(graph_steps=16)
    ws = [Worker("127.0.0.1:0", cfg) for _ in range(2)]
    for w in ws:
        w.trainer = _FakeGraphTrainer()
        monkeypatch.setattr(w, "_use_graph", lambda: True)
    cuts = [[], []]
    for i, w in enumerate(ws):
        step = 0
        while step < 100:
            if i == 1 and step in (16, 48):
                w.trainer.load_shard()  # only this rank re-captures
            want = min(100 - step, 10 - step % 10)  # a log boundary every 10 steps
            ran = w._run_chunk(want)
            assert w.trainer.ran == step + ran
            step += ran
            cuts[i].append(step)
    assert cuts[0] == cuts[1]
    # eager mode cuts the same chunks
    w = Worker("127.0.0.1:0", cfg)
    w.trainer = _FakeGraphTrainer()
    monkeypatch.setattr(w, "_use_graph", lambda: False)
    assert w._run_chunk(40) == 16 and w._run_chunk(3) == 3


def test_worker_chunk_failure_counts_completed_steps_and_releases_lock(monkeypatch):
    """an eager chunk takes train_lock per step (so RPC handlers wait at
    most one step), and a collective failing at step k of a chunk raises ChunkBroken carrying
    the k steps that completed, which the loop adds to the step / sample counters."""
    from serverless_learn_amd.parallel.dp import GroupBroken
    from serverless_learn_amd.runtime.local_cluster import fast_config
    from serverless_learn_amd.runtime.worker import ChunkBroken, Worker

    import threading

    w = Worker("127.0.0.1:0", fast_config(graph_steps=16))

    def lock_free() -> bool:  # train_lock is an RLock: probe it from another thread
        out = []

        def probe():
            got = w.train_lock.acquire(blocking=False)
            if got:
                w.train_lock.release()
            out.append(got)
        th = threading.Thread(target=probe)
        th.start()
        th.join()
        return out[0]

    class Failing(_FakeGraphTrainer):
        batch = 8

        def __init__(self, fail_at):
            super().__init__()
            self.fail_at = fail_at

        def step(self):
            assert not lock_free()  # the worker holds train_lock during a step
            if self.ran == self.fail_at:
                raise GroupBroken("peer died")
            self.ran += 1

    w.trainer = Failing(fail_at=5)
    monkeypatch.setattr(w, "_use_graph", lambda: False)
    with pytest.raises(ChunkBroken) as ei:
        w._run_chunk(10)
    assert ei.value.done == 5 and isinstance(ei.value, GroupBroken)
    assert lock_free()  # released after the failure
    w.step, w.samples = 100, 0
    w._account_steps(100, ei.value.done)
    assert (w.step, w.samples) == (105, 5 * 8)
    # graph mode: a failure in the capture step reports 0 completed steps
    t = Failing(fail_at=0)
    w.trainer = t
    monkeypatch.setattr(w, "_use_graph", lambda: True)
    with pytest.raises(ChunkBroken) as ei:
        w._run_chunk(10)
    assert ei.value.done == 0


def test_worker_drops_graphs_before_regroup_and_multirank_rccl_capture_is_opt_in():
    """a re-form frees BOTH captured graphs through drop_graphs (which
    syncs the device first); capturing a multi-rank RCCL group's collectives is opt-in."""
    from serverless_learn_amd.runtime.local_cluster import fast_config
    from serverless_learn_amd.runtime.worker import Worker

    w = Worker("127.0.0.1:0", fast_config())

    class T(_FakeGraphTrainer):
        dropped = 0

        def drop_graphs(self):
            T.dropped += 1
            self.graph = None
            self.graph_unrolled = None

    t = T()
    t.graph, t.graph_unrolled = object(), object()
    w.trainer = t
    w._drop_graphs()
    assert T.dropped == 1 and t.graph is None and t.graph_unrolled is None

    class G:
        active, backend, world = True, "nccl", 2

    w.group = G()
    w.device = torch.device("cuda", 0)
    t.allreduce = lambda g: None
    assert w._use_graph() is False
    w.cfg.graph_collectives = True
    assert w._use_graph() is True
    t.allreduce = None
    w.cfg.graph_collectives = False
    assert w._use_graph() is True  # no host-side collective in the step: always captured


def test_worker_aborts_communicator_before_draining_graphs_that_hold_collectives(monkeypatch):
    """a replayed graph can sit inside a collective whose peer died, and
    the watchdog does not see it, so draining the device first would hang the regroup.  When
    the group is broken, or when the captured graphs hold collectives, _drop_graphs aborts the
    communicator (teardown) BEFORE the device drain; graphs of kernels only drain with the
    group untouched."""
    from serverless_learn_amd.runtime.local_cluster import fast_config
    from serverless_learn_amd.runtime.worker import Worker

    events = []

    class T(_FakeGraphTrainer):
        def drop_graphs(self):
            events.append("drain")  # FusedMLPTrainer.drop_graphs syncs the device here
            self.graph = self.graph_unrolled = None

    class G:
        backend, world = "nccl", 2

        def __init__(self, broken):
            self.broken, self.pg = broken, object()

        @property
        def active(self):
            return self.pg is not None

        def teardown(self):
            events.append("abort")
            self.pg = None

    w = Worker("127.0.0.1:0", fast_config(graph_steps=4))
    monkeypatch.setattr(w, "_use_graph", lambda: True)
    for broken, collectives, want in ((True, False, ["abort", "drain"]), (False, True, ["abort", "drain"]),
                                      (False, False, ["drain"])):
        events.clear()
        t = T()
        t.allreduce = (lambda g: None) if collectives else None
        w.trainer, w.group = t, G(broken)
        w._run_chunk(4)  # eager first step + capture: records whether the graphs hold collectives
        assert w._graph_collectives is collectives
        w._drop_graphs()
        assert events == want, (broken, collectives, events)
        assert not w._graph_collectives


def test_allreduce_async_enqueue_failure_is_group_broken():
    """an enqueue that fails on an aborted communicator must surface as
    GroupBroken (which the training loop handles by re-forming) on both the sum path and
    the op path."""
    from serverless_learn_amd.parallel.dp import ElasticGroup, GroupBroken

    class DeadPG:
        def allreduce(self, *a):
            raise RuntimeError("communicator aborted")

    for op in (None, torch.distributed.ReduceOp.MAX):
        g = ElasticGroup(backend="gloo")
        g.pg = DeadPG()
        with pytest.raises(GroupBroken):
            g.allreduce_async(torch.zeros(2), op)
        assert g.broken


def test_share_gpu_env_caps_hardware_queues_only_when_processes_share_a_gpu():
    """Several processes on one GPU: GPU_MAX_HW_QUEUES is capped so their queues stay within the
    GPU's budget (4+ processes at HIP's 4 each were time-sliced, profiles/r06_ranks); one or two
    processes keep the default, and a lower value already set is kept."""
    from serverless_learn_amd.utils.gpu_share import QUEUE_BUDGET, share_gpu_env

    assert share_gpu_env({}, 1) == {}
    assert share_gpu_env({"GPU_MAX_HW_QUEUES": "4"}, 2) == {"GPU_MAX_HW_QUEUES": "4"}
    assert share_gpu_env({"GPU_MAX_HW_QUEUES": "4"}, 4) == {"GPU_MAX_HW_QUEUES": "2"}
    assert share_gpu_env({}, 8) == {"GPU_MAX_HW_QUEUES": "1"}
    assert share_gpu_env({"GPU_MAX_HW_QUEUES": "1"}, 3) == {"GPU_MAX_HW_QUEUES": "1"}
    for n in range(3, 17):
        assert n * int(share_gpu_env({}, n)["GPU_MAX_HW_QUEUES"]) <= max(QUEUE_BUDGET, n)


def test_reserve_port_stays_below_the_ephemeral_range_and_binds():
    """Ports handed to processes that bind them later come from below the kernel's ephemeral
    range (outgoing connections never take them) and are distinct within a process."""
    import socket

    from serverless_learn_amd.utils.ports import _ephemeral_low, reserve_port

    ports = [reserve_port() for _ in range(32)]
    assert len(set(ports)) == len(ports)
    assert all(10000 <= p < max(10001, _ephemeral_low()) for p in ports)
    s = socket.socket()
    s.bind(("127.0.0.1", ports[0]))
    s.close()


def test_rendezvous_round_abandoned_by_rank0_is_left_by_a_late_rank():
    """A rank arriving just as rank 0 gives up on a round (its check-in wait timed out) must
    not wait out a whole timeout in that dead round: it checks in to the round rank 0 opens
    next, and both build the group there (the r06_full7 elastic GPU failure: rank 1 joined
    round 1 as rank 0 abandoned it, and each then waited 20 s for the other)."""
    import datetime
    import threading
    import time

    import torch.distributed as dist

    from serverless_learn_amd.parallel.dp import ElasticGroup, GroupCancelled
    from serverless_learn_amd.utils.ports import reserve_port

    port = reserve_port()
    master = dist.TCPStore("127.0.0.1", port, is_master=True, wait_for_workers=False,
                           timeout=datetime.timedelta(seconds=30))
    rdv = f"127.0.0.1:{port}"
    g0, g1 = ElasticGroup(backend="gloo", timeout_s=0.6), ElasticGroup(backend="gloo", timeout_s=10)
    ep0 = dist.PrefixStore("sl/e5", g0._store(rdv))
    ep1 = dist.PrefixStore("sl/e5", g1._store(rdv))
    with pytest.raises(TimeoutError):
        g0._open_round(ep0, 5, 0, 2)  # nobody checks in to round 1: rank 0 abandons it
    got = {}
    t1 = threading.Thread(target=lambda: got.setdefault("r1", g1._open_round(ep1, 5, 1, 2)))
    t1.start()  # rank 1 sees round 1 (the abandoned one) and checks in there
    time.sleep(0.3)
    assert int(ep0.add("in1", 0)) == 1 and "r1" not in got
    t0 = time.monotonic()
    assert g0._open_round(ep0, 5, 0, 2) == 2  # rank 0's retry: rank 1 moves over at once
    t1.join(5)
    assert got.get("r1") == 2 and time.monotonic() - t0 < 2.0

    # end to end: both ranks build a gloo group after the abandoned round
    gg = [ElasticGroup(backend="gloo", timeout_s=10) for _ in range(2)]
    ok = {}
    ths = [threading.Thread(target=lambda r=r: ok.setdefault(r, gg[r].reform(6, r, 2, rdv))) for r in range(2)]
    for th in ths:
        th.start()
    for th in ths:
        th.join(30)
    assert ok == {0: True, 1: True}
    x = torch.tensor([float(1)])
    y = torch.tensor([float(2)])
    ws = [threading.Thread(target=gg[0].allreduce_, args=(x,)), threading.Thread(target=gg[1].allreduce_, args=(y,))]
    for w in ws:
        w.start()
    for w in ws:
        w.join(30)
    assert float(x) == float(y) == 3.0

    # a rendezvous for a membership that is no longer current ends as soon as that is seen
    g2 = ElasticGroup(backend="gloo", timeout_s=20)
    flag = {"stale": False}
    threading.Timer(0.2, lambda: flag.update(stale=True)).start()
    t0 = time.monotonic()
    assert not g2.reform(7, 0, 2, rdv, cancelled=lambda: flag["stale"])
    assert time.monotonic() - t0 < 2.0 and g2.broken
    with pytest.raises(GroupCancelled):
        g2._open_round(dist.PrefixStore("sl/e8", g2._store(rdv)), 8, 1, 2, cancelled=lambda: True)
    del master


def test_replaced_step_graphs_are_retired_until_a_sync_reaps_them():
    """A trainer's replaced graph is kept alive (its destructor would wait for in-flight
    launches with the GIL held, r06_full7) until ``reap_graphs`` -- after a device sync, or
    in ``drop_graphs`` / ``capture`` -- frees it."""
    import gc
    import weakref

    from serverless_learn_amd.utils.graphs import GraphSlots

    class G:
        pass

    class T(GraphSlots):
        device = torch.device("cpu")

    t = T()
    assert t.graph is None and t.graph_unrolled is None and t.retired_graphs == 0
    a, b, k = G(), G(), G()
    ra, rk = weakref.ref(a), weakref.ref(k)
    t.graph, t.graph_unrolled = a, k
    t.graph = a  # same object: nothing retired
    assert t.retired_graphs == 0
    del a, k
    t.graph = None
    t.graph_unrolled = None
    t.graph = b
    gc.collect()
    assert ra() is not None and rk() is not None and t.retired_graphs == 2
    t.reap_graphs()
    gc.collect()
    assert ra() is None and rk() is None and t.retired_graphs == 0 and t.graph is b


def test_regroup_forms_the_view_current_after_its_drains(monkeypatch):
    """The drains before a re-form (leaving the exchange, dropping graphs) can take up to the
    exchange's dead-peer timeout.  The worker must then form the view current at that moment:
    a newer epoch if one arrived, nothing while it re-registers (epoch 0), and the epoch read
    before the drains when it is still current (r06_full7: w0 formed a stale epoch 4 for 20 s)."""
    from serverless_learn_amd.runtime.local_cluster import fast_config
    from serverless_learn_amd.runtime.worker import Worker

    w = Worker("127.0.0.1:0", fast_config())
    calls = []

    class G:
        backend, world, epoch, rank = "gloo", 3, 3, 0
        broken, active = True, False

        def reform(self, epoch, rank, world, rdv, cancelled=None):
            calls.append((epoch, rank, world, cancelled()))
            return False

    def view(epoch, rank=0, world=2):
        return {"epoch": epoch, "peers": [], "rank": rank, "world": world, "rendezvous": "x:1", "resume_file": 0}

    for after, want in ((view(8, 1), [(8, 1, 2, False)]), (view(0, -1, 0), []), (view(4), [(4, 0, 2, False)])):
        calls.clear()
        w.group, w.view = G(), view(4)
        monkeypatch.setattr(w, "_drop_xgmi", lambda healthy=False, after=after: setattr(w, "view", after))
        monkeypatch.setattr(w, "_drop_graphs", lambda: None)
        monkeypatch.setattr(w._stop, "wait", lambda s=None: None)
        w._maybe_regroup()
        assert calls == want, (after["epoch"], calls)


def test_xgmi_probe_decision_is_group_wide_and_always_unmaps(monkeypatch):
    """parallel.xgmi.probe: every rank returns a failure when any rank's probe exchange fails
    (wrong sums, a barrier timeout, or a mapping error), each probe exchange is closed only
    after the group agreed, and a clean group returns "" (CPU: a fake exchange does the sums)."""
    from serverless_learn_amd.parallel import xgmi

    monkeypatch.setattr(torch.cuda, "synchronize", lambda *a, **k: None)
    events = []

    def fake(mode):
        class Ex:
            def __init__(self, n, rank, world, device, allgather, all_ok, two_shot=False):
                if mode == "map":
                    raise RuntimeError("xgmi exchange unavailable: hipIpcOpenMemHandle(rank 1) failed (1)")
                self.rank, self.world, self.two = rank, world, two_shot

            def allreduce_(self, t, scale=1.0):
                w = self.world
                t.copy_((t - self.rank - 1) * w + w * (w + 1) // 2)
                if mode == "sums" and self.two:
                    t[5] += 1

            def error(self):
                return mode == "timeout"

            def close(self, sync=True):
                events.append(("close", self.two))
        return Ex

    def all_ok_from(peer_ok):
        def all_ok(ok):
            events.append(("agree", ok))
            return ok and peer_ok
        return all_ok

    dev = torch.device("cpu")
    for mode, peer_ok, want_err in (("clean", True, ""), ("clean", False, "a peer failed"), ("sums", True, "two-shot probe call 0: 1 of"),
                                    ("timeout", True, "one-shot probe: barrier timed out"), ("map", True, "one-shot probe: xgmi exchange unavailable")):
        events.clear()
        monkeypatch.setattr(xgmi, "XgmiExchange", fake(mode))
        err = xgmi.probe(2, 4, dev, lambda b: [b] * 4, all_ok_from(peer_ok), n=64)
        assert (err == "") if not want_err else err.startswith(want_err), (mode, peer_ok, err)
        agrees = [e for e in events if e[0] == "agree"]
        closes = [e for e in events if e[0] == "close"]
        if mode == "map":
            assert closes == [] and len(agrees) == 1
        else:
            # each exchange closes right after its agreement; a failed first one ends the probe
            assert events[0][0] == "agree" and events[1] == ("close", False)
            assert len(agrees) == (2 if (not want_err or mode == "sums") else 1)


def test_gloo_teardown_does_not_wait_for_collectives_queued_on_a_dead_peer():
    """A survivor tearing down its broken gloo group must not sit in the group's destructor
    until a collective it posted to a dead peer times out (r06_elastic_abort: a 17 s regroup)."""
    import datetime
    import threading
    import time

    import torch.distributed as dist

    from serverless_learn_amd.parallel.dp import ElasticGroup
    from serverless_learn_amd.utils.ports import reserve_port

    port = reserve_port()
    master = dist.TCPStore("127.0.0.1", port, is_master=True, wait_for_workers=False,
                           timeout=datetime.timedelta(seconds=30))
    gg = [ElasticGroup(backend="gloo", timeout_s=8) for _ in range(2)]
    ok = {}
    ths = [threading.Thread(target=lambda r=r: ok.setdefault(r, gg[r].reform(1, r, 2, f"127.0.0.1:{port}")))
           for r in range(2)]
    for th in ths:
        th.start()
    for th in ths:
        th.join(30)
    assert ok == {0: True, 1: True}
    work = gg[0].allreduce_async(torch.ones(4))  # rank 1 never joins: pending until the timeout
    assert work is not None
    t0 = time.monotonic()
    gg[0].teardown()
    assert time.monotonic() - t0 < 2.0 and not gg[0].active and len(gg[0]._retired) == 1
    gg[1].teardown()
    del master
