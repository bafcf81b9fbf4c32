"""Exact resume (checkpoint format v2: parameters + momentum + batch cursor + BatchNorm running
statistics), the ResNet engine's eval-mode forward, and the runtime worker running the fused
engine from hipGraph chunks (reference state message: proto :81-83)."""
import numpy as np
import pytest
import torch

from serverless_learn_amd.ckpt import format as ckfmt

pytestmark = pytest.mark.gpu


def _roundtrip(tr):
    """Save a trainer's full state through the checkpoint byte format and decode it."""
    n = tr.n_params
    mom = tr.mom[:n].cpu().numpy() if tr.mom is not None else None
    buf = ckfmt.encode(tr.get_flat().cpu().numpy(), {"model": tr.model_name, "step": 0}, mom, tr.state_extra())
    return ckfmt.decode_full(buf)


def _restore(tr, state):
    meta, params, mom, extra = state
    tr.set_flat(torch.from_numpy(params))
    if mom is not None:
        tr.mom[:tr.n_params].copy_(torch.from_numpy(mom))
    tr.load_state_extra(extra)


def test_mlp_resume_is_bit_exact():
    """Save at step k, resume in a fresh trainer, run m steps: bit-equal to k + m uninterrupted
    steps (parameters and momentum), because the batch cursor travels in the checkpoint."""
    from serverless_learn_amd.data.synthetic import make_mnist_like
    from serverless_learn_amd.models.mlp import FusedMLPTrainer

    x, y = make_mnist_like(4 * 2048, seed=3)
    x, y = torch.from_numpy(x), torch.from_numpy(y)
    k, m = 5, 6
    a = FusedMLPTrainer(batch=2048, device="cuda:0", seed=1)
    a.load_shard(x, y)
    for _ in range(k):
        a.step()
    state = _roundtrip(a)
    assert int(state[3]["cursor"][0]) == k
    for _ in range(m):
        a.step()
    b = FusedMLPTrainer(batch=2048, device="cuda:0", seed=99)  # different init: everything must come from the file
    b.load_shard(x, y)
    _restore(b, state)
    for _ in range(m):
        b.step()
    torch.cuda.synchronize()
    assert torch.equal(a.get_flat(), b.get_flat())
    assert torch.equal(a.mom, b.mom)
    assert int(a.cursor.item()) == int(b.cursor.item()) == k + m


def test_resnet_resume_restores_running_stats_and_cursor():
    from serverless_learn_amd.data.synthetic import make_cifar_like
    from serverless_learn_amd.models.resnet_engine import FusedResNetTrainer

    x, y = make_cifar_like(4 * 32, seed=5)
    x, y = torch.from_numpy(x), torch.from_numpy(y)
    a = FusedResNetTrainer(batch=32, device="cuda:0", seed=2)
    a.load_shard(x, y)
    for _ in range(3):
        a.step()
    state = _roundtrip(a)
    b = FusedResNetTrainer(batch=32, device="cuda:0", seed=7)
    b.load_shard(x, y)
    _restore(b, state)
    torch.cuda.synchronize()
    assert torch.equal(a.get_flat(), b.get_flat()) and torch.equal(a.mom, b.mom)
    assert int(b.cursor.item()) == 3
    for name, (rm, rv) in a.running_stats().items():
        brm, brv = b.running_stats()[name]
        assert torch.equal(rm, brm) and torch.equal(rv, brv), name
    # the stats are real (moved away from the (0, 1) init) and keep evolving identically
    rm0, rv0 = a.running_stats()["stem_bn"] if "stem_bn" in a.running_stats() else next(iter(a.running_stats().values()))
    assert float(rm0.abs().sum()) > 0 and float((rv0 - 1).abs().sum()) > 0
    assert int(a.cursor.item()) == 3
    # the default build's BN / weight-gradient sums use cross-workgroup atomics, so two runs of
    # the same step are not bit-equal (the deterministic build's bit-exact resume is the next
    # test): the resumed step must move the weights the same way and advance the same cursor
    w0 = a.get_flat()
    a.step()
    b.step()
    torch.cuda.synchronize()
    da, db = (a.get_flat() - w0).double(), (b.get_flat() - w0).double()
    cos = float(torch.dot(da, db) / (da.norm() * db.norm()))
    assert cos > 0.95, cos
    assert int(a.cursor.item()) == int(b.cursor.item()) == 4


def test_resnet_resume_is_bit_exact_in_deterministic_build():
    """Save at step k, resume in a fresh engine, run m steps: with the deterministic kernel build
    (SL_DETERMINISTIC=1: fixed-point cross-workgroup sums, no split-K atomics) parameters,
    momentum, BatchNorm running statistics and cursor are bit-identical to the uninterrupted
    run.  Runs in a child process, since a process loads one kernel library."""
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, SL_DETERMINISTIC="1")
    out = subprocess.run([sys.executable, os.path.join(root, "scripts", "resnet_resume_det.py"), "32", "3", "2"],
                         env=env, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    r = json.loads(out.stdout.strip().splitlines()[-1])
    assert r["deterministic_build"] and r["finite"], r
    assert r["params_identical"] and r["mom_identical"] and r["running_stats_identical"], r
    assert r["cursor"] == [5, 5], r


def test_resnet_eval_uses_running_statistics():
    """Eval forward = fp32 torch reference in eval mode (F.batch_norm with the engine's running
    statistics) on the same weights; it differs from the batch-statistics forward."""
    from serverless_learn_amd.data.synthetic import make_cifar_like
    from serverless_learn_amd.models.resnet import ref_forward
    from serverless_learn_amd.models.resnet_engine import FusedResNetTrainer

    x, y = make_cifar_like(3 * 32, seed=11)
    x, y = torch.from_numpy(x), torch.from_numpy(y)
    tr = FusedResNetTrainer(batch=32, device="cuda:0", seed=4, lr=0.05)
    tr.load_shard(x, y)
    for _ in range(6):
        tr.step()
    torch.cuda.synchronize()
    xe, ye = x[:64], y[:64]
    st = tr.evaluate(xe, ye)
    running = {k: (m.detach().cpu().clone(), v.detach().cpu().clone()) for k, (m, v) in tr.running_stats().items()}
    flat = tr.get_flat().cpu()
    with torch.no_grad():
        logits = ref_forward(tr.spec, flat, xe, training=False, running=running)
        ref_loss = float(torch.nn.functional.cross_entropy(logits, ye.long()))
        ref_acc = float((logits.argmax(1) == ye.long()).float().mean())
        batch_logits = ref_forward(tr.spec, flat, xe, training=True, running=None)
        batch_loss = float(torch.nn.functional.cross_entropy(batch_logits, ye.long()))
    assert st.samples == 64
    assert abs(st.loss - ref_loss) < 0.03 * max(1.0, ref_loss), (st.loss, ref_loss)
    assert abs(st.accuracy - ref_acc) <= 4 / 64, (st.accuracy, ref_acc)
    assert abs(ref_loss - batch_loss) > 1e-3  # running statistics really differ from batch statistics
    # evaluation leaves the training state alone
    assert int(tr.cursor.item()) == 6


def test_worker_runs_graph_chunks_near_engine_speed():
    """The runtime worker trains from hipGraph chunks (Config.graph): its reported samples/s
    (FlowFeedback) reaches >= 90 % of the bare engine's on the same GPU and batch."""
    import time

    from serverless_learn_amd.data.synthetic import make_mnist_like
    from serverless_learn_amd.models.mlp import FusedMLPTrainer
    from serverless_learn_amd.proto import messages as pb
    from serverless_learn_amd.runtime.local_cluster import LocalCluster, fast_config

    B = 65536
    x, y = make_mnist_like(2 * B, seed=0)
    eng = FusedMLPTrainer(batch=B, device="cuda:0")
    eng.load_shard(torch.from_numpy(x), torch.from_numpy(y))
    eng.step()
    eng.capture(warmup=0, unroll=16)
    eng.steps(32)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.steps(320)
    torch.cuda.synchronize()
    engine_rate = 320 * B / (time.perf_counter() - t0)
    del eng
    torch.cuda.empty_cache()

    c = LocalCluster(fast_config(device="cuda:0", batch=B, shard_records=2 * B, log_every=320, graph_steps=16))
    try:
        w = c.add_worker(sync="none")
        assert c.wait_for(lambda: w.step >= 1300, 240), w.step
        fb = pb.FlowFeedback.FromString(w._check_up(pb.PeerList().SerializeToString(), None))
        assert w.graph_chunks > 0
        assert fb.samples_per_sec >= 0.9 * engine_rate, (fb.samples_per_sec, engine_rate)
        assert fb.group_world == 1 and fb.group_samples_per_sec > 0
    finally:
        c.stop()
