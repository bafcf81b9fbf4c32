"""GPU paths of the runtime: pinned ingest ring into HBM, K7 gossip kernel, K5 SGD."""
import numpy as np
import pytest
import torch

from serverless_learn_amd.parallel.gossip import GossipState

pytestmark = pytest.mark.gpu


def test_ingest_ring_lands_bytes_in_hbm():
    from serverless_learn_amd._core import core
    from serverless_learn_amd.wire.codec import iter_chunks

    data = np.random.default_rng(0).integers(0, 256, size=9_500_001, dtype=np.uint8).tobytes()
    ring = core().IngestRing(1 << 20, 3, 0)
    assert ring.pinned and ring.has_device
    dst = torch.empty(len(data), dtype=torch.uint8, device="cuda")
    ring.begin(dst.data_ptr(), len(data), True)
    for msg in iter_chunks(data, 1_000_000):
        ring.feed_chunk(msg)
    assert ring.finish() == len(data)
    assert bytes(dst.cpu().numpy()) == data


def _ref_serve(m, o, d, a):
    m = m.astype(np.float64).copy()
    m[:d.size] += a * d
    m = m.astype(np.float32).astype(np.float64)
    return m, m - o.astype(np.float64)


def test_gossip_kernel_matches_reference_math():
    rng = np.random.default_rng(1)
    n = 100_003
    m0 = rng.standard_normal(n).astype(np.float32)
    o0 = (m0 - rng.standard_normal(n).astype(np.float32) * 0.1).astype(np.float32)
    d = rng.standard_normal(n - 7)
    g = GossipState(torch.from_numpy(m0).cuda(), 0.5)
    g.old.copy_(torch.from_numpy(o0))
    reply = g.serve(d)
    m_ref, r_ref = _ref_serve(m0, o0, d, 0.5)
    np.testing.assert_allclose(g.model.cpu().numpy(), m_ref.astype(np.float32), rtol=0, atol=0)
    np.testing.assert_allclose(reply, r_ref, rtol=0, atol=0)
    assert torch.equal(g.old, g.model)


def test_gossip_echo_free_client_absorb():
    n = 4096
    m = torch.randn(n, device="cuda")
    g = GossipState(m, 0.5, compat=False)
    sent = g.make_delta()  # zeros right after construction
    reply = np.random.default_rng(2).standard_normal(n)
    before = g.model.clone().cpu().double().numpy()
    g.absorb(reply, sent)
    expect = (before + 0.5 * (reply - 0.5 * sent)).astype(np.float32)
    np.testing.assert_allclose(g.model.cpu().numpy(), expect, atol=1e-6)


def test_gossip_absorb_kernel_keeps_in_flight_progress():
    """K7b on device: o advances by exactly what was shared; a step taken during the RPC stays pending."""
    rng = np.random.default_rng(3)
    n = 65_537
    m0 = rng.standard_normal(n).astype(np.float32)
    g = GossipState(torch.from_numpy(m0).cuda(), 0.5, compat=False)
    g.model += 1.0
    sent = g.make_delta()
    step = torch.from_numpy(rng.standard_normal(n).astype(np.float32)).cuda()
    g.model += step                                  # training during the RPC
    reply = rng.standard_normal(n)
    before_m = g.model.clone()
    before_o = g.old.clone()
    g.absorb(reply, sent)
    r = reply - 0.5 * sent
    m_ref = (before_m.cpu().double().numpy() + 0.5 * r).astype(np.float32)
    o_ref = (before_o.cpu().double().numpy() + sent + 0.5 * r).astype(np.float32)
    np.testing.assert_array_equal(g.model.cpu().numpy(), m_ref)
    np.testing.assert_array_equal(g.old.cpu().numpy(), o_ref)
    np.testing.assert_allclose(g.make_delta(), step.cpu().double().numpy(), atol=1e-5)


def test_sgd_flat_kernel_matches_torch():
    from serverless_learn_amd.ops.optim import sgd_flat

    n = 1_000_003
    w = torch.randn(n, device="cuda")
    g = torch.randn(n, device="cuda")
    mom = torch.randn(n, device="cuda")
    shadow = torch.empty(n, dtype=torch.bfloat16, device="cuda")
    w_ref, m_ref = w.clone(), mom.clone()
    sgd_flat(w, g, mom, lr=0.1, momentum=0.9, weight_decay=1e-4, shadow=shadow)
    d = g + 1e-4 * w_ref
    m_ref = 0.9 * m_ref + d
    w_ref -= 0.1 * m_ref
    torch.testing.assert_close(w, w_ref, rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(mom, m_ref, rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(shadow.float(), w.bfloat16().float(), rtol=0, atol=0)


def test_gpu_worker_trains_from_pushed_shard():
    from serverless_learn_amd.runtime.local_cluster import LocalCluster, fast_config

    c = LocalCluster(fast_config(device="cuda:0", batch=1024, shard_records=16384, log_every=20))
    try:
        w = c.add_worker(sync="none")
        assert c.wait_for(lambda: w.step >= 200, 120), w.step
        assert w.ring.pinned
        st = w.trainer.stats()
        assert st.accuracy > 0.8, st
    finally:
        c.stop()


def test_device_synth_matches_numpy_reference():
    """K8: the on-device Philox generator reproduces the numpy reference (u8 +-1 at fp32 rounding ties)."""
    import numpy as np

    from serverless_learn_amd.data.device_synth import synth_on_device, synth_reference

    for kind, first in (("mnist", 0), ("cifar", 1234567)):
        img, lab = synth_on_device(kind, 96, seed=0xABCDEF0123, first=first)
        ref_img, ref_lab = synth_reference(kind, 96, seed=0xABCDEF0123, first=first)
        torch.cuda.synchronize()
        assert np.array_equal(lab.cpu().numpy(), ref_lab)
        diff = np.abs(img.cpu().numpy().astype(int) - ref_img.astype(int))
        assert diff.max() <= 1 and (diff > 0).mean() < 0.01, (kind, diff.max(), (diff > 0).mean())


@pytest.mark.parametrize("argv", [
    ["--steps", "4", "--warmup", "2", "--ingest", "local", "--batch", "4096"],
    ["--model", "resnet18", "--steps", "2", "--warmup", "1", "--ingest", "device", "--batch", "64"],
])
def test_bench_prints_the_driver_json_contract(argv, capsys):
    """bench.py's one JSON line: the fields the driver reads, the BASELINE.json metric for the
    MLP, whole-job value = global batch x steps / time."""
    import json
    import os

    import bench

    assert bench.main(argv) == 0
    line = [ln for ln in capsys.readouterr().out.splitlines() if ln.startswith("{")][-1]
    out = json.loads(line)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in out, k
    for k in ("model", "global_batch", "seq_len", "parallelism"):
        assert k in out["config"], k
    assert out["n_gpus"] == 1 and out["steps"] == int(argv[argv.index("--steps") + 1])
    assert out["higher_is_better"] is True and out["scaling"] == "weak" and out["dtype"] == "bf16"
    assert "synthetic" in out["data"] and out["config"]["parallelism"] == "dp1"
    b = out["config"]["global_batch"]
    assert abs(out["value"] - b / (out["ms_per_step"] / 1e3)) / out["value"] < 0.03  # ms_per_step is rounded
    if "--model" not in argv:
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        with open(os.path.join(root, "BASELINE.json")) as f:
            assert out["metric"] == json.load(f)["metric"]


def test_bench_two_ranks_autotune_and_replicas():
    """bench.py with 2 ranks (gloo rehearsal on the one GPU): the xGMI exchange is set up, one-shot,
    two-shot and the process group are timed before the timed region, the replicas end identical,
    and the JSON reports the whole-job value for dp2."""
    import json
    import os
    import socket
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = ["timeout", "-k", "10", "150", sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node=2", "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "8", "--warmup", "3", "--batch", "4096",
           "--dist-backend", "gloo", "--oversubscribe", "--ingest", "local"]
    p = subprocess.run(cmd, cwd=root, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=170)
    assert p.returncode == 0, p.stdout[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith('{"metric"')]
    assert len(lines) == 1, p.stdout[-4000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "dp2" and out["config"]["global_batch"] == 8192
    assert out["replicas_identical"] is True and "replica_fallback" not in out
    at = out["allreduce_autotune"]
    assert {"xgmi_ms", "xgmi_two_shot_ms", "pg_ms"} <= set(at), at
    best = min(at["xgmi_ms"], at["xgmi_two_shot_ms"], at["pg_ms"])
    names = {"xgmi_ms": "xgmi-ipc", "xgmi_two_shot_ms": "xgmi-ipc-two-shot", "pg_ms": "gloo"}
    fastest = {names[k] for k in names if at[k] == best}  # (rounded values may tie)
    assert out["config"]["collective_backend"] in fastest, (out["config"]["collective_backend"], at)
    assert abs(out["value"] - 8192 / (out["ms_per_step"] / 1e3)) / out["value"] < 0.03


def _bench_self_launch(extra, timeout=240):
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = ["timeout", "-k", "10", str(timeout), sys.executable, os.path.join(root, "bench.py"), *extra]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run(cmd, cwd=root, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                       timeout=timeout + 20, env=env)
    assert p.returncode == 0, p.stdout[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith('{"metric"')]
    assert len(lines) == 1, p.stdout[-4000:]
    return json.loads(lines[0])


@pytest.mark.parametrize("model,extra", [
    ("mlp", ["--batch", "4096", "--steps", "8", "--warmup", "3", "--ingest", "local"]),
    ("resnet18", ["--batch", "64", "--steps", "3", "--warmup", "2", "--ingest", "device", "--bucket-mb", "4"]),
])
def test_bench_self_launches_two_ranks(model, extra):
    """``bench.py --gpus 2`` with no launcher spawns the two rank processes itself (here sharing the
    one GPU over gloo, --oversubscribe) and reports a real dp2 number: both models, replicas
    identical after the timed steps (the ResNet path through the async bucket hooks)."""
    out = _bench_self_launch(["--gpus", "2", "--oversubscribe", "--dist-backend", "gloo", "--model", model, *extra])
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "dp2"
    assert out["dist"]["world_size"] == 2 and out["dist"]["launcher"] == "bench.py"
    assert out["dist"]["ranks_share_gpus"] is True
    assert out["replicas_identical"] is True, out
    b = int(extra[extra.index("--batch") + 1])
    assert out["config"]["global_batch"] == 2 * b


@pytest.mark.parametrize("mode", ["once", "always"])
def test_bench_diverged_replicas_retime_or_refuse(mode):
    """The N>1 safety net end to end (2 gloo ranks sharing the GPU, the process-group path):
    rank 1's weights are perturbed before the replica check.  Once: bench.py re-syncs, re-times
    with the uncaptured process group and reports the new number with replica_fallback.  Always:
    exit 2 and no JSON line -- a diverged run never prints a number."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = ["timeout", "-k", "10", "200", sys.executable, os.path.join(root, "bench.py"), "--gpus", "2",
           "--oversubscribe", "--dist-backend", "gloo", "--allreduce", "pg", "--batch", "4096", "--steps", "6",
           "--warmup", "2", "--ingest", "local"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["SL_BENCH_FORCE_DIVERGE"] = mode
    p = subprocess.run(cmd, cwd=root, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=230,
                       env=env)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith('{"metric"')]
    if mode == "once":
        assert p.returncode == 0, p.stdout[-4000:]
        import json

        out = json.loads(lines[-1])
        assert out["replica_fallback"] == "replicas diverged" and out["replicas_identical"] is True
        assert out["config"]["hipgraph"] is False
    else:
        assert p.returncode != 0 and not lines, p.stdout[-4000:]
        assert "no number reported" in p.stdout
