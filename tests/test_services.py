"""All RPCs of the three services, in-process on ephemeral ports."""
import time

import numpy as np
import pytest

from serverless_learn_amd.ckpt.format import CKPT_BASE
from serverless_learn_amd.data.synthetic import decode_shard
from serverless_learn_amd.proto import messages as pb
from serverless_learn_amd.runtime.file_server import FILE_NUM_MD, FileServer
from serverless_learn_amd.runtime.local_cluster import _Sink, fast_config
from serverless_learn_amd.runtime.master import Master
from serverless_learn_amd.runtime.transport import Channels, RpcFailure
from serverless_learn_amd.runtime.worker import Worker
from serverless_learn_amd.wire import codec


@pytest.fixture
def ch():
    c = Channels(default_timeout=5.0)
    yield c
    c.close()


@pytest.fixture
def fs():
    f = FileServer(fast_config(shard_records=512), addr="127.0.0.1:0").start()
    yield f
    f.stop()


def test_file_server_push_and_checkup(fs, ch):
    sink = _Sink()
    try:
        out = pb.PushOutcome.FromString(ch.unary(fs.addr, "FileServer", "DoPush",
                                                 pb.Push(recipient_addr=sink.server.addr, file_num=3).SerializeToString()))
        assert out.ok and out.bytes == sink.data.size
        hdr, x, y = decode_shard(sink.data.tobytes())
        assert hdr["n"] == 512 and hdr["shard_index"] == 3 and x.shape == (512, 784)
        lf = pb.LoadFeedback.FromString(ch.unary(fs.addr, "FileServer", "CheckUp", pb.Empty().SerializeToString()))
        assert lf.bytes_sent == out.bytes and lf.files >= 1
    finally:
        sink.server.stop()


def test_unknown_file_is_ok_false_and_server_survives(fs, ch):
    # reference: exit(1) on file_num != 0 (file_server.cc:107-110)
    out = pb.PushOutcome.FromString(ch.unary(fs.addr, "FileServer", "DoPush",
                                             pb.Push(recipient_addr="127.0.0.1:1", file_num=CKPT_BASE + 5)
                                             .SerializeToString()))
    assert not out.ok and "unknown" in out.error
    pb.LoadFeedback.FromString(ch.unary(fs.addr, "FileServer", "CheckUp", pb.Empty().SerializeToString()))


def test_push_to_dead_worker_fails_cleanly(fs, ch):
    out = pb.PushOutcome.FromString(ch.unary(fs.addr, "FileServer", "DoPush",
                                             pb.Push(recipient_addr="127.0.0.1:1", file_num=0).SerializeToString(),
                                             timeout=30))
    assert not out.ok


def test_reference_dummy_dataset(ch):
    cfg = fast_config(dataset="reference-dummy", dummy_file_length=3_000_000)
    f = FileServer(cfg, addr="127.0.0.1:0").start()
    sink = _Sink()
    try:
        out = pb.PushOutcome.FromString(ch.unary(f.addr, "FileServer", "DoPush",
                                                 pb.Push(recipient_addr=sink.server.addr, file_num=0)
                                                 .SerializeToString()))
        assert out.ok
        from serverless_learn_amd._core import core

        assert sink.data.tobytes() == core().reference_dummy_file(3_000_000)
        bad = pb.PushOutcome.FromString(ch.unary(f.addr, "FileServer", "DoPush",
                                                 pb.Push(recipient_addr=sink.server.addr, file_num=1)
                                                 .SerializeToString()))
        assert not bad.ok
    finally:
        sink.server.stop()
        f.stop()


def test_file_store_roundtrip(fs, ch):
    data = bytes(range(256)) * 9000
    md = ((FILE_NUM_MD, str(CKPT_BASE + 1)),)
    out = pb.PushOutcome.FromString(ch.stream_unary(fs.addr, "FileStore", "StoreFile", codec.iter_chunks(data),
                                                    metadata=md))
    assert out.ok and out.bytes == len(data)
    fl = pb.FileList.FromString(ch.unary(fs.addr, "FileStore", "ListFiles", pb.Empty().SerializeToString()))
    assert CKPT_BASE + 1 in list(fl.file_nums)
    rej = pb.PushOutcome.FromString(ch.stream_unary(fs.addr, "FileStore", "StoreFile", codec.iter_chunks(b"xx"),
                                                    metadata=((FILE_NUM_MD, "4"),)))
    assert not rej.ok


def test_master_register_is_idempotent_and_ps_exchange(ch):
    m = Master(fast_config(), addr="127.0.0.1:0").start(loops=False)
    try:
        info = pb.WorkerBirthInfo(addr="127.0.0.1:9", incarnation=5).SerializeToString()
        a1 = pb.RegisterBirthAck.FromString(ch.unary(m.addr, "Master", "RegisterBirth", info))
        a2 = pb.RegisterBirthAck.FromString(ch.unary(m.addr, "Master", "RegisterBirth", info))
        assert a1.ok and a2.ok and a1.epoch == a2.epoch == 1
        assert m.registry.members() == ["127.0.0.1:9"]
        # PS exchange semantics (master.cc:95-114): m += .5 d ; reply m - o ; o = m
        r1 = codec.decode_update(ch.unary(m.addr, "Master", "ExchangeUpdates", codec.encode_update(np.array([2.0, 4.0]))))
        np.testing.assert_allclose(r1, [1.0, 2.0])
        r2 = codec.decode_update(ch.unary(m.addr, "Master", "ExchangeUpdates", codec.encode_update(np.array([2.0]))))
        np.testing.assert_allclose(r2, [1.0, 0.0])
        mem = pb.PeerList.FromString(ch.unary(m.addr, "MasterControl", "GetMembership", pb.Empty().SerializeToString()))
        assert list(mem.peer_addrs) == ["127.0.0.1:9"] and mem.world_size == 1
        d = pb.RegisterBirthAck.FromString(ch.unary(m.addr, "MasterControl", "Deregister", info))
        assert d.ok and d.epoch == 2 and len(m.registry) == 0
    finally:
        m.stop()


def test_worker_rpcs_checkup_exchange_receivefile(ch):
    cfg = fast_config(sync="gossip", model="simulate", master_addr="127.0.0.1:1")
    w = Worker("127.0.0.1:0", cfg).start()
    try:
        fb = pb.FlowFeedback.FromString(ch.unary(w.addr, "Worker", "CheckUp",
                                                 pb.PeerList(peer_addrs=[w.addr, "x:1"], epoch=4, rank=0,
                                                             world_size=2).SerializeToString()))
        assert fb.state in ("idle", "training")
        assert w.view["peers"] == [w.addr, "x:1"] and w.view["epoch"] == 4
        # the simulated model starts empty and grows to the incoming length (worker.cc:85-89)
        r = codec.decode_update(ch.unary(w.addr, "Worker", "ExchangeUpdates", codec.encode_update(np.array([2.0, 2.0]))))
        np.testing.assert_allclose(r[:2], [1.0, 1.0], atol=0)
        # ReceiveFile without metadata (a reference-style sender) is accepted and counted
        ack = pb.ReceiveFileAck.FromString(ch.stream_unary(w.addr, "Worker", "ReceiveFile",
                                                           codec.iter_chunks(b"\x01" * 2_500_000)))
        assert ack.ok and w.bytes_ingested == 2_500_000
    finally:
        w.stop(leave=False)


def test_deadline_expiry_on_hung_peer(ch, monkeypatch):
    monkeypatch.setenv("SL_FAULT", "hang:CheckUp")
    w = Worker("127.0.0.1:0", fast_config(model="simulate", master_addr="127.0.0.1:1")).start()
    try:
        t0 = time.monotonic()
        with pytest.raises(RpcFailure) as ei:
            ch.unary(w.addr, "Worker", "CheckUp", pb.PeerList().SerializeToString(), timeout=0.5)
        assert ei.value.retryable and time.monotonic() - t0 < 3
    finally:
        w.fault.release()
        w.stop(leave=False)


def test_receive_file_short_stream_is_rejected(ch):
    """A stream that ends before the announced size is not acked (nor trained on)."""
    from serverless_learn_amd.data.synthetic import make_shard
    from serverless_learn_amd.runtime.file_server import FILE_SIZE_MD

    w = Worker("127.0.0.1:0", fast_config(model="simulate", master_addr="127.0.0.1:1")).start()
    try:
        data = bytes(make_shard(256, shard_index=0, num_shards=1, seed=0, dataset="synthetic-mnist"))
        md = ((FILE_NUM_MD, "0"), (FILE_SIZE_MD, str(len(data))))
        short = pb.ReceiveFileAck.FromString(ch.stream_unary(w.addr, "Worker", "ReceiveFile",
                                                             codec.iter_chunks(data[:len(data) // 2]), metadata=md))
        assert not short.ok and w._pending_shard is None
        # a header that claims more records than the file holds is rejected too
        md2 = ((FILE_NUM_MD, "0"), (FILE_SIZE_MD, str(len(data) // 2)))
        bad = pb.ReceiveFileAck.FromString(ch.stream_unary(w.addr, "Worker", "ReceiveFile",
                                                           codec.iter_chunks(data[:len(data) // 2]), metadata=md2))
        assert not bad.ok and w._pending_shard is None
        full = pb.ReceiveFileAck.FromString(ch.stream_unary(w.addr, "Worker", "ReceiveFile",
                                                            codec.iter_chunks(data), metadata=md))
        assert full.ok and w._pending_shard is not None
    finally:
        w.stop(leave=False)


def test_idempotent_rpc_retries_until_listener_is_back(ch):
    """An idempotent unary RPC (FileServer.CheckUp) to a server that is restarting is
    re-sent with back-off inside its one deadline and succeeds once the listener is up;
    a non-idempotent one (ExchangeUpdates) fails at once; a dead peer still fails within
    the deadline."""
    import socket
    import threading

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    addr = f"127.0.0.1:{port}"
    started = {}

    def start_later():
        time.sleep(0.4)
        started["fs"] = FileServer(fast_config(shard_records=256), addr=addr).start()

    th = threading.Thread(target=start_later)
    th.start()
    try:
        t0 = time.monotonic()
        raw = ch.unary(addr, "FileServer", "CheckUp", pb.Empty().SerializeToString(), timeout=4.0)
        pb.LoadFeedback.FromString(raw)
        assert ch.retried >= 1 and time.monotonic() - t0 < 4.0
    finally:
        th.join()
        started["fs"].stop()
    # nothing listens any more: fails within the deadline, never hangs past it
    t0 = time.monotonic()
    with pytest.raises(RpcFailure):
        ch.unary(addr, "FileServer", "CheckUp", pb.Empty().SerializeToString(), timeout=0.8)
    assert time.monotonic() - t0 < 2.0
    before = ch.retried
    with pytest.raises(RpcFailure):
        ch.unary(addr, "Worker", "ExchangeUpdates", codec.encode_update(np.zeros(2)), timeout=0.8)
    assert ch.retried == before
