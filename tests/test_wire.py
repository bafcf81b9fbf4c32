"""Wire contract: golden bytes, codec round trips, descriptor/.proto agreement."""
import numpy as np
import pytest
from hypothesis import given, settings, strategies as st

from serverless_learn_amd.proto import messages as pb
from serverless_learn_amd.wire import codec


def test_update_golden_bytes():
    # packed f64 -> 0a 10 | 1.0 | 2.0
    want = bytes.fromhex("0a10" "000000000000f03f" "0000000000000040")
    assert pb.Update(delta=[1.0, 2.0]).SerializeToString() == want
    assert codec.encode_update(np.array([1.0, 2.0])) == want
    assert codec.encode_update(np.array([1.0, 2.0], np.float32)) == want


def test_reference_method_paths_served_by_descriptor():
    paths = {f"/{pb.PACKAGE}.{s}/{m.name}" for s, ms in pb.PROTO.services.items() for m in ms}
    for p in pb.REFERENCE_METHODS:
        assert p in paths
    assert pb.method_def("Worker", "ReceiveFile").client_streaming
    assert pb.PACKAGE == "serverless_learn"


def test_original_messages_keep_field_numbers():
    expect = {
        "WorkerBirthInfo": {"addr": 1}, "RegisterBirthAck": {"ok": 1},
        "Push": {"recipient_addr": 1, "file_num": 2}, "PushOutcome": {"ok": 1},
        "Chunk": {"data": 1}, "ReceiveFileAck": {"ok": 1}, "PeerList": {"peer_addrs": 1},
        "Update": {"delta": 1}, "FlowFeedback": {}, "LoadFeedback": {}, "Empty": {},
    }
    for msg, fields in expect.items():
        got = {f.name: f.number for f in pb.PROTO.messages[msg]}
        for name, num in fields.items():
            assert got[name] == num, (msg, name)


def test_additive_fields_are_skipped_by_an_original_parser():
    # An "old" PeerList parser (only field 1) must read our extended message.
    from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

    fdp = descriptor_pb2.FileDescriptorProto(name="old.proto", package="old", syntax="proto3")
    m = fdp.message_type.add(name="PeerList")
    m.field.add(name="peer_addrs", number=1, type=9, label=3)
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fdp)
    Old = message_factory.GetMessageClass(pool.FindMessageTypeByName("old.PeerList"))
    new = pb.PeerList(peer_addrs=["a:1", "b:2"], epoch=7, rank=1, world_size=2, rendezvous="h:1")
    old = Old.FromString(new.SerializeToString())
    assert list(old.peer_addrs) == ["a:1", "b:2"]


def test_flow_feedback_with_step_phases_parses_with_the_original_empty_schema():
    """FlowFeedback is empty in the original (/root/reference/src/protos/serverless_learn.proto:73-75):
    an original parser skips every additive field, the step-time breakdown (fields 11-16) included,
    and an original (empty) FlowFeedback decodes here with all phases zero."""
    from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

    fdp = descriptor_pb2.FileDescriptorProto(name="old_fb.proto", package="old", syntax="proto3")
    fdp.message_type.add(name="FlowFeedback")
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fdp)
    Old = message_factory.GetMessageClass(pool.FindMessageTypeByName("old.FlowFeedback"))
    new = pb.FlowFeedback(step=9, samples_per_sec=1e6, step_ms=0.11, data_wait_ms=0.01, compute_ms=0.09,
                          exchange_ms=0.015, update_ms=0.008, exchange_gbps=71.8)
    raw = new.SerializeToString()
    old = Old.FromString(raw)
    assert old.SerializeToString() == b"" or old.ByteSize() >= 0  # parsed (unknown fields kept or dropped)
    back = pb.FlowFeedback.FromString(Old().SerializeToString())
    assert back.compute_ms == 0.0 and back.exchange_gbps == 0.0
    got = {f.name: f.number for f in pb.PROTO.messages["FlowFeedback"]}
    assert [got[k] for k in ("step_ms", "data_wait_ms", "compute_ms", "exchange_ms", "update_ms",
                             "exchange_gbps")] == [11, 12, 13, 14, 15, 16]
    assert pb.FlowFeedback.FromString(raw).exchange_gbps == 71.8


@settings(max_examples=60, deadline=None)
@given(st.lists(st.floats(allow_nan=False, allow_infinity=True, width=64), max_size=300))
def test_update_roundtrip_f64(vals):
    arr = np.array(vals, np.float64)
    msg = codec.encode_update(arr)
    assert msg == pb.Update(delta=vals).SerializeToString()
    back = codec.decode_update(msg, "float64")
    np.testing.assert_array_equal(back, arr)


def test_update_decode_accepts_unpacked_and_unknown_fields():
    # unpacked doubles (tag 0x09) interleaved with an unknown varint field 7
    raw = bytes([0x09]) + np.float64(3.5).tobytes() + bytes([0x38, 0x05]) + bytes([0x09]) + np.float64(-1).tobytes()
    np.testing.assert_array_equal(codec.decode_update(raw, "float64"), [3.5, -1.0])
    assert list(pb.Update.FromString(raw).delta) == [3.5, -1.0]


def test_update_decode_rejects_truncation():
    msg = codec.encode_update(np.arange(10.0))
    with pytest.raises(ValueError):
        codec.decode_update(msg[:-3], "float64")


@settings(max_examples=30, deadline=None)
@given(st.binary(max_size=5000))
def test_chunk_roundtrip(data):
    msg = codec.encode_chunk(data)
    assert msg == pb.Chunk(data=data).SerializeToString()
    assert bytes(codec.chunk_payload(msg)) == data


def test_iter_chunks_uses_reference_chunk_size():
    buf = bytes(range(256)) * 10000  # 2.56 MB
    parts = list(codec.iter_chunks(buf))
    assert len(parts) == 3
    assert b"".join(bytes(codec.chunk_payload(p)) for p in parts) == buf
    assert len(codec.chunk_payload(parts[0])) == 1_000_000


def test_reference_dummy_file_is_deterministic():
    from serverless_learn_amd._core import core

    a = core().reference_dummy_file(4096)
    assert a == core().reference_dummy_file(4096)
    assert len(set(a)) > 200
