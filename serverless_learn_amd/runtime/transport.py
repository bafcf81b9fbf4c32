"""gRPC transport: raw-bytes generic handlers + a cached, deadline-aware client.

Reference transport: the synchronous gRPC C++ API with
insecure credentials, a brand-new channel per call site
(/root/reference/src/master.cc:258,284, worker.cc:210, file_server.cc:111-113,
flagged ``// TODO (PERF)`` at master.cc:257), no deadlines (a hung peer blocks
the caller's loop forever) and the default 4 MiB receive cap.

Here: handlers are registered on the exact method paths
(``/serverless_learn.<Service>/<Method>``) with NO serializers, so handlers see
wire bytes and decode them with the C++ codec (hot messages) or the
descriptor-built classes; channels are cached per address; every call has a
deadline; message caps are raised so a full-model ``Update`` fits.
"""
from __future__ import annotations

import threading
from concurrent import futures

import grpc

from ..proto import messages as pb

_RETRYABLE = {grpc.StatusCode.UNAVAILABLE, grpc.StatusCode.DEADLINE_EXCEEDED}


class RpcFailure(RuntimeError):
    def __init__(self, path: str, addr: str, code, details: str):
        super().__init__(f"{path} -> {addr}: {code.name if code else '?'} {details}")
        self.code = code
        self.path = path
        self.addr = addr

    @property
    def retryable(self) -> bool:
        return self.code in _RETRYABLE


def _options(max_message_bytes: int):
    return [
        ("grpc.max_receive_message_length", max_message_bytes),
        ("grpc.max_send_message_length", max_message_bytes),
    ]


class RpcServer:
    """A gRPC server hosting one or more services of the serverless_learn package."""

    def __init__(self, addr: str, max_workers: int = 16, max_message_bytes: int = 256 << 20):
        self._server = grpc.server(futures.ThreadPoolExecutor(max_workers=max_workers,
                                                              thread_name_prefix="sl-rpc"),
                                   options=_options(max_message_bytes) + [("grpc.so_reuseport", 0)])
        self.port = self._server.add_insecure_port(addr)
        if self.port == 0:
            raise OSError(f"could not bind {addr}")
        host = addr.rsplit(":", 1)[0]
        self.addr = f"{host}:{self.port}"
        self._started = False

    def add_service(self, service: str, handlers: dict) -> None:
        """``handlers``: method name -> fn(request_bytes_or_iterator, context) -> response bytes."""
        table = {}
        for method, fn in handlers.items():
            md = pb.method_def(service, method)
            if md.client_streaming and not md.server_streaming:
                table[method] = grpc.stream_unary_rpc_method_handler(fn)
            elif not md.client_streaming and not md.server_streaming:
                table[method] = grpc.unary_unary_rpc_method_handler(fn)
            else:
                raise NotImplementedError(f"{service}.{method}: streaming responses are not in the protocol")
        self._server.add_generic_rpc_handlers(
            (grpc.method_handlers_generic_handler(f"{pb.PACKAGE}.{service}", table),))

    def start(self) -> "RpcServer":
        self._server.start()
        self._started = True
        return self

    def stop(self, grace: float | None = 0.5) -> None:
        if self._started:
            self._server.stop(grace).wait()
            self._started = False

    def wait(self) -> None:
        self._server.wait_for_termination()


class Channels:
    """Per-address channel cache with deadlines (fixes master.cc:257's TODO(PERF))."""

    def __init__(self, max_message_bytes: int = 256 << 20, default_timeout: float = 5.0):
        self._lock = threading.Lock()
        self._channels: dict[str, grpc.Channel] = {}
        self._stubs: dict[tuple, object] = {}
        self._opts = _options(max_message_bytes)
        self.default_timeout = default_timeout

    def channel(self, addr: str) -> grpc.Channel:
        with self._lock:
            ch = self._channels.get(addr)
            if ch is None:
                ch = grpc.insecure_channel(addr, options=self._opts)
                self._channels[addr] = ch
            return ch

    def _stub(self, addr: str, service: str, method: str, kind: str):
        key = (addr, service, method)
        with self._lock:
            s = self._stubs.get(key)
        if s is None:
            ch = self.channel(addr)
            path = pb.method_path(service, method)
            s = ch.unary_unary(path) if kind == "uu" else ch.stream_unary(path)
            with self._lock:
                self._stubs[key] = s
        return s

    def unary(self, addr: str, service: str, method: str, request: bytes, timeout: float | None = None,
              metadata=None) -> bytes:
        stub = self._stub(addr, service, method, "uu")
        try:
            return stub(request, timeout=timeout or self.default_timeout, metadata=metadata)
        except grpc.RpcError as e:  # pragma: no cover - exercised by failure tests
            raise RpcFailure(pb.method_path(service, method), addr, e.code(), e.details() or "") from None

    def stream_unary(self, addr: str, service: str, method: str, requests, timeout: float | None = None,
                     metadata=None) -> bytes:
        stub = self._stub(addr, service, method, "su")
        try:
            return stub(requests, timeout=timeout or self.default_timeout, metadata=metadata)
        except grpc.RpcError as e:
            raise RpcFailure(pb.method_path(service, method), addr, e.code(), e.details() or "") from None

    def forget(self, addr: str) -> None:
        with self._lock:
            ch = self._channels.pop(addr, None)
            for k in [k for k in self._stubs if k[0] == addr]:
                del self._stubs[k]
        if ch is not None:
            ch.close()

    def close(self) -> None:
        with self._lock:
            chans = list(self._channels.values())
            self._channels.clear()
            self._stubs.clear()
        for ch in chans:
            ch.close()


def metadata_dict(context) -> dict:
    return {k: v for k, v in (context.invocation_metadata() or ())}
