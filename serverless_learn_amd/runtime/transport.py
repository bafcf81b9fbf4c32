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
deadline; message caps are raised so a full-model ``Update`` fits.  Every call served and
every call made is timed into the owning role's ``sl_rpc_seconds`` histogram (method, side,
final status code) -- the reference times nothing.
"""
from __future__ import annotations

import random
import threading
import time
from concurrent import futures

import grpc

from ..proto import messages as pb

_RETRYABLE = {grpc.StatusCode.UNAVAILABLE, grpc.StatusCode.DEADLINE_EXCEEDED}

# Unary RPCs that may be re-sent after a transient failure: re-delivery has no extra effect
# (CheckUp replaces the receiver's view, the others read state or set it to the same value).
# ExchangeUpdates mixes models and DoPush re-streams a whole shard: never retried here.  The
# reference only logs a failed call (master.cc:156-158, :192-194).
IDEMPOTENT = frozenset({
    ("Worker", "CheckUp"), ("FileServer", "CheckUp"), ("MasterControl", "GetMembership"),
    ("FileStore", "ListFiles"), ("MasterControl", "ReportCheckpoint"), ("MasterControl", "Deregister"),
    ("Master", "RegisterBirth"),
})


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


def _status_name(context, default: str) -> str:
    code = context.code() if context is not None and hasattr(context, "code") else None
    return code.name if code is not None else default


class RpcServer:
    """A gRPC server hosting one or more services of the serverless_learn package.
    ``metrics`` (utils.metrics.Metrics): every handled call is timed, with its status code."""

    def __init__(self, addr: str, max_workers: int = 16, max_message_bytes: int = 256 << 20, metrics=None):
        self.metrics = metrics
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
            if self.metrics is not None:
                fn = self._timed(f"{service}/{method}", fn)
            if md.client_streaming and not md.server_streaming:
                table[method] = grpc.stream_unary_rpc_method_handler(fn)
            elif not md.client_streaming and not md.server_streaming:
                table[method] = grpc.unary_unary_rpc_method_handler(fn)
            else:
                raise NotImplementedError(f"{service}.{method}: streaming responses are not in the protocol")
        self._server.add_generic_rpc_handlers(
            (grpc.method_handlers_generic_handler(f"{pb.PACKAGE}.{service}", table),))

    def _timed(self, name: str, fn):
        m = self.metrics

        def handler(request, context):
            t0 = time.perf_counter()
            code = "UNKNOWN"
            try:
                out = fn(request, context)
                code = _status_name(context, "OK")
                return out
            except Exception:
                code = _status_name(context, "UNKNOWN")  # context.abort() sets it before raising
                raise
            finally:
                m.rpc("server", name, code, time.perf_counter() - t0)
        return handler

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

    def __init__(self, max_message_bytes: int = 256 << 20, default_timeout: float = 5.0, retries: int = 4,
                 backoff_s: float = 0.05, metrics=None):
        self.metrics = metrics      # utils.metrics.Metrics: client-side latency per call
        self.retries = retries      # extra attempts for idempotent unary RPCs
        self.backoff_s = backoff_s  # first back-off; doubles per attempt, +-50 % jitter
        self.retried = 0            # attempts re-sent (metrics / tests)
        self._lock = threading.Lock()
        self._channels: dict[str, grpc.Channel] = {}
        self._stubs: dict[tuple, object] = {}
        # reconnect quickly: gRPC's default first reconnect back-off is 1 s, during which every
        # call on the channel fails at once (a retry could never see a restarted listener)
        self._opts = _options(max_message_bytes) + [
            ("grpc.initial_reconnect_backoff_ms", 100), ("grpc.min_reconnect_backoff_ms", 100),
            ("grpc.max_reconnect_backoff_ms", 2000)]
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
              metadata=None, idempotent: bool | None = None) -> bytes:
        """One unary call with a deadline.  Idempotent methods (``IDEMPOTENT``, or
        ``idempotent=True``) are re-sent with bounded exponential back-off on UNAVAILABLE /
        DEADLINE_EXCEEDED, all attempts inside the ONE deadline ``timeout`` -- so a caller's
        failure-detection timing (the master's miss counting) is unchanged: a peer that is
        really gone still fails within ``timeout``, while a dropped connection or a restarting
        listener no longer costs a miss."""
        t0 = time.perf_counter()
        code = "OK"
        try:
            return self._unary(addr, service, method, request, timeout, metadata, idempotent)
        except RpcFailure as f:
            code = f.code.name if f.code else "UNKNOWN"
            raise
        finally:
            if self.metrics is not None:
                self.metrics.rpc("client", f"{service}/{method}", code, time.perf_counter() - t0)

    def _unary(self, addr, service, method, request, timeout, metadata, idempotent) -> bytes:
        stub = self._stub(addr, service, method, "uu")
        budget = timeout or self.default_timeout
        deadline = time.monotonic() + budget
        retry = (service, method) in IDEMPOTENT if idempotent is None else idempotent
        attempt = 0
        while True:
            left = deadline - time.monotonic()
            try:
                return stub(request, timeout=max(0.001, left), metadata=metadata)
            except grpc.RpcError as e:
                fail = RpcFailure(pb.method_path(service, method), addr, e.code(), e.details() or "")
            wait = self.backoff_s * (2 ** attempt) * (0.5 + random.random())
            if not (retry and fail.retryable and attempt < self.retries
                    and deadline - time.monotonic() > wait + 0.01):
                raise fail
            attempt += 1
            with self._lock:
                self.retried += 1
            time.sleep(wait)

    def stream_unary(self, addr: str, service: str, method: str, requests, timeout: float | None = None,
                     metadata=None) -> bytes:
        stub = self._stub(addr, service, method, "su")
        t0 = time.perf_counter()
        code = "OK"
        try:
            return stub(requests, timeout=timeout or self.default_timeout, metadata=metadata)
        except grpc.RpcError as e:
            code = e.code().name if e.code() else "UNKNOWN"
            raise RpcFailure(pb.method_path(service, method), addr, e.code(), e.details() or "") from None
        finally:
            if self.metrics is not None:
                self.metrics.rpc("client", f"{service}/{method}", code, time.perf_counter() - t0)

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
