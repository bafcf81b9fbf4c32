"""Prometheus metrics for every role (the reference only
prints free text, /root/reference/src/master.cc:81,89,139-143).

Metrics are derived from the structured log events the roles already emit
(:mod:`serverless_learn_amd.utils.log`), so instrumentation lives in one
place: every event increments ``sl_events_total{role,event,level}`` and the
numeric fields of a few well-known events feed gauges / counters / histograms:

* ``train``         -> ``sl_step`` / ``sl_loss`` / ``sl_samples_per_second`` gauges
* ``received_file`` -> ``sl_ingested_bytes_total``, ``sl_ingest_seconds`` histogram
* ``push``          -> ``sl_pushed_bytes_total{ok}``, ``sl_push_seconds`` histogram
* ``register_birth`` / ``deregister`` / ``evict`` -> ``sl_membership_epoch`` gauge
* any ``epoch`` / ``world`` field -> ``sl_membership_epoch`` / ``sl_world_size``
* ``train``'s step-time breakdown -> ``sl_step_phase_ms{phase}``, ``sl_exchange_gbps``

Besides the log events, the transport reports every RPC it serves or makes (SURVEY.md §5.1,
"per-RPC latency histograms"): ``sl_rpc_seconds{role,side,method,code}`` -- side ``server`` /
``client``, method ``Service/Method``, the final gRPC status code (a client call's retries
included in its one observation).

Each role owns a :class:`Metrics` (its own registry: several roles may share
a process in tests and the local cluster).  ``SL_METRICS_PORT`` /
``--metrics-port`` > 0 serves it over HTTP at ``/metrics``.
"""
from __future__ import annotations

import threading

try:  # an optional dependency: roles run (and log) without it
    from prometheus_client import CollectorRegistry, Counter, Gauge, Histogram, generate_latest
    from prometheus_client.exposition import start_http_server

    AVAILABLE = True
except Exception:  # pragma: no cover - exercised only where prometheus_client is missing
    AVAILABLE = False

_BUCKETS = (0.001, 0.005, 0.02, 0.05, 0.1, 0.25, 0.5, 1.0, 2.5, 5.0, 10.0, 30.0)
# RPC latencies: control-plane calls take ~0.1-1 ms on one host, a 100 MB push seconds
_RPC_BUCKETS = (0.0001, 0.00025, 0.0005, 0.001, 0.0025, 0.005, 0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1.0, 2.5,
                5.0, 10.0, 30.0)
_PHASES = ("step_ms", "data_wait_ms", "compute_ms", "exchange_ms", "update_ms")


class Metrics:
    def __init__(self, role: str):
        self.role = role
        self._lock = threading.Lock()
        self.enabled = AVAILABLE
        self.port = 0
        if not AVAILABLE:
            return
        r = self.registry = CollectorRegistry()
        self.events = Counter("sl_events", "structured log events", ["role", "event", "level"], registry=r)
        self.step = Gauge("sl_step", "training steps completed", ["role"], registry=r)
        self.loss = Gauge("sl_loss", "last reported training loss", ["role"], registry=r)
        self.rate = Gauge("sl_samples_per_second", "training throughput (samples/s)", ["role"], registry=r)
        self.epoch = Gauge("sl_membership_epoch", "membership epoch", ["role"], registry=r)
        self.world = Gauge("sl_world_size", "members of the data-parallel group", ["role"], registry=r)
        self.job_rate = Gauge("sl_job_samples_per_second", "whole-job training throughput (samples/s) "
                              "derived by the master from the workers' feedback", ["role"], registry=r)
        self.group_rate = Gauge("sl_group_samples_per_second", "data-parallel group throughput (samples/s, "
                                "all-reduced over the group)", ["role"], registry=r)
        self.ingested = Counter("sl_ingested_bytes", "bytes landed by ReceiveFile", ["role"], registry=r)
        self.ingest_s = Histogram("sl_ingest_seconds", "ReceiveFile duration", ["role"], buckets=_BUCKETS,
                                  registry=r)
        self.pushed = Counter("sl_pushed_bytes", "bytes streamed by pushes", ["role", "ok"], registry=r)
        self.push_s = Histogram("sl_push_seconds", "push duration", ["role"], buckets=_BUCKETS, registry=r)
        self.rpc_s = Histogram("sl_rpc_seconds", "gRPC call latency by side (server / client), method and "
                               "final status code", ["role", "side", "method", "code"], buckets=_RPC_BUCKETS,
                               registry=r)
        self.phase_ms = Gauge("sl_step_phase_ms", "per-step time by phase over the last log interval "
                              "(wall step, loop waits; device compute / exchange / update of one probed step)",
                              ["role", "phase"], registry=r)
        self.exchange_gbps = Gauge("sl_exchange_gbps", "gradient exchange algorithm bandwidth of the probed step",
                                   ["role"], registry=r)

    # ---- fed by the transport ---------------------------------------------------------
    def rpc(self, side: str, method: str, code: str, seconds: float) -> None:
        if not self.enabled:
            return
        self.rpc_s.labels(self.role, side, method, code).observe(seconds)

    def rpc_count(self, side: str, method: str, code: str = "OK") -> int:
        """Observations so far of one (side, method, code) series (tests, feedback)."""
        if not self.enabled:
            return 0
        for metric in self.registry.collect():
            if metric.name != "sl_rpc_seconds":
                continue
            for smp in metric.samples:
                lb = smp.labels
                if (smp.name.endswith("_count") and lb.get("side") == side and lb.get("method") == method
                        and lb.get("code") == code):
                    return int(smp.value)
        return 0

    # ---- fed by Logger ----------------------------------------------------------
    def observe(self, level: str, event: str, fields: dict) -> None:
        if not self.enabled:
            return
        role = self.role
        with self._lock:
            self.events.labels(role, event, level).inc()
            if "epoch" in fields and isinstance(fields["epoch"], (int, float)) and fields["epoch"] >= 0:
                self.epoch.labels(role).set(fields["epoch"])
            if "world" in fields and isinstance(fields["world"], (int, float)):
                self.world.labels(role).set(fields["world"])
            if event == "train":
                for k, g in (("step", self.step), ("loss", self.loss), ("samples_per_sec", self.rate)):
                    if isinstance(fields.get(k), (int, float)):
                        g.labels(role).set(fields[k])
                if isinstance(fields.get("group_samples_per_sec"), (int, float)):
                    self.group_rate.labels(role).set(fields["group_samples_per_sec"])
                for ph in _PHASES:
                    if isinstance(fields.get(ph), (int, float)):
                        self.phase_ms.labels(role, ph[:-3]).set(fields[ph])
                if isinstance(fields.get("exchange_gbps"), (int, float)):
                    self.exchange_gbps.labels(role).set(fields["exchange_gbps"])
            elif event == "job":
                if isinstance(fields.get("samples_per_sec"), (int, float)):
                    self.job_rate.labels(role).set(fields["samples_per_sec"])
            elif event == "received_file":
                if isinstance(fields.get("bytes"), (int, float)):
                    self.ingested.labels(role).inc(fields["bytes"])
                if isinstance(fields.get("s"), (int, float)):
                    self.ingest_s.labels(role).observe(fields["s"])
            elif event == "push":
                ok = "true" if fields.get("ok") else "false"
                if isinstance(fields.get("bytes"), (int, float)):
                    self.pushed.labels(role, ok).inc(fields["bytes"])
                if isinstance(fields.get("s"), (int, float)):
                    self.push_s.labels(role).observe(fields["s"])

    # ---- exposition -----------------------------------------------------------------
    def text(self) -> str:
        return generate_latest(self.registry).decode() if self.enabled else ""

    def serve(self, port: int, addr: str = "0.0.0.0") -> int:
        """Serve /metrics on ``port`` (0 = an ephemeral port); returns the bound port."""
        if not self.enabled:
            return 0
        server, _thread = start_http_server(port, addr=addr, registry=self.registry)
        self.port = server.server_address[1]
        self._server = server
        return self.port

    def close(self) -> None:
        srv = getattr(self, "_server", None)
        if srv is not None:
            srv.shutdown()
            srv.server_close()
            self._server = None
