"""Typed runtime configuration.

The reference is configured only at compile time: ``#define``s in
/root/reference/src/serverless_learn.h:5-12 (addresses, gossip and simulated
training intervals), file constants in /root/reference/src/master.cc:43,46,60
(push/checkup intervals, LEARN_RATE) and /root/reference/src/file_server.cc:40,46
(dummy file and chunk size); the only runtime flag is the worker's argv[1]
(/root/reference/src/worker.cc:234-239).

Here every knob is a dataclass field whose DEFAULT EQUALS THE REFERENCE
CONSTANT, overridable by ``SL_<FIELD>`` environment variables and by CLI flags
(:func:`add_cli_args` / :func:`from_args`).
"""
from __future__ import annotations

import argparse
import dataclasses
import os
from dataclasses import dataclass, field


@dataclass
class Config:
    # --- well-known endpoints (serverless_learn.h:5,8) ---
    master_addr: str = "localhost:50052"
    file_server_addr: str = "localhost:50053"
    # --- cadences, milliseconds (serverless_learn.h:10,12; master.cc:43,46) ---
    gossip_interval_ms: int = 5000
    simulated_train_interval_ms: int = 2000
    push_interval_ms: int = 5000
    checkup_interval_ms: int = 5000
    ps_broadcast_interval_ms: int = 0  # master -> random worker PS exchange (master.cc:268-293, never
                                       # started in the reference; it would run every 5000 ms); 0 = off
    # --- learning constants (master.cc:60) ---
    learn_rate: float = 0.5            # gossip / PS mixing coefficient alpha
    # --- data plane (file_server.cc:40,46) ---
    chunk_size: int = 1_000_000
    dummy_file_length: int = 100_000_000
    dataset: str = "synthetic-mnist"   # | "synthetic-cifar" | "reference-dummy" (byte-exact reference file 0)
    shard_records: int = 127_388       # records per shard: a 100,000,000-byte shard
    num_shards: int = 0                # 0 = one shard per worker
    push_policy: str = "on_change"     # "on_change" | "periodic" (reference: re-push every interval)
    store_dir: str = ""                # persist uploaded checkpoints here (file server)
    # --- failure detection / transport (new; reference has none) ---
    rpc_timeout_s: float = 5.0
    max_misses: int = 3                # evict after this many failed heartbeats
    max_message_bytes: int = 256 << 20
    rendezvous_port: int = 0           # master's collective rendezvous store (0 = pick free)
    metrics_port: int = 0              # > 0: serve Prometheus /metrics on this port (0 = off)
    # --- worker training ---
    sync: str = "allreduce"            # allreduce | gossip | ps | none
    gossip_compat: bool = False        # reproduce the reference's alpha^2 echo exactly
    device: str = "auto"               # auto | cpu | cuda[:N]
    model: str = "mlp"                 # mlp | resnet18 | simulate (reference: vector += 1)
    batch: int = 1024
    lr: float = 0.05
    momentum: float = 0.9
    weight_decay: float = 0.0
    seed: int = 0
    checkpoint_every: int = 0          # steps between checkpoints (rank 0); 0 = off
    max_steps: int = 0                 # 0 = run until stopped
    log_every: int = 50
    graph: bool = True                 # capture the fused step in a hipGraph when possible
    graph_steps: int = 16              # steps per graph replay chunk (error / metrics checks between chunks)
    graph_collectives: bool = False    # also capture a multi-rank RCCL group's collectives into the step graph
    dp_backend: str = "auto"           # auto (nccl = RCCL on GPU, gloo on CPU) | nccl | gloo
    dp_timeout_s: float = 30.0         # collective / rendezvous timeout of the data-parallel group
    xgmi: bool = True                  # MLP on a GPU group: all-reduce through IPC-mapped buffers over xGMI
    extra: dict = field(default_factory=dict)

    @classmethod
    def from_env(cls, **overrides) -> "Config":
        cfg = cls()
        for f in dataclasses.fields(cls):
            key = "SL_" + f.name.upper()
            if key in os.environ and f.name != "extra":
                setattr(cfg, f.name, _coerce(f, os.environ[key]))
        for k, v in overrides.items():
            setattr(cfg, k, v)
        return cfg

    @property
    def gossip_interval(self) -> float:
        return self.gossip_interval_ms / 1000.0

    @property
    def push_interval(self) -> float:
        return self.push_interval_ms / 1000.0

    @property
    def ps_broadcast_interval(self) -> float:
        return self.ps_broadcast_interval_ms / 1000.0

    @property
    def checkup_interval(self) -> float:
        return self.checkup_interval_ms / 1000.0


def _coerce(f, raw: str):
    t = f.type if isinstance(f.type, type) else {"int": int, "float": float, "bool": bool, "str": str}.get(str(f.type), str)
    if t is bool:
        return raw.strip().lower() in ("1", "true", "yes", "on")
    return t(raw)


def add_cli_args(ap: argparse.ArgumentParser, only=None) -> None:
    for f in dataclasses.fields(Config):
        if f.name == "extra" or (only is not None and f.name not in only):
            continue
        flag = "--" + f.name.replace("_", "-")
        if f.type in (bool, "bool"):
            ap.add_argument(flag, type=lambda s: s.lower() in ("1", "true", "yes", "on"), default=None)
        else:
            t = {"int": int, "float": float, "str": str}.get(str(f.type), f.type if isinstance(f.type, type) else str)
            ap.add_argument(flag, type=t, default=None)


def from_args(args: argparse.Namespace) -> Config:
    cfg = Config.from_env()
    for f in dataclasses.fields(Config):
        v = getattr(args, f.name, None)
        if v is not None:
            setattr(cfg, f.name, v)
    return cfg
