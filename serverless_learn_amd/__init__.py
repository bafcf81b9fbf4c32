"""serverless_learn_amd -- an MI355X-native serverless-learning runtime.

Same capabilities and wire protocol as sheaconlon/serverless_learn (master,
file server and ephemeral workers speaking package ``serverless_learn`` over
gRPC), with real training on MI355X: hand-written gfx950 HIP kernels for the
model math, RCCL all-reduce over xGMI for data parallelism, pinned-buffer
shard ingest and a wire-compatible checkpoint format.
"""
__version__ = "0.1.0"
