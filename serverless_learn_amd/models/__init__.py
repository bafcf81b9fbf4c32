"""Model registry: the worker asks for a trainer by name (``Config.model``).

Every trainer exposes the same small interface -- ``load_shard``, ``step``,
``stats``, ``get_flat``/``set_flat``, ``params``/``mom`` (flat fp32 vectors),
``allreduce`` (gradient hook), ``n_params``, ``model_name``, ``set_world`` --
so the runtime (gossip, parameter server, all-reduce DP, checkpoints) is
model-agnostic: everything travels as one flat parameter vector, exactly what
the reference's ``Update{repeated double delta}`` carries (proto :81-83).
"""
from __future__ import annotations

import torch

MODELS = ("mlp", "resnet18")


def make_trainer(model: str, device: torch.device, **kw):
    """A GPU (hand-written HIP kernels) or CPU (torch reference) trainer."""
    cuda = torch.device(device).type == "cuda"
    if model == "mlp":
        from . import mlp

        return mlp.FusedMLPTrainer(device=device, **kw) if cuda else mlp.CPUTrainer(**kw)
    if model in ("resnet18", "resnet18-cifar"):
        from . import resnet

        if cuda:
            from .resnet_engine import FusedResNetTrainer

            return FusedResNetTrainer(device=device, **kw)
        return resnet.CPUResNetTrainer(**kw)
    raise ValueError(f"unknown model {model!r} (choose from {MODELS})")
