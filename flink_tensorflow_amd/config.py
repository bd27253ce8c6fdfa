"""Typed engine configuration.

The reference configures jobs through positional CLI args, programmatic
``env.setParallelism`` and constructor arguments, and ignores the Flink ``Configuration``
handed to ``open`` (``LIB/common/functions/util/ModelAwareFunction.scala:15``).  Here one
``EngineConfig`` carries every engine knob; it is loaded from (lowest to highest
precedence) defaults → a YAML file → ``FT_*`` environment variables → CLI flags, applied
to a :class:`~flink_tensorflow_amd.runtime.StreamExecutionEnvironment`, and visible to
every operator as ``parameters.engine`` in ``open(parameters)``
(also ``get_runtime_context().config.engine``).
"""
from __future__ import annotations

import argparse
import contextlib
import dataclasses
import os
from dataclasses import dataclass, field
from typing import Any

_HBM_BYTES_MI355X = 288 * 1024 ** 3


@dataclass
class EngineConfig:
    parallelism: int = 1               # subtasks per operator (one per GPU for GPU operators)
    max_batch: int = 256               # micro-batch size of batched model operators
    max_delay_ms: float = 10.0         # micro-batch flush timeout
    precision: str = "bf16"            # compiled CNN plans: bf16 | fp8
    batch_buckets: tuple = (64, 256)   # captured plan sizes for dynamic batching
    arena_fraction: float = 0.9        # share of HBM a subtask's plans may claim
    use_hip_graph: bool = True
    pipeline_depth: int = 3            # in-flight micro-batches per GPU (pinned ring slots)
    checkpoint_interval_s: float | None = None
    checkpoint_dir: str | None = None
    restart_attempts: int = 0
    restart_delay_s: float = 0.0
    channel_capacity: int = 1024
    log_level: str = "INFO"
    # ---- compiler / kernel selection (FT_<NAME> env vars or YAML): every default is the
    # measured-fastest choice; these switch a fusion OFF for A/B runs.  Variants measured
    # slower were removed with their kernels (graph/compiler.py LITE_TILE comment)
    sibling_conv_fusion: bool = True   # fp8: an Inception module's sibling 1x1 convs as one multi-output GEMM
    fuse_preprocess_stem: bool = True  # resize-free preprocess folded into the s2d RGB stem conv
    fuse_block_tails: bool = True      # ResNet block boundary: expand + next reduce in one kernel
    decimate_tails: bool = True        # stage-1 tail output stored at the stride-2 reader's pixels
    recompute_tails: bool = True       # stage-1 residual stream recomputed from 64-ch sources, not re-read
    chain_max_links: int = 2           # ... over at most this many links (3: -2 %, profiles/r06_chain)
    pw_res_kernel: bool = True         # identity-residual expand convs on the persistent kernel
    conv3x3c64_kernel: bool = True     # 64-channel 3x3 convs with the filter bank in LDS
    # cache-resident batch slices: the plan's leading run of large-activation layers (every
    # tensor >= chain_min_hw pixels per image: Inception-v3's 149x149 .. 71x71 stem) runs once
    # per slice of chain_batch images, its intermediates in slice-sized buffers that stay in
    # the 256 MiB Infinity Cache.  -1 = auto (32-image slices, never over a persistent
    # weight-resident kernel: ResNet-50's stage 1 measured slower sliced), 0 = off
    chain_batch: int = -1
    chain_min_hw: int = 5041
    chain_edge: bool = True            # ... plus the layers leaving that resolution (stride-2 readers)
    wd_fused_step: bool = True         # Wide&Deep: hand-fused GPU step instead of autograd
    # Wide&Deep under DP (parallel/sparse_exchange.py): "owner" (default) = deduplicated rows
    # to their owner rank (row % world), owner-side Adagrad, updated rows back, with exact
    # per-step sizes (host-synced counts, not capturable); "bucketed" = the same in
    # fixed-capacity per-peer buckets — static shapes, no host sync, the DP step captured in
    # a hipGraph — whose overflow (CapacityExceeded) is recovered by a job restart with
    # doubled slack, so a job operator refuses it without a restart strategy;
    # "allgather" = the padded all-gather of one row per lookup (capturable, most bytes)
    wd_sparse_exchange: str = "owner"
    wd_bucket_slack: float = 2.0       # bucket capacity = slack x (slots / world) + 64
    extra: dict = field(default_factory=dict)

    # ------------------------------------------------------------------ sources
    @classmethod
    def field_names(cls) -> list[str]:
        return [f.name for f in dataclasses.fields(cls) if f.name != "extra"]

    def _coerce(self, name: str, value: Any) -> Any:
        cur = getattr(self, name)
        typ = {f.name: f.type for f in dataclasses.fields(self)}[name]
        if value is None:
            return None
        if isinstance(value, str):
            if "tuple" in str(typ):
                return tuple(int(v) for v in value.replace(" ", "").split(",") if v)
            if "bool" in str(typ):
                return value.lower() in ("1", "true", "yes", "on")
            if "int" in str(typ) and "float" not in str(typ):
                return int(value)
            if "float" in str(typ):
                return float(value)
            return value
        if isinstance(cur, tuple) and isinstance(value, (list, tuple)):
            return tuple(value)
        return value

    def update(self, values: dict) -> "EngineConfig":
        for k, v in values.items():
            if k in self.field_names():
                setattr(self, k, self._coerce(k, v))
            else:
                self.extra[k] = v
        self.validate()
        return self

    @classmethod
    def from_yaml(cls, path: str, base: "EngineConfig | None" = None) -> "EngineConfig":
        import yaml

        with open(path) as f:
            data = yaml.safe_load(f) or {}
        return (base or cls()).update(data)

    @classmethod
    def from_env(cls, base: "EngineConfig | None" = None, prefix: str = "FT_", environ=None) -> "EngineConfig":
        environ = os.environ if environ is None else environ
        vals = {}
        for name in cls.field_names():
            key = prefix + name.upper()
            if key in environ:
                vals[name] = environ[key]
        return (base or cls()).update(vals)

    @classmethod
    def add_arguments(cls, ap: argparse.ArgumentParser) -> None:
        for name in cls.field_names():
            ap.add_argument("--" + name.replace("_", "-"), dest=f"cfg_{name}", default=None)
        ap.add_argument("--config", dest="cfg_yaml", default=None, help="YAML engine config")

    @classmethod
    def load(cls, argv: list[str] | None = None, environ=None) -> "EngineConfig":
        """defaults → YAML (``--config`` or ``FT_CONFIG``) → ``FT_*`` env → CLI flags."""
        ap = argparse.ArgumentParser(add_help=False)
        cls.add_arguments(ap)
        ns, _ = ap.parse_known_args(argv if argv is not None else [])
        environ = os.environ if environ is None else environ
        cfg = cls()
        yml = ns.cfg_yaml or environ.get("FT_CONFIG")
        if yml:
            cfg = cls.from_yaml(yml, cfg)
        cfg = cls.from_env(cfg, environ=environ)
        cli = {n: getattr(ns, f"cfg_{n}") for n in cls.field_names() if getattr(ns, f"cfg_{n}") is not None}
        return cfg.update(cli)

    # ------------------------------------------------------------------ checks / use
    def validate(self) -> None:
        if self.parallelism < 1:
            raise ValueError("parallelism must be >= 1")
        if self.max_batch < 1 or self.max_delay_ms < 0:
            raise ValueError("max_batch >= 1 and max_delay_ms >= 0 required")
        if self.precision not in ("bf16", "fp8"):
            raise ValueError("precision must be bf16 or fp8")
        if not 0 < self.arena_fraction <= 1:
            raise ValueError("arena_fraction must be in (0, 1]")
        if self.wd_sparse_exchange not in ("bucketed", "owner", "allgather"):
            raise ValueError("wd_sparse_exchange must be bucketed, owner or allgather")
        if self.wd_bucket_slack <= 0:
            raise ValueError("wd_bucket_slack must be positive")
        if self.batch_buckets and sorted(self.batch_buckets) != list(self.batch_buckets):
            self.batch_buckets = tuple(sorted(self.batch_buckets))

    def arena_bytes(self, device=None) -> int:
        """HBM budget of one subtask's plans (288 GB per MI355X unless the device says)."""
        total = _HBM_BYTES_MI355X
        try:
            import torch

            if device is not None and torch.cuda.is_available():
                total = torch.cuda.get_device_properties(device).total_memory
        except Exception:  # noqa: BLE001
            pass
        return int(total * self.arena_fraction)

    def apply(self, env) -> Any:
        """Configures a ``StreamExecutionEnvironment`` and exposes the config to operators."""
        from .runtime.checkpoint import RestartStrategy

        set_current(self)
        env.set_parallelism(self.parallelism)
        env.config.channel_capacity = self.channel_capacity
        env.config.global_job_parameters["engine"] = self
        if self.checkpoint_interval_s and self.checkpoint_dir:
            env.enable_checkpointing(self.checkpoint_interval_s, self.checkpoint_dir)
        if self.restart_attempts > 0:
            env.set_restart_strategy(RestartStrategy.fixed_delay(self.restart_attempts, self.restart_delay_s))
        import logging

        logging.getLogger("flink_tensorflow_amd").setLevel(self.log_level.upper())
        return env

    def to_dict(self) -> dict:
        d = dataclasses.asdict(self)
        d["batch_buckets"] = list(self.batch_buckets)
        return d


_CURRENT: EngineConfig | None = None


def current() -> EngineConfig:
    """The process's engine configuration: the one last applied to an environment, else
    defaults + ``FT_*`` environment variables (read once).  The graph compiler and the
    model zoo read their kernel-selection fields from here."""
    global _CURRENT
    if _CURRENT is None:
        _CURRENT = EngineConfig.from_env()
    return _CURRENT


def set_current(cfg: EngineConfig | None) -> None:
    global _CURRENT
    _CURRENT = cfg


@contextlib.contextmanager
def override(**fields):
    """Temporarily replaces fields of the current configuration (tests, A/B benches)."""
    old = current()
    new = dataclasses.replace(old, extra=dict(old.extra))
    new.update(fields)
    set_current(new)
    try:
        yield new
    finally:
        set_current(old)
