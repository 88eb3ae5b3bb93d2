"""The one diagnostic switchboard: ``DISTRIFLOW_DIAG="name=value,name=value"``.

Measurement aids only — A/B switches for engine variants that were measured (docs/RESULTS.md) and
either lost or came out neutral, plus the escape hatches of the fused fast paths.  Production never
sets ``DISTRIFLOW_DIAG``; every switch defaults to the shipped path.  The native kernels read the same
variable (csrc/diag.h).  User-facing configuration (``DISTRIFLOW_BACKEND``, ``DISTRIFLOW_ALLREDUCE``,
the watchdog timeouts, ``DISTRIFLOW_METRICS``, ``DISTRIFLOW_DEBUG_SYNC``) is not here: see config.py.

Python switches (default in brackets):
  lenet_fused [1]          whole-network LeNet-5 kernels (0: per-layer kernels)
  lenet_fused_update [1]   the reduce launch applies the SGD update (0: separate optimizer launch)
  async_fused [1]          async PS step = train + reduce/apply (0: pull / compute / apply launches)
  ps_excl_fused [1]        async PS with one rank, models other than the fused LeNet-5: admission + next claim
                           in one workgroup and the model's optimizer launch gated on the decision (0: pull /
                           refresh / compute / ps_apply launches)
  ps_owner_apply [-1]      async PS apply path at world > 1: 1 owner-applies (gradients pushed into the shard
                           owners' inbox rings with plain stores, drained into the shards in sequence order by
                           the lock holder; no remote atomics), 0 per-element CAS adds, -1 both timed at setup on
                           the real topology and the faster taken (AsyncPSTrainer._calibrate_apply)
  kcnn_fused [1]           the reference CNN's conv block as one forward + one backward kernel
  fold_dropout [1]         dropout folded into producer epilogues
  khead_fused [1]          the reference CNN's dense head (4608 -> 128 -> C + CE) as one split-K launch
                           plus the fused head weight-gradient launch (0: per-layer GEMMs + head kernels)
  lenet_succ [1]           LeNet-5 reduce launch: successor ownership (each slot's partials handed to the next
                           slot's workgroups as {epoch, value} granules; 0: arrival tickets + slab reload)
  multistep [1]            bench.py unrolls up to 64 steps per hipGraph (0: one replay per step)
  graph_steps [64]         most steps unrolled into one multi-step hipGraph
  fused_selftest [1]       real-kernel self-test of the multi-rank fused LeNet-5 step before its first use
                           (0: trust the LL exchange's own setup self-test)
  wgrad_overlap [0]        ResNet weight gradients on a side stream (round 2: +3 %; with the halo-tiled
                           kernels, whose workgroups fill whole CUs, in-order is faster: 83.7 k vs 79.5 k
                           images/s, profiles/r3/resnet18_b256_stream_overlap_ab.txt)
  proj_overlap [0]         ResNet projection shortcut on a side stream (in order is faster with the halo
                           kernels: 87.0 k vs 85.0 k images/s, profiles/r3/resnet18_b256_inorder_ab.txt)
  concurrent_backward [0]  head weight gradients on side streams (measured slower)
  bn_fused [0]             BatchNorm statistics and the apply / dx pass in one launch (in-launch hand-off to
                           the resident workgroups).  Correct (tests/test_kernels_gpu.py), but the hand-off
                           chain stays and the streaming pass runs at the statistics grid: ResNet-18 B=256
                           83.4 k vs 85.0 k images/s (profiles/r4/resnet18_bn_fused_ab.txt)
  bn_acc [1]               BatchNorm statistics accumulated by the producing kernels' epilogues (fp64 adds into
                           replicas, csrc/bn_acc.h) and finalised by the consuming apply / dx pass: no
                           statistics launches (0: the statistics passes of csrc/bn.hip, bitwise reproducible)
  bn_acc_rep [8]           accumulator replicas per BatchNorm and direction (1..16)
  bn_epilogue [0]          BatchNorm statistics finalised inside the producing conv launches instead of
                           separate statistics passes (correct, but the write-through + ticket tail each
                           conv workgroup then pays costs more than the passes: ResNet-18 B=256 72.3 k vs
                           73 k images/s, profiles/r3/resnet18_bn_in_launch_step.txt)
"""
from __future__ import annotations

import os

_DEFAULTS = {"lenet_fused": 1, "lenet_fused_update": 1, "async_fused": 1, "ps_owner_apply": -1, "ps_excl_fused": 1, "kcnn_fused": 1, "khead_fused": 1, "fold_dropout": 1,
             "lenet_succ": 1, "multistep": 1, "graph_steps": 64, "fused_selftest": 1, "wgrad_overlap": 0, "proj_overlap": 0, "concurrent_backward": 0, "bn_epilogue": 0,
             "bn_fused": 0, "bn_acc": 1, "bn_acc_rep": 8}


def diag(name: str) -> int:
    """Value of switch ``name`` (its documented default unless DISTRIFLOW_DIAG overrides it)."""
    if name not in _DEFAULTS:
        raise KeyError(f"unknown diagnostic switch {name!r}")
    spec = os.environ.get("DISTRIFLOW_DIAG", "")
    for item in spec.split(","):
        k, _, v = item.strip().partition("=")
        if k == name and v:
            return int(v)
    return _DEFAULTS[name]


def on(name: str) -> bool:
    return diag(name) != 0


def active() -> dict:
    """Every switch set away from its default (recorded by bench.py so a diagnostic run is never
    mistaken for a production number)."""
    return {k: diag(k) for k in _DEFAULTS if diag(k) != _DEFAULTS[k]}
