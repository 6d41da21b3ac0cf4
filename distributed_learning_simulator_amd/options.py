"""Runtime options of the engine and kernels: one object, read at call time.

These are measurement / comparison switches (alternating A/B runs, tests), not part of the
experiment config surface of the reference. They used to be import-time module constants
(`DLS_*` environment variables read once when a module loaded), so a session could not change
them and tests had to patch module globals. Now:

* `OPTIONS` holds every switch; the code paths read `OPTIONS.<name>` when they run;
* the environment variables of the same switches still seed the defaults (scripts/ab_env.sh);
* a run can set them from its config (`runtime_options: {planes: false, streams: 1}` in the
  YAML or `++<group>.runtime_options.streams=1` on the command line; Session applies them),
  programmatically (`options.update(streams=1)`), or for a block (`with options.override(...)`);
* the native launch knobs (tile rules of csrc/) are forwarded to the extension
  (`set_native_option`) when set.

Defaults are the measured-best settings; each field's comment says what the other setting does.
"""

from __future__ import annotations

import contextlib
import dataclasses
import os
import threading


def _env_bool(name: str, default: bool) -> bool:
    v = os.environ.get(name)
    return default if v is None else v not in ("0", "", "false", "False")


def _env_int(name: str, default: int) -> int:
    v = os.environ.get(name)
    return default if v is None or v == "" else int(v)


@dataclasses.dataclass
class RuntimeOptions:
    # --- fp32 (split-bf16) activation operands
    planes: bool = dataclasses.field(default_factory=lambda: _env_bool("DLS_PLANES", True))
    """BatchNorms emit bf16 (hi, lo) planes for the LDS-DMA plane / halo GEMMs (off: every conv
    splits its operand in registers)."""
    fused_sgd: bool = dataclasses.field(default_factory=lambda: _env_bool("DLS_FUSED_SGD", True))
    """SGD steps of the weights whose plane / halo wgrad kernels can apply them (csrc/sgd_epi.h)
    run in those kernels; the flat step covers the rest (engine.params.FusedSGD)."""
    tfm_planes: bool = dataclasses.field(default_factory=lambda: _env_bool("DLS_TFM_PLANES", True))
    """Transformer split-plane producers: the FFN hidden activation and its gradient (linear1 /
    linear2 epilogues) and the dropout backward of the residual-branch linears (out_proj /
    linear2) write planes for the plane GEMMs (off: fp32 only). (Attention outputs writing planes
    measured +0.4-0.5 s per FedOBD stage-1 round each, profiles/r5_c6_ab_tfm_planes.txt: removed.)"""
    # --- BatchNorm fusions
    bn_bwd_parts: bool = dataclasses.field(default_factory=lambda: _env_bool("DLS_BN_BWD_PARTS", True))
    """BN backward partial sums from the consuming conv's dgrad epilogue (off: own reduction)."""
    bn_fused_halo: bool = dataclasses.field(default_factory=lambda: _env_bool("DLS_BN_FUSED_HALO", True))
    """A BN(+ReLU) whose only reader is a 3x3 stride-1 conv (ResNet BasicBlock bn1) is applied in
    that conv's halo loader (ops.functional DeferredBN; off: BN apply pass + plane conv)."""
    bn_res_fold: bool = dataclasses.field(default_factory=lambda: _env_bool("DLS_BN_RES_FOLD", True))
    """A ResNet downsample shortcut's BN is applied inside the block's last BN apply, which reads
    its raw input as the residual (ops.functional DeferredRes; off: its own apply pass)."""
    dense_bn_halo: bool = dataclasses.field(default_factory=lambda: _env_bool("DLS_DENSE_BN_HALO", True))
    """DenseNet growth convs apply their BN + ReLU in the halo loader over the block buffer's
    channel prefix (off: BN apply pass + implicit-GEMM conv)."""
    halo_wgrad: bool = dataclasses.field(default_factory=lambda: _env_bool("DLS_HALO_WGRAD", True))
    """3x3 stride-1 weight gradients of 64-512-channel convs (ResNet layers 1-3) on the LDS-halo
    kernel (csrc/conv_halo_wgrad.hip; off: the implicit-GEMM TN kernel)."""
    bn_bwd_in_wgrad: bool = dataclasses.field(default_factory=lambda: _env_bool("DLS_BN_BWD_IN_WGRAD", True))
    """A training BN(+ReLU) whose input gradient feeds only a 3x3 stride-1 conv's backward (ResNet
    BasicBlock bn1 / identity-block bn2, layers 1-3) computes its coefficients only: that conv's halo
    weight gradient applies the BN backward in its dY loader and writes dX's planes for the dgrad
    (ops.functional DeferredBNBwd; off: the BN backward's own apply pass writes them)."""
    dense_wgrad_halo: bool = dataclasses.field(default_factory=lambda: _env_bool("DLS_DENSE_WGRAD_HALO", True))
    """DenseNet growth-conv weight gradients on the LDS-halo kernel (the normalised prefix staged
    once per pixel tile for all nine taps; off: the implicit-GEMM TN kernel)."""
    dense_dgrad_fused: bool = dataclasses.field(default_factory=lambda: _env_bool("DLS_DENSE_DGRAD_FUSED", True))
    """DenseNet growth-conv input gradients fused with the BN backward (csrc/conv_dense_dgrad.hip:
    dX̂ recomputed in a sums pass and an apply pass instead of stored and read twice; off: the
    implicit-GEMM dgrad + the BN backward passes)."""
    dense_y_recompute: bool = dataclasses.field(default_factory=lambda: _env_bool("DLS_DENSE_Y_RECOMPUTE", True))
    """With the fused dgrad and the halo weight gradient, DenseNet training stores no normalised
    activation: both backward kernels rebuild relu(BN(x)) from the raw prefix and the forward's
    (scale, shift), bitwise (off: the forward's halo conv writes it for them)."""
    dense_stats_cache: bool = dataclasses.field(default_factory=lambda: _env_bool("DLS_DENSE_STATS_CACHE", True))
    """DenseNet blocks (fused growth convs) sum each channel's statistics once, from the producing
    conv's epilogue, into running fp64 sums the BN coefficients read (off: a statistics pass over
    the prefix per layer)."""
    # --- reductions
    deterministic: bool = dataclasses.field(default_factory=lambda: _env_bool("DLS_DETERMINISTIC", True))
    """Split-K weight gradients and column sums folded in a fixed order (off: fp32 atomics)."""
    # --- step execution
    streams: int = dataclasses.field(default_factory=lambda: _env_int("DLS_STREAMS", 2))
    """Sub-cohort HIP streams trained concurrently on one GPU."""
    ragged_steps: bool = dataclasses.field(default_factory=lambda: _env_bool("DLS_RAGGED_STEPS", True))
    """A cohort's clients are ordered by shard size, so in an epoch's last steps (where only the
    clients with the largest shards still have a batch) the active clients are a row prefix and
    the step runs those rows only (off: every step runs all K rows, idle ones masked)."""
    skip_invalid: bool = dataclasses.field(default_factory=lambda: _env_bool("DLS_SKIP_INVALID", True))
    """Halo convolutions skip the images past a client's valid samples (a partial last batch):
    weight gradients because their dY and X are zeros written by the BatchNorms, forward / dgrad
    tiles whose only readers are BatchNorm passes that stop at the valid rows (off: computed)."""
    graphs: bool = dataclasses.field(default_factory=lambda: _env_bool("DLS_GRAPHS", True))
    """HIP-graph replay of whole training steps (off: eager steps)."""
    max_graphs: int = dataclasses.field(default_factory=lambda: _env_int("DLS_MAX_GRAPHS", 3))
    """Captured step graphs kept per trainer (each owns a private memory pool): a round uses the
    full cohort's and its ragged epoch-end step's (ragged_steps)."""
    eval_max_images: int = dataclasses.field(default_factory=lambda: _env_int("DLS_EVAL_MAX_IMAGES", 4096))
    """Images per evaluation launch (M models x batches): larger launches fill the GPU better and
    cost activation memory; past 4096 they measured slower (GTG utility of 32 models: 38.8 ms per
    model at 4096 vs 39.9 at 8192 and 40.5 at 16384, profiles/r6_c16_eval_max_images.log; the
    headline's one-model test pass equal). Per sub-cohort stream: evaluate() keeps up to `streams` launches in
    flight on separate streams (whose freed blocks the caching allocator does not share), so its
    peak activation memory is about streams x this many images' worth."""
    shared_planes: bool = dataclasses.field(default_factory=lambda: _env_bool("DLS_SHARED_PLANES", True))
    """Shared-model steps (sign-SGD / sync-SGD): every client reads the one shared row's weight
    planes (rep = K) and its activations' planes (off: register-split GEMMs; sign-SGD ResNet-50
    3.51 vs 3.18 s per vote step)."""
    # --- native launch knobs (csrc/, forwarded to the extension; None = the kernel's own default)
    native: dict = dataclasses.field(default_factory=dict)
    """e.g. {"pl_min_wg": 0, "conv_gl": 0, "attn_mfma": 0, "halo_wgrad_unroll": 2}."""


OPTIONS = RuntimeOptions()
_FIELDS = {f.name for f in dataclasses.fields(RuntimeOptions)}


_NATIVE_UNSET = -1000000  # (csrc/dls.h kOptUnset: back to the environment / kernel default)


def _push_native(native: dict) -> None:
    if not native:
        return
    try:
        from .ops import hip
    except ImportError:  # no extension (CPU box): nothing to forward
        return
    for k, v in native.items():
        hip._C.set_native_option(str(k), _NATIVE_UNSET if v is None else int(v))


def update(**kw) -> dict:
    """Set options; returns the previous values of the ones changed."""
    old = {}
    for k, v in kw.items():
        if k not in _FIELDS:
            raise KeyError(f"unknown runtime option {k!r}; known: {sorted(_FIELDS)}")
        old[k] = getattr(OPTIONS, k)
        if k == "native":
            merged = dict(OPTIONS.native)
            merged.update(v or {})
            v = {n: x for n, x in merged.items() if x is not None}
        else:
            v = type(old[k])(v)
        setattr(OPTIONS, k, v)
    if "native" in kw:
        _push_native(kw["native"] or {})
    if "skip_invalid" in kw:  # (mirrored by the native halo launches, csrc/dls.h g_opt_halo_skip)
        _push_native({"halo_skip": int(OPTIONS.skip_invalid)})
    return old


def _restore(old: dict, kw: dict) -> None:
    """Undo update(**kw), given the previous values it returned."""
    old = dict(old)
    native_prev = old.pop("native", None)
    for k, v in old.items():
        setattr(OPTIONS, k, v)
    if native_prev is not None:  # knobs the update set go back to their previous value (or unset)
        update(native={n: native_prev.get(n) for n in (kw.get("native") or {})})


@contextlib.contextmanager
def override(**kw):
    """Temporarily set options (tests, A/B loops)."""
    old = update(**kw)
    try:
        yield OPTIONS
    finally:
        _restore(old, kw)


def config_options(config) -> dict:
    """A run's `runtime_options:` mapping (config extra key)."""
    extra = getattr(config, "extra", None) or {}
    return dict(extra.get("runtime_options") or {})


_scope_lock = threading.Lock()
_scope = {"count": 0, "opts": None, "saved": None}


@contextlib.contextmanager
def scoped(opts: dict | None):
    """A run's runtime options for its duration (Session.__init__ / Session.run): applied when the
    first run in the process enters, restored when the last one leaves — they never leak into a
    later run. The kernels read the process-wide OPTIONS while they run, so concurrent runs
    (training.train with practitioners: threads) must agree on them: a run whose options differ
    from those of the runs in flight is refused instead of switching their kernels mid-step."""
    opts = dict(opts or {})
    with _scope_lock:
        if _scope["count"] and opts != _scope["opts"]:
            raise RuntimeError(f"concurrent runs with different runtime_options: {opts} vs {_scope['opts']}")
        if _scope["count"] == 0:
            _scope["saved"] = update(**opts) if opts else {}
            _scope["opts"] = opts
        _scope["count"] += 1
    try:
        yield OPTIONS
    finally:
        with _scope_lock:
            _scope["count"] -= 1
            if _scope["count"] == 0:
                _restore(_scope["saved"], _scope["opts"])
                _scope["saved"] = _scope["opts"] = None


def apply_config(config) -> None:
    """Set a run's `runtime_options:` process-wide, unscoped (scripts; Session uses `scoped`)."""
    opts = config_options(config)
    if opts:
        update(**opts)
