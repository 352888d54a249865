"""One typed, validated, rank-checked run-time configuration for the whole framework.

Every switch that changes which kernels or algorithms run lives here as a field of the frozen
:class:`Config` dataclass. The process's configuration is read ONCE from the environment (the
``BH_*`` variable named next to each field), validated (an unknown value raises instead of silently
falling back), and then only changed through :func:`set` / :func:`override`. The native extension
gets its switches from here too (``_C.set_knobs``, csrc/include/bh/knobs.h): no kernel or Python
module reads ``os.environ`` for a run-time decision any more.

Ranks must agree: a rank that runs another fold mode or loss-scaler mode computes different numbers
and may issue different collectives. :func:`check_ranks` all-gathers a digest of the configuration
and raises on the first mismatch; ``parallel.DistributedDataParallel`` and ``bench.py`` call it when
a multi-rank process group is up.

Round 5 removed the A/B switches whose losing side had been kept in the code (second-stream weight
gradients and their reductions, the 3x3 BatchNorm-sums epilogue, 64-channel igemm tiles, the
c1x1 occupancy target, register-staged GEMM loads, the 16-wide flash kernels, the BatchNorm launch
geometry overrides): their measurements stay in profiles/, the code paths are gone.

Not configuration (left as environment variables on purpose): build flags (``BH_ARCH``,
``BH_DEBUG``, ``BH_AUTOBUILD``, _build.py / _native.py) and test-harness plumbing
(``BH_TEST_WORLD_SIZE``, ``BH_DIST_TEST_CHILD``, ``BH_ARGS_VERBOSE``, ``BH_TEST_OPDUMP``).
"""
from __future__ import annotations

import contextlib
import dataclasses
import hashlib
import os
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional

_BOOL = {"1": True, "true": True, "on": True, "yes": True, "0": False, "false": False, "off": False, "no": False}


@dataclass(frozen=True)
class Config:
    # -- amp
    amp_device_scaler: bool = field(default=False, metadata=dict(env="BH_AMP_DEVICE_SCALER", doc=(
        "device-resident dynamic loss scale: no host sync per step, overflow skips on the device")))
    amp_python_scaler: bool = field(default=False, metadata=dict(env="BH_AMP_PYTHON_SCALER", doc=(
        "the reference's python-only scaler (per-tensor checks, no multi-tensor kernel); tests")))
    amp_fused_master_step: bool = field(default=False, metadata=dict(env="BH_AMP_FUSED_MASTER", doc=(
        "opt-in, O2/O5 + FusedLAMB/FusedAdam: the step reads the scaled 16-bit grads and writes the model "
        "copy; the fp32 master .grad stay None until amp.master_params() (clip through it, not param_groups)")))
    # -- ResNet / convolution paths (models/resnet.py)
    fold_bn: bool = field(default=True, metadata=dict(env="BH_FOLD_BN", doc=(
        "BatchNorm statistics / apply folded into the convolutions")))
    fold_apply: str = field(default="all", metadata=dict(env="BH_FOLD_APPLY", choices=("all", "bn1", "bn2", "none"),
                                                         doc="which BatchNorm applies run inside the next conv"))
    bn_res_fold: str = field(default="pro", metadata=dict(env="BH_BN_RES_FOLD", choices=("pro", "all", "off"),
                                                          doc="bottleneck tail (conv3 + bn3 + residual) as one node"))
    ds_fold: str = field(default="stride1", metadata=dict(env="BH_DS_FOLD", choices=("off", "stride1", "all"),
                                                          doc="downsample BatchNorm folded into the tail node"))
    mask_producer: str = field(default="any", metadata=dict(env="BH_MASK_PRODUCER", choices=("off", "fast", "any"),
                                                            doc="residual ReLU mask applied in conv1's dgrad"))
    stem_stats: bool = field(default=True, metadata=dict(env="BH_STEM_STATS", doc=(
        "the stem conv's epilogue reduces the stem BatchNorm statistics")))
    own_gemm: str = field(default="fwd,plain", metadata=dict(env="BH_OWN_GEMM", doc=(
        "comma list of {fwd, bwd, plain, resid}: strip/ping-pong GEMMs instead of hipBLASLt")))
    conv_tune: bool = field(default=False, metadata=dict(env="BH_CONV_TUNE", doc=(
        "time own vs MIOpen per conv shape (rank 0's pick broadcast)")))
    conv3x3_bwd_epi: bool = field(default=False, metadata=dict(env="BH_CONV3X3_BWD_EPI", doc=(
        "stride-1 3x3 data gradient of a BatchNorm-prologue conv reduces that BatchNorm's backward sums "
        "in its epilogue (no separate reduction pass)")))
    conv_wgrad: str = field(default="own", metadata=dict(env="BH_CONV_WGRAD", choices=("own", "miopen"),
                                                         doc="weight gradients of the stride-1 convs"))
    conv1x1_s2: str = field(default="wgrad", metadata=dict(env="BH_CONV1X1_S2", choices=("wgrad", "gather", "miopen"),
                                                           doc="stride-2 1x1 conv paths"))
    gemm_n64: bool = field(default=True, metadata=dict(env="BH_GEMM_N64", doc=(
        "the streaming 64-column MFMA GEMM for the 64-channel 1x1 convs")))
    syncbn_stats: str = field(default="allreduce", metadata=dict(env="BH_SYNCBN_STATS",
                                                                 choices=("allreduce", "allgather"),
                                                                 doc="SyncBN statistics exchange"))
    groupbn_ipc: bool = field(default=True, metadata=dict(env="BH_GROUPBN_IPC", doc=(
        "contrib.groupbn exchanges statistics over HIP IPC peer memory")))
    # -- transformer paths
    mha_fused: bool = field(default=True, metadata=dict(env="BH_MHA_FUSED", doc="MFMA fused attention kernels"))
    attn_flash_only: bool = field(default=False, metadata=dict(env="BH_ATTN_FLASH_ONLY", doc=(
        "flash kernels also for sk <= 128 (benchmarks)")))
    fused_mlp: bool = field(default=True, metadata=dict(env="BH_FUSED_MLP", doc="fused MLP block in transformer_lm"))
    flash_attn: bool = field(default=True, metadata=dict(env="BH_FLASH_ATTN", doc="flash attention in transformer_lm"))
    dense_wgrad_mfma: bool = field(default=True, metadata=dict(env="BH_DENSE_WGRAD", native="dense_wgrad", doc=(
        "dense weight gradients on the MFMA kernels (gemm_tn / 1x1 wgrad, bindings/dense.cpp weight_grad)")))
    embed_native: bool = field(default=True, metadata=dict(env="BH_EMBED_NATIVE", doc="native embedding backward"))
    ln_residual_grad: bool = field(default=True, metadata=dict(env="BH_LN_RESID", doc=(
        "pre-LN blocks: the residual add's input gradient is summed inside the LayerNorm dx kernel")))
    gemm_table: str = field(default="", metadata=dict(env="BH_GEMM_TABLE", doc=(
        "tuned GEMM dispatch table path ('' = the packaged default)")))
    # -- native switches (pushed into the extension, bh::knob)
    dense_mfma: bool = field(default=True, metadata=dict(env="BH_DENSE_MFMA", native="dense_mfma", doc=(
        "FusedDense / MLP GEMMs with fused epilogues on the MFMA kernel")))
    dense_tune: bool = field(default=False, metadata=dict(env="BH_DENSE_TUNE", native="dense_tune", doc=(
        "time MFMA vs hipBLASLt per dense shape once")))
    gemm_tile: int = field(default=0, metadata=dict(env="BH_GEMM_TILE", native="gemm_tile", choices=(0, 1, 2, 3, 4),
                                                    doc="GEMM tile: 0 auto, 1 small, 2 big, 3 mid, 4 ping-pong"))
    conv3x3_nb: int = field(default=2, metadata=dict(env="BH_CONV3X3_NB", native="conv3x3_nb", choices=(2, 3), doc=(
        "direct 3x3 conv: LDS weight buffers (3: next step's fragments pre-read; measured 0.5% slower "
        "end to end, profiles/conv3x3_nb_sw_ab_r6.txt)")))
    conv3x3_sw: bool = field(default=False, metadata=dict(env="BH_CONV3X3_SW", native="conv3x3_sw", doc=(
        "direct 3x3 conv, plain epilogue: operands swapped so it stores 8-byte channel runs (measured "
        "slower, profiles/conv3x3_nb_sw_ab_r6.txt)")))
    ln_bwd_fused: bool = field(default=False, metadata=dict(env="BH_LN_BWD_FUSED", native="ln_bwd_fused", doc=(
        "LayerNorm backward: dx and the gamma / beta partials in one row-pipelined pass (else two passes; "
        "the two-pass backward measured 0.6 % faster per BERT-large step, profiles/ln_bwd_fused_ab_r6.txt)")))
    igemm_lds: bool = field(default=False, metadata=dict(env="BH_IGEMM_LDS", native="igemm_lds", doc=(
        "stride-2 3x3 implicit GEMM: both operands staged in LDS by LDS-DMA (measured slower than the "
        "register-staged A fragments, profiles/igemm_lds_ab_r6.txt)")))
    gemm_log: bool = field(default=False, metadata=dict(env="BH_GEMM_LOG", native="gemm_log", rank_checked=False,
                                                        doc="log the GEMM kernel picked per shape (debugging)"))

    def __post_init__(self):
        for f in dataclasses.fields(self):
            v = getattr(self, f.name)
            want = {"bool": bool, "str": str, "int": int}[f.type if isinstance(f.type, str) else f.type.__name__]
            if not isinstance(v, want) or (want is int and isinstance(v, bool)):
                raise TypeError(f"Config.{f.name} must be {want.__name__}, got {v!r}")
            choices = f.metadata.get("choices")
            if choices is not None and v not in choices:
                raise ValueError(f"Config.{f.name}={v!r}: expected one of {choices}")
        kinds = {k for k in self.own_gemm.split(",") if k}
        if not kinds <= {"fwd", "bwd", "plain", "resid"}:
            raise ValueError(f"Config.own_gemm={self.own_gemm!r}: kinds must be among fwd, bwd, plain, resid")

    @classmethod
    def from_env(cls, environ=None) -> "Config":
        env = os.environ if environ is None else environ
        kw = {}
        for f in dataclasses.fields(cls):
            raw = env.get(f.metadata["env"])
            if raw is None:
                continue
            kw[f.name] = _parse(f, raw)
        return cls(**kw)

    def digest(self) -> str:
        """Hash of every field that changes what a rank computes. Diagnostic fields
        (``rank_checked=False``) are left out, and the GEMM table enters by its CONTENT, so two ranks
        reading copies of one table at different paths agree."""
        parts = []
        for f in dataclasses.fields(self):
            if not f.metadata.get("rank_checked", True):
                continue
            v = getattr(self, f.name)
            if f.name == "gemm_table" and v:
                v = _file_digest(v)
            parts.append(f"{f.name}={v!r}")
        return hashlib.sha256(";".join(parts).encode()).hexdigest()[:16]

    def native_knobs(self) -> Dict[str, int]:
        return {f.metadata["native"]: int(getattr(self, f.name)) for f in dataclasses.fields(self)
                if "native" in f.metadata}


def _file_digest(path: str) -> str:
    try:
        with open(path, "rb") as fh:
            return "sha256:" + hashlib.sha256(fh.read()).hexdigest()
    except OSError:
        return "missing:" + os.path.basename(path)


# legacy spellings of the pre-config environment values
_ALIASES = {
    "bn_res_fold": {"0": "off", "1": "pro"},
    "ds_fold": {"0": "off", "1": "stride1"},
    "fold_apply": {"1": "all", "0": "none"},
    "mask_producer": {"0": "off", "1": "any"},
    "conv_wgrad": {"gemm": "own"},
    "conv1x1_s2": {"0": "miopen"},
    "own_gemm": {"1": "fwd,bwd,plain,resid", "all": "fwd,bwd,plain,resid", "0": "", "none": ""},
}


def _parse(f, raw: str):
    t = f.type if isinstance(f.type, str) else f.type.__name__
    name = f.metadata["env"]
    if t == "bool":
        v = _BOOL.get(raw.strip().lower())
        if v is None:
            raise ValueError(f"{name}={raw!r}: expected 0/1")
        return v
    if t == "int":
        try:
            return int(raw)
        except ValueError:
            raise ValueError(f"{name}={raw!r}: expected an integer") from None
    if f.name == "own_gemm":
        raw = ",".join(k.strip() for k in raw.strip().lower().split(",") if k.strip())
    return _ALIASES.get(f.name, {}).get(raw, raw)


_current: Optional[Config] = None
_listeners: List[Callable[[Config], None]] = []


def get() -> Config:
    """The process's configuration (read from the environment on first use)."""
    global _current
    if _current is None:
        _current = Config.from_env()
    return _current


def set(**changes) -> Config:  # noqa: A001 - module-level API: config.set(...)
    """Replace fields (validated); modules that cache switches and the native extension are updated."""
    global _current
    _current = dataclasses.replace(get(), **changes)
    _publish(_current)
    return _current


@contextlib.contextmanager
def override(**changes):
    """``with config.override(fold_bn=False): ...`` -- restored on exit."""
    old = get()
    set(**changes)
    try:
        yield get()
    finally:
        set(**dataclasses.asdict(old))


def on_change(fn: Callable[[Config], None]) -> None:
    """``fn(config)`` now and after every :func:`set` (modules that keep switches in globals)."""
    _listeners.append(fn)
    fn(get())


def push_native(module=None) -> None:
    """Hand the native switches to the extension (``_native`` calls this once it is loaded)."""
    mod = module
    if mod is None:
        from . import _native

        if not _native.available():
            return
        mod = _native.module()
    setter = getattr(mod, "set_knobs", None)
    if setter is not None:
        setter(get().native_knobs())


def _publish(c: Config) -> None:
    for fn in list(_listeners):
        fn(c)
    try:
        from . import _native

        if _native.loaded():
            push_native(_native.module())
    except ImportError:
        pass


def check_ranks(group=None) -> str:
    """All ranks of ``group`` run the same configuration (raises RuntimeError naming the first rank
    that differs); returns the digest. A no-op without an initialised multi-rank process group."""
    import torch
    import torch.distributed as dist

    d = get().digest()
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) <= 1:
        return d
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else "cpu"
    mine = torch.tensor([int(d, 16) & ((1 << 62) - 1)], dtype=torch.int64, device=dev)
    every = [torch.empty_like(mine) for _ in range(dist.get_world_size(group))]
    dist.all_gather(every, mine, group=group)
    vals = [int(t.item()) for t in every]
    for r, v in enumerate(vals):
        if v != vals[0]:
            raise RuntimeError(f"beforeholiday_amd.config differs between ranks (rank 0 vs rank {r}); "
                               f"this rank runs {describe()}")
    return d


def describe() -> str:
    c = get()
    return ", ".join(f"{f.name}={getattr(c, f.name)!r}" for f in dataclasses.fields(c))
