"""Read checkpoints written in the reference's ZeRO layout and load them into this framework.

Layout (reference runtime/engine.py:3259-3380 ``_save_checkpoint`` / ``_save_zero_checkpoint``,
runtime/zero/stage_1_and_2.py:2472-2512 ``state_dict``, runtime/zero/stage3.py ``_rigid_state_dict``,
checkpoint/constants.py):

  <dir>/<tag>/mp_rank_00_model_states.pt            ZeRO-0/1/2: ``module`` (bit16 weights),
                                                    ``param_shapes`` (per group: name -> shape),
                                                    ``lr_scheduler``, ``global_steps`` ...
  <dir>/<tag>/zero_pp_rank_<r>_mp_rank_00_model_states.pt   ZeRO-3 (per rank, ``param_shapes``)
  <dir>/<tag>/zero_pp_rank_<r>_mp_rank_00_optim_states.pt   ``optimizer_state_dict`` =
      stage 1/2: ``single_partition_of_fp32_groups`` (per group, this rank's unpadded fp32
                 partition), ``base_optimizer_state`` (torch state of the padded partition, or the
                 elastic per-group list), ``param_slice_mappings`` (per group: name ->
                 fragment_address(numel, start) inside this rank's partition), ``loss_scaler``
                 (a pickled LossScaler object), ``zero_stage`` (pickled ZeroStageEnum) ...
      stage 3:   ``fp32_flat_groups`` (per sub-group flat fp32 partitions; every parameter is
                 split on its own into ceil(numel / dp) pieces), ``optimizer_state_dict``.

Everything is read with ``torch.load(weights_only=True)``: the reference's pickled classes
(``DynamicLossScaler``, ``LossScaler``, ``ZeroStageEnum``, ``fragment_address``) are mapped to inert
stand-ins registered as safe globals under their reference import paths, so nothing from the file
is executed. The merged full fp32 weights and Adam moments are then written into the live engine
through the layout-independent ``safe_set_full_*`` API (utils/tensor_fragment.py), so a reference
checkpoint resumes under any ZeRO stage / data-parallel degree / slice layout of this framework.
Parity against files written by the reference itself is unpinned (the reference is not importable
here); the tests build files with the reference's key schema and pickled class paths.
"""
import collections
import dataclasses
import enum
import glob
import os
import re

import torch


# ------------------------------------------------------------------- inert stand-in classes
class _StandIn:
    """Attribute bag: the unpickler restores the object's __dict__ (BUILD) and nothing else."""

    def __init__(self, *a, **kw):
        pass

    def state(self):
        return dict(self.__dict__)


class RefLossScaler(_StandIn):
    pass


class RefDynamicLossScaler(_StandIn):
    pass


class RefZeroStageEnum(int, enum.Enum):
    disabled = 0
    optimizer_states = 1
    gradients = 2
    weights = 3


@dataclasses.dataclass
class RefFragmentAddress:
    numel: int = 0
    start: int = 0


_SAFE = [
    (RefLossScaler, "deepspeed.runtime.fp16.loss_scaler.LossScaler"),
    (RefDynamicLossScaler, "deepspeed.runtime.fp16.loss_scaler.DynamicLossScaler"),
    (RefZeroStageEnum, "deepspeed.runtime.zero.config.ZeroStageEnum"),
    (RefFragmentAddress, "deepspeed.utils.tensor_fragment.fragment_address"),
]


def load_file(path, mmap=True):
    """torch.load(weights_only=True) with the reference's pickled classes mapped to stand-ins;
    memory-mapped, so merging touches only the slices it copies."""
    with torch.serialization.safe_globals(_SAFE):
        return torch.load(path, map_location="cpu", weights_only=True, mmap=mmap)


# ------------------------------------------------------------------------------- discovery
def _tag_dir(checkpoint_dir, tag=None):
    if tag is None:
        with open(os.path.join(checkpoint_dir, "latest")) as f:
            tag = f.read().strip()
    return os.path.join(checkpoint_dir, str(tag))


def _rank_files(d, suffix):
    """Per-rank files; the reference's BF16_Optimizer writes them with a ``bf16_`` prefix
    (runtime/engine.py:2927)."""
    files = glob.glob(os.path.join(d, f"zero_pp_rank_*_mp_rank_00{suffix}"))
    if not files and suffix == "_optim_states.pt":
        files = glob.glob(os.path.join(d, f"bf16_zero_pp_rank_*_mp_rank_00{suffix}"))
    return sorted(files, key=lambda f: int(re.search(r"zero_pp_rank_(\d+)_", os.path.basename(f)).group(1)))


def is_reference_checkpoint(checkpoint_dir, tag=None):
    """True for a checkpoint in the reference's ZeRO layout (no ``unit_layout`` of this framework)."""
    try:
        d = _tag_dir(checkpoint_dir, tag)
    except OSError:
        return False
    files = _rank_files(d, "_optim_states.pt")
    if not files:
        return False
    osd = load_file(files[0]).get("optimizer_state_dict", {})
    return "unit_layout" not in osd and ("single_partition_of_fp32_groups" in osd or "fp32_flat_groups" in osd)


def _stage(osd):
    z = osd.get("zero_stage", 0)
    return int(z.value if isinstance(z, enum.Enum) else z)


def _numel(shape):
    n = 1
    for s in shape:
        n *= int(s)
    return n


# ---------------------------------------------------------------------------------- merging
def _base_states_12(osd, g, nranks_state):
    """Per-group optimizer state tensors of one rank: {key: flat tensor} (elastic or torch form)."""
    bos = osd.get("base_optimizer_state")
    if bos is None:
        return {}
    if isinstance(bos, list):  # elastic: per group lean (unpadded) state
        return {k: v for k, v in bos[g].items() if torch.is_tensor(v) and v.dim() == 1}
    st = bos.get("state", {}).get(g, {})
    return {k: v for k, v in st.items() if torch.is_tensor(v) and v.dim() == 1}


def _step_of(osds):
    osd = osds[0]
    if "base_optimizer_state_step" in osd:
        return int(osd["base_optimizer_state_step"])
    bos = osd.get("base_optimizer_state") or osd.get("optimizer_state_dict")
    if isinstance(bos, dict):
        for st in bos.get("state", {}).values():
            if "step" in st:
                s = st["step"]
                return int(s.item() if torch.is_tensor(s) else s)
        for pg in bos.get("param_groups", []):
            if "step" in pg:
                return int(pg["step"])
    return 0


def read_reference_checkpoint(checkpoint_dir, tag=None):
    """-> {"fp32": {name: tensor}, "state": {name: {key: tensor}}, "step": int, "zero_stage": int,
    "model_states": rank-0 model-states dict (bit16 ``module`` for stage 0/1/2), "loss_scaler": dict}."""
    d = _tag_dir(checkpoint_dir, tag)
    optim_files = _rank_files(d, "_optim_states.pt")
    if not optim_files:
        raise FileNotFoundError(f"no zero_pp_rank_*_optim_states.pt under {d}")
    osds = [load_file(f)["optimizer_state_dict"] for f in optim_files]
    stage = _stage(osds[0])
    if os.path.basename(optim_files[0]).startswith("bf16_") and "zero_stage" not in osds[0]:
        # BF16_Optimizer (reference runtime/bf16_optimizer.py:467-477): ZeRO-1 layout -- fp32
        # partitions + param_slice_mappings, base-optimizer state keyed by group index
        stage = 1
    world = len(osds)
    model_file = os.path.join(d, "mp_rank_00_model_states.pt")
    if not os.path.exists(model_file):
        zf = _rank_files(d, "_model_states.pt")
        model_file = zf[0] if zf else None
    ms = load_file(model_file) if model_file else {}
    shapes = ms.get("param_shapes")
    fp32, state = {}, collections.defaultdict(dict)
    if stage in (1, 2):
        groups = len(osds[0]["single_partition_of_fp32_groups"])
        for g in range(groups):
            maps = [o.get("param_slice_mappings", [None] * groups)[g] for o in osds]
            parts = [o["single_partition_of_fp32_groups"][g] for o in osds]
            sts = [_base_states_12(o, g, world) for o in osds]
            keys = set(sts[0]) if sts else set()
            if maps[0] is not None:  # exact per-rank fragments
                names = list(maps[0].keys())
                for m in maps[1:]:
                    names += [n for n in m.keys() if n not in names]
                for name in names:
                    frags = [(r, m[name]) for r, m in enumerate(maps) if name in m]
                    fp32[name] = torch.cat([parts[r].narrow(0, fa.start, fa.numel) for r, fa in frags])
                    for k in keys:
                        state[name][k] = torch.cat([sts[r][k].narrow(0, fa.start, fa.numel) for r, fa in frags])
            else:  # walk the group's parameter order over the rank-concatenated partitions
                flat = torch.cat(parts)
                flat_st = {k: torch.cat([s[k] for s in sts]) for k in keys}
                off = 0
                for name, shp in shapes[g].items():
                    n = _numel(shp)
                    fp32[name] = flat.narrow(0, off, n)
                    for k in keys:
                        state[name][k] = flat_st[k].narrow(0, off, n)
                    off += n
    elif stage == 3:
        flats = [torch.cat(o["fp32_flat_groups"]) for o in osds]
        tsd = [o.get("optimizer_state_dict", {}) for o in osds]
        keys = set()
        if tsd[0].get("state"):
            keys = {k for k, v in next(iter(tsd[0]["state"].values())).items() if torch.is_tensor(v) and v.dim() == 1}
        flat_st = {k: [torch.cat([tsd[r]["state"][i][k] for i in sorted(tsd[r]["state"])]) for r in range(world)]
                   for k in keys}
        merged = collections.OrderedDict()
        for grp in shapes:
            merged.update(grp)
        off = 0
        for name, shp in merged.items():
            n = _numel(shp)
            part = -(-n // world)
            fp32[name] = torch.cat([f.narrow(0, off, part) for f in flats]).narrow(0, 0, n)
            for k in keys:
                state[name][k] = torch.cat([f.narrow(0, off, part) for f in flat_st[k]]).narrow(0, 0, n)
            off += part
    else:
        raise ValueError(f"reference checkpoint with zero_stage {stage}: use the module weights directly")
    for name, shp in (ms.get("param_shapes") and
                      {k: v for grp in ms["param_shapes"] for k, v in grp.items()} or {}).items():
        if name in fp32:
            fp32[name] = fp32[name].reshape(shp)
            for k in state.get(name, {}):
                state[name][k] = state[name][k].reshape(shp)
    ls = osds[0].get("loss_scaler")
    ls = ls.state() if isinstance(ls, _StandIn) else (ls if isinstance(ls, dict) else {})
    return {"fp32": fp32, "state": dict(state), "step": _step_of(osds), "zero_stage": stage,
            "model_states": ms, "loss_scaler": ls, "dp_world_size": world}


# ---------------------------------------------------------------------------------- loading
def load_reference_checkpoint(engine, checkpoint_dir, tag=None, load_optimizer_states=True,
                              load_lr_scheduler_states=True, strict=True):
    """Resume ``engine`` from a reference-layout ZeRO checkpoint (any saved stage / dp degree)."""
    from ..utils.tensor_fragment import safe_set_full_fp32_param, safe_set_full_optimizer_state
    ck = read_reference_checkpoint(checkpoint_dir, tag)
    names = {p: n for n, p in engine.module.named_parameters()}
    missing = [n for p, n in names.items() if p.requires_grad and n not in ck["fp32"]]
    if strict and missing:
        raise KeyError(f"reference checkpoint lacks parameters: {missing[:5]}{' ...' if len(missing) > 5 else ''}")
    opt = engine.optimizer
    key_map = {"exp_avg": "exp_avg", "exp_avg_sq": "exp_avg_sq", "sum": "sum"}
    for p, n in names.items():
        if n not in ck["fp32"]:
            continue
        if hasattr(p, "_sxe_zero"):
            safe_set_full_fp32_param(p, ck["fp32"][n])
            if load_optimizer_states:
                for k, v in ck["state"].get(n, {}).items():
                    if k in key_map:
                        try:
                            safe_set_full_optimizer_state(p, v, key_map[k])
                        except KeyError:
                            pass  # this optimizer keeps no such state
        else:
            with torch.no_grad():
                p.copy_(ck["fp32"][n].to(p.device, p.dtype))
    if load_optimizer_states and hasattr(opt, "master"):
        for g, m in enumerate(opt.master):
            st = opt.optimizer.state.get(m) if hasattr(opt, "optimizer") else None
            if st is not None and "step" in st:
                st["step"] = ck["step"] if not torch.is_tensor(st["step"]) else torch.tensor(float(ck["step"]))
    if hasattr(opt, "loss_scaler") and ck["loss_scaler"]:
        ls = ck["loss_scaler"]
        sd = {"cur_scale": float(ls.get("cur_scale", 1.0)), "dynamic": bool(ls.get("dynamic", False)),
              "cur_iter": int(ls.get("cur_iter", 0)), "last_overflow_iter": int(ls.get("last_overflow_iter", -1)),
              "cur_hysteresis": int(ls.get("cur_hysteresis", ls.get("delayed_shift", 1)))}
        opt.loss_scaler.load_state_dict(sd)
    ms = ck["model_states"]
    if load_lr_scheduler_states and engine.lr_scheduler is not None and ms.get("lr_scheduler"):
        engine.lr_scheduler.load_state_dict(ms["lr_scheduler"])
    engine.global_steps = int(ms.get("global_steps", ck["step"]))
    engine.global_samples = int(ms.get("global_samples", 0))
    engine.skipped_steps = int(ms.get("skipped_steps", 0))
    return ck
