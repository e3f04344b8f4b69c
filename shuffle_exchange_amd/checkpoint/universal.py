"""Universal checkpoints: parallelism-independent, per-parameter fp32 weights + optimizer moments.

Parity: reference checkpoint/ds_to_universal.py (extract ZeRO shards -> per-parameter
``fp32.pt`` / ``exp_avg.pt`` / ``exp_avg_sq.pt`` under ``<out>/zero/<param name>/``, copy the model
states) and the engine's ``load_universal_checkpoint`` path (runtime/engine.py, ``checkpoint:
{load_universal: true}``), which re-partitions those tensors for the *current* data-parallel /
Shuffle-exchange layout -- so a run saved on 8 GPUs resumes on 4 or 16.

Writing is offline (CPU, no process group) and streaming: the rank files are memory-mapped and
consumed one unit at a time, so peak host memory is about one unit's full fp32 tensors (not every
rank's whole state: ~840 GB for a 70B model). Checkpoints in the reference's own ZeRO layout are
converted too (checkpoint/reference_format.py). Loading slices each parameter's fp32 tensor and
moments straight into this rank's chunk of its flat unit (no full-model materialisation per rank).
"""
import argparse
import glob
import json
import os
import shutil

import torch

from ..utils.zero_to_fp32 import _load, _optim_files, _tag_dir

STATE_KEYS = ("exp_avg", "exp_avg_sq")


def _numel(shape):
    n = 1
    for x in shape:
        n *= x
    return n


def _convert_reference(checkpoint_dir, output_dir, tag):
    from .reference_format import _tag_dir as ref_tag_dir
    from .reference_format import read_reference_checkpoint
    ck = read_reference_checkpoint(checkpoint_dir, tag)
    zdir = os.path.join(output_dir, "zero")
    for name, t in ck["fp32"].items():
        pdir = os.path.join(zdir, name)
        os.makedirs(pdir, exist_ok=True)
        torch.save(t.clone(), os.path.join(pdir, "fp32.pt"))
        for k, v in ck["state"].get(name, {}).items():
            if k in STATE_KEYS:
                torch.save(v.clone(), os.path.join(pdir, f"{k}.pt"))
    with open(os.path.join(output_dir, "universal_meta.json"), "w") as f:
        json.dump({"step": ck["step"], "source_zero_stage": ck["zero_stage"], "source_format": "reference",
                   "source_dp": ck["dp_world_size"]}, f)
    d = ref_tag_dir(checkpoint_dir, tag)
    for mf in glob.glob(os.path.join(d, "*model_states.pt")):
        shutil.copy(mf, output_dir)
    return output_dir


def convert_to_universal(checkpoint_dir, output_dir, tag=None):
    from .reference_format import is_reference_checkpoint
    if is_reference_checkpoint(checkpoint_dir, tag):
        return _convert_reference(checkpoint_dir, output_dir, tag)
    d = _tag_dir(checkpoint_dir, tag)
    states = [_load(f, mmap=True)["optimizer_state_dict"] for f in _optim_files(d)]
    s0 = states[0]
    stage = s0.get("zero_stage", 0)
    layout = s0["unit_layout"]
    if stage == 3:
        masters = [s["fp32_flat_groups"] for s in states]
        S = s0["partition_count"]
        opt_states = [s["optimizer_state_dict"] for s in states]
    else:
        masters = [s["single_partition_of_fp32_groups"] for s in states]
        S = s0.get("slice_count", 1) if stage in (1, 2) else 1
        opt_states = [s["base_optimizer_state"] for s in states]
    S = int(S if not isinstance(S, (list, tuple)) else S[0])
    n_slices = max(1, len(states) // S) if stage else 1
    zdir = os.path.join(output_dir, "zero")
    os.makedirs(zdir, exist_ok=True)
    step = None
    for g, units in enumerate(layout):
        off = 0
        for u in units:
            chunk = u["chunk"]

            def full(tensors_by_rank):
                acc = None
                for j in range(n_slices):
                    parts = [tensors_by_rank[j * S + r][off:off + chunk].float() for r in range(S)]
                    f = torch.cat(parts) if S > 1 else parts[0]
                    acc = f.clone() if acc is None else acc.add_(f)
                return acc / n_slices

            flats = {"fp32": full([m[g] for m in masters])}
            for k in STATE_KEYS:
                per_rank = []
                for os_ in opt_states:
                    st = os_["state"].get(g, os_["state"].get(str(g), {}))
                    if k not in st:
                        break
                    per_rank.append(st[k])
                    step = st.get("step", step)
                if len(per_rank) == len(opt_states):
                    flats[k] = full(per_rank)
            for name, shape, o in zip(u["params"], u["shapes"], u["offsets"]):
                n = _numel(shape)
                pdir = os.path.join(zdir, name)
                os.makedirs(pdir, exist_ok=True)
                for k, f in flats.items():
                    torch.save(f[o:o + n].view(shape).clone(), os.path.join(pdir, f"{k}.pt"))
            off += chunk
    meta = {"step": int(step) if step is not None else 0, "source_zero_stage": stage, "source_partition": S,
            "source_slices": n_slices}
    with open(os.path.join(output_dir, "universal_meta.json"), "w") as f:
        json.dump(meta, f)
    for mf in glob.glob(os.path.join(d, "*model_states.pt")):
        shutil.copy(mf, output_dir)
    return output_dir


def load_universal_into_optimizer(opt, universal_dir, name_of):
    """Fill this rank's fp32 master chunks and Adam moments from a universal checkpoint, then
    refresh the bit16 shards. ``name_of``: {param: name}."""
    with open(os.path.join(universal_dir, "universal_meta.json")) as f:
        meta = json.load(f)
    zdir = os.path.join(universal_dir, "zero")
    for g, units in enumerate(opt.units):
        m = opt.master[g]
        st = opt.optimizer.state[m]
        base = 0
        for u in units:
            lo = u.rank * u.chunk if hasattr(u, "rank") else 0
            hi = lo + u.chunk
            for p, o, n in zip(u.params, u.offsets, u.numels):
                a, b = max(o, lo), min(o + n, hi)
                if a >= b:
                    continue
                pdir = os.path.join(zdir, name_of[p])
                for key, dst in [("fp32", m.data)] + [(k, st[k]) for k in STATE_KEYS if k in st]:
                    path = os.path.join(pdir, f"{key}.pt")
                    if not os.path.exists(path):
                        continue
                    src = torch.load(path, map_location="cpu", weights_only=True).reshape(-1)
                    dst[base + (a - lo):base + (b - lo)].copy_(src[a - o:b - o].to(dst.device))
            base += u.chunk
        if "step" in st:
            st["step"] = meta.get("step", st["step"])
    for units in opt.units:
        for u in units:
            u.shard.copy_(u.master)
    if hasattr(opt, "_allgather_params"):
        opt._allgather_params()
    elif hasattr(opt, "_refresh_persistent"):
        opt._refresh_persistent()
    return meta


def main(argv=None):
    ap = argparse.ArgumentParser(description="convert a ZeRO checkpoint to a universal checkpoint")
    ap.add_argument("--input_folder", required=True)
    ap.add_argument("--output_folder", required=True)
    ap.add_argument("--tag", default=None)
    a = ap.parse_args(argv)
    print(convert_to_universal(a.input_folder, a.output_folder, a.tag))


if __name__ == "__main__":
    main()
