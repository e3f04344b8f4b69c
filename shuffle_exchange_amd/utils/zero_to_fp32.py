#!/usr/bin/env python3
"""Consolidate a ZeRO (stage 0/1/2/3, incl. Shuffle-exchange slices) checkpoint into one fp32
state dict -- offline, on the CPU, no GPUs or process group needed.

Parity: reference utils/zero_to_fp32.py (``get_fp32_state_dict_from_zero_checkpoint``,
``convert_zero_checkpoint_to_fp32_state_dict``, ``load_state_dict_from_zero_checkpoint``, CLI).

Our optimizer files carry a ``unit_layout`` (per param group: units with param names / shapes /
offsets / padded size / chunk). Rank r of a ZeRO partition group owns chunk r of every unit, and
its fp32 master for a group is the concatenation of its chunks, so the full flat unit is the
rank-ordered concatenation of chunks -- no padding arithmetic as in the reference. With
Shuffle-exchange slices every slice holds a complete (slice-local) fp32 copy; the consolidated
weights are their mean, which is exactly what the slice-averaged bit16 model holds after RR.

Usage: python -m shuffle_exchange_amd.utils.zero_to_fp32 CHECKPOINT_DIR OUTPUT_FILE [-t TAG]
"""
import argparse
import glob
import os
import re

import torch


def _load(path, mmap=False):
    # files written by this framework; mmap=True maps the tensors instead of reading them, so a
    # consumer that slices one unit at a time only pages in that unit (streaming conversion)
    return torch.load(path, map_location="cpu", weights_only=False, mmap=mmap)


def _tag_dir(checkpoint_dir, tag=None):
    if tag is None:
        latest = os.path.join(checkpoint_dir, "latest")
        if not os.path.isfile(latest):
            raise ValueError(f"no 'latest' file in {checkpoint_dir}; pass tag explicitly")
        with open(latest) as f:
            tag = f.read().strip()
    d = os.path.join(checkpoint_dir, str(tag))
    if not os.path.isdir(d):
        raise FileNotFoundError(d)
    return d


def _optim_files(d):
    files = glob.glob(os.path.join(d, "*zero_pp_rank_*_mp_rank_*_optim_states.pt"))

    def key(f):
        m = re.search(r"zero_pp_rank_(\d+)_mp_rank_(\d+)", os.path.basename(f))
        return (int(m.group(2)), int(m.group(1)))
    return sorted(files, key=key)


def _reference_reader():
    """The reference-layout reader when the package is importable; the copy of this script that
    save_checkpoint drops into every tag directory runs without it (own checkpoints only)."""
    try:
        from shuffle_exchange_amd.checkpoint.reference_format import is_reference_checkpoint, read_reference_checkpoint
    except ImportError:
        return None
    return is_reference_checkpoint, read_reference_checkpoint


def get_fp32_state_dict_from_zero_checkpoint(checkpoint_dir, tag=None, exclude_frozen_parameters=False):
    ref = _reference_reader()
    if ref is not None and ref[0](checkpoint_dir, tag):  # written in the reference's ZeRO layout
        return dict(ref[1](checkpoint_dir, tag)["fp32"])
    if tag is None and not os.path.isfile(os.path.join(checkpoint_dir, "latest")) and _optim_files(checkpoint_dir):
        d = checkpoint_dir  # pointed at the tag directory itself (the copied script: `python zero_to_fp32.py . out`)
    else:
        d = _tag_dir(checkpoint_dir, tag)
    files = _optim_files(d)
    if not files:
        raise FileNotFoundError(f"no ZeRO optimizer files in {d}")
    states = [_load(f)["optimizer_state_dict"] for f in files]
    s0 = states[0]
    stage = s0.get("zero_stage", 0)
    layout = s0["unit_layout"]
    if stage == 3:
        masters = [s["fp32_flat_groups"] for s in states]
        S = s0["partition_count"]
    else:
        masters = [s["single_partition_of_fp32_groups"] for s in states]
        S = s0.get("slice_count", 1) if stage in (1, 2) else 1
    S = int(S if not isinstance(S, (list, tuple)) else S[0])
    n_slices = max(1, len(states) // S) if stage in (1, 2, 3) else 1
    sd = {}
    for g, units in enumerate(layout):
        off = 0
        for u in units:
            chunk = u["chunk"]
            flat = None
            for j in range(n_slices):
                parts = [masters[j * S + r][g][off:off + chunk].float() for r in range(S)]
                f = torch.cat(parts) if S > 1 else parts[0]
                flat = f.clone() if flat is None else flat.add_(f)
            if n_slices > 1:
                flat /= n_slices
            for name, shape, o in zip(u["params"], u["shapes"], u["offsets"]):
                n = 1
                for x in shape:
                    n *= x
                sd[name] = flat[o:o + n].view(shape).clone().float()
            off += chunk
    # frozen params / buffers from the model-states file(s)
    model_files = sorted(glob.glob(os.path.join(d, "*model_states.pt")))
    if model_files:
        ms = _load(model_files[0])
        mod = ms.get("module") or {}
        for k in ms.get("buffer_names", []):
            if k in mod and k not in sd:
                sd[k] = mod[k]
        if not exclude_frozen_parameters:
            frags = ms.get("frozen_param_fragments") or {}
            for k in ms.get("frozen_param_shapes", {}):
                if k not in sd and k in mod:
                    sd[k] = mod[k].float()
                elif k not in sd and k in frags:  # ZeRO-2/3 files without a module state
                    sd[k] = frags[k].float()
        # tied weights: the parameter that is not stored shares the data of the one that is
        for k, src in (ms.get("shared_params") or {}).items():
            if src in sd:
                sd[k] = sd[src]
    return sd


def convert_zero_checkpoint_to_fp32_state_dict(checkpoint_dir, output_file, tag=None, exclude_frozen_parameters=False,
                                               safe_serialization=False):
    sd = get_fp32_state_dict_from_zero_checkpoint(checkpoint_dir, tag, exclude_frozen_parameters)
    os.makedirs(os.path.dirname(os.path.abspath(output_file)), exist_ok=True)
    if safe_serialization:
        from safetensors.torch import save_file
        save_file({k: v.contiguous() for k, v in sd.items()}, output_file)
    else:
        torch.save(sd, output_file)
    return output_file


def load_state_dict_from_zero_checkpoint(model, checkpoint_dir, tag=None):
    sd = get_fp32_state_dict_from_zero_checkpoint(checkpoint_dir, tag)
    model = model.cpu()
    model.load_state_dict(sd, strict=False)
    return model


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("checkpoint_dir")
    ap.add_argument("output_file")
    ap.add_argument("-t", "--tag", default=None)
    ap.add_argument("--exclude_frozen_parameters", action="store_true")
    ap.add_argument("--safe_serialization", action="store_true")
    a = ap.parse_args(argv)
    out = convert_zero_checkpoint_to_fp32_state_dict(a.checkpoint_dir, a.output_file, a.tag,
                                                     a.exclude_frozen_parameters, a.safe_serialization)
    print(f"saved fp32 state dict to {out}")


if __name__ == "__main__":
    main()
