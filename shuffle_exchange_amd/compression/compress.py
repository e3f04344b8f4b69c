"""Model compression: quantization-aware training, pruning (sparse / row / head / channel) and layer
reduction, driven by the ``compression_training`` config block.

Parity: reference compression/basic_layer.py (``LinearLayer_Compress`` :121 with
enable_weight_quantization / enable_activation_quantization / enable_sparse_pruning /
enable_row_pruning / enable_head_pruning and their ``fix_*`` finalisers; ``Embedding_Compress``
:65 (weight quantization), ``Conv2dLayer_Compress`` :404 (weight / activation quantization, sparse
and channel pruning), ``BNLayer_Compress`` :611 (follows its conv's channel mask)), compress.py
(``init_compression`` / ``redundancy_clean``, layer reduction from a teacher model),
scheduler.py (``compression_scheduler`` turning techniques on at ``schedule_offset``).

Fake quantization uses a straight-through estimator; masks are recomputed from the live weights
at every enabled forward (magnitude criteria), and ``redundancy_clean`` bakes them in (and for row
pruning physically shrinks the layer and the consumer's input columns).
"""
import re

import torch
import torch.nn as nn
import torch.nn.functional as F


class _STEQuant(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, bits, groups, symmetric):
        from ..runtime.quantize import fake_quantize
        g = groups if x.numel() % groups == 0 else 1
        return fake_quantize(x, int(bits), g, symmetric)

    @staticmethod
    def backward(ctx, g):
        return g, None, None, None


class LinearLayer_Compress(nn.Linear):
    def __init__(self, *args, **kw):
        super().__init__(*args, **kw)
        self.weight_quantization_enabled = False
        self.activation_quantization_enabled = False
        self.sparse_pruning_enabled = False
        self.row_pruning_enabled = False
        self.head_pruning_enabled = False
        self.wq = {}
        self.aq = {}
        self.sparse_mask = None
        self.row_mask = None
        self.head_mask = None

    @classmethod
    def from_linear(cls, lin):
        new = cls(lin.in_features, lin.out_features, bias=lin.bias is not None, device=lin.weight.device,
                  dtype=lin.weight.dtype)
        with torch.no_grad():
            new.weight.copy_(lin.weight)
            if lin.bias is not None:
                new.bias.copy_(lin.bias)
        return new

    # -------------------------------------------------------------------------------- enabling
    def enable_weight_quantization(self, start_bits, target_bits, quantization_period, weight_quantization_enabled_in_forward=True,
                                   quantization_type="symmetric", num_groups=1):
        self.wq = dict(bits=start_bits, target=target_bits, period=max(1, quantization_period), step=0,
                       symmetric=quantization_type == "symmetric", groups=num_groups)
        self.weight_quantization_enabled = True

    def enable_activation_quantization(self, bits, quantization_type="symmetric", range_calibration="dynamic"):
        self.aq = dict(bits=bits, symmetric=quantization_type == "symmetric")
        self.activation_quantization_enabled = True

    def enable_sparse_pruning(self, ratio, method="l1"):
        self.sparse_ratio, self.sparse_method = ratio, method
        self.sparse_pruning_enabled = True

    def enable_row_pruning(self, ratio, method="l1"):
        self.row_ratio = ratio
        self.row_pruning_enabled = True

    def enable_head_pruning(self, ratio, num_heads, method="l1"):
        self.head_ratio, self.num_heads = ratio, num_heads
        self.head_pruning_enabled = True

    # ------------------------------------------------------------------------------ masks
    def _sparse(self):
        k = int(self.weight.numel() * self.sparse_ratio)
        thr = self.weight.detach().abs().flatten().kthvalue(max(1, self.weight.numel() - k)).values
        return (self.weight.detach().abs() > thr).to(self.weight.dtype)

    def _rows(self):
        n = self.weight.shape[0]
        keep = max(1, int(round(n * self.row_ratio)))
        score = self.weight.detach().abs().sum(1)
        m = torch.zeros(n, dtype=self.weight.dtype, device=self.weight.device)
        m[score.topk(keep).indices] = 1
        return m

    def _heads(self):
        h = self.num_heads
        d = self.weight.shape[1] // h
        keep = max(1, int(round(h * self.head_ratio)))
        score = self.weight.detach().abs().view(self.weight.shape[0], h, d).sum((0, 2))
        m = torch.zeros(h, dtype=self.weight.dtype, device=self.weight.device)
        m[score.topk(keep).indices] = 1
        return m.repeat_interleave(d)

    def effective_weight(self):
        w = self.weight
        if self.sparse_pruning_enabled:
            self.sparse_mask = self._sparse()
            w = w * self.sparse_mask
        if self.row_pruning_enabled:
            self.row_mask = self._rows()
            w = w * self.row_mask[:, None]
        if self.head_pruning_enabled:
            self.head_mask = self._heads()
            w = w * self.head_mask[None, :]
        if self.weight_quantization_enabled:
            q = self.wq
            if self.training:
                q["step"] += 1
                if q["bits"] > q["target"] and q["step"] % q["period"] == 0:
                    q["bits"] -= 1
            w = _STEQuant.apply(w, q["bits"], q["groups"], q["symmetric"])
        return w

    def forward(self, x, skip_bias=False):
        if self.activation_quantization_enabled:
            x = _STEQuant.apply(x, self.aq["bits"], 1, self.aq["symmetric"])
        b = None if skip_bias else self.bias
        if self.row_pruning_enabled and b is not None:
            b = b * self._rows()
        return F.linear(x, self.effective_weight(), b)

    # ---------------------------------------------------------------------------- finalising
    @torch.no_grad()
    def fix_all(self):
        self.weight.copy_(self.effective_weight())
        for a in ("sparse_pruning_enabled", "head_pruning_enabled", "weight_quantization_enabled",
                  "activation_quantization_enabled"):
            setattr(self, a, False)


class Embedding_Compress(nn.Embedding):
    """Embedding with (scheduled) fake weight quantization (reference basic_layer.py:65)."""

    def __init__(self, *args, **kw):
        super().__init__(*args, **kw)
        self.weight_quantization_enabled = False
        self.wq = {}

    @classmethod
    def from_embedding(cls, emb):
        new = cls(emb.num_embeddings, emb.embedding_dim, padding_idx=emb.padding_idx, device=emb.weight.device,
                  dtype=emb.weight.dtype)
        with torch.no_grad():
            new.weight.copy_(emb.weight)
        return new

    enable_weight_quantization = LinearLayer_Compress.enable_weight_quantization

    def effective_weight(self):
        w = self.weight
        if self.weight_quantization_enabled:
            q = self.wq
            if self.training:
                q["step"] += 1
                if q["bits"] > q["target"] and q["step"] % q["period"] == 0:
                    q["bits"] -= 1
            w = _STEQuant.apply(w, q["bits"], q["groups"], q["symmetric"])
        return w

    def forward(self, ids):
        return F.embedding(ids, self.effective_weight(), self.padding_idx, self.max_norm, self.norm_type,
                           self.scale_grad_by_freq, self.sparse)

    @torch.no_grad()
    def fix_all(self):
        self.weight.copy_(self.effective_weight())
        self.weight_quantization_enabled = False


class Conv2dLayer_Compress(nn.Conv2d):
    """Conv2d with fake weight / activation quantization, sparse pruning and output-channel pruning
    (reference basic_layer.py:404). Channel scores are the L1 norms of the output filters."""

    def __init__(self, *args, **kw):
        super().__init__(*args, **kw)
        self.weight_quantization_enabled = False
        self.activation_quantization_enabled = False
        self.sparse_pruning_enabled = False
        self.channel_pruning_enabled = False
        self.wq, self.aq = {}, {}
        self.sparse_mask = self.channel_mask = None

    @classmethod
    def from_conv(cls, c):
        new = cls(c.in_channels, c.out_channels, c.kernel_size, stride=c.stride, padding=c.padding,
                  dilation=c.dilation, groups=c.groups, bias=c.bias is not None, padding_mode=c.padding_mode,
                  device=c.weight.device, dtype=c.weight.dtype)
        with torch.no_grad():
            new.weight.copy_(c.weight)
            if c.bias is not None:
                new.bias.copy_(c.bias)
        return new

    enable_weight_quantization = LinearLayer_Compress.enable_weight_quantization
    enable_activation_quantization = LinearLayer_Compress.enable_activation_quantization
    enable_sparse_pruning = LinearLayer_Compress.enable_sparse_pruning
    _sparse = LinearLayer_Compress._sparse

    def enable_channel_pruning(self, ratio, method="l1"):
        self.channel_ratio = ratio
        self.channel_pruning_enabled = True

    def _channels(self):
        n = self.weight.shape[0]
        keep = max(1, int(round(n * self.channel_ratio)))
        score = self.weight.detach().abs().flatten(1).sum(1)
        m = torch.zeros(n, dtype=self.weight.dtype, device=self.weight.device)
        m[score.topk(keep).indices] = 1
        return m

    def effective_weight(self):
        w = self.weight
        if self.sparse_pruning_enabled:
            self.sparse_mask = self._sparse()
            w = w * self.sparse_mask
        if self.channel_pruning_enabled:
            self.channel_mask = self._channels()
            w = w * self.channel_mask.view(-1, 1, 1, 1)
        if self.weight_quantization_enabled:
            q = self.wq
            if self.training:
                q["step"] += 1
                if q["bits"] > q["target"] and q["step"] % q["period"] == 0:
                    q["bits"] -= 1
            w = _STEQuant.apply(w, q["bits"], q["groups"], q["symmetric"])
        return w

    def forward(self, x):
        if self.activation_quantization_enabled:
            x = _STEQuant.apply(x, self.aq["bits"], 1, self.aq["symmetric"])
        b = self.bias
        if self.channel_pruning_enabled and b is not None:
            b = b * self._channels()
        return self._conv_forward(x, self.effective_weight(), b)

    @torch.no_grad()
    def fix_all(self):
        self.weight.copy_(self.effective_weight())
        if self.channel_pruning_enabled and self.bias is not None:
            self.bias.mul_(self._channels())
        for a in ("sparse_pruning_enabled", "weight_quantization_enabled", "activation_quantization_enabled"):
            setattr(self, a, False)


class BNLayer_Compress(nn.BatchNorm2d):
    """BatchNorm2d that drops the channels its producing conv pruned (reference basic_layer.py:611)."""

    @classmethod
    def from_bn(cls, bn):
        new = cls(bn.num_features, eps=bn.eps, momentum=bn.momentum, affine=bn.affine,
                  track_running_stats=bn.track_running_stats, device=bn.running_mean.device
                  if bn.running_mean is not None else None)
        new.load_state_dict(bn.state_dict())
        return new

    @torch.no_grad()
    def fix_channel_pruning_helper(self, keep):
        for name in ("weight", "bias"):
            t = getattr(self, name)
            if t is not None:
                setattr(self, name, nn.Parameter(t[keep].clone()))
        for name in ("running_mean", "running_var"):
            t = getattr(self, name)
            if t is not None:
                setattr(self, name, t[keep].clone())
        self.num_features = len(keep)


def _match(name, patterns):
    return any(re.search(p, name) for p in patterns)


def _groups(cfg_block):
    shared = cfg_block.get("shared_parameters", {})
    for gname, g in cfg_block.get("different_groups", {}).items():
        yield shared, g.get("params", {}), g.get("modules", ["*"]), g.get("related_modules")


def init_compression(model, deepspeed_config, teacher_model=None, mpu=None):
    """Replace matching nn.Linear modules by LinearLayer_Compress and apply layer reduction."""
    cfg = deepspeed_config if isinstance(deepspeed_config, dict) else {}
    if isinstance(deepspeed_config, str):
        import json
        with open(deepspeed_config) as f:
            cfg = json.load(f)
    ct = cfg.get("compression_training", cfg)
    lr = ct.get("layer_reduction", {})
    if lr.get("enabled"):
        model = _layer_reduction(model, lr, teacher_model)
    wanted = []
    for tech in ("weight_quantization", "activation_quantization", "sparse_pruning", "row_pruning", "head_pruning",
                 "channel_pruning"):
        blk = ct.get(tech, {})
        if blk.get("shared_parameters", {}).get("enabled"):
            for _, _, mods, _ in _groups(blk):
                wanted += [m.replace("*", ".*") for m in mods]
    if not wanted:
        return model
    bn_wanted = []
    for _, _, _, rel in _groups(ct.get("channel_pruning", {})):
        for r in rel or []:
            bn_wanted += [x.replace("*", ".*") for x in (r if isinstance(r, list) else [r])]
    for name, mod in list(model.named_modules()):
        for cname, child in list(mod.named_children()):
            full = f"{name}.{cname}" if name else cname
            if isinstance(child, nn.Linear) and not isinstance(child, LinearLayer_Compress) and _match(full, wanted):
                setattr(mod, cname, LinearLayer_Compress.from_linear(child))
            elif isinstance(child, nn.Conv2d) and not isinstance(child, Conv2dLayer_Compress) and _match(full, wanted):
                setattr(mod, cname, Conv2dLayer_Compress.from_conv(child))
            elif (isinstance(child, nn.Embedding) and not isinstance(child, Embedding_Compress)
                  and _match(full, wanted)):
                setattr(mod, cname, Embedding_Compress.from_embedding(child))
            elif (isinstance(child, nn.BatchNorm2d) and not isinstance(child, BNLayer_Compress)
                  and bn_wanted and _match(full, bn_wanted)):
                setattr(mod, cname, BNLayer_Compress.from_bn(child))
    model._sxe_compression_config = ct
    return model


def _layer_reduction(model, lr, teacher=None):
    prefix = lr["module_name_prefix"]
    keep = lr.get("teacher_layer", list(range(lr["keep_number_layer"])))
    layers = model.get_submodule(prefix)
    src = teacher.get_submodule(prefix) if teacher is not None else layers
    new = nn.ModuleList([src[i] for i in keep])
    parent, _, leaf = prefix.rpartition(".")
    setattr(model.get_submodule(parent) if parent else model, leaf, new)
    if teacher is not None:
        for other in lr.get("other_module_name", []):
            parent, _, leaf = other.rpartition(".")
            setattr(model.get_submodule(parent) if parent else model, leaf, teacher.get_submodule(other))
    if hasattr(model, "cfg") and hasattr(model.cfg, "num_hidden_layers"):
        model.cfg.num_hidden_layers = len(new)
    return model


# technique -> the method a compressible layer must have for it to apply
_ENABLER = {"weight_quantization": "enable_weight_quantization",
            "activation_quantization": "enable_activation_quantization",
            "sparse_pruning": "enable_sparse_pruning", "row_pruning": "enable_row_pruning",
            "head_pruning": "enable_head_pruning", "channel_pruning": "enable_channel_pruning"}


class compression_scheduler:
    """Turns each technique on at its ``schedule_offset`` (reference compression/scheduler.py:12)."""

    def __init__(self, model, compression_config):
        self.model = model
        self.ct = compression_config.get("compression_training", compression_config)
        self.training_steps = 0
        self.done = set()

    def _apply(self, tech, fn):
        blk = self.ct.get(tech, {})
        sh = blk.get("shared_parameters", {})
        if not sh.get("enabled") or tech in self.done:
            return
        if self.training_steps < sh.get("schedule_offset", 0):
            return
        for shared, params, mods, _ in _groups(blk):
            pats = [m.replace("*", ".*") for m in mods]
            for name, m in self.model.named_modules():
                if _match(name, pats) and hasattr(m, _ENABLER[tech]):
                    fn(m, shared, params)
        self.done.add(tech)

    def step(self, step_zero_check=False):
        if not step_zero_check:
            self.training_steps += 1
        self._apply("weight_quantization", lambda m, s, p: m.enable_weight_quantization(
            p.get("start_bits", 8), p.get("target_bits", 8), p.get("quantization_period", 1),
            quantization_type=s.get("quantization_type", "symmetric"), num_groups=s.get("quantize_groups", 1)))
        self._apply("activation_quantization", lambda m, s, p: m.enable_activation_quantization(
            p.get("bits", 8), s.get("quantization_type", "symmetric")))
        self._apply("sparse_pruning", lambda m, s, p: m.enable_sparse_pruning(p.get("dense_ratio", 0.5),
                                                                             s.get("method", "l1")))
        self._apply("row_pruning", lambda m, s, p: m.enable_row_pruning(p.get("dense_ratio", 0.5)))
        self._apply("head_pruning", lambda m, s, p: m.enable_head_pruning(p.get("dense_ratio", 0.5),
                                                                         s.get("num_heads", 1)))
        self._apply("channel_pruning", lambda m, s, p: m.enable_channel_pruning(p.get("dense_ratio", 0.5),
                                                                               s.get("method", "l1")))


def redundancy_clean(model, deepspeed_config=None, mpu=None):
    """Bake masks / quantization into the weights; row-pruned layers physically shrink together
    with the input columns of the layer named in ``related_modules``."""
    ct = (deepspeed_config or {}).get("compression_training", deepspeed_config or {})
    related = {}
    for _, _, mods, rel in _groups(ct.get("row_pruning", {})):
        if rel:
            for m, r in zip(mods, rel):
                related[m] = r
    rows_of, chans_of = {}, {}
    for name, m in list(model.named_modules()):  # phase 1: bake every mask / quantizer
        if isinstance(m, LinearLayer_Compress):
            if m.row_pruning_enabled:
                rows_of[name] = m._rows()
            m.fix_all()
        elif isinstance(m, Conv2dLayer_Compress):
            if m.channel_pruning_enabled:
                chans_of[name] = m._channels()
            m.fix_all()
        elif isinstance(m, Embedding_Compress):
            m.fix_all()
    _drop_channels(model, ct, chans_of)
    for name, m in list(model.named_modules()):  # phase 2: physically drop pruned rows / columns
        if name not in rows_of:
            continue
        keep = rows_of[name].nonzero().squeeze(1)
        with torch.no_grad():
            m.weight = nn.Parameter(m.weight[keep].clone())
            if m.bias is not None:
                m.bias = nn.Parameter(m.bias[keep].clone())
        m.out_features = len(keep)
        m.row_pruning_enabled = False
        for pat, rel in related.items():
            if re.search(pat.replace("*", ".*"), name):
                for rname in (rel if isinstance(rel, list) else [rel]):
                    for n2, m2 in model.named_modules():
                        if re.search(rname.replace("*", ".*"), n2) and isinstance(m2, nn.Linear):
                            with torch.no_grad():
                                m2.weight = nn.Parameter(m2.weight[:, keep].clone())
                            m2.in_features = len(keep)
    return model


def _drop_channels(model, ct, chans_of):
    """Channel pruning, physically: the pruned conv loses output filters, and each of its
    ``related_modules`` (BatchNorm -> its channels, a following conv -> its input channels) follows."""
    related = {}
    for _, _, mods, rel in _groups(ct.get("channel_pruning", {})):
        if rel:
            for m, r in zip(mods, rel):
                related[m] = r if isinstance(r, list) else [r]
    mods = dict(model.named_modules())
    for name, mask in chans_of.items():
        m = mods[name]
        keep = mask.nonzero().squeeze(1)
        with torch.no_grad():
            m.weight = nn.Parameter(m.weight[keep].clone())
            if m.bias is not None:
                m.bias = nn.Parameter(m.bias[keep].clone())
        m.out_channels = len(keep)
        m.channel_pruning_enabled = False
        for pat, rels in related.items():
            if not re.search(pat.replace("*", ".*"), name):
                continue
            for rname in rels:
                for n2, m2 in mods.items():
                    if not re.search(rname.replace("*", ".*"), n2):
                        continue
                    if isinstance(m2, BNLayer_Compress):
                        m2.fix_channel_pruning_helper(keep)
                    elif isinstance(m2, nn.Conv2d) and m2.groups == 1:
                        with torch.no_grad():
                            m2.weight = nn.Parameter(m2.weight[:, keep].clone())
                        m2.in_channels = len(keep)
