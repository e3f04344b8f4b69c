"""Dominant Hessian eigenvalue per parameter block by power iteration on Hessian-vector products.

Parity: reference runtime/eigenvalue.py ``Eigenvalue`` :13 (max_iter, tol, stability, layer_name /
layer_num blocks, used to scale MoQ quantization periods). The HVP is
d/dp (g(p) . v) with ``create_graph`` on the first gradient; blocks are the parameters of each
``layer_name[i]`` submodule.
"""
import torch


class Eigenvalue:
    def __init__(self, verbose=False, max_iter=100, tol=1e-2, stability=1e-6, gas_boundary_resolution=1,
                 layer_name="", layer_num=0):
        self.verbose, self.max_iter, self.tol, self.stability = verbose, max_iter, tol, stability
        self.gas_boundary_resolution = gas_boundary_resolution
        self.layer_name, self.layer_num = layer_name, layer_num

    @staticmethod
    def _normalize(vs):
        n = torch.sqrt(sum((v * v).sum() for v in vs))
        return [v / (n + 1e-12) for v in vs]

    def _blocks(self, module):
        if self.layer_name:
            layers = module.get_submodule(self.layer_name)
            return [[p for p in layers[i].parameters() if p.requires_grad] for i in range(self.layer_num or len(layers))]
        return [[p for p in module.parameters() if p.requires_grad]]

    def compute_eigenvalue(self, module, loss_fn, scale=1.0):
        """loss_fn() -> scalar loss (re-evaluated here with a differentiable graph).
        Returns {block_index: (eigenvalue, layer_index)} like the reference's post-processing."""
        blocks = self._blocks(module)
        loss = loss_fn()
        out = {}
        for bi, params in enumerate(blocks):
            grads = torch.autograd.grad(loss, params, create_graph=True, retain_graph=True)
            v = self._normalize([torch.randn_like(p) for p in params])
            eig = 0.0
            for it in range(self.max_iter):
                hv = torch.autograd.grad(grads, params, grad_outputs=v, retain_graph=True)
                hv = [h.detach() + self.stability * x for h, x in zip(hv, v)]
                new = float(sum((h * x).sum() for h, x in zip(hv, v)))
                v = self._normalize(hv)
                if it > 0 and abs(new - eig) / (abs(eig) + 1e-6) < self.tol:
                    eig = new
                    break
                eig = new
            out[bi] = (eig * scale, bi)
        return out
