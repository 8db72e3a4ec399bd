"""Block-wise Hessian max-eigenvalue estimation by power iteration (Hessian-vector products via double backward).

Reference parity: runtime/eigenvalue.py (``Eigenvalue`` :13, ``compute_eigenvalue`` :71, ``post_process``):
one eigenvalue per layer block (``layer_name`` + ``layer_num``), used by MoQ to pick per-block quantization
periods. Requires the loss graph to be built with ``create_graph=True`` gradients.
"""
import torch

from ..utils.logging import log_dist


class Eigenvalue:

    def __init__(self, verbose=False, max_iter=100, tol=1e-2, stability=1e-6, gas_boundary_resolution=1,
                 layer_name="", layer_num=0):
        self.verbose = verbose
        self.max_iter = max_iter
        self.tol = tol
        self.stability = stability
        self.gas_boundary_resolution = gas_boundary_resolution
        self.layer_name = layer_name
        self.layer_num = layer_num

    @staticmethod
    def nan_to_num(x):
        return torch.nan_to_num(x, nan=0.0, posinf=0.0, neginf=0.0)

    def normalize(self, v):
        norm = torch.sqrt(sum(torch.sum(x * x) for x in v)) + self.stability
        return [x / norm for x in v]

    @staticmethod
    def inner_product(xs, ys):
        return sum(torch.sum(x * y) for x, y in zip(xs, ys))

    def get_layers(self, module):
        obj = module
        for name in self.layer_name.split(".") if self.layer_name else []:
            obj = getattr(obj, name)
        return obj

    def compute_eigenvalue(self, module, loss=None, device=None, scale=1.0):
        """Returns {block_index: (eigenvalue, layer_index)} using grads of ``loss`` w.r.t. each block's params."""
        blocks = self.get_layers(module) if self.layer_name else [module]
        results = {}
        for i, block in enumerate(list(blocks)[:self.layer_num or None]):
            params = [p for p in block.parameters() if p.requires_grad]
            if not params:
                continue
            grads = torch.autograd.grad(loss, params, create_graph=True, allow_unused=True)
            pairs = [(p, g) for p, g in zip(params, grads) if g is not None]
            if not pairs:
                continue
            ps, gs = zip(*pairs)
            v = self.normalize([torch.randn_like(p) for p in ps])
            eig = None
            for _ in range(self.max_iter):
                hv = torch.autograd.grad(gs, ps, grad_outputs=v, retain_graph=True)
                hv = [self.nan_to_num(h.detach()) for h in hv]
                new = self.inner_product(hv, v).item()
                v = self.normalize(hv)
                if eig is not None and abs(new - eig) / (abs(eig) + self.stability) < self.tol:
                    eig = new
                    break
                eig = new
            results[i] = (eig * scale if eig is not None else 0.0, i)
            if self.verbose:
                log_dist(f"block {i} eigenvalue {eig}", ranks=[0])
        return self.post_process(results)

    def post_process(self, value_dict):
        """Normalise by the max |eigenvalue| (reference: relative eigenvalues feed MoQ's periods)."""
        if not value_dict:
            return value_dict
        m = max(abs(v[0]) for v in value_dict.values()) or 1.0
        return {k: (abs(v[0]) / m, v[1]) for k, v in value_dict.items()}
