"""RAdam (radam.py:5-94) with the reference's exact step semantics.

Dense update over every parameter each step (untouched hash rows still get
their moments decayed), N_sma >= 5 rectification threshold (so no update for
the first five steps at beta2 = 0.99), weight decay applied as p -= wd*lr*p,
and the 10-entry step buffer.  The per-element update runs in one HIP launch
over every parameter (hn_radam_step); the scalar rectification terms are
computed on the host exactly as the reference does.
"""
from __future__ import annotations

import math

import torch
from torch.optim.optimizer import Optimizer

from . import functional as HF


class RAdam(Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0,
                 degenerated_to_sgd=False):
        if lr < 0.0:
            raise ValueError(f"Invalid learning rate: {lr}")
        if eps < 0.0:
            raise ValueError(f"Invalid epsilon value: {eps}")
        if not 0.0 <= betas[0] < 1.0 or not 0.0 <= betas[1] < 1.0:
            raise ValueError(f"Invalid beta parameters: {betas}")
        self.degenerated_to_sgd = degenerated_to_sgd
        if isinstance(params, (list, tuple)) and len(params) > 0 and isinstance(params[0], dict):
            for g in params:
                if "betas" in g and (g["betas"][0] != betas[0] or g["betas"][1] != betas[1]):
                    g["buffer"] = [[None, None, None] for _ in range(10)]
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay,
                        buffer=[[None, None, None] for _ in range(10)])
        super().__init__(params, defaults)

    def _coeffs(self, group, step):
        beta1, beta2 = group["betas"]
        buffered = group["buffer"][int(step % 10)]
        if step == buffered[0]:
            return buffered[1], buffered[2]
        buffered[0] = step
        beta2_t = beta2 ** step
        n_sma_max = 2 / (1 - beta2) - 1
        n_sma = n_sma_max - 2 * step * beta2_t / (1 - beta2_t)
        buffered[1] = n_sma
        if n_sma >= 5:
            step_size = math.sqrt((1 - beta2_t) * (n_sma - 4) / (n_sma_max - 4) * (n_sma - 2) / n_sma
                                  * n_sma_max / (n_sma_max - 2)) / (1 - beta1 ** step)
        elif self.degenerated_to_sgd:
            step_size = 1.0 / (1 - beta1 ** step)
        else:
            step_size = -1
        buffered[2] = step_size
        return n_sma, step_size

    @torch.no_grad()
    def step(self, closure=None):
        """All parameters of all groups in one HIP launch (hn_radam_step)."""
        loss = closure() if closure is not None else None
        work = []
        for group in self.param_groups:
            beta1, beta2 = group["betas"]
            for p in group["params"]:
                if p.grad is None:
                    continue
                grad = p.grad
                if grad.is_sparse:
                    raise RuntimeError("RAdam does not support sparse gradients")
                state = self.state[p]
                if len(state) == 0:
                    state["step"] = 0
                    state["exp_avg"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                    state["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                state["step"] += 1
                n_sma, step_size = self._coeffs(group, state["step"])
                mode = 2 if n_sma >= 5 else (1 if step_size > 0 else 0)
                lr, wd = group["lr"], group["weight_decay"]
                c = {"beta1": beta1, "beta2": beta2, "one_minus_beta1": 1 - beta1,
                     "one_minus_beta2": 1 - beta2, "eps": group["eps"], "neg_wd_lr": -wd * lr,
                     "neg_step_lr": -step_size * lr if mode else 0.0, "mode": mode,
                     "has_wd": int(wd != 0)}
                work.append((p, grad.contiguous(), state["exp_avg"], state["exp_avg_sq"], c))
        if work:
            HF.radam_step(work)
        return loss
