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

    def _prepare(self, group, p):
        """Advance p's step and return its (exp_avg, exp_avg_sq, coeffs)."""
        beta1, beta2 = group["betas"]
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
        return state["exp_avg"], state["exp_avg_sq"], c

    @torch.no_grad()
    def take_step(self, p):
        """Hand p's next update to a fused kernel: advances p's state exactly
        as step() would and returns (p, exp_avg, exp_avg_sq, coeffs) for
        functional.render_bwd(table_step=...); the next step() leaves p
        alone.  Call it at the point of the iteration where step() would run
        for p (same lr)."""
        for group in self.param_groups:
            if any(q is p for q in group["params"]):
                m, v, c = self._prepare(group, p)
                self._fused = getattr(self, "_fused", set()) | {id(p)}
                return p, m, v, c
        raise ValueError("RAdam.take_step: not a parameter of this optimizer")

    @torch.no_grad()
    def step(self, closure=None):
        """All parameters of all groups in one HIP launch (hn_radam_step);
        parameters handed to take_step since the last step() are skipped."""
        loss = closure() if closure is not None else None
        work = []
        fused, self._fused = getattr(self, "_fused", set()), set()
        for group in self.param_groups:
            for p in group["params"]:
                if id(p) in fused or p.grad is None:
                    continue
                grad = p.grad
                if grad.is_sparse:
                    raise RuntimeError("RAdam does not support sparse gradients")
                m, v, c = self._prepare(group, p)
                work.append((p, grad.contiguous(), m, v, c))
        if work:
            HF.radam_step(work)
        return loss

    # -- reference-compatible state dict --------------------------------------
    # The reference's embedding group holds the 16 per-level nn.Embedding
    # weights (run_nerf_helpers.py:61-62, :132-135); here it holds ONE stacked
    # table [L, 2^T, F] (HashEmbedder.table, marked with ``_hn_levels``).  The
    # optimizer state dict is converted both ways so that a checkpoint written
    # by either side (run_nerf.py:663-680) loads into the other: the stacked
    # parameter is listed as L consecutive params whose exp_avg / exp_avg_sq are
    # its per-level slices, with the shared step counter.
    @staticmethod
    def _levels(p) -> int:
        return int(getattr(p, "_hn_levels", 0) or 0)

    def state_dict(self):
        xchg = getattr(self, "sharded_state", None)
        if xchg is not None and xchg.stale:
            # data-parallel sharded table step (train.ShardedTableStep): the
            # table's moments live on the ranks' shards; the full-size copy
            # here is out of date until every rank has gathered them
            raise RuntimeError("RAdam.state_dict: the hash table's moments are sharded over the ranks and the "
                               "optimizer's copy is stale; call Trainer.sync_optimizer_state() on every rank first")
        sd = super().state_dict()
        if not any(self._levels(p) for g in self.param_groups for p in g["params"]):
            return sd
        state, groups, nxt = {}, [], 0
        for gsd, group in zip(sd["param_groups"], self.param_groups):
            ids = []
            for old, p in zip(gsd["params"], group["params"]):
                st = sd["state"].get(old)
                n = self._levels(p)
                for l in range(max(n, 1)):
                    if st is not None:
                        state[nxt] = st if not n else {
                            k: (v[l] if torch.is_tensor(v) and v.dim() == p.dim() else v)
                            for k, v in st.items()}
                    ids.append(nxt)
                    nxt += 1
            groups.append({**gsd, "params": ids})
        return {"state": state, "param_groups": groups}

    def load_state_dict(self, state_dict):
        """Accepts this optimizer's own state dict and the reference's (one
        param entry per hash level in the embedding group)."""
        sd_groups = state_dict["param_groups"]
        if len(sd_groups) != len(self.param_groups):
            return super().load_state_dict(state_dict)   # torch raises its own error
        state, groups, nxt = {}, [], 0
        src = state_dict["state"]
        for gsd, group in zip(sd_groups, self.param_groups):
            ids = list(gsd["params"])
            own = len(group["params"])
            expanded = sum(max(self._levels(p), 1) for p in group["params"])
            if len(ids) == own:                        # this optimizer's own layout
                new_ids = []
                for i in ids:
                    if i in src:
                        state[nxt] = src[i]
                    new_ids.append(nxt)
                    nxt += 1
                groups.append({**gsd, "params": new_ids})
                continue
            if len(ids) != expanded:
                raise ValueError(
                    f"loaded state dict has a group with {len(ids)} params; this optimizer's group has "
                    f"{own} (or {expanded} with per-level hash tables)")
            new_ids, k = [], 0
            for p in group["params"]:
                n = self._levels(p)
                if not n:
                    if ids[k] in src:
                        state[nxt] = src[ids[k]]
                    k += 1
                else:
                    parts = [src.get(i) for i in ids[k:k + n]]
                    k += n
                    if any(s is not None for s in parts):
                        if any(s is None for s in parts):
                            raise ValueError("per-level hash-table state is missing for some levels")
                        steps = {int(s["step"]) for s in parts}
                        if len(steps) != 1:
                            raise ValueError(f"per-level hash-table steps differ: {sorted(steps)}")
                        state[nxt] = {"step": steps.pop(),
                                      "exp_avg": torch.stack([s["exp_avg"] for s in parts], 0),
                                      "exp_avg_sq": torch.stack([s["exp_avg_sq"] for s in parts], 0)}
                new_ids.append(nxt)
                nxt += 1
            groups.append({**gsd, "params": new_ids})
        out = super().load_state_dict({"state": state, "param_groups": groups})
        # data-parallel sharded table step: the table's moments live on the
        # ranks' shards, seeded once from optimizer.state; the loaded moments
        # must reach the shards too, or training would silently continue on the
        # old ones
        xchg = getattr(self, "sharded_state", None)
        if xchg is not None:
            xchg.load_state(self.state.get(xchg.table))
        return out
