"""Architecture-parameter optimiser (reference ``fedml_api/model/cv/darts/architect.py:13-392``).

All reference update rules are provided:

* ``step(..., unrolled=False)`` — first-order DARTS (alpha gradient of the validation loss);
* ``step(..., unrolled=True)`` — second-order DARTS: validation loss at the one-step-unrolled weights
  ``w' = w - eta (m*mom + dL_train/dw + wd w)``, minus ``eta`` times the finite-difference Hessian-vector
  product ``(grad_a L_train(w+) - grad_a L_train(w-)) / 2R``, ``R = 0.01/||dL_val/dw'||``;
* ``step_v2`` / ``step_wa`` — alpha gradient = val gradient + lambda * train gradient;
* ``step_single_level`` — train-loss alpha gradient only; ``step_AOS`` — plain val-loss backward;
* ``step_v2_2ndorder`` / ``step_v2_2ndorder2`` — the unrolled variant of ``step_v2`` (the second one takes
  the Hessian-vector product of the validation term on the validation batch).

The unrolled model is evaluated with ``torch.func.functional_call`` on the live module and a flat weight
vector instead of deep-copying a new network per step.  The optimiser is Adam(lr=arch_learning_rate,
betas=(0.5, 0.999), weight_decay=arch_weight_decay) as in the reference.
"""
from __future__ import annotations

import torch
from torch.func import functional_call


def _flat(ts):
    return torch.cat([t.reshape(-1) for t in ts])


def _grads(loss, ts):
    """``autograd.grad`` with zeros for inputs the loss does not touch (e.g. unused normal-cell alphas)."""
    gs = torch.autograd.grad(loss, ts, allow_unused=True)
    return [torch.zeros_like(t) if g is None else g for g, t in zip(gs, ts)]


class Architect:
    def __init__(self, model, criterion, args, device=None, grad_sync=None):
        """``grad_sync(list_of_grads)``: optional in-place cross-rank average of the alpha gradients (data-
        parallel search, one process per GPU); called right before every Adam step."""
        self.model = model
        self.grad_sync = grad_sync
        self.criterion = criterion
        self.device = device
        self.network_momentum = args.momentum
        self.network_weight_decay = args.weight_decay
        self.optimizer = torch.optim.Adam(self._arch(), lr=args.arch_learning_rate, betas=(0.5, 0.999),
                                          weight_decay=args.arch_weight_decay)

    # ---------------------------------------------------------------------------------------------
    def _net(self):
        return self.model.module if hasattr(self.model, "module") else self.model

    def _arch(self):
        return self._net().arch_parameters()

    def _weights(self):
        return self._net().weight_parameters()

    def _weight_names(self):
        ids = {id(p) for p in self._arch()}
        return [n for n, p in self._net().named_parameters() if id(p) not in ids]

    def _loss(self, x, y, params=None):
        net = self._net()
        out = net(x) if params is None else functional_call(net, params, (x,))
        return self.criterion(out, y)

    def _set_grads(self, grads):
        for v, g in zip(self._arch(), grads):
            v.grad = g.detach().clone()

    def _opt_step(self):
        if self.grad_sync is not None:
            self.grad_sync([a.grad for a in self._arch() if a.grad is not None])
        self.optimizer.step()

    def _alpha_grad(self, x, y):
        return _grads(self._loss(x, y), self._arch())

    # ---------------------------------------------------------------------------------------------
    def _unrolled_params(self, x, y, eta, network_optimizer):
        ws = self._weights()
        theta = _flat([w.detach() for w in ws])
        try:
            mom = _flat([network_optimizer.state[w]["momentum_buffer"] for w in ws]) * self.network_momentum
        except (KeyError, TypeError, AttributeError):
            mom = torch.zeros_like(theta)
        g = _flat(torch.autograd.grad(self._loss(x, y), ws)) + self.network_weight_decay * theta
        new = theta - eta * (mom + g)
        params, off = {}, 0
        for n, w in zip(self._weight_names(), ws):
            params[n] = new[off:off + w.numel()].view_as(w).detach().requires_grad_(True)
            off += w.numel()
        for n, b in self._net().named_buffers():  # the unrolled model keeps its own BN statistics
            params[n] = b.detach().clone()
        for n, a in zip(("alphas_normal", "alphas_reduce"), self._arch()):
            params[n] = a
        return params

    def _unrolled_grads(self, params, x, y):
        """(d alpha, d w') of the loss at the unrolled weights."""
        loss = self._loss(x, y, params)
        names = self._weight_names()
        grads = _grads(loss, list(self._arch()) + [params[n] for n in names])
        na = len(self._arch())
        return list(grads[:na]), list(grads[na:])

    def _hessian_vector_product(self, vector, x, y, r=1e-2):
        ws = self._weights()
        R = r / _flat(vector).norm()
        with torch.no_grad():
            for p, v in zip(ws, vector):
                p.add_(v, alpha=float(R))
        gp = self._alpha_grad(x, y)
        with torch.no_grad():
            for p, v in zip(ws, vector):
                p.sub_(v, alpha=2 * float(R))
        gn = self._alpha_grad(x, y)
        with torch.no_grad():
            for p, v in zip(ws, vector):
                p.add_(v, alpha=float(R))
        return [(a - b) / (2 * R) for a, b in zip(gp, gn)]

    def _second_order_alpha(self, params, xa, ya, xh, yh, eta):
        da, dw = self._unrolled_grads(params, xa, ya)
        ig = self._hessian_vector_product(dw, xh, yh)
        return [g - eta * h for g, h in zip(da, ig)]

    # ---------------------------------------------------------------------------------------------
    def step(self, input_train, target_train, input_valid, target_valid, eta, network_optimizer, unrolled):
        self.optimizer.zero_grad()
        if unrolled:
            params = self._unrolled_params(input_train, target_train, eta, network_optimizer)
            self._set_grads(self._second_order_alpha(params, input_valid, target_valid, input_train, target_train,
                                                     eta))
        else:
            self._loss(input_valid, target_valid).backward()
        self._opt_step()

    def step_v2(self, input_train, target_train, input_valid, target_valid, lambda_train_regularizer,
                lambda_valid_regularizer=1.0):
        self.optimizer.zero_grad()
        gt = self._alpha_grad(input_train, target_train)
        gv = self._alpha_grad(input_valid, target_valid)
        self._set_grads([v + lambda_train_regularizer * t for t, v in zip(gt, gv)])
        self._opt_step()

    def step_wa(self, input_train, target_train, input_valid, target_valid, lambda_regularizer):
        self.step_v2(input_train, target_train, input_valid, target_valid, lambda_regularizer)

    def step_single_level(self, input_train, target_train):
        self.optimizer.zero_grad()
        self._set_grads(self._alpha_grad(input_train, target_train))
        self._opt_step()

    def step_AOS(self, input_train, target_train, input_valid, target_valid):  # noqa: N802
        self.optimizer.zero_grad()
        self._loss(input_valid, target_valid).backward()
        self._opt_step()

    def step_v2_2ndorder(self, input_train, target_train, input_valid, target_valid, eta, network_optimizer,
                         lambda_train_regularizer, lambda_valid_regularizer=1.0, hvp_on_valid=False):
        self.optimizer.zero_grad()
        params = self._unrolled_params(input_train, target_train, eta, network_optimizer)
        hx, hy = (input_valid, target_valid) if hvp_on_valid else (input_train, target_train)
        gv = self._second_order_alpha(params, input_valid, target_valid, hx, hy, eta)
        gt = self._second_order_alpha(params, input_train, target_train, input_train, target_train, eta)
        self._set_grads([v + lambda_train_regularizer * t for t, v in zip(gt, gv)])
        self._opt_step()

    def step_v2_2ndorder2(self, *a, **kw):
        kw["hvp_on_valid"] = True
        self.step_v2_2ndorder(*a, **kw)
