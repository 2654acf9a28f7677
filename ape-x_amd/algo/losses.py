"""Learner losses and the parameter update (reference utils.py:44-97).

``compute_loss``: double-DQN n-step target with a PER-weighted Huber(1) loss::

    a*  = argmax_a Q_online(s')          y = r + gamma^n Q_target(s', a*) (1 - d)
    d_i = |y - Q_online(s, a)|           loss = mean(w * huber(d))
    prio = 0.9 max(d) + 0.1 d + 1e-6     (batch-max mixing)

``compute_loss_AQL`` is the same over candidate sets, with the candidates sampled at
s_t re-used to evaluate s' (utils.py:47-49).  Priorities are returned as a NumPy
array like the reference (host sync); engines that keep priorities on device use
``compute_loss_device`` (returns a device tensor) or the fused HIP loss kernel.

``update_parameters`` returns the reference's *reported* norm
``(sum_p ||g_p||^(1/2))^(1/2)`` while clipping with the true global L2;
``update_parameters_ex`` returns both.
"""
from __future__ import annotations

import torch


def _td_terms(q_values, next_q_values, tgt_next_q_values, actions, rewards, dones, n_steps, gamma):
    q_a = q_values.gather(1, actions.unsqueeze(1)).squeeze(1)
    next_actions = next_q_values.max(1)[1].unsqueeze(1)
    next_q_a = tgt_next_q_values.gather(1, next_actions).squeeze(1)
    target = rewards + (gamma ** n_steps) * next_q_a * (1 - dones)
    return torch.abs(target.detach() - q_a)


def huber_weighted(td_error, weights):
    loss = torch.where(td_error < 1, 0.5 * td_error ** 2, td_error - 0.5)
    return (loss * weights).mean()


def priorities_from_td(td_error):
    return 0.9 * torch.max(td_error) + 0.1 * td_error + 1e-6


def compute_loss_device(model, tgt_model, batch, n_steps, gamma=0.99):
    states, actions, rewards, next_states, dones, weights = batch
    q_values = model(states)
    with torch.no_grad():
        next_q_values = model(next_states)
        tgt_next_q_values = tgt_model(next_states)
    td = _td_terms(q_values, next_q_values, tgt_next_q_values, actions, rewards, dones, n_steps, gamma)
    return huber_weighted(td, weights), priorities_from_td(td).detach()


def compute_loss(model, tgt_model, batch, n_steps, gamma=0.99):
    loss, prios = compute_loss_device(model, tgt_model, batch, n_steps, gamma)
    return loss, prios.cpu().numpy()


def compute_loss_AQL(model, tgt_model, batch, n_steps, gamma=0.99):
    states, actions, rewards, next_states, dones, a_mu, weights = batch
    q_values = model(states, a_mu)
    next_q_values = model(next_states, a_mu)
    tgt_next_q_values = tgt_model(next_states, a_mu)
    td = _td_terms(q_values, next_q_values, tgt_next_q_values, actions, rewards, dones, n_steps, gamma)
    return huber_weighted(td, weights), priorities_from_td(td).detach().cpu().numpy()


def reference_grad_norm(parameters) -> torch.Tensor:
    """The reference's logged 'grad_norm': (sum_p ||g_p||_2^(1/2))^(1/2)."""
    total = 0.0
    for p in parameters:
        if p.grad is not None:
            total = total + p.grad.detach().norm(2) ** 0.5
    return total ** 0.5


def update_parameters_ex(loss, model, optimizer, max_norm):
    optimizer.zero_grad()
    loss.backward()
    params = [p for p in model.parameters() if p.grad is not None]
    ref_norm = reference_grad_norm(params)
    l2 = torch.nn.utils.clip_grad_norm_(params, max_norm)
    optimizer.step()
    return ref_norm, l2


def update_parameters(loss, model, optimizer, max_norm):
    return update_parameters_ex(loss, model, optimizer, max_norm)[0]
