"""RL algorithm layer: losses, parameter update, schedules, epsilon ladder."""
from .losses import (compute_loss, compute_loss_AQL, compute_loss_device, huber_weighted, priorities_from_td,
                     reference_grad_norm, update_parameters, update_parameters_ex)
from .schedules import actor_epsilon, beta_by_frame, epsilon_by_frame

__all__ = ["compute_loss", "compute_loss_AQL", "compute_loss_device", "huber_weighted", "priorities_from_td",
           "reference_grad_norm", "update_parameters", "update_parameters_ex", "actor_epsilon", "beta_by_frame",
           "epsilon_by_frame"]
