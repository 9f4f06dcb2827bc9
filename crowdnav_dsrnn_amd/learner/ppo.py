"""PPO (pytorchBaselines/a2c_ppo_acktr/algo/ppo.py:7-118) with an optional data-parallel all-reduce.

Single process: the reference's update, operation for operation. With torch.distributed initialised
(world > 1, one process per GPU, backend "nccl" = RCCL over xGMI):
  * advantages are normalised with the global mean and unbiased std (one all_reduce of [sum, sumsq, n]);
  * after backward, the gradients are flattened into one bucket (973,983 fp32 = 3.9 MB for the DSRNN)
    and all-reduced (SUM, then / world) before clip_grad_norm_ and the Adam step, so every rank applies
    the same update;
  * the reported losses are averaged over ranks.
"""
import torch
import torch.nn as nn
import torch.optim as optim


def _dist():
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        return dist
    return None


class PPO:
    def __init__(self, actor_critic, clip_param, ppo_epoch, num_mini_batch, value_loss_coef, entropy_coef, lr=None,
                 eps=None, max_grad_norm=None, use_clipped_value_loss=True):
        self.actor_critic = actor_critic
        self.clip_param = clip_param
        self.ppo_epoch = ppo_epoch
        self.num_mini_batch = num_mini_batch
        self.value_loss_coef = value_loss_coef
        self.entropy_coef = entropy_coef
        self.max_grad_norm = max_grad_norm
        self.use_clipped_value_loss = use_clipped_value_loss
        self.optimizer = optim.Adam(actor_critic.parameters(), lr=lr, eps=eps)
        self.dist = _dist()
        if self.dist is not None:   # start from identical weights on every rank
            for p in actor_critic.parameters():
                self.dist.broadcast(p.data, 0)

    def _normalised_advantages(self, rollouts):
        adv = rollouts.returns[:-1] - rollouts.value_preds[:-1]
        if self.dist is None:
            return (adv - adv.mean()) / (adv.std() + 1e-5)
        stats = torch.stack([adv.sum(), (adv * adv).sum(), torch.tensor(float(adv.numel()), device=adv.device)])
        stats = stats.double()
        self.dist.all_reduce(stats)
        s, ss, n = stats[0], stats[1], stats[2]
        mean = s / n
        std = torch.sqrt(torch.clamp((ss - n * mean * mean) / (n - 1), min=0.0))
        return (adv - mean.float()) / (std.float() + 1e-5)

    def _allreduce_grads(self):
        grads = [p.grad for p in self.actor_critic.parameters() if p.grad is not None]
        flat = torch.cat([g.reshape(-1) for g in grads])
        self.dist.all_reduce(flat)
        flat /= self.dist.get_world_size()
        o = 0
        for g in grads:
            g.copy_(flat[o:o + g.numel()].view_as(g))
            o += g.numel()

    def update(self, rollouts):
        advantages = self._normalised_advantages(rollouts)
        acc = None
        for _ in range(self.ppo_epoch):
            if self.actor_critic.is_recurrent:
                gen = rollouts.recurrent_generator(advantages, self.num_mini_batch)
            else:
                gen = rollouts.feed_forward_generator(advantages, self.num_mini_batch)
            for (obs_b, hxs_b, actions_b, value_preds_b, return_b, masks_b, old_logp_b, adv_targ) in gen:
                values, action_log_probs, dist_entropy, _ = self.actor_critic.evaluate_actions(
                    obs_b, hxs_b, masks_b, actions_b)
                ratio = torch.exp(action_log_probs - old_logp_b)
                surr1 = ratio * adv_targ
                surr2 = torch.clamp(ratio, 1.0 - self.clip_param, 1.0 + self.clip_param) * adv_targ
                action_loss = -torch.min(surr1, surr2).mean()
                if self.use_clipped_value_loss:
                    value_pred_clipped = value_preds_b + (values - value_preds_b).clamp(-self.clip_param,
                                                                                      self.clip_param)
                    value_losses = (values - return_b).pow(2)
                    value_losses_clipped = (value_pred_clipped - return_b).pow(2)
                    value_loss = 0.5 * torch.max(value_losses, value_losses_clipped).mean()
                else:
                    value_loss = 0.5 * (return_b - values).pow(2).mean()
                self.optimizer.zero_grad()
                (value_loss * self.value_loss_coef + action_loss - dist_entropy * self.entropy_coef).backward()
                if self.dist is not None:
                    self._allreduce_grads()
                nn.utils.clip_grad_norm_(self.actor_critic.parameters(), self.max_grad_norm)
                self.optimizer.step()
                # accumulated on the device: one host sync per update instead of three per minibatch
                d = torch.stack([value_loss.detach(), action_loss.detach(), dist_entropy.detach()]).double()
                acc = d if acc is None else acc + d
        if self.dist is not None:
            self.dist.all_reduce(acc)
            acc = acc / self.dist.get_world_size()
        vals = acc.double().cpu().tolist()
        n = self.ppo_epoch * self.num_mini_batch
        value_loss_epoch, action_loss_epoch, dist_entropy_epoch = (x / n for x in vals)
        return value_loss_epoch, action_loss_epoch, dist_entropy_epoch
