"""Cosine LR schedule with linear warm-up (reference graphphysics/utils/scheduler.py:8-67)."""
import numpy as np
import torch


class CosineWarmupScheduler(torch.optim.lr_scheduler._LRScheduler):
    def __init__(self, optimizer, warmup: int, max_iters: int, min_lr_factor: float = 0.001,
                 last_epoch: int = -1):
        self.warmup = warmup
        self.max_iters = max_iters
        self.min_lr_factor = min_lr_factor
        super().__init__(optimizer, last_epoch)

    def get_lr(self):
        f = self.get_lr_factor(epoch=self.last_epoch)
        return [base * f for base in self.base_lrs]

    def get_lr_factor(self, epoch: int) -> float:
        epoch += 1
        f = 0.5 * (1 + np.cos(np.pi * epoch / self.max_iters))
        if epoch <= self.warmup:
            f *= epoch * 1.0 / self.warmup
        return max(f, self.min_lr_factor)
