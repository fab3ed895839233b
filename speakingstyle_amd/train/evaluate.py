"""Validation pass (reference ``evaluate.py:18-88``): loss means over ``val.txt``
weighted by sub-batch size, one synthesized sample logged.  With DP each rank
evaluates a shard and the sums are all-reduced.  ``named_param`` defaults to the
FiLM scalars (the reference's standalone ``evaluate.py`` crashes on ``None``, D5)."""
from __future__ import annotations

import torch
from torch.utils.data import DataLoader

from ..data.dataset import Dataset, to_device
from ..models.loss import FastSpeech2Loss
from ..parallel import ddp
from ..utils.logging import log_scalars, synth_one_sample


@torch.no_grad()
def evaluate(model, step, configs, logger=None, vocoder=None, named_param=None):
    preprocess_config, model_config, train_config = configs
    world, rank = ddp.world_size(), ddp.rank()
    dataset = Dataset("val.txt", preprocess_config, train_config, sort=False, drop_last=False,
                      shard=(rank, world) if world > 1 else None)
    loader = DataLoader(dataset, batch_size=train_config["optimizer"]["batch_size"], shuffle=False,
                        collate_fn=dataset.collate_fn, num_workers=2)
    loss_fn = FastSpeech2Loss(preprocess_config, train_config)
    device = next(model.parameters()).device
    sums = torch.zeros(7, dtype=torch.float64, device=device)
    batch = output = None
    for batchs in loader:
        for batch in batchs:
            batch = to_device(batch, device)
            output = model(*batch[2:])
            named = named_param if named_param is not None else model.film_scalars()
            losses = loss_fn(batch, output, named)
            n = len(batch[0])
            for i in range(6):
                sums[i] += float(losses[i]) * n
            sums[6] += n
    if world > 1:
        torch.distributed.all_reduce(sums)
    means = (sums[:6] / sums[6].clamp(min=1)).tolist()
    message = ("Validation Step {}, Total Loss: {:.4f}, Mel Loss: {:.4f}, Mel PostNet Loss: {:.4f}, "
               "Pitch Loss: {:.4f}, Energy Loss: {:.4f}, Duration Loss: {:.4f}").format(step, *means)
    if logger is not None:
        log_scalars(logger, step, losses=means)
        if batch is not None:
            synth_one_sample(batch, output, vocoder, model_config, preprocess_config, logger, step, "Validation")
    return message
